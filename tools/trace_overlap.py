"""Do kernels overlap in time?  Reads a rocprofv3 --kernel-trace CSV directory and reports,
over the dispatches in start order, how often a kernel starts before the previous one ends
and by how much, plus each kernel's mean duration and the mean start-to-start interval.

    python tools/trace_overlap.py gpurun_out/.../trace_dir [--last 200]
"""
import argparse
import csv
import glob
import json
import os

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=200, help="only the last N dispatches")
    args = ap.parse_args()
    rows = []
    for path in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"].split("(")[0][-60:], r.get("Queue_Id", "")))
    rows.sort()
    rows = rows[-args.last:]
    ov, gaps = [], []
    end_max = None
    for s, e, _, _ in rows:
        if end_max is not None:
            (ov if s < end_max else gaps).append(abs(end_max - s) / 1e3)
        end_max = e if end_max is None else max(end_max, e)
    by = {}
    for s, e, k, q in rows:
        by.setdefault(k, []).append((e - s) / 1e3)
    starts = np.array([s for s, _, _, _ in rows], dtype=np.float64)
    print(json.dumps({
        "dispatches": len(rows),
        "overlapping_starts": len(ov), "overlap_us_mean": round(float(np.mean(ov)), 2) if ov else 0.0,
        "gap_us_mean": round(float(np.mean(gaps)), 2) if gaps else 0.0,
        "span_us": round((rows[-1][1] - rows[0][0]) / 1e3, 1) if rows else 0.0,
        "queues": sorted({q for _, _, _, q in rows}),
        "kernel_us_mean": {k: round(float(np.mean(v)), 2) for k, v in by.items()},
        "start_interval_us_mean": round(float(np.mean(np.diff(starts))) / 1e3, 2) if len(rows) > 1 else 0.0,
    }, indent=1))


if __name__ == "__main__":
    main()
