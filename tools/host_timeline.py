"""Timeline of host-API calls from a rocprofv3 --kernel-trace --memory-copy-trace directory:
kernels and copies merged in start order, cut into calls at each host-to-device copy, and
per call the mean duration of every operation plus the gaps between them.

    python tools/host_timeline.py gpurun_out/.../trace_dir [--last 100]
"""
import argparse
import collections
import csv
import glob
import json
import os

import numpy as np


def load(d):
    ev = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                           "K:" + r["Kernel_Name"].split("(")[0].split("<")[0][-28:]))
    for path in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or "COPY"
                size = r.get("Bytes") or r.get("Size") or ""
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                           "C:" + kind.replace("MEMORY_COPY_", "")[-16:] + (f":{size}" if size else "")))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=100, help="calls at the end of the trace")
    args = ap.parse_args()
    ev = load(args.dir)
    calls, cur = [], []
    for e in ev:
        # a call starts at the first host-to-device copy after other work (an overlapped
        # upload is several copies in a row)
        if "HOST_TO_DEVICE" in e[2] and cur and "HOST_TO_DEVICE" not in cur[-1][2]:
            calls.append(cur)
            cur = []
        cur.append(e)
    if cur:
        calls.append(cur)
    calls = calls[-args.last:]
    shape = collections.Counter(tuple(x[2] for x in c) for c in calls).most_common(1)[0][0]
    same = [c for c in calls if tuple(x[2] for x in c) == shape]
    ops = []
    for i, name in enumerate(shape):
        dur = [(c[i][1] - c[i][0]) / 1e3 for c in same]
        gap = [(c[i][0] - c[i - 1][1]) / 1e3 for c in same] if i else [0.0]
        ops.append({"op": name, "us_mean": round(float(np.mean(dur)), 2),
                    "gap_before_us_mean": round(float(np.mean(gap)), 2)})
    span = [(c[-1][1] - c[0][0]) / 1e3 for c in same]
    print(json.dumps({"calls": len(calls), "calls_of_main_shape": len(same), "ops": ops,
                      "device_span_us_mean": round(float(np.mean(span)), 2)}, indent=1))


if __name__ == "__main__":
    main()
