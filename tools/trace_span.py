"""Per-launch cost of the detector from a rocprofv3 --kernel-trace directory, in bench.py's
terms: over the last N dispatches of the kernel (the timed region of a bench run; the settle
and warm-up launches come before it), the span from the first start to the last end divided
by N (= roofline.kernel_ms_avg when launch lanes overlap the launches) and the mean of the
dispatches' own durations (= roofline.launch_ms_avg; with one lane the two agree).

    python tools/trace_span.py TRACE_DIR [--last 50] [--kernel fast_sweep_kernel]
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=50)
    ap.add_argument("--kernel", default="fast_sweep_kernel")
    args = ap.parse_args()
    ev = []
    for path in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                if args.kernel in r["Kernel_Name"]:
                    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                               r.get("Queue_Id", "")))
    ev.sort()
    if not ev:
        raise SystemExit(f"no {args.kernel} dispatches under {args.dir}")
    last = ev[-args.last:]
    span = (max(e[1] for e in last) - last[0][0]) / 1e6
    dur = [(e[1] - e[0]) / 1e6 for e in last]
    print(json.dumps({"kernel": args.kernel, "dispatches_total": len(ev), "window": len(last),
                      "span_ms_per_launch": round(span / len(last), 4),
                      "duration_ms_mean": round(sum(dur) / len(dur), 4),
                      "queues": sorted({e[2] for e in last})}))


if __name__ == "__main__":
    main()
