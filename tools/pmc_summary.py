"""Summarise rocprofv3 --pmc CSV output per kernel: counter totals per dispatch.

    python tools/pmc_summary.py gpurun_out/pmc_a [gpurun_out/pmc_b ...] [--kernel fast_sweep]

Each directory is one --pmc pass (rocprofv3 -d DIR -o p --output-format csv).  Counter
values of a dispatch are summed over the rows rocprofv3 writes for it, then averaged over
the dispatches of every kernel whose name contains --kernel.
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(dirname, kernel):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for path in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if kernel not in row["Kernel_Name"]:
                    continue
                d = row["Dispatch_Id"]
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
                names[d] = row["Kernel_Name"][:80]
    return per, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="fast_sweep")
    args = ap.parse_args()
    out = {}
    for d in args.dirs:
        per, names = load(d, args.kernel)
        if not per:
            continue
        acc = collections.defaultdict(list)
        for disp, counters in per.items():
            for k, v in counters.items():
                acc[k].append(v)
        for k, vs in acc.items():
            out[k] = sum(vs) / len(vs)
        out.setdefault("_dispatches", {})[os.path.basename(d)] = len(per)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
