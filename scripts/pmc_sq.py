#!/usr/bin/env python3
"""Per-kernel means of the counters in rocprofv3 counter_collection CSVs
(one or more passes), with the last N dispatches of each kernel (the probe's
timed launches come last).

    python scripts/pmc_sq.py gpurun_out/sq1/run_counter_collection.csv [...] [--last 5]
"""
import argparse
import collections
import csv
import re


def short(name):
    m = re.search(r"(\w+_kernel)<([^>]*)>", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--last", type=int, default=5)
    args = ap.parse_args()
    table = collections.defaultdict(dict)  # kernel -> counter -> [values by dispatch]
    for path in args.csv:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        order = collections.defaultdict(list)
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                d = int(r["Dispatch_Id"])
                if d not in per[k]:
                    order[k].append(d)
                per[k][(d, r["Counter_Name"])] += float(r["Counter_Value"])
        for k, vals in per.items():
            ds = sorted(set(d for d, _ in vals))[-args.last:]
            names = sorted(set(c for _, c in vals))
            for c in names:
                xs = [vals[(d, c)] for d in ds if (d, c) in vals]
                table[k][c] = sum(xs) / len(xs)
    for k, cs in table.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"  {c:28s} {v:16.1f}")


if __name__ == "__main__":
    main()
