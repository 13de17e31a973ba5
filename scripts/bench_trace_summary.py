#!/usr/bin/env python3
"""Per-config kernel durations from a rocprofv3 --kernel-trace CSV of bench.py.

bench.py's default run times C2, then C3, C4 and C5 (the c3 / c4 / c5_strong
keys) in one process.  Each config's checksum launches share one (kernel,
grid size) pair -- C2 and C5 are the same rstream instantiation but different
grids -- so launches are grouped by that pair, in order of first appearance,
and each group's LAST K launches (the K timed steps; the settle and warm-up
launches come before them) are averaged.  Groups with fewer than K launches
(the data generator, the e2e leg's chunk launches) are listed for reference.

    python scripts/bench_trace_summary.py gpurun_out/prof_all/run_kernel_trace.csv --last 20
"""
import argparse
import csv
import re
import statistics


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=20)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    groups: dict = {}
    for r in rows:
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':58s} {'grid':>10s} {'launches':>8s} {'avg_all_us':>11s} "
          f"{'avg_last%d_us' % args.last:>12s} {'min':>9s} {'max':>9s}")
    for (name, grid), d in groups.items():
        tail = d[-args.last:]
        mark = "" if len(d) >= args.last else "  (fewer than K launches)"
        print(f"{name:58s} {grid:10d} {len(d):8d} {statistics.mean(d):11.2f} {statistics.mean(tail):12.2f} "
              f"{min(tail):9.2f} {max(tail):9.2f}{mark}")


if __name__ == "__main__":
    main()
