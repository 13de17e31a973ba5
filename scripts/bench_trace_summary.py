#!/usr/bin/env python3
"""Per-config kernel durations from a rocprofv3 --kernel-trace CSV of bench.py.

bench.py's default run times C2, then the c3 / c4 / c5_strong / fill / slots /
receive / segment keys, one config after another in one process.  Each config
starts by generating its batch on the device (a synth_kernel launch), which
cuts the trace into configs; inside each config the library's launches are
grouped by (kernel, grid size) and each group's LAST K launches (the K timed
steps; the settle and warm-up launches come before them) are averaged; the
config's per-step time is the sum over its groups.

    python scripts/bench_trace_summary.py gpurun_out/prof_all/run_kernel_trace.csv --last 20 \\
        --names c2,c5_strong,fill,slots,receive,segment,c3,c4
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
    ap.add_argument("--names", default="")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    # every config's batch is generated on the device first (tcpck_synth_*): a
    # synth_kernel launch opens the next config
    phases = []
    for r in rows:
        if "synth_kernel" in r["Kernel_Name"] or not phases:
            phases.append([])
        phases[-1].append(r)
    timed = []
    for ph in phases:
        groups: dict = {}
        for r in ph:
            if "tcpck" not in r["Kernel_Name"] or "synth_kernel" in r["Kernel_Name"]:
                continue
            key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
            groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if any(len(d) >= args.last for d in groups.values()):
            timed.append(groups)
    names = args.names.split(",") if args.names else []
    print(f"{'config':10s} {'kernel':58s} {'grid':>10s} {'launches':>8s} {'avg_last%d_us' % args.last:>12s} "
          f"{'min':>9s} {'max':>9s}")
    for i, groups in enumerate(timed):
        label = names[i] if i < len(names) else f"phase{i}"
        total = 0.0
        for (name, grid), d in groups.items():
            if len(d) < args.last:
                continue
            tail = d[-args.last:]
            total += statistics.mean(tail)
            print(f"{label:10s} {name:58s} {grid:10d} {len(d):8d} {statistics.mean(tail):12.2f} "
                  f"{min(tail):9.2f} {max(tail):9.2f}")
        print(f"{label:10s} {'(per step, all kernels above)':58s} {'':10s} {'':8s} {total:12.2f}")


if __name__ == "__main__":
    main()
