#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, with the
average over the LAST K launches of the dominant checksum kernel (the bench's
timed launches come last; the settle/warm-up launches before them include the
idle GPU's clock ramp).

    python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv [--last 20]
"""
import argparse
import csv
import statistics

KERNELS = ("rstream_kernel", "vvstream_kernel", "seg_kernel", "jumbo_kernel", "sstream_kernel", "segment_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=20)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ck = [r for r in rows if any(k in r["Kernel_Name"] for k in KERNELS)]
    if not ck:
        raise SystemExit("no checksum kernel in trace")
    name = ck[-1]["Kernel_Name"]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ck if r["Kernel_Name"] == name]
    tail = d[-args.last:]
    print(f"kernel: {name}")
    print(f"launches: {len(d)}  all: avg {statistics.mean(d):.2f} us  min {min(d):.2f}  max {max(d):.2f}")
    print(f"last {len(tail)}: avg {statistics.mean(tail):.2f} us  min {min(tail):.2f}  max {max(tail):.2f}")


if __name__ == "__main__":
    main()
