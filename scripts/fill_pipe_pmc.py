#!/usr/bin/env python3
"""HBM bytes per pipelined FILL call from rocprofv3 --pmc passes of
scripts/fill_pipe_probe.py --pmc-calls N (one K per run, FETCH_SIZE and
WRITE_SIZE in separate runs, /opt/skills/guides/MI355X_MICROARCH.md: both in
KiB, FETCH_SIZE doubled on gfx950 for wide streaming reads).

    python scripts/fill_pipe_pmc.py DIR_PREFIX N  ->  per K: read GB, written GB per call

DIR_PREFIX_<K>_{fetch,write}/run_counter_collection.csv; only the FILL's own
kernels (OURS) count -- the batch generator and torch's clone are excluded.
"""
import csv
import glob
import sys

OURS = ("vvstream_kernel", "rstream_kernel", "patch_fields_kernel", "seg_kernel", "sstream_kernel")


def total(path: str, counter: str) -> float:
    s = 0.0
    with open(path) as f:
        for r in csv.DictReader(f):
            if not any(k in r["Kernel_Name"] for k in OURS) or r.get("Counter_Name", counter) != counter:
                continue
            s += float(r["Counter_Value"])
    return s


def main():
    prefix, calls = sys.argv[1], int(sys.argv[2])
    for d in sorted(glob.glob(f"{prefix}_*_fetch")):
        k = d[len(prefix) + 1:-len("_fetch")]
        f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        w = glob.glob(f"{prefix}_{k}_write/**/*counter_collection.csv", recursive=True)
        if not f or not w:
            continue
        rd = 2 * 1024 * total(f[0], "FETCH_SIZE") / calls / 1e9
        wr = 1024 * total(w[0], "WRITE_SIZE") / calls / 1e9
        print(f"K {k:>4s}: read {rd:.3f} GB  written {wr:.3f} GB  per call")


if __name__ == "__main__":
    main()
