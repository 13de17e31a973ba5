"""Summarise the rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_summary.json.

Input: gpurun_out/pmc_<cfg>_{fetch,write}/run_counter_collection.csv from
`STEPS="pmc_c2 pmc_c3 pmc_c4" bash scripts/gpu_check.sh` (one counter per pass:
FETCH_SIZE and WRITE_SIZE do not fit one pass of the 4 TCC slots).

Each config's two passes must carry the same libtcpck.so sha256 (written by
gpu_check.sh beside the CSVs); the entry is stamped with it and bench.py uses
it only while that very library is the one loaded.

Units and corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section):
both counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced streaming read (16 B/lane), so it is doubled; WRITE_SIZE is
exact.  HBM bytes per launch = 1024 * (2 * FETCH_SIZE + WRITE_SIZE), averaged
over the launches of the dominant (checksum) kernel.  The raw CSVs are copied
to profiles/<round>/ next to the summary.
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("rstream_kernel", "vvstream_kernel", "seg_kernel", "jumbo_kernel", "sstream_kernel", "segment_kernel",
           "header_swap_kernel", "header_extract_kernel", "patch_fields_kernel", "gstream_kernel")
CONFIGS = ("c2", "c3", "c4", "c5", "slots", "segment", "receive", "fill", "fill_noout", "fill_c3", "c2_rfc")


def per_launch(path: str, counter: str):
    """Mean counter value per launch of each step kernel, summed over the step's
    kernels (two for `receive`: VERIFY, then the header pass; and for `fill`:
    the stream, then the field-block pass)."""
    vals: dict[str, list[float]] = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            key = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if r["Counter_Name"] != counter or key is None:
                continue
            vals.setdefault(key, []).append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no checksum-kernel rows for {counter} in {path}")
    return " + ".join(sorted(vals)), sum(statistics.mean(v) for v in vals.values()), min(len(v) for v in vals.values())


def main(rnd: str = "r01", *only: str) -> None:
    """rnd: the profiles/ subdirectory for the CSVs; only: the configs to
    update (default: every config with both passes under gpurun_out/)."""
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    out_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(out_path) as f:
            summary = json.load(f)
    except (OSError, ValueError):
        summary = {}
    for cfg in CONFIGS:
        if only and cfg not in only:
            continue
        fp = os.path.join(src, f"pmc_{cfg}_fetch", "run_counter_collection.csv")
        wp = os.path.join(src, f"pmc_{cfg}_write", "run_counter_collection.csv")
        if not (os.path.exists(fp) and os.path.exists(wp)):
            continue
        # the library both passes ran (scripts/gpu_check.sh writes its sha256 beside them)
        shas = set()
        for ph in ("fetch", "write"):
            sp = os.path.join(src, f"pmc_{cfg}_{ph}_lib.sha256")
            if os.path.exists(sp):
                shas.add(open(sp).read().split()[0])
        if len(shas) != 1:
            print(f"{cfg}: skipped, library stamps {sorted(shas) or 'missing'}")
            continue
        kname, fetch_kib, n = per_launch(fp, "FETCH_SIZE")
        _, write_kib, _ = per_launch(wp, "WRITE_SIZE")
        read_b = 2.0 * fetch_kib * 1024.0
        write_b = write_kib * 1024.0
        summary[cfg] = {
            "kernel": kname,
            "launches": n,
            "fetch_size_kib_raw": round(fetch_kib, 3),
            "write_size_kib_raw": round(write_kib, 3),
            "hbm_read_bytes_per_launch": int(read_b),
            "hbm_write_bytes_per_launch": int(write_b),
            "hbm_bytes_per_launch": int(read_b + write_b),
            "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count on 16-B/lane streams); write = WRITE_SIZE KiB",
            "source": f"profiles/{rnd}/pmc_{cfg}_{{fetch,write}}.csv",
            "lib_sha256": shas.pop(),
        }
        shutil.copy(fp, os.path.join(dst, f"pmc_{cfg}_fetch.csv"))
        shutil.copy(wp, os.path.join(dst, f"pmc_{cfg}_write.csv"))
        print(cfg, json.dumps(summary[cfg]))
    with open(out_path, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    if any(a.startswith("-") for a in sys.argv[1:]):
        raise SystemExit("usage: pmc_summary.py [round] [config ...]")
    main(*sys.argv[1:])
