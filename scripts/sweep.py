#!/usr/bin/env python3
"""In-process A/B sweep of the checksum kernel variants on the BASELINE configs.

    python scripts/sweep.py [--configs c2,c3,c4] [--rounds 5] [--reps 10]

Every variant of include/tcpck_tuning.h runs on the same resident batch,
interleaved over several rounds (cdna_hip_programming.md 5.4 rule 24); each
launch is timed with HIP events on the launch stream.  Results are checked
against the AUTO kernel's output before timing.  Prints one line per variant
(median / min GB/s, % of the 8 TB/s roof) and writes gpurun_out/sweep.json.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from synth_np import mixed_layout  # noqa: E402


def build(cfg):
    if cfg == "c2":
        count, L = 1 << 20, 1492
    elif cfg == "c4":
        count, L = 256 << 10, 65536
    else:
        count, L = 4 << 20, None
    if L:
        a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, count, seed=42)
        return dict(fixed=True, arena=a, count=count, L=L, bytes=count * L)
    off, ln, total = mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
    return dict(fixed=False, arena=a, off=d_off, ln=d_ln, count=count, bytes=int(ln.astype(np.int64).sum()),
                min_len=int(ln.min()), max_len=int(ln.max()))


def variants(w):
    v = [("auto", tcpck.KERNEL_AUTO, 0)]
    v += [(f"seg {n}", tcpck.KERNEL_SEG, p) for p, n in tcpck.SEG_SHAPES.items()]
    v += [(f"vvstream v{p}", tcpck.KERNEL_VVSTREAM, p) for p in (0, 1, 2, 3, 4)]
    if w["fixed"] and w["L"] <= 16384:
        v += [(f"rstream v{p}", tcpck.KERNEL_RSTREAM, p) for p in (0, 1, 2, 9, 10, 11, 12, 13)]
    return v


def launch(ctx, w, out, kernel, param, stream):
    if w["fixed"]:
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, w["arena"], w["L"], w["L"], w["count"], out, kernel, param,
                           stream=stream)
    else:
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, w["arena"], w["off"], w["ln"], w["count"], out, kernel, param,
                         total_bytes=w["bytes"], min_len=w["min_len"], max_len=w["max_len"], packed=True,
                         stream=stream)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c2,c3,c4")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=10)
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    stream = torch.cuda.current_stream()
    report = {}
    for cfg in args.configs.split(","):
        w = build(cfg)
        algo = w["bytes"] + 2 * w["count"]
        ref = torch.empty(w["count"], dtype=torch.int16, device="cuda")
        launch(ctx, w, ref, tcpck.KERNEL_AUTO, 0, stream)
        vs = variants(w)
        times = {name: [] for name, _, _ in vs}
        out = torch.empty_like(ref)
        for name, k, prm in vs:  # correctness + warm-up
            out.zero_()
            launch(ctx, w, out, k, prm, stream)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), f"{cfg} {name}: results differ from AUTO"
        for _ in range(args.rounds):
            for name, k, prm in vs:
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(args.reps)]
                for s, e in ev:
                    s.record(stream)
                    launch(ctx, w, out, k, prm, stream)
                    e.record(stream)
                torch.cuda.synchronize()
                times[name] += [s.elapsed_time(e) for s, e in ev]
        rows = []
        for name, _, _ in vs:
            t = np.array(times[name])
            med, mn = float(np.median(t)), float(t.min())
            rows.append({"variant": name, "median_ms": med, "min_ms": mn,
                         "GBps_median": algo / med / 1e6, "GBps_best": algo / mn / 1e6,
                         "frac_median": algo / med / 1e6 / 8000.0})
            print(f"{cfg} {name:12s} median {med:8.4f} ms  {algo / med / 1e6:7.1f} GB/s "
                  f"({algo / med / 1e6 / 80:.1f}%)  best {algo / mn / 1e6:7.1f} GB/s", flush=True)
        report[cfg] = {"algorithmic_bytes": algo, "rows": rows}
        del w
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sweep.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
