#!/usr/bin/env python3
"""Grid oversubscription probe for the run-per-wave kernels.

With exactly one wave per resident slot, the SIMD's issue arbitration (by age)
finishes slot-0 waves ~2x earlier than slot-7 waves and the last ones stream
alone.  Launching M x the resident grid lets the dispatcher refill freed slots
with fresh (smaller) runs.  Each (variant, M) is checked bit-exactly against
the seg kernel, then timed: median HIP-event launch time over interleaved
rounds, in this one process (compare numbers within one run only: boxes differ
by a few percent).

    python scripts/oversub.py [--what c2,c5,c4,v256,v96,c3] [--variants 0,10] [--ms 1,8,32]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

# name: (image length, count, kernel, default variants)
FIXED = {"c2": (1492, 1 << 20, tcpck.KERNEL_RSTREAM, (0, 10)),
         "c5": (1492, 8 << 20, tcpck.KERNEL_RSTREAM, (0,)),
         "c5v": (1492, 8 << 20, tcpck.KERNEL_VVSTREAM, (0, 1)),
         "c2v": (1492, 1 << 20, tcpck.KERNEL_VVSTREAM, (0, 1)),
         "c4": (65536, 256 << 10, tcpck.KERNEL_SEG, (3,)),
         "c4r": (65536, 256 << 10, tcpck.KERNEL_RSTREAM, (0, 10)),
         "c4v": (65536, 256 << 10, tcpck.KERNEL_VVSTREAM, (0, 1)),
         "v256": (256, 6 << 20, tcpck.KERNEL_VVSTREAM, (0, 1)),
         "v96": (96, 16 << 20, tcpck.KERNEL_VVSTREAM, (0, 1))}


def timed(fn, params, rounds=8, reps=3):
    s = torch.cuda.current_stream()
    t = {p: [] for p in params}
    for _ in range(rounds):
        for p in params:
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                fn(p)
                e1.record(s)
                torch.cuda.synchronize()
                t[p].append(e0.elapsed_time(e1))
    return {p: float(np.median(v)) for p, v in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="c2,c5,c4,v256,v96,c3")
    ap.add_argument("--variants", default="")
    ap.add_argument("--ms", default="1,4,8,12,16,24,32,64")
    args = ap.parse_args()
    ms = [int(m) for m in args.ms.split(",")]
    ctx = tcpck.Context(0, probe=True)
    for what in args.what.split(","):
        if what in FIXED:
            L, n, kern, variants = FIXED[what]
            if args.variants:
                variants = [int(v) for v in args.variants.split(",")]
            a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
            tcpck.synth_fixed(a, L, L, n, seed=42)
            ref = torch.empty(n, dtype=torch.int16, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, ref, tcpck.KERNEL_SEG, 0)
            out = torch.empty(n, dtype=torch.int16, device="cuda")

            def run(p):
                ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, kern, p)
            nbytes = n * L + 2 * n
            label = f"L={L:5d} n={n:9d} kernel {kern}"
        elif what == "c3":
            from synth_np import mixed_layout
            variants = [int(v) for v in args.variants.split(",")] if args.variants else (2, 3)
            off, ln, total = mixed_layout(4 << 20, seed=42)
            n = ln.size
            a = torch.empty(total, dtype=torch.uint8, device="cuda")
            d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
            ref = torch.empty(n, dtype=torch.int16, device="cuda")
            ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, ref, tcpck.KERNEL_SEG, 0)
            out = torch.empty(n, dtype=torch.int16, device="cuda")

            def run(p):
                ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_VVSTREAM, p, packed=True,
                                 total_bytes=total)
            nbytes = total + 2 * n
            label = "C3 vvstream"
        else:
            raise SystemExit(f"unknown --what {what}")
        params = []
        for p in [v | (m << 16) for v in variants for m in ms]:
            out.zero_()
            try:
                run(p)
            except tcpck.TcpckError:  # variant not defined for this kernel
                continue
            torch.cuda.synchronize()
            assert torch.equal(out, ref), (what, p)
            params.append(p)
        med = timed(run, params)
        for p in params:
            gbs = nbytes / (med[p] * 1e-3) / 1e9
            print(f"{label} variant {p & 0xFF:2d} x{p >> 16:<3d} {med[p]:8.4f} ms {gbs:7.1f} GB/s "
                  f"({gbs / 80:.1f}%)", flush=True)
        del a, ref, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
