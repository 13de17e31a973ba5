#!/usr/bin/env python3
"""FILL of fixed images >= 1 KiB by kernel: AUTO against rstream's policy (variant
20).  Back-to-back launches after a clock settle, interleaved rounds; every
candidate's arena and results checked against seg first.  (A variant 25 that kept
each image's 128-B field line in registers and wrote it back whole when the image
ended measured 57.6 % against 69.0 % at 1492 B and was removed:
profiles/r01/fill_line_writeback_probe.log.)

    python scripts/fill_wb_probe.py [--lengths 1024,1492,...] [--bytes 1.5e9]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck as K  # noqa: E402
from xcd_probe import b2b  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lengths", default="1024,1492,2000,4096,9000,65536")
    ap.add_argument("--bytes", type=float, default=1.5e9)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ops", default="fill")
    args = ap.parse_args()
    ctx = K.Context(0)
    s = torch.cuda.current_stream()
    cands = [("auto", None, 0), ("rstream v20", K.KERNEL_RSTREAM, 20)]
    for L in [int(x) for x in args.lengths.split(",")]:
        n = int(args.bytes) // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, L, L, n, seed=42)
        a0 = a.clone()
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(K.OP_FILL, a, L, L, n, ref, K.KERNEL_SEG, 0)
        filled = a.clone()
        out = torch.empty(n, dtype=torch.int16, device="cuda")

        for opname in args.ops.split(","):
            op = K.OP_FILL if opname == "fill" else K.OP_CHECKSUM

            def run(c, op=op):
                if c[1] is None:
                    ctx.batch_fixed(op, a, L, L, n, out, stream=s)
                else:
                    ctx.batch_fixed_ex(op, a, L, L, n, out, c[1], c[2], stream=s)
            for c in cands:  # parity: from the unfilled arena, results and bytes equal seg's
                a.copy_(a0)
                out.zero_()
                run(c, K.OP_FILL)
                torch.cuda.synchronize()
                assert torch.equal(out, ref) and torch.equal(a, filled), f"{c[0]} L={L}"
                run(c, K.OP_CHECKSUM)  # a filled image sums to 0xFFFF -> checksum 0
                torch.cuda.synchronize()
                assert not bool(out.any()), f"{c[0]} L={L} checksum of filled images"
            t = {c[0]: [] for c in cands}
            for _ in range(args.rounds):
                for c in cands:
                    t[c[0]].append(b2b(lambda c=c: run(c), s, reps=20, rounds=1))
            for c in cands:
                ms = float(np.median(t[c[0]]))
                gbs = (n * L + 2 * n) / (ms * 1e-3) / 1e9
                print(f"L={L:6d} {opname:8s} {c[0]:22s} {ms:.4f} ms  {gbs:7.1f} GB/s ({100 * gbs / PEAK:5.1f}%)",
                      flush=True)
        del a, a0, filled, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
