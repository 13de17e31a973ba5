#!/usr/bin/env python3
"""C2 FILL (1M x 1492-B images, fixed stride) on rstream by steps in flight
(variant 20: U4, 23: U8, 24: U2) and grid multiple M (param >> 16; 0 = the
policy's, 32 at C2).  Back to back after a clock settle; results and arena checked
against seg's FILL first (FILL is idempotent on the filled arena).

    C2F_MS=8,16,32,64 python scripts/c2_fill_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck as K  # noqa: E402
from xcd_probe import b2b  # noqa: E402


def main():
    ctx = K.Context(0)
    s = torch.cuda.current_stream()
    L, n = 1492, int(os.environ.get("C2F_N", 1 << 20))
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    K.synth_fixed(a, L, L, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(K.OP_FILL, a, L, L, n, ref, K.KERNEL_SEG, 0)
    snap = a.clone()
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ms_ = [int(x) for x in os.environ.get("C2F_MS", "8,16,32,64").split(",")]
    params = [20] + [v | (m << 16) for v in (20, 23, 24) for m in ms_] + [20]
    for p in params:
        fn = (lambda p=p: ctx.batch_fixed_ex(K.OP_FILL, a, L, L, n, out, K.KERNEL_RSTREAM, p, stream=s))
        fn()
        torch.cuda.synchronize()
        assert torch.equal(out, ref) and torch.equal(a, snap), p
        ms = b2b(fn, s, reps=20, rounds=3)
        print(f"C2 fill rstream variant {p & 0xFF} x{p >> 16}: {ms:.4f} ms ({(n * L + 2 * n) / ms / 1e6 / 80:.1f}%)",
              flush=True)


if __name__ == "__main__":
    main()
