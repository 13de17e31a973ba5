#!/usr/bin/env python3
"""C3 FILL (send path of the mixed batch) on vvstream by steps in flight (U4 / U8)
and grid multiple M, against the policy (variant 28: U8, M by size = 32 at C3).
Back to back after a clock settle; FILL is idempotent on the filled arena, and
every candidate's results and arena are checked against seg's FILL first.

    C3F_MS=8,16,32,64 C3F_N=4194304 python scripts/c3_fill_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck as K  # noqa: E402
from synth_np import mixed_layout  # noqa: E402
from xcd_probe import b2b  # noqa: E402


def main():
    ctx = K.Context(0)
    s = torch.cuda.current_stream()
    off, ln, total = mixed_layout(int(os.environ.get("C3F_N", 4 << 20)), seed=42)
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    K.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(K.OP_FILL, a, d_off, d_ln, n, ref, K.KERNEL_SEG, 0)
    snap = a.clone()
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ms_ = [int(x) for x in os.environ.get("C3F_MS", "8,16,32,64").split(",")]
    params = [28] + [v | (m << 16) for v in (26, 27) for m in ms_] + [28]
    for p in params:
        fn = (lambda p=p: ctx.batch_var_ex(K.OP_FILL, a, d_off, d_ln, n, out, K.KERNEL_VVSTREAM, p, packed=True,
                                           total_bytes=total, stream=s))
        fn()
        torch.cuda.synchronize()
        assert torch.equal(out, ref) and torch.equal(a, snap), p
        ms = b2b(fn, s, reps=20, rounds=3)
        print(f"C3 fill vvstream variant {p & 0xFF} x{p >> 16}: {ms:.4f} ms ({(total + 2 * n) / ms / 1e6 / 80:.1f}%)",
              flush=True)


if __name__ == "__main__":
    main()
