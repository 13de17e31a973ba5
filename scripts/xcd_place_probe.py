#!/usr/bin/env python3
"""Placement sensitivity of the XCD-aware run order: the C2 batch (1M x 1492 B)
at several offsets inside one 4 GiB allocation, rstream variant 10 (default
block order) vs 14 (XCD order), 32x grid.  Median of back-to-back rounds."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=5):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1) / reps)
    return float(np.median(t))


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    n, L = 1 << 20, 1492
    big = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    print(f"base address {big.data_ptr():#x}", flush=True)
    for off in (0, 4096, 1 << 20, 96 << 20, (256 << 20) + 128, 1 << 30, (1 << 31) + (3 << 20)):
        a = big[off:off + n * L]
        K.synth_fixed(a, L, L, n, seed=42)
        res = {}
        for v in (10, 14):
            p = v | (32 << 16)
            res[v] = b2b(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_RSTREAM, p, stream=s), s)
        for v in (0x3800, 0x3801):
            res[v] = b2b(lambda: ctx.diag_stream(v, a, n * L, out, stream=s), s)
        pct = {v: (n * L + 2 * n) / ms / 1e6 / 80 for v, ms in res.items()}
        print(f"offset {off:>11d}: rstream default {pct[10]:.1f}%  xcd {pct[14]:.1f}%   "
              f"bare x32 default {pct[0x3800]:.1f}%  xcd {pct[0x3801]:.1f}%", flush=True)


if __name__ == "__main__":
    main()
