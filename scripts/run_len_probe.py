#!/usr/bin/env python3
"""rstream grid for packed images of 2-4 KiB (AUTO's rstream range ends at
4 KiB): the policy's grid (runs of 4-8 KiB, a fractional number of images per
wave) against one image per wave (M = 255 caps at the image count) and M = 16
/ 32, at C2's byte size.  Companion of scripts/pow2_probe.py."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=3):
    for _ in range(5):
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
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    total = 1564475392
    for L in (2600, 3000, 3500, 4000, 4096):
        n = total // L
        arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(arena, L, L, n, seed=42, stream=s)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        alg = n * L + 2 * n
        row = []
        for label, p in (("AUTO", None), ("M 16", 20 | (16 << 16)), ("M 32", 20 | (32 << 16)), ("M 48", 20 | (48 << 16)),
                         ("1/wave", 20 | (255 << 16))):
            if p is None:
                fn = lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s)
            else:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, kernel=tcpck.KERNEL_RSTREAM,
                                                param=p, stream=s)
            ms = b2b(fn, s)
            row.append(f"{label} {alg / ms / 1e6 / 80:5.1f} %")
        print(f"L {L:5d} x {n:7d}  (policy: {n / 262144:4.2f} images per wave)  " + "   ".join(row), flush=True)
        del arena


if __name__ == "__main__":
    main()
