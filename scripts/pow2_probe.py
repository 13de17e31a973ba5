#!/usr/bin/env python3
"""rstream on packed power-of-two images (512 B - 4 KiB go to rstream under
AUTO): does the run length matter when every run starts at a multiple of a
power of two?  Each wave streams per_wave = count / (8 x 256 x 4 x M) images;
this sweeps the grid multiplier M (param bits 16-23) for 1024 / 1492 / 2048 /
4096-B images at C2's byte size (1.5 GB) and prints the run length, against
AUTO.  Back-to-back launches, median of 3 rounds of 20."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=3):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
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
    for L in (4096, 2048, 1024, 1492):
        n = total // L
        arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(arena, L, L, n, seed=42, stream=s)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        alg = n * L + 2 * n
        ms = b2b(lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s), s)
        ref = out.clone()
        print(f"L {L:5d} x {n:7d}  AUTO          {ms * 1e3:7.1f} us  {alg / ms / 1e6 / 80:5.1f} %", flush=True)
        for M in (3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40, 48, 64):
            p = 20 | (M << 16)
            ms = b2b(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, kernel=tcpck.KERNEL_RSTREAM,
                                                param=p, stream=s), s)
            waves = min(8 * 256 * 4 * M, n)
            per = n / waves
            ok = torch.equal(out, ref)
            print(f"L {L:5d} x {n:7d}  M {M:3d} ({per:5.2f} images = {per * L / 1024:6.2f} KiB per run)  "
                  f"{ms * 1e3:7.1f} us  {alg / ms / 1e6 / 80:5.1f} %  {'' if ok else 'MISMATCH'}", flush=True)
        del arena


if __name__ == "__main__":
    main()
