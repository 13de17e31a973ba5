#!/usr/bin/env python3
"""Kernel time vs batch size: separates fixed per-launch cost (ramp-up, tail)
from steady-state bandwidth.  Fits t = t0 + bytes / BW over batch sizes.

    python scripts/scaling.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def time_launch(fn, reps=15):
    stream = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        fn()
        e.record(stream)
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts)), float(np.min(ts))


def main():
    ctx = tcpck.Context(0, probe=True)
    stream = torch.cuda.current_stream()
    max_bytes = 24 << 30
    arena = torch.empty(max_bytes, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, 65536, 65536, max_bytes // 65536, seed=1)
    out = torch.empty(16 << 20, dtype=torch.int16, device="cuda")
    tiny = torch.zeros(1 << 12, dtype=torch.uint8, device="cuda")
    print("empty-ish launch (1 image):", time_launch(lambda: ctx.batch_fixed_ex(
        tcpck.OP_CHECKSUM, tiny, 1492, 1492, 1, out, tcpck.KERNEL_SEG, 2, stream=stream)), flush=True)
    cases = [("rstream 1492", 1492, tcpck.KERNEL_RSTREAM, 10), ("vvstream 1492", 1492, tcpck.KERNEL_VVSTREAM, 4),
             ("seg G16 1492", 1492, tcpck.KERNEL_SEG, 2), ("seg G64U4 64K", 65536, tcpck.KERNEL_SEG, 3),
             ("vvstream 96", 96, tcpck.KERNEL_VVSTREAM, 4)]
    for name, L, k, p in cases:
        xs, ys = [], []
        for gb in (0.25, 0.5, 1, 1.5, 2, 4, 8, 16):
            n = int(gb * (1 << 30)) // L
            if n * L > max_bytes or n > out.numel():
                continue
            med, mn = time_launch(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, k, p,
                                                             stream=stream))
            algo = n * L + 2 * n
            xs.append(algo)
            ys.append(med * 1e-3)
            print(f"{name:16s} {algo / 1e9:7.3f} GB  median {med:8.4f} ms  {algo / med / 1e6:7.1f} GB/s  "
                  f"best {algo / mn / 1e6:7.1f}", flush=True)
        A = np.vstack([np.ones(len(xs)), np.array(xs)]).T
        (t0, inv_bw), *_ = np.linalg.lstsq(A, np.array(ys), rcond=None)
        print(f"{name:16s} fit: t0 = {t0 * 1e6:6.1f} us, steady BW = {1 / inv_bw / 1e9:7.1f} GB/s "
              f"({1 / inv_bw / 8e12 * 100:.1f}% of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
