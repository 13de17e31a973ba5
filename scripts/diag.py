#!/usr/bin/env python3
"""Timing ablations of the stream kernel (include/tcpck_tuning.h variants 4-7):
128-B aligned runs, boundary handling removed, scan removed.  Variants 6/7
produce wrong checksums by design (timing only).  Interleaved rounds in one
process; median GB/s per variant and batch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

VARIANTS = [("stream U4 a16", tcpck.KERNEL_STREAM, 0), ("stream U4 a128", tcpck.KERNEL_STREAM, 4),
            ("stream U2 a128", tcpck.KERNEL_STREAM, 5), ("scan only a128", tcpck.KERNEL_STREAM, 6),
            ("pure a128", tcpck.KERNEL_STREAM, 7), ("span T16", tcpck.KERNEL_SPAN, 16),
            ("seg G64U4", tcpck.KERNEL_SEG, 3), ("seg G16U6", tcpck.KERNEL_SEG, 2),
            ("fstream U4", tcpck.KERNEL_FSTREAM, 0), ("fstream U2", tcpck.KERNEL_FSTREAM, 1 << 16),
            ("fstream U4 T32", tcpck.KERNEL_FSTREAM, 32), ("fstream U4 T8", tcpck.KERNEL_FSTREAM, 8)]


def main():
    ctx = tcpck.Context(0)
    stream = torch.cuda.current_stream()
    arena = torch.empty(17 << 30, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, 65536, 65536, (17 << 30) // 65536, seed=3)
    out = torch.empty(12 << 20, dtype=torch.int16, device="cuda")
    for L, total in ((1492, 1 << 30), (1492, int(1.5 * (1 << 30))), (1492, 16 << 30), (65536, 16 << 30)):
        n = total // L
        times = {v[0]: [] for v in VARIANTS}
        for _ in range(4):
            for name, k, p in VARIANTS:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, k, p, stream=stream)
                fn()
                for _ in range(5):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record(stream)
                    fn()
                    e.record(stream)
                    torch.cuda.synchronize()
                    times[name].append(s.elapsed_time(e))
        algo = n * L + 2 * n
        for name, _, _ in VARIANTS:
            med = float(np.median(times[name]))
            print(f"L={L:5d} {algo / 1e9:6.2f} GB  {name:15s} {med:8.4f} ms  {algo / med / 1e6:7.1f} GB/s "
                  f"({algo / med / 1e6 / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
