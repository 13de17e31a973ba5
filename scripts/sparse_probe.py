#!/usr/bin/env python3
"""Sparse read patterns: fixed slots (stride S, image L) at equal density and
different block sizes, through sstream (reads only the images' chunks) -- does
the rate depend on the density or on the contiguous block size?  % of the 8 TB/s
roof in image bytes (= the lines read, L a multiple of 128)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from slot_probe import PEAK, timed  # noqa: E402

CASES = [(256, 128), (512, 256), (1024, 512), (2048, 1024), (4096, 2048), (8192, 4096), (16384, 8192),
         (65536, 32768), (1024, 256), (2048, 512), (4096, 1024), (8192, 2048), (16384, 4096), (2048, 1536),
         (4096, 3072), (8192, 6144), (1024, 1024), (4096, 4096)]


VARIANTS = [int(x) for x in os.environ.get("SP_VARIANTS", "0,4,8").split(",")]
MS = [int(x) for x in os.environ.get("SP_MS", "4,8,16,32").split(",")]


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    arena = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")
    arena.fill_(7)
    for S, L in CASES:
        n = (3 << 30) // S
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        row = []
        for v in VARIANTS:
            for m in MS:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, S, L, n, out, tcpck.KERNEL_SSTREAM,  # noqa
                                                v | (m << 16), stream=s)
                ms = timed(fn, s)
                row.append(f"v{v}/M{m} {n * L / (ms * 1e-3) / PEAK * 100:5.1f}")
        print(f"slot {S:6d} image {L:6d} density {L / S:4.2f}  " + "  ".join(row), flush=True)
        del out


if __name__ == "__main__":
    main()
