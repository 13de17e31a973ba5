#!/usr/bin/env python3
"""C5 (8M x 1492 B = 12.5 GB) in one launch vs split into sub-launches of
1M, 2M or 4M images on the same stream (rstream policy, grid by size).  Is the
per-launch size, not the arena size, what costs the large batch ~3 %?"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    N, L = 8 << 20, 1492
    a = torch.empty(N * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, N, seed=42)
    ref = torch.empty(N, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, N, ref, tcpck.KERNEL_SEG, 0)
    out = torch.empty(N, dtype=torch.int16, device="cuda")

    def launch(sub, m):
        for i in range(0, N, sub):
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a[i * L:(i + sub) * L], L, L, sub, out[i:i + sub],
                               tcpck.KERNEL_RSTREAM, 20 | (m << 16), stream=s)

    cases = [(N, 0), (N, 128), (N, 64), (4 << 20, 0), (2 << 20, 0), (1 << 20, 0), (1 << 19, 0)]
    for sub, m in cases:
        out.zero_()
        launch(sub, m)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (sub, m)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        launch(N, 0)
        torch.cuda.synchronize()
    for _ in range(2):
        for sub, m in cases:
            res = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(4):
                    launch(sub, m)
                e1.record(s)
                torch.cuda.synchronize()
                res.append(e0.elapsed_time(e1) / 4)
            ms = float(np.median(res))
            print(f"C5 in launches of {sub >> 20 if sub >= 1 << 20 else sub / (1 << 20)}M images"
                  f"{' (M=' + str(m) + ')' if m else ''}: {ms:.4f} ms ({(N * L + 2 * N) / ms / 1e6 / 80:.1f}%)",
                  flush=True)


if __name__ == "__main__":
    main()
