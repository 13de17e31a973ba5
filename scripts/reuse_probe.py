#!/usr/bin/env python3
"""Does the C2 rate depend on cache reuse across launches?  The MI355X's
256 MB MALL sits behind the L2s and FETCH_SIZE does not see its hits.  C2
(1M x 1492 B = 1.57 GB) launched back to back over the same arena, and
rotating over 2, 4 and 8 distinct arenas (3.1-12.5 GB): a stream that gained
from lines left by the previous launch would slow down when rotating."""
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
    n, L = 1 << 20, 1492
    arenas = []
    for i in range(8):
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42, first_index=i * n)
        arenas.append(a)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for a in arenas:
            ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out, stream=s)
        torch.cuda.synchronize()
    for _ in range(2):
        for k in (1, 2, 4, 8, 1):
            reps = 24
            res = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for r in range(reps):
                    ctx.batch_fixed(tcpck.OP_CHECKSUM, arenas[r % k], L, L, n, out, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                res.append(e0.elapsed_time(e1) / reps)
            ms = float(np.median(res))
            print(f"C2 rotating over {k} arena(s) ({k * n * L / 1e9:5.2f} GB): {ms * 1e3:7.1f} us "
                  f"({(n * L + 2 * n) / ms / 1e6 / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
