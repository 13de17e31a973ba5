#!/usr/bin/env python3
"""C4 rotation multiplier sweep (seg W16, XCD order, SegArgs::rot = param bits
8-15): image k's chunk walk starts at chunk ((k rot) mod 64) 64.  Three
interleaved passes over the multipliers, median per multiplier; results
compared with rot 0.  Optional argv[1]: image length (default 65536)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=10, rounds=3):
    for _ in range(3):
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
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    n = (16 << 30) // L
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=42, stream=s)
    alg = n * L + 2 * n
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s)
        torch.cuda.synchronize()
    ref = out.clone()
    rots = [0, 1, 3, 5, 7, 9, 11, 13, 17, 21, 25, 27, 29, 31, 33, 37, 41, 45, 49, 53, 57, 61, 63]
    times = {r: [] for r in rots}
    same = True
    for _ in range(3):
        for r in rots:
            p = (1 << 24) | (r << 8)
            ms = b2b(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, kernel=tcpck.KERNEL_SEG,
                                                param=p, stream=s), s)
            times[r].append(ms)
            same = same and torch.equal(out, ref)
    for r in rots:
        ms = float(np.median(times[r]))
        print(f"L {L:6d}  rot {r:3d}  {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof  "
              f"(passes {', '.join(f'{t * 1e3:.0f}' for t in times[r])})", flush=True)
    print("results identical:", same, flush=True)


if __name__ == "__main__":
    main()
