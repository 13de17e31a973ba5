#!/usr/bin/env python3
"""Byte runs across image edges (experimental bstream) against AUTO on packed
fixed images: C4 (256K x 64 KiB), 16 KiB, 9000 B, C2's 1492 B.  Run sizes
4-32 KiB, 4 / 8 steps in flight.  Results compared with AUTO's.  Back to
back, median of rounds, % of the roof in image bytes + results."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=10, rounds=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
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
    for L, n in ((65536, 256 << 10), (16384, 1 << 20), (9000, (1536 << 20) // 9000), (1492, 1 << 20)):
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ws = torch.zeros(n, dtype=torch.int64, device="cuda")
        ctx.set_debug(ws)
        ms = b2b(lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, ref, stream=s), s)
        print(f"{L:6d} B x {n}: AUTO              {ms * 1e3:8.1f} us  {(n * L + 2 * n) / ms / 1e6 / 80:5.1f} %",
              flush=True)
        for v in (12, 13, 14, 15, 256 | 13, 256 | 14):
            ms = b2b(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, tcpck.KERNEL_BSTREAM, v,
                                                stream=s), s)
            torch.cuda.synchronize()
            same = torch.equal(out, ref) and not ws.any().item()
            print(f"{L:6d} B x {n}: bstream {1 << (v & 31):6d} B U{8 if v & 256 else 4} {ms * 1e3:8.1f} us  "
                  f"{(n * L + 2 * n) / ms / 1e6 / 80:5.1f} %  same: {same}", flush=True)
        ctx.set_debug(None)
        del a, ws


if __name__ == "__main__":
    main()
