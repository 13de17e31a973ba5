#!/usr/bin/env python3
"""C4 (256K x 64 KiB packed): seg's W-wave jumbo shapes (W8/U4, W16/U2, W16/U4)
with the XCD-chunked order, one image per block (M = 0) or grid-stride blocks
at M x the resident grid, against AUTO.  Results compared with AUTO's.  Back
to back, median of rounds."""
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
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    L, n = 65536, 256 << 10
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, n, seed=42)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ms = b2b(lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, ref, stream=s), s)
    print(f"AUTO                 {ms * 1e3:8.1f} us  {(n * L + 2 * n) / ms / 1e6 / 80:5.1f} %", flush=True)
    for shape, name in ((8, "W8/U4"), (9, "W16/U2"), (10, "W16/U4")):
        for m in (0, 2, 4, 8, 16):
            p = shape | (m << 16) | (1 << 24)  # param = SegShape + 1: 8 W8/U4, 9 W16/U2, 10 W16/U4
            ms = b2b(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, tcpck.KERNEL_SEG, p, stream=s), s)
            torch.cuda.synchronize()
            print(f"{name:7s} M{m:<3d}          {ms * 1e3:8.1f} us  {(n * L + 2 * n) / ms / 1e6 / 80:5.1f} %  "
                  f"same: {torch.equal(out, ref)}", flush=True)


if __name__ == "__main__":
    main()
