#!/usr/bin/env python3
"""FILL on packed fixed images: the stream with in-place 2-B field stores
(rstream policy, variant 20) against the stream writing only the results
followed by a pass that rewrites each field's 64-B block whole (variant 25),
with CHECKSUM for reference.  1.5 GB per size, median of back-to-back rounds.
(The same pass after vvstream's stream on C3 and on 96-384 B fixed images
lost 12-40 %, profiles/r02/fill_defer_vv_probe.log: the pass's cost grows with
the image count, and there are many small images.  After sstream in fixed
slots it was equal or slower, profiles/r02/fill_defer_slots_probe.log.)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=5):
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
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [512, 1024, 1492, 2048, 4096]
    for L in sizes:
        n = (1492 << 20) // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        R = tcpck.KERNEL_RSTREAM
        runs = [("CHECKSUM", lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, R, 20, stream=s)),
                ("FILL in-stream", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, out, R, 20, stream=s)),
                ("FILL + block pass", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, out, R, 25, stream=s))]
        if L > 4096:  # jumbo: AUTO (seg's W-wave kernels from 24 KiB) for comparison
            runs.append(("FILL AUTO", lambda: ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, out, stream=s)))
        for name, fn in runs:
            ms = b2b(fn, s)
            print(f"{L:5d} B x {n}: {name:18s} {ms * 1e3:8.1f} us  {(n * L + 2 * n) / ms / 1e6 / 80:5.1f} % of the roof",
                  flush=True)
        del a


if __name__ == "__main__":
    main()
