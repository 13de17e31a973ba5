#!/usr/bin/env python3
"""C2 CHECKSUM on rstream: the grid (M x the resident grid) re-measured on the
round-4 kernel, next to AUTO (M = 32 at C2's size, profiles/r01/oversub_c2c3.log).
Interleaved rounds of 20 back-to-back launches; results compared with AUTO's."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def timed(fn, s, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    K = tcpck
    L, n = 1492, 1 << 20
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    K.synth_fixed(a, L, L, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(K.OP_CHECKSUM, a, L, L, n, ref)
    fns, outs = {}, {}
    for label, p in [("auto", None)] + [(f"M{m}", 20 | (m << 16)) for m in (8, 16, 24, 32, 48, 64, 96, 128)]:
        o = torch.empty(n, dtype=torch.int16, device="cuda")
        outs[label] = o
        fns[label] = ((lambda o=o: ctx.batch_fixed(K.OP_CHECKSUM, a, L, L, n, o, stream=s)) if p is None else
                      (lambda o=o, p=p: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, o, K.KERNEL_RSTREAM, p,
                                                           stream=s)))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for f in fns.values():
            f()
        torch.cuda.synchronize()
    times = {k: [] for k in fns}
    for _ in range(9):
        for k, f in fns.items():
            times[k].append(timed(f, s))
    algo = n * L + 2 * n
    for k in fns:
        ms = float(np.median(times[k]))
        print(f"C2 CHECKSUM rstream {k:5s} {ms * 1e3:7.1f} us  {100 * algo / (ms * 1e-3) / 8e12:5.1f} %  "
              f"{'ok' if torch.equal(outs[k], ref) else 'DIFFERS'}", flush=True)


if __name__ == "__main__":
    main()
