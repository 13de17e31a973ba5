#!/usr/bin/env python3
"""C3 CHECKSUM on vvstream: steps in flight (U4 vs U8) and grid size, re-measured
on the round-4 kernel (probe library; round 1 chose U8 at 32x when the kernel was
slower: profiles/r01/oversub_c2c3.log).  Interleaved rounds of 20 back-to-back
launches, results compared with AUTO's."""
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
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    rng = np.random.default_rng(42)
    n = 1 << 22
    ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(ln.sum())
    arena = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    K.synth_var(arena, d_off, d_len, int(ln.max()), n, seed=42)
    hints = dict(total_bytes=total, min_len=int(ln.min()), max_len=int(ln.max()), packed=True)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_var(K.OP_CHECKSUM, arena, d_off, d_len, n, ref, **hints)
    cases = [("auto", None)]
    for u, v in (("U4", 2), ("U8", 3)):
        for m in (16, 24, 32, 48, 64):
            cases.append((f"{u} x{m}", v | 8 | 16 | (m << 16)))
    outs = {}
    fns = {}
    for label, p in cases:
        o = torch.empty(n, dtype=torch.int16, device="cuda")
        outs[label] = o
        if p is None:
            fns[label] = (lambda o=o: ctx.batch_var(K.OP_CHECKSUM, arena, d_off, d_len, n, o, stream=s, **hints))
        else:
            fns[label] = (lambda o=o, p=p: ctx.batch_var_ex(K.OP_CHECKSUM, arena, d_off, d_len, n, o,
                                                           K.KERNEL_VVSTREAM, p, stream=s, **hints))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for f in fns.values():
            f()
        torch.cuda.synchronize()
    times = {k: [] for k in fns}
    for _ in range(7):
        for k, f in fns.items():
            times[k].append(timed(f, s))
    algo = total + 2 * n
    for k in fns:
        ms = float(np.median(times[k]))
        ok = torch.equal(outs[k], ref)
        print(f"C3 CHECKSUM {k:8s} {ms * 1e3:7.1f} us  {100 * algo / (ms * 1e-3) / 8e12:5.1f} %  "
              f"{'ok' if ok else 'DIFFERS'}", flush=True)


if __name__ == "__main__":
    main()
