#!/usr/bin/env python3
"""FILL on vvstream with every step read with the default cache policy (variant
flag 32, "keep") against the policy's nt reads (variant 28): fixed images below
512 B and packed variable mixes, back-to-back launches after a clock settle.

    python scripts/keep_probe.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

PEAK = 8000.0


def timeit(run, rounds=3):
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(rounds):
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20)
    return float(np.median(ts))


def report(name, ms, nbytes):
    gbs = nbytes / (ms * 1e-3) / 1e9
    print(f"{name:44s} {ms:.4f} ms {gbs:7.1f} GB/s ({100 * gbs / PEAK:5.1f}%)", flush=True)


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    target = 1.5e9
    for L in (96, 160, 192, 320, 480):
        n = int(target) // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.25:
            ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, out, tcpck.KERNEL_VVSTREAM, 28, stream=s)
            torch.cuda.synchronize()
        for p in (28, 60, 28, 60):
            ms = timeit(lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, out, tcpck.KERNEL_VVSTREAM, p, stream=s))
            report(f"fixed L={L} fill vvstream {p}", ms, n * L + 2 * n)
        ms = timeit(lambda: ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, out, stream=s))
        report(f"fixed L={L} fill auto", ms, n * L + 2 * n)
        del a, out
    from synth_np import mixed_layout
    for name, payloads in (("mix 32/64/96+32", (32, 64, 96)), ("mix 64/96/224+32", (64, 96, 224)),
                           ("C3 mix", (64, 576, 1460))):
        count = int(target) // (32 + int(np.mean(payloads)))
        rng = np.random.default_rng(42)
        ln = (np.asarray(payloads, np.int64)[rng.integers(0, len(payloads), count)] + 32).astype(np.uint32)
        if name == "C3 mix":
            off, ln, total = mixed_layout(count, seed=42)
        else:
            off = np.zeros(count, np.uint64)
            off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
            total = int(ln.astype(np.int64).sum())
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        lmin, lmax = int(ln.min()), int(ln.max())
        for p in (28, 60, 28, 60):
            ms = timeit(lambda: ctx.batch_var_ex(tcpck.OP_FILL, a, d_off, d_ln, count, out, tcpck.KERNEL_VVSTREAM, p,
                                                 packed=True, total_bytes=total, stream=s))
            report(f"{name} fill vvstream {p}", ms, total + 2 * count)
        ms = timeit(lambda: ctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, count, out, total_bytes=total,
                                          min_len=lmin, max_len=lmax, packed=True, stream=s))
        report(f"{name} fill auto", ms, total + 2 * count)
        del a, out, d_off, d_ln


if __name__ == "__main__":
    main()
