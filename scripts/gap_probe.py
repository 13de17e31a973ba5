#!/usr/bin/env python3
"""Gapped (non-packed) layouts: fixed stride > image length (MSS slots) and
variable images in fixed slots (recvmmsg arenas).  AUTO (seg) by layout; rate
counts image bytes only.  Median back-to-back."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def timed(fn, s, reps=20, rounds=4):
    for _ in range(10):
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
    K = tcpck
    for S, L in ((1536, 1492), (2048, 1492), (128, 96), (160, 96), (256, 96), (96, 64), (1492, 1492)):
        n = (1566572544 // S)
        a = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, S, L, n, seed=3)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ms = timed(lambda: ctx.batch_fixed(K.OP_CHECKSUM, a, S, L, n, out, stream=s), s)
        ms3 = timed(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, S, L, n, out, K.KERNEL_VVSTREAM, 4, stream=s), s)
        print(f"fixed stride {S} len {L}: vvstream (hull) {ms3:.4f} ms image bytes "
              f"{n * L / ms3 / 1e6 / 80:.1f}%  hull {n * S / ms3 / 1e6 / 80:.1f}%", flush=True)
        for shape in (1, 2, 3, 5):
            ms2 = timed(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, S, L, n, out, K.KERNEL_SEG, shape, stream=s), s)
            print(f"fixed stride {S} len {L}: seg shape {shape} {ms2:.4f} ms image bytes "
                  f"{n * L / ms2 / 1e6 / 80:.1f}%  hull {n * S / ms2 / 1e6 / 80:.1f}%", flush=True)
        print(f"fixed stride {S} len {L}: AUTO {ms:.4f} ms  image bytes {n * L / ms / 1e6 / 80:.1f}%  "
              f"hull {n * S / ms / 1e6 / 80:.1f}%", flush=True)
        del a, out
        torch.cuda.empty_cache()
    from synth_np import mixed_layout
    _, ln, _ = mixed_layout(1 << 20, seed=5)
    n = ln.size
    off = np.arange(n, dtype=np.uint64) * 1536
    a = torch.empty(n * 1536, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    K.synth_var(a, d_off, d_ln, 1492, n, seed=3)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    tot = int(ln.astype(np.int64).sum())
    ms = timed(lambda: ctx.batch_var(K.OP_CHECKSUM, a, d_off, d_ln, n, out, total_bytes=tot, stream=s), s)
    print(f"var in 1536-B slots (96/608/1492): AUTO {ms:.4f} ms image bytes {tot / ms / 1e6 / 80:.1f}%  "
          f"hull {n * 1536 / ms / 1e6 / 80:.1f}%", flush=True)


if __name__ == "__main__":
    main()
