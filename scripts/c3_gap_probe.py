#!/usr/bin/env python3
"""Where C3's gap to C2 comes from: the same bytes through the packed
variable path (offsets + lengths, vvstream) and through the fixed paths (no
descriptors: vvstream FIXED, rstream), at 736-B images (C3's mean, 4M
images), and C3's own mix.  Back to back, median of rounds, % of the roof in
image bytes + results."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

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
    from synth_np import mixed_layout
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    n = 4 << 20
    for name, L in (("736 B x 4M", 736), ("C3 mix", None)):
        if L:
            off = np.arange(n, dtype=np.uint64) * np.uint64(L)
            ln = np.full(n, L, np.uint32)
            total = n * L
        else:
            off, ln, total = mixed_layout(n, seed=42)
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        img = int(ln.astype(np.int64).sum())
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
        runs = [("var AUTO (vvstream)", lambda: ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, **kw))]
        for m in (16, 32, 64):
            runs.append((f"var vvstream M{m}", lambda m=m: ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out,
                                                                         8, 28 | (m << 16), **kw)))
        if L:
            runs += [("fixed AUTO (rstream)", lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out, stream=s)),
                     ("fixed vvstream", lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, 8, 28,
                                                                   stream=s))]
        for label, fn in runs:
            ms = b2b(fn, s)
            print(f"{name:12s} {label:22s} {ms * 1e3:8.1f} us  {(img + 2 * n) / ms / 1e6 / 80:5.1f} % of the roof",
                  flush=True)
        del a


if __name__ == "__main__":
    main()
