#!/usr/bin/env python3
"""What a second batch changes (round 5): C2 / C3 CHECKSUM launched back to
back over ONE arena, over 2 or 4 identical arenas taken in turn (separate
allocations, or 2 halves of one allocation), and over one arena with a 512-MB
read of another buffer between steps (evicts the 256-MB Infinity Cache, few
pages).  If one arena is faster because the next step finds the previous
step's lines in the Infinity Cache, the flush removes it like extra arenas
do; if it is address translation (more pages in use), extra arenas cost and
the flush does not.

Run under `rocprofv3 --kernel-trace`: every variant begins with a synth
launch (a phase boundary for scripts/bench_trace_summary.py) and the kernel
durations there exclude the flush.  Also prints HIP-event step times (the
flush included for that variant)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402


def timed(fn, s, steps=40):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    flush = torch.ones(512 << 20, dtype=torch.uint8, device="cuda")
    sink = torch.empty(1, dtype=torch.int64, device="cuda")
    for case in ("c2", "c3"):
        if case == "c2":
            n, L = 1 << 20, 1492
            size = n * L
            gen = lambda a: tcpck.synth_fixed(a, L, L, n, seed=42, stream=s)
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            run = lambda a: ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out, stream=s)
            img = size
        else:
            n = 4 << 20
            off, ln, size = synth_np.mixed_layout(n, seed=42)
            d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            gen = lambda a: tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42, stream=s)
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            img = int(ln.astype(np.int64).sum())
            kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
            run = lambda a: ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, **kw)
        for variant in ("1 arena", "2 arenas", "4 arenas", "2 halves of one allocation", "1 arena + flush"):
            if variant == "2 halves of one allocation":
                big = torch.empty(2 * size + 256, dtype=torch.uint8, device="cuda")
                arenas = [big[:size], big[size + 128:2 * size + 128]]  # 128-B apart: even, line-aligned
            else:
                k = {"1 arena": 1, "2 arenas": 2, "4 arenas": 4, "1 arena + flush": 1}[variant]
                arenas = [torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(k)]
            for a in arenas:
                gen(a)  # (the first synth launch opens the phase in a kernel trace)
            torch.cuda.synchronize()
            turn = [0]

            def step():
                run(arenas[turn[0] % len(arenas)])
                turn[0] += 1
                if variant.endswith("flush"):
                    flush.view(torch.int64).sum()
            ms = timed(step, s)
            print(f"{case} {variant:28s} {ms * 1e3:7.1f} us per step (HIP events{', flush included' if 'flush' in variant else ''})"
                  f"  {(img + 2 * n) / ms / 1e6 / 80:5.1f} %", flush=True)
            del arenas
            if variant == "2 halves of one allocation":
                del big
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
