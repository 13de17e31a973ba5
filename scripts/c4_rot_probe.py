#!/usr/bin/env python3
"""C4 (256K x 64-KiB packed jumbo images, seg W16: one image per 1024-thread
block): does reading every image from the same offset at the same time cost
(the blocks in flight hold consecutive images, 64 KiB apart)?  The W-wave
shapes can start image k's chunk walk at chunk ((k rot) mod (n / 64)) 64 and
wrap (SegArgs::rot = seg param bits 8-15).  CHECKSUM and
FILL timed against AUTO, results (and FILL's fields) compared.  Back-to-back
launches, median of 5 rounds of 10."""
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
    W16 = 9  # seg shape kShapeW16 + 1
    cases = [(65536, 256 << 10), (32768, 512 << 10), (16384, 1 << 20)]
    for L, n in cases:
        arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(arena, L, L, n, seed=42, stream=s)
        alg = n * L + 2 * n
        res = {}
        forms = [("AUTO", None), ("seg W-shape, XCD order", 1 << 24), ("+ rot 1", (1 << 24) | (1 << 8)),
                 ("+ rot 37", (1 << 24) | (37 << 8)), ("+ rot 29", (1 << 24) | (29 << 8)), ("rot 1, default order", 1 << 8)]
        for label, p in forms:
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            if p is None:
                fn = lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s)
            else:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, kernel=tcpck.KERNEL_SEG,
                                                param=p, stream=s)
            ms = b2b(fn, s)
            torch.cuda.synchronize()
            res[label] = out.clone()
            print(f"L {L:6d} x {n:7d}  {label:24s} {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof",
                  flush=True)
        ref = res["AUTO"]
        print(f"L {L:6d}  results identical: {all(torch.equal(v, ref) for v in res.values())}", flush=True)
        if L == 65536:  # FILL: AUTO (seg W16 in-stream) against the rotated form
            fres = {}
            for label, p in (("FILL AUTO", None), ("FILL + rot 1", (1 << 24) | (1 << 8)), ("FILL + rot 29", (1 << 24) | (29 << 8))):
                out = torch.empty(n, dtype=torch.int16, device="cuda")
                if p is None:
                    fn = lambda: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, out, stream=s)
                else:
                    fn = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, kernel=tcpck.KERNEL_SEG,
                                                    param=p, stream=s)
                ms = b2b(fn, s)
                torch.cuda.synchronize()
                fres[label] = (out.clone(), arena[28::L].clone(), arena[29::L].clone())
                print(f"L {L:6d} x {n:7d}  {label:24s} {ms * 1e3:8.1f} us  {(alg + 2 * n) / ms / 1e6 / 80:5.1f} % of "
                      f"the roof", flush=True)
            a, b = fres["FILL AUTO"], fres["FILL + rot 1"]
            print("FILL results and fields identical:", all(torch.equal(x, y) for x, y in zip(a, b)), flush=True)
        del arena


if __name__ == "__main__":
    main()
