#!/usr/bin/env python3
"""Small power-of-two fixed images (stride == len, 32-1024 B): gstream (G = len/16
lanes per image, DPP group sums) against the kernels AUTO used before it
(vvstream FIXED below 512 B, rstream from 512 B), back-to-back launches (the
bench's timing: one HIP-event pair around 20 launches) after a clock settle,
interleaved rounds so that DVFS drift hits every kernel alike.

    python scripts/gstream_probe.py [--bytes 1.5e9] [--lengths 32,64,...] [--ops checksum,fill]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

PEAK = 8000.0  # GB/s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=float, default=1.5e9)
    ap.add_argument("--lengths", default="32,64,128,256,512,1024")
    ap.add_argument("--ops", default="checksum,fill")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--gs", default="", help="gstream params to compare (variant | oversub << 16), e.g. 0x100000,0x200002")
    args = ap.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    ops = {"checksum": tcpck.OP_CHECKSUM, "fill": tcpck.OP_FILL}
    cands = [("auto", None, 0), ("gstream U4", tcpck.KERNEL_GSTREAM, 0),
             ("gstream U4 default loads", tcpck.KERNEL_GSTREAM, 0x80), ("gstream U2", tcpck.KERNEL_GSTREAM, 2),
             ("vvstream policy", tcpck.KERNEL_VVSTREAM, 28), ("rstream policy", tcpck.KERNEL_RSTREAM, 20)]
    if args.gs:
        cands = [("auto", None, 0)] + [(f"gstream#{i} {int(p, 0) & 0xFFFF:#x} x{int(p, 0) >> 16}", tcpck.KERNEL_GSTREAM, int(p, 0))
                                       for i, p in enumerate(args.gs.split(","))]
    for L in [int(x) for x in args.lengths.split(",")]:
        n = int(args.bytes) // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, ref, tcpck.KERNEL_SEG, 0, stream=s)
        for opname in args.ops.split(","):
            op = ops[opname]
            live = [c for c in cands if not (c[1] == tcpck.KERNEL_RSTREAM and L < 512)]

            def run(c):
                if c[1] is None:
                    ctx.batch_fixed(op, a, L, L, n, out, stream=s)
                else:
                    ctx.batch_fixed_ex(op, a, L, L, n, out, c[1], c[2], stream=s)
            if op == tcpck.OP_CHECKSUM:  # parity spot check of every candidate against seg
                for c in live:
                    out.zero_()
                    run(c)
                    torch.cuda.synchronize()
                    assert torch.equal(out, ref), f"{c[0]} L={L} differs from seg"
            t = {c[0]: [] for c in live}
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.25:  # settle the clocks
                run(live[0])
                torch.cuda.synchronize()
            for _ in range(args.rounds):
                for c in live:
                    for _ in range(3):
                        run(c)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(20):
                        run(c)
                    e1.record(s)
                    torch.cuda.synchronize()
                    t[c[0]].append(e0.elapsed_time(e1) / 20)
            for c in live:
                ms = float(np.median(t[c[0]]))
                gbs = (n * L + 2 * n) / (ms * 1e-3) / 1e9
                print(f"L={L:5d} {opname:8s} {c[0]:22s} {ms:.4f} ms  {gbs:7.1f} GB/s ({100 * gbs / PEAK:5.1f}%)",
                      flush=True)
        del a, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
