#!/usr/bin/env python3
"""Kernel choice vs image size: the data behind run_fixed / run_var's AUTO policy.

For packed batches of ~1.5 GB with one image length L (fixed stride, and the
same bytes as a variable layout) and for a few length mixes, times every
applicable kernel (median of interleaved HIP-event launches) after checking
its results against the seg kernel.  Prints one line per (layout, kernel).

    python scripts/policy_sweep.py [--bytes 1564475392] [--reps 6]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

FIXED_L = [16, 32, 64, 96, 128, 192, 256, 320, 384, 448, 512, 640, 768, 1024, 1492, 2048, 3000, 4096]
MIXES = {"32/1492": (0, 1460), "96/608/1492": (64, 576, 1460), "32..1492": (0, 32, 64, 128, 256, 512, 1024, 1460),
         "608/1492": (576, 1460)}


def time_runs(runs, reps, stream, per=10):
    """Median over `reps` rounds of `per` back-to-back launches (interleaved by round)."""
    t = {r[0]: [] for r in runs}
    for label, fn in runs:  # settle
        for _ in range(per):
            fn()
    torch.cuda.synchronize()
    for _ in range(reps):
        for label, fn in runs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(per):
                fn()
            b.record(stream)
            torch.cuda.synchronize()
            t[label].append(a.elapsed_time(b) / per)
    return {k: float(np.median(v)) for k, v in t.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--bytes", type=int, default=1564475392)
    p.add_argument("--reps", type=int, default=6)
    p.add_argument("--no-mixes", action="store_true")
    p.add_argument("--no-fixed", action="store_true")
    p.add_argument("--lengths", default="", help="comma list of fixed image lengths (default: all)")
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    fixed_l = [int(x) for x in args.lengths.split(",")] if args.lengths else FIXED_L
    for L in ([] if args.no_fixed else fixed_l):
        n = args.bytes // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, L, L, n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, ref, K.KERNEL_SEG, 0)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        off = torch.arange(n, dtype=torch.int64, device="cuda") * L
        ln = torch.full((n,), L, dtype=torch.int32, device="cuda")
        cand = [("auto", lambda: ctx.batch_fixed(K.OP_CHECKSUM, a, L, L, n, out, stream=s)),
                ("seg", lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_SEG, 0, stream=s)),
                ("rstream 20", lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_RSTREAM, 20,
                                                          stream=s)),
                ("vvstream fix 28", lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_VVSTREAM, 28,
                                                               stream=s)),
                ("gstream 0", lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_GSTREAM, 0,
                                                         stream=s)),
                ("var vvstream 28", lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, off, ln, n, out, K.KERNEL_VVSTREAM, 28,
                                                             packed=True, total_bytes=n * L, stream=s))]
        runs = []
        for label, fn in cand:
            try:
                out.zero_()
                fn()
                torch.cuda.synchronize()
            except tcpck.TcpckError:
                continue
            if not torch.equal(out, ref):
                print(f"L={L} {label}: WRONG RESULTS", flush=True)
                continue
            runs.append((label, fn))
        for label, ms in time_runs(runs, args.reps, s).items():
            gbs = (n * L + 2 * n) / (ms * 1e-3) / 1e9
            print(f"fixed L={L:5d} {label:14s} {ms:8.4f} ms {gbs:7.1f} GB/s ({gbs / 80:5.1f}%)", flush=True)
        del a, ref, out, off, ln
        torch.cuda.empty_cache()
    for name, payloads in ({} if args.no_mixes else MIXES).items():
        rng = np.random.default_rng(1)
        mean = np.mean(payloads) + 32
        n = int(args.bytes / mean)
        ln_np = (np.asarray(payloads, np.uint32)[rng.integers(0, len(payloads), n)] + 32).astype(np.uint32)
        off_np = np.zeros(n, np.uint64)
        off_np[1:] = np.cumsum(ln_np[:-1].astype(np.uint64))
        total = int(off_np[-1] + ln_np[-1])
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        off, ln = torch.from_numpy(off_np).cuda(), torch.from_numpy(ln_np).cuda()
        K.synth_var(a, off, ln, int(ln_np.max()), n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(K.OP_CHECKSUM, a, off, ln, n, ref, K.KERNEL_SEG, 0)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        lay = dict(total_bytes=total, min_len=int(ln_np.min()), max_len=int(ln_np.max()), packed=True)
        cand = [("auto", lambda: ctx.batch_var(K.OP_CHECKSUM, a, off, ln, n, out, stream=s, **lay)),
                ("seg", lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, off, ln, n, out, K.KERNEL_SEG, 0, stream=s, **lay)),
                ("vvstream 28", lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, off, ln, n, out, K.KERNEL_VVSTREAM, 28,
                                                         stream=s, **lay)),
                ("sstream 0", lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, off, ln, n, out, K.KERNEL_SSTREAM, 0,
                                                       stream=s, sorted=True, **lay))]
        runs = []
        for label, fn in cand:
            out.zero_()
            fn()
            torch.cuda.synchronize()
            if not torch.equal(out, ref):
                print(f"mix {name} {label}: WRONG RESULTS", flush=True)
                continue
            runs.append((label, fn))
        for label, ms in time_runs(runs, args.reps, s).items():
            gbs = (total + 2 * n) / (ms * 1e-3) / 1e9
            print(f"mix {name:12s} {label:14s} {ms:8.4f} ms {gbs:7.1f} GB/s ({gbs / 80:5.1f}%)", flush=True)
        del a, ref, out, off, ln
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
