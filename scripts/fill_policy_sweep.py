#!/usr/bin/env python3
"""FILL: AUTO's choice against every applicable form, by image length (round 4).

Round 3 changed FILL's costs (write-through field passes, the update form), and
round 4's line-form probe found one stale AUTO choice (1-KiB FILL on gstream);
this sweep re-checks the rest.  Packed fixed batches of ~1.5 GB of one image
length, and packed offset lists of a few length mixes; each form is timed back
to back (median of rounds after a settle) and its arena compared with AUTO's.

    python scripts/fill_policy_sweep.py [--lengths 32,64,...] [--no-mixes]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402

FIXED_L = [32, 48, 64, 96, 128, 192, 256, 320, 384, 448, 512, 640, 768, 1024, 1492, 2048]
MIXES = {"96/608/1492": (64, 576, 1460), "608/1492": (576, 1460), "32..1492": (0, 32, 64, 128, 256, 512, 1024, 1460),
         "64/1460": (32, 1428)}
UPD = 1 << 28  # TCPCK_PARAM_FILL_UPDATE


def b2b(fn, s, reps=10, rounds=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:
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


def run_cases(label, cases, arena, want, algo, s):
    best = None
    for name, fn in cases:
        try:
            fn()
            torch.cuda.synchronize()
        except tcpck.TcpckError:
            print(f"{label:14s} {name:14s} rejected", flush=True)
            arena.copy_(want)
            continue
        same = torch.equal(arena, want)
        arena.copy_(want)
        ms = b2b(fn, s)
        arena.copy_(want)
        frac = algo / (ms * 1e-3) / 8e12
        print(f"{label:14s} {name:14s} {ms * 1e3:8.1f} us  {100 * frac:5.1f} %  {'ok' if same else 'ARENA DIFFERS'}",
              flush=True)
        if name != "auto" and same and (best is None or ms < best[1]):
            best = (name, ms)
    return best


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--bytes", type=int, default=1564475392)
    p.add_argument("--lengths", default="")
    p.add_argument("--no-mixes", action="store_true")
    p.add_argument("--no-fixed", action="store_true")
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    lengths = [int(x) for x in args.lengths.split(",")] if args.lengths else FIXED_L
    for L in ([] if args.no_fixed else lengths):
        n = args.bytes // L
        arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(arena, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed(K.OP_FILL, arena, L, L, n, out, stream=s)
        torch.cuda.synchronize()
        want = arena.clone()

        def ex(kernel, param):
            return lambda: ctx.batch_fixed_ex(K.OP_FILL, arena, L, L, n, out, kernel, param, stream=s)
        cases = [("auto", lambda: ctx.batch_fixed(K.OP_FILL, arena, L, L, n, out, stream=s)),
                 ("seg", ex(K.KERNEL_SEG, 0)), ("vv28", ex(K.KERNEL_VVSTREAM, 28)), ("vv28+32", ex(K.KERNEL_VVSTREAM, 60)),
                 ("vv28+64", ex(K.KERNEL_VVSTREAM, 92)), ("vv28 upd", ex(K.KERNEL_VVSTREAM, 28 | UPD))]
        if L >= 30:
            cases += [("rs25", ex(K.KERNEL_RSTREAM, 25)), ("rs20", ex(K.KERNEL_RSTREAM, 20)),
                      ("rs20 upd", ex(K.KERNEL_RSTREAM, 20 | UPD))]
        if L % 16 == 0 and (L & (L - 1) == 0 or L <= 240) and L <= 1024:
            cases += [("gs0", ex(K.KERNEL_GSTREAM, 0)), ("gs0x80", ex(K.KERNEL_GSTREAM, 0x80)),
                      ("gs0x401", ex(K.KERNEL_GSTREAM, 0x401))]
        best = run_cases(f"fixed {L}", cases, arena, want, n * L + 2 * n, s)
        print(f"fixed {L:6d}  best explicit: {best}", flush=True)
        del arena, want, out
        torch.cuda.empty_cache()
    if args.no_mixes:
        return
    for name, pays in MIXES.items():
        rng = np.random.default_rng(7)
        lens = 32 + np.asarray(pays)[rng.integers(0, len(pays), 1 << 22)]
        csum = np.cumsum(lens)
        n = int(np.searchsorted(csum, args.bytes))
        lens = lens[:n].astype(np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
        total = int(lens.sum())
        arena = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off = torch.from_numpy(offs.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens.view(np.int32)).cuda()
        K.synth_var(arena, d_off, d_len, int(lens.max()), n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        hints = dict(total_bytes=total, min_len=int(lens.min()), max_len=int(lens.max()), packed=True)
        ctx.batch_var(K.OP_FILL, arena, d_off, d_len, n, out, stream=s, **hints)
        torch.cuda.synchronize()
        want = arena.clone()

        def exv(kernel, param):
            return lambda: ctx.batch_var_ex(K.OP_FILL, arena, d_off, d_len, n, out, kernel, param, stream=s, **hints)
        cases = [("auto", lambda: ctx.batch_var(K.OP_FILL, arena, d_off, d_len, n, out, stream=s, **hints)),
                 ("seg", exv(K.KERNEL_SEG, 0)), ("vv28", exv(K.KERNEL_VVSTREAM, 28)),
                 ("vv28+32", exv(K.KERNEL_VVSTREAM, 60)), ("vv28+64", exv(K.KERNEL_VVSTREAM, 92)),
                 ("vv28 upd", exv(K.KERNEL_VVSTREAM, 28 | UPD)), ("ss0", exv(K.KERNEL_SSTREAM, 0)),
                 ("ss128", exv(K.KERNEL_SSTREAM, 128))]
        best = run_cases(f"mix {name}", cases, arena, want, total + 2 * n, s)
        print(f"mix {name}  best explicit: {best}", flush=True)
        del arena, want, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
