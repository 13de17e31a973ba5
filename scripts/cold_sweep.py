#!/usr/bin/env python3
"""C2 / C3 kernel choices re-measured COLD (round 5): every step on one of two
identical arenas taken in turn, so no step finds the previous step's lines in
the Infinity Cache (scripts/arena_reuse_probe.py: one arena re-read step after
step ran 2-3 % faster, and a 512-MB read of another buffer between steps
removes that exactly like a second arena does).  The round-1..4 choices (grid
multiplier M, steps in flight U, the L2-kept first step, the XCD-chunked
order) were measured on one arena; here each is re-timed both ways.

rstream params: variant | M << 16 (18: v_dot2 + buffer loads + XCD-chunked
order; 20: 18 + the run's first step with the default cache policy = AUTO;
22: every step default policy; 23 / 24: 20 with 8 / 2 steps in flight; 31 =
20 (since round 5 only the run's first line kept), 32: 20 before round 5
(the whole first step kept); 14 /
15: each XCD one contiguous region of runs, 4 / 8 steps in flight; 21: 14 +
the first step default policy).
vvstream params: 2 / 3 = equal-count runs U4 / U8, + 8 XCD-chunked order, +
16 first step default policy (AUTO: 4 | 8 | 16 = 28, U8 at M 32)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402

VARIANTS, MS, VMS = [], [], []


def b2b(fn, s, reps=20, rounds=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
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


def sweep(name, arenas, run, params, algo, s):
    for label, p in params:
        res = []
        for k in (2, 1):
            turn = [0]

            def step():
                run(arenas[turn[0] % k], p)
                turn[0] += 1
            ms = b2b(step, s)
            res.append(f"{k} arena{'s' if k > 1 else ''} {ms * 1e3:7.1f} us {algo / ms / 1e6 / 80:5.1f} %")
        print(f"{name} {label:34s} " + " | ".join(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c2,c3", help="c2, c3, diag (the bare C2-size stream)")
    ap.add_argument("--rs", default="20,18,22,23,24", help="rstream variants (C2)")
    ap.add_argument("--ms", default="16,32,64", help="grid multipliers (C2)")
    ap.add_argument("--vms", default="16,32,64", help="grid multipliers (C3)")
    ap.add_argument("--sms", default="2,4,8,16", help="grid multipliers (slots)")
    ap.add_argument("--c2n", type=int, default=1 << 20, help="images of the c2 case (8388608: C5 on one GPU)")
    ap.add_argument("--c3n", type=int, default=4 << 20, help="images of the c3 case (C3's mix)")
    ap.add_argument("--c3forms", default="U8 xcd keep,U8 xcd,U4 xcd keep", help="vvstream forms swept (c3)")
    ap.add_argument("--sorders", default="scatter,xcd-chunked,default order", help="block orders (slots)")
    args = ap.parse_args()
    VARIANTS[:] = [int(x) for x in args.rs.split(",")]
    MS[:] = [int(x) for x in args.ms.split(",")]
    VMS[:] = [int(x) for x in args.vms.split(",") if x]
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    if "c2" in args.cases.split(","):
        n, L = args.c2n, 1492
        arenas = []
        for _ in range(2):
            a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
            tcpck.synth_fixed(a, L, L, n, seed=42)
            arenas.append(a)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        run = lambda a, p: (ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out, stream=s) if p is None else
                            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, tcpck.KERNEL_RSTREAM, p, stream=s))
        if "diag" in args.cases:  # the bare stream (no checksum, XCD regions, 32x): the ceiling, cold and warm
            dout = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
            sweep("c2", arenas, lambda a, p: ctx.diag_stream(p, a, n * L, dout, stream=s),
                  [("AUTO warm-up", 0x3801), ("bare stream 0x3801 (xcd)", 0x3801), ("bare stream 0x3800", 0x3800)],
                  n * L + 2 * n, s)
        params = [("AUTO warm-up", None), ("AUTO", None)]
        for v in VARIANTS:
            for m in MS:
                params.append((f"rstream {v} M{m}", v | (m << 16)))
        sweep("c2", arenas, run, params, n * L + 2 * n, s)
        del arenas, out
        torch.cuda.empty_cache()
    if "c3" in args.cases.split(",") or "c3fixed" in args.cases:
        n = args.c3n
        off, ln, total = synth_np.mixed_layout(n, seed=42)
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        arenas = []
        for _ in range(2):
            a = torch.empty(total, dtype=torch.uint8, device="cuda")
            tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
            arenas.append(a)
        img = int(ln.astype(np.int64).sum())
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
        run = lambda a, p: (ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, **kw) if p is None else
                            ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_VVSTREAM, p, **kw))
        params = [("AUTO warm-up", None), ("AUTO", None)] if "c3" in args.cases.split(",") else [("AUTO", None)]
        params += [] if "c3" not in args.cases.split(",") else [("vvstream policy, whole first step kept (5)", 5 | 8 | 16), ("vvstream policy (AUTO)", 4 | 8 | 16),
                   ("vvstream policy, no kept line", 4 | 8)]
        for base, lab in ((3 | 8 | 16, "U8 xcd keep"), (3 | 8, "U8 xcd"), (2 | 8 | 16, "U4 xcd keep")):
            if lab not in args.c3forms.split(","):
                continue
            for m in VMS:
                params.append((f"vvstream {lab} M{m}", base | (m << 16)))
        sweep("c3", arenas, run, params, img + 2 * n, s)
        if "c3fixed" in args.cases:  # C3's bytes as a 736-B fixed stride: no descriptors, the same boundary density
            L = 736
            n2 = img // L
            run2 = lambda a, p: (ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n2, out, stream=s) if p is None else
                                 ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n2, out, p[0], p[1], stream=s))
            sweep("736", arenas, run2, [("AUTO (rstream)", None), ("vvstream FIXED policy", (tcpck.KERNEL_VVSTREAM, 28))],
                  n2 * L + 2 * n2, s)
    if "slots" in args.cases.split(","):
        # the bench's receive ring, VERIFY (the `slots` key): sstream's block order and grid, cold
        n, SL = 1 << 20, 2048
        rng = np.random.default_rng(42)
        ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
        off = np.arange(n, dtype=np.uint64) * np.uint64(SL)
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        arenas = []
        for _ in range(2):
            a = torch.empty(n * SL, dtype=torch.uint8, device="cuda")
            tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
            arenas.append(a)
        img = int(ln.astype(np.int64).sum())
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), sorted=True, stream=s)
        run = lambda a, p: (ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, **kw) if p is None else
                            ctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, tcpck.KERNEL_SSTREAM, p, **kw))
        params = [("AUTO warm-up", None), ("AUTO", None)]
        for order, lab in ((8, "scatter"), (0 | 1, "xcd-chunked"), (4, "default order")):
            if lab not in args.sorders.split(","):
                continue
            for m in (int(x) for x in args.sms.split(",")):
                params.append((f"sstream {lab} M{m}", order | 1 | (m << 16)))
        sweep("slots", arenas, run, params, img + n, s)
    ctx.close()


if __name__ == "__main__":
    main()
