#!/usr/bin/env python3
"""FILL as the layout's CHECKSUM pass + a field-update pass (c = ~(~C - f)
mod 2^16 from the old field f, written as the field's 64-B block) against
AUTO's in-stream FILL (TCPCK_PARAM_FILL_INSTREAM), with CHECKSUM for
reference.  Both FILL results (arena and out) are compared byte for byte on
the same input.  ~1.5 GB per layout, median of back-to-back rounds."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

UPD, INS = 1 << 28, 1 << 29


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


def report(name, runs, img_bytes, n, s, check):
    ms = {}
    for label, fn in runs:
        ms[label] = b2b(fn, s)
        print(f"{name:24s} {label:14s} {ms[label] * 1e3:8.1f} us  "
              f"{(img_bytes + 2 * n) / ms[label] / 1e6 / 80:5.1f} % of the roof", flush=True)
    print(f"{name:24s} results identical: {check()}", flush=True)


def fixed_case(ctx, s, L, S):
    n = (1536 << 20) // S
    a = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, S, L, n, seed=42)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    A = tcpck.KERNEL_AUTO

    def check():
        b = a.clone()
        o1 = torch.empty_like(out)
        ctx.batch_fixed_ex(tcpck.OP_FILL, b, S, L, n, o1, A, INS, stream=s)
        c = a.clone()
        o2 = torch.empty_like(out)
        ctx.batch_fixed_ex(tcpck.OP_FILL, c, S, L, n, o2, A, 0, stream=s)
        torch.cuda.synchronize()
        r = bool(torch.equal(b, c) and torch.equal(o1, o2))
        del b, c
        return r

    runs = [("CHECKSUM", lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, S, L, n, out, A, 0, stream=s)),
            ("FILL instream", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, a, S, L, n, out, A, INS, stream=s)),
            ("FILL update", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, a, S, L, n, out, A, 0, stream=s))]
    report(f"fixed {L}/{S}", runs, n * L, n, s, check)
    del a


def var_case(ctx, s, kind):
    from synth_np import mixed_layout
    if kind == "c3":
        n = 4 << 20
        off, ln, total = mixed_layout(n, seed=42)
        flags = dict(packed=True)
    else:  # receive slots: the mix in 2048-B slots
        n = 1 << 20
        rng = np.random.default_rng(42)
        ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
        off = np.arange(n, dtype=np.uint64) * np.uint64(2048)
        total = n * 2048
        flags = dict(sorted=True)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    img = int(ln.astype(np.int64).sum())
    kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), stream=s, **flags)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    A = tcpck.KERNEL_AUTO

    def check():
        b = a.clone()
        o1 = torch.empty_like(out)
        ctx.batch_var_ex(tcpck.OP_FILL, b, d_off, d_ln, n, o1, A, INS, **kw)
        c = a.clone()
        o2 = torch.empty_like(out)
        ctx.batch_var_ex(tcpck.OP_FILL, c, d_off, d_ln, n, o2, A, 0, **kw)
        torch.cuda.synchronize()
        r = bool(torch.equal(b, c) and torch.equal(o1, o2))
        del b, c
        return r

    runs = [("CHECKSUM", lambda: ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, A, 0, **kw)),
            ("FILL instream", lambda: ctx.batch_var_ex(tcpck.OP_FILL, a, d_off, d_ln, n, out, A, INS, **kw)),
            ("FILL update", lambda: ctx.batch_var_ex(tcpck.OP_FILL, a, d_off, d_ln, n, out, A, 0, **kw))]
    report(f"var {kind}", runs, img, n, s, check)
    del a


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--fixed", default="64/64,96/96,128/128,256/256,512/512,1024/1024,1492/1492,4096/4096,"
                                       "9000/9000,65536/65536,1492/2048,96/256,9000/16384,9000/9216")
    p.add_argument("--var", default="c3,slots")
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    for spec in filter(None, args.fixed.split(",")):
        L, S = (int(x) for x in spec.split("/"))
        fixed_case(ctx, s, L, S)
    for kind in filter(None, args.var.split(",")):
        var_case(ctx, s, kind)


if __name__ == "__main__":
    main()
