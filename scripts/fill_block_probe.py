#!/usr/bin/env python3
"""FILL with each field's whole 64-B block written from the stream's own
registers (vvstream BLK, param | 128), against AUTO's FILL
(C3: vvstream CHECKSUM + the field-update pass; C2: rstream's deferred fields)
and the CHECKSUM stream alone, on C3's packed mix and on C2-shaped batches.
Back-to-back launches, median of 5 rounds of 10; every FILL form's arena and
results compared with AUTO's.

  --only LABEL[,LABEL]   run just these forms (for rocprofv3 --pmc passes)
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
import synth_np  # noqa: E402

VV_POLICY = 4 | 8 | 16  # tcpck_api.hip kVvPolicy
BLK = 128
MS = []


def b2b(fn, s, reps=10, rounds=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
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


def case(ctx, s, name, off, ln, total, only, fixed=None):
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
    pristine = a.clone()
    img = int(ln.astype(np.int64).sum())
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    V = tcpck.KERNEL_VVSTREAM
    if fixed:
        run = lambda op, p, o=out: ctx.batch_fixed_ex(op, a, fixed, fixed, n, o, V, p, stream=s)
        auto = lambda o=out: ctx.batch_fixed(tcpck.OP_FILL, a, fixed, fixed, n, o, stream=s)
    else:
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
        run = lambda op, p, o=out: ctx.batch_var_ex(op, a, d_off, d_ln, n, o, V, p, **kw)
        auto = lambda o=out: ctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, n, o, **kw)
    forms = [("CHECKSUM", lambda: run(tcpck.OP_CHECKSUM, VV_POLICY)),
             ("FILL_AUTO", auto),
             ("FILL_AUTO_noout", lambda: auto(None)),
             ("FILL_BLK", lambda: run(tcpck.OP_FILL, VV_POLICY | BLK)),
             ("FILL_BLK_noout", lambda: run(tcpck.OP_FILL, VV_POLICY | BLK, None))]
    for m in MS:
        forms.append((f"FILL_BLK_M{m}", lambda m=m: run(tcpck.OP_FILL, VV_POLICY | BLK | (m << 16))))
    ref = None
    for label, fn in forms:
        if only and label not in only:
            continue
        a.copy_(pristine)
        time.sleep(0.05)  # phase boundary in a kernel trace
        ms = b2b(fn, s)
        torch.cuda.synchronize()
        algo = img + (2 * n if "noout" not in label else 0) + (2 * n if label.startswith("FILL") else 0)
        print(f"{name:30s} {label:16s} {ms * 1e3:8.1f} us  {algo / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
        if label.startswith("FILL"):
            got = (out.clone() if "noout" not in label else None, a.clone())
            if ref is None and label == "FILL_AUTO":
                ref = got
            elif ref is not None:
                same = torch.equal(got[1], ref[1]) and (got[0] is None or torch.equal(got[0], ref[0]))
                print(f"{name:30s} {label:16s} arena/results == FILL_AUTO's: {same}", flush=True)
    del a, pristine


def packed(ln):
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    return off, ln, int(ln.astype(np.int64).sum())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default="")
    p.add_argument("--cases", default="c3,c2var,c2fixed,mix608")
    p.add_argument("--ms", default="16,64", help="grid multipliers M of the extra FILL_BLK_M<M> forms")
    args = p.parse_args()
    MS[:] = [int(x) for x in args.ms.split(",") if x]
    only = set(x for x in args.only.split(",") if x)
    cases = args.cases.split(",")
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(1)
    if "c3" in cases:
        off, ln, total = synth_np.mixed_layout(4 << 20, seed=42)
        case(ctx, s, "C3 4M 96/608/1492 packed", off, ln, total, only)
    n = 1 << 20
    if "c2var" in cases:
        case(ctx, s, "1M x 1492 packed (offset list)", *packed(np.full(n, 1492, np.uint32)), only)
    if "c2fixed" in cases:
        case(ctx, s, "C2 1M x 1492 fixed", np.arange(n, dtype=np.uint64) * 1492, np.full(n, 1492, np.uint32),
             n * 1492, only, fixed=1492)
    if "mix608" in cases:
        case(ctx, s, "2M 608/1492 packed", *packed(np.asarray((608, 1492), np.uint32)[rng.integers(0, 2, 2 << 20)]),
             only)
    ctx.close()


if __name__ == "__main__":
    main()
