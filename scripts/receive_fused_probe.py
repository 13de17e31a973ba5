#!/usr/bin/env python3
"""RECEIVE into a header array on sstream layouts: the VERIFY pass followed by
the separate header pass (TCPCK_PARAM_RECEIVE_TWO_PASS) against sstream
writing each run's headers itself after the run's verdicts (one launch),
with the stream read nt (variant 0) or with the default cache policy
(variant 16, the header lines still in L2 when the run's end re-reads them),
and (round 3) each header emitted from the stream's registers as the step is
consumed (variant 32; 96: with write-through sc0 sc1 nt stores), and the
header pass with write-through array stores (tcpck_probe_receive_ex's
PROBE_RECEIVE_HDR_WT, probe build).
VERIFY alone for reference.  Results compared byte for byte.  Median of
back-to-back rounds.  (Before round 3's fix the VERIFY-only closure took the
lengths' min/max on the host per call: its small-ring lines, ~300 us, were
host-bound; the kernel takes 140 us, profiles/r03/receive_small_ring_trace.txt.)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402

TWO = 1 << 30


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


def case(ctx, s, name, n, slot, ln, fixed_len=None):
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
    img = int(ln.astype(np.int64).sum())
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    S = tcpck.KERNEL_SSTREAM
    if fixed_len:
        kw = dict(stride=slot, length=fixed_len, stream=s)
    else:
        kw = dict(offsets=d_off, lengths=d_ln, total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()),
                  sorted=True, stream=s)

    def verify():
        if fixed_len:
            ctx.batch_fixed(tcpck.OP_VERIFY, a, slot, fixed_len, n, ok, stream=s)
        else:
            ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, total_bytes=img, min_len=kw["min_len"],
                          max_len=kw["max_len"], sorted=True, stream=s)

    runs = [("VERIFY only", verify),
            ("two passes", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=TWO, **kw)),
            ("fused nt", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=0, **kw)),
            ("fused keep", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=16, **kw)),
            ("in-stream", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=32, **kw)),
            ("in-str WT", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=96, **kw)),
            ("2 passes WT", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=TWO,
                                                      probe_flags=tcpck.PROBE_RECEIVE_HDR_WT, **kw)),
            ("2 passes KH", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=TWO | 16, **kw)),
            ("concurrent", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=0,
                                                     probe_flags=tcpck.PROBE_RECEIVE_CONCURRENT, **kw)),
            ("concurrent A", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=0, param=0,
                                                       probe_flags=tcpck.PROBE_RECEIVE_CONCURRENT, **kw)),
            ("AUTO", lambda: ctx.batch_receive(a, n, ok, hdr, **kw))]
    res = {}
    for label, fn in runs:
        ms = b2b(fn, s)
        if label != "VERIFY only":
            torch.cuda.synchronize()
            res[label] = (ok.clone(), hdr.clone())
        alg = img + n + (0 if label == "VERIFY only" else 32 * n)
        print(f"{name:28s} {label:12s} {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof "
              f"(image bytes + verdicts + headers)", flush=True)
    ref = res["two passes"]
    same = all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in res.values())
    print(f"{name:28s} results identical: {same}", flush=True)
    del a, hdr


def sweep(ctx, s, rng, n):
    """--sweep: VERIFY against the in-stream RECEIVE (param 32) over slot
    sizes, grid multipliers M (param bits 16-23; 0 = the policy's) and block
    orders (+4 default, else scattered)."""
    mix = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    img = int(mix.astype(np.int64).sum())
    S = tcpck.KERNEL_SSTREAM
    for slot in (1536, 2048, 2560, 4096):
        off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
        a = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(mix).cuda()
        tcpck.synth_var(a, d_off, d_ln, int(mix.max()), n, seed=42)
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        kw = dict(offsets=d_off, lengths=d_ln, total_bytes=img, min_len=int(mix.min()), max_len=int(mix.max()),
                  sorted=True, stream=s)
        for order in (0, 4):
            for m in (0, 1, 2, 4, 8, 16):
                p = (m << 16) | order
                tv = b2b(lambda: ctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, kernel=S, param=p,
                                                  total_bytes=img, min_len=int(mix.min()), max_len=int(mix.max()),
                                                  sorted=True, stream=s), s)
                tr = b2b(lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=p | 32, **kw), s)
                print(f"slot {slot:5d} order {order} M {m:2d}   VERIFY {tv * 1e3:7.1f} us   in-stream RECEIVE "
                      f"{tr * 1e3:7.1f} us   (+{(tr - tv) * 1e3:5.1f})", flush=True)
        del a, hdr


def wide(ctx, s, rng, n):
    """--wide: the receive ring's header pass as the product form (8 lanes per
    image, u16 loads) against two lanes per image with one 16-B load each and
    the load cache bits default / nt / sc0 sc1 / sc1 (tcpck_probe_receive_ex:
    PROBE_RECEIVE_HDR_WIDE | form << 4, probe build); time per RECEIVE step and
    the results compared."""
    mix = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    img = int(mix.astype(np.int64).sum())
    S = tcpck.KERNEL_SSTREAM
    slot = 2048
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(mix).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(mix.max()), n, seed=42)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    kw = dict(offsets=d_off, lengths=d_ln, total_bytes=img, min_len=int(mix.min()), max_len=int(mix.max()),
              sorted=True, stream=s)
    res = {}
    W, F = tcpck.PROBE_RECEIVE_HDR_WIDE, tcpck.PROBE_RECEIVE_HDR_FIRST
    for label, f in (("two passes", 0), ("wide default", W), ("wide nt", W | (1 << 4)), ("wide sc0 sc1", W | (2 << 4)),
                     ("wide sc1", W | (3 << 4)), ("header first", F), ("hdr first wide", F | W)):
        ms = b2b(lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=TWO, probe_flags=f, **kw), s)
        torch.cuda.synchronize()
        res[label] = (ok.clone(), hdr.clone())
        print(f"ring 1M x 2048 (bench mix)   {label:14s} {ms * 1e3:8.1f} us", flush=True)
    ref = res["two passes"]
    print("results identical:", all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in res.values()),
          flush=True)


def order(ctx, s, rng, n):
    """--order (round 4): the receive ring's header pass with the images in
    another order (tcpck_probe_receive_ex ORDER: 1 XCD-chunked blocks, 2 blocks
    scattered over the batch, 3 each block's images 1/128 of the batch apart)
    against the product's in-order pass, and VERIFY alone; per RECEIVE step,
    the header pass = RECEIVE - VERIFY.  Results compared."""
    mix = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    img = int(mix.astype(np.int64).sum())
    S = tcpck.KERNEL_SSTREAM
    slot = 2048
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(mix).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(mix.max()), n, seed=42)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    kw = dict(offsets=d_off, lengths=d_ln, total_bytes=img, min_len=int(mix.min()), max_len=int(mix.max()),
              sorted=True, stream=s)
    ver = b2b(lambda: ctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, kernel=S, param=0, total_bytes=img,
                                       min_len=int(mix.min()), max_len=int(mix.max()), sorted=True, stream=s), s)
    print(f"ring 1M x 2048 (bench mix)   VERIFY only    {ver * 1e3:8.1f} us", flush=True)
    res = {}
    for label, f in (("in order", 0), ("XCD-chunked", 1 << 8), ("scattered", 2 << 8), ("transposed", 3 << 8),
                     ("in order", 0)):
        ms = b2b(lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=TWO, probe_flags=f, **kw), s)
        torch.cuda.synchronize()
        res[label] = (ok.clone(), hdr.clone())
        print(f"ring 1M x 2048 (bench mix)   {label:14s} {ms * 1e3:8.1f} us  header pass {(ms - ver) * 1e3:6.1f} us",
              flush=True)
    ref = res["in order"]
    print("results identical:", all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in res.values()),
          flush=True)


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(42)
    n = 1 << 20
    if "--wide" in sys.argv:
        wide(ctx, s, rng, n)
        return
    if "--sweep" in sys.argv:
        sweep(ctx, s, rng, n)
        return
    if "--order" in sys.argv:
        order(ctx, s, rng, n)
        return
    mix = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    case(ctx, s, "ring 1M x 2048 (bench mix)", n, 2048, mix)
    case(ctx, s, "ring 1M x 1536 (bench mix)", n, 1536, mix)
    case(ctx, s, "fixed 1492 in 2048-B slots", n, 2048, np.full(n, 1492, np.uint32), fixed_len=1492)
    small = (rng.integers(16, 128, 4 * n) * 2).astype(np.uint32)
    case(ctx, s, "ring 4M x 256 (32-254 B)", 4 * n, 256, small)


if __name__ == "__main__":
    main()
