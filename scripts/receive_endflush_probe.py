#!/usr/bin/env python3
"""RECEIVE on sstream rings: where does the in-stream header form's extra
time go?  (Round 3, profiles/r03/receive_endflush_probe.log: the stores
themselves -- the records built and staged but never stored cost nothing,
stored after the run's stream they cost as much as inside it.  The HDR 4-6
kernel variants this drove were measured and removed; the script needs them
back in tcpck_sstream.hip to run.)  Forms (probe build, kernel SSTREAM):
  VERIFY only                     the verdicts alone
  two passes                      VERIFY + the separate header pass (AUTO's form for MSS rings)
  in-stream  (param 32)           records from the stream's registers, staged in LDS, stored 256 B
                                  at a time inside the stream loop
  end-flush  (param 32 | 128)     the same records kept in LDS until the run's stream has ended,
                                  then stored 1 KiB per instruction (+ 16: write-through stores)
  no-store   (param 32 | 64 | 128) the records built and staged but never stored (diagnostic)
Results of every storing form compared byte for byte with the two-pass form.
--small: the 4M x 256-B ring of 32-254-B datagrams, VERIFY at grid multipliers
M = 1..16 against the in-stream RECEIVE (VERIFY alone measured slower than
the RECEIVE there in profiles/r03/receive_fused_probe_staged.log)."""
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


def ring(ctx, s, name, n, slot, ln, fixed_len=None, small=False):
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

    lo, hi = int(ln.min()), int(ln.max())  # once: per call they kept the host behind small-ring kernels

    def verify(p=None):
        if fixed_len:
            if p is None:
                ctx.batch_fixed(tcpck.OP_VERIFY, a, slot, fixed_len, n, ok, stream=s)
            else:
                ctx.batch_fixed_ex(tcpck.OP_VERIFY, a, slot, fixed_len, n, ok, kernel=S, param=p, stream=s)
        elif p is None:
            ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, total_bytes=img, min_len=lo, max_len=hi,
                          sorted=True, stream=s)
        else:
            ctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, kernel=S, param=p, total_bytes=img,
                             min_len=lo, max_len=hi, sorted=True, stream=s)

    if small:
        for m in (0, 1, 2, 4, 8, 16):
            tv = b2b(lambda: verify(m << 16), s)
            tr = b2b(lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=(m << 16) | 32, **kw), s)
            print(f"{name:28s} M {m:2d}  VERIFY {tv * 1e3:7.1f} us   in-stream RECEIVE {tr * 1e3:7.1f} us", flush=True)
        tv = b2b(lambda: verify(), s)
        print(f"{name:28s} AUTO VERIFY {tv * 1e3:7.1f} us", flush=True)
    runs = [("VERIFY only", lambda: verify()),
            ("two passes", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=TWO, **kw)),
            ("in-stream", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=32, **kw)),
            ("end-flush", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=32 | 128, **kw)),
            ("end-flush WT", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=32 | 128 | 16, **kw)),
            ("no-store", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=S, param=32 | 64 | 128, **kw)),
            ("AUTO", lambda: ctx.batch_receive(a, n, ok, hdr, **kw))]
    res = {}
    for label, fn in runs:
        if label != "VERIFY only":
            hdr.fill_(0xA5)
            ok.fill_(7)
        ms = b2b(fn, s)
        if label not in ("VERIFY only", "no-store"):
            torch.cuda.synchronize()
            res[label] = (ok.clone(), hdr.clone())
        alg = img + n + (0 if label == "VERIFY only" else 32 * n)
        print(f"{name:28s} {label:12s} {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof "
              f"(image bytes + verdicts + headers)", flush=True)
    ref = res["two passes"]
    same = all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in res.values())
    print(f"{name:28s} results identical: {same}", flush=True)
    del a, hdr


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(42)
    n = 1 << 20
    mix = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    ring(ctx, s, "ring 1M x 2048 (bench mix)", n, 2048, mix)
    ring(ctx, s, "ring 1M x 1536 (bench mix)", n, 1536, mix)
    ring(ctx, s, "fixed 1492 in 2048-B slots", n, 2048, np.full(n, 1492, np.uint32), fixed_len=1492)
    small = (rng.integers(16, 128, 4 * n) * 2).astype(np.uint32)
    ring(ctx, s, "ring 4M x 256 (32-254 B)", 4 * n, 256, small, small="--small" in sys.argv)


if __name__ == "__main__" and "--trace" not in sys.argv:
    main()


def trace():
    """--trace: the 4M x 256-B ring, 20 launches each of VERIFY (AUTO), the
    no-store RECEIVE and the in-stream RECEIVE, for rocprofv3 --kernel-trace."""
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(42)
    n = 4 << 20
    ln = (rng.integers(16, 128, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(256)
    a = torch.empty(n * 256, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    kw = dict(offsets=d_off, lengths=d_ln, total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()),
              sorted=True, stream=s)
    for label, fn in (("verify", lambda: ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok,
                                                       total_bytes=kw["total_bytes"], min_len=kw["min_len"],
                                                       max_len=kw["max_len"], sorted=True, stream=s)),
                      ("no-store", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=tcpck.KERNEL_SSTREAM,
                                                             param=32 | 64 | 128, **kw)),
                      ("in-stream", lambda: ctx.batch_receive(a, n, ok, hdr, kernel=tcpck.KERNEL_SSTREAM, param=32,
                                                              **kw))):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        print(label, "done", flush=True)


if __name__ == "__main__" and "--trace" in sys.argv:
    trace()
