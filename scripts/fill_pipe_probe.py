#!/usr/bin/env python3
"""Pipelined FILL: the field pass of chunk i on a context
stream beside the stream pass of chunk i + 1 (tcpck_api.hip fill_pipelined),
against the serial form (stream over all images, then the field pass), at C3
(4M packed 96/608/1492, the update form) and C2 (1M x 1492 fixed, rstream's
deferred fields), with and without a results buffer.

Timed like bench.py: two identical batches taken in turn (cold), 250 ms of
settle launches, then median of 5 rounds of 10 back-to-back launches between
HIP events on the launch stream (the pipelined call joins the pipe stream back
into it, so the end event covers every field pass).  Every form's arena and
results are compared with the serial form's.

Hypothesis (written before the run): the field pass is
bound by sub-64-B merge writes (~44 us per 1M fields, ~3.9 TB/s of HBM
traffic), not by HBM bandwidth, so beside a stream at ~7.2 TB/s it should take
part of the slack: C3 636 -> <= 560 us (fill_c3 >= 0.66) if the overlap is
real.  Stop rule: if no K in {4, 8, 16} beats serial by >= 3 % at C3, FILL is
closed.

  --ks 0,2,4,8,16,32   chunk counts (0 = serial; + 256: the chunks on the caller's
                       stream only, no pipe stream -- the chunking cost alone)
  --prio 0,-1          pipe stream priorities
  --only c3,c3_noout,c2,c2_noout
  --pmc-calls N        (under rocprofv3 --pmc, one K per run) N FILLs and no timing;
                       scripts/fill_pipe_pmc.py sums the counters per call
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


def timed(fn, s, reps=10, rounds=5):
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
    return float(np.median(t)), float(min(t)), float(max(t))


def run_case(ctx, s, name, ks, prios, reps, rounds, pmc_calls=0):
    n_c3 = 4 << 20
    if name.startswith("c3"):
        off, ln, total = synth_np.mixed_layout(n_c3, seed=42)
        n = ln.size
        img = int(ln.astype(np.int64).sum())
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        arenas = []
        for _ in range(2):
            a = torch.empty(total, dtype=torch.uint8, device="cuda")
            tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42, stream=s)
            arenas.append(a)
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)

        def call(a, o):
            ctx.batch_var_ex(tcpck.OP_FILL, a, d_off, d_ln, n, o, tcpck.KERNEL_AUTO, 0, **kw)

        def checksum(a, o):
            ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, o, tcpck.KERNEL_AUTO, 0, **kw)
    else:
        n, L = 1 << 20, 1492
        img = n * L
        arenas = []
        for _ in range(2):
            a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
            tcpck.synth_fixed(a, L, L, n, seed=42, stream=s)
            arenas.append(a)

        def call(a, o):
            ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, o, tcpck.KERNEL_AUTO, 0, stream=s)

        def checksum(a, o):
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, o, tcpck.KERNEL_AUTO, 0, stream=s)
    pristine = arenas[0].clone()
    noout = name.endswith("_noout")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    algo_fill = img + 2 * n + (0 if noout else 2 * n)
    turn = [0]

    def step(fn, o):
        def f():
            fn(arenas[turn[0] & 1], o)
            turn[0] += 1
        return f

    if pmc_calls:  # rocprofv3 --pmc runs: exactly pmc_calls FILLs of each form, nothing else timed
        for k in ks:
            ctx.set_fill_pipe(k, prios[0])
            for _ in range(pmc_calls):
                step(call, None if noout else out)()
            torch.cuda.synchronize()
            print(f"{name:10s} FILL K {k}: {pmc_calls} calls", flush=True)
        ctx.set_fill_pipe(-1, 0)
        return
    ms, lo, hi = timed(step(checksum, out), s, reps, rounds)
    print(f"{name:10s} CHECKSUM          {ms * 1e3:8.1f} us [{lo * 1e3:.1f}, {hi * 1e3:.1f}]  "
          f"{(img + 2 * n) / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
    ref = None
    for prio in prios:
        for k in ks:
            if k == 0 and prio != prios[0]:
                continue
            ctx.set_fill_pipe(k, prio)
            for a in arenas:
                a.copy_(pristine)
            torch.cuda.synchronize()
            time.sleep(0.05)
            ms, lo, hi = timed(step(call, None if noout else out), s, reps, rounds)
            kk = k & 0xFF
            label = ("serial" if k == 0 else f"pipe K{kk:<2d} prio{prio:+d}" if not k & tcpck.PROBE_PIPE_ONE_STREAM
                     else f"chunks K{kk:<2d} 1-strm")
            line = (f"{name:10s} FILL {label:14s} {ms * 1e3:8.1f} us [{lo * 1e3:.1f}, {hi * 1e3:.1f}]  "
                    f"{algo_fill / ms / 1e6 / 80:5.1f} % of the roof")
            got = (None if noout else out.clone(), arenas[0].clone(), arenas[1].clone())
            if ref is None:
                ref = got
            else:
                same = all(torch.equal(x, y) for x, y in zip(got, ref) if x is not None)
                line += f"  == serial: {same}"
            print(line, flush=True)
    ctx.set_fill_pipe(-1, 0)
    del arenas, pristine
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ks", default="0,2,4,8,16,32")
    p.add_argument("--prio", default="0,-1")
    p.add_argument("--only", default="c3,c3_noout,c2,c2_noout")
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--pmc-calls", type=int, default=0,
                   help="for rocprofv3 --pmc: only this many FILL calls per K (one K per run), no timing")
    args = p.parse_args()
    print(__doc__.split("Hypothesis")[1].split("--ks")[0].strip(), flush=True)
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    ks = [int(x) for x in args.ks.split(",")]
    prios = [int(x) for x in args.prio.split(",")]
    for name in args.only.split(","):
        run_case(ctx, s, name, ks, prios, args.reps, args.rounds, args.pmc_calls)
    ctx.close()


if __name__ == "__main__":
    main()
