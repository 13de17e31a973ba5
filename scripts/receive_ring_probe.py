#!/usr/bin/env python3
"""The receive ring (bench key `receive`: 1M 2048-B slots, 96/608/1492-B
datagrams, SORTED offset list, verdicts + host-order header array) timed the
honest way -- on rings taken in turn, so no step finds the previous step's
lines in the 256-MB Infinity Cache -- and, for comparison, on one ring.

Forms: AUTO (since round 5 the header pass FIRST: its 128 MB of first lines
are then in the Infinity Cache when the VERIFY stream reads them), the header
pass after VERIFY (tcpck_probe.h PROBE_RECEIVE_HDR_AFTER, the order before
round 5), sstream emitting each header from the stream's registers (one
launch; AUTO's form for rings of small datagrams, kernel SSTREAM param 32),
VERIFY alone.  --layout: the bench ring (offset list), 1492-B
images in 2048-B fixed slots, or C2's packed fixed 1492-B images.  Back-to-back launches, median of 5 rounds; verdicts and header
arrays compared with AUTO's."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=5):
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rings", type=int, default=3)
    p.add_argument("--slot", type=int, default=2048)
    p.add_argument("--layout", default="ring", choices=["ring", "slots1492", "c2"])
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    count, L = 1 << 20, args.slot
    rng = np.random.default_rng(42)
    ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, count)] + 32).astype(np.uint32)
    if args.layout != "ring":
        ln[:] = 1492
        L = 1492 if args.layout == "c2" else L
    off = np.arange(count, dtype=np.uint64) * np.uint64(L)
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    rings = []
    for _ in range(args.rings):
        a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
        rings.append(a)
    img = int(ln.astype(np.int64).sum())
    algo = img + 32 * count + count
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(count * 32, dtype=torch.uint8, device="cuda")
    if args.layout == "ring":
        kw = dict(offsets=d_off, lengths=d_ln, total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()),
                  sorted=True, stream=s)
        verify = lambda a: ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, count, ok, total_bytes=img,
                                         min_len=int(ln.min()), max_len=int(ln.max()), sorted=True, stream=s)
    else:
        kw = dict(stride=L, length=1492, stream=s)
        verify = lambda a: ctx.batch_fixed(tcpck.OP_VERIFY, a, L, 1492, count, ok, stream=s)
    forms = {
        "AUTO (headers first)": lambda a: ctx.batch_receive(a, count, ok, hdr, **kw),
        "headers after VERIFY": lambda a: ctx.batch_receive(a, count, ok, hdr, kernel=tcpck.KERNEL_AUTO,
                                                            probe_flags=tcpck.PROBE_RECEIVE_HDR_AFTER, **kw),
        "sstream, headers in-stream": lambda a: ctx.batch_receive(a, count, ok, hdr, kernel=tcpck.KERNEL_SSTREAM,
                                                                  param=32, **kw),
        "VERIFY alone": verify,
    }
    ref = None
    for name, fn in forms.items():
        for n in (args.rings, 1):
            turn = [0]

            def step():
                fn(rings[turn[0] % n])
                turn[0] += 1
            ms = b2b(step, s)
            a_bytes = algo if "VERIFY alone" not in name else img + count
            print(f"{name:30s} rings {n}: {ms * 1e3:7.1f} us  {a_bytes / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
        torch.cuda.synchronize()
        if "VERIFY alone" in name:
            continue
        got = (ok.clone(), hdr.clone())
        if ref is None:
            ref = got
        else:
            print(f"{name:30s} verdicts/headers == AUTO's: {torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])}",
                  flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
