#!/usr/bin/env python3
"""Receive batch cost (ReceivePacket's front half, socket-manager.h:181-184):
the verdict pass (TCPCK_OP_VERIFY) alone, the header N2H pass
(tcpck_batch_header_swap) alone, both back to back on one stream, and
TCPCK_OP_RECEIVE (the same two passes in one call), and
tcpck_batch_receive into a dense header array -- on
C2's layout (1M x 1492 B packed), 1M x 1492 B in 2048-B slots and a 1M-entry
offset list.  Median of back-to-back rounds after a settle."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


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


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    n, L = 1 << 20, 1492
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    for name, stride in (("C2 packed", L), ("2048-B slots", 2048)):
        a = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, stride, L, n, seed=42)
        ctx.batch_fixed(tcpck.OP_FILL, a, stride, L, n, None)
        runs = [
            ("VERIFY", lambda: ctx.batch_fixed(tcpck.OP_VERIFY, a, stride, L, n, ok, stream=s)),
            ("header N2H", lambda: ctx.batch_header_swap(a, n, stride=stride, stream=s)),
            ("VERIFY + N2H", lambda: (ctx.batch_fixed(tcpck.OP_VERIFY, a, stride, L, n, ok, stream=s),
                                      ctx.batch_header_swap(a, n, stride=stride, stream=s))),
            ("OP_RECEIVE", lambda: ctx.batch_fixed(tcpck.OP_RECEIVE, a, stride, L, n, ok, stream=s)),
            ("receive->hdr", lambda: ctx.batch_receive(a, n, ok, hdr, stride=stride, length=L, stream=s)),
        ]
        for what, fn in runs:
            ms = b2b(fn, s)
            print(f"{name:14s} {n} x {L}: {what:14s} {ms * 1e3:9.1f} us  {n * L / ms / 1e6:8.1f} GB/s of images",
                  flush=True)
        del a
    # offset list: the same images as a 1M-entry list (sorted)
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, n, seed=42)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * L
    ln = torch.full((n,), L, dtype=torch.int32, device="cuda")
    hints = dict(total_bytes=n * L, min_len=L, max_len=L, packed=True, sorted=True)
    runs = [
        ("VERIFY", lambda: ctx.batch_var(tcpck.OP_VERIFY, a, off, ln, n, ok, stream=s, **hints)),
        ("header N2H", lambda: ctx.batch_header_swap(a, n, offsets=off, stream=s)),
        ("receive->hdr", lambda: ctx.batch_receive(a, n, ok, hdr, offsets=off, lengths=ln, stream=s, **hints)),
    ]
    for what, fn in runs:
        ms = b2b(fn, s)
        print(f"{'offset list':14s} {n} x {L}: {what:14s} {ms * 1e3:9.1f} us  {n * L / ms / 1e6:8.1f} GB/s of images",
              flush=True)


if __name__ == "__main__":
    main()
