#!/usr/bin/env python3
"""Retransmit batch cost on the C2 layout (1M x 1492 B): tcpck_batch_set_ack
(ACK rewrite + incremental checksum update, one scalar ACK or one per image)
vs the reference's way, a full recompute of every image (FILL).  Median of
back-to-back rounds after a settle."""
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
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, n, seed=42)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, None)
    acks = torch.arange(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    runs = [
        ("set_ack, one ACK", lambda: ctx.batch_set_ack(a, n, ack=77, stride=L, stream=s)),
        ("set_ack, one ACK + out", lambda: ctx.batch_set_ack(a, n, ack=77, stride=L, out=out, stream=s)),
        ("set_ack, per-image ACKs + out", lambda: ctx.batch_set_ack(a, n, acks=acks, stride=L, out=out, stream=s)),
        ("full recompute (FILL)", lambda: ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, out, stream=s)),
    ]
    for name, fn in runs:
        ms = b2b(fn, s)
        print(f"C2 {n} images: {name:32s} {ms * 1e3:9.1f} us  {n / ms / 1e6:8.2f} G images/s", flush=True)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, n, ok)
    torch.cuda.synchronize()
    assert bool(ok.all())


if __name__ == "__main__":
    main()
