#!/usr/bin/env python3
"""Does the distance between a copy's source and destination set its rate?
The diag copy kernel (tcpck_diag_stream variant 0x5000, scripts/copy_probe.py)
copies the first `half` bytes of a buffer to the next `half`, so the
destination sits exactly `half` bytes after the source; here `half` is
1.5 GiB plus a small delta (128 B to 1 MiB), which moves the destination
relative to the source's HBM channel and bank interleave without changing the
bytes moved.  Two cold-ish buffers taken in turn, back to back, median of 5
rounds; % of the 8 TB/s roof in read + write bytes.  Timing only (the copy is
checked once at the end)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=10, rounds=5):
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--deltas", default="0,128,256,512,1024,2048,4096,8192,16384,65536,262144,1048448")
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    base = 1536 << 20
    size = 2 * (base + (2 << 20))
    bufs = [torch.randint(0, 255, (size,), dtype=torch.uint8, device="cuda") for _ in range(2)]
    out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    forms = [("runs U4 nt M8", 0x5000 | 1 | (1 << 2) | (8 << 8)),
             ("grid-stride U2 nt M8", 0x5000 | 0 | (1 << 2) | 16 | (8 << 8))]
    for name, v in forms:
        for d in (int(x) for x in args.deltas.split(",")):
            half = base + d
            turn = [0]

            def step():
                ctx.diag_stream(v, bufs[turn[0] % 2], 2 * half, out, stream=s)
                turn[0] += 1
            ms = b2b(step, s)
            print(f"{name:22s} dst - src = 1.5 GiB + {d:8d} B: {ms * 1e3:7.1f} us  "
                  f"{2 * half / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
    torch.cuda.synchronize()
    b = bufs[0]
    half = base + int(args.deltas.split(",")[-1])
    ctx.diag_stream(forms[0][1], b, 2 * half, out, stream=s)
    torch.cuda.synchronize()
    print(f"copy verified: {torch.equal(b[:half], b[half:2 * half])}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
