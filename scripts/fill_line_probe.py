#!/usr/bin/env python3
"""FILL on packed fixed images: the line form (rstream 31) against AUTO's
deferred form (rstream 25) and CHECKSUM.  (round 4)

25: the stream reads every byte and writes the results, then one write-through
2-B store per field -- the memory side reads each field's 64-B block to merge
it.  31: the stream skips every field's 128-B line, then a pass reads each
field line and writes it back whole (a full-line write needs no merge read).
Median of rounds of 20 back-to-back steps after a settle; every FILL's arena is
compared with the 25 form's.  The line form lost (profiles/r04/fill_line_probe.log,
DESIGN.md section 8) and rstream variant 31 was removed with it: its cases are
rejected by the current libraries."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=7):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--lengths", default="1492,512,1024,2048,4096,9000")
    ap.add_argument("--bytes", type=float, default=1.5644e9)
    args = ap.parse_args()
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    R = tcpck.KERNEL_RSTREAM
    for L in [int(x) for x in args.lengths.split(",")]:
        n = int(args.bytes) // L
        arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(arena, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        algo = n * L + 2 * n
        ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 25, stream=s)
        torch.cuda.synchronize()
        want = arena.clone()
        cases = [("fill25", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 25, stream=s), True),
                 ("line31", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 31, stream=s), True),
                 ("auto", lambda: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, out, stream=s), True),
                 ("noout", lambda: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, None, stream=s), True),
                 ("checksum", lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s), False),
                 ("fill25", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 25, stream=s), True),
                 ("line31", lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 31, stream=s), True)]
        for label, fn, full in cases:
            ms = b2b(fn, s)
            same = ""
            if full:
                torch.cuda.synchronize()
                same = "arena == 25's" if torch.equal(arena, want) else "ARENA DIFFERS"
                arena.copy_(want)
            frac = algo / (ms * 1e-3) / 8e12
            print(f"{L:6d} B x {n:8d}  {label:9s} {ms * 1e3:8.1f} us  {100 * frac:5.1f} % of the roof  {same}",
                  flush=True)
        del arena, want, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
