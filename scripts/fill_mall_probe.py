#!/usr/bin/env python3
"""FILL on C2's layout: can the field pass write whole 64-B blocks without
reading HBM?  (round 4, probe library)

AUTO's FILL is rstream's deferred stream (results only, variant 25's stream)
then one write-through 2-B store per field; a 2-B store makes the memory side
read the 64-B block to merge it (profiles/r03/fill_blind.log: blind 64-B
writes 20 us per 1M fields, 2-B stores 38-42 us).  Here the stream reads each
field's 64-B block with the DEFAULT cache policy (rstream 29; the rest nt), so
the block may still be cached -- C2's 1M field lines are 128 MB, half the
memory-side Infinity Cache -- when a block pass reads it and writes it back
whole (TCPCK_KERNEL_PATCH form 0).  Sequences, each back to back (median of
rounds of 20 steps after a settle):

  auto        AUTO FILL (product)
  s30+p28     the policy's deferred stream alone, then the product's 2-B
              write-through pass (== auto, as two calls)
  s29+p28     field blocks default-policy, then the 2-B pass
  s29+pB      field blocks default-policy, then the 64-B block pass with
              store bits B (TCPCK_KERNEL_PATCH param: 0x00 plain, 0x03 nt,
              0x05 sc1, 0x07 sc1 nt... 0x08 sc0 sc1 nt)
  s30+p08     control: the block pass without the default-policy reads
  s29 / s30 / checksum   the streams alone
  .../C       the same over the batch in C pieces, each piece's pass right
              after its stream (the pieces' field lines fit the caches)

Every FILL sequence's arena is compared with AUTO's."""
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
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    L, n = 1492, 1 << 20
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=42)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    R, P = tcpck.KERNEL_RSTREAM, tcpck.KERNEL_PATCH
    algo = n * L + 4 * n  # image bytes + fields + results

    def seq(stream_v, patch_p, chunks=1):
        """The stream then the pass, over the batch in `chunks` pieces (each
        piece's pass right after its stream: its blocks read at most 1/chunks
        of the batch ago)."""
        m = n // chunks
        a0, o0 = arena.data_ptr(), out.data_ptr()

        def f():
            for c in range(chunks):
                a, o = a0 + c * m * L, o0 + 2 * c * m
                ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, m, o, R, stream_v, stream=s)
                if patch_p is not None:
                    ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, m, o, P, patch_p, stream=s)
        return f

    ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, out, stream=s)
    torch.cuda.synchronize()
    want = arena.clone()
    cases = [("auto", lambda: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, out, stream=s), True),
             ("s30+p28", seq(30, 0x28), True), ("s29+p28", seq(29, 0x28), True),
             ("s29+p08", seq(29, 0x08), True), ("s29+p00", seq(29, 0x00), True), ("s29+p03", seq(29, 0x03), True),
             ("s29+p05", seq(29, 0x05), True), ("s29+p07", seq(29, 0x07), True), ("s30+p08", seq(30, 0x08), True),
             ("s30+p00", seq(30, 0x00), True),
             ("s29+p08/4", seq(29, 0x08, 4), True), ("s29+p08/8", seq(29, 0x08, 8), True),
             ("s30+p28/8", seq(30, 0x28, 8), True), ("s29+p28/8", seq(29, 0x28, 8), True),
             ("s29", seq(29, None), False), ("s30", seq(30, None), False),
             ("checksum", lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s), False),
             ("auto", lambda: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, out, stream=s), True)]
    for label, fn, full in cases:
        ms = b2b(fn, s)
        same = ""
        if full:
            torch.cuda.synchronize()
            same = "arena == AUTO's" if torch.equal(arena, want) else "ARENA DIFFERS"
            arena.copy_(want)
        frac = algo / (ms * 1e-3) / 8e12
        print(f"C2 FILL  {label:9s} {ms * 1e3:8.1f} us  {100 * frac:5.1f} % of the roof  {same}", flush=True)


if __name__ == "__main__":
    main()
