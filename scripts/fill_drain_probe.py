#!/usr/bin/env python3
"""Where does FILL's extra time go?  

C2's layout (1M x 1492-B images, fixed stride).  AUTO's FILL is rstream's
stream writing only the results, then launch_patch_fields rewriting each
field's 64-B block (variant 25).  Its stream ran 246 us against CHECKSUM's
211 us.  Phases, each back to back after a settle, separated by a 50-ms host
pause so scripts/fill_drain_summary.py can cut the kernel trace:

  stream         CHECKSUM (rstream 20, results to out[])
  fill           AUTO FILL: stream (results only) + block pass
  fill+sleepS    the same with an S-us spin kernel after the block pass (no memory traffic)
  stream+sleepS  control: CHECKSUM + the same spin
  patch          the block pass alone (TCPCK_KERNEL_PATCH, tcpck_probe.h)
  instream       FILL with the 2-B field stores inside the stream (rstream 20)
  spB            CHECKSUM stream, then the block pass alone with its stores'
                 cache bits B - 1 (sc0 1 | nt 2 | sc1 4; sp0: plain C++ store)

Run under `rocprofv3 --kernel-trace` (per-kernel durations) and, separately,
`--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (where the field writes leave L2)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--phases", default="stream,fill,fill+sleep20,fill+sleep100,stream+sleep20,patch,instream,fill")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--settle-ms", type=float, default=200)
    a = ap.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    L, n = 1492, 1 << 20
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=42)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    R = tcpck.KERNEL_RSTREAM
    # spin-kernel cycles per us (torch.cuda._sleep counts s_memtime ticks): calibrate once
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    torch.cuda._sleep(1_000_000)
    e1.record(s)
    torch.cuda.synchronize()
    per_us = 1_000_000 / (e0.elapsed_time(e1) * 1e3)

    def step_fn(ph):
        parts = ph.split("+")
        base, sleep_us = parts[0], 0
        if len(parts) > 1:
            sleep_us = int(parts[1].replace("sleep", ""))
        if base == "stream":
            f = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, R, 20, stream=s)
        elif base == "fill":
            f = lambda: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, out, stream=s)
        elif base == "patch":
            f = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, tcpck.KERNEL_PATCH, 0, stream=s)
        elif base.startswith("sp"):  # stream, then the block pass with store bits (sp0 plain, spB: 1 + bits)
            bits = int(base[2:])

            def f():
                ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, R, 20, stream=s)
                ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, tcpck.KERNEL_PATCH, bits, stream=s)
        elif base.startswith("sg"):  # stream, then the probe pass: sgG_B (granularity G, bits B - 1)
            g, b = base[2:].split("_")
            prm = (int(g) << 4) | int(b)

            def f():
                ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, R, 20, stream=s)
                ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, tcpck.KERNEL_PATCH, prm, stream=s)
        elif base == "instream26":  # in-stream 2-B field stores, sc0 sc1 nt
            f = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 26, stream=s)
        elif base == "block":  # rstream variant 27: whole 64-B field blocks written from the stream
            f = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 27, stream=s)
        elif base == "blockend":  # variant 28: the run's blocks stored after its last load
            f = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 28, stream=s)
        elif base == "instream":
            f = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, out, R, 20, stream=s)
        else:
            raise SystemExit(f"unknown phase {ph}")
        if not sleep_us:
            return f
        cyc = int(sleep_us * per_us)

        def g():
            f()
            torch.cuda._sleep(cyc)
        return g

    print(f"spin: {per_us:.1f} cycles/us", flush=True)
    for ph in a.phases.split(","):
        fn = step_fn(ph)
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < a.settle_ms:
            for _ in range(4):
                fn()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.steps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        print(f"{ph:16s} {e0.elapsed_time(e1) / a.steps * 1e3:8.1f} us per step (HIP events, {a.steps} steps)",
              flush=True)
        time.sleep(0.05)  # phase boundary for the trace summary


if __name__ == "__main__":
    main()
