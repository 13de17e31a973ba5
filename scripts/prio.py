#!/usr/bin/env python3
"""rstream arbitration experiments: wave priority by slot and occupancy caps.
Interleaved rounds in one process; median GB/s.  Then per-wave stamps of the
graded-priority build."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402

R = tcpck.KERNEL_RSTREAM
VARIANTS = [("U4", 0), ("U2", 1), ("U8", 2), ("U4 prio-graded", 4), ("U4 prio-half", 5), ("U8 prio-graded", 6),
            ("U2 prio-graded", 8), ("U8 cap4", 2 | 4 << 8), ("U8 cap4 prio", 6 | 4 << 8), ("U4 cap6", 0 | 6 << 8),
            ("U4 cap4", 0 | 4 << 8), ("U8 cap2", 2 | 2 << 8), ("U4 cap6 prio", 4 | 6 << 8)]


def main():
    ctx = tcpck.Context(0, probe=True)
    stream = torch.cuda.current_stream()
    L = 1492
    nmax = (16 << 30) // L
    arena = torch.empty(nmax * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, nmax, seed=9)
    out = torch.empty(nmax, dtype=torch.int16, device="cuda")
    ref = torch.empty_like(out)
    for n in (1 << 20, nmax):
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, ref, tcpck.KERNEL_SEG, 2, stream=stream)
        times = {v[0]: [] for v in VARIANTS}
        for name, p in VARIANTS:
            out.zero_()
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, R, p, stream=stream)
            torch.cuda.synchronize()
            assert torch.equal(out[:n], ref[:n]), name
        for _ in range(4):
            for name, p in VARIANTS:
                for _ in range(5):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record(stream)
                    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, R, p, stream=stream)
                    e.record(stream)
                    torch.cuda.synchronize()
                    times[name].append(s.elapsed_time(e))
        algo = n * L + 2 * n
        for name, _ in VARIANTS:
            med = float(np.median(times[name]))
            print(f"{algo / 1e9:6.2f} GB  {name:16s} {med:8.4f} ms  {algo / med / 1e6:7.1f} GB/s "
                  f"({algo / med / 1e6 / 80:.1f}%)", flush=True)
    # stamps with graded priority
    n = 1 << 20
    dbg = torch.zeros(4 * 16384, dtype=torch.int64, device="cuda")
    ctx.set_debug(dbg)
    for stamp_variant in (3, 7):
        dbg.zero_()
        for _ in range(2):
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, R, stamp_variant, stream=stream)
        torch.cuda.synchronize()
        d = dbg.cpu().numpy().reshape(-1, 4)
        d = d[d[:, 1] > 0]
        t0 = d[:, 0].min()
        st, en = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0
        slot = d[:, 2] & 0xF
        row = " ".join(f"{int(k)}:{(en - st)[slot == k].mean():.0f}" for k in np.unique(slot))
        print(f"variant {stamp_variant}: end median/p90/max {np.median(en):.1f}/{np.percentile(en, 90):.1f}/"
              f"{en.max():.1f} us; mean duration by slot {row}", flush=True)
    ctx.set_debug(None)


if __name__ == "__main__":
    main()
