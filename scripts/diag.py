#!/usr/bin/env python3
"""Timing ablations of the stream kernel (include/tcpck_tuning.h variants 4-7):
128-B aligned runs, boundary handling removed, scan removed.  Variants 6/7
produce wrong checksums by design (timing only).  Interleaved rounds in one
process; median GB/s per variant and batch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

VARIANTS = [("stream U4 a16", tcpck.KERNEL_STREAM, 0), ("stream U4 a128", tcpck.KERNEL_STREAM, 4),
            ("stream U2 a128", tcpck.KERNEL_STREAM, 5), ("scan only a128", tcpck.KERNEL_STREAM, 6),
            ("pure a128", tcpck.KERNEL_STREAM, 7), ("span T16", tcpck.KERNEL_SPAN, 16),
            ("seg G64U4", tcpck.KERNEL_SEG, 3), ("seg G16U6", tcpck.KERNEL_SEG, 2),
            ("fstream U4", tcpck.KERNEL_FSTREAM, 0), ("fstream U2", tcpck.KERNEL_FSTREAM, 1 << 16),
            ("rstream U4", tcpck.KERNEL_RSTREAM, 0), ("rstream U2", tcpck.KERNEL_RSTREAM, 1),
            ("rstream U8", tcpck.KERNEL_RSTREAM, 2)]


def main():
    ctx = tcpck.Context(0)
    stream = torch.cuda.current_stream()
    arena = torch.empty(17 << 30, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, 65536, 65536, (17 << 30) // 65536, seed=3)
    out = torch.empty(12 << 20, dtype=torch.int16, device="cuda")
    stamps(ctx, arena, out, stream)
    for L, total in ((1492, 1 << 30), (1492, int(1.5 * (1 << 30))), (1492, 16 << 30), (65536, 16 << 30)):
        n = total // L
        times = {v[0]: [] for v in VARIANTS}
        for _ in range(4):
            for name, k, p in VARIANTS:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, k, p, stream=stream)
                fn()
                for _ in range(5):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record(stream)
                    fn()
                    e.record(stream)
                    torch.cuda.synchronize()
                    times[name].append(s.elapsed_time(e))
        algo = n * L + 2 * n
        for name, _, _ in VARIANTS:
            med = float(np.median(times[name]))
            print(f"L={L:5d} {algo / 1e9:6.2f} GB  {name:15s} {med:8.4f} ms  {algo / med / 1e6:7.1f} GB/s "
                  f"({algo / med / 1e6 / 80:.1f}%)", flush=True)


def stamps(ctx, arena, out, stream):
    """Per-wave start/end times of one C2-sized rstream launch (tail analysis)."""
    L, n = 1492, 1 << 20
    dbg = torch.zeros(2 * 256 * 8 * 4 * 2, dtype=torch.int64, device="cuda")
    ctx.set_debug(dbg)
    for _ in range(3):
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, tcpck.KERNEL_RSTREAM, 3, stream=stream)
    torch.cuda.synchronize()
    ctx.set_debug(None)
    d = dbg.cpu().numpy().reshape(-1, 2)
    d = d[d[:, 1] > 0]
    t0 = d[:, 0].min()
    st, en = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0  # 100 MHz -> us
    dur = en - st
    print(f"stamps: waves {len(d)}  start max {st.max():.2f} us  end min/median/p99/max "
          f"{en.min():.1f}/{np.median(en):.1f}/{np.percentile(en, 99):.1f}/{en.max():.1f} us  "
          f"wave duration min/median/max {dur.min():.1f}/{np.median(dur):.1f}/{dur.max():.1f} us", flush=True)
    wid = np.nonzero(dbg.cpu().numpy().reshape(-1, 2)[:, 1] > 0)[0]
    by = {}
    for x in range(8):
        sel = ((wid // 4) % 8) == x
        by[x] = float(np.median(en[sel])) if sel.any() else 0.0
    print("stamps: median end by block-id mod 8 (XCD group):", {k: round(v, 1) for k, v in by.items()}, flush=True)


if __name__ == "__main__":
    main()
