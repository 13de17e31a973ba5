#!/usr/bin/env python3
"""Raw streaming rate of the diag micro-kernels (tcpck_diag.hip): per-step
overhead and per-lane stride experiments.  Interleaved rounds, median GB/s."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402

NAMES = {0: "1x16B U4 scan", 1: "1x16B U4 noscan", 2: "2x16B U2 scan", 3: "2x16B U2 noscan",
         4: "4x16B U1 scan", 5: "2x16B U4 scan", 6: "4x16B U2 scan", 7: "1x16B U2 scan",
         8: "dyn U4 16K units", 9: "dyn U4 32K units", 10: "dyn U4 8K units", 11: "dyn U8 32K units",
         4 << 8: "1x16B U4 scan x4", 8 << 8: "1x16B U4 scan x8", 16 << 8: "1x16B U4 scan x16",
         32 << 8: "1x16B U4 scan x32"}


def main():
    ctx = tcpck.Context(0, probe=True)
    stream = torch.cuda.current_stream()
    buf = torch.empty(17 << 30, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(buf, 65536, 65536, (17 << 30) // 65536, seed=1)
    out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    for nbytes in (1566572544, 17 << 30):
        times = {v: [] for v in NAMES}
        for _ in range(4):
            for v in NAMES:
                ctx.diag_stream(v, buf, nbytes, out, stream=stream)
                for _ in range(5):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record(stream)
                    ctx.diag_stream(v, buf, nbytes, out, stream=stream)
                    e.record(stream)
                    torch.cuda.synchronize()
                    times[v].append(s.elapsed_time(e))
        for v, name in NAMES.items():
            med = float(np.median(times[v]))
            print(f"{nbytes / 1e9:6.2f} GB {name:18s} {med:8.4f} ms {nbytes / med / 1e6:7.1f} GB/s "
                  f"({nbytes / med / 1e6 / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
