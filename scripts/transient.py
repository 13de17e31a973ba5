#!/usr/bin/env python3
"""Launch-duration time series over a long back-to-back run (per-launch HIP
events): how long the clock/power transient after the GPU goes busy lasts,
i.e. how many warm-up launches the bench needs before its timed region.
    python scripts/transient.py [--what c3|c2] [--n 400]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="c3")
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--idle", type=float, default=2.0, help="idle seconds before the series")
    args = ap.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    if args.what == "c3":
        from synth_np import mixed_layout
        off, ln, total = mixed_layout(4 << 20, seed=42)
        n = ln.size
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
        lmin, lmax = int(ln.min()), int(ln.max())

        def run():
            ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, total_bytes=total, min_len=lmin,
                          max_len=lmax, packed=True, stream=s)
        nbytes = total + 2 * n
    else:
        L, n = (1492, 1 << 20) if args.what == "c2" else (65536, 256 << 10)
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)

        def run():
            ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out, stream=s)
        nbytes = n * L + 2 * n
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    time.sleep(args.idle)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.n)]
    for e0, e1 in ev:
        e0.record(s)
        run()
        e1.record(s)
    torch.cuda.synchronize()
    d = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
    t = np.cumsum(d + 0.010)
    for i in range(0, args.n, 10):
        seg = d[i:i + 10]
        print(f"{args.what} launches {i:4d}-{i + 9:4d} (t={t[i]:7.1f} ms) mean {seg.mean():.4f} ms "
              f"min {seg.min():.4f} max {seg.max():.4f}  {nbytes / seg.mean() / 1e6 / 80:.1f}%", flush=True)


if __name__ == "__main__":
    main()
