#!/usr/bin/env python3
"""Back-to-back vs isolated launch time for kernel choices on one workload:
the bench times K launches in a row (one event bracket), the probes time one
launch at a time.  python scripts/b2b_probe.py [--what c3|c2]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="c3")
    ap.add_argument("--params", default="")
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
        kern = tcpck.KERNEL_VVSTREAM
        lmin, lmax = int(ln.min()), int(ln.max())
        params = [int(p, 0) for p in args.params.split(",")] if args.params else \
            [4, 3 | (32 << 16), 2 | (32 << 16), 2 | (16 << 16), 2 | (8 << 16), 1 | (1 << 16)]

        def run(p):
            if p < 0:
                ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, total_bytes=total, min_len=lmin,
                              max_len=lmax, packed=True, stream=s)
            else:
                ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, kern, p, packed=True,
                                 total_bytes=total, stream=s)
        nbytes = total + 2 * n
        params = [-1] + params
    else:
        L, n = 1492, 1 << 20
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        kern = tcpck.KERNEL_RSTREAM
        params = [int(p, 0) for p in args.params.split(",")] if args.params else \
            [0, 0 | (8 << 16), 0 | (32 << 16), 10 | (8 << 16), 10 | (32 << 16)]

        def run(p):
            if p < 0:
                ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out, stream=s)
            else:
                ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, kern, p, stream=s)
        nbytes = n * L + 2 * n
        params = [-1] + params
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    iso = {p: [] for p in params}
    b2b = {p: [] for p in params}
    for _ in range(4):
        for p in params:
            for _ in range(5):
                run(p)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                run(p)
            e1.record(s)
            torch.cuda.synchronize()
            b2b[p].append(e0.elapsed_time(e1) / 20)
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                run(p)
                e1.record(s)
                torch.cuda.synchronize()
                iso[p].append(e0.elapsed_time(e1))
    for p in params:
        bi, bb = float(np.median(iso[p])), float(np.median(b2b[p]))
        name = "AUTO" if p < 0 else f"variant {p & 0xFF} x{p >> 16}"
        print(f"{args.what} {name:18s} isolated {bi:.4f} ms ({nbytes / bi / 1e6 / 80:.1f}%)  "
              f"back-to-back {bb:.4f} ms ({nbytes / bb / 1e6 / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
