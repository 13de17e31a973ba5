#!/usr/bin/env python3
"""rvstream (rstream's scalar walk over packed offset lists, round 5) against
AUTO's kernel (vvstream, or seg above 32 KiB) on packed variable batches of
several densities, measured cold: two identical batches taken in turn
(scripts/arena_reuse_probe.py).  CHECKSUM; ~1.5-3 GB per batch; back-to-back
launches, median of 5 rounds; results compared with AUTO's.

  --mixes NAME[,NAME]   c3, u64_256, u256_1024, u512_1536, c1492, u2k_8k, u8k_24k
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402

MIXES = {"c3": None, "u64_256": (64, 256), "u256_1024": (256, 1024), "u512_1536": (512, 1536), "c1492": (1492, 1492),
         "u2k_8k": (2048, 8192), "u8k_24k": (8192, 24576)}


def b2b(fn, s, reps=20, rounds=5):
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
    p.add_argument("--mixes", default=",".join(MIXES))
    p.add_argument("--forms", default="0,1,2", help="rvstream variants (0 policy U4, 1 U8, 2 U2, 3 U4 + run table, 4 U2 + run table)")
    p.add_argument("--ms", default="0", help="rvstream grid multipliers (0 = by size)")
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(7)
    for name in args.mixes.split(","):
        spec = MIXES[name]
        if spec is None:
            off, ln, total = synth_np.mixed_layout(4 << 20, seed=42)
        else:
            lo, hi = spec
            n = int((2 << 30) // ((lo + hi) // 2))
            ln = (rng.integers(lo // 2, hi // 2 + 1, n) * 2).astype(np.uint32)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
            total = int(off[-1]) + int(ln[-1])
        n = ln.size
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        arenas = []
        for _ in range(2):
            a = torch.empty(total, dtype=torch.uint8, device="cuda")
            tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
            arenas.append(a)
        img = int(ln.astype(np.int64).sum())
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
        forms = [("AUTO warm-up", None), ("AUTO", None)]
        if name == "c1492":  # the same bytes as a fixed stride: AUTO's fixed kernel (rstream)
            forms.append(("fixed stride AUTO", -1))
        for v in (int(x) for x in args.forms.split(",")):
            for m in (int(x) for x in args.ms.split(",")):
                forms.append((f"rvstream {v} M{m or 'policy'}", v | (m << 16)))
        ref = None
        for label, prm in forms:
            turn = [0]

            def step():
                a = arenas[turn[0] % 2]
                turn[0] += 1
                if prm == -1:
                    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, 1492, 1492, n, out, stream=s)
                elif prm is None:
                    ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, **kw)
                else:
                    ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_RVSTREAM, prm, **kw)
            ms = b2b(step, s)
            torch.cuda.synchronize()
            same = ""
            if ref is None:
                ref = out.clone()
            else:
                same = f"  results == AUTO's: {torch.equal(out, ref)}"
            print(f"{name:10s} mean {img // n:5d} B {label:22s} {ms * 1e3:8.1f} us  "
                  f"{(img + 2 * n) / ms / 1e6 / 80:5.1f} %{same}", flush=True)
        del arenas, out
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
