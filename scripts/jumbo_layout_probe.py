#!/usr/bin/env python3
"""Jumbo images outside the packed fixed layout: gapped fixed slots (e.g. 9000-B
images in 9216-B receive slots) and packed variable batches of jumbo images.
AUTO (seg with the length-based W shape above 4 / 16 KiB) against vvstream's
policy (variant 28: gapped slots streamed as virtual images, packed variable as
one run).  CHECKSUM, back to back after a clock settle; every candidate checked
against seg's results first.

    python scripts/jumbo_layout_probe.py [--fill]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck as K  # noqa: E402
from xcd_probe import b2b  # noqa: E402

PEAK = 8000.0


def report(label, fn, nbytes, s, chk):
    fn()
    torch.cuda.synchronize()
    chk()
    ms = b2b(fn, s, reps=20, rounds=3)
    gbs = nbytes / (ms * 1e-3) / 1e9
    print(f"{label:44s} {ms:.4f} ms {gbs:7.1f} GB/s ({100 * gbs / PEAK:5.1f}%)", flush=True)


def main():
    op = K.OP_FILL if "--fill" in sys.argv else K.OP_CHECKSUM  # FILL: idempotent on the filled arena
    ctx = K.Context(0)
    s = torch.cuda.current_stream()
    for L, S in ((4500, 4608), (9000, 9216), (9000, 9088), (20000, 20480), (40000, 40960)):
        n = int(1.5e9) // S
        a = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, S, L, n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(op, a, S, L, n, ref, K.KERNEL_SEG, 0)
        snap = a.clone()

        def chk():
            assert torch.equal(out, ref) and torch.equal(a, snap)
        report(f"gapped {L}/{S} auto", lambda: ctx.batch_fixed(op, a, S, L, n, out, stream=s), n * L + 2 * n, s, chk)
        report(f"gapped {L}/{S} vvstream 28", lambda: ctx.batch_fixed_ex(op, a, S, L, n, out, K.KERNEL_VVSTREAM, 28,
                                                                       stream=s), n * L + 2 * n, s, chk)
        del snap
        del a, ref, out
        torch.cuda.empty_cache()
    rng = np.random.default_rng(5)
    for pay in ((8968,), (4468, 8968), (8968, 19968, 39968), (19968,), (39968, 60000)):
        n = int(1.5e9) // (int(np.mean(pay)) + 32)
        ln = (np.asarray(pay, np.uint32)[rng.integers(0, len(pay), n)] + 32).astype(np.uint32)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        total = int(off[-1] + ln[-1])
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        K.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(op, a, d_off, d_ln, n, ref, K.KERNEL_SEG, 0)
        snap = a.clone()
        lay = dict(packed=True, total_bytes=total, min_len=int(ln.min()), max_len=int(ln.max()))

        def chk():
            assert torch.equal(out, ref) and torch.equal(a, snap)
        lab = "/".join(str(p + 32) for p in pay)
        report(f"packed var {lab} auto", lambda: ctx.batch_var(op, a, d_off, d_ln, n, out, stream=s, **lay),
               total + 2 * n, s, chk)
        report(f"packed var {lab} vvstream 28", lambda: ctx.batch_var_ex(op, a, d_off, d_ln, n, out,
                                                                         K.KERNEL_VVSTREAM, 28, stream=s, **lay),
               total + 2 * n, s, chk)
        del a, ref, out, d_off, d_ln, snap
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
