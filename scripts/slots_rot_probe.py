#!/usr/bin/env python3
"""Receive slots (sstream over an offset list): the waves in flight start their
runs together at equally spaced slots (32 images of 2048 B: 64 KiB apart) and
advance at similar rates.  RunArgs::rot (sstream param bits 8-15) streams wave
w's run from image (w rot) mod n on, wrapping.  VERIFY and CHECKSUM on the
bench's slots layout (1M x 2048-B slots, 96/608/1492-B images) and on 1536 /
4096-B slots, against rot 0; results compared.  Three interleaved passes,
median.  Round 3 (profiles/r03/slots_rot_probe.log): bit-exact, but every
multiplier ran 158 us against 133 us in order, at 1536 / 2048 / 4096-B slots;
the RunArgs::rot form was removed (the script needs it back to run)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=3):
    for _ in range(5):
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
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(42)
    n = 1 << 20
    mix = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    img = int(mix.astype(np.int64).sum())
    lo, hi = int(mix.min()), int(mix.max())
    for slot in (2048, 1536, 4096):
        off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
        a = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(mix).cuda()
        tcpck.synth_var(a, d_off, d_ln, hi, n, seed=42)
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        cs = torch.empty(n, dtype=torch.int16, device="cuda")
        kw = dict(total_bytes=img, min_len=lo, max_len=hi, sorted=True, stream=s)
        ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, **kw)
        ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, cs, **kw)
        torch.cuda.synchronize()
        ref_ok, ref_cs = ok.clone(), cs.clone()
        rots = [0, 1, 3, 5, 13, 29, 37, 61]
        tv = {r: [] for r in rots}
        same = True
        for _ in range(3):
            for r in rots:
                p = r << 8
                tv[r].append(b2b(lambda: ctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok,
                                                          kernel=tcpck.KERNEL_SSTREAM, param=p, **kw), s))
                ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, cs, kernel=tcpck.KERNEL_SSTREAM, param=p, **kw)
                torch.cuda.synchronize()
                same = same and torch.equal(ok, ref_ok) and torch.equal(cs, ref_cs)
        for r in rots:
            ms = float(np.median(tv[r]))
            print(f"slot {slot:5d}  rot {r:3d}  VERIFY {ms * 1e3:7.1f} us  {(img + n) / ms / 1e6 / 80:5.1f} % of the roof  "
                  f"(passes {', '.join(f'{t * 1e3:.1f}' for t in tv[r])})", flush=True)
        print(f"slot {slot:5d}  results identical (VERIFY and CHECKSUM): {same}", flush=True)
        del a


if __name__ == "__main__":
    main()
