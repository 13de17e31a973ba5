#!/usr/bin/env python3
"""Slotted (gapped) layouts -- the device-resident receive arena: images in
fixed-size slots (NIC/recvmmsg slots of S bytes), fixed or variable length.
Times AUTO and explicit kernels back to back (median of rounds) and reports
image bytes / time as % of the 8 TB/s roof, plus the 128-B lines the images
touch (the least HBM traffic any kernel can move) as % of the roof.

    python scripts/slot_probe.py [--ops checksum,verify,fill] [--kernels auto,seg,slot]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

PEAK = 8.0e12
OPS = {"checksum": tcpck.OP_CHECKSUM, "verify": tcpck.OP_VERIFY, "fill": tcpck.OP_FILL}


def timed(fn, s, reps=20, rounds=5, settle_ms=60.0):
    import time
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:  # the idle GPU's clock ramp (profiles/DESIGN_history_r01-r04.md section 4)
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


def lines_touched(off, ln):
    a = off.astype(np.int64)
    e = a + ln.astype(np.int64)
    return int(((e + 127) // 128 - a // 128).sum()) * 128


def layouts(target_bytes):
    rng = np.random.default_rng(7)
    out = []
    for S, L in ((2048, 1492), (1536, 1492), (4096, 1492), (2048, 1024), (256, 96), (16384, 9000)):
        n = target_bytes // S
        out.append((f"fixed {L} in {S}-B slots", S, L, n, None, None))
    for S, mix in ((2048, (96, 608, 1492)), (1536, (96, 608, 1492)), (2048, (32, 1492)), (2048, (1492,)),
                   (1600, (64, 200, 576, 1024, 1492))):
        n = target_bytes // S
        ln = np.asarray(mix, np.uint32)[rng.integers(0, len(mix), n)]
        off = np.arange(n, dtype=np.uint64) * np.uint64(S)
        out.append((f"var {'/'.join(map(str, mix))} in {S}-B slots", S, None, n, off, ln))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="checksum,verify,fill")
    ap.add_argument("--kernels", default="auto,seg,ss,ss4,ss8")
    ap.add_argument("--bytes", type=int, default=1 << 31)
    args = ap.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    kern = {"auto": (K.KERNEL_AUTO, 0), "seg": (K.KERNEL_SEG, 0)}
    kern["ss"] = (K.KERNEL_SSTREAM, 0)
    kern["ss4"] = (K.KERNEL_SSTREAM, 1)
    kern["ss8"] = (K.KERNEL_SSTREAM, 2)
    for name, S, L, n, off, ln in layouts(args.bytes):
        arena = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        if off is None:
            K.synth_fixed(arena, S, L, n, seed=3)
            img = n * L
            o = np.arange(n, dtype=np.uint64) * np.uint64(S)
            lt = lines_touched(o, np.full(n, L, np.uint32))
        else:
            d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            K.synth_var(arena, d_off, d_ln, int(ln.max()), n, seed=3)
            img = int(ln.astype(np.int64).sum())
            lt = lines_touched(off, ln)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        for op in args.ops.split(","):
            for kn in args.kernels.split(","):
                if kn not in kern:
                    continue
                k, p = kern[kn]
                if off is None:
                    fn = lambda: ctx.batch_fixed_ex(OPS[op], arena, S, L, n, out, k, p, stream=s)  # noqa: E731
                else:
                    fn = lambda: ctx.batch_var_ex(OPS[op], arena, d_off, d_ln, n, out, k, p,  # noqa: E731
                                                  total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()),
                                                  sorted=True, stream=s)
                try:
                    ms = timed(fn, s)
                except tcpck.TcpckError as e:
                    print(f"{name:42s} {op:8s} {kn:5s} n/a ({e})", flush=True)
                    continue
                print(f"{name:42s} {op:8s} {kn:5s} {ms * 1e3:9.1f} us  image bytes {img / (ms * 1e-3) / PEAK * 100:5.1f} %"
                      f"  lines {lt / (ms * 1e-3) / PEAK * 100:5.1f} %  (image/line bytes {img / lt:.3f})", flush=True)
        del arena, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
