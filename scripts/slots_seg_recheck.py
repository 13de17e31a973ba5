#!/usr/bin/env python3
"""Re-check of the AUTO grids on the final binary for two bench lines: the
`slots` ring (1M 2048-B slots, 96/608/1492-B images, offset list, VERIFY on
sstream: U4/U8, block orders, M) and `segment` (1.5 GiB stream -> 1460-B
segments in 1504-B slots: variant, M).  Results compared with AUTO's.  Back to
back, median of rounds."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
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
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    # slots
    n = 1 << 20
    rng = np.random.default_rng(42)
    ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(2048)
    a = torch.empty(n * 2048, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    img = int(ln.astype(np.int64).sum())
    kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), sorted=True, stream=s)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ref = torch.empty(n, dtype=torch.uint8, device="cuda")
    ms = b2b(lambda: ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, n, ref, **kw), s)
    print(f"slots AUTO                  {ms * 1e3:7.1f} us  {(img + n) / ms / 1e6 / 80:5.1f} %", flush=True)
    for v, vn in ((0, "policy"), (2, "U8 XCD"), (1, "U4 XCD"), (9, "U4 scatter"), (10, "U8 scatter"), (5, "U4 default")):
        for m in (2, 4, 8, 16):
            p = v | (m << 16)
            ms = b2b(lambda: ctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, tcpck.KERNEL_SSTREAM, p, **kw), s)
            torch.cuda.synchronize()
            print(f"slots {vn:10s} M{m:<3d}        {ms * 1e3:7.1f} us  {(img + n) / ms / 1e6 / 80:5.1f} %  "
                  f"same: {torch.equal(ok, ref)}", flush=True)
    del a
    # segment
    P, seg, stride = 1536 << 20, 1460, 1504
    payload = torch.empty(P, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(payload, 1492, 1492, P // 1492, seed=42)
    cnt = (P + seg - 1) // seg
    images = torch.empty(cnt * stride, dtype=torch.uint8, device="cuda")
    out = torch.empty(cnt, dtype=torch.int16, device="cuda")
    sref = torch.empty(cnt, dtype=torch.int16, device="cuda")
    hdr = np.zeros(32, np.uint8)
    hdr[0:4], hdr[4:8], hdr[12:14], hdr[14:16] = [127, 0, 0, 1], [127, 0, 0, 1], [0x3C, 0x8C], [0x3C, 0x8D]
    rw = P + cnt * 32 + P
    ms = b2b(lambda: ctx.batch_segment(payload, P, seg, hdr, 1001, images, stride, sref, stream=s), s)
    print(f"segment AUTO                {ms * 1e3:7.1f} us  {rw / ms / 1e6 / 80:5.1f} % (read + write)", flush=True)
    for v, vn in ((0, "policy"), (1, "U8"), (2, "default st"), (8, "dflt order")):
        for m in (16, 32, 64, 128):
            p = v | (m << 16)
            ms = b2b(lambda: ctx.batch_segment(payload, P, seg, hdr, 1001, images, stride, out, param=p, stream=s), s)
            torch.cuda.synchronize()
            print(f"segment {vn:10s} M{m:<3d}      {ms * 1e3:7.1f} us  {rw / ms / 1e6 / 80:5.1f} %  "
                  f"same: {torch.equal(out, sref)}", flush=True)


if __name__ == "__main__":
    main()
