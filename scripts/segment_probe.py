#!/usr/bin/env python3
"""tcpck_batch_segment throughput: a device-resident send stream cut into
checksummed images.  Reports payload GiB/s and the HBM traffic rate (stream
read + images written) as % of the 8 TB/s roof, next to a plain device copy of
the same bytes (torch copy_, the copy ceiling) -- back to back, one process.

    python scripts/segment_probe.py [--params 0,1,2,3,8] [--ms 0,8,16,32,64] [--arenas 2]

--arenas 2 takes two payload streams and two image arenas in turn (cold: no
step finds the previous step's lines in the Infinity Cache, as bench.py).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from slot_probe import PEAK, timed  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="0,1,2,3,8")
    ap.add_argument("--ms", default="0")
    ap.add_argument("--cases", default="1460:1504,1024:1056,1448:1488,9000:9040,65532:65568")
    ap.add_argument("--bytes", type=int, default=1536 << 20)
    ap.add_argument("--arenas", type=int, default=1)
    args = ap.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    P = args.bytes
    payloads = []
    for _ in range(args.arenas):
        payload = torch.empty(P, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(payload, 1492, 1492, P // 1492, seed=5)
        payloads.append(payload)
    tmpl = np.arange(32, dtype=np.uint8)
    dst = torch.empty(P, dtype=torch.uint8, device="cuda")
    ms = timed(lambda: dst.copy_(payload), s)
    print(f"device copy of {P / 1e9:.2f} GB: {ms * 1e3:.1f} us = {2 * P / (ms * 1e-3) / PEAK * 100:.1f} % of the roof "
          f"(read + write)", flush=True)
    del dst
    for case in args.cases.split(","):
        seg, stride = map(int, case.split(":"))
        n = (P + seg - 1) // seg
        images_l = [torch.empty(n * stride, dtype=torch.uint8, device="cuda") for _ in range(args.arenas)]
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        traffic = P + n * stride + 2 * n
        row = []
        for p in map(int, args.params.split(",")):
            for m in map(int, args.ms.split(",")):
                prm = p | (m << 16)
                turn = [0]

                def fn():
                    k = turn[0] % args.arenas
                    turn[0] += 1
                    ctx.batch_segment(payloads[k], P, seg, tmpl, 1000, images_l[k], stride, out, param=prm, stream=s)
                t = timed(fn, s)
                row.append(f"p{p}/M{m} {t * 1e3:7.1f} us {P / (t * 1e-3) / GIB:6.0f} GiB/s {traffic / (t * 1e-3) / PEAK * 100:5.1f} %")
        print(f"seg {seg:5d} stride {stride:5d}: " + " | ".join(row), flush=True)
        del images_l, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
