#!/usr/bin/env python3
"""Cost of FILL's in-place field write (tcpck_diag.hip diag_fill_kernel): the bare
stream over 1.5 GB of 1492-B images plus one store per image of W bytes at the
checksum field, W = 0 (none), 2, 4, 16, 32, 64, 128.  Median back-to-back."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    nbytes = 1492 << 20
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(buf, 1492, 1492, 1 << 20, seed=1)
    out = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
    if "--store-policy" in sys.argv:
        # store cache-policy bits (bit 0 sc0, bit 1 nt, bit 4 sc1) on the 2-B and 64-B field stores
        names = {0x1000: "no write", 0x1001: "2 B", 0x1005: "64 B"}
        for w, base in ((2, 0x4000), (64, 0x4100)):
            for aux in (0, 1, 2, 3, 16, 17, 18, 19):
                names[base | aux] = f"{w} B aux {aux}"
    else:
        names = {0x1000 | k: v for k, v in {
            0: "no write", 1: "2 B", 2: "4 B", 3: "16 B", 4: "32 B", 5: "64 B", 6: "128 B",
            7: "2 B, write-only pass", 8: "none, then a 2-B write-only pass"}.items()}
    t = {v: [] for v in names}
    for v in names:
        for _ in range(20):
            ctx.diag_stream(v, buf, nbytes, out, stream=s)
    torch.cuda.synchronize()
    for _ in range(5):
        for v in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                ctx.diag_stream(v, buf, nbytes, out, stream=s)
            e1.record(s)
            torch.cuda.synchronize()
            t[v].append(e0.elapsed_time(e1) / 10)
    for v, name in names.items():
        ms = float(np.median(t[v]))
        print(f"1492-B images, field write {name:8s} {ms:8.4f} ms  read rate {nbytes / ms / 1e6:7.1f} GB/s "
              f"({nbytes / ms / 1e6 / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
