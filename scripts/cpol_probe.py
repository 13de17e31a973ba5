#!/usr/bin/env python3
"""Load cache-policy bits on the bare stream (tcpck_diag.hip diag_cpol_kernel):
aux = sc0 (1) | nt (2) | sc1 (16), 1.57 GB and 17 GB, median back-to-back.
Round 5: the 1.57-GB case also cold -- consecutive launches alternate between
two 1.57-GB regions 4 GiB apart, so none finds the previous one's lines in the
Infinity Cache (scripts/arena_reuse_probe.py)."""
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
    buf = torch.empty(17 << 30, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(buf, 65536, 65536, (17 << 30) // 65536, seed=1)
    out = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
    auxes = {0: "default", 2: "nt", 1: "sc0", 3: "sc0 nt", 16: "sc1", 18: "sc1 nt", 17: "sc0 sc1", 19: "sc0 sc1 nt"}
    for nbytes, reps, cold in ((1566572544, 10, False), (1566572544, 10, True), (17 << 30, 3, False)):
        t = {a: [] for a in auxes}
        srcs = [buf, buf[4 << 30:]] if cold else [buf]
        for a in auxes:
            for i in range(reps * 2):
                ctx.diag_stream(0x2000 | a, srcs[i % len(srcs)], nbytes, out, stream=s)
        torch.cuda.synchronize()
        for _ in range(5):
            for a in auxes:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for i in range(reps):
                    ctx.diag_stream(0x2000 | a, srcs[i % len(srcs)], nbytes, out, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                t[a].append(e0.elapsed_time(e1) / reps)
        for a, name in auxes.items():
            ms = float(np.median(t[a]))
            print(f"{nbytes / 1e9:6.2f} GB {'cold' if cold else 'warm'} loads {name:12s} {ms:8.4f} ms {nbytes / ms / 1e6:7.1f} GB/s "
                  f"({nbytes / ms / 1e6 / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
