#!/usr/bin/env python3
"""RFC 1071 mode vs the reference mode on the C2 batch: AUTO (rstream for both
now), seg (round 1's RFC path).  % of the 8 TB/s roof, back to back."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from slot_probe import PEAK, timed  # noqa: E402


def main():
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    for L in (1492, 1024, 4096):
        n = 1566572544 // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        row = []
        for name, op, mode, k, p in (("ref auto", 0, 0, 0, 0), ("rfc auto", 0, 1, 0, 0),
                                     ("rfc seg", 0, 1, tcpck.KERNEL_SEG, 0), ("rfc fill auto", 1, 1, 0, 0),
                                     ("ref fill auto", 1, 0, 0, 0)):
            fn = lambda: ctx.batch_fixed_ex(op, a, L, L, n, out, k, p, mode=mode, stream=s)  # noqa
            ms = timed(fn, s)
            row.append(f"{name} {(n * L + 2 * n) / (ms * 1e-3) / PEAK * 100:5.1f} %")
        print(f"{n} x {L} B: " + " | ".join(row), flush=True)
        del a, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
