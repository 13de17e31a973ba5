#!/usr/bin/env python3
"""FILL through rstream: 2-B field stores (variant 20, the policy) against the
64-B field-block write-back (variant 25), back to back, 1.5 GB batches.
% of the 8 TB/s roof in algorithmic bytes (images + 2 B per result)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from slot_probe import PEAK, timed  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    for L in (512, 1024, 1492, 2000, 4096, 9000):
        n = (1566572544 // L)
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=3)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        row = []
        for name, k, p in (("auto", tcpck.KERNEL_AUTO, 0), ("rs20", tcpck.KERNEL_RSTREAM, 20),
                           ("rs25", tcpck.KERNEL_RSTREAM, 25), ("ck20", -1, 20)):
            if k == -1:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, tcpck.KERNEL_RSTREAM, p, stream=s)  # noqa
            else:
                fn = lambda: ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, out, k, p, stream=s)  # noqa
            ms = timed(fn, s)
            row.append(f"{name} {ms * 1e3:6.1f} us {(n * L + 2 * n) / (ms * 1e-3) / PEAK * 100:5.1f} %")
        print(f"FILL {L:5d} B: " + " | ".join(row), flush=True)
        del a, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
