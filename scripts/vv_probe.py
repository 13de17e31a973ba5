#!/usr/bin/env python3
"""C3 on vvstream by variant (0/1 byte split U4/U8, 2/3 count split, 4 policy) and grid
oversubscription.  Bit-exact check against the seg kernel first; then median
HIP-event launch time over interleaved rounds."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from synth_np import mixed_layout  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    off, ln, total = mixed_layout(4 << 20, seed=42)
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, ref, tcpck.KERNEL_SEG, 0)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    params = [4] + [v | (m << 16) for v in (2, 3) for m in (8, 16, 32, 48, 64)] + [0 | (1 << 16), 1 | (1 << 16)]
    for p in params:
        out.zero_()
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_VVSTREAM, p, packed=True,
                         total_bytes=total)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), p
    t = {p: [] for p in params}
    for _ in range(8):
        for p in params:
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_VVSTREAM, p, packed=True,
                                 total_bytes=total, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                t[p].append(e0.elapsed_time(e1))
    for p in params:
        ms = float(np.median(t[p]))
        gbs = (total + 2 * n) / (ms * 1e-3) / 1e9
        print(f"C3 vvstream variant {p & 0xFF} x{p >> 16}  {ms:8.4f} ms {gbs:7.1f} GB/s ({gbs / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
