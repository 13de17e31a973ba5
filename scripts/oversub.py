#!/usr/bin/env python3
"""Grid oversubscription vs the slot-age tail (rstream / vstream).

With exactly one wave per resident slot, the SIMD's issue arbitration (by
age) finishes slot-0 waves ~2x earlier than slot-7 waves and the last ones
stream alone.  Launching M x the resident grid lets the dispatcher refill freed
slots with fresh (smaller) runs.  Median HIP-event launch time, interleaved.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    for L, n, kern, variants in ((1492, 1 << 20, tcpck.KERNEL_RSTREAM, (0, 1, 10)),
                                 (1492, 8 << 20, tcpck.KERNEL_RSTREAM, (0,)),
                                 (65536, 256 << 10, tcpck.KERNEL_SEG, (3,)),
                                 (256, 6 << 20, tcpck.KERNEL_VSTREAM, (2,)),
                                 (96, 16 << 20, tcpck.KERNEL_VSTREAM, (2,))):
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, ref, tcpck.KERNEL_SEG, 0)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        params = [v | (m << 16) for v in variants for m in (1, 4, 8, 12, 16, 24, 32, 64)]
        for p in params:
            out.zero_()
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, kern, p)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), (L, p)
        t = {p: [] for p in params}
        for _ in range(8):
            for p in params:
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, kern, p, stream=s)
                    e1.record(s)
                    torch.cuda.synchronize()
                    t[p].append(e0.elapsed_time(e1))
        for p in params:
            ms = float(np.median(t[p]))
            gbs = (n * L + 2 * n) / (ms * 1e-3) / 1e9
            print(f"L={L:5d} n={n:9d} kernel {kern} variant {p & 0xFF:2d} x{p >> 16}  {ms:8.4f} ms "
                  f"{gbs:7.1f} GB/s ({gbs / 80:.1f}%)", flush=True)
        del a, ref, out
        torch.cuda.empty_cache()
    # C3 on vvstream
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from synth_np import mixed_layout
    off, ln, total = mixed_layout(4 << 20, seed=42)
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, ref, tcpck.KERNEL_SEG, 0)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    params = [v | (m << 16) for v in (0, 2) for m in (1, 2, 4, 8, 16)]
    for p in params:
        out.zero_()
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_VVSTREAM, p, packed=True)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), p
    t = {p: [] for p in params}
    for _ in range(8):
        for p in params:
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, tcpck.KERNEL_VVSTREAM, p, packed=True,
                                 stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                t[p].append(e0.elapsed_time(e1))
    for p in params:
        ms = float(np.median(t[p]))
        gbs = (total + 2 * n) / (ms * 1e-3) / 1e9
        print(f"C3 vvstream variant {p & 0xFF} x{p >> 16}  {ms:8.4f} ms {gbs:7.1f} GB/s ({gbs / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
