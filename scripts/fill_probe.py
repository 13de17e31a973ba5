#!/usr/bin/env python3
"""Send-side FILL throughput by kernel (back-to-back launches, median of rounds),
packed C3 layout and fixed C2 / small fixed images.  FILL is idempotent, so the
same arena is refilled every launch; results are checked against seg first."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from synth_np import mixed_layout  # noqa: E402


def bench(label, fn, nbytes, s, check):
    fn()
    torch.cuda.synchronize()
    check()
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    med = []
    for _ in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        med.append(e0.elapsed_time(e1) / 20)
    ms = float(np.median(med))
    print(f"{label:36s} {ms:8.4f} ms ({nbytes / ms / 1e6 / 80:.1f}%)", flush=True)


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    off, ln, total = mixed_layout(4 << 20, seed=42)
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    K.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(K.OP_FILL, a, d_off, d_ln, n, ref, K.KERNEL_SEG, 0)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    lay = dict(total_bytes=total, min_len=int(ln.min()), max_len=int(ln.max()), packed=True)

    def chk():
        assert torch.equal(out, ref)
    for label, fn in (("C3 fill vvstream policy", lambda: ctx.batch_var_ex(K.OP_FILL, a, d_off, d_ln, n, out,
                                                                           K.KERNEL_VVSTREAM, 4, stream=s, **lay)),
                      ("C3 fill auto", lambda: ctx.batch_var(K.OP_FILL, a, d_off, d_ln, n, out, stream=s, **lay)),
                      ("C3 checksum auto", lambda: ctx.batch_var(K.OP_CHECKSUM, a, d_off, d_ln, n, out, stream=s,
                                                                 **lay))):
        bench(label, fn, total + 2 * n, s, chk if "fill" in label else (lambda: None))
    del a, ref, out
    torch.cuda.empty_cache()
    for L, n in ((1492, 1 << 20), (96, 16 << 20), (256, 6 << 20)):
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, L, L, n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(K.OP_FILL, a, L, L, n, ref, K.KERNEL_SEG, 0)
        out = torch.empty(n, dtype=torch.int16, device="cuda")

        def chk():
            assert torch.equal(out, ref)
        runs = [("rstream", K.KERNEL_RSTREAM, 10), ("vvstream fixed", K.KERNEL_VVSTREAM, 4), ("auto", None, 0)]
        if L == 1492:  # rstream policy (20) vs every step read with the default cache policy (22)
            runs += [("rstream v20", K.KERNEL_RSTREAM, 20), ("rstream v22", K.KERNEL_RSTREAM, 22)]
        for label, kern, p in runs:
            for op in (K.OP_FILL, K.OP_CHECKSUM):
                if kern is None:
                    fn = (lambda op=op: ctx.batch_fixed(op, a, L, L, n, out, stream=s))
                else:
                    fn = (lambda op=op, kern=kern, p=p: ctx.batch_fixed_ex(op, a, L, L, n, out, kern, p, stream=s))
                name = "fill" if op == K.OP_FILL else "checksum"
                bench(f"fixed L={L} {name} {label}", fn, n * L + 2 * n, s,
                      chk if op == K.OP_FILL else (lambda: None))
        del a, ref, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
