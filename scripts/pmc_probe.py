#!/usr/bin/env python3
"""Launches for SQ counter passes (run under rocprofv3 --pmc ...): the C2 batch
through rstream (policy) and through vvstream's fixed mode, and the C3 batch
through vvstream (policy), a few launches each after a settle.  Compare the
kernels' instruction mix and stall buckets with scripts/pmc_sq.py.

    rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES ... -d gpurun_out/sq1 -o run \
        --output-format csv -- python3 scripts/pmc_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

K = tcpck


def run(fn, n=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        fn()
        torch.cuda.synchronize()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()


def main():
    ctx = tcpck.Context(0, probe=True)
    n, L = 1 << 20, 1492
    if "--rs" in sys.argv:  # rstream 18 vs 20 (default-policy first step): FETCH_SIZE per launch
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        for v in (18, 20):
            run(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_RSTREAM, v | (32 << 16)))
        print("ok", flush=True)
        return
    if "--vv" in sys.argv:  # C3 vvstream policy without / with the L2-kept first step
        from synth_np import mixed_layout
        off, ln, total = mixed_layout(4 << 20, seed=42)
        n = ln.size
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        K.synth_var(a, d_off, d_ln, 1492, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        for v in (12, 28):
            run(lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, out, K.KERNEL_VVSTREAM, v, packed=True,
                                         total_bytes=total))
        print("ok", flush=True)
        return
    if "--ss" in sys.argv:  # sstream: variable images in 2048-B slots vs fixed 1492 B in 4-KiB slots (same density)
        import numpy as np
        S = 2048
        n = (1 << 31) // S
        rng = np.random.default_rng(7)
        ln = np.asarray((96, 608, 1492), np.uint32)[rng.integers(0, 3, n)]
        off = np.arange(n, dtype=np.uint64) * np.uint64(S)
        a = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        K.synth_var(a, d_off, d_ln, 1492, n, seed=3)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        run(lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, out, K.KERNEL_SSTREAM, 0,
                                     total_bytes=int(ln.sum())))
        del a, out
        S, L = 4096, 1492
        n = (1 << 31) // S
        a = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        K.synth_fixed(a, S, L, n, seed=3)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        run(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, S, L, n, out, K.KERNEL_SSTREAM, 0))
        print("ok", flush=True)
        return
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    K.synth_fixed(a, L, L, n, seed=42)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    run(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_RSTREAM, 20 | (32 << 16)))
    run(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_VVSTREAM, 27 | (32 << 16)))
    del a, out
    from synth_np import mixed_layout
    off, ln, total = mixed_layout(4 << 20, seed=42)
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    K.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    run(lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, out, K.KERNEL_VVSTREAM, 28, packed=True,
                                 total_bytes=total))
    print("ok", flush=True)


if __name__ == "__main__":
    main()
