#!/usr/bin/env python3
"""XCD-aware run order (dev::xcd_block): bare stream (diag) and the checksum
kernels, default block order vs the blocks of one XCD taking consecutive runs.
Median of back-to-back rounds.  Run one workload per process (--what c2, ...):
a batch allocated after other large buffers were freed can land on fragmented
memory, which hides the effect.

    python scripts/xcd_probe.py --what bare|c2|c5|c3|c4
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402

K = tcpck


_SETTLED = [False]


def b2b(fn, s, reps=20, rounds=5):
    # the first config measured in a process would otherwise pay the idle GPU's
    # clock ramp (profiles/r01/transient.log): settle ~300 ms of launches first
    warm = 10
    if not _SETTLED[0]:
        _SETTLED[0] = True
        import time
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            for _ in range(8):
                fn()
            torch.cuda.synchronize()
    for _ in range(warm):
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


def fixed_case(ctx, s, label, n, L, runs, reps):
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    K.synth_fixed(a, L, L, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, ref, K.KERNEL_SEG, 0)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    for name, kern, p in runs:
        ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, kern, p)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), name
        ms = b2b(lambda: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, kern, p, stream=s), s, reps=reps)
        print(f"{label} {name}: {ms:.4f} ms ({(n * L + 2 * n) / ms / 1e6 / 80:.1f}%)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="c2")
    ap.add_argument("--m-sweep", action="store_true")
    ap.add_argument("--cap-sweep", action="store_true")
    what = ap.parse_args().what
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    if what == "bare":
        buf = torch.empty(17 << 30, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(buf, 65536, 65536, (17 << 30) // 65536, seed=1)
        dout = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
        for nbytes in (1566572544, 17 << 30):
            for k, m in ((2, 8), (8, 32)):
                for x in (0, 1):
                    v = 0x3000 | (k << 8) | x
                    ms = b2b(lambda: ctx.diag_stream(v, buf, nbytes, dout, stream=s), s,
                             reps=20 if nbytes < 4e9 else 4)
                    print(f"bare stream {nbytes / 1e9:5.2f} GB x{m} {'xcd' if x else 'default'}: {ms:.4f} ms "
                          f"({nbytes / ms / 1e6 / 80:.1f}%)", flush=True)
    elif what in ("c2", "c5"):
        n = (1 << 20) if what == "c2" else (8 << 20)
        runs = [(f"rstream v{v} x{m}", K.KERNEL_RSTREAM, v | (m << 16))
                for v, m in ((18, 32), (20, 32), (23, 32), (24, 32), (20, 0), (23, 0), (24, 0))]
        runs += [("vvstream fixed x32", K.KERNEL_VVSTREAM, 3 | (32 << 16)),
                 ("vvstream fixed x32 xcd16", K.KERNEL_VVSTREAM, 11 | (32 << 16)),
                 ("vvstream fixed x32 xcd16 first-step", K.KERNEL_VVSTREAM, 27 | (32 << 16))]
        fixed_case(ctx, s, what, n, 1492, runs, 20 if what == "c2" else 4)
    elif what == "c4":
        runs = [(f"seg G64U4 x{m}{' xcd16' if x else ''}", K.KERNEL_SEG, 3 | (m << 16) | (x << 24))
                for m in (1, 8) for x in (0, 1)]
        runs += [(f"rstream v{v} x{m}", K.KERNEL_RSTREAM, v | (m << 16))
                 for v, m in ((18, 32), (20, 0))]
        runs += [(f"seg {n} x{m} xcd16", K.KERNEL_SEG, sh | (m << 16) | (1 << 24))
                 for n, sh in (("W4/U4", 7), ("W16/U2", 9)) for m in (32, 64, 128, 255, 0)]
        fixed_case(ctx, s, "c4", 256 << 10, 65536, runs, 4)
    elif what == "jumbo":
        # jumbo lengths: rstream (whole images per wave) vs W waves per image
        for L in (4096, 6144, 8192, 12288, 16384, 32768, 65536, 131072):
            n = (4 << 30) // L
            runs = [("AUTO", K.KERNEL_AUTO, 0)]
            runs += [("rstream v20", K.KERNEL_RSTREAM, 20)] if L <= 65536 else []
            runs += [(f"seg {nm} xcd16", K.KERNEL_SEG, sh | (1 << 24))
                     for nm, sh in (("G64/U4", 3), ("W2/U4", 11), ("W4/U4", 7), ("W8/U4", 8), ("W16/U2", 9))]
            fixed_case(ctx, s, f"jumbo L={L}", n, L, runs, 8)
            torch.cuda.empty_cache()
    elif what in ("c3", "c3big", "c3u"):
        from synth_np import mixed_layout
        # c3u: the C3 mix with payloads of 66/578/1462 B (images 2 mod 4: the unaligned table path)
        pay = (66, 578, 1462) if what == "c3u" else (64, 576, 1460)
        off, ln, total = mixed_layout((16 if what == "c3big" else 4) << 20, seed=42, payloads=pay)
        n = ln.size
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        K.synth_var(a, d_off, d_ln, 1492, n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, ref, K.KERNEL_SEG, 0)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        params = (12, 28, 11 | (32 << 16), 27 | (32 << 16), 10 | (32 << 16), 26 | (32 << 16), 12, 28)
        if what == "c3big":  # 16M images, ~12 GB: the policy's M (128) vs 32 and 64
            params = (28, 27 | (32 << 16), 27 | (64 << 16), 27 | (128 << 16), 28)
        if "--m-sweep" in sys.argv:  # grid multiple with the policy's flags, U8 and U4
            params = tuple(v | (m << 16) for v in (27, 26) for m in (8, 16, 32, 48)) + (28,)
        if what == "c3u":
            params = (28, 27 | (32 << 16), 27 | (6 << 8) | (24 << 16), 26 | (8 << 8) | (24 << 16), 28)
        if "--cap-sweep" in sys.argv:  # blocks per CU (LDS padding) x grid multiple, U8 + flags
            params = tuple(27 | (c << 8) | (m << 16) for c, m in ((8, 16), (8, 20), (8, 24), (7, 24), (6, 24),
                                                                  (6, 28), (5, 32)))
            params += tuple(26 | (c << 8) | (m << 16) for c, m in ((8, 16), (8, 20), (8, 24), (8, 32))) + (28,)
        for p in params:
            ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, out, K.KERNEL_VVSTREAM, p, packed=True,
                             total_bytes=total)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), p
            ms = b2b(lambda: ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, out, K.KERNEL_VVSTREAM, p,
                                              packed=True, total_bytes=total, stream=s), s)
            print(f"{what} vvstream variant {p & 0xFF} cap {(p >> 8) & 0xFF} x{p >> 16}: {ms:.4f} ms ({(total + 2 * n) / ms / 1e6 / 80:.1f}%)",
                  flush=True)
    elif what == "iso":
        # what separates C3 from the fixed layouts on vvstream: the descriptors
        # (packed var over uniform lengths vs the same fixed batch) and the end
        # density (744-B vs 1492-B images)
        for L, n in ((1492, 1 << 20), (744, 2 << 20)):
            a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
            K.synth_fixed(a, L, L, n, seed=42)
            ref = torch.empty(n, dtype=torch.int16, device="cuda")
            ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, ref, K.KERNEL_SEG, 0)
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            d_off = torch.arange(n, dtype=torch.int64, device="cuda") * L
            d_ln = torch.full((n,), L, dtype=torch.int32, device="cuda")
            runs = [("fixed", lambda st=None: ctx.batch_fixed_ex(K.OP_CHECKSUM, a, L, L, n, out, K.KERNEL_VVSTREAM, 12,
                                                                 **({"stream": st} if st else {}))),
                    ("var  ", lambda st=None: ctx.batch_var_ex(K.OP_CHECKSUM, a, d_off, d_ln, n, out, K.KERNEL_VVSTREAM,
                                                               12, packed=True, total_bytes=n * L,
                                                               **({"stream": st} if st else {})))]
            for name, fn in runs:
                out.zero_()
                fn()
                torch.cuda.synchronize()
                assert torch.equal(out, ref), name
                ms = b2b(lambda: fn(s), s)
                print(f"iso L={L} {name} vvstream policy: {ms:.4f} ms ({(n * L + 2 * n) / ms / 1e6 / 80:.1f}%)",
                      flush=True)
            del a, out, ref, d_off, d_ln
    else:
        raise SystemExit(f"unknown --what {what}")


if __name__ == "__main__":
    main()
