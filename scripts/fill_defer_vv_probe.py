#!/usr/bin/env python3
"""FILL with the fields deferred to the write-through field pass on vvstream
layouts (round 3): C3's packed mix and other packed / gapped batches, the
stream storing the fields itself (kVvPolicy, variant 28) against the stream
writing only the results + launch_patch_fields (variant 28 | 64), CHECKSUM for
reference; the same for sstream's fixed slots (variant 0 against 0 | 128),
and for gapped layouts also the CHECKSUM + field-update form.  ~1.5-3 GB per
case, median of back-to-back rounds; results and arenas compared."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402


def b2b(fn, s, reps=10, rounds=5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
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


def case(ctx, s, name, off, ln, total, fixed=None, kernel=None, base=28, defer=64, defer_param=None):
    n = ln.size
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
    img = int(ln.astype(np.int64).sum())
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    V = tcpck.KERNEL_VVSTREAM if kernel is None else kernel
    if fixed:
        stride, L = fixed
        run = lambda op, p: ctx.batch_fixed_ex(op, a, stride, L, n, out, V, p, stream=s)
        auto = lambda: ctx.batch_fixed(tcpck.OP_FILL, a, stride, L, n, out, stream=s)
    else:
        kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
        run = lambda op, p: ctx.batch_var_ex(op, a, d_off, d_ln, n, out, V, p, **kw)
        auto = lambda: ctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, n, out, **kw)
    res = {}
    runs = [("CHECKSUM", lambda: run(tcpck.OP_CHECKSUM, base)), ("FILL in-stream", lambda: run(tcpck.OP_FILL, base)),
            ("FILL deferred", lambda: run(tcpck.OP_FILL, base | defer if defer_param is None else defer_param)), ("FILL AUTO", auto)]
    runs.append(("FILL update", lambda: run(tcpck.OP_FILL, base | tcpck.PARAM_FILL_UPDATE)))
    for label, fn in runs:
        time.sleep(0.05)  # phase boundary for scripts/fill_drain_summary.py
        ms = b2b(fn, s)
        torch.cuda.synchronize()
        if label.startswith("FILL"):
            res[label] = (out.clone(), a.clone())
        print(f"{name:34s} {label:15s} {ms * 1e3:8.1f} us  {(img + 4 * n) / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
    ref = res["FILL in-stream"]
    same = all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in res.values())
    print(f"{name:34s} results and arenas identical: {same}", flush=True)
    del a


def packed(ln):
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    return off, ln, int(ln.astype(np.int64).sum())


def sweep(ctx, s):
    """Packed variable mixes around AUTO's update threshold (448 B): the in-stream
    FILL with default-policy reads (variant 60, AUTO below it), the stream's
    policy variant (28), and the update form."""
    rng = np.random.default_rng(3)
    for lo, hi in ((32, 256), (64, 512), (128, 640), (192, 768), (256, 896), (64, 1460)):
        n = int((2 << 30) // ((lo + hi) // 2 + 32))
        ln = (rng.integers(lo // 2, hi // 2 + 1, n) * 2 + 32).astype(np.uint32)
        case(ctx, s, f"{n // 1024}K x {lo + 32}-{hi + 32} B packed", *packed(ln), base=60)


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    if "--sweep" in sys.argv:
        return sweep(ctx, s)
    rng = np.random.default_rng(1)
    n = 1 << 20
    case(ctx, s, "C2 1M x 1492 fixed (rstream)", np.arange(n, dtype=np.uint64) * 1492, np.full(n, 1492, np.uint32),
         n * 1492, fixed=(1492, 1492), kernel=tcpck.KERNEL_RSTREAM, base=20, defer_param=25)
    off, ln, total = synth_np.mixed_layout(4 << 20, seed=42)
    case(ctx, s, "C3 4M 96/608/1492 packed", off, ln, total)
    case(ctx, s, "1M x 1492 packed (var)", *packed(np.full(1 << 20, 1492, np.uint32)))
    case(ctx, s, "2M 608/1492 packed", *packed(np.asarray((608, 1492), np.uint32)[rng.integers(0, 2, 2 << 20)]))
    case(ctx, s, "3M 512/608 packed", *packed(np.asarray((512, 608), np.uint32)[rng.integers(0, 2, 3 << 20)]))
    case(ctx, s, "4M 256-1024 packed", *packed((rng.integers(128, 513, 4 << 20) * 2).astype(np.uint32)))
    n = 1 << 20
    case(ctx, s, "1M x 1492 in 1536-B slots (hull)", np.arange(n, dtype=np.uint64) * 1536, np.full(n, 1492, np.uint32),
         n * 1536, fixed=(1536, 1492))
    S = tcpck.KERNEL_SSTREAM
    for stride, L, cnt in ((2048, 1492, n), (4096, 1492, n // 2), (1024, 608, 2 * n), (9216, 9000, n // 6),
                           (16384, 9000, n // 8)):
        case(ctx, s, f"{cnt // 1024}K x {L} in {stride}-B slots (sstream)", np.arange(cnt, dtype=np.uint64) * stride,
             np.full(cnt, L, np.uint32), cnt * stride, fixed=(stride, L), kernel=S, base=0, defer=128)
    case(ctx, s, "171K x 9000 in 9216-B slots (hull)", np.arange(n // 6, dtype=np.uint64) * 9216,
         np.full(n // 6, 9000, np.uint32), (n // 6) * 9216, fixed=(9216, 9000))


if __name__ == "__main__":
    main()
