#!/usr/bin/env python3
"""Where C3's vvstream launch spends its wave time: per
wave, s_memrealtime (100 MHz) stamps at entry, once the run's descriptors are
in (offsets / lengths -> span), once the first step's data has been summed,
and at the end (probe library, RunArgs::dbg; tcpck_probe.h).  The same
analysis on C3's bytes as a fixed 736-B stride (vvstream FIXED: no
descriptors, the same boundary density) separates the descriptor wait from
the rest.

Prints per layout: the launch's span, the mean wave's phases (descriptor
wait, first-data wait, streaming), the share of all wave-time spent before
the first data, and the number of streaming waves over the launch (start
ramp, steady state, tail)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402

VV_POLICY = 4 | 8 | 16


def analyse(name, d, img_bytes):
    d = d.reshape(-1, 8)
    d = d[d[:, 3] > 0]
    t0 = d[:, 0].min()
    st, de, fi, en = [(d[:, i] - t0) / 100.0 for i in range(4)]
    span = en.max()
    wave = en - st
    pre = fi - st
    print(f"{name}: waves {len(d)}, launch span {span:.1f} us ({img_bytes / span / 1e6 / 8:.1%} of the roof for the "
          f"image bytes); runs {np.median(d[:, 6]) / 1024:.1f} KiB median", flush=True)
    print(f"  per wave (mean / median us): total {wave.mean():.2f}/{np.median(wave):.2f}, descriptors "
          f"{(de - st).mean():.2f}/{np.median(de - st):.2f}, first data {pre.mean():.2f}/{np.median(pre):.2f}, "
          f"streaming {(en - fi).mean():.2f}/{np.median(en - fi):.2f}", flush=True)
    print(f"  wave-time before the first data: {pre.sum() / wave.sum():.1%} of all wave-time "
          f"(descriptors {(de - st).sum() / wave.sum():.1%})", flush=True)
    # waves resident over time, and how many of them are streaming, in 2-us buckets
    edges = np.arange(0, span + 2, 2.0)
    res = np.array([((st <= t) & (en > t)).sum() for t in edges])
    strm = np.array([((fi <= t) & (en > t)).sum() for t in edges])
    steady = res[len(res) // 4: 3 * len(res) // 4].mean()
    print(f"  resident waves steady {steady:.0f}; streaming share of resident waves in the middle half "
          f"{strm[len(res) // 4: 3 * len(res) // 4].sum() / max(1, res[len(res) // 4: 3 * len(res) // 4].sum()):.1%}",
          flush=True)
    tail = span - np.percentile(en, 50)
    ramp = np.argmax(res >= 0.9 * res.max()) * 2.0
    last90 = (np.nonzero(res >= 0.9 * steady)[0].max() + 1) * 2.0
    print(f"  ramp to 90% residency {ramp:.1f} us; residency >= 90% of steady until {last90:.1f} us; tail after "
          f"that {span - last90:.1f} us; median wave end {np.percentile(en, 50):.1f} us (tail {tail:.1f})", flush=True)


def run(ctx, s, name, arena, launch, nwaves_max, img_bytes, reps=3):
    dbg = torch.zeros(8 * (nwaves_max + 8), dtype=torch.int64, device="cuda")
    for _ in range(30):  # settle the clocks
        launch()
    torch.cuda.synchronize()
    ctx.set_debug(dbg)
    for _ in range(reps):
        dbg.zero_()
        launch()
        torch.cuda.synchronize()
    ctx.set_debug(None)
    analyse(name, dbg.cpu().numpy(), img_bytes)


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    img = int(ln.astype(np.int64).sum())
    kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True)
    for m in (0, 16, 64):
        run(ctx, s, f"C3 packed offsets, vvstream M {m or 'policy'}", a,
            lambda m=m: ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, count, out, tcpck.KERNEL_VVSTREAM,
                                         VV_POLICY | (m << 16), **kw), count, img)
    L = 736  # C3's mean image: the same bytes, no descriptors
    n2 = img // L
    run(ctx, s, "736-B fixed stride, vvstream FIXED", a,
        lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n2, out, tcpck.KERNEL_VVSTREAM, VV_POLICY),
        n2, n2 * L)
    ctx.close()


if __name__ == "__main__":
    main()
