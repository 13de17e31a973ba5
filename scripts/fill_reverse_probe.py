#!/usr/bin/env python3
"""FILL's field pass in reverse image order (tcpck_probe.h
TCPCK_PROBE_PARAM_PATCH_REVERSE) against AUTO's index order, on C2's fixed
layout (rstream's deferred form + the 2-B write-through pass) and C3's mix
(vvstream CHECKSUM + the field-update pass), with and without a results
buffer.  The stream ends on the arena's last lines; a pass that starts there
may find their blocks still in the 256-MB Infinity Cache when it merges its
2-B writes.  Timed on one arena and on arenas taken in turn (no step sees the
previous step's lines); back-to-back launches, median of 5 rounds; arenas and
results compared with AUTO's."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402


def b2b(fn, s, reps=20, rounds=5):
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--arenas", type=int, default=2)
    p.add_argument("--cases", default="c2,c3")
    args = p.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    REV = tcpck.PROBE_PARAM_PATCH_REVERSE
    for case in args.cases.split(","):
        if case == "c2":
            n, L = 1 << 20, 1492
            arenas = []
            for _ in range(args.arenas):
                a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
                tcpck.synth_fixed(a, L, L, n, seed=42)
                arenas.append(a)
            img = n * L
            call = lambda a, o, prm: ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, n, o, tcpck.KERNEL_AUTO, prm, stream=s)
        else:
            n = 4 << 20
            off, ln, total = synth_np.mixed_layout(n, seed=42)
            d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            arenas = []
            for _ in range(args.arenas):
                a = torch.empty(total, dtype=torch.uint8, device="cuda")
                tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
                arenas.append(a)
            img = int(ln.astype(np.int64).sum())
            kw = dict(total_bytes=img, min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
            call = lambda a, o, prm: ctx.batch_var_ex(tcpck.OP_FILL, a, d_off, d_ln, n, o, tcpck.KERNEL_AUTO, prm,
                                                      **kw)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ref = None
        for label, o, prm in (("AUTO", out, 0), ("AUTO reversed pass", out, REV), ("AUTO no results", None, 0),
                              ("no results, reversed pass", None, REV)):
            for k in (args.arenas, 1):
                turn = [0]

                def step():
                    call(arenas[turn[0] % k], o, prm)
                    turn[0] += 1
                ms = b2b(step, s)
                algo = img + 2 * n + (2 * n if o is not None else 0)
                print(f"{case} {label:28s} arenas {k}: {ms * 1e3:7.1f} us  {algo / ms / 1e6 / 80:5.1f} % of the roof",
                      flush=True)
            torch.cuda.synchronize()
            got = (arenas[0].clone(), out.clone() if o is not None else None)
            if ref is None:
                ref = got
            else:
                same = torch.equal(got[0], ref[0]) and (got[1] is None or torch.equal(got[1], ref[1]))
                print(f"{case} {label:28s} arena/results == AUTO's: {same}", flush=True)
        del arenas, out
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
