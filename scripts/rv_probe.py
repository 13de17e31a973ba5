#!/usr/bin/env python3
"""Where does the variable-layout run-stream kernel lose against the fixed one?

Times KERNEL_RVSTREAM variants, span and stream on three packed layouts of
about the same byte count -- C3 (mixed 96/608/1492-B images), C2 expressed as
a variable layout (1M x 1492 B), and all-96-B images (boundary-dense) -- and
rstream on the fixed-stride form of the C2 bytes.  Every result is checked
against the seg kernel first.  Median of interleaved HIP-event launch times.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from synth_np import mixed_layout  # noqa: E402


def layout(name):
    if name == "c3":
        off, ln, total = mixed_layout(4 << 20, seed=42)
    elif name == "c2var":
        n = 1 << 20
        ln = np.full(n, 1492, np.uint32)
        off = np.arange(n, dtype=np.uint64) * np.uint64(1492)
        total = n * 1492
    else:  # all 96-B images
        n = (1564475392 // 96)
        ln = np.full(n, 96, np.uint32)
        off = np.arange(n, dtype=np.uint64) * np.uint64(96)
        total = n * 96
    return off, ln, total


def main():
    ctx = tcpck.Context(0)
    stream = torch.cuda.current_stream()
    for name in ("c2var", "c3", "all96"):
        off, ln, total = layout(name)
        n = ln.size
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        tcpck.synth_var(a, d_off, d_ln, int(ln.max()), n, seed=42)
        ref = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, ref, tcpck.KERNEL_SEG, 0)
        runs = [(f"rvstream v{v}", "var", tcpck.KERNEL_RVSTREAM, v) for v in (0, 3)]
        runs += [(f"vvstream v{v}", "var", tcpck.KERNEL_VVSTREAM, v) for v in (0, 1, 2, 3)]
        runs += [("span T16", "var", tcpck.KERNEL_SPAN, 16), ("stream U4", "var", tcpck.KERNEL_STREAM, 0)]
        if name != "c3":
            L = int(ln[0])
            runs += [(f"rstream v{v} (fixed)", "fixed", tcpck.KERNEL_RSTREAM, v) for v in (0, 9, 10, 11)]
        out = torch.empty(n, dtype=torch.int16, device="cuda")

        def launch(kind, k, p):
            if kind == "var":
                ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, n, out, k, p, packed=True, stream=stream)
            else:
                ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, n, out, k, p, stream=stream)

        ok = {}
        for label, kind, k, p in runs:
            out.zero_()
            launch(kind, k, p)
            torch.cuda.synchronize()
            ok[label] = bool(torch.equal(out, ref))
        times = {r[0]: [] for r in runs}
        for _ in range(8):
            for label, kind, k, p in runs:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
                for i in range(3):
                    ev[2 * i].record(stream)
                    launch(kind, k, p)
                    ev[2 * i + 1].record(stream)
                torch.cuda.synchronize()
                times[label] += [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(3)]
        for label, *_ in runs:
            ms = float(np.median(times[label]))
            gbs = (total + 2 * n) / (ms * 1e-3) / 1e9
            print(f"{name:6s} {label:22s} {ms:8.4f} ms {gbs:8.1f} GB/s ({gbs / 80:.1f}%) ok={ok[label]}", flush=True)
        del a, d_off, d_ln, ref, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
