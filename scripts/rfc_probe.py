#!/usr/bin/env python3
"""RFC 1071 mode vs the reference mode on the C2 batch: AUTO (rstream for both
now), seg (round 1's RFC path).  % of the 8 TB/s roof, back to back."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "scripts"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from slot_probe import PEAK, timed  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    for L in (1492, 1024, 4096):
        n = 1566572544 // L
        a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        row = []
        for name, op, mode, k, p in (("ref auto", 0, 0, 0, 0), ("rfc auto", 0, 1, 0, 0),
                                     ("rfc seg", 0, 1, tcpck.KERNEL_SEG, 0), ("rfc fill auto", 1, 1, 0, 0),
                                     ("ref fill auto", 1, 0, 0, 0)):
            fn = lambda: ctx.batch_fixed_ex(op, a, L, L, n, out, k, p, mode=mode, stream=s)  # noqa
            ms = timed(fn, s)
            row.append(f"{name} {(n * L + 2 * n) / (ms * 1e-3) / PEAK * 100:5.1f} %")
        print(f"{n} x {L} B: " + " | ".join(row), flush=True)
        del a, out
        torch.cuda.empty_cache()
    from synth_np import mixed_layout
    for pay, name in (((64, 576, 1460), "C3"), ((66, 578, 1462), "C3 2-mod-4")):
        off, ln, total = mixed_layout(4 << 20, seed=42, payloads=pay)
        n = ln.size
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
        tcpck.synth_var(a, d_off, d_ln, 1494, n, seed=42)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        img = int(ln.astype("int64").sum())
        row = []
        for rname, mode, k in (("ref auto", 0, 0), ("rfc auto", 1, 0), ("rfc seg", 1, tcpck.KERNEL_SEG)):
            fn = lambda: ctx.batch_var_ex(0, a, d_off, d_ln, n, out, k, 0, mode=mode, total_bytes=img,  # noqa
                                          min_len=int(ln.min()), max_len=int(ln.max()), packed=True, stream=s)
            ms = timed(fn, s)
            row.append(f"{rname} {(img + 2 * n) / (ms * 1e-3) / PEAK * 100:5.1f} %")
        print(f"{name} {n} images: " + " | ".join(row), flush=True)
        del a, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
