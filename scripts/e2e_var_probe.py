#!/usr/bin/env python3
"""End to end (pinned host -> GPU -> host, PCIe included) beyond C2's
CHECKSUM (bench.py's `e2e` key): C3's mixed packed batch through
tcpck_host_batch_var (the host scan of offsets / lengths, chunks of images,
their descriptors H2D, kernel, results D2H), and the send-path FILL on C2's
layout through tcpck_host_batch_fixed (results D2H, then bytes 28-29 patched
into the host images).  Median of 5 passes; every result compared with the
device-resident path on the same bytes.

Hypothesis: every host-memory form is bound by PCIe
(C2 CHECKSUM 49-57 GiB/s of image bytes); C3 adds 12 B of descriptors per
732-B image (+1.6 % of the bytes moved) and the host scan, so it should run
within a few percent of C2's rate; FILL moves only 2 B per image back, so it
should match CHECKSUM.
"""
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import tcpck  # noqa: E402
import synth_np  # noqa: E402

GIB = float(1 << 30)


def timed(fn, reps=5):
    fn()  # staging allocation, clocks
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return statistics.median(t), min(t), max(t)


def main():
    print(__doc__.split("Hypothesis")[1].strip(), flush=True)
    ctx = tcpck.Context(0)
    ctx.set_chunk_bytes(64 << 20)
    # C3: 4M images of 96 / 608 / 1492 B, packed
    off, ln, total = synth_np.mixed_layout(4 << 20, seed=42)
    n = ln.size
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(d, d_off, d_ln, 1492, n, seed=42)
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, d, d_off, d_ln, n, ref, total_bytes=total, min_len=int(ln.min()),
                  max_len=int(ln.max()), packed=True)
    h = torch.empty(total, dtype=torch.uint8).pin_memory()
    h.copy_(d.cpu())
    out = torch.empty(n, dtype=torch.int16).pin_memory()
    med, lo, hi = timed(lambda: ctx.host_batch_var(tcpck.OP_CHECKSUM, h, off, ln, n, out))
    same = bool(torch.equal(out, ref.cpu()))
    print(f"C3 CHECKSUM host batch: {total / med / GIB:6.2f} GiB/s of image bytes (median of 5; "
          f"{total / hi / GIB:.2f}-{total / lo / GIB:.2f}), results == device path: {same}", flush=True)
    del d, d_off, d_ln, h, out, ref
    torch.cuda.empty_cache()
    # C2 FILL (send path) from host memory
    L, n = 1492, 1 << 20
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(d, L, L, n, seed=42)
    h = torch.empty(n * L, dtype=torch.uint8).pin_memory()
    h.copy_(d.cpu())
    ctx.batch_fixed(tcpck.OP_FILL, d, L, L, n, None)
    want = d.cpu()
    med, lo, hi = timed(lambda: ctx.host_batch_fixed(tcpck.OP_FILL, h, L, L, n, None))
    same = bool(torch.equal(h, want))
    print(f"C2 FILL host batch:     {n * L / med / GIB:6.2f} GiB/s of image bytes (median of 5; "
          f"{n * L / hi / GIB:.2f}-{n * L / lo / GIB:.2f}), arena == device path's: {same}", flush=True)
    out = torch.empty(n, dtype=torch.int16).pin_memory()
    med, lo, hi = timed(lambda: ctx.host_batch_fixed(tcpck.OP_CHECKSUM, h, L, L, n, out))
    print(f"C2 CHECKSUM host batch: {n * L / med / GIB:6.2f} GiB/s of image bytes (median of 5; "
          f"{n * L / hi / GIB:.2f}-{n * L / lo / GIB:.2f})", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
