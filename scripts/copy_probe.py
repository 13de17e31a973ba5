#!/usr/bin/env python3
"""Device copy ceiling on this part: 1.61 GB copied HBM -> HBM by the diag copy
kernel (tcpck_diag_stream variant 0x5000: contiguous runs per wave or a
grid-stride float4 copy; loads in flight, store cache policy, grid size) and
by torch copy_, as % of the 8 TB/s roof in read + write bytes.  The ceiling
batched segmentation (a read stream + a write stream of the same size) is
judged against.  Back to back, median of rounds."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


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


def main():
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    half = 1536 * (1 << 20)
    buf = torch.randint(0, 255, (2 * half,), dtype=torch.uint8, device="cuda")
    out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    dst = torch.empty(half, dtype=torch.uint8, device="cuda")
    ms = b2b(lambda: dst.copy_(buf[:half]), s)
    print(f"torch copy_            {ms * 1e3:7.1f} us  {2 * half / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
    best = (0, None)
    for gs in (0, 16):
        for u, un in ((0, 2), (1, 4), (2, 8)):
            for sp, sn in ((0, "default"), (1, "nt"), (2, "sc1")):
                for m in ((1, 4, 8, 16) if not gs else (1, 2, 4, 8)):
                    v = 0x5000 | u | (sp << 2) | gs | (m << 8)
                    ms = b2b(lambda: ctx.diag_stream(v, buf, 2 * half, out, stream=s), s)
                    frac = 2 * half / ms / 1e6 / 80
                    best = max(best, (frac, v))
                    print(f"{'grid-stride' if gs else 'runs':11s} U{un} {sn:7s} M{m:<3d} {ms * 1e3:7.1f} us  "
                          f"{frac:5.1f} % of the roof", flush=True)
    torch.cuda.synchronize()
    assert torch.equal(buf[:half], buf[half:2 * half]), "copy mismatch"
    print(f"best {best[0]:.1f} % (variant {best[1]:#x}); copies verified", flush=True)


if __name__ == "__main__":
    main()
