#!/usr/bin/env python3
"""Device copy rate against the copied size (round 4): is the guide's
"6.29 TB/s measured (float4 copy, 79%)" (MI355X_MICROARCH.md) a large-buffer
HBM figure, or one helped by the 256 MB Infinity Cache?  Our 1.5 GiB copies
stop at 67.7 % of the roof (profiles/r02/copy_probe.log), the ceiling
batched segmentation is judged against.  torch copy_ and the diag copy kernel
(runs of 1 KiB steps, U2, nt stores, 8x the resident grid: copy_probe.py's
best) at 64 MiB .. 6 GiB; % of the roof in read + write bytes."""
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
    out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    best = 0x5000 | 0 | (1 << 2) | (8 << 8)  # runs, U2, nt stores, M8
    for mib in (64, 128, 256, 512, 1024, 1536, 3072, 6144):
        half = mib << 20
        buf = torch.randint(0, 255, (2 * half,), dtype=torch.uint8, device="cuda")
        dst = torch.empty(half, dtype=torch.uint8, device="cuda")
        t_torch = b2b(lambda: dst.copy_(buf[:half]), s)
        t_diag = b2b(lambda: ctx.diag_stream(best, buf, 2 * half, out, stream=s), s)
        torch.cuda.synchronize()
        ok = torch.equal(buf[:half], buf[half:])
        print(f"copy {mib:5d} MiB   torch {t_torch * 1e3:9.1f} us {2 * half / t_torch / 1e6 / 80:5.1f} %   "
              f"diag {t_diag * 1e3:9.1f} us {2 * half / t_diag / 1e6 / 80:5.1f} %   copied ok: {ok}", flush=True)
        del buf, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
