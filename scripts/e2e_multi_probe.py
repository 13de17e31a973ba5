#!/usr/bin/env python3
"""End to end (pinned host -> GPU -> host) through tcpck_host_batch_fixed and
tcpck_host_batch_fixed_multi with 1, 2, 4 contexts, C2's batch (1M x 1492 B).
On a one-GPU box every context shares device 0 and its one PCIe link, so this
measures the sharding's overhead, not multi-GPU scaling."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    L, n = 1492, 1 << 20
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(d, L, L, n, seed=42)
    h = torch.empty(n * L, dtype=torch.uint8).pin_memory()
    h.copy_(d.cpu())
    out = torch.empty(n, dtype=torch.int16).pin_memory()
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    ctxs = [tcpck.Context(0, probe=True) for _ in range(4)]
    ctxs[0].batch_fixed(tcpck.OP_CHECKSUM, d, L, L, n, ref)
    torch.cuda.synchronize()
    ref = ref.cpu()
    runs = [("one ctx", lambda: ctxs[0].host_batch_fixed(tcpck.OP_CHECKSUM, h, L, L, n, out))]
    for k in (1, 2, 4):
        runs.append((f"multi x{k}", lambda k=k: tcpck.host_batch_fixed_multi(ctxs[:k], tcpck.OP_CHECKSUM, h, L, L, n,
                                                                             out)))
    for name, fn in runs:
        fn()
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        dt = float(np.median(t))
        print(f"{name:10s} {dt * 1e3:8.2f} ms  {n * L / dt / 2**30:6.1f} GiB/s  same: {torch.equal(out, ref)}",
              flush=True)


if __name__ == "__main__":
    main()
