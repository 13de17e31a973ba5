#!/usr/bin/env python3
"""C5 (8M x 1492 B on one GPU) timed under different allocation histories in
one process: first, after C4's 16 GiB arena was freed with empty_cache (a
fresh hipMalloc), and after it was freed into torch's cache (the C5 arena
then reuses C4's block).  bench.py's Workload/measure, HIP events."""
import argparse
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", default="c5,c4,c5e,c4,c5k,c5k")
    a = ap.parse_args()
    import torch
    import tcpck
    args = argparse.Namespace(steps=20, warmup=5, settle_ms=250.0, per_launch_events=False)
    ctx = tcpck.Context(0)
    stream = torch.cuda.current_stream()
    for item in a.orders.split(","):
        name = item[:2]
        w = bench.Workload(name, ctx, stream, 0, 1)
        _, ms, _, _, _ = bench.measure(w, args, 1, stream, "cuda")
        frac = w.algo_bytes / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBS
        ptr = w.arena.data_ptr()
        print(f"{item:5s} {ms * 1e3:9.1f} us  frac {frac:.4f}  arena 0x{ptr:x}", flush=True)
        del w
        torch.cuda.synchronize()
        if not item.endswith("k"):
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
