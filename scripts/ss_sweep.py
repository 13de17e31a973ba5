#!/usr/bin/env python3
"""sstream grid sweep on slotted layouts: U4/U8 x oversubscription M x block
order, back to back in one process (% of the 8 TB/s roof in image bytes).

    python scripts/ss_sweep.py [--ms 1,2,4,8,16,32,64] [--variants 1,2,5]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402
import tcpck  # noqa: E402
from slot_probe import PEAK, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,2,4,8,16,32,64")
    ap.add_argument("--variants", default="1,2,5")
    ap.add_argument("--ops", default="checksum")
    args = ap.parse_args()
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    rng = np.random.default_rng(7)
    cases = []
    for S, mix in ((2048, (1492,)), (2048, (96, 608, 1492)), (1536, (96, 608, 1492)), (2048, (32, 1492))):
        n = (1 << 31) // S
        ln = np.asarray(mix, np.uint32)[rng.integers(0, len(mix), n)]
        cases.append((f"var {'/'.join(map(str, mix))} in {S}", S, None, n, np.arange(n, dtype=np.uint64) * np.uint64(S), ln))
    for S, L in ((2048, 1492), (4096, 1492), (256, 96), (16384, 9000), (2048, 1024)):
        cases.append((f"fixed {L} in {S}", S, L, (1 << 31) // S, None, None))
    ops = {"checksum": K.OP_CHECKSUM, "fill": K.OP_FILL, "verify": K.OP_VERIFY}
    for name, S, L, n, off, ln in cases:
        arena = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        if off is None:
            K.synth_fixed(arena, S, L, n, seed=3)
            img = n * L
        else:
            d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            K.synth_var(arena, d_off, d_ln, int(ln.max()), n, seed=3)
            img = int(ln.astype(np.int64).sum())
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        for opn in args.ops.split(","):
            op = ops[opn]
            row = []
            for v in map(int, args.variants.split(",")):
                for m in map(int, args.ms.split(",")):
                    p = v | (m << 16)
                    if off is None:
                        fn = lambda: ctx.batch_fixed_ex(op, arena, S, L, n, out, K.KERNEL_SSTREAM, p, stream=s)  # noqa
                    else:
                        fn = lambda: ctx.batch_var_ex(op, arena, d_off, d_ln, n, out, K.KERNEL_SSTREAM, p,  # noqa
                                                      total_bytes=img, stream=s)
                    ms = timed(fn, s)
                    row.append(f"v{v}/M{m} {img / (ms * 1e-3) / PEAK * 100:5.1f}")
            print(f"{name:28s} {opn:8s} " + "  ".join(row), flush=True)
        del arena, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
