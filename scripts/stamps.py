#!/usr/bin/env python3
"""Per-wave timing of one C2-sized rstream launch, grouped by hardware placement.

Uses the stamp build of the rstream kernel (variant 3): each wave records
{start, end} (s_memrealtime, 100 MHz), HW_ID and XCC_ID.  Prints the spread of
wave durations and their mean by XCC, SE, CU, SIMD and wave slot, to tell what
makes identical runs finish at different times."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    L, n = 1492, 1 << 20
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=5)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    dbg = torch.zeros(4 * 65536, dtype=torch.int64, device="cuda")  # 4 x u64 per wave of the x1 grid
    ctx.set_debug(dbg)
    for rep in range(3):
        dbg.zero_()
        # variant 3 (stamps) on the resident grid only (x1): one stamp slot per wave
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, tcpck.KERNEL_RSTREAM, 3 | (1 << 16))
        torch.cuda.synchronize()
    ctx.set_debug(None)
    d = dbg.cpu().numpy().reshape(-1, 4)
    d = d[d[:, 1] > 0]
    t0 = d[:, 0].min()
    st = (d[:, 0] - t0) / 100.0
    en = (d[:, 1] - t0) / 100.0
    dur = en - st
    hw = d[:, 2].astype(np.int64)
    fields = {"xcc": d[:, 3] & 0xF, "se": (hw >> 13) & 0x7, "sh": (hw >> 12) & 1, "cu": (hw >> 8) & 0xF,
              "simd": (hw >> 4) & 3, "slot": hw & 0xF}
    print(f"waves {len(d)}; start spread {st.max():.2f} us; end min/median/p90/max "
          f"{en.min():.1f}/{np.median(en):.1f}/{np.percentile(en, 90):.1f}/{en.max():.1f} us", flush=True)
    for name, v in fields.items():
        keys = np.unique(v)
        row = " ".join(f"{int(k)}:{dur[v == k].mean():.0f}" for k in keys)
        print(f"mean duration by {name:4s} -> {row}", flush=True)
    # rank correlation with slot inside a SIMD (arbitration age)
    key = fields["xcc"] * 4096 + fields["se"] * 512 + fields["sh"] * 256 + fields["cu"] * 16 + fields["simd"] * 4
    order = np.argsort(st)
    print("slowest 10 waves:", [(int(fields['xcc'][i]), int(fields['cu'][i]), int(fields['simd'][i]),
                                 int(fields['slot'][i]), round(float(dur[i]), 1))
                                for i in np.argsort(-dur)[:10]], flush=True)
    print("fastest 10 waves:", [(int(fields['xcc'][i]), int(fields['cu'][i]), int(fields['simd'][i]),
                                 int(fields['slot'][i]), round(float(dur[i]), 1))
                                for i in np.argsort(dur)[:10]], flush=True)
    # within each SIMD: durations sorted by start order
    groups = {}
    for i in order:
        groups.setdefault(int(key[i]), []).append(float(dur[i]))
    lens = [len(g) for g in groups.values()]
    width = max(lens)
    mat = np.full((len(groups), width), np.nan)
    for r, g in enumerate(groups.values()):
        mat[r, :len(g)] = g
    print("mean duration by start order within a SIMD:", np.round(np.nanmean(mat, axis=0), 1).tolist(), flush=True)


if __name__ == "__main__":
    main()
