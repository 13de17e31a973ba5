#!/usr/bin/env python3
"""Which XCD runs which block: rstream's stamp build (variant 3, resident grid,
default block order) records XCC_ID per wave; prints blockIdx % 8 against
XCC_ID, i.e. whether dispatch is round-robin on this box."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def main():
    ctx = tcpck.Context(0, probe=True)
    props = torch.cuda.get_device_properties(0)
    print(f"device: {props.name} CUs {props.multi_processor_count} mem {props.total_memory / 2**30:.0f} GiB "
          f"gcn {getattr(props, 'gcnArchName', '?')}", flush=True)
    L, n = 1492, 1 << 20
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=5)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    dbg = torch.zeros(4 * 65536, dtype=torch.int64, device="cuda")
    ctx.set_debug(dbg)
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out, tcpck.KERNEL_RSTREAM, 3 | (1 << 16))
    torch.cuda.synchronize()
    ctx.set_debug(None)
    d = dbg.cpu().numpy().reshape(-1, 4)
    waves = np.nonzero(d[:, 1] > 0)[0]
    blk = waves // 4
    xcc = d[waves, 3] & 0xF
    print(f"waves stamped: {waves.size}, blocks {blk.max() + 1}", flush=True)
    tab = np.zeros((8, 16), np.int64)
    for b, x in zip(blk % 8, xcc):
        tab[b, x] += 1
    for b in range(8):
        print(f"blockIdx % 8 = {b}: waves per XCC_ID {tab[b, :8].tolist()}", flush=True)


if __name__ == "__main__":
    main()
