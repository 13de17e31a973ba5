#!/usr/bin/env python3
"""vvstream A/B on one box (round 4): libtcpck.so (A) against a
libtcpck_probe.so built for this run only with one change switched off (B).
All three changes lost or tied and were removed with their build switches
(logs profiles/r04/vv_stage_ab.log, vv_cache_ab.log,
rs_qsel_ab.log): re-running this needs the change and its -D switch back.

  default  A: results staged in a VGPR, 64 per store (as rstream); B:
           -DTCPCK_VV_NOSTAGE, each step's results stored from inside the step
           loop (the round-1..3 form)
  --cache  A: the pending ends kept in a VGPR across steps (CACHE_E); B:
           -DTCPCK_VV_NOCACHE, the ends re-read from LDS and balloted every step
  --qsel   rstream (tcpck_rstream.hip) A: a 4-B-aligned boundary's P from one
           readlane of the lane's exclusive prefix + its v_dot2 partial (QSEL);
           B: -DTCPCK_RS_NOQSEL, six readlanes and a scalar word sum
The AUTO CHECKSUM / VERIFY on C3's packed 4M mix and on packed fixed 96/256-B
images, interleaved rounds of 20 back-to-back launches; results compared."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def timed(fn, s, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def ab(label, fa, fb, outa, outb, algo, s, rounds=9):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        fa()
        fb()
        torch.cuda.synchronize()
    ta, tb = [], []
    for _ in range(rounds):
        ta.append(timed(fa, s))
        tb.append(timed(fb, s))
    same = torch.equal(outa, outb)
    ma, mb = float(np.median(ta)), float(np.median(tb))
    na, nb = (("cached", "per-step") if "--cache" in sys.argv else
              (("qsel", "6-read") if "--qsel" in sys.argv else ("staged", "unstaged")))
    print(f"{label:26s} {na} {ma * 1e3:7.1f} us ({100 * algo / (ma * 1e-3) / 8e12:5.1f} %)   "
          f"{nb} {mb * 1e3:7.1f} us ({100 * algo / (mb * 1e-3) / 8e12:5.1f} %)   results {'equal' if same else 'DIFFER'}",
          flush=True)


def main_qsel(A, B, s, K):
    for L, mode in ((1492, 0), (1492, 1), (512, 0), (1024, 0), (2048, 0), (3000, 0)):
        m = 1564475392 // L
        arena = torch.empty(m * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(arena, L, L, m, seed=42)
        for op, dt, name in ((K.OP_CHECKSUM, torch.int16, "CHECKSUM"), (K.OP_VERIFY, torch.uint8, "VERIFY")):
            oa = torch.empty(m, dtype=dt, device="cuda")
            ob = torch.empty(m, dtype=dt, device="cuda")
            ab(f"rstream {L} {name} m{mode}",
               lambda: A.batch_fixed_ex(op, arena, L, L, m, oa, K.KERNEL_RSTREAM, 20, mode=mode, stream=s),
               lambda: B.batch_fixed_ex(op, arena, L, L, m, ob, K.KERNEL_RSTREAM, 20, mode=mode, stream=s), oa, ob,
               m * L + 2 * m, s)
        del arena
        torch.cuda.empty_cache()
    n = 8 << 20  # C5 on one GPU
    arena = torch.empty(n * 1492, dtype=torch.uint8, device="cuda")
    K.synth_fixed(arena, 1492, 1492, n, seed=42)
    oa = torch.empty(n, dtype=torch.int16, device="cuda")
    ob = torch.empty(n, dtype=torch.int16, device="cuda")
    ab("rstream C5 8M CHECKSUM", lambda: A.batch_fixed(K.OP_CHECKSUM, arena, 1492, 1492, n, oa, stream=s),
       lambda: B.batch_fixed(K.OP_CHECKSUM, arena, 1492, 1492, n, ob, stream=s), oa, ob, n * 1494, s, rounds=5)


def main():
    A = tcpck.Context(0)
    B = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    K = tcpck
    if "--qsel" in sys.argv:
        main_qsel(A, B, s, K)
        return
    rng = np.random.default_rng(42)
    n = 1 << 22
    ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(ln.sum())
    arena = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    K.synth_var(arena, d_off, d_len, int(ln.max()), n, seed=42)
    hints = dict(total_bytes=total, min_len=int(ln.min()), max_len=int(ln.max()), packed=True)
    for op, name, dt in ((K.OP_CHECKSUM, "C3 CHECKSUM", torch.int16), (K.OP_VERIFY, "C3 VERIFY", torch.uint8)):
        oa = torch.empty(n, dtype=dt, device="cuda")
        ob = torch.empty(n, dtype=dt, device="cuda")
        ab(name, lambda: A.batch_var(op, arena, d_off, d_len, n, oa, stream=s, **hints),
           lambda: B.batch_var(op, arena, d_off, d_len, n, ob, stream=s, **hints), oa, ob, total + 2 * n, s)
    del arena
    torch.cuda.empty_cache()
    for L in (96, 256, 448, 736, 1492, 4096):
        m = 1564475392 // L
        arena = torch.empty(m * L, dtype=torch.uint8, device="cuda")
        K.synth_fixed(arena, L, L, m, seed=42)
        oa = torch.empty(m, dtype=torch.int16, device="cuda")
        ob = torch.empty(m, dtype=torch.int16, device="cuda")
        ab(f"fixed {L} CHECKSUM vv28", lambda: A.batch_fixed_ex(K.OP_CHECKSUM, arena, L, L, m, oa, K.KERNEL_VVSTREAM, 28,
                                                                stream=s),
           lambda: B.batch_fixed_ex(K.OP_CHECKSUM, arena, L, L, m, ob, K.KERNEL_VVSTREAM, 28, stream=s), oa, ob,
           m * L + 2 * m, s)
        del arena
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
