#!/usr/bin/env python3
"""C4 (256K x 64-KiB packed jumbo images) as virtual pieces on rstream.

An image's checksum is ~(sum of its LE u16 words mod 2^16) (tcp-header.h:252-263),
and a ring sum splits: the image sum is the sum of its pieces' sums.  So the
16 GiB arena can be streamed as 64 KiB / P pieces of P bytes per image by
rstream (the C2/C5 kernel, 92-93 % of the roof on 1492-B images), each piece's
checksum c_p = ~s_p, and the image's checksum = ~(sum of ~c_p) mod 2^16.  This
probe times rstream on the pieces (P = 1024 .. 16384) against AUTO's C4 kernel
(seg jumbo W16) and checks the combined result (torch) against AUTO's.
Back-to-back launches, median of 5 rounds of 10.
Round 3 (profiles/r03/c4_pieces_probe.log): every piece size ran 85.5-87.0 %
against seg W16's 90.9 % (rstream on the whole 64-KiB images 88.4 %), so the
product form this drove (rstream variant 30 + a combine pass) was removed; its
lines here need it back to run.  The torch-combined lines run as they are."""
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
    while time.perf_counter() - t0 < 0.3:
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
    L, n = 65536, 256 << 10
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=42, stream=s)
    alg = n * L + 2 * n
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ms = b2b(lambda: ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, n, out, stream=s), s)
    print(f"AUTO (C4 kernel)        {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
    ref = out.clone()
    for P in [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("1024", "2048", "4096", "8192", "16384", "65536"))]:
        k = L // P
        outp = torch.empty(n * k, dtype=torch.int16, device="cuda")
        for label, param in (("policy", 20), ("M 64", 20 | (64 << 16)), ("M 255", 20 | (255 << 16))):
            try:
                ms = b2b(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, P, P, n * k, outp, kernel=tcpck.KERNEL_RSTREAM,
                                                    param=param, stream=s), s)
            except tcpck.TcpckError as e:
                print(f"rstream P={P:5d} {label}: {e}", flush=True)
                continue
            raw = (~outp.to(torch.int32)) & 0xFFFF
            comb = (~(raw.view(n, k).sum(dim=1) & 0xFFFF)) & 0xFFFF
            same = torch.equal(comb.to(torch.int32), ref.to(torch.int32) & 0xFFFF)
            a2 = n * L + 2 * n * k
            print(f"rstream P={P:5d} {label:10s} {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof "
                  f"(C4 bytes; {a2 / ms / 1e6 / 80:5.1f} % with the piece results)  combined == AUTO: {same}", flush=True)
        del outp
        if k >= 8:  # the product form: run_pieces (rstream variant 30) = the stream + launch_piece_combine
            param = 30 | ((k // 8) << 8)
            out2 = torch.empty(n, dtype=torch.int16, device="cuda")
            ms = b2b(lambda: ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, L, L, n, out2, kernel=tcpck.KERNEL_RSTREAM,
                                                param=param, stream=s), s)
            same = torch.equal(out2, ref)
            ok = torch.empty(n, dtype=torch.uint8, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_VERIFY, arena, L, L, n, ok, kernel=tcpck.KERNEL_RSTREAM, param=param, stream=s)
            torch.cuda.synchronize()
            vsame = torch.equal(ok, (ref == 0).to(torch.uint8))
            print(f"run_pieces np={k:3d} (P={P:5d}) {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof  "
                  f"== AUTO: {same}, VERIFY == (AUTO == 0): {vsame}", flush=True)


def fill():
    """--fill: C4 FILL, AUTO (seg W16 in-stream) against the pieces' CHECKSUM +
    the write-through field-update pass (np 16), outputs and arenas compared."""
    L, n = 65536, 256 << 10
    ctx = tcpck.Context(0, probe=True)
    s = torch.cuda.current_stream()
    arena = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(arena, L, L, n, seed=42, stream=s)
    alg = n * L + 2 * n + 2 * n
    res = {}
    for label, fn in (("AUTO", lambda o: ctx.batch_fixed(tcpck.OP_FILL, arena, L, L, n, o, stream=s)),
                      ("pieces+update", lambda o: ctx.batch_fixed_ex(tcpck.OP_FILL, arena, L, L, n, o,
                                                                     kernel=tcpck.KERNEL_RSTREAM,
                                                                     param=30 | (2 << 8) | tcpck.PARAM_FILL_UPDATE,
                                                                     stream=s))):
        o = torch.empty(n, dtype=torch.int16, device="cuda")
        ms = b2b(lambda: fn(o), s)
        torch.cuda.synchronize()
        res[label] = (o.clone(), arena[28::L].clone(), arena[29::L].clone())
        print(f"C4 FILL {label:14s} {ms * 1e3:8.1f} us  {alg / ms / 1e6 / 80:5.1f} % of the roof", flush=True)
    a, b = res["AUTO"], res["pieces+update"]
    print("results and fields identical:", all(torch.equal(x, y) for x, y in zip(a, b)), flush=True)


if __name__ == "__main__" and "--fill" in sys.argv:
    fill()
elif __name__ == "__main__":
    main()
