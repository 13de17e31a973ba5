#!/usr/bin/env python3
"""Receive ring in chunks (round 4): the bench's ring (1M datagrams of 96/608/1492 B
in 2048-B slots, offset list, SORTED) as K tcpck_batch_receive calls over
consecutive image ranges, so each chunk's header pass follows its own VERIFY
stream while that stream's lines may still sit in the 256 MB Infinity Cache
(the whole ring streams 834 MB).  K = 1 is the product's single call.  Back to
back, median of rounds; verdicts and headers compared with K = 1."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tcp-stack_amd")]

import torch  # noqa: E402
import tcpck  # noqa: E402


def b2b(fn, s, reps=20, rounds=7):
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
    ctx = tcpck.Context(0)
    s = torch.cuda.current_stream()
    n = 1 << 20
    rng = np.random.default_rng(42)
    ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, n)] + 32).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(2048)
    a = torch.empty(n * 2048, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=42)
    img = int(ln.astype(np.int64).sum())
    algo = img + n + 32 * n
    ref_ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ref_hdr = torch.empty(32 * n, dtype=torch.uint8, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(32 * n, dtype=torch.uint8, device="cuda")

    def run(K, o, h):
        m = n // K
        calls = []
        for c in range(K):
            k0 = c * m
            cnt = m if c < K - 1 else n - k0
            sub = ln[k0:k0 + cnt]
            calls.append((k0, cnt, dict(total_bytes=int(sub.astype(np.int64).sum()), min_len=int(sub.min()),
                                        max_len=int(sub.max()), sorted=True)))

        def f():
            for k0, cnt, kw in calls:
                ctx.batch_receive(a, cnt, o.data_ptr() + k0, h.data_ptr() + 32 * k0,
                                  offsets=d_off.data_ptr() + 8 * k0, lengths=d_ln.data_ptr() + 4 * k0, stream=s, **kw)
        return f

    run(1, ref_ok, ref_hdr)()
    torch.cuda.synchronize()
    for K in (1, 2, 4, 8, 16, 1):
        ok.zero_()
        hdr.zero_()
        f = run(K, ok, hdr)
        ms = b2b(f, s)
        same = torch.equal(ok, ref_ok) and torch.equal(hdr, ref_hdr)
        print(f"receive ring in {K:2d} chunk(s)  {ms * 1e3:7.1f} us  {100 * algo / (ms * 1e-3) / 8e12:5.1f} %  "
              f"{'same' if same else 'DIFFERS'}", flush=True)


if __name__ == "__main__":
    main()
