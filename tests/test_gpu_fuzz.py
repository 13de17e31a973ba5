"""Randomised parity of the AUTO policy (tcpck_batch_fixed / tcpck_batch_var /
tcpck_batch_segment / tcpck_batch_receive): seeded random layouts -- fixed
strides and lengths around every policy boundary, packed / sorted-with-gaps /
unordered offset lists, empty and jumbo images, misaligned arenas, both modes,
every op (RECEIVE in place and into a header array too), right and wrong SORTED
hints -- each checked against the oracle (oracle/ref16.c, pinned to the
reference's golden vectors).  Sizes stay small (<= 16 MB per case); the seeds
are fixed, so a failure names a reproducible case.  TCPCK_FUZZ_BASE /
TCPCK_FUZZ_SEEDS (environment) shift and widen the seed range for longer bug
hunts (defaults: 0 and 200 / 200 / 80)."""
import os

import numpy as np
import pytest

BASE = int(os.environ.get("TCPCK_FUZZ_BASE", "0"))
NSEEDS = int(os.environ.get("TCPCK_FUZZ_SEEDS", "0"))

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available()
    c = tcpck.Context(0)
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


LENS = [2, 14, 16, 30, 32, 34, 48, 64, 96, 98, 128, 240, 256, 448, 510, 512, 514, 1024, 1460, 1492, 1494, 2048,
        4094, 4096, 4098, 8192, 9000, 16384, 20000, 32768, 40000, 65534, 65536]


def check_fill(arena_np, offs, lens, mode, run):
    """FILL through `run`, then compare the results and every arena byte with the
    reference's per-image send path (socket-manager.cc:9-10)."""
    from oracle import ref16 as R
    out = run()
    exp_arena = arena_np.copy()
    exp = np.array([R.fill_np(exp_arena[int(o):int(o) + int(n)], mode) for o, n in zip(offs, lens)], np.uint16)
    np.testing.assert_array_equal(out, exp)
    return exp_arena


def check_receive(ctx, arena_np, mis, offs, lens, mode, seed, layout):
    """RECEIVE on a fresh copy of the arena (ReceivePacket's front half,
    socket-manager.h:182-184): into a header array (arena untouched) or in
    place, by seed; verdicts and bytes against oracle.ref16.receive_np."""
    from oracle import ref16 as R
    buf = dev(arena_np)
    n = len(offs)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    exp = arena_np.copy()
    exp_ok = R.receive_np(exp[mis:], offs, lens, mode)
    if seed % 2:
        hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        ctx.batch_receive(buf.data_ptr() + mis, n, ok, hdr, mode=mode, **layout)
        o = np.asarray(offs, np.int64)
        np.testing.assert_array_equal(host(hdr).reshape(n, 32), exp[mis:][o[:, None] + np.arange(32)[None, :]])
        np.testing.assert_array_equal(host(buf), arena_np)
    else:
        ctx.batch_receive(buf.data_ptr() + mis, n, ok, None, mode=mode, **layout)
        np.testing.assert_array_equal(host(buf), exp)
    np.testing.assert_array_equal(host(ok), exp_ok)


@pytest.mark.parametrize("seed", range(BASE, BASE + (NSEEDS or 200)))
def test_fuzz_fixed(ctx, oracle_c, seed):
    import tcpck
    rng = np.random.default_rng(1000 + seed)
    length = int(rng.choice(LENS))
    gap = int(rng.choice([0, 0, 0, 2, 16, 44, length // 3 * 2, 556, 2048]))
    stride = length + gap
    if rng.random() < 0.3:
        stride = (stride + 15) // 16 * 16  # slots of a multiple of 16 B
    stride = max(stride, length)
    count = int(max(1, min(rng.integers(1, 60000), (16 << 20) // max(stride, 1))))
    mis = int(rng.choice([0, 2, 4, 6, 14, 126]))
    mode = int(rng.random() < 0.35)
    arena_np = rng.integers(0, 256, count * stride + 256, dtype=np.uint8)
    if rng.random() < 0.2:
        arena_np[:] = 0xFF
    buf = dev(arena_np)
    ptr = buf.data_ptr() + mis
    view = arena_np[mis:]
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, ptr, stride, length, count, out, mode=mode)
    exp = oracle_c.batch(view, stride=stride, length=length, count=count, mode=mode, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp, err_msg=f"{stride}/{length}x{count} mis {mis}")
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, ptr, stride, length, count, ok, mode=mode)
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))
    if length >= 30:
        offs = np.arange(count, dtype=np.int64) * stride
        lens = np.full(count, length, np.int64)

        def run():
            ctx.batch_fixed(tcpck.OP_FILL, ptr, stride, length, count, out, mode=mode)
            return host(out).view(np.uint16)
        exp_arena = check_fill(view, offs, lens, mode, run)
        np.testing.assert_array_equal(host(buf)[mis:], exp_arena, err_msg=f"{stride}/{length}x{count} fill arena")
        np.testing.assert_array_equal(host(buf)[:mis], arena_np[:mis])
        # the reference's call shape: no results buffer (the context's scratch)
        buf.copy_(dev(arena_np))
        ctx.batch_fixed(tcpck.OP_FILL, ptr, stride, length, count, None, mode=mode)
        np.testing.assert_array_equal(host(buf)[mis:], exp_arena, err_msg=f"{stride}/{length}x{count} fill, no out")
    if length >= 32 and mis % 2 == 0:
        check_receive(ctx, arena_np, mis, np.arange(count, dtype=np.int64) * stride, np.full(count, length, np.uint32),
                      mode, seed, dict(stride=stride, length=length))


@pytest.mark.parametrize("seed", range(BASE, BASE + (NSEEDS or 200)))
def test_fuzz_var(ctx, oracle_c, seed):
    import tcpck
    rng = np.random.default_rng(2000 + seed)
    kind = rng.choice(["packed", "sorted", "slots", "unordered"])
    dist = rng.choice(["c3", "small", "tiny", "jumbo", "mixed"])
    count = int(rng.integers(1, 30000))
    if dist == "c3":
        ln = np.asarray((96, 608, 1492), np.uint32)[rng.integers(0, 3, count)]
    elif dist == "small":
        ln = (rng.integers(15, 260, count) * 2).astype(np.uint32)
    elif dist == "tiny":
        ln = (rng.integers(0, 20, count) * 2).astype(np.uint32)
    elif dist == "jumbo":
        count = min(count, 200)
        ln = (rng.integers(2000, 33000, count) * 2).astype(np.uint32)
    else:
        ln = np.asarray(rng.choice(LENS, count), np.uint32)
    lens64 = ln.astype(np.uint64)
    if kind == "packed":
        off = np.zeros(count, np.uint64)
        off[1:] = np.cumsum(lens64[:-1])
    elif kind == "slots":
        slot = int((ln.max() + 15) // 16 * 16 + rng.choice([0, 16, 512]))
        off = np.arange(count, dtype=np.uint64) * np.uint64(slot)
    else:
        gaps = (rng.integers(0, 64, count) * 2).astype(np.uint64)
        off = np.zeros(count, np.uint64)
        off[1:] = np.cumsum(lens64[:-1] + gaps[:-1])
        if kind == "unordered":
            perm = rng.permutation(count)
            off, ln = off[perm].copy(), ln[perm].copy()
    total = int((off + ln.astype(np.uint64)).max()) + 256 if count else 256
    if total > (24 << 20):
        return
    mis = int(rng.choice([0, 2, 8]))
    mode = int(rng.random() < 0.35)
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    buf = dev(arena_np)
    ptr = buf.data_ptr() + mis
    view = arena_np[mis:]
    d_off, d_ln = dev(off), dev(ln)
    hints = dict(total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                 packed=kind == "packed", sorted=kind in ("sorted", "slots") or (kind == "unordered" and rng.random() < 0.5))
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, ptr, d_off, d_ln, count, out, mode=mode, **hints)
    exp = oracle_c.batch(view, off, ln, mode=mode, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp, err_msg=f"{kind}/{dist} x{count} mode {mode}")
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, ptr, d_off, d_ln, count, ok, mode=mode, **hints)
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))
    if ln.min() >= 30:  # FILL's precondition

        def run():
            ctx.batch_var(tcpck.OP_FILL, ptr, d_off, d_ln, count, out, mode=mode, **hints)
            return host(out).view(np.uint16)
        exp_arena = check_fill(view, off, ln, mode, run)
        np.testing.assert_array_equal(host(buf)[mis:], exp_arena, err_msg=f"{kind}/{dist} fill arena")
        buf.copy_(dev(arena_np))  # again with no results buffer (the context's scratch)
        ctx.batch_var(tcpck.OP_FILL, ptr, d_off, d_ln, count, None, mode=mode, **hints)
        np.testing.assert_array_equal(host(buf)[mis:], exp_arena, err_msg=f"{kind}/{dist} fill arena, no out")
    if ln.min() >= 32 and kind != "unordered":  # RECEIVE's in-place headers must not overlap
        check_receive(ctx, arena_np, mis, off.astype(np.int64), ln, mode, seed,
                      dict(offsets=d_off, lengths=d_ln, **hints))


@pytest.mark.parametrize("seed", range(BASE, BASE + (NSEEDS or 80)))
def test_fuzz_segment(ctx, seed):
    from oracle import ref16 as R
    rng = np.random.default_rng(3000 + seed)
    seg = int(rng.choice([4, 8, 16, 100, 512, 1024, 1448, 1460, 4096, 8192, 9000, 16384, 32768, 65532]))
    nbytes = int(rng.integers(1, min(12 << 20, seg * 2000) // 2 + 1)) * 2
    stride = (32 + seg + 15) // 16 * 16 + 16 * int(rng.choice([0, 0, 1, 7]))
    mode = int(rng.random() < 0.35)
    mis = int(rng.choice([0, 4, 12]))
    payload = rng.integers(0, 256, nbytes, dtype=np.uint8)
    tmpl = rng.integers(0, 256, 32, dtype=np.uint8)
    seq0 = int(rng.integers(0, 1 << 32))
    n = (nbytes + seg - 1) // seg
    pbuf = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
    pbuf[mis:mis + nbytes] = dev(payload)
    images = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_segment(pbuf.data_ptr() + mis, nbytes, seg, tmpl, seq0, images, stride, out, mode=mode)
    exp, _, exp_cs = R.segment_np(payload, seg, tmpl, seq0, stride=stride, mode=mode)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp_cs, err_msg=f"seg {seg} bytes {nbytes}")
    np.testing.assert_array_equal(host(images), exp)
