"""GPU parity tests: the HIP path (through the C ABI) against the oracle.

* golden vectors (the reference's own outputs) for checksum / fill / verify,
  at unaligned offsets, through every kernel shape;
* seeded random batches (fixed stride and variable length) against the C
  oracle, bit-exact;
* BASELINE.json's full configs (C2 1M x 1492 B, C3 4M mixed, C4 256K x 64 KiB)
  against the oracle (C2, C3 in full; C4 on a sample of images) and through
  size-independent properties (fill -> verify all true, single-byte
  corruption detected exactly where injected);
* the host-memory (PCIe, end-to-end) batch path.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    from conftest import RoutedContext
    c = RoutedContext(0)  # libtcpck.so; measurement-only variants on libtcpck_probe.so
    yield c
    c.close()


def dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy()


SHAPE_HINTS = {"small": 100, "mss": 1500, "jumbo": 65536}


def golden_arrays(golden, kind):
    cases = golden.by_kind(kind)
    off = np.array([c["off"] for c in cases], np.uint64)
    ln = np.array([c["len"] for c in cases], np.uint32)
    exp = np.array([c["expected"] for c in cases])
    return cases, off, ln, exp


@pytest.mark.parametrize("shape", list(SHAPE_HINTS))
def test_golden_checksum(ctx, golden, shape):
    import tcpck
    cases, off, ln, exp = golden_arrays(golden, "checksum")
    arena = dev(golden.blob)
    out = torch.empty(len(cases), dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, arena, dev(off), dev(ln), len(cases), out,
                  total_bytes=SHAPE_HINTS[shape] * len(cases))
    got = host(out).view(np.uint16)
    bad = [(c["name"], int(g), c["expected"]) for c, g in zip(cases, got) if g != c["expected"]]
    assert not bad, bad[:10]


@pytest.mark.parametrize("shape", list(SHAPE_HINTS))
def test_golden_fill_and_verify(ctx, golden, shape):
    import tcpck
    cases, off, ln, exp = golden_arrays(golden, "fill")
    arena = dev(golden.blob)
    out = torch.zeros(len(cases), dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_FILL, arena, dev(off), dev(ln), len(cases), out,
                  total_bytes=SHAPE_HINTS[shape] * len(cases))
    got = host(out).view(np.uint16)
    np.testing.assert_array_equal(got, exp.astype(np.uint16))
    a = host(arena)
    for c in cases:
        np.testing.assert_array_equal(a[c["off"]:c["off"] + c["len"]],
                                      golden.blob[c["fill_off"]:c["fill_off"] + c["len"]],
                                      err_msg=c["name"])
    vcases, voff, vln, vexp = golden_arrays(golden, "verify")
    ok = torch.zeros(len(vcases), dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, dev(golden.blob), dev(voff), dev(vln), len(vcases), ok,
                  total_bytes=SHAPE_HINTS[shape] * len(vcases))
    np.testing.assert_array_equal(host(ok), vexp.astype(np.uint8))


def test_synth_generator_matches_host_restatement(ctx):
    import tcpck
    import synth_np
    for stride, length, kind in ((1492, 1492, 0), (104, 96, 0), (640, 608, 2), (96, 96, 1), (34, 34, 0)):
        n = 37
        a = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, stride, length, n, seed=42, first_index=1000, kind=kind)
        np.testing.assert_array_equal(host(a), synth_np.arena_fixed(42, n, stride, length, 1000, kind))


@pytest.mark.parametrize("stride,length", [(1492, 1492), (1504, 1492), (96, 96), (608, 608),
                                           (1490, 1490), (1496, 1494), (32, 32), (34, 30),
                                           (2, 2), (8, 0), (4096, 4094), (65536, 65536),
                                           (65538, 65534)])
@pytest.mark.parametrize("mode", [0, 1])
def test_fixed_random_vs_oracle(ctx, oracle_c, stride, length, mode):
    import tcpck
    rng = np.random.default_rng(stride * 7 + length + mode)
    count = max(3, min(20000, (24 << 20) // stride))
    arena_np = rng.integers(0, 256, count * stride, dtype=np.uint8)
    if mode == 0 and length >= 4:
        arena_np[:length] = 0xFF  # an adversarial all-ones image
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, stride, length, count, out, mode=mode)
    exp = oracle_c.batch(arena_np, stride=stride, length=length, count=count, mode=mode, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, arena, stride, length, count, ok, mode=mode)
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("shape", list(SHAPE_HINTS))
def test_var_random_ragged_vs_oracle(ctx, oracle_c, mode, shape):
    """Ragged lengths 0..3000 (even), unordered offsets, gaps: every kernel shape."""
    import tcpck
    rng = np.random.default_rng(100 + mode)
    count = 30000
    ln = (rng.integers(0, 1501, count) * 2).astype(np.uint32)
    ln[:50] = np.arange(0, 100, 2)
    gaps = (rng.integers(0, 9, count) * 2).astype(np.uint64)
    off = np.zeros(count, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gaps[:-1])
    total = int(off[-1] + ln[-1]) + 64
    perm = rng.permutation(count)
    off, ln = off[perm], ln[perm]
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, dev(arena_np), dev(off), dev(ln), count, out, mode=mode,
                  total_bytes=SHAPE_HINTS[shape] * count)
    exp = oracle_c.batch(arena_np, off, ln, mode=mode, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("mode", [0, 1])
def test_fill_random_vs_oracle(ctx, oracle_c, mode):
    """Send-side insertion: garbage in bytes 28-29 must not matter, result stored raw."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(200 + mode)
    stride, length, count = 1500, 1492, 5000
    arena_np = rng.integers(0, 256, stride * count, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_FILL, arena, stride, length, count, out, mode=mode)
    got_arena = host(arena)
    exp = np.empty(count, np.uint16)
    for k in range(count):
        img = arena_np[k * stride:k * stride + length].copy()
        exp[k] = R.fill_np(img, mode)
        np.testing.assert_array_equal(got_arena[k * stride:k * stride + length], img)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, arena, stride, length, count, ok, mode=mode)
    assert bool(host(ok).all())
    # FILL with out == NULL writes only the arena
    arena2 = dev(arena_np)
    ctx.batch_fixed(tcpck.OP_FILL, arena2, stride, length, count, None, mode=mode)
    np.testing.assert_array_equal(host(arena2), got_arena)


def test_argument_errors(ctx):
    import tcpck
    a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    o = torch.zeros(16, dtype=torch.int16, device="cuda")
    with pytest.raises(tcpck.TcpckError) as e:
        ctx.batch_fixed(tcpck.OP_CHECKSUM, a, 60, 59, 4, o)
    assert e.value.status == tcpck.EINVAL
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed(tcpck.OP_FILL, a, 28, 28, 4, o)
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed(7, a, 64, 64, 4, o)
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, 64, 64, 0, o)  # empty batch is a no-op


# ---- BASELINE.json configs at full size ------------------------------------------

def _synth_fixed_dev(count, stride, length, seed=42, first_index=0):
    import tcpck
    a = torch.empty(count * stride, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, stride, length, count, seed=seed, first_index=first_index)
    return a


def test_c2_full_1m_x_1492_vs_oracle(ctx, oracle_c):
    import tcpck
    count, L = 1 << 20, 1492
    a = _synth_fixed_dev(count, L, L)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out)
    exp = oracle_c.batch(host(a), stride=L, length=L, count=count, threads=16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    # fill -> verify round trip at full size, then corruption is caught exactly
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, None)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok)
    assert int(ok.sum().item()) == count
    rng = np.random.default_rng(3)
    bad = np.unique(rng.integers(0, count, 1000))
    pos = torch.from_numpy(bad.astype(np.int64) * L + rng.integers(0, L, bad.size)).cuda()
    a[pos] ^= 0x40
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok)
    fails = np.nonzero(host(ok) == 0)[0]
    np.testing.assert_array_equal(fails, bad)


def test_c3_full_4m_mixed_vs_oracle(ctx, oracle_c):
    import tcpck
    import synth_np
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, count, out, total_bytes=int(ln.sum()),
                  min_len=96, max_len=1492, packed=False)
    exp = oracle_c.batch(host(a), off, ln, threads=16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)


def test_c3_full_fill_update_then_verify(ctx, oracle_c):
    """C3 at full size through AUTO's send path (round 3: packed variable batches
    take CHECKSUM's stream + the write-through field-update pass): every result
    against the oracle's FILL on a sample and every image verifying afterwards;
    the bytes outside the fields unchanged."""
    import tcpck
    import synth_np
    from oracle import ref16 as R
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
    before = host(a).copy()
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, count, out, total_bytes=int(ln.sum()), min_len=96, max_len=1492,
                  packed=True)
    got = host(out).view(np.uint16)
    after = host(a)
    rng = np.random.default_rng(4)
    idx = np.unique(np.concatenate([rng.integers(0, count, 5000), [0, count - 1]]))
    for k in idx:
        o, n = int(off[k]), int(ln[k])
        img = before[o:o + n].copy()
        assert R.fill_np(img) == got[k], k
        np.testing.assert_array_equal(after[o:o + n], img, err_msg=f"image {k}")
    fields = (off.astype(np.int64)[:, None] + np.array([28, 29])[None, :]).reshape(-1)
    mask = np.ones(total, bool)
    mask[fields] = False
    np.testing.assert_array_equal(after[mask], before[mask])  # nothing but bytes 28-29 written
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, count, ok, total_bytes=int(ln.sum()), packed=True)
    assert int(ok.sum(dtype=torch.int64).item()) == count
    np.testing.assert_array_equal(oracle_c.batch(after, off, ln, threads=16)[idx], np.zeros(idx.size, np.uint16))


def test_receive_small_ring_full_size(ctx, oracle_c):
    """The small-datagram receive ring AUTO sends to the in-stream header form
    (4M x 32-254-B datagrams in 256-B slots, a third valid): verdicts and every
    header byte against the numpy receive path, the ring unchanged."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(21)
    n, slot = 4 << 20, 256
    ln = (rng.integers(16, 128, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = rng.integers(0, 256, n * slot, dtype=np.uint8)
    for k in range(0, n, 3 * 4096):  # some valid images (FILLed like the send path)
        R.fill_np(a[k * slot:k * slot + int(ln[k])])
    d = dev(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(d, n, ok, hdr, offsets=dev(off), lengths=dev(ln), total_bytes=int(ln.sum()),
                      min_len=int(ln.min()), max_len=int(ln.max()), sorted=True)
    exp_ok = (oracle_c.batch(a, off, ln, threads=16) == 0).astype(np.uint8)
    assert exp_ok.sum() >= n // (3 * 4096)
    np.testing.assert_array_equal(host(ok), exp_ok)
    o = off.astype(np.int64)
    np.testing.assert_array_equal(host(hdr).reshape(n, 32), a[o[:, None] + R.HEADER_PERM[None, :]])
    np.testing.assert_array_equal(host(d), a)


@pytest.mark.parametrize("L", [32, 256])
def test_small_pow2_above_4gib_sampled(ctx, oracle_c, L):
    """Pure-ACK-sized images in a 4.5 GiB arena (byte offsets past 2^32): gstream
    CHECKSUM against the oracle on a sample (both sides of the 4 GiB line, the
    batch end), then the AUTO send path (FILL, gstream) -> VERIFY over every image,
    and CHECKSUM of the filled batch is 0 everywhere except the corrupted images."""
    import tcpck
    count = (9 << 29) // L
    a = _synth_fixed_dev(count, L, L, seed=11)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, count, out, tcpck.KERNEL_GSTREAM, 0)
    got = host(out).view(np.uint16)
    edge = (1 << 32) // L
    idx = np.unique(np.concatenate([np.arange(0, count, 100003), np.arange(edge - 40, edge + 40),
                                    np.arange(count - 70, count)]))
    sample = host(a.view(count, L)[torch.from_numpy(idx).cuda()]).reshape(-1)
    exp = oracle_c.batch(sample, stride=L, length=L, count=idx.size)
    np.testing.assert_array_equal(got[idx], exp)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, None)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok)
    assert int(ok.sum(dtype=torch.int64).item()) == count
    rng = np.random.default_rng(5)
    bad = np.unique(np.concatenate([rng.integers(0, count, 500), [edge, count - 1]]))
    pos = torch.from_numpy(bad.astype(np.int64) * L + rng.integers(0, L, bad.size)).cuda()
    a[pos] ^= 0x11
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, count, out, tcpck.KERNEL_GSTREAM, 2)
    np.testing.assert_array_equal(np.nonzero(host(out) != 0)[0], bad)
    del a


def test_c4_jumbo_256k_x_64k_sampled(ctx, oracle_c):
    import tcpck
    count, L = 256 << 10, 65536
    a = _synth_fixed_dev(count, L, L)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out)
    got = host(out).view(np.uint16)
    idx = np.unique(np.concatenate([np.arange(0, count, 997), [count - 1]]))
    sample = host(a.view(count, L)[torch.from_numpy(idx).cuda()]).reshape(-1)
    exp = oracle_c.batch(sample, stride=L, length=L, count=idx.size, threads=16)
    np.testing.assert_array_equal(got[idx], exp)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, None)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok)
    assert int(ok.sum().item()) == count
    del a
    torch.cuda.empty_cache()


# ---- host-memory (end-to-end) path -------------------------------------------------

@pytest.mark.parametrize("op", [0, 1, 2])
def test_host_batch_fixed_vs_oracle(ctx, oracle_c, op):
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(300 + op)
    stride, length, count = 1492, 1492, 50000
    arena = rng.integers(0, 256, stride * count, dtype=np.uint8)
    ctx.set_chunk_bytes(8 << 20)  # several chunks, both streams
    if op == tcpck.OP_VERIFY:
        for k in range(0, count, 2):
            R.fill_np(arena[k * stride:(k + 1) * stride])
    before = arena.copy()
    out = np.zeros(count, np.uint8 if op == tcpck.OP_VERIFY else np.uint16)
    ctx.host_batch_fixed(op, arena, stride, length, count, out)
    if op == tcpck.OP_CHECKSUM:
        np.testing.assert_array_equal(out, oracle_c.batch(before, stride=stride, length=length, count=count))
    elif op == tcpck.OP_VERIFY:
        exp = oracle_c.batch(before, stride=stride, length=length, count=count) == 0
        np.testing.assert_array_equal(out, exp.astype(np.uint8))
        assert out[::2].all()
    else:
        for k in range(0, count, 101):
            img = before[k * stride:(k + 1) * stride].copy()
            assert R.fill_np(img) == out[k]
            np.testing.assert_array_equal(arena[k * stride:(k + 1) * stride], img)


def test_host_batch_var_vs_oracle(ctx, oracle_c):
    import tcpck
    import synth_np
    rng = np.random.default_rng(400)
    count = 100000
    off, ln, total = synth_np.mixed_layout(count, seed=7)
    arena = rng.integers(0, 256, total, dtype=np.uint8)
    out = np.zeros(count, np.uint16)
    ctx.set_chunk_bytes(16 << 20)
    ctx.host_batch_var(tcpck.OP_CHECKSUM, arena, off, ln, count, out)
    np.testing.assert_array_equal(out, oracle_c.batch(arena, off, ln, threads=8))


@pytest.mark.parametrize("op", [0, 1, 2])
def test_host_batch_var_slots_vs_oracle(ctx, oracle_c, op):
    """Host receive arena in 2048-B slots (recv_burst's layout): the host sees the
    offsets ascend and passes TCPCK_LAYOUT_SORTED, so the chunks run on sstream."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(401 + op)
    count = 60000
    ln = np.asarray((96, 608, 1492), np.uint32)[rng.integers(0, 3, count)]
    off = np.arange(count, dtype=np.uint64) * 2048 + 2
    arena = rng.integers(0, 256, count * 2048 + 16, dtype=np.uint8)
    before = arena.copy()
    out = np.zeros(count, np.uint16 if op != 2 else np.uint8)
    ctx.set_chunk_bytes(16 << 20)
    ctx.host_batch_var(op, arena, off, ln, count, out)
    if op == 1:
        exp = np.array([R.fill_np(before[int(off[k]):int(off[k]) + int(ln[k])]) for k in range(count)], np.uint16)
        np.testing.assert_array_equal(out, exp)
        np.testing.assert_array_equal(arena, before)  # fill_np patched `before` in place, as the reference
    else:
        exp = oracle_c.batch(arena, off, ln, threads=8)
        np.testing.assert_array_equal(out, exp if op == 0 else (exp == 0).astype(np.uint8))



def test_host_batch_recovers_after_failed_stage_growth(ctx, oracle_c):
    """a staging-buffer growth that fails with ENOMEM must
    leave the context usable.  A 30-TiB chunk request fails inside ensure_stage
    before the host arena is touched; the next normal-size batch must run on the
    previous buffers and be bit-exact."""
    import tcpck
    rng = np.random.default_rng(310)
    stride = length = 1492
    count = 20000
    arena = rng.integers(0, 256, stride * count, dtype=np.uint8)
    out = np.zeros(count, np.uint16)
    ctx.set_chunk_bytes(8 << 20)
    ctx.host_batch_fixed(tcpck.OP_CHECKSUM, arena, stride, length, count, out)
    exp = oracle_c.batch(arena, stride=stride, length=length, count=count)
    np.testing.assert_array_equal(out, exp)
    ctx.set_chunk_bytes(1 << 45)
    with pytest.raises(tcpck.TcpckError) as e:
        # 32 images per chunk at a 1-TiB stride: ~31 TiB of staging, far above HBM
        ctx.host_batch_fixed(tcpck.OP_CHECKSUM, arena, 1 << 40, length, 64, out)
    assert e.value.status == tcpck.ENOMEM
    ctx.set_chunk_bytes(8 << 20)
    out[:] = 0
    ctx.host_batch_fixed(tcpck.OP_CHECKSUM, arena, stride, length, count, out)
    np.testing.assert_array_equal(out, exp)
    torch.cuda.synchronize()
    t = torch.ones(1 << 20, device="cuda") * 2  # torch's own launch checks see no stale error
    assert float(t.sum().item()) == 2.0 * (1 << 20)


@pytest.mark.parametrize("length", [96, 1492, 9000])
@pytest.mark.parametrize("op", [0, 1, 2])
def test_single_image_any_stride(ctx, oracle_c, length, op):
    """count == 1 with stride < len (e.g. 0) is a valid batch of
    one image, on the device and the host path alike."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(320 + length + op)
    img = rng.integers(0, 256, length, dtype=np.uint8)
    if op == tcpck.OP_VERIFY:
        R.fill_np(img)
    exp_img = img.copy()
    exp = R.fill_np(exp_img) if op == tcpck.OP_FILL else oracle_c.one(img)
    want = np.uint8(exp == 0) if op == tcpck.OP_VERIFY else np.uint16(exp)
    dt = torch.uint8 if op == tcpck.OP_VERIFY else torch.int16
    for stride in (0, 2, length):
        a = dev(img)
        o = torch.zeros(1, dtype=dt, device="cuda")
        ctx.batch_fixed(op, a, stride, length, 1, o)
        got = host(o).view(np.uint8 if op == tcpck.OP_VERIFY else np.uint16)[0]
        assert got == want, (stride, got, want)
        if op == tcpck.OP_FILL:
            np.testing.assert_array_equal(host(a), exp_img)
        h = img.copy()
        ho = np.zeros(1, np.uint8 if op == tcpck.OP_VERIFY else np.uint16)
        ctx.host_batch_fixed(op, h, stride, length, 1, ho)
        assert ho[0] == want, (stride, ho[0], want)
        if op == tcpck.OP_FILL:
            np.testing.assert_array_equal(h, exp_img)


def test_host_batch_fixed_rejects_wrapping_stride(ctx):
    """the host fixed path has the device path's overflow guard."""
    import tcpck
    arena = np.zeros(4096, np.uint8)
    out = np.zeros(4, np.uint16)
    with pytest.raises(tcpck.TcpckError) as e:
        ctx.host_batch_fixed(tcpck.OP_CHECKSUM, arena, (1 << 63), 1492, 4, out)
    assert e.value.status == tcpck.EINVAL
    with pytest.raises(tcpck.TcpckError) as e:
        ctx.batch_fixed(tcpck.OP_CHECKSUM, dev(arena), (1 << 63), 1492, 4,
                        torch.zeros(4, dtype=torch.int16, device="cuda"))
    assert e.value.status == tcpck.EINVAL

# ---- retransmit: batched ACK rewrite + incremental update ----

@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("layout", ["fixed", "var"])
@pytest.mark.parametrize("per_image", [False, True])
def test_set_ack_vs_resend_oracle(ctx, mode, layout, per_image):
    """tcpck_batch_set_ack after FILL == the reference's resend path (ACK
    rewrite, socket-internal.h:376-377, then SendPacket's full recompute,
    socket-manager.cc:9-10) on every image: arena bytes and checksums."""
    import tcpck
    import synth_np
    from oracle import ref16 as R
    rng = np.random.default_rng(500 + mode + 2 * per_image)
    if layout == "fixed":
        stride, length, count = 1500, 1492, 20000
        off = np.arange(count, dtype=np.int64) * stride
        ln = np.full(count, length, np.int64)
        total = stride * count
    else:
        count = 20000
        off, ln, total = synth_np.mixed_layout(count, seed=11)
        gaps = 2 * (np.arange(count) % 3 == 0)  # 2-B gaps: starts that are 2 mod 4
        off = off.astype(np.int64) + np.cumsum(gaps)
        total = int(off[-1] + ln[-1])
    arena_np = rng.integers(0, 256, total + 64, dtype=np.uint8)
    arena = dev(arena_np)
    d_off = dev(off.astype(np.uint64))
    d_ln = dev(ln.astype(np.uint32))
    ctx.batch_var(tcpck.OP_FILL, arena, d_off, d_ln, count, None, mode=mode)
    filled = host(arena)
    acks = rng.integers(0, 2**32, count, dtype=np.uint64).astype(np.uint32) if per_image else np.uint32(0x9ABCDEF1)
    out = torch.zeros(count, dtype=torch.int16, device="cuda")
    kw = dict(acks=dev(acks)) if per_image else dict(ack=int(acks))
    if layout == "fixed":
        ctx.batch_set_ack(arena, count, stride=stride, out=out, mode=mode, **kw)
    else:
        ctx.batch_set_ack(arena, count, offsets=d_off, out=out, mode=mode, **kw)
    exp_arena = filled.copy()
    exp = R.resend_batch_np(exp_arena, off, ln, acks, mode)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    np.testing.assert_array_equal(host(arena), exp_arena)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, arena, d_off, d_ln, count, ok, mode=mode)
    assert bool(host(ok).all())


def test_set_ack_c2_full_size_roundtrip(ctx, oracle_c):
    """BASELINE C2 (1M x 1492 B): FILL, then two successive ACK rewrites; every image
    verifies and the checksums equal a fresh FILL of the rewritten images."""
    import tcpck
    count, L = 1 << 20, 1492
    a = _synth_fixed_dev(count, L, L)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, None)
    acks = torch.arange(count, dtype=torch.int32, device="cuda") * 7 + 12345
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_set_ack(a, count, ack=0xFFFFFFFF, stride=L)
    ctx.batch_set_ack(a, count, acks=acks, stride=L, out=out)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok)
    assert bool(host(ok).all())
    b = a.clone()
    refill = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_FILL, b, L, L, count, refill)
    assert torch.equal(out, refill) and torch.equal(a, b)
    hdr = host(a[: 64])
    assert hdr[20:24].tolist() == list((12345).to_bytes(4, "big"))


def test_set_ack_argument_errors(ctx):
    import tcpck
    a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_set_ack(a, 4, stride=63)   # odd stride
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_set_ack(a, 4, stride=28)   # images shorter than the header
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_set_ack(a, 4, stride=64, mode=5)
    ctx.batch_set_ack(a, 0, stride=64)       # empty batch is a no-op


# ---- AUTO policy boundaries: rstream / jumbo W-shapes / vvstream / gstream hand-overs ----------


@pytest.mark.parametrize("length", [32, 48, 64, 96, 240, 256, 1024])
@pytest.mark.parametrize("mis", [0, 2, 16])
def test_auto_fill_small_pow2_alignment(ctx, length, mis):
    """AUTO FILL of power-of-two images (and multiples of 16 B up to 240 B) takes gstream only for a 16-B aligned arena;
    any other pointer goes to the general kernels -- same arena bytes and results."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length * 3 + mis)
    count = 5000
    arena_np = rng.integers(0, 256, count * length + 64, dtype=np.uint8)
    buf = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_FILL, buf.data_ptr() + mis, length, length, count, out)
    exp_arena = arena_np.copy()
    img = exp_arena[mis:]
    exp = np.array([R.fill_np(img[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    np.testing.assert_array_equal(host(buf), exp_arena)

@pytest.mark.parametrize("length", [30, 32, 34, 48, 64, 96, 128, 240, 256, 258, 272, 510, 512, 1024, 1026, 4094, 4096,
                                    4098, 5000, 6144, 8192, 8194, 9000, 16384, 16386, 24578, 28000, 32768, 32770,
                                    49152, 60000, 98304])
@pytest.mark.parametrize("mode", [0, 1])
def test_auto_policy_boundaries_fixed(ctx, oracle_c, length, mode):
    """Packed fixed batches at every length where the AUTO policy changes kernel or
    waves per image: CHECKSUM, FILL (arena and results) and VERIFY against the oracle."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + 7 * mode)
    count = max(8, min(4000, (48 << 20) // length))
    arena_np = rng.integers(0, 256, count * length, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, length, length, count, out, mode=mode)
    exp = oracle_c.batch(arena_np, stride=length, length=length, count=count, mode=mode, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ctx.batch_fixed(tcpck.OP_FILL, arena, length, length, count, out, mode=mode)
    filled = host(arena)
    exp_arena = arena_np.copy()
    exp_fill = np.array([R.fill_np(exp_arena[k * length:(k + 1) * length], mode) for k in range(count)],
                        np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp_fill)
    np.testing.assert_array_equal(filled, exp_arena)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, arena, length, length, count, ok, mode=mode)
    assert bool(host(ok).all())


@pytest.mark.parametrize("length,stride", [(4500, 4608), (9000, 9216), (9000, 9088), (20000, 20480),
                                           (40000, 40960), (65536, 69632), (9000, 12000), (4098, 4100)])
def test_auto_policy_jumbo_gapped(ctx, oracle_c, length, stride):
    """Jumbo images in slots: small gaps go to vvstream (virtual gap images), larger
    ones and FILL to seg.  CHECKSUM, FILL (results, fields, untouched gaps), VERIFY."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + stride)
    count = max(8, min(1200, (48 << 20) // stride))
    arena_np = rng.integers(0, 256, count * stride, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, stride, length, count, out)
    np.testing.assert_array_equal(host(out).view(np.uint16),
                                  oracle_c.batch(arena_np, stride=stride, length=length, count=count, threads=8))
    ctx.batch_fixed(tcpck.OP_FILL, arena, stride, length, count, out)
    exp_arena = arena_np.copy()
    exp = np.array([R.fill_np(exp_arena[k * stride:k * stride + length]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    np.testing.assert_array_equal(host(arena), exp_arena)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, arena, stride, length, count, ok)
    assert bool(host(ok).all())


@pytest.mark.parametrize("typical", [6000, 12000, 20000, 24000, 40000, 60000])
def test_auto_policy_jumbo_var(ctx, oracle_c, typical):
    """Variable layouts whose typical length selects a W-waves-per-image shape, with
    lengths spread around it (some far shorter, some zero), packed and with gaps."""
    import tcpck
    rng = np.random.default_rng(typical)
    count = 1500
    ln = (rng.integers(0, 2 * typical, count) // 2 * 2).astype(np.uint32)
    ln[::97] = 0
    for gaps in (False, True):
        g = (rng.integers(0, 3, count) * 2) if gaps else np.zeros(count, np.int64)
        off = (np.concatenate([[0], np.cumsum(ln[:-1].astype(np.int64) + g[:-1])])).astype(np.uint64)
        total = int(off[-1] + ln[-1])
        arena_np = rng.integers(0, 256, total + 16, dtype=np.uint8)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_var(tcpck.OP_CHECKSUM, dev(arena_np), dev(off), dev(ln), count, out,
                      total_bytes=int(ln.sum()), packed=not gaps)
        np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np, off, ln, threads=8))


@pytest.mark.parametrize("length,stride", [(1492, 2048), (1024, 2048), (96, 256), (1492, 4096), (30, 64),
                                           (9000, 16384), (1494, 2048), (1492, 2000)])
@pytest.mark.parametrize("mis", [0, 6])
def test_auto_policy_fixed_slots(ctx, oracle_c, length, stride, mis):
    """Slots with larger gaps: sstream where the slot is a multiple of 16 B, else
    seg.  CHECKSUM, FILL (results, fields, untouched gaps), VERIFY."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + stride + mis)
    count = max(8, min(20000, (48 << 20) // stride))
    arena_np = rng.integers(0, 256, count * stride + 16, dtype=np.uint8)
    buf = dev(arena_np)
    ptr = buf.data_ptr() + mis
    view = arena_np[mis:]
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, ptr, stride, length, count, out)
    np.testing.assert_array_equal(host(out).view(np.uint16),
                                  oracle_c.batch(view, stride=stride, length=length, count=count, threads=8))
    ctx.batch_fixed(tcpck.OP_FILL, ptr, stride, length, count, out)
    exp_arena = view.copy()
    exp = np.array([R.fill_np(exp_arena[k * stride:k * stride + length]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    np.testing.assert_array_equal(host(buf)[mis:], exp_arena)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, ptr, stride, length, count, ok)
    assert bool(host(ok).all())


@pytest.mark.parametrize("slot,mix", [(2048, (96, 608, 1492)), (1536, (32, 1492)), (2050, (34, 606, 1494)),
                                      (65600, (40, 65536))])
@pytest.mark.parametrize("hint", ["sorted", "none", "sorted_wrong"])
def test_auto_policy_var_slots(ctx, oracle_c, slot, mix, hint):
    """Variable images in receive slots: with TCPCK_LAYOUT_SORTED AUTO takes
    sstream for CHECKSUM/VERIFY (seg without the hint, and for FILL); a wrong
    SORTED hint (shuffled offsets) costs speed, never correctness."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(slot + len(mix) + len(hint))
    count = max(8, min(30000, (64 << 20) // slot))
    ln = np.asarray(mix, np.uint32)[rng.integers(0, len(mix), count)]
    off = np.arange(count, dtype=np.uint64) * np.uint64(slot)
    if hint == "sorted_wrong":
        perm = rng.permutation(count)
        off, ln = off[perm].copy(), ln[perm].copy()
    arena_np = rng.integers(0, 256, count * slot + 16, dtype=np.uint8)
    arena = dev(arena_np)
    d_off, d_ln = dev(off), dev(ln)
    kw = dict(total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()), sorted=hint != "none")
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, arena, d_off, d_ln, count, out, **kw)
    exp = oracle_c.batch(arena_np, off, ln, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, arena, d_off, d_ln, count, ok, **kw)
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))
    ctx.batch_var(tcpck.OP_FILL, arena, d_off, d_ln, count, out, **kw)
    exp_arena = arena_np.copy()
    expf = np.array([R.fill_np(exp_arena[int(off[k]):int(off[k]) + int(ln[k])]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), expf)
    np.testing.assert_array_equal(host(arena), exp_arena)
    ctx.batch_var(tcpck.OP_VERIFY, arena, d_off, d_ln, count, ok, **kw)
    assert bool(host(ok).all())


def test_concurrent_threads_and_streams(ctx, oracle_c):
    """The ABI is reentrant (the reference calls the checksum from
    several threads unlocked): four host threads, each on its own HIP stream
    and its own layout, launch batches concurrently on one ctx and on a second
    ctx; every result equals the oracle."""
    import threading
    import tcpck
    import synth_np
    ctx2 = tcpck.Context(0)
    rng = np.random.default_rng(77)
    jobs = []
    for t in range(4):
        if t % 2 == 0:
            L, n = (1492, 96)[t // 2], 30000
            a = rng.integers(0, 256, n * L, dtype=np.uint8)
            jobs.append(("fixed", a, L, n, oracle_c.batch(a, stride=L, length=L, count=n, threads=4)))
        else:
            off, ln, total = synth_np.mixed_layout(30000, seed=t)
            a = rng.integers(0, 256, total, dtype=np.uint8)
            jobs.append(("var", a, (off, ln, total), 30000, oracle_c.batch(a, off, ln, threads=4)))
    errors = []

    def worker(t):
        try:
            c = ctx if t < 2 else ctx2
            s = torch.cuda.Stream()
            kind, a, geo, n, exp = jobs[t]
            with torch.cuda.stream(s):
                buf = torch.from_numpy(a).cuda()
                out = torch.empty(n, dtype=torch.int16, device="cuda")
                if kind == "var":
                    off, ln, total = geo
                    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            s.synchronize()
            for _ in range(50):
                if kind == "fixed":
                    c.batch_fixed(tcpck.OP_CHECKSUM, buf, geo, geo, n, out, stream=s)
                else:
                    c.batch_var(tcpck.OP_CHECKSUM, buf, d_off, d_ln, n, out, total_bytes=int(ln.sum()), packed=True,
                                stream=s)
            s.synchronize()
            if not np.array_equal(out.cpu().numpy().view(np.uint16), exp):
                errors.append(f"thread {t}: mismatch")
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(f"thread {t}: {e!r}")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    ctx2.close()
    assert not errors, errors
