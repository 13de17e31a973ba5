"""GPU parity: rvstream, rstream's scalar boundary walk over packed offset
lists (TCPCK_KERNEL_RVSTREAM, round 5; libtcpck_probe.so only).

Every result against the oracle (oracle/ref16.c restating
include/tcp-header.h:252-263, pinned by tests/golden): CHECKSUM u16 and VERIFY
u8, on packed batches of many densities -- empty and 2-B images, 16-B images,
jumbo images, lengths = 2 mod 4 -- at several grids (so runs of 1 to > 128
images, run edges everywhere), misaligned arenas, batches whose runs end in
zero-length images, and on layouts that are NOT packed (gaps, overlaps,
shuffled offsets), which the runs detect and recompute exactly.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def pctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = tcpck.Context(0, probe=True)
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _lens(kind, n, rng):
    if kind == "c3":
        return np.asarray((96, 608, 1492))[rng.integers(0, 3, n)]
    if kind == "small":
        return rng.integers(0, 65, n) * 2
    if kind == "mixed":
        return rng.integers(0, 2049, n) * 2
    if kind == "jumbo":
        return rng.integers(0, 16385, n) * 2
    if kind == "zeros":  # many empty images, runs ending in them
        ln = rng.integers(1, 400, n) * 2
        ln[rng.random(n) < 0.3] = 0
        return ln
    if kind == "2mod4":
        return rng.integers(0, 300, n) * 4 + 2
    raise ValueError(kind)


def _run(ctx, oracle_c, ln, mis, op, param, seed, offsets=None):
    import tcpck
    rng = np.random.default_rng(seed)
    ln = ln.astype(np.uint32)
    if offsets is None:
        off = np.zeros(ln.size, np.int64)
        off[1:] = np.cumsum(ln[:-1].astype(np.int64))
        off += mis
    else:
        off = offsets
    total = int((off + ln).max()) + 64 if ln.size else 64
    a = rng.integers(0, 256, total, dtype=np.uint8)
    exp = oracle_c.batch(a, off.astype(np.uint64), ln, threads=16)
    out = (torch.full((ln.size,), -1, dtype=torch.int16, device="cuda") if op == tcpck.OP_CHECKSUM else
           torch.full((ln.size,), 255, dtype=torch.uint8, device="cuda"))
    packed = offsets is None
    ctx.batch_var_ex(op, dev(a), dev(off.astype(np.uint64)), dev(ln), ln.size, out, tcpck.KERNEL_RVSTREAM, param,
                     total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                     packed=packed)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    if op == tcpck.OP_CHECKSUM:
        np.testing.assert_array_equal(got.view(np.uint16), exp)
    else:
        np.testing.assert_array_equal(got, (exp == 0).astype(np.uint8))


@pytest.mark.parametrize("kind", ["c3", "small", "mixed", "jumbo", "zeros", "2mod4"])
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 129, 5000])
@pytest.mark.parametrize("m", [0, 1, 32])
def test_rvstream_checksum(pctx, oracle_c, kind, n, m):
    import tcpck
    seed = zlib.crc32(f"{kind}/{n}/{m}".encode())
    rng = np.random.default_rng(seed)
    _run(pctx, oracle_c, _lens(kind, n, rng), 2 * (seed % 64), tcpck.OP_CHECKSUM, m << 16, seed)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("m", [0, 2, 16, 256])
@pytest.mark.parametrize("op", ["checksum", "verify"])
def test_rvstream_variants_grids(pctx, oracle_c, variant, m, op):
    """60000 images of C3's mix (runs from 1 to thousands of images): every result."""
    import tcpck
    seed = zlib.crc32(f"{variant}/{m}/{op}".encode())
    rng = np.random.default_rng(seed)
    o = tcpck.OP_CHECKSUM if op == "checksum" else tcpck.OP_VERIFY
    _run(pctx, oracle_c, _lens("c3", 60000, rng), 6, o, variant | (m << 16), seed)


def test_rvstream_verify_filled(pctx, oracle_c):
    """VERIFY on images after the reference's insert: all 1, then one bit flipped per 7th image."""
    import tcpck
    import synth_np
    n = 200000
    off, ln, total = synth_np.mixed_layout(n, seed=5)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, n, seed=5)
    pctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, n, None)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hints = dict(total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()), packed=True)
    pctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, tcpck.KERNEL_RVSTREAM, 0, **hints)
    assert int(ok.sum(dtype=torch.int64).item()) == n
    bad = np.arange(0, n, 7)
    h = a.cpu().numpy()
    pos = off[bad].astype(np.int64) + 40
    h[pos] ^= 0x10
    a.copy_(torch.from_numpy(h))
    pctx.batch_var_ex(tcpck.OP_VERIFY, a, d_off, d_ln, n, ok, tcpck.KERNEL_RVSTREAM, 0, **hints)
    want = np.ones(n, np.uint8)
    want[bad] = 0
    np.testing.assert_array_equal(ok.cpu().numpy(), want)


@pytest.mark.parametrize("layout", ["gaps", "overlap", "shuffled"])
def test_rvstream_not_packed_recomputes(pctx, oracle_c, layout):
    """Offsets that are not back to back (the PACKED hint wrong): the runs whose
    lengths do not add up to their span take the exact per-image pass."""
    import tcpck
    rng = np.random.default_rng(["gaps", "overlap", "shuffled"].index(layout))
    n = 20000
    ln = (rng.integers(8, 800, n) * 2).astype(np.uint32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(ln[:-1].astype(np.int64))
    if layout == "gaps":
        off += np.cumsum(rng.integers(0, 3, n) * 2)
    elif layout == "overlap":
        off = np.maximum(off - np.cumsum(rng.integers(0, 2, n) * 2), 0)
    else:
        off = off[rng.permutation(n)]
    _run(pctx, oracle_c, ln, 0, tcpck.OP_CHECKSUM, 0, 11, offsets=off)


def test_rvstream_c3_full(pctx, oracle_c):
    """C3's whole batch (4M images, the bench's seeds)."""
    import tcpck
    import synth_np
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    pctx.batch_var_ex(tcpck.OP_CHECKSUM, a, d_off, d_ln, count, out, tcpck.KERNEL_RVSTREAM, 0,
                     total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                     packed=True)
    exp = oracle_c.batch(a.cpu().numpy(), off, ln, threads=16)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp)


def test_rvstream_rejects(pctx):
    import tcpck
    a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    off = dev(np.arange(4, dtype=np.uint64) * 1024)
    ln = dev(np.full(4, 1024, np.uint32))
    out = torch.empty(4, dtype=torch.int16, device="cuda")
    for op, mode, o in ((tcpck.OP_FILL, 0, out), (tcpck.OP_CHECKSUM, 1, out), (tcpck.OP_CHECKSUM, 0, None)):
        with pytest.raises(tcpck.TcpckError):
            pctx.batch_var_ex(op, a, off, ln, 4, o, tcpck.KERNEL_RVSTREAM, 0, mode=mode)


def test_rvstream_refused_by_the_product(built_lib):
    """Not AUTO's kernel: the product library refuses it (hipErrorInvalidValue)."""
    import tcpck
    c = tcpck.Context(0)
    try:
        a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
        off = dev(np.arange(4, dtype=np.uint64) * 1024)
        ln = dev(np.full(4, 1024, np.uint32))
        out = torch.empty(4, dtype=torch.int16, device="cuda")
        with pytest.raises(tcpck.TcpckError):
            c.batch_var_ex(tcpck.OP_CHECKSUM, a, off, ln, 4, out, tcpck.KERNEL_RVSTREAM, 0, packed=True)
    finally:
        c.close()
