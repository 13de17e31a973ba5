"""GPU parity: vvstream's whole-block FILL (param | 128, BLK).

Each field leaves as its whole 64-B block from the stream's registers, so the
block's other 62 bytes -- possibly another run's image, or bytes past the
run's span -- are written back too: they must come back unchanged.  Every
arena byte, the bytes around the batch included, is compared with the
reference's insert (src/socket-manager.cc:9-10: field zeroed, then
CalculateChecksum, include/tcp-header.h:252-263, stored raw at bytes 28-29),
through oracle/ref16.c (pinned by tests/golden); the results too.

Cases: packed offset lists of 64 B .. 4 KiB images (4-B and 2-B aligned ends,
the prefix table's u32 and packed u16 forms), C3's mix, fixed packed strides,
batches that start and end off the 64-B grid (blocks reaching outside the
batch take the 2-B store), tiny batches, several grid sizes (run edges in
different places), images below 64 B (the exact per-image fallback), and no
results buffer.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_gpu_full_paths import expected_fill  # noqa: E402

VV_POLICY = 4 | 8 | 16
BLK = 128


@pytest.fixture(scope="module")
def pctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = tcpck.Context(0, probe=True)
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _run_var(ctx, oracle_c, ln, pad_lo, pad_hi, m, with_out, seed):
    import tcpck
    rng = np.random.default_rng(seed)
    off = np.zeros(ln.size, np.int64)
    off[1:] = np.cumsum(ln[:-1].astype(np.int64))
    off += pad_lo
    total = int(off[-1] + ln[-1]) + pad_hi
    a_h = rng.integers(0, 256, total, dtype=np.uint8)
    want = expected_fill(a_h, off, ln, oracle_c)
    a = dev(a_h)
    out = torch.full((ln.size,), -1, dtype=torch.int16, device="cuda") if with_out else None
    img = int(ln.astype(np.int64).sum())
    ctx.batch_var_ex(tcpck.OP_FILL, a, dev(off.astype(np.uint64)), dev(ln.astype(np.uint32)), ln.size, out,
                     tcpck.KERNEL_VVSTREAM, VV_POLICY | BLK | (m << 16), total_bytes=img, min_len=int(ln.min()),
                     max_len=int(ln.max()), packed=True)
    np.testing.assert_array_equal(host(a), want)
    if with_out:
        fw = want[off + 28].astype(np.uint16) | (want[off + 29].astype(np.uint16) << 8)
        np.testing.assert_array_equal(host(out).view(np.uint16), fw)


@pytest.mark.parametrize("lens", ["64-4096", "64-256", "c3", "1492", "2mod4"])
@pytest.mark.parametrize("pad_lo", [0, 2, 6, 64, 126])
@pytest.mark.parametrize("m", [0, 1, 16, 64])
def test_blk_var_packed(pctx, oracle_c, lens, pad_lo, m):
    rng = np.random.default_rng(zlib.crc32(f"{lens}/{pad_lo}/{m}".encode()))
    n = 60000
    if lens == "64-4096":
        ln = rng.integers(32, 2049, n) * 2
    elif lens == "64-256":
        ln = rng.integers(32, 129, n) * 2
    elif lens == "c3":
        ln = np.asarray((96, 608, 1492))[rng.integers(0, 3, n)]
    elif lens == "1492":
        ln = np.full(n, 1492)
    else:  # every length 2 mod 4: ends alternate between 4-B and 2-B alignment
        ln = rng.integers(16, 400, n) * 4 + 2
    _run_var(pctx, oracle_c, ln.astype(np.uint32), pad_lo, 2 + 2 * (pad_lo % 7), m, True, pad_lo + m)


@pytest.mark.parametrize("count", [1, 2, 3, 63, 64, 65, 257])
@pytest.mark.parametrize("L", [64, 66, 96, 1492])
def test_blk_var_tiny(pctx, oracle_c, count, L):
    """Tiny batches: every block near the batch's edges."""
    _run_var(pctx, oracle_c, np.full(count, L, np.uint32), 6, 10, 0, True, count * 10 + L)


def test_blk_var_short_images_fall_back(pctx, oracle_c):
    """Images below 64 B (two fields may share a block): the runs holding one
    take the exact per-image pass -- same bytes."""
    rng = np.random.default_rng(5)
    ln = rng.integers(32, 800, 50000) * 2
    ln[rng.integers(0, ln.size, 40)] = 30
    _run_var(pctx, oracle_c, ln.astype(np.uint32), 4, 4, 0, True, 5)


@pytest.mark.parametrize("with_out", [False, True])
def test_blk_var_c3_full(pctx, oracle_c, with_out):
    """C3's batch (4M images, 3.07 GB), bench seeds: whole arena exact."""
    import tcpck
    import synth_np
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=44)
    want = expected_fill(host(a), off, ln, oracle_c)
    out = torch.empty(count, dtype=torch.int16, device="cuda") if with_out else None
    pctx.batch_var_ex(tcpck.OP_FILL, a, d_off, d_ln, count, out, tcpck.KERNEL_VVSTREAM, VV_POLICY | BLK,
                      total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                      packed=True)
    np.testing.assert_array_equal(host(a), want)
    if with_out:
        o = off.astype(np.int64)
        fw = want[o + 28].astype(np.uint16) | (want[o + 29].astype(np.uint16) << 8)
        np.testing.assert_array_equal(host(out).view(np.uint16), fw)


@pytest.mark.parametrize("L", [64, 66, 96, 250, 1492, 4098])
@pytest.mark.parametrize("count", [1, 5, 64, 1000, 70001])
@pytest.mark.parametrize("pad_lo", [0, 2, 38])
def test_blk_fixed_packed(pctx, oracle_c, L, count, pad_lo):
    import tcpck
    rng = np.random.default_rng(L * 3 + count + pad_lo)
    total = pad_lo + count * L + 6
    a_h = rng.integers(0, 256, total, dtype=np.uint8)
    offs = pad_lo + np.arange(count, dtype=np.int64) * L
    want = expected_fill(a_h, offs, np.full(count, L), oracle_c)
    buf = dev(a_h)
    view = buf[pad_lo:]
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    pctx.batch_fixed_ex(tcpck.OP_FILL, view, L, L, count, out, tcpck.KERNEL_VVSTREAM, VV_POLICY | BLK)
    np.testing.assert_array_equal(host(buf), want)
    fw = want[offs + 28].astype(np.uint16) | (want[offs + 29].astype(np.uint16) << 8)
    np.testing.assert_array_equal(host(out).view(np.uint16), fw)


def test_blk_rejected_where_it_does_not_apply(pctx):
    """BLK is reference-mode FILL without gaps: RFC 1071, CHECKSUM and gapped strides are refused."""
    import tcpck
    a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = torch.empty(64, dtype=torch.int16, device="cuda")
    for op, mode, stride in ((tcpck.OP_FILL, 1, 512), (tcpck.OP_CHECKSUM, 0, 512), (tcpck.OP_FILL, 0, 640)):
        with pytest.raises(tcpck.TcpckError):
            pctx.batch_fixed_ex(op, a, stride, 512, 64, out, tcpck.KERNEL_VVSTREAM, VV_POLICY | BLK, mode=mode)
