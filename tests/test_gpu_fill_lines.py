"""FILL's line form (rstream variant 31): the stream sums every image outside
the 128-B lines holding the checksum fields, then one pass per image reads its
field line, adds the image's words there (and at the start of the next image's
field line), and writes the line back whole with the checksum in bytes 28-29
(tcpck_rstream.hip FLAV bit 8, tcpck_header.hip fill_lines_kernel).

Against the oracle's FILL (socket-manager.cc:9-10: Checksum() = 0, then
CalculateChecksum, include/tcp-header.h:252-263): every arena byte, every
result, and the bytes around the arena untouched -- every line alignment of
the arena (the first image's line may begin before it), stale fields, all-0xFF
and all-zero images, both modes, small and odd counts, past the context
scratch (no results buffer), and C2 at full size."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LINE_FILL = 31


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available()
    c = tcpck.Context(0)
    yield c
    c.close()


def expected_fill(a, mis, length, count, mode):
    """The arena after FILL and the results (oracle: fields zeroed, then summed)."""
    from oracle import ref16 as R
    exp = a.copy()
    v = exp[mis:mis + count * length].reshape(count, length)
    v[:, 28:30] = 0
    off = np.arange(count, dtype=np.int64) * length
    ln = np.full(count, length, np.int64)
    want = (R.ref16_batch_np(exp[mis:], off, ln, mode)).astype(np.uint16)
    v[:, 28:30] = want.view(np.uint8).reshape(count, 2)
    return exp, want


def run(ctx, a, mis, length, count, mode, pad=256):
    import tcpck
    buf = torch.from_numpy(a).cuda()
    out = torch.full((count,), 0x5A5A, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, buf.data_ptr() + pad + mis, length, length, count, out, tcpck.KERNEL_RSTREAM,
                       LINE_FILL, mode=mode)
    torch.cuda.synchronize()
    return buf.cpu().numpy(), out.cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("length", [256, 258, 300, 510, 512, 1024, 1460, 1492, 2048, 3000, 4096, 9000])
@pytest.mark.parametrize("mis", [0, 2, 28, 36, 62, 98, 100, 126])
@pytest.mark.parametrize("mode", [0, 1])
def test_line_fill_vs_oracle(ctx, length, mis, mode):
    """Every arena alignment relative to the 128-B line (so each image's
    field line starts before, at or after the image start), guard bytes
    before and after the arena unchanged."""
    rng = np.random.default_rng(length * 1000 + mis * 2 + mode)
    pad = 256
    count = max(3, min(6000, (8 << 20) // length)) + (length % 7)
    a = rng.integers(0, 256, pad + mis + count * length + pad, dtype=np.uint8)
    got, out = run(ctx, a, mis, length, count, mode, pad)
    exp, want = expected_fill(a[pad:], mis, length, count, mode)
    np.testing.assert_array_equal(out, want)
    np.testing.assert_array_equal(got[:pad], a[:pad])
    np.testing.assert_array_equal(got[pad:], exp)


@pytest.mark.parametrize("count", [1, 2, 3, 63, 64, 65, 127, 129, 257, 2049])
@pytest.mark.parametrize("mis", [0, 100])
def test_line_fill_counts(ctx, count, mis):
    rng = np.random.default_rng(count * 3 + mis)
    length, pad = 1492, 256
    a = rng.integers(0, 256, pad + mis + count * length + pad, dtype=np.uint8)
    got, out = run(ctx, a, mis, length, count, 0, pad)
    exp, want = expected_fill(a[pad:], mis, length, count, 0)
    np.testing.assert_array_equal(out, want)
    np.testing.assert_array_equal(got[:pad], a[:pad])
    np.testing.assert_array_equal(got[pad:], exp)


@pytest.mark.parametrize("fill_byte", [0x00, 0xFF])
@pytest.mark.parametrize("mode", [0, 1])
def test_line_fill_constant_images(ctx, fill_byte, mode):
    """All-zero / all-0xFF images: sums at 0 and at the fold's edges."""
    length, pad, mis, count = 1492, 256, 36, 5000
    a = np.full(pad + mis + count * length + pad, fill_byte, np.uint8)
    got, out = run(ctx, a, mis, length, count, mode, pad)
    exp, want = expected_fill(a[pad:], mis, length, count, mode)
    np.testing.assert_array_equal(out, want)
    np.testing.assert_array_equal(got[pad:], exp)


def test_line_fill_then_verify(ctx):
    """FILL's line form, then VERIFY on the same arena: every image checks."""
    import tcpck
    rng = np.random.default_rng(77)
    length, count = 1492, 100000
    a = torch.from_numpy(rng.integers(0, 256, count * length + 64, dtype=np.uint8)).cuda()
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, a.data_ptr() + 2, length, length, count, out, tcpck.KERNEL_RSTREAM, LINE_FILL)
    ok = torch.zeros(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a.data_ptr() + 2, length, length, count, ok)
    torch.cuda.synchronize()
    assert int(ok.sum()) == count


def test_line_fill_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    out = torch.empty(4096, dtype=torch.int16, device="cuda")
    with pytest.raises(tcpck.TcpckError):  # a line may hold two fields below 256 B
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 254, 254, 64, out, tcpck.KERNEL_RSTREAM, LINE_FILL)
    with pytest.raises(tcpck.TcpckError):  # CHECKSUM has no fields
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 512, 512, 64, out, tcpck.KERNEL_RSTREAM, LINE_FILL)
    with pytest.raises(tcpck.TcpckError):  # the pass's input: a results buffer (explicit kernels)
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 512, 512, 64, None, tcpck.KERNEL_RSTREAM, LINE_FILL)
    assert not a.cpu().numpy().any()


def test_line_fill_c2_full(ctx, oracle_c):
    """C2 at full size (1M x 1492 B) through the line form, every result and
    every arena byte against the C oracle (16 threads)."""
    import tcpck
    length, count = 1492, 1 << 20
    a = torch.empty(count * length, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, length, length, count, seed=42)
    h = a.cpu().numpy().copy()
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, a, length, length, count, out, tcpck.KERNEL_RSTREAM, LINE_FILL)
    torch.cuda.synchronize()
    v = h.reshape(count, length)
    v[:, 28:30] = 0
    off = np.arange(count, dtype=np.uint64) * np.uint64(length)
    ln = np.full(count, length, np.uint32)
    want = oracle_c.batch(h, off, ln, threads=16).astype(np.uint16)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    v[:, 28:30] = want.view(np.uint8).reshape(count, 2)
    np.testing.assert_array_equal(a.cpu().numpy(), h)
