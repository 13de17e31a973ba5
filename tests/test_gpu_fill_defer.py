"""FILL with the field stores deferred to a second pass (rstream variant 25:
the stream writes only the results, then one write-through 2-B store per
field): every arena byte and result against the oracle's FILL
(socket-manager.cc:9-10), including the images at the batch's edges; and the
probe build's other forms of that pass (64-B blocks, 16-B chunks, 128-B lines,
each store policy) write the same bytes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available()
    from conftest import RoutedContext
    c = RoutedContext(0)  # libtcpck.so; measurement-only variants on libtcpck_probe.so
    yield c
    c.close()


@pytest.mark.parametrize("length", [64, 66, 100, 512, 514, 1024, 1460, 1492, 2048, 4094, 4096, 6000, 9000, 16384])
@pytest.mark.parametrize("mis", [0, 2, 30, 36, 62])
@pytest.mark.parametrize("mode", [0, 1])
def test_fill_defer_vs_oracle(ctx, oracle_c, length, mis, mode):
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length * 8 + mis + mode)
    count = max(1, min(20000, (16 << 20) // length))
    a = rng.integers(0, 256, count * length + 128, dtype=np.uint8)
    buf = torch.from_numpy(a).cuda()
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, buf.data_ptr() + mis, length, length, count, out, tcpck.KERNEL_RSTREAM, 25,
                       mode=mode)
    torch.cuda.synchronize()
    exp = a.copy()
    v = exp[mis:]
    want = np.array([R.fill_np(v[k * length:(k + 1) * length], mode) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    np.testing.assert_array_equal(buf.cpu().numpy(), exp)


def test_fill_defer_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = torch.empty(1024, dtype=torch.int16, device="cuda")
    with pytest.raises(tcpck.TcpckError):  # results are the pass's input: out required
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 512, 512, 64, None, tcpck.KERNEL_RSTREAM, 25)
    with pytest.raises(tcpck.TcpckError):  # CHECKSUM has no fields to defer
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 512, 512, 64, out, tcpck.KERNEL_RSTREAM, 25)



@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_odd_arena_rejected(ctx, op):
    """An odd arena address puts every u16 word of the images at an odd
    address; the kernels pair bytes by address, so the C ABI rejects it
    (TCPCK_EINVAL) for every op and layout rather than compute other words."""
    import tcpck
    a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = torch.empty(1024, dtype=torch.int16, device="cuda")
    off = torch.arange(16, dtype=torch.int64, device="cuda") * 1024
    ln = torch.full((16,), 512, dtype=torch.int32, device="cuda")
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed(op, a.data_ptr() + 1, 512, 512, 64, out)
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_var(op, a.data_ptr() + 1, off, ln, 16, out)
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_set_ack(a.data_ptr() + 1, 16, stride=512)
    assert not a.cpu().numpy().any()


@pytest.mark.parametrize("length", [512, 1492, 4096, 9000])
@pytest.mark.parametrize("with_out", [True, False])
def test_fill_auto_rstream(ctx, length, with_out):
    """AUTO FILL on packed fixed images: with a results buffer the policy
    defers the fields to the field pass, without one it stores them in the
    stream -- same arena either way."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + with_out)
    count = max(1, (8 << 20) // length)
    a = rng.integers(0, 256, count * length, dtype=np.uint8)
    buf = torch.from_numpy(a).cuda()
    out = torch.empty(count, dtype=torch.int16, device="cuda") if with_out else None
    ctx.batch_fixed(tcpck.OP_FILL, buf, length, length, count, out)
    torch.cuda.synchronize()
    exp = a.copy()
    want = np.array([R.fill_np(exp[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
    if with_out:
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    np.testing.assert_array_equal(buf.cpu().numpy(), exp)


@pytest.mark.parametrize("form", [0x00, 0x08, 0x07, 0x18, 0x10, 0x28, 0x27, 0x20, 0x38, 0x30, 0xC8, 0xC0])
def test_field_pass_forms(ctx, form):
    """TCPCK_KERNEL_PATCH (libtcpck_probe.so): the field pass alone, every
    granularity (form >> 4: 64-B block, 16-B chunk, 2-B field, 128-B line, 12:
    32-B block) and
    store policy (form & 15: 1 + cache bits, 0 plain) stores out[k] into bytes
    28-29 of image k and leaves every other byte as it was."""
    import tcpck
    rng = np.random.default_rng(form)
    L, count, mis = 1492, 3000, 6
    a = rng.integers(0, 256, count * L + 256, dtype=np.uint8)
    sums = rng.integers(0, 1 << 16, count, dtype=np.uint16)
    buf = torch.from_numpy(a).cuda()
    out = torch.from_numpy(sums.view(np.int16)).cuda()
    ctx.probe.batch_fixed_ex(tcpck.OP_FILL, buf.data_ptr() + mis, L, L, count, out, tcpck.KERNEL_PATCH, form)
    torch.cuda.synchronize()
    exp = a.copy()
    for k in range(count):
        exp[mis + k * L + 28:mis + k * L + 30] = sums[k:k + 1].view(np.uint8)
    np.testing.assert_array_equal(buf.cpu().numpy(), exp)


@pytest.mark.parametrize("length", [128, 130, 190, 512, 514, 1024, 1460, 1492, 2048, 4094, 9000, 16384])
@pytest.mark.parametrize("mis", [0, 2, 36, 126])
@pytest.mark.parametrize("count", [1, 17, 20000])
@pytest.mark.parametrize("with_out", [True, False])
@pytest.mark.parametrize("variant", [27, 28])
def test_fill_block_vs_oracle(ctx, length, mis, count, with_out, variant):
    """rstream variants 27 / 28 (libtcpck_probe.so): each field's whole 64-B
    block written from the stream's registers with the checksum in place (28:
    a short run's blocks after its last load).  Every
    arena byte (the blocks also hold the previous image's tail), the bytes
    before and after the batch, and the results against the oracle's FILL
    (socket-manager.cc:9-10); misalignments put image 0's block before the
    arena (the field stored alone)."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length * 8 + mis + count + with_out + variant)
    count = max(1, min(count, (8 << 20) // length))
    a = rng.integers(0, 256, count * length + 256, dtype=np.uint8)
    buf = torch.from_numpy(a).cuda()
    out = torch.empty(count, dtype=torch.int16, device="cuda") if with_out else None
    ctx.batch_fixed_ex(tcpck.OP_FILL, buf.data_ptr() + mis, length, length, count, out, tcpck.KERNEL_RSTREAM,
                       variant)
    torch.cuda.synchronize()
    exp = a.copy()
    v = exp[mis:]
    want = np.array([R.fill_np(v[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
    if with_out:
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    np.testing.assert_array_equal(buf.cpu().numpy(), exp)


def test_fill_block_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = torch.empty(1024, dtype=torch.int16, device="cuda")
    with pytest.raises(tcpck.TcpckError):  # fields < 128 B apart: blocks would overlap a neighbour's
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 96, 96, 64, out, tcpck.KERNEL_RSTREAM, 27)
