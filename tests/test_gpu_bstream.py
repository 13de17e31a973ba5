"""Experimental byte-run stream (TCPCK_KERNEL_BSTREAM, tcpck_bstream.hip):
runs that ignore image edges, cut images combined by per-part atomics in a
zeroed u64 workspace.  CHECKSUM and VERIFY against the oracle
(tcp-header.h:252-263) over image sizes below, at and above the run size,
misaligned arenas, several run sizes and loads in flight; the workspace must
be all zero again after every launch, and a second launch must agree."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available()
    c = tcpck.Context(0)
    yield c
    c.set_debug(None)
    c.close()


@pytest.mark.parametrize("length", [2, 30, 1492, 4096, 4098, 6000, 8192, 9000, 12290, 16384, 65534, 65536, 200000])
@pytest.mark.parametrize("mis", [0, 2, 126])
@pytest.mark.parametrize("variant", [0, 10, 12, 16, 256, 256 | 14])
def test_bstream_vs_oracle(ctx, oracle_c, length, mis, variant):
    import tcpck
    rng = np.random.default_rng(length + mis + variant)
    count = int(max(1, min(3000, (24 << 20) // length)))
    a = rng.integers(0, 256, count * length + 256, dtype=np.uint8)
    buf = torch.from_numpy(a).cuda()
    ws = torch.zeros(count, dtype=torch.int64, device="cuda")
    ctx.set_debug(ws)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ptr = buf.data_ptr() + mis
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, ptr, length, length, count, out, tcpck.KERNEL_BSTREAM, variant)
    torch.cuda.synchronize()
    exp = oracle_c.batch(a[mis:], stride=length, length=length, count=count)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp)
    assert not ws.any().item(), "workspace not left zero"
    # valid images verify, the rest do not
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, ptr, length, length, count, ok, tcpck.KERNEL_BSTREAM, variant)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ok.cpu().numpy(), (exp == 0).astype(np.uint8))
    assert not ws.any().item()
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, ptr, length, length, count, out, tcpck.KERNEL_BSTREAM, variant)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp)
    ctx.set_debug(None)


def test_bstream_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    out = torch.empty(64, dtype=torch.int16, device="cuda")
    ctx.set_debug(None)
    with pytest.raises(tcpck.TcpckError):  # no workspace
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 8192, 8192, 64, out, tcpck.KERNEL_BSTREAM, 0)
    ws = torch.zeros(64, dtype=torch.int64, device="cuda")
    ctx.set_debug(ws)
    with pytest.raises(tcpck.TcpckError):  # FILL is not a bstream op
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 8192, 8192, 64, out, tcpck.KERNEL_BSTREAM, 0)
    with pytest.raises(tcpck.TcpckError):  # RFC 1071
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 8192, 8192, 64, out, tcpck.KERNEL_BSTREAM, 0, mode=1)
    with pytest.raises(tcpck.TcpckError):  # gapped
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 8192, 8000, 64, out, tcpck.KERNEL_BSTREAM, 0)
    ctx.set_debug(None)
