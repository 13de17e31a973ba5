"""GPU parity at the largest image sizes the C ABI takes (SURVEY §8c edge
cases: maximum sizes).  The reference checksums any `size_` its TcpPacket
holds (include/tcp-header.h:252-263, a uint32_t accumulator truncated to
16 bits, so the REF sum is mod 2^16 at any length); the C ABI's image length
is a uint32_t.  Images of 1 MiB to 3 GiB, fixed strides and packed offset
lists, every op, both modes, through AUTO (seg's W-wave jumbo shapes), against
the oracle (oracle/ref16.c, pinned by tests/golden)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def c(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    ctx = tcpck.Context(0)
    yield ctx
    ctx.close()


def results(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16) if t.dtype == torch.int16 else t.cpu().numpy()


@pytest.mark.parametrize("L,count", [((1 << 20) + 2, 5), (16 << 20, 3), ((256 << 20) + 6, 1)])
@pytest.mark.parametrize("mode", [0, 1], ids=["ref", "rfc1071"])
def test_fixed_large(c, oracle_c, L, count, mode):
    import tcpck
    a = torch.empty(L * count, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, count, seed=L % 1000 + mode)
    host = a.cpu().numpy()
    want = oracle_c.batch(host, stride=L, length=L, count=count, mode=mode)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    c.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out, mode=mode)
    np.testing.assert_array_equal(results(out), want)
    c.batch_fixed(tcpck.OP_FILL, a, L, L, count, out, mode=mode)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    c.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok, mode=mode)
    assert (results(ok) == 1).all()
    filled = a.cpu().numpy()
    for k in range(count):  # only bytes 28-29 of each image changed
        h = host[k * L:(k + 1) * L].copy()
        h[28:30] = 0
        fw = int(oracle_c.one(h, mode))
        assert filled[k * L + 28] == (fw & 0xFF) and filled[k * L + 29] == fw >> 8
        assert np.array_equal(np.delete(filled[k * L:(k + 1) * L], [28, 29]), np.delete(h, [28, 29]))


@pytest.mark.parametrize("mode", [0, 1], ids=["ref", "rfc1071"])
def test_packed_list_with_huge_images(c, oracle_c, mode):
    import tcpck
    ln = np.asarray([2, 70000, 1 << 20, 32, 5 << 20, 96, (9 << 20) + 4, 1492], np.uint32)
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    total = int(ln.astype(np.int64).sum())
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    tcpck.synth_var(a, d_off, d_ln, int(ln.max()), ln.size, seed=7 + mode)
    want = oracle_c.batch(a.cpu().numpy(), off, ln, mode=mode)
    out = torch.empty(ln.size, dtype=torch.int16, device="cuda")
    c.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, ln.size, out, mode=mode, total_bytes=total, min_len=2,
                max_len=int(ln.max()), packed=True)
    np.testing.assert_array_equal(results(out), want)


def test_one_3gib_image(c, oracle_c):
    """One image of 3 GiB + 2 B (the C ABI's uint32_t length; above 2^31):
    CHECKSUM in both modes and VERIFY after FILL."""
    import tcpck
    L = (3 << 30) + 2
    a = torch.empty(L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, 1, seed=33)
    host = a.cpu().numpy()
    out = torch.empty(1, dtype=torch.int16, device="cuda")
    for mode in (0, 1):
        c.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, 1, out, mode=mode)
        assert int(results(out)[0]) == int(oracle_c.one(host, mode)), mode
    del host
    c.batch_fixed(tcpck.OP_FILL, a, L, L, 1, None)
    ok = torch.empty(1, dtype=torch.uint8, device="cuda")
    c.batch_fixed(tcpck.OP_VERIFY, a, L, L, 1, ok)
    assert int(results(ok)[0]) == 1
