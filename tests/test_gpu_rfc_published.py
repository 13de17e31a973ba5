"""GPU parity of the opt-in RFC 1071 mode against a PUBLISHED answer
(VERDICT r05 item 3): RFC 1071 section 3's worked example, bytes
00 01 f2 03 f4 f5 f6 f7 -> folded sum 0xddf2 (big-endian words), checksum
0x0d22 in this library's little-endian raw convention (stored bytes 22 0d =
0x220d read big-endian; tests/test_oracle.py pins the restatements to it).

The example is embedded at the start of images whose other bytes are zero
(zero words leave a one's complement sum unchanged), so every image of every
layout below has that checksum, through each kernel AUTO picks in RFC 1071
mode: vvstream (8-B and 32-B packed images), rstream (1492-B packed), sstream
(1492-B images in 2048-B slots), seg (an unordered offset list), and FILL on
32-B headers (the field at bytes 28-29 zeroed, then 22 0d stored).  Contrast
the reference arithmetic (include/tcp-header.h:253-262, no fold): 0x0d23.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

EXAMPLE = np.frombuffer(bytes.fromhex("0001f203f4f5f6f7"), np.uint8)
RFC = 0x0D22
REF = 0x0D23


@pytest.fixture(scope="module")
def c(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    ctx = tcpck.Context(0)
    yield ctx
    ctx.close()


def arena_of(count, stride, length):
    a = np.zeros(count * stride, np.uint8)
    for k in range(count):
        a[k * stride:k * stride + 8] = EXAMPLE
    return torch.from_numpy(a).cuda()


def results(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("stride,length", [(8, 8), (32, 32), (1492, 1492), (2048, 1492), (96, 96)])
@pytest.mark.parametrize("mode", [0, 1], ids=["ref", "rfc1071"])
def test_fixed_layouts(c, stride, length, mode):
    import tcpck
    count = 20000
    a = arena_of(count, stride, length)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    c.batch_fixed(tcpck.OP_CHECKSUM, a, stride, length, count, out, mode=mode)
    assert (results(out) == (RFC if mode else REF)).all()


def test_unordered_offset_list(c):
    """seg (offsets neither packed nor sorted) in RFC 1071 mode."""
    import tcpck
    count, slot = 5000, 256
    a = arena_of(count, slot, 200)
    perm = np.random.default_rng(5).permutation(count).astype(np.uint64) * np.uint64(slot)
    off = torch.from_numpy(perm).cuda()
    ln = torch.full((count,), 200, dtype=torch.int32, device="cuda")
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    c.batch_var(tcpck.OP_CHECKSUM, a, off, ln, count, out, mode=tcpck.MODE_RFC1071, total_bytes=200 * count,
                min_len=200, max_len=200)
    assert (results(out) == RFC).all()


@pytest.mark.parametrize("with_out", [True, False], ids=["out", "noout"])
def test_fill_32b_headers(c, with_out):
    """FILL in RFC 1071 mode on 32-B headers carrying the example (a stale
    field is zeroed first): bytes 28-29 become 22 0d, VERIFY then passes."""
    import tcpck
    count = 50000
    host = np.zeros(count * 32, np.uint8)
    for k in range(count):
        host[k * 32:k * 32 + 8] = EXAMPLE
        host[k * 32 + 28:k * 32 + 30] = (0xAB, 0xCD)  # stale field
    a = torch.from_numpy(host).cuda()
    out = torch.empty(count, dtype=torch.int16, device="cuda") if with_out else None
    c.batch_fixed(tcpck.OP_FILL, a, 32, 32, count, out, mode=tcpck.MODE_RFC1071)
    got = a.cpu().numpy().reshape(count, 32)
    assert (got[:, 28] == 0x22).all() and (got[:, 29] == 0x0D).all()
    assert (got[:, :8] == EXAMPLE).all()
    if with_out:
        assert (results(out) == RFC).all()
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    c.batch_fixed(tcpck.OP_VERIFY, a, 32, 32, count, ok, mode=tcpck.MODE_RFC1071)
    torch.cuda.synchronize()
    assert bool((ok == 1).all().item())
