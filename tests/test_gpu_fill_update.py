"""FILL as a CHECKSUM pass + a field-update pass (TCPCK_PARAM_FILL_UPDATE,
AUTO's choice in reference mode with a results buffer for jumbo images in
slots): the zero-field
checksum is derived from the stored one and the old field, c = ~(~C - f) mod
2^16, and written as the field's 64-B block (or a 2-B store where the block
could touch another field or leave the batch).  Every arena byte and result
against the oracle's FILL (socket-manager.cc:9-10: zero bytes 28-29, then
CalculateChecksum, tcp-header.h:252-263), through every CHECKSUM kernel the
pass can follow, on fixed, packed and gapped layouts."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

UPD = 1 << 28
INS = 1 << 29


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available()
    from conftest import RoutedContext
    c = RoutedContext(0)  # libtcpck.so; measurement-only variants on libtcpck_probe.so
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def expect_fill(arena, offs, lens):
    from oracle import ref16 as R
    exp = arena.copy()
    want = np.array([R.fill_np(exp[int(o):int(o) + int(n)]) if n >= 30 else 0 for o, n in zip(offs, lens)], np.uint16)
    return exp, want


def run_fixed(ctx, a, mis, stride, length, count, kernel, param):
    import tcpck
    buf = dev(a)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, buf.data_ptr() + mis, stride, length, count, out, kernel, param)
    torch.cuda.synchronize()
    return buf.cpu().numpy(), out.cpu().numpy().view(np.uint16)


# (kernel, param) pairs the update pass follows; None = applies to every layout
KERNELS = {
    "auto": (0, 0),
    "auto+flag": (0, UPD),
    "rstream": (5, 20 | UPD),
    "vvstream": (8, 28 | UPD),
    "seg": (1, UPD),
    "sstream": (10, UPD),
}


@pytest.mark.parametrize("length", [64, 66, 96, 126, 512, 1024, 1492, 4094, 4096, 9000, 65536])
@pytest.mark.parametrize("mis", [0, 2, 30, 62])
@pytest.mark.parametrize("kname", ["auto", "rstream", "vvstream", "seg"])
def test_update_fixed_packed(ctx, length, mis, kname):
    rng = np.random.default_rng(length * 31 + mis)
    kernel, param = KERNELS[kname]
    if kname == "rstream" and length < 512:
        kernel, param = 0, UPD
    count = max(1, min(20000, (12 << 20) // length))
    a = rng.integers(0, 256, count * length + 128, dtype=np.uint8)
    got, res = run_fixed(ctx, a, mis, length, length, count, kernel, param)
    exp, want = expect_fill(a[mis:], np.arange(count) * length, np.full(count, length))
    np.testing.assert_array_equal(res, want)
    np.testing.assert_array_equal(got[mis:], exp)
    np.testing.assert_array_equal(got[:mis], a[:mis])


@pytest.mark.parametrize("length,stride", [(64, 80), (96, 256), (1492, 2048), (1492, 1504), (9000, 9216),
                                           (9000, 16384), (30, 64), (62, 64), (200, 4096)])
@pytest.mark.parametrize("kname", ["auto", "vvstream", "seg", "sstream"])
def test_update_fixed_slots(ctx, length, stride, kname):
    rng = np.random.default_rng(length + stride)
    kernel, param = KERNELS[kname]
    if kname == "sstream" and stride % 16:
        kernel, param = 0, UPD
    count = max(1, min(20000, (12 << 20) // stride))
    a = rng.integers(0, 256, count * stride + 64, dtype=np.uint8)
    got, res = run_fixed(ctx, a, 2, stride, length, count, kernel, param)
    exp, want = expect_fill(a[2:], np.arange(count) * stride, np.full(count, length))
    np.testing.assert_array_equal(res, want)
    np.testing.assert_array_equal(got[2:], exp)
    np.testing.assert_array_equal(got[:2], a[:2])


@pytest.mark.parametrize("fields", ["random", "ones", "zero", "valid"])
def test_update_field_values(ctx, fields):
    """The old field is what the update subtracts: random, all-ones, zero and
    already-valid fields (a FILL twice) give the same arena as the in-stream
    FILL, and the wrap cases (~C - f below 0) are exact mod 2^16."""
    import tcpck
    rng = np.random.default_rng(7)
    L, n = 1492, 4096
    a = rng.integers(0, 256, n * L, dtype=np.uint8)
    v = a.reshape(n, L)
    if fields == "ones":
        v[:, 28:30] = 0xFF
    elif fields == "zero":
        v[:, 28:30] = 0
    if fields == "valid":
        exp, _ = expect_fill(a, np.arange(n) * L, np.full(n, L))
        a = exp
    got, res = run_fixed(ctx, a, 0, L, L, n, 0, UPD)
    exp, want = expect_fill(a, np.arange(n) * L, np.full(n, L))
    np.testing.assert_array_equal(res, want)
    np.testing.assert_array_equal(got, exp)
    got2, res2 = run_fixed(ctx, a, 0, L, L, n, 0, INS)
    np.testing.assert_array_equal(got2, got)
    np.testing.assert_array_equal(res2, res)


@pytest.mark.parametrize("dist", ["c3", "short", "mixed", "jumbo"])
@pytest.mark.parametrize("layout", ["packed", "packed-nohint", "sorted", "unordered"])
@pytest.mark.parametrize("mis", [0, 2, 40])
def test_update_var(ctx, dist, layout, mis):
    """Offset lists: the block write only for PACKED batches where the fields
    are >= 64 B apart and the block stays inside images k-1..k (lengths[k] >=
    96, lengths[k-1] >= 64), else 2-B accesses; images < 30 B keep their plain
    checksum and are not written."""
    import tcpck
    rng = np.random.default_rng(zlib.crc32(f"{dist}/{layout}/{mis}".encode()))
    n = 3000 if dist != "jumbo" else 200
    if dist == "c3":
        ln = np.asarray((96, 608, 1492), np.uint32)[rng.integers(0, 3, n)]
    elif dist == "short":
        ln = (rng.integers(0, 70, n) * 2).astype(np.uint32)  # 0..138 B: every block/2-B rule boundary
    elif dist == "mixed":
        ln = np.asarray((28, 30, 32, 62, 64, 66, 94, 96, 98, 1460), np.uint32)[rng.integers(0, 10, n)]
    else:
        ln = (rng.integers(2000, 33000, n) * 2).astype(np.uint32)
    l64 = ln.astype(np.uint64)
    if layout.startswith("packed"):
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(l64[:-1])
    else:
        gaps = (rng.integers(0, 40, n) * 2).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(l64[:-1] + gaps[:-1])
        if layout == "unordered":
            p = rng.permutation(n)
            off, ln = off[p].copy(), ln[p].copy()
    total = int((off + ln.astype(np.uint64)).max()) + 128
    a = rng.integers(0, 256, total + mis, dtype=np.uint8)
    buf = dev(a)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    hints = dict(total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                 packed=layout == "packed", sorted=layout == "sorted")
    ctx.batch_var_ex(tcpck.OP_FILL, buf.data_ptr() + mis, dev(off), dev(ln), n, out, 0, UPD, **hints)
    torch.cuda.synchronize()
    exp, want = expect_fill(a[mis:], off, ln)
    from oracle import ref16 as R
    short = ln < 30
    if short.any():  # no field: the plain checksum (seg's FILL does the same)
        plain = np.array([R.ref16_np(a[mis:][int(o):int(o) + int(m)]) for o, m in zip(off[short], ln[short])],
                         np.uint16)
        want[short] = plain
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    np.testing.assert_array_equal(buf.cpu().numpy()[mis:], exp)
    np.testing.assert_array_equal(buf.cpu().numpy()[:mis], a[:mis])


def test_update_not_taken(ctx):
    """No results buffer, or RFC 1071 mode: the in-stream FILL (the update
    identity is exact only mod 2^16); results match the oracle either way."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(3)
    L, n = 1492, 2048
    a = rng.integers(0, 256, n * L, dtype=np.uint8)
    buf = dev(a)
    ctx.batch_fixed(tcpck.OP_FILL, buf, L, L, n, None)
    exp, _ = expect_fill(a, np.arange(n) * L, np.full(n, L))
    np.testing.assert_array_equal(buf.cpu().numpy(), exp)
    buf = dev(a)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_FILL, buf, L, L, n, out, mode=1)
    exp = a.copy()
    want = np.array([R.fill_np(exp[k * L:(k + 1) * L], 1) for k in range(n)], np.uint16)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    np.testing.assert_array_equal(buf.cpu().numpy(), exp)
