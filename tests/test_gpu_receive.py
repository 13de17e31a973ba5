"""GPU parity of the receive path's front half (ReceivePacket,
include/socket-manager.h:181-184): the batched verdict (TCPCK_OP_VERIFY) on the
network-order images, then tcpck_batch_header_swap (TcpHeaderN2H,
tcp-header.h:208-221) in place -- against the reference's own receive path on
known wire images (tests/golden/receive_golden.*, tests/golden/gen_receive.cc)
and against the oracle (oracle.ref16.receive_np / header_swap_np) on random
arenas: fixed strides and offset lists, 2-B-aligned images, damaged packets,
every arena byte (payloads and gaps untouched), and at C2's full size through
the involution (N2H twice = identity) plus sampled images."""
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


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("mis", [0, 2, 16, 30])
@pytest.mark.parametrize("hinted", [False, True])
def test_receive_golden(ctx, receive_golden, mis, hinted):
    """VERIFY + N2H on the reference's wire images == the reference's receive
    path: the 96 verdicts and every byte of the arena afterwards."""
    import tcpck
    g = receive_golden
    buf = torch.zeros(g.wire.size + 64, dtype=torch.uint8, device="cuda")
    buf[mis:mis + g.wire.size] = dev(g.wire)
    ptr = buf.data_ptr() + mis
    d_off, d_len = dev(g.offsets), dev(g.lengths)
    ok = torch.empty(len(g.offsets), dtype=torch.uint8, device="cuda")
    hints = dict(total_bytes=int(g.lengths.sum()), min_len=int(g.lengths.min()), max_len=int(g.lengths.max()),
                 sorted=True) if hinted else {}
    s = torch.cuda.Stream()
    ctx.batch_var(tcpck.OP_VERIFY, ptr, d_off, d_len, len(g.offsets), ok, stream=s, **hints)
    ctx.batch_header_swap(ptr, len(g.offsets), offsets=d_off, stream=s)
    s.synchronize()
    np.testing.assert_array_equal(host(ok), g.ok)
    got = host(buf)
    np.testing.assert_array_equal(got[mis:mis + g.wire.size], g.host)
    assert not got[:mis].any() and not got[mis + g.wire.size:].any()


def test_header_swap_golden_fields(ctx, receive_golden):
    """After the device N2H the accessors' host-order fields read right."""
    g = receive_golden
    buf = dev(g.wire)
    ctx.batch_header_swap(buf, len(g.offsets), offsets=dev(g.offsets))
    a = host(buf)
    o = g.offsets.astype(np.int64)
    seq = a[o[:, None] + np.arange(16, 20)[None, :]].copy().view("<u4").ravel()
    win = a[o[:, None] + np.arange(26, 28)[None, :]].copy().view("<u2").ravel()
    np.testing.assert_array_equal(seq, g.fields["seq"].astype(np.uint32))
    np.testing.assert_array_equal(win, g.fields["window"].astype(np.uint16))


@pytest.mark.parametrize("stride,count", [(32, 1), (32, 1000), (34, 777), (64, 4096), (96, 3),
                                          (1492, 5000), (1500, 4099), (2048, 2048), (9000, 300),
                                          (65536, 17), (36, 70001)])
@pytest.mark.parametrize("mis", [0, 2, 6])
def test_header_swap_fixed_vs_oracle(ctx, stride, count, mis):
    from oracle import ref16 as R
    rng = np.random.default_rng(stride * 7 + count + mis)
    a = rng.integers(0, 256, count * stride + 64, dtype=np.uint8)
    buf = dev(a)
    ctx.batch_header_swap(buf.data_ptr() + mis, count, stride=stride)
    exp = a.copy()
    R.header_swap_np(exp[mis:], np.arange(count, dtype=np.int64) * stride)
    np.testing.assert_array_equal(host(buf), exp)


@pytest.mark.parametrize("count", [1, 2, 63, 64, 65, 1000, 50000])
@pytest.mark.parametrize("kind", ["sorted", "unordered", "overlapping_pages"])
def test_header_swap_offsets_vs_oracle(ctx, count, kind):
    from oracle import ref16 as R
    rng = np.random.default_rng(count * 3 + len(kind))
    lens = (rng.integers(16, 800, count) * 2).astype(np.uint64)
    gaps = (rng.integers(0, 40, count) * 2).astype(np.uint64)
    off = np.zeros(count, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + gaps[:-1])
    if kind == "unordered":
        off = off[rng.permutation(count)]
    elif kind == "overlapping_pages":  # headers 32 B apart: neighbours share cache lines
        off = np.arange(count, dtype=np.uint64) * 32
        off = off[rng.permutation(count)]
    total = int(off.max()) + 2048
    a = rng.integers(0, 256, total, dtype=np.uint8)
    buf = dev(a)
    ctx.batch_header_swap(buf, count, offsets=dev(off))
    exp = a.copy()
    R.header_swap_np(exp, off.astype(np.int64))
    np.testing.assert_array_equal(host(buf), exp)


def test_receive_c2_full_size(ctx, oracle_c):
    """C2's layout (1M x 1492 B, 1.49 GB): FILL, damage 1 image in 1000,
    VERIFY, N2H.  Verdicts exact; N2H checked on 4096 sampled images against
    the oracle, then N2H again must restore the arena (every byte, via a
    checksum of checksums: the arena verifies exactly as before)."""
    import tcpck
    from oracle import ref16 as R
    n, L = 1 << 20, 1492
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, n, seed=11)
    cs = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, cs)
    bad = np.arange(500, n, 1000, dtype=np.int64)
    a[torch.from_numpy(bad * L + 40).cuda()] ^= 0x10
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, n, ok)
    exp_ok = np.ones(n, np.uint8)
    exp_ok[bad] = 0
    np.testing.assert_array_equal(host(ok), exp_ok)
    rng = np.random.default_rng(5)
    pick = np.sort(rng.choice(n, 4096, replace=False))
    idx = torch.from_numpy((pick[:, None] * L + np.arange(32)[None, :]).ravel()).cuda()
    before = host(a[idx]).reshape(-1, 32)
    ctx.batch_header_swap(a, n, stride=L)
    after = host(a[idx]).reshape(-1, 32)
    np.testing.assert_array_equal(after, before[:, R.HEADER_PERM])
    ctx.batch_header_swap(a, n, stride=L)  # H2N: back to network order
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, n, ok)
    np.testing.assert_array_equal(host(ok), exp_ok)
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, cs)
    got = host(cs).view(np.uint16)
    assert (got[exp_ok == 1] == 0).all() and (got[exp_ok == 0] != 0).all()


def test_header_swap_argument_errors(ctx):
    import tcpck
    a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_header_swap(a, 4, stride=63)                # odd stride
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_header_swap(a, 4, stride=30)                # shorter than the header
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_header_swap(a.data_ptr() + 1, 4, stride=64)  # odd arena
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_header_swap(0, 4, stride=64)                 # null arena
    ctx.batch_header_swap(a, 0, stride=64)                     # empty batch is a no-op
    ctx.batch_header_swap(a, 1, stride=0)                      # one image: stride unused
    torch.cuda.synchronize()
    assert not host(a).any()


# ---- TCPCK_OP_RECEIVE: verdicts + N2H in one call --------------------------------

def _fixed_case(rng, stride, length, count, mis=0, mode=0, damage_every=7):
    """Random images at mis + k * stride with valid checksums (as sent), every
    damage_every-th one damaged in its payload."""
    from oracle import ref16 as R
    a = rng.integers(0, 256, count * stride + 64, dtype=np.uint8)
    offs = np.arange(count, dtype=np.int64) * stride
    v = a[mis:]
    for o in offs:
        R.fill_np(v[o:o + length], mode)
    v[offs[::damage_every] + length // 2] ^= 0x5A
    return a, offs


@pytest.mark.parametrize("length", [32, 34, 96, 510, 512, 514, 1000, 1022, 1024, 1026, 1460, 1492, 1500, 2048,
                                    3000, 4094, 4096, 4098, 9000])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("mis", [0, 2, 62])
def test_receive_op_fixed_packed(ctx, length, mode, mis):
    """AUTO RECEIVE on packed fixed images (every verdict kernel the policy
    picks, then the header pass) == the oracle's receive path: the verdicts and
    every arena byte."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length * 4 + mode * 2 + mis)
    count = max(1, min(30000, (24 << 20) // length))
    a, offs = _fixed_case(rng, length, length, count, mis, mode)
    buf = dev(a)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_RECEIVE, buf.data_ptr() + mis, length, length, count, ok, mode=mode)
    exp = a.copy()
    exp_ok = R.receive_np(exp[mis:], offs, np.full(count, length), mode)
    np.testing.assert_array_equal(host(ok), exp_ok)
    assert 0 < exp_ok.sum() < count or count == 1  # intact and damaged images
    np.testing.assert_array_equal(host(buf), exp, err_msg=f"{length} mode {mode} mis {mis}")


@pytest.mark.parametrize("variant", [0, 10, 20, 21, 23, 24])
def test_receive_op_rstream_variants(ctx, variant):
    """Explicit rstream variants under RECEIVE: same verdicts and bytes."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(variant)
    L, count = 1492, 20000
    a, offs = _fixed_case(rng, L, L, count)
    buf = dev(a)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_RECEIVE, buf, L, L, count, ok, tcpck.KERNEL_RSTREAM, variant)
    exp = a.copy()
    exp_ok = R.receive_np(exp, offs, np.full(count, L))
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(buf), exp)


@pytest.mark.parametrize("stride,length", [(1536, 1492), (2048, 1492), (9216, 9000), (16384, 9000), (128, 96),
                                           (64, 32), (4096, 1500)])
def test_receive_op_fixed_slots(ctx, stride, length):
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(stride + length)
    count = max(1, min(20000, (24 << 20) // stride))
    a, offs = _fixed_case(rng, stride, length, count)
    buf = dev(a)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_RECEIVE, buf, stride, length, count, ok)
    exp = a.copy()
    exp_ok = R.receive_np(exp, offs, np.full(count, length))
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(buf), exp)


@pytest.mark.parametrize("hinted", [False, True])
@pytest.mark.parametrize("mode", [0, 1])
def test_receive_op_var_golden(ctx, receive_golden, hinted, mode):
    """RECEIVE through tcpck_batch_var on the reference's wire images (REF) and
    against the oracle (RFC 1071)."""
    import tcpck
    from oracle import ref16 as R
    g = receive_golden
    buf = dev(g.wire)
    ok = torch.empty(len(g.offsets), dtype=torch.uint8, device="cuda")
    hints = dict(total_bytes=int(g.lengths.sum()), min_len=int(g.lengths.min()), max_len=int(g.lengths.max()),
                 sorted=True) if hinted else {}
    ctx.batch_var(tcpck.OP_RECEIVE, buf, dev(g.offsets), dev(g.lengths), len(g.offsets), ok, mode=mode, **hints)
    exp = g.wire.copy()
    exp_ok = R.receive_np(exp, g.offsets, g.lengths, mode)
    if mode == 0:
        np.testing.assert_array_equal(exp_ok, g.ok)
        np.testing.assert_array_equal(exp, g.host)
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(buf), exp)


def test_receive_op_c2_full_size(ctx):
    """C2 (1M x 1492 B): RECEIVE twice restores the
    network order (the second pass's verdicts are on host-order headers, so
    they are not compared), then VERIFY gives the first verdicts again; 4096
    sampled headers checked against the permutation after the first pass."""
    import tcpck
    from oracle import ref16 as R
    n, L = 1 << 20, 1492
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, n, seed=3)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, None)
    bad = np.arange(123, n, 997, dtype=np.int64)
    a[torch.from_numpy(bad * L + 100).cuda()] ^= 0x01
    rng = np.random.default_rng(9)
    pick = np.sort(rng.choice(n, 4096, replace=False))
    idx = torch.from_numpy((pick[:, None] * L + np.arange(32)[None, :]).ravel()).cuda()
    before = host(a[idx]).reshape(-1, 32)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_RECEIVE, a, L, L, n, ok)
    exp_ok = np.ones(n, np.uint8)
    exp_ok[bad] = 0
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(a[idx]).reshape(-1, 32), before[:, R.HEADER_PERM])
    ctx.batch_fixed(tcpck.OP_RECEIVE, a, L, L, n, ok)
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, n, ok)
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(a[idx]).reshape(-1, 32), before)


def test_receive_op_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    ok = torch.empty(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed(tcpck.OP_RECEIVE, a, 30, 30, 4, ok)               # images < 32 B
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed(tcpck.OP_RECEIVE, a.data_ptr() + 1, 64, 64, 4, ok)  # odd arena
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed(tcpck.OP_RECEIVE, a, 64, 64, 4, None)             # no verdict buffer
    h, o = np.zeros(256, np.uint8), np.zeros(4, np.uint8)
    with pytest.raises(tcpck.TcpckError):
        ctx.host_batch_fixed(tcpck.OP_RECEIVE, h, 64, 64, 4, o)           # host batches: not taken


# ---- tcpck_batch_receive: headers into a dense array, arena untouched ----------------

def _expect_hdr(arena, offs):
    from oracle import ref16 as R
    o = np.asarray(offs, np.int64)
    return arena[o[:, None] + R.HEADER_PERM[None, :]].reshape(-1)


@pytest.mark.parametrize("length", [32, 96, 512, 1024, 1026, 1460, 1492, 4096, 9000])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("mis", [0, 2, 30])
def test_batch_receive_hdr_fixed(ctx, length, mode, mis):
    """Packed fixed images: verdicts, every header byte, the arena unchanged."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + 7 * mode + mis)
    count = max(1, min(30000, (24 << 20) // length))
    a, offs = _fixed_case(rng, length, length, count, mis, mode)
    buf = dev(a)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    hdr = torch.full((count * 32,), 0xEE, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(buf.data_ptr() + mis, count, ok, hdr, stride=length, length=length, mode=mode)
    exp_ok = (R.ref16_batch_np(a[mis:], offs, np.full(count, length), mode) == 0).astype(np.uint8)
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(hdr), _expect_hdr(a[mis:], offs))
    np.testing.assert_array_equal(host(buf), a)


@pytest.mark.parametrize("stride,length", [(2048, 1492), (1536, 1492), (16384, 9000), (64, 32)])
def test_batch_receive_hdr_slots(ctx, stride, length):
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(stride)
    count = max(1, min(20000, (24 << 20) // stride))
    a, offs = _fixed_case(rng, stride, length, count)
    buf = dev(a)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(count * 32, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(buf, count, ok, hdr, stride=stride, length=length)
    np.testing.assert_array_equal(host(ok), (R.ref16_batch_np(a, offs, np.full(count, length)) == 0).astype(np.uint8))
    np.testing.assert_array_equal(host(hdr), _expect_hdr(a, offs))
    np.testing.assert_array_equal(host(buf), a)


@pytest.mark.parametrize("hinted", [False, True])
def test_batch_receive_hdr_golden(ctx, receive_golden, hinted):
    """The reference's wire images through an offset list: the verdicts and
    the host-order headers equal the reference's after ReceivePacket's N2H."""
    g = receive_golden
    buf = dev(g.wire)
    n = len(g.offsets)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    hints = dict(total_bytes=int(g.lengths.sum()), min_len=int(g.lengths.min()), max_len=int(g.lengths.max()),
                 sorted=True) if hinted else {}
    ctx.batch_receive(buf, n, ok, hdr, offsets=dev(g.offsets), lengths=dev(g.lengths), **hints)
    np.testing.assert_array_equal(host(ok), g.ok)
    o = g.offsets.astype(np.int64)
    np.testing.assert_array_equal(host(hdr).reshape(n, 32), g.host[o[:, None] + np.arange(32)[None, :]])
    np.testing.assert_array_equal(host(buf), g.wire)


def test_batch_receive_hdr_c2_full_size(ctx):
    """C2 (1M x 1492 B): verdicts exact, 8192 sampled headers, the
    arena still verifies exactly as before (it is not written)."""
    import tcpck
    from oracle import ref16 as R
    n, L = 1 << 20, 1492
    a = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, n, seed=21)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, n, None)
    bad = np.arange(77, n, 1009, dtype=np.int64)
    a[torch.from_numpy(bad * L + 500).cuda()] ^= 0x80
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(a, n, ok, hdr, stride=L, length=L)
    exp_ok = np.ones(n, np.uint8)
    exp_ok[bad] = 0
    np.testing.assert_array_equal(host(ok), exp_ok)
    pick = np.sort(np.random.default_rng(2).choice(n, 8192, replace=False))
    idx = torch.from_numpy((pick[:, None] * L + np.arange(32)[None, :]).ravel()).cuda()
    raw = host(a[idx]).reshape(-1, 32)
    got = host(hdr).reshape(n, 32)[pick]
    np.testing.assert_array_equal(got, raw[:, R.HEADER_PERM])
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, n, ok)
    np.testing.assert_array_equal(host(ok), exp_ok)


def test_batch_receive_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    ok = torch.empty(64, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(64 * 32 + 8, dtype=torch.uint8, device="cuda")
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_receive(a, 4, ok, hdr.data_ptr() + 2, stride=64, length=64)  # header array not 4-B aligned
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_receive(a, 4, ok, hdr, stride=64, length=30)                 # images < 32 B
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_receive(a, 4, None, hdr, stride=64, length=64)               # no verdicts
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_receive(a, 4, ok, hdr, offsets=dev(np.zeros(4, np.uint64)))  # offsets without lengths
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_receive(a, 4, ok, hdr, stride=64, length=64, mode=7)
    ctx.batch_receive(a, 0, ok, hdr, stride=64, length=64)                     # empty: no-op


@pytest.mark.parametrize("slot", [64, 1536, 2048, 9216])
@pytest.mark.parametrize("mis", [0, 16, 2, 6])
@pytest.mark.parametrize("mode", [0, 1])
def test_batch_receive_hdr_ring(ctx, slot, mis, mode):
    """A datagram ring through an offset list with the SORTED hint (the
    compacted slot stream, then the header pass): 16-B aligned and unaligned
    starts, both modes."""
    from oracle import ref16 as R
    rng = np.random.default_rng(slot + mis + 100 * mode)
    n = max(1, min(40000, (32 << 20) // slot))
    ln = (rng.integers(16, slot // 2 + 1, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = rng.integers(0, 256, n * slot + 64, dtype=np.uint8)
    v = a[mis:]
    for o, l in zip(off[::3], ln[::3]):  # a third of them valid, as sent
        R.fill_np(v[int(o):int(o) + int(l)], mode)
    buf = dev(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(buf.data_ptr() + mis, n, ok, hdr, offsets=dev(off), lengths=dev(ln), mode=mode,
                      total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()), sorted=True)
    exp_ok = (R.ref16_batch_np(v, off, ln, mode) == 0).astype(np.uint8)
    assert exp_ok.sum() >= len(off[::3])
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(hdr), _expect_hdr(v, off.astype(np.int64)))
    np.testing.assert_array_equal(host(buf), a)


@pytest.mark.parametrize("variant", [0, 1, 2, 4, 8])
def test_batch_receive_sstream_variants(ctx, variant):
    """RECEIVE through tcpck_batch_var_ex(KERNEL_SSTREAM), every variant
    (U4 / U8, block orders): VERIFY + the header pass, same bytes."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(variant)
    n, slot = 30000, 2048
    ln = (rng.integers(16, 1024, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = rng.integers(0, 256, n * slot, dtype=np.uint8)
    buf = dev(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.batch_var_ex(tcpck.OP_RECEIVE, buf, dev(off), dev(ln), n, ok, tcpck.KERNEL_SSTREAM, variant,
                     total_bytes=int(ln.sum()), sorted=True)
    exp = a.copy()
    exp_ok = R.receive_np(exp, off.astype(np.int64), ln)
    np.testing.assert_array_equal(host(ok), exp_ok)
    np.testing.assert_array_equal(host(buf), exp)


# ---- RECEIVE with the headers written by sstream itself (one launch) -------------------

@pytest.mark.parametrize("variant", [0, 1, 2, 4, 8, 16, 17, 18, 32, 33, 34, 36, 40, 96, 98, 1 << 30])
@pytest.mark.parametrize("layout", ["ring", "ring-mis", "ring-short", "ring-64", "unordered", "fixed-slots",
                                    "fixed-mis", "fixed-64"])
@pytest.mark.parametrize("hdr_mis", [0, 4])
def test_batch_receive_fused_hdr(ctx, variant, layout, hdr_mis):
    """tcpck_batch_receive_ex on KERNEL_SSTREAM: each wave writes its run's
    host-order headers after its verdicts (variant + 16: the stream read with
    the default cache policy; + 32: each header from the stream's registers,
    + 64 with nt stores -- runs holding a misaligned or < 32-B image fall back
    to the per-run conversion; 1 << 30: the separate header pass instead).
    Rings (16-B and 2-B aligned starts), unordered offsets (the per-image
    fallback), fixed slots; 64-256-B rings and 64-B fixed images (+ 32: every
    run's records staged in LDS, up to 17 images per step); header arrays 16-B
    and only 4-B aligned; both modes.  Verdicts, every header byte, the arena
    unchanged."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(variant % 97 + 10 * len(layout) + hdr_mis)
    mode = int(rng.random() < 0.5)
    n, slot = 20000, 2048
    mis = 6 if layout.endswith("mis") else 0
    ln = (rng.integers(16, 1000, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    if layout == "unordered":
        off = off[rng.permutation(n)].copy()
    if layout.startswith("fixed"):
        ln[:] = 64 if layout == "fixed-64" else 1492
    if layout == "ring-64":  # every image >= 64 B, up to 17 per compacted step
        ln = (rng.integers(32, 129, n) * 2).astype(np.uint32)
    if layout == "ring-short":  # some runs hold images below 32 B (headers past the image end)
        ln[rng.integers(0, n, 40)] = (rng.integers(1, 16, 40) * 2).astype(np.uint32)
    a = rng.integers(0, 256, n * slot + 64, dtype=np.uint8)
    v = a[mis:]
    for o, l in zip(off[::3], ln[::3]):
        if l >= 30:
            R.fill_np(v[int(o):int(o) + int(l)], mode)
    buf = dev(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hbuf = torch.full((n * 32 + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    hdr = hbuf.data_ptr() + hdr_mis
    if layout.startswith("fixed"):
        ctx.batch_receive(buf.data_ptr() + mis, n, ok, hdr, stride=slot, length=int(ln[0]), mode=mode,
                          kernel=tcpck.KERNEL_SSTREAM, param=variant)
    else:
        ctx.batch_receive(buf.data_ptr() + mis, n, ok, hdr, offsets=dev(off), lengths=dev(ln), mode=mode,
                          total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                          sorted=layout != "unordered", kernel=tcpck.KERNEL_SSTREAM, param=variant)
    exp_ok = (R.ref16_batch_np(v, off, ln, mode) == 0).astype(np.uint8)
    np.testing.assert_array_equal(host(ok), exp_ok)
    h = host(hbuf)
    np.testing.assert_array_equal(h[hdr_mis:hdr_mis + 32 * n], _expect_hdr(v, off.astype(np.int64)))
    assert (h[:hdr_mis] == 0xEE).all() and (h[hdr_mis + 32 * n:] == 0xEE).all()
    np.testing.assert_array_equal(host(buf), a)


def test_batch_receive_fused_rejects_other_ops(ctx):
    """The fused header write exists for RECEIVE only: a plain VERIFY through
    sstream never touches a header array (there is none to pass), and a
    CHECKSUM/FILL never reaches it."""
    import tcpck
    rng = np.random.default_rng(5)
    n, slot = 1000, 2048
    a = rng.integers(0, 256, n * slot, dtype=np.uint8)
    buf = dev(a)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf, slot, 1492, n, out, tcpck.KERNEL_SSTREAM, 16)
    from oracle import ref16 as R
    np.testing.assert_array_equal(host(out).view(np.uint16),
                                  R.ref16_batch_np(a, np.arange(n) * slot, np.full(n, 1492)))
