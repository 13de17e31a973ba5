"""GPU parity of the compacted slot stream (KERNEL_SSTREAM, tcpck_sstream.hip)
against the oracle (oracle/ref16.c, pinned to the reference's golden vectors):
variable-length images in fixed receive slots (the batched recvfrom buffer of
src/network-service.cc:39,49-56), fixed slots with gaps, any offset order,
overlapping and chunk-sharing images, empty and 2-B images, misaligned arena
pointers, runs of exactly 256 images; CHECKSUM, FILL (arena byte-exact, gap
bytes untouched) and VERIFY with corruptions."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

VARIANTS = [0, 1, 2, 5, 10]  # 0 policy, 1 U4, 2 U8; +4 default block order, +8 scattered


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


def fill_oracle(arena_np, off, ln):
    """The reference's send path per image, in index order (socket-manager.cc:9-10)."""
    from oracle import ref16 as R
    a = arena_np.copy()
    exp = np.empty(len(off), np.uint16)
    for k in range(len(off)):
        o, n = int(off[k]), int(ln[k])
        exp[k] = R.fill_np(a[o:o + n])
    return exp, a


def slot_layout(count, slot, lengths, seed, lead=0):
    """count slots of `slot` bytes; image k at k * slot + lead, length drawn from `lengths`."""
    rng = np.random.default_rng(seed)
    ln = np.asarray(lengths, np.uint32)[rng.integers(0, len(lengths), count)]
    off = np.arange(count, dtype=np.uint64) * np.uint64(slot) + np.uint64(lead)
    return off, ln, int(count * slot + lead)


SLOTS = [
    (64, (2, 30, 32, 48, 64)),
    (1536, (96, 608, 1492)),
    (2048, (32, 96, 608, 1492)),
    (2048, (1492,)),
    (2050, (34, 606, 1494)),        # 2-mod-4 starts and lengths: u16 prefix table
    (1600, (64, 200, 576, 1024, 1492)),
    (9216, (40, 9000)),
    (65600, (65536, 1500)),
]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("slot,lengths", SLOTS)
@pytest.mark.parametrize("count", [1, 2, 63, 64, 65, 255, 256, 257, 3001, 40000])
def test_sstream_var_slots(ctx, oracle_c, variant, slot, lengths, count):
    import tcpck
    if count * slot > (160 << 20):
        count = (160 << 20) // slot
    off, ln, total = slot_layout(count, slot, lengths, seed=count + slot + variant)
    rng = np.random.default_rng(count * 7 + slot)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    buf = dev(arena_np)
    d_off, d_ln = dev(off), dev(ln)
    exp0 = None
    for mis in (0, 2, 14):
        for oversub in (0, 1, 8):
            out = torch.empty(count, dtype=torch.int16, device="cuda")
            ctx.batch_var_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, d_off, d_ln, count, out,
                             tcpck.KERNEL_SSTREAM, variant | (oversub << 16), total_bytes=int(ln.sum()))
            exp = oracle_c.batch(arena_np[mis:], off, ln, threads=8)
            np.testing.assert_array_equal(host(out).view(np.uint16), exp)
            if mis == 0:
                exp0 = exp
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var_ex(tcpck.OP_VERIFY, buf, d_off, d_ln, count, ok, tcpck.KERNEL_SSTREAM, variant)
    np.testing.assert_array_equal(host(ok), (exp0 == 0).astype(np.uint8))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("slot,lengths", [s for s in SLOTS if min(s[1]) >= 30])
@pytest.mark.parametrize("count", [1, 65, 257, 5000])
def test_sstream_var_fill_verify(ctx, variant, slot, lengths, count):
    """Send path in slots: the field is zeroed in the stream, the result lands in
    out[k] and in bytes 28-29; every other byte (gaps included) is untouched;
    then every image verifies and corrupted images are found exactly."""
    import tcpck
    if count * slot > (160 << 20):
        count = (160 << 20) // slot
    off, ln, total = slot_layout(count, slot, lengths, seed=count * 3 + slot)
    rng = np.random.default_rng(count + slot + variant)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    for mis in (0, 2, 94):
        buf = dev(arena_np)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(tcpck.OP_FILL, buf.data_ptr() + mis, dev(off), dev(ln), count, out,
                         tcpck.KERNEL_SSTREAM, variant, total_bytes=int(ln.sum()))
        exp, exp_arena = fill_oracle(arena_np[mis:], off, ln)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
        got = host(buf)
        np.testing.assert_array_equal(got[mis:], exp_arena)
        np.testing.assert_array_equal(got[:mis], arena_np[:mis])
    # out == NULL: the arena alone
    buf = dev(arena_np)
    ctx.batch_var_ex(tcpck.OP_FILL, buf, dev(off), dev(ln), count, None, tcpck.KERNEL_SSTREAM, variant)
    exp, exp_arena = fill_oracle(arena_np, off, ln)
    got = host(buf)
    np.testing.assert_array_equal(got, exp_arena)
    bad = rng.choice(count, min(count, 40), replace=False)
    for k in bad:
        got[int(off[k]) + int(rng.integers(0, int(ln[k])))] ^= 0x42
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var_ex(tcpck.OP_VERIFY, dev(got), dev(off), dev(ln), count, ok, tcpck.KERNEL_SSTREAM, variant)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], np.sort(bad))


FIXED_SLOTS = [(16, 2), (16, 16), (32, 30), (64, 32), (80, 34), (256, 96), (1536, 1492), (2048, 1492),
               (2048, 1494), (2048, 2048), (4096, 1492), (16384, 9000), (65536, 65504), (65536, 65536)]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride,length", FIXED_SLOTS)
@pytest.mark.parametrize("count", [1, 2, 65, 3001, 40000])
def test_sstream_fixed_slots(ctx, oracle_c, variant, stride, length, count):
    import tcpck
    if count * stride > (200 << 20):
        count = (200 << 20) // stride
    rng = np.random.default_rng(stride + length + count + variant)
    arena_np = rng.integers(0, 256, count * stride + 128, dtype=np.uint8)
    buf = dev(arena_np)
    for mis in (0, 2, 6, 14):
        for oversub in (0, 1, 8):
            out = torch.empty(count, dtype=torch.int16, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, stride, length, count, out,
                               tcpck.KERNEL_SSTREAM, variant | (oversub << 16))
            np.testing.assert_array_equal(host(out).view(np.uint16),
                                          oracle_c.batch(arena_np[mis:], stride=stride, length=length, count=count,
                                                         threads=8))
    if length >= 30:
        for mis in (0, 6):
            arena = dev(arena_np)
            out = torch.empty(count, dtype=torch.int16, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_FILL, arena.data_ptr() + mis, stride, length, count, out,
                               tcpck.KERNEL_SSTREAM, variant)
            off = np.arange(count, dtype=np.uint64) * stride
            exp, exp_arena = fill_oracle(arena_np[mis:], off, np.full(count, length, np.uint32))
            np.testing.assert_array_equal(host(out).view(np.uint16), exp)
            got = host(arena)
            np.testing.assert_array_equal(got[mis:], exp_arena)  # gap bytes untouched
            ok = torch.empty(count, dtype=torch.uint8, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_VERIFY, arena.data_ptr() + mis, stride, length, count, ok,
                               tcpck.KERNEL_SSTREAM, variant)
            assert bool(ok.all().item())


def test_sstream_fixed_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    o = torch.zeros(1024, dtype=torch.int16, device="cuda")
    for stride, length in ((1500, 1492), (1492, 1492), (2056, 2058)):  # stride % 16 != 0, or stride < len
        with pytest.raises(tcpck.TcpckError):
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, stride, length, 100, o, tcpck.KERNEL_SSTREAM, 0)
    with pytest.raises(tcpck.TcpckError):  # RFC 1071: images below 128 KiB (exact u32 sums)
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1 << 18, 1 << 17, 2, o, tcpck.KERNEL_SSTREAM, 0, mode=1)
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 32, 28, 100, o, tcpck.KERNEL_SSTREAM, 0)


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("case", ["shuffled", "reversed", "overlap", "chunk_share", "empty", "tiny", "mixed_jumbo",
                                  "packed"])
@pytest.mark.parametrize("count", [1, 256, 257, 4096, 20000])
def test_sstream_any_offsets(ctx, oracle_c, variant, case, count):
    """Any offset list: out-of-order, overlapping and chunk-sharing images, empty
    and 2-B images, jumbo images; runs that start below their first image fall
    back to the exact per-image pass."""
    import tcpck
    rng = np.random.default_rng(count * 13 + variant + len(case))
    if case == "mixed_jumbo":
        ln = rng.choice(np.array([2, 40, 1492, 9000, 65536, 70000], np.uint32), count)
        ln = ln[: max(1, min(count, 2000))]
    elif case == "empty":
        ln = rng.choice(np.array([0, 0, 2, 96, 1492], np.uint32), count)
    elif case == "tiny":
        ln = (rng.integers(0, 9, count) * 2).astype(np.uint32)
    else:
        ln = (rng.integers(0, 800, count) * 2).astype(np.uint32)
    n = ln.size
    if case == "chunk_share" or case == "packed":  # back to back (2-B aligned): neighbours share 16-B chunks
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    elif case == "overlap":
        off = np.cumsum(rng.integers(0, 400, n).astype(np.uint64) * 2)
    else:
        gaps = rng.integers(0, 300, n).astype(np.uint64) * 2
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gaps[:-1])
    if case == "shuffled":
        perm = rng.permutation(n)
        off, ln = off[perm], ln[perm]
    elif case == "reversed":
        off, ln = off[::-1].copy(), ln[::-1].copy()
    total = int((off + ln.astype(np.uint64)).max()) + 128
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    buf = dev(arena_np)
    for mis in (0, 2):
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, dev(off), dev(ln), n, out, tcpck.KERNEL_SSTREAM,
                         variant, total_bytes=int(ln.sum()))
        np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np[mis:], off, ln, threads=8))


@pytest.mark.parametrize("variant", [0, 2])
def test_sstream_golden(ctx, golden, variant):
    """Every golden checksum image made by the reference header (0..65536 B), each in a 64-KiB + 128-B slot."""
    import tcpck
    cases = golden.by_kind("checksum")
    slot = 65536 + 128
    arena_np = np.zeros(len(cases) * slot, np.uint8)
    off = np.arange(len(cases), dtype=np.uint64) * slot + 6
    ln = np.array([c["len"] for c in cases], np.uint32)
    for k, c in enumerate(cases):
        arena_np[int(off[k]):int(off[k]) + c["len"]] = golden.image(c)
    out = torch.empty(len(cases), dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, dev(arena_np), dev(off), dev(ln), len(cases), out, tcpck.KERNEL_SSTREAM,
                     variant)
    np.testing.assert_array_equal(host(out).view(np.uint16), np.array([c["expected"] for c in cases], np.uint16))


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("case", ["packed_2mod16", "gaps_2mod4", "reversed_gaps"])
def test_sstream_fill_any_offsets(ctx, variant, case):
    """FILL on offset lists whose images share 16-B chunks with their neighbours
    (packed at 2-B offsets), 2-mod-4 gaps, and reversed order (per-image pass)."""
    import tcpck
    rng = np.random.default_rng(len(case) * 17 + variant)
    count = 9000
    ln = (rng.integers(15, 800, count) * 2).astype(np.uint32)
    gaps = np.zeros(count, np.uint64) if case == "packed_2mod16" else (rng.integers(0, 40, count) * 2 + 2).astype(np.uint64)
    off = np.zeros(count, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gaps[:-1])
    off += np.uint64(2)
    if case == "reversed_gaps":
        off, ln = off[::-1].copy(), ln[::-1].copy()
    total = int((off + ln.astype(np.uint64)).max()) + 64
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_FILL, arena, dev(off), dev(ln), count, out, tcpck.KERNEL_SSTREAM, variant)
    exp, exp_arena = fill_oracle(arena_np, off, ln)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    np.testing.assert_array_equal(host(arena), exp_arena)


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("slot,lengths", SLOTS[:-1])
@pytest.mark.parametrize("count", [1, 257, 40000])
def test_sstream_rfc1071(ctx, oracle_c, variant, slot, lengths, count):
    """RFC 1071 on the slot stream: exact u32 prefix tables (dword or word
    positions), folded differences; CHECKSUM, VERIFY (AUTO with the SORTED hint)
    and FILL against the RFC oracle."""
    import tcpck
    from oracle import ref16 as R
    if count * slot > (160 << 20):
        count = (160 << 20) // slot
    off, ln, total = slot_layout(count, slot, lengths, seed=count + slot + 7 * variant)
    rng = np.random.default_rng(count * 11 + slot)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    if count > 2:
        k = count // 2
        arena_np[int(off[k]):int(off[k]) + int(ln[k])] = 0xFF
    arena = dev(arena_np)
    d_off, d_ln = dev(off), dev(ln)
    exp = oracle_c.batch(arena_np, off, ln, mode=1, threads=8)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, arena, d_off, d_ln, count, out, tcpck.KERNEL_SSTREAM, variant, mode=1)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, arena, d_off, d_ln, count, ok, mode=1, sorted=True, total_bytes=int(ln.sum()),
                  min_len=int(ln.min()), max_len=int(ln.max()))
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))
    if min(lengths) >= 30:
        ctx.batch_var_ex(tcpck.OP_FILL, arena, d_off, d_ln, count, out, tcpck.KERNEL_SSTREAM, variant, mode=1)
        exp_arena = arena_np.copy()
        expf = np.array([R.fill_np(exp_arena[int(off[k]):int(off[k]) + int(ln[k])], 1) for k in range(count)],
                        np.uint16)
        np.testing.assert_array_equal(host(out).view(np.uint16), expf)
        np.testing.assert_array_equal(host(arena), exp_arena)


@pytest.mark.parametrize("stride,length", [(2048, 1492), (2048, 1494), (256, 96), (16384, 9000), (80, 34)])
def test_sstream_rfc1071_fixed_auto(ctx, oracle_c, stride, length):
    import tcpck
    count = max(8, min(30000, (48 << 20) // stride))
    rng = np.random.default_rng(stride + length)
    arena_np = rng.integers(0, 256, count * stride, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, stride, length, count, out, mode=1)
    np.testing.assert_array_equal(host(out).view(np.uint16),
                                  oracle_c.batch(arena_np, stride=stride, length=length, count=count, mode=1,
                                                 threads=8))
