"""GPU parity of every kernel and variant (include/tcpck_tuning.h) against the
reference's golden vectors and the oracle: seg (each shape), rstream (each
variant) and vvstream (each variant; packed variable, fixed and gapped fixed
layouts), all three ops, misaligned arenas, wrong layout hints, tiny and empty
images, and grid oversubscription."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SEG = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]  # 7-11: 4, 8, 16, 16, 2 waves per image
RSTREAM = [0, 1, 2, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24]  # 9-13: v_dot2 sums and/or buffer loads; 14-21 XCD orders (20, 21: default-policy first step)
VVSTREAM = [0, 1, 2, 3, 4, 28, 36, 60]  # 0/1 byte split U4/U8, 2/3 count split, 4 policy; +8 XCD order, +16 L2-kept first step, +32 FILL default-policy reads


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


def var_kernels():
    import tcpck
    return ([(tcpck.KERNEL_SEG, p) for p in SEG] + [(tcpck.KERNEL_VVSTREAM, v) for v in VVSTREAM] +
            [(tcpck.KERNEL_SSTREAM, v) for v in (0, 1, 2)])


def fixed_kernels():  # sstream's fixed mode takes slots of a multiple of 16 B only (tests/test_gpu_sstream.py)
    import tcpck
    return ([(k, p) for k, p in var_kernels() if k != tcpck.KERNEL_SSTREAM] +
            [(tcpck.KERNEL_RSTREAM, v) for v in RSTREAM])


def packed_layout(count, seed, payloads, header=32):
    rng = np.random.default_rng(seed)
    ln = (np.asarray(payloads, np.int64)[rng.integers(0, len(payloads), count)] + header).astype(np.uint32)
    off = np.zeros(count, np.uint64)
    if count > 1:
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    return off, ln, int(ln.astype(np.int64).sum())


def _fill_oracle(arena_np, off, ln):
    exp_arena = arena_np.copy()
    exp = np.empty(len(off), np.uint16)
    from oracle import ref16 as R
    for k in range(len(off)):
        o, n = int(off[k]), int(ln[k])
        exp[k] = R.fill_np(exp_arena[o:o + n])
    return exp, exp_arena


def packed_golden(golden, min_len=16):
    """Golden checksum images of length >= min_len, re-packed back to back."""
    cases = [c for c in golden.by_kind("checksum") if c["len"] >= min_len]
    imgs = [golden.image(c) for c in cases]
    ln = np.array([c["len"] for c in cases], np.uint32)
    off = np.zeros(len(cases), np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    return np.concatenate(imgs), off, ln, np.array([c["expected"] for c in cases], np.uint16)


# ---- every kernel ----------------------------------------------------------
@pytest.mark.parametrize("kernel,param", var_kernels())
def test_packed_golden_all_kernels(ctx, golden, kernel, param):
    import tcpck
    arena, off, ln, exp = packed_golden(golden)
    out = torch.empty(len(exp), dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, dev(arena), dev(off), dev(ln), len(exp), out, kernel, param,
                     packed=True)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("variant", VVSTREAM)
def test_vvstream_golden_all_lengths(ctx, golden, variant):
    """Every golden checksum image (0..65536 B, incl. < 16 B and empty) packed back to back."""
    import tcpck
    arena, off, ln, exp = packed_golden(golden, min_len=0)
    out = torch.empty(len(exp), dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, dev(arena), dev(off), dev(ln), len(exp), out, tcpck.KERNEL_VVSTREAM,
                     variant, packed=True)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("kernel,param", fixed_kernels())
@pytest.mark.parametrize("length", [16, 32, 96, 606, 1492, 1494, 4096])
def test_fixed_packed_all_kernels(ctx, oracle_c, kernel, param, length):
    import tcpck
    rng = np.random.default_rng(length + param)
    count = 3001
    arena_np = rng.integers(0, 256, count * length, dtype=np.uint8)
    arena_np[length * 5:length * 6] = 0xFF
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, dev(arena_np), length, length, count, out, kernel, param)
    exp = oracle_c.batch(arena_np, stride=length, length=length, count=count, threads=8)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("kernel,param", fixed_kernels())
@pytest.mark.parametrize("mis", [2, 6, 14])
def test_misaligned_arena_pointer(ctx, oracle_c, kernel, param, mis):
    """The arena pointer itself need not be 16-B aligned (e.g. a sliced buffer)."""
    import tcpck
    rng = np.random.default_rng(mis * 31 + param)
    L, count = 1492, 2000
    arena_np = rng.integers(0, 256, count * L + 64, dtype=np.uint8)
    buf = dev(arena_np)
    ptr = buf.data_ptr() + mis
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, ptr, L, L, count, out, kernel, param)
    exp = oracle_c.batch(arena_np[mis:], stride=L, length=L, count=count)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    if kernel == tcpck.KERNEL_RSTREAM:
        return  # fixed layouts only
    off = (np.arange(count, dtype=np.uint64) * L)
    ln = np.full(count, L, np.uint32)
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, ptr, dev(off), dev(ln), count, out, kernel, param, packed=True)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("kernel,param", var_kernels())
def test_var_mixed_with_gaps_and_short_images(ctx, oracle_c, kernel, param):
    """Packed C3-style batch with a wrong packed hint (a few gaps) and images below 16 B."""
    import tcpck
    import synth_np
    rng = np.random.default_rng(param + 100 * kernel)
    count = 20000
    off, ln, total = synth_np.mixed_layout(count, seed=param)
    off = off.copy()
    ln = ln.copy()
    for k in rng.integers(1, count, 40):
        off[k:] += 6
    ln[rng.integers(0, count, 15)] = 8
    total = int(off[-1] + ln[-1]) + 64
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, dev(arena_np), dev(off), dev(ln), count, out, kernel, param, packed=True)
    np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np, off, ln, threads=8))


def test_run_kernels_reject(ctx):
    import tcpck
    a = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    o = torch.zeros(1024, dtype=torch.int16, device="cuda")
    off = torch.arange(8, dtype=torch.int64, device="cuda") * 1000
    ln = torch.full((8,), 1000, dtype=torch.int32, device="cuda")
    with pytest.raises(tcpck.TcpckError):  # rstream: gaps
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1500, 1492, 100, o, tcpck.KERNEL_RSTREAM, 0)
    with pytest.raises(tcpck.TcpckError):  # RFC 1071 on rstream: the policy's variant (20) only
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1492, 1492, 100, o, tcpck.KERNEL_RSTREAM, 0, mode=1)
    with pytest.raises(tcpck.TcpckError):  # RFC 1071 on vvstream: not with the FILL default-policy reads (+32)
        ctx.batch_fixed_ex(tcpck.OP_FILL, a, 96, 96, 100, o, tcpck.KERNEL_VVSTREAM, 36, mode=1)
    with pytest.raises(tcpck.TcpckError):  # RFC 1071 on sstream: images below 128 KiB
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1 << 18, 1 << 17, 2, o, tcpck.KERNEL_SSTREAM, 0, mode=1)
    with pytest.raises(tcpck.TcpckError):  # removed kernels
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1492, 1492, 100, o, 2, 0)
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, a, off, ln, 8, o, 7, 0)


# ---- run-stream kernel (KERNEL_RSTREAM = 5: fixed stride == len, scalar boundary walk) ----


@pytest.mark.parametrize("variant", RSTREAM)
@pytest.mark.parametrize("length", [16, 18, 30, 32, 96, 606, 1024, 1026, 1492, 1494, 4096, 9000, 65536])
@pytest.mark.parametrize("count", [1, 2, 7, 64, 65, 3001, 70001])
def test_rstream_fixed_vs_oracle(ctx, oracle_c, variant, length, count):
    import tcpck
    if count * length > (64 << 20):
        count = (64 << 20) // length
    rng = np.random.default_rng(length * 7 + count + variant)
    arena_np = rng.integers(0, 256, count * length + 128, dtype=np.uint8)  # room for mis <= 126
    arena_np[:length] = 0xFF
    buf = dev(arena_np)
    for mis in (0, 2, 14, 126):
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, length, length, count, out,
                           tcpck.KERNEL_RSTREAM, variant)
        exp = oracle_c.batch(arena_np[mis:], stride=length, length=length, count=count, threads=8)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("variant", RSTREAM)
@pytest.mark.parametrize("length", [30, 32, 96, 128, 130, 196, 1024, 1492, 1494, 2000, 9000])
def test_rstream_fill_verify(ctx, variant, length):
    """Includes 2-mod-4 lengths (fields at every 16-B phase) and jumbo images."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + 10 * variant)
    count = 9000 if length < 4096 else 1500
    arena_np = rng.integers(0, 256, count * length, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, arena, length, length, count, out, tcpck.KERNEL_RSTREAM, variant)
    exp_arena = arena_np.copy()
    exp = np.array([R.fill_np(exp_arena[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    got = host(arena)
    np.testing.assert_array_equal(got, exp_arena)
    bad = rng.choice(count, 64, replace=False)
    for k in bad:
        got[k * length + int(rng.integers(0, length))] ^= 0x24
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, dev(got), length, length, count, ok, tcpck.KERNEL_RSTREAM, variant)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], np.sort(bad))


# ---- prefix-table run stream (KERNEL_VVSTREAM = 8): packed variable and fixed layouts ----
@pytest.mark.parametrize("variant", VVSTREAM)
@pytest.mark.parametrize("payloads", [(64, 576, 1460), (-16, 0, 1460), (-16,), (0, 9000, 65504), (-32, 64, 1460)])
@pytest.mark.parametrize("count", [1, 2, 63, 64, 65, 255, 256, 257, 1000, 70001])
def test_vvstream_var_vs_oracle(ctx, oracle_c, variant, payloads, count):
    """Includes 16-B images and, with payload -32, empty images."""
    import tcpck
    off, ln, total = packed_layout(count, count * 5 + len(payloads), payloads)
    if total > (96 << 20):
        return
    rng = np.random.default_rng(count + 3 * variant)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    buf = dev(arena_np)
    d_off, d_ln = dev(off), dev(ln)
    for mis in (0, 2, 126):
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, d_off, d_ln, count, out,
                         tcpck.KERNEL_VVSTREAM, variant, packed=True, total_bytes=total)
        np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np[mis:], off, ln, threads=8))


@pytest.mark.parametrize("variant", [0, 2, 4])
@pytest.mark.parametrize("payloads", [(-30, -28, -20), (-32, -30), (-32, -2, 1460), (-30, 64, 9000)])
@pytest.mark.parametrize("count", [1, 65, 257, 5000, 70001])
def test_vvstream_tiny_images(ctx, oracle_c, variant, payloads, count):
    """0..14-B images (up to 512 ends per 1 KiB step), several ends per 16-B
    chunk, zero-length runs at the batch end."""
    import tcpck
    off, ln, total = packed_layout(count, count * 7 + len(payloads), payloads)
    rng = np.random.default_rng(count + variant)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    buf = dev(arena_np)
    d_off, d_ln = dev(off), dev(ln)
    for mis in (0, 2, 126):
        for oversub in (1, 8):
            out = torch.empty(count, dtype=torch.int16, device="cuda")
            ctx.batch_var_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, d_off, d_ln, count, out,
                             tcpck.KERNEL_VVSTREAM, variant | (oversub << 16), packed=True)
            np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np[mis:], off, ln, threads=8))
    ln2 = ln.copy()
    ln2[-3:] = 0
    off2 = np.zeros(count, np.uint64)
    if count > 1:
        off2[1:] = np.cumsum(ln2[:-1].astype(np.uint64))
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, buf, dev(off2), dev(ln2), count, out, tcpck.KERNEL_VVSTREAM, variant,
                     packed=True)
    np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np, off2, ln2, threads=8))


@pytest.mark.parametrize("variant", VVSTREAM)
def test_vvstream_not_packed_and_verify(ctx, oracle_c, variant):
    """A wrong packed hint (gaps) costs speed, never correctness: waves fall back."""
    import tcpck
    import synth_np
    rng = np.random.default_rng(40 + variant)
    count = 30000
    off, ln, _ = synth_np.mixed_layout(count, seed=9)
    off = off.copy()
    for k in rng.integers(1, count, 25):
        off[k:] += 10
    total = int(off[-1] + ln[-1]) + 64
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, dev(arena_np), dev(off), dev(ln), count, out,
                     tcpck.KERNEL_VVSTREAM, variant, packed=True)
    np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np, off, ln, threads=8))
    # fill with the same wrong hint: results and the arena equal the per-image oracle
    arena = dev(arena_np)
    ctx.batch_var_ex(tcpck.OP_FILL, arena, dev(off), dev(ln), count, out, tcpck.KERNEL_VVSTREAM, variant,
                     packed=True)
    exp, exp_arena = _fill_oracle(arena_np, off, ln)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    np.testing.assert_array_equal(host(arena), exp_arena)
    # verify on a packed, filled batch with corruptions
    off, ln, total = packed_layout(count, 77, (64, 576, 1460))
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    _, arena_np = _fill_oracle(arena_np, off, ln)
    bad = rng.choice(count, 60, replace=False)
    for k in bad:
        arena_np[int(off[k]) + int(rng.integers(0, int(ln[k])))] ^= 0x81
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var_ex(tcpck.OP_VERIFY, dev(arena_np), dev(off), dev(ln), count, ok, tcpck.KERNEL_VVSTREAM, variant,
                     packed=True)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], np.sort(bad))


@pytest.mark.parametrize("variant", VVSTREAM)
@pytest.mark.parametrize("payloads", [(64, 576, 1460), (-2, 0), (-2,), (0, 9000), (64,)])
@pytest.mark.parametrize("count", [1, 64, 65, 257, 3000, 40000])
def test_vvstream_fill_var(ctx, variant, payloads, count):
    """Send-side fill on packed variable layouts: the field (bytes 28-29) is zeroed
    in the stream and the result lands in out[k] and in the field; stale fields."""
    import tcpck
    off, ln, total = packed_layout(count, count + 11 * variant, payloads)
    rng = np.random.default_rng(count * 3 + variant)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    for mis in (0, 2, 94):
        buf = dev(arena_np)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(tcpck.OP_FILL, buf.data_ptr() + mis, dev(off), dev(ln), count, out,
                         tcpck.KERNEL_VVSTREAM, variant | (8 << 16 if variant == 2 else 0), packed=True,
                         total_bytes=total)
        exp, exp_arena = _fill_oracle(arena_np[mis:], off, ln)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
        np.testing.assert_array_equal(host(buf)[mis:], exp_arena)
        np.testing.assert_array_equal(host(buf)[:mis], arena_np[:mis])


@pytest.mark.parametrize("variant", [0, 1, 4])
@pytest.mark.parametrize("length", [2, 14, 16, 30, 32, 34, 64, 96, 100, 256, 608, 1492])
@pytest.mark.parametrize("count", [1, 63, 1000, 77777])
def test_vvstream_fixed_vs_oracle(ctx, oracle_c, variant, length, count):
    import tcpck
    rng = np.random.default_rng(length * 31 + count + variant)
    arena_np = rng.integers(0, 256, count * length + 128, dtype=np.uint8)
    buf = dev(arena_np)
    for mis in (0, 6, 100):
        for oversub in (0, 4, 32):
            out = torch.empty(count, dtype=torch.int16, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, length, length, count, out,
                               tcpck.KERNEL_VVSTREAM, variant | (oversub << 16))
            np.testing.assert_array_equal(host(out).view(np.uint16),
                                          oracle_c.batch(arena_np[mis:], stride=length, length=length, count=count,
                                                         threads=8))


@pytest.mark.parametrize("variant", [0, 1, 4])
@pytest.mark.parametrize("stride,length", [(4, 2), (34, 32), (100, 2), (128, 96), (1000, 30), (1536, 1492),
                                           (2048, 1492), (70000, 65504)])
@pytest.mark.parametrize("count", [1, 2, 65, 3001, 40000])
def test_vvstream_fixed_gapped(ctx, oracle_c, variant, stride, length, count):
    """stride > length: the run streams the gaps too, as virtual images whose sums are dropped."""
    import tcpck
    if count * stride > (600 << 20):
        count = (600 << 20) // stride
    rng = np.random.default_rng(stride + length + count + variant)
    arena_np = rng.integers(0, 256, count * stride + 128, dtype=np.uint8)
    buf = dev(arena_np)
    for mis in (0, 2, 50):
        for oversub in (0, 8):
            out = torch.empty(count, dtype=torch.int16, device="cuda")
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, stride, length, count, out,
                               tcpck.KERNEL_VVSTREAM, variant | (oversub << 16))
            np.testing.assert_array_equal(host(out).view(np.uint16),
                                          oracle_c.batch(arena_np[mis:], stride=stride, length=length, count=count,
                                                         threads=8))
    if length >= 30:
        arena = dev(arena_np)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_FILL, arena, stride, length, count, out, tcpck.KERNEL_VVSTREAM, variant)
        off = np.arange(count, dtype=np.uint64) * stride
        exp, exp_arena = _fill_oracle(arena_np, off, np.full(count, length, np.uint32))
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
        np.testing.assert_array_equal(host(arena), exp_arena)  # gap bytes untouched
        ok = torch.empty(count, dtype=torch.uint8, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_VERIFY, arena, stride, length, count, ok, tcpck.KERNEL_VVSTREAM, variant)
        assert bool(ok.all().item())


@pytest.mark.parametrize("variant", [0, 4])
@pytest.mark.parametrize("length", [30, 32, 96, 1492])
def test_vvstream_fixed_fill_verify(ctx, variant, length):
    import tcpck
    count = 20000
    rng = np.random.default_rng(length + variant)
    arena_np = rng.integers(0, 256, count * length, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, arena, length, length, count, out, tcpck.KERNEL_VVSTREAM, variant)
    off = np.arange(count, dtype=np.uint64) * length
    ln = np.full(count, length, np.uint32)
    exp, exp_arena = _fill_oracle(arena_np, off, ln)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    got = host(arena)
    np.testing.assert_array_equal(got, exp_arena)
    bad = rng.choice(count, 40, replace=False)
    for k in bad:
        got[int(k) * length + int(rng.integers(0, length))] ^= 0x24
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, dev(got), length, length, count, ok, tcpck.KERNEL_VVSTREAM, variant)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], np.sort(bad))
    with pytest.raises(tcpck.TcpckError):
        ctx.batch_fixed_ex(tcpck.OP_FILL, arena, 28, 28, 100, out, tcpck.KERNEL_VVSTREAM, variant)


# ---- grid oversubscription (param bits 16..23): more, shorter runs per launch ----
@pytest.mark.parametrize("kernel,variant,length", [(5, 0, 1492), (5, 10, 1024), (8, 4, 96), (8, 0, 256), (8, 1, 34)])
@pytest.mark.parametrize("oversub", [2, 8, 32])
def test_oversubscribed_fixed(ctx, oracle_c, kernel, variant, length, oversub):
    import tcpck
    count = (48 << 20) // length
    rng = np.random.default_rng(length + oversub)
    arena_np = rng.integers(0, 256, count * length + 128, dtype=np.uint8)
    buf = dev(arena_np)
    for mis in (0, 6):
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, length, length, count, out, kernel,
                           variant | (oversub << 16))
        exp = oracle_c.batch(arena_np[mis:], stride=length, length=length, count=count, threads=8)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)


@pytest.mark.parametrize("variant", [0, 2, 4])
@pytest.mark.parametrize("oversub", [0, 2, 8, 16, 32])
def test_oversubscribed_vvstream(ctx, oracle_c, variant, oversub):
    import tcpck
    import synth_np
    count = 60000
    off, ln, total = synth_np.mixed_layout(count, seed=oversub + variant)
    rng = np.random.default_rng(variant)
    arena_np = rng.integers(0, 256, total, dtype=np.uint8)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var_ex(tcpck.OP_CHECKSUM, dev(arena_np), dev(off), dev(ln), count, out, tcpck.KERNEL_VVSTREAM,
                     variant | (oversub << 16), packed=True, total_bytes=total)
    np.testing.assert_array_equal(host(out).view(np.uint16), oracle_c.batch(arena_np, off, ln, threads=8))


# ---- group stream (KERNEL_GSTREAM = 9: fixed stride == len, len a power of two in [32, 1024]) ----

GSTREAM = [0, 1, 2, 4, 0x10, 0x20, 0x22, 0x40, 0x80, 0x100, 0x200, 0x201, 0x202]  # include/tcpck_tuning.h
GS_LENGTHS = [32, 64, 128, 256, 512, 1024]


@pytest.mark.parametrize("variant", GSTREAM)
@pytest.mark.parametrize("length", GS_LENGTHS)
@pytest.mark.parametrize("count", [1, 2, 31, 33, 64, 65, 3001, 70001])
def test_gstream_fixed_vs_oracle(ctx, oracle_c, variant, length, count):
    """Every length and ragged counts (partial last step, fewer images than one step),
    the arena at 16-B (not 128-B) alignment too, and grid oversubscription."""
    import tcpck
    rng = np.random.default_rng(length * 11 + count + variant)
    arena_np = rng.integers(0, 256, count * length + 128, dtype=np.uint8)
    arena_np[:length] = 0xFF
    arena_np[length:2 * length] = 0
    buf = dev(arena_np)
    for mis, oversub in ((0, 0), (16, 0), (112, 1), (0, 8)):
        out = torch.full((count + 1,), -1, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, length, length, count, out,
                           tcpck.KERNEL_GSTREAM, variant | (oversub << 16))
        exp = oracle_c.batch(arena_np[mis:], stride=length, length=length, count=count, threads=8)
        got = host(out).view(np.uint16)
        np.testing.assert_array_equal(got[:count], exp)
        assert got[count] == 0xFFFF  # nothing written past the batch


@pytest.mark.parametrize("variant", GSTREAM)
@pytest.mark.parametrize("length", GS_LENGTHS)
def test_gstream_fill_verify(ctx, variant, length):
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length + 13 * variant)
    count = 9001
    arena_np = rng.integers(0, 256, count * length, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, arena, length, length, count, out, tcpck.KERNEL_GSTREAM, variant)
    exp_arena = arena_np.copy()
    exp = np.array([R.fill_np(exp_arena[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    got = host(arena)
    np.testing.assert_array_equal(got, exp_arena)
    # FILL without an output array writes the fields only
    arena2 = dev(arena_np)
    ctx.batch_fixed_ex(tcpck.OP_FILL, arena2, length, length, count, None, tcpck.KERNEL_GSTREAM, variant)
    np.testing.assert_array_equal(host(arena2), exp_arena)
    bad = rng.choice(count, 64, replace=False)
    for k in bad:
        got[k * length + int(rng.integers(0, length))] ^= 0x24
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, dev(got), length, length, count, ok, tcpck.KERNEL_GSTREAM, variant)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], np.sort(bad))


GS_WRITEBACK = [0x400, 0x800, 0x401, 0xC00]  # FILL only: whole-chunk write-back
# multiples of 16 B up to 240 B that are not powers of two: P = 64 / G images per step
GS_NP_LENGTHS = [48, 80, 96, 112, 144, 176, 192, 240]
GS_NP = [0, 1, 2, 4, 0x80]


@pytest.mark.parametrize("variant", GS_NP)
@pytest.mark.parametrize("length", GS_NP_LENGTHS)
@pytest.mark.parametrize("count", [1, 9, 11, 65, 3001])
def test_gstream_np_vs_oracle(ctx, oracle_c, variant, length, count):
    """Steps of P = 64 / G whole images (idle lanes at the top of the wave), ragged
    counts, 16-B misaligned arenas, grid oversubscription."""
    import tcpck
    rng = np.random.default_rng(length * 13 + count + variant)
    arena_np = rng.integers(0, 256, count * length + 128, dtype=np.uint8)
    arena_np[:length] = 0xFF
    buf = dev(arena_np)
    for mis, oversub in ((0, 0), (16, 0), (48, 1), (0, 8)):
        out = torch.full((count + 1,), -1, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, length, length, count, out,
                           tcpck.KERNEL_GSTREAM, variant | (oversub << 16))
        exp = oracle_c.batch(arena_np[mis:], stride=length, length=length, count=count, threads=8)
        got = host(out).view(np.uint16)
        np.testing.assert_array_equal(got[:count], exp)
        assert got[count] == 0xFFFF  # nothing written past the batch
        ok = torch.full((count + 1,), 7, dtype=torch.uint8, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_VERIFY, buf.data_ptr() + mis, length, length, count, ok,
                           tcpck.KERNEL_GSTREAM, variant | (oversub << 16))
        np.testing.assert_array_equal(host(ok)[:count], (exp == 0).astype(np.uint8))
        assert host(ok)[count] == 7


@pytest.mark.parametrize("variant", GS_NP + [0x400, 0x401])
@pytest.mark.parametrize("length", GS_NP_LENGTHS)
@pytest.mark.parametrize("count", [1, 11, 9001])
def test_gstream_np_fill(ctx, variant, length, count):
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length * 5 + count + variant)
    for mis in (0, 16):
        arena_np = rng.integers(0, 256, count * length + 256 + mis, dtype=np.uint8)
        arena = dev(arena_np)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_FILL, arena.data_ptr() + mis, length, length, count, out,
                           tcpck.KERNEL_GSTREAM, variant)
        exp_arena = arena_np.copy()
        body = exp_arena[mis:mis + count * length]  # a view: fill_np writes the fields in place
        exp = np.array([R.fill_np(body[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
        np.testing.assert_array_equal(host(arena), exp_arena)


@pytest.mark.parametrize("variant", GS_WRITEBACK)
@pytest.mark.parametrize("length", GS_LENGTHS)
@pytest.mark.parametrize("count", [1, 33, 9001])
def test_gstream_fill_writeback(ctx, variant, length, count):
    """The write-back FILL rewrites every chunk of the batch: the images must come back
    byte-exact except the field, and the guard bytes after the batch untouched."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length * 7 + count + variant)
    for mis in (0, 16):
        arena_np = rng.integers(0, 256, count * length + 256 + mis, dtype=np.uint8)
        arena = dev(arena_np)
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_FILL, arena.data_ptr() + mis, length, length, count, out,
                           tcpck.KERNEL_GSTREAM, variant)
        exp_arena = arena_np.copy()
        body = exp_arena[mis:mis + count * length]
        exp = np.array([R.fill_np(body[k * length:(k + 1) * length]) for k in range(count)], np.uint16)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
        np.testing.assert_array_equal(host(arena), exp_arena)
    with pytest.raises(tcpck.TcpckError):  # CHECKSUM / VERIFY have nothing to write back
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, length, length, count, out, tcpck.KERNEL_GSTREAM, variant)


def test_gstream_golden_header_only(ctx, golden):
    """Header-only images (MakeTcpPacket(0), 32 B) from the golden fixtures, packed at stride 32."""
    import tcpck
    cases = [c for c in golden.by_kind("checksum") if c["len"] == 32]
    assert cases
    arena_np = np.concatenate([golden.image(c) for c in cases])
    out = torch.empty(len(cases), dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, dev(arena_np), 32, 32, len(cases), out, tcpck.KERNEL_GSTREAM, 0)
    np.testing.assert_array_equal(host(out).view(np.uint16), np.array([c["expected"] for c in cases], np.uint16))


def test_gstream_reject(ctx):
    import tcpck
    a = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    o = torch.zeros(4096, dtype=torch.int16, device="cuda")
    for stride, length in ((272, 272), (100, 100), (16, 16), (2048, 2048), (64, 32), (1492, 1492)):
        with pytest.raises(tcpck.TcpckError):
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, stride, length, 100, o, tcpck.KERNEL_GSTREAM, 0)
    with pytest.raises(tcpck.TcpckError):  # arena not 16-B aligned
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a.data_ptr() + 2, 64, 64, 100, o, tcpck.KERNEL_GSTREAM, 0)
    with pytest.raises(tcpck.TcpckError):  # RFC 1071 mode: seg only
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 64, 64, 100, o, tcpck.KERNEL_GSTREAM, 0, mode=1)
    for v in (3, 8, 0x30, 0x1000):  # no such variant
        with pytest.raises(tcpck.TcpckError):
            ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 64, 64, 100, o, tcpck.KERNEL_GSTREAM, v)
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 64, 64, 0, o, tcpck.KERNEL_GSTREAM, 0)  # empty batch: no-op


@pytest.mark.parametrize("length", [512, 1024, 1492, 1494, 2000, 4096, 9000, 65536])
@pytest.mark.parametrize("kind", ["random", "ones", "zeros", "sum_ffff"])
def test_rstream_rfc1071_vs_oracle(ctx, oracle_c, length, kind):
    """Opt-in RFC 1071 mode on rstream (the policy's variant 20): the run prefix is
    an exact u32 word sum, so the image differences fold exactly -- including
    all-0xFF images, all-zero images (+0 vs -0) and images whose word sum is a
    multiple of 0xFFFF.  CHECKSUM, FILL (arena) and VERIFY against the RFC oracle."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(length)
    count = max(16, min(60000, (64 << 20) // length))  # several images per run: boundaries inside runs
    if kind == "random":
        arena_np = rng.integers(0, 256, count * length, dtype=np.uint8)
    elif kind == "ones":
        arena_np = np.full(count * length, 0xFF, np.uint8)
    elif kind == "zeros":
        arena_np = np.zeros(count * length, np.uint8)
    else:  # word sums that are multiples of 0xFFFF: a 0xFFFF word, the rest zero
        arena_np = np.zeros(count * length, np.uint8)
        arena_np[(np.arange(count) * length + 40)] = 0xFF
        arena_np[(np.arange(count) * length + 41)] = 0xFF
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    arena = dev(arena_np)
    exp = oracle_c.batch(arena_np, stride=length, length=length, count=count, mode=1, threads=8)
    for oversub in (0, 1, 16):
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, length, length, count, out, tcpck.KERNEL_RSTREAM,
                           20 | (oversub << 16), mode=1)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, length, length, count, out, mode=1)  # AUTO
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ctx.batch_fixed_ex(tcpck.OP_FILL, arena, length, length, count, out, tcpck.KERNEL_RSTREAM, 20, mode=1)
    exp_arena = arena_np.copy()
    expf = np.array([R.fill_np(exp_arena[k * length:(k + 1) * length], 1) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), expf)
    np.testing.assert_array_equal(host(arena), exp_arena)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, arena, length, length, count, ok, tcpck.KERNEL_RSTREAM, 20, mode=1)
    exp_ok = (oracle_c.batch(exp_arena, stride=length, length=length, count=count, mode=1, threads=8) == 0)
    np.testing.assert_array_equal(host(ok).astype(bool), exp_ok)


def test_rstream_rfc1071_rejects(ctx):
    import tcpck
    a = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    o = torch.zeros(16, dtype=torch.int16, device="cuda")
    with pytest.raises(tcpck.TcpckError):  # RFC 1071 on rstream: the policy's variant only
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1492, 1492, 16, o, tcpck.KERNEL_RSTREAM, 10, mode=1)
    with pytest.raises(tcpck.TcpckError):  # images of 128 KiB and more: the exact u32 sum could wrap
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, 1 << 17, 1 << 17, 4, o, tcpck.KERNEL_RSTREAM, 20, mode=1)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 28])
@pytest.mark.parametrize("payloads", [(64, 576, 1460), (66, 578, 1462), (-30, -2, 0, 64), (0, 9000, 65504)])
@pytest.mark.parametrize("count", [1, 65, 257, 5000, 70001])
def test_vvstream_rfc1071_var(ctx, oracle_c, variant, payloads, count):
    """RFC 1071 on vvstream, packed variable layouts: the u32 prefix table at dword
    positions (4-B aligned ends) or at every word position (2-mod-4 ends), exact
    sums folded.  CHECKSUM and VERIFY against the RFC oracle, misaligned arenas."""
    import tcpck
    off, ln, total = packed_layout(count, count + len(payloads) + variant, payloads)
    if total > (96 << 20):
        return
    rng = np.random.default_rng(count * 3 + variant)
    arena_np = rng.integers(0, 256, total + 128, dtype=np.uint8)
    if count > 3:
        k = count // 2
        arena_np[int(off[k]):int(off[k]) + int(ln[k])] = 0xFF  # an all-ones image
    buf = dev(arena_np)
    d_off, d_ln = dev(off), dev(ln)
    for mis in (0, 2):
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_var_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, d_off, d_ln, count, out, tcpck.KERNEL_VVSTREAM,
                         variant, mode=1, packed=True, total_bytes=total)
        exp = oracle_c.batch(arena_np[mis:], off, ln, mode=1, threads=8)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, buf, d_off, d_ln, count, ok, mode=1, packed=True, total_bytes=total,
                  min_len=int(ln.min()), max_len=int(ln.max()))  # AUTO
    np.testing.assert_array_equal(host(ok), (oracle_c.batch(arena_np, off, ln, mode=1, threads=8) == 0).astype(np.uint8))


@pytest.mark.parametrize("stride,length", [(32, 32), (96, 96), (98, 98), (256, 256), (510, 510), (128, 96),
                                           (1536, 1492), (1000, 998)])
@pytest.mark.parametrize("count", [1, 63, 4000, 100000])
def test_vvstream_rfc1071_fixed_fill(ctx, oracle_c, stride, length, count):
    """RFC 1071 on vvstream's fixed and gapped modes: CHECKSUM, FILL (arena byte-exact)
    and VERIFY; packed small images through AUTO as well."""
    import tcpck
    from oracle import ref16 as R
    if count * stride > (64 << 20):
        count = (64 << 20) // stride
    rng = np.random.default_rng(stride + length + count)
    arena_np = rng.integers(0, 256, count * stride + 64, dtype=np.uint8)
    arena = dev(arena_np)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    exp = oracle_c.batch(arena_np, stride=stride, length=length, count=count, mode=1, threads=8)
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, arena, stride, length, count, out, tcpck.KERNEL_VVSTREAM, 4, mode=1)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    if stride == length:
        ctx.batch_fixed(tcpck.OP_CHECKSUM, arena, stride, length, count, out, mode=1)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    ctx.batch_fixed_ex(tcpck.OP_FILL, arena, stride, length, count, out, tcpck.KERNEL_VVSTREAM, 4, mode=1)
    exp_arena = arena_np.copy()
    expf = np.array([R.fill_np(exp_arena[k * stride:k * stride + length], 1) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), expf)
    np.testing.assert_array_equal(host(arena), exp_arena)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, arena, stride, length, count, ok, tcpck.KERNEL_VVSTREAM, 4, mode=1)
    np.testing.assert_array_equal(host(ok).astype(bool),
                                  oracle_c.batch(exp_arena, stride=stride, length=length, count=count, mode=1,
                                                 threads=8) == 0)


# ---- seg W-wave shapes with the chunk-walk rotation (SegArgs::rot = param bits 8-15) ----
# AUTO's C4 form (seg W16, rot 29, tcpck_api.hip kSegW16Rot): image k's chunks are
# read from 1-KiB step (rot k) mod (chunks / 64) on, wrapping; every byte is still
# summed once, so results are the unrotated ones (include/tcp-header.h:252-263).
@pytest.mark.parametrize("shape", [11, 7, 8, 9])  # W2, W4, W8, W16
@pytest.mark.parametrize("rot", [1, 29, 64, 255])
@pytest.mark.parametrize("length,stride", [(65536, 65536), (65534, 65536), (49152, 49152), (40000, 40000),
                                           (16384, 16384), (9000, 9216), (2048, 2048), (131072, 131072)])
def test_seg_wave_shapes_rotated(ctx, oracle_c, shape, rot, length, stride):
    import tcpck
    from oracle import ref16 as R
    count = max(3, min(300, (24 << 20) // stride))
    rng = np.random.default_rng(length + 7 * rot + shape)
    arena_np = rng.integers(0, 256, count * stride + 128, dtype=np.uint8)
    arena_np[:length] = 0xFF
    buf = dev(arena_np)
    param = (1 << 24) | (rot << 8) | shape
    for mis in (0, 2, 126):
        out = torch.empty(count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, buf.data_ptr() + mis, stride, length, count, out, tcpck.KERNEL_SEG, param)
        exp = oracle_c.batch(arena_np[mis:], stride=stride, length=length, count=count, threads=8)
        np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    # FILL in place, then VERIFY with a few images damaged
    img = arena_np[:count * stride].copy()
    a = dev(img)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_FILL, a, stride, length, count, out, tcpck.KERNEL_SEG, param)
    exp_img = img.copy()
    exp = np.array([R.fill_np(exp_img[k * stride:k * stride + length]) for k in range(count)], np.uint16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    got = host(a)
    np.testing.assert_array_equal(got, exp_img)
    bad = np.sort(rng.choice(count, 3, replace=False))
    for k in bad:
        got[k * stride + int(rng.integers(0, length))] ^= 0x81
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_VERIFY, dev(got), stride, length, count, ok, tcpck.KERNEL_SEG, param)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], bad)


@pytest.mark.parametrize("length", [49152, 57344, 65520, 65536])
def test_auto_packed_w16_rotated(ctx, oracle_c, length):
    """AUTO on packed jumbo images that take seg W16 (rot 29): CHECKSUM, VERIFY and RECEIVE's verdicts."""
    import tcpck
    from oracle import ref16 as R
    count = 400
    rng = np.random.default_rng(length)
    img = rng.integers(0, 256, count * length, dtype=np.uint8)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, dev(img), length, length, count, out)
    np.testing.assert_array_equal(host(out).view(np.uint16),
                                  oracle_c.batch(img, stride=length, length=length, count=count, threads=8))
    for k in range(count):
        R.fill_np(img[k * length:(k + 1) * length])
    bad = np.sort(rng.choice(count, 7, replace=False))
    for k in bad:
        img[k * length + int(rng.integers(0, length))] ^= 0x10
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, dev(img), length, length, count, ok)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], bad)
    hdr = torch.empty(count * 32, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(dev(img), count, ok, hdr, stride=length, length=length)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], bad)
