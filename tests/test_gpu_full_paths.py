"""GPU parity, round 4: the exact kernels the bench times, compared in full.

* C3 through bench.py's own call (packed=True with its total_bytes / min_len /
  max_len hints: AUTO -> vvstream), all 4,194,304 results against the oracle;
* C4 (256K x 64 KiB, AUTO -> seg W16 with the rotated chunk walk) -- all
  262,144 results against the oracle, the 16 GiB arena copied to the host in
  1 GiB chunks; then single-byte corruptions placed in image k's first and
  last rotated 1-KiB steps (steps (29 k) mod 64 and the one before it) are
  caught exactly;
* FILL without a results buffer (the reference's call shape,
  src/socket-manager.cc:9-10): the context's scratch keeps AUTO's two-pass
  forms; the whole arena byte-exact against the oracle's fill at C2 (both
  modes) and C3, past the scratch's 8M images (chunks) on fixed and offset-list
  layouts, and from two streams in turn;
* RECEIVE under AUTO with TCPCK_PARAM_RECEIVE_TWO_PASS: the
  separate header pass runs and the results equal the fused form's.

Oracle: oracle/ref16.c restating include/tcp-header.h:252-263, pinned by
tests/golden (tests/test_oracle.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = tcpck.Context(0)  # libtcpck.so, AUTO only
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def expected_fill(arena: np.ndarray, offs, lens, oracle_c, mode=0) -> np.ndarray:
    """The arena after the reference's insert on every image of >= 30 B
    (socket-manager.cc:9-10: field zeroed, CalculateChecksum, stored raw)."""
    h = arena.copy()
    o = np.asarray(offs, np.int64)
    ln = np.asarray(lens, np.int64)
    has = ln >= 30
    f = o[has] + 28
    h[f] = 0
    h[f + 1] = 0
    c = oracle_c.batch(h, o.astype(np.uint64), ln.astype(np.uint32), mode=mode, threads=16)[has]
    h[f] = (c & 0xFF).astype(np.uint8)
    h[f + 1] = (c >> 8).astype(np.uint8)
    return h


# ---- C3: the bench's call, every result ------------------------------------------

def test_c3_full_bench_call_vvstream_vs_oracle(ctx, oracle_c):
    """bench.py's C3 step exactly (Workload 'mixed': packed=True, total_bytes,
    min_len, max_len): all 4M results against the oracle."""
    import tcpck
    import synth_np
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42)
    img_bytes = int(ln.astype(np.int64).sum())
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_var(tcpck.OP_CHECKSUM, a, d_off, d_ln, count, out, total_bytes=img_bytes,
                  min_len=int(ln.min()), max_len=int(ln.max()), packed=True)
    exp = oracle_c.batch(host(a), off, ln, threads=16)
    np.testing.assert_array_equal(host(out).view(np.uint16), exp)
    # VERIFY through the same kernel: exactly the images whose checksum is 0
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, count, ok, total_bytes=img_bytes, min_len=int(ln.min()),
                  max_len=int(ln.max()), packed=True)
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))


# ---- C4: every result of the rotated W16 walk ------------------------------------------

def _c4_results_host(a, count, L, oracle_c, chunk_images=16384):
    exp = np.empty(count, np.uint16)
    view = a.view(count, L)
    for k0 in range(0, count, chunk_images):
        k1 = min(count, k0 + chunk_images)
        h = host(view[k0:k1]).reshape(-1)  # 1 GiB at a time
        exp[k0:k1] = oracle_c.batch(h, stride=L, length=L, count=k1 - k0, threads=16)
        del h
    return exp


def test_c4_full_all_results_and_rotated_step_corruption(ctx, oracle_c):
    import tcpck
    count, L = 256 << 10, 65536
    a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, count, seed=42)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out)
    got = host(out).view(np.uint16).copy()
    exp = _c4_results_host(a, count, L, oracle_c)
    np.testing.assert_array_equal(got, exp)
    # corruptions in image k's first and last 1-KiB steps of its rotated walk
    # (kSegW16Rot = 29: the walk starts at step (29 k) mod 64 and wraps)
    rng = np.random.default_rng(29)
    ks = np.unique(np.concatenate([rng.integers(0, count, 1500), [0, 1, 63, 64, count - 1]]))
    first = ks * 29 % 64
    last = (first + 63) % 64
    which = rng.integers(0, 2, ks.size)
    step = np.where(which == 0, first, last)
    pos = ks * L + step * 1024 + rng.integers(0, 1024, ks.size)
    d_pos = torch.from_numpy(pos.astype(np.int64)).cuda()
    a[d_pos] ^= 0x01  # bit 0 of one byte: the word sum moves by 1 or 256
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out)
    after = host(out).view(np.uint16)
    np.testing.assert_array_equal(np.nonzero(after != got)[0], ks)
    sample = host(a.view(count, L)[torch.from_numpy(ks).cuda()]).reshape(-1)
    np.testing.assert_array_equal(after[ks], oracle_c.batch(sample, stride=L, length=L, count=ks.size, threads=16))
    # and VERIFY (the same rotated walk) after a FILL: exactly the corrupted images fail
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, None)
    a[d_pos] ^= 0x01
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, count, ok)
    np.testing.assert_array_equal(np.nonzero(host(ok) == 0)[0], ks)
    del a
    torch.cuda.empty_cache()


# ---- FILL without a results buffer --------------------------------------------------

@pytest.mark.parametrize("mode", [0, 1])
def test_fill_noout_c2_full_arena_exact(ctx, oracle_c, mode):
    """C2 FILL with out=None: every arena byte against the reference's insert."""
    import tcpck
    count, L = 1 << 20, 1492
    a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, count, seed=43)
    offs = np.arange(count, dtype=np.int64) * L
    want = expected_fill(host(a), offs, np.full(count, L), oracle_c, mode)
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, None, mode=mode)
    np.testing.assert_array_equal(host(a), want)
    # and with a results buffer: the same arena, results = the stored fields
    tcpck.synth_fixed(a, L, L, count, seed=43)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, out, mode=mode)
    np.testing.assert_array_equal(host(a), want)
    np.testing.assert_array_equal(host(out).view(np.uint16), want[offs + 28] | (want[offs + 29].astype(np.uint16) << 8))


def test_fill_noout_c3_full_arena_exact(ctx, oracle_c):
    """C3 FILL with out=None and the bench's hints (the update form through the
    scratch): every arena byte against the reference's insert, then VERIFY."""
    import tcpck
    import synth_np
    count = 4 << 20
    off, ln, total = synth_np.mixed_layout(count, seed=42)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=44)
    want = expected_fill(host(a), off, ln, oracle_c)
    hints = dict(total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()), packed=True)
    ctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, count, None, **hints)
    np.testing.assert_array_equal(host(a), want)
    ok = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, count, ok, **hints)
    assert int(ok.sum(dtype=torch.int64).item()) == count


@pytest.mark.parametrize("length", [96, 1492])
def test_fill_noout_fixed_chunks_past_scratch(ctx, oracle_c, length):
    """More images than the scratch holds (8M): the batch runs in chunks, the
    last one short (one image: its stride is not read)."""
    import tcpck
    count = (8 << 20) + 1 if length == 96 else (8 << 20) + 5
    a = torch.empty(count * length, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, length, length, count, seed=45)
    offs = np.arange(count, dtype=np.int64) * length
    want = expected_fill(host(a), offs, np.full(count, length), oracle_c)
    ctx.batch_fixed(tcpck.OP_FILL, a, length, length, count, None)
    np.testing.assert_array_equal(host(a), want)
    del a
    torch.cuda.empty_cache()


@pytest.mark.parametrize("packed", [True, False])
def test_fill_noout_var_chunks_past_scratch(ctx, oracle_c, packed):
    """An offset list of 9M images of 30-200 B (packed: vvstream), or with
    gaps and a few images below 30 B that hold no field (seg): chunks of 8M
    through the scratch, offsets and lengths advanced."""
    import tcpck
    rng = np.random.default_rng(46 + packed)
    count = 9 << 20
    ln = (rng.integers(15, 101, count) * 2).astype(np.uint32)
    if not packed:
        ln[rng.integers(0, count, 1000)] = 16
    gap = np.zeros(count, np.int64) if packed else rng.integers(0, 3, count) * 2
    off = np.zeros(count, np.int64)
    off[1:] = np.cumsum(ln[:-1].astype(np.int64) + gap[:-1])
    total = int(off[-1] + ln[-1])
    a_h = rng.integers(0, 256, total, dtype=np.uint8)
    want = expected_fill(a_h, off, ln, oracle_c)
    a = dev(a_h)
    hints = dict(total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                 packed=packed, sorted=not packed)
    ctx.batch_var(tcpck.OP_FILL, a, dev(off.astype(np.uint64)), dev(ln), count, None, **hints)
    np.testing.assert_array_equal(host(a), want)


@pytest.mark.parametrize("count", [1, 2, 3, 65, 4097])
@pytest.mark.parametrize("length", [30, 96, 1492, 9000, 65536])
@pytest.mark.parametrize("mode", [0, 1])
def test_fill_noout_small_batches(ctx, oracle_c, count, length, mode):
    """out=None on tiny and odd-sized batches through every AUTO route (fixed
    packed, and the same bytes as a packed offset list): arena byte-exact."""
    import tcpck
    rng = np.random.default_rng(count * 7 + length + mode)
    a_h = rng.integers(0, 256, count * length + 2, dtype=np.uint8)[2:]  # (an even, not 16-B aligned start)
    offs = np.arange(count, dtype=np.int64) * length
    want = expected_fill(a_h, offs, np.full(count, length), oracle_c, mode)
    buf = dev(a_h)
    ctx.batch_fixed(tcpck.OP_FILL, buf, length, length, count, None, mode=mode)
    np.testing.assert_array_equal(host(buf), want)
    buf = dev(a_h)
    ln = np.full(count, length, np.uint32)
    ctx.batch_var(tcpck.OP_FILL, buf, dev(offs.astype(np.uint64)), dev(ln), count, None, mode=mode,
                  total_bytes=count * length, min_len=length, max_len=length, packed=True)
    np.testing.assert_array_equal(host(buf), want)


def test_fill_noout_explicit_kernel_stays_in_stream(ctx, oracle_c):
    """The scratch is AUTO's: an explicit kernel with out=None keeps its own
    in-stream form (tcpck_tuning.h) -- the same arena either way."""
    import tcpck
    count, L = 4096, 1492
    a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, count, seed=49)
    want = expected_fill(host(a), np.arange(count, dtype=np.int64) * L, np.full(count, L), oracle_c)
    ctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, count, None, tcpck.KERNEL_RSTREAM, 20)
    np.testing.assert_array_equal(host(a), want)


def test_fill_noout_two_streams_in_turn(ctx, oracle_c):
    """The scratch shared by FILLs on two streams (each waits for the other's
    last use): both arenas byte-exact."""
    import tcpck
    count, L = 1 << 18, 1492
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    arenas, wants = [], []
    for seed in (47, 48):
        a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
        tcpck.synth_fixed(a, L, L, count, seed=seed)
        arenas.append(a)
        wants.append(expected_fill(host(a), np.arange(count, dtype=np.int64) * L, np.full(count, L), oracle_c))
    torch.cuda.synchronize()
    for _ in range(3):  # FILL is idempotent: the field is zeroed before the sum
        ctx.batch_fixed(tcpck.OP_FILL, arenas[0], L, L, count, None, stream=s1)
        ctx.batch_fixed(tcpck.OP_FILL, arenas[1], L, L, count, None, stream=s2)
    torch.cuda.synchronize()
    for a, w in zip(arenas, wants):
        np.testing.assert_array_equal(host(a), w)


# ---- RECEIVE: TCPCK_PARAM_RECEIVE_TWO_PASS under AUTO --------------------------------

def _kernel_names(fn):
    """Device kernels one call launched (torch.profiler), or None when the
    profiler records no device activity on this box."""
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if "kernel" in e.name}
    return names or None


def _ring(rng, n, slot, lmin, lmax, mode):
    from oracle import ref16 as R
    ln = (rng.integers(lmin // 2, lmax // 2 + 1, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = rng.integers(0, 256, n * slot, dtype=np.uint8)
    for o, l in zip(off[::3], ln[::3]):
        R.fill_np(a[int(o):int(o) + int(l)], mode)
    return a, off, ln


@pytest.mark.parametrize("layout", ["slots96", "slots64", "ring"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("hdr_mis", [0, 4])
@pytest.mark.parametrize("two_pass", [False, True])
def test_auto_receive_small_images_two_pass(ctx, layout, mode, hdr_mis, two_pass):
    """AUTO RECEIVE on small images in wide slots (96 / 64 B in 256-B slots:
    sstream with the headers from its registers) and on a ring of 32-254-B
    datagrams; the header array 16-B aligned and only 4-B aligned; with and
    without TCPCK_PARAM_RECEIVE_TWO_PASS.  Verdicts, every header byte, the
    arena untouched."""
    import tcpck
    from oracle import ref16 as R
    rng = np.random.default_rng(["slots96", "slots64", "ring"].index(layout) * 100 + 10 * mode + hdr_mis)
    n, slot = 20000, 256
    if layout == "ring":
        a, off, ln = _ring(rng, n, slot, 32, 254, mode)
    else:
        L = 96 if layout == "slots96" else 64
        a, off, ln = _ring(rng, n, slot, L, L, mode)
    buf = dev(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hbuf = torch.full((n * 32 + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    hdr = hbuf.data_ptr() + hdr_mis
    param = tcpck.PARAM_RECEIVE_TWO_PASS if two_pass else 0
    kw = dict(mode=mode, kernel=tcpck.KERNEL_AUTO, param=param)
    if layout == "ring":
        kw.update(offsets=dev(off), lengths=dev(ln), total_bytes=int(ln.sum()), min_len=int(ln.min()),
                  max_len=int(ln.max()), sorted=True)
    else:
        kw.update(stride=slot, length=int(ln[0]))
    ctx.batch_receive(buf, n, ok, hdr, **kw)
    exp_ok = (R.ref16_batch_np(a, off, ln, mode) == 0).astype(np.uint8)
    np.testing.assert_array_equal(host(ok), exp_ok)
    o = off.astype(np.int64)
    hb = host(hbuf)
    np.testing.assert_array_equal(hb[hdr_mis:hdr_mis + 32 * n], a[o[:, None] + R.HEADER_PERM[None, :]].reshape(-1))
    np.testing.assert_array_equal(hb[:hdr_mis], np.full(hdr_mis, 0xEE, np.uint8))
    np.testing.assert_array_equal(host(buf), a)


@pytest.mark.parametrize("layout", ["slots96", "ring"])
def test_auto_receive_two_pass_runs_the_header_pass(ctx, layout):
    """TCPCK_PARAM_RECEIVE_TWO_PASS under AUTO keeps the separate header pass
    (tcpck_tuning.h): header_extract_kernel runs with the bit and does not
    without it (AUTO's sstream writes the headers from its registers)."""
    import tcpck
    rng = np.random.default_rng(7)
    n, slot = 20000, 256
    a, off, ln = _ring(rng, n, slot, 32 if layout == "ring" else 96, 254 if layout == "ring" else 96, 0)
    buf = dev(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    kw = dict(kernel=tcpck.KERNEL_AUTO)
    if layout == "ring":
        kw.update(offsets=dev(off), lengths=dev(ln), total_bytes=int(ln.sum()), min_len=int(ln.min()),
                  max_len=int(ln.max()), sorted=True)
    else:
        kw.update(stride=slot, length=96)
    fused = _kernel_names(lambda: ctx.batch_receive(buf, n, ok, hdr, param=0, **kw))
    two = _kernel_names(lambda: ctx.batch_receive(buf, n, ok, hdr, param=tcpck.PARAM_RECEIVE_TWO_PASS, **kw))
    if fused is None or two is None:
        pytest.skip("torch.profiler records no device kernels on this box")
    assert not any("header_extract_kernel" in k for k in fused), fused
    assert any("header_extract_kernel" in k for k in two), two
    assert any("sstream_kernel" in k for k in two), two
