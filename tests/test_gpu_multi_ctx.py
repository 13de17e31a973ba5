"""Host batches over several contexts at once (tcpck_host_batch_*_multi: one
context per GPU, contiguous shards, one host thread each).  On a one-GPU box
the contexts share device 0, which exercises the same sharding, threads and
per-context staging; results, FILL's arena bytes and VERIFY verdicts against
the oracle (tcp-header.h:252-263; send path socket-manager.cc:9-10)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctxs(built_lib):
    import tcpck
    assert torch.cuda.is_available()
    cs = [tcpck.Context(0) for _ in range(3)]
    for c in cs:
        c.set_chunk_bytes(4 << 20)  # several chunks per shard
    yield cs
    for c in cs:
        c.close()


def fill_expect(a, offs, lens):
    from oracle import ref16 as R
    exp = a.copy()
    want = np.array([R.fill_np(exp[int(o):int(o) + int(n)]) for o, n in zip(offs, lens)], np.uint16)
    return exp, want


@pytest.mark.parametrize("length", [96, 1492, 9000])
@pytest.mark.parametrize("nctx", [1, 2, 3, "same"])
@pytest.mark.parametrize("count", [1, 2, 5000])
def test_multi_fixed(ctxs, oracle_c, length, nctx, count):
    import tcpck
    use = [ctxs[0], ctxs[0]] if nctx == "same" else ctxs[:nctx]
    rng = np.random.default_rng(length + count + len(use))
    a = rng.integers(0, 256, count * length, dtype=np.uint8)
    out = np.zeros(count, np.uint16)
    tcpck.host_batch_fixed_multi(use, tcpck.OP_CHECKSUM, a, length, length, count, out)
    exp = oracle_c.batch(a, stride=length, length=length, count=count)
    np.testing.assert_array_equal(out, exp)
    ok = np.zeros(count, np.uint8)
    tcpck.host_batch_fixed_multi(use, tcpck.OP_VERIFY, a, length, length, count, ok)
    np.testing.assert_array_equal(ok, (exp == 0).astype(np.uint8))
    exp_a, want = fill_expect(a, np.arange(count) * length, np.full(count, length))
    b = a.copy()
    tcpck.host_batch_fixed_multi(use, tcpck.OP_FILL, b, length, length, count, out)
    np.testing.assert_array_equal(out, want)
    np.testing.assert_array_equal(b, exp_a)
    c = a.copy()
    tcpck.host_batch_fixed_multi(use, tcpck.OP_FILL, c, length, length, count, None)
    np.testing.assert_array_equal(c, exp_a)


@pytest.mark.parametrize("layout", ["packed", "slots"])
@pytest.mark.parametrize("nctx", [1, 2, 3])
def test_multi_var(ctxs, oracle_c, layout, nctx):
    """Variable lengths: shards balanced by bytes (a 1492-B image is 15.5x a
    96-B one); packed and in receive slots."""
    import tcpck
    rng = np.random.default_rng(7 * nctx + len(layout))
    n = 20000
    ln = np.asarray((96, 608, 1492), np.uint32)[rng.integers(0, 3, n)]
    if layout == "packed":
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        total = int(ln.sum())
    else:
        off = np.arange(n, dtype=np.uint64) * np.uint64(2048)
        total = n * 2048
    a = rng.integers(0, 256, total, dtype=np.uint8)
    out = np.zeros(n, np.uint16)
    tcpck.host_batch_var_multi(ctxs[:nctx], tcpck.OP_CHECKSUM, a, off, ln, n, out)
    exp = oracle_c.batch(a, off, ln)
    np.testing.assert_array_equal(out, exp)
    b = a.copy()
    tcpck.host_batch_var_multi(ctxs[:nctx], tcpck.OP_FILL, b, off, ln, n, out)
    exp_a, want = fill_expect(a, off, ln)
    np.testing.assert_array_equal(out, want)
    np.testing.assert_array_equal(b, exp_a)
    ok = np.zeros(n, np.uint8)
    tcpck.host_batch_var_multi(ctxs[:nctx], tcpck.OP_VERIFY, b, off, ln, n, ok)
    assert ok.all()


def test_multi_errors_propagate(ctxs):
    """A shard's argument error comes back as the call's status."""
    import tcpck
    a = np.zeros(4096, np.uint8)
    out = np.zeros(8, np.uint16)
    with pytest.raises(tcpck.TcpckError):  # odd length
        tcpck.host_batch_fixed_multi(ctxs[:2], tcpck.OP_CHECKSUM, a, 101, 101, 8, out)
    off = np.arange(8, dtype=np.uint64) * 64
    ln = np.full(8, 20, np.uint32)
    with pytest.raises(tcpck.TcpckError):  # FILL of images < 30 B
        tcpck.host_batch_var_multi(ctxs[:2], tcpck.OP_FILL, a, off, ln, 8, out)


# ---- distinct devices (skipped on a one-GPU box; runs wherever >= 2 GPUs exist) ----

def _device_count():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.skipif(_device_count() < 2, reason="needs >= 2 GPUs (contexts on distinct devices)")
@pytest.mark.parametrize("length", [1492, 65536])
def test_multi_fixed_distinct_devices(built_lib, oracle_c, length):
    """tcpck_host_batch_fixed_multi with one context per GPU (one
    contiguous shard per device, no exchange): CHECKSUM against the oracle, then
    FILL -> VERIFY, and every call leaves the calling thread's current device as
    it found it (the ABI's DeviceGuard)."""
    import tcpck
    ndev = _device_count()
    cs = [tcpck.Context(d) for d in range(ndev)]
    try:
        for c in cs:
            c.set_chunk_bytes(8 << 20)
        count = 4096 if length == 1492 else 96
        rng = np.random.default_rng(length + ndev)
        a = rng.integers(0, 256, count * length, dtype=np.uint8)
        out = np.zeros(count, np.uint16)
        torch.cuda.set_device(0)
        tcpck.host_batch_fixed_multi(cs, tcpck.OP_CHECKSUM, a, length, length, count, out)
        assert torch.cuda.current_device() == 0
        np.testing.assert_array_equal(out, oracle_c.batch(a, stride=length, length=length, count=count))
        b = a.copy()
        tcpck.host_batch_fixed_multi(cs, tcpck.OP_FILL, b, length, length, count, out)
        exp_a, want = fill_expect(a, np.arange(count) * length, np.full(count, length))
        np.testing.assert_array_equal(out, want)
        np.testing.assert_array_equal(b, exp_a)
        ok = np.zeros(count, np.uint8)
        tcpck.host_batch_fixed_multi(cs, tcpck.OP_VERIFY, b, length, length, count, ok)
        assert ok.all()
    finally:
        for c in cs:
            c.close()


@pytest.mark.skipif(_device_count() < 2, reason="needs >= 2 GPUs (contexts on distinct devices)")
def test_device_batches_on_distinct_devices(built_lib, oracle_c):
    """Device-resident batches: one context and one C2-layout shard per GPU,
    each on its own device's current stream, results equal to the oracle."""
    import tcpck
    ndev = _device_count()
    L, per = 1492, 20000
    rng = np.random.default_rng(ndev)
    a = rng.integers(0, 256, ndev * per * L, dtype=np.uint8)
    exp = oracle_c.batch(a, stride=L, length=L, count=ndev * per)
    for d in range(ndev):
        with tcpck.Context(d) as c, torch.cuda.device(d):
            arena = torch.from_numpy(a[d * per * L:(d + 1) * per * L]).to(f"cuda:{d}")
            out = torch.empty(per, dtype=torch.int16, device=f"cuda:{d}")
            c.batch_fixed(tcpck.OP_CHECKSUM, arena, L, L, per, out, stream=torch.cuda.current_stream(d))
            torch.cuda.synchronize(d)
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), exp[d * per:(d + 1) * per])
