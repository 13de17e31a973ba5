"""GPU parity of RECEIVE's combined form (round 4): where AUTO's VERIFY is the
slot stream and the header pass follows (MSS-sized rings and slots), the stream
sums each image's tail (bytes 128 ..) and the header pass sums the head (its
first line), combines both into the verdict and writes the host-order header
(tcpck_api.hip receive_combined, tcpck_header.hip header_combine_kernel).

Against the reference's receive path (ReceivePacket's verdict + TcpHeaderN2H,
include/socket-manager.h:181-184) restated by oracle.ref16: verdicts, every
header byte, the arena untouched -- around the 128-B head boundary, with runs
of short images (whose empty tails borrow the next tail's start), 2-B aligned
images, both modes, wrong SORTED hints, and past the context scratch's 8M
images (chunks)."""
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
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def check(ctx, a, off, ln, mode, mis=0, hdr_mis=0, hints=None, fixed=None):
    """RECEIVE into a header array; compare verdicts, headers and the arena."""
    from oracle import ref16 as R
    n = len(off)
    buf = dev(a)
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    hbuf = torch.full((n * 32 + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    kw = dict(mode=mode)
    if fixed:
        kw.update(stride=fixed[0], length=fixed[1])
    else:
        kw.update(offsets=dev(off.astype(np.uint64)), lengths=dev(ln.astype(np.uint32)), **(hints or {}))
    ctx.batch_receive(buf.data_ptr() + mis, n, ok, hbuf.data_ptr() + hdr_mis, **kw)
    v = a[mis:]
    exp_ok = (R.ref16_batch_np(v, off, ln, mode) == 0).astype(np.uint8)
    np.testing.assert_array_equal(host(ok), exp_ok)
    o = np.asarray(off, np.int64)
    hb = host(hbuf)
    np.testing.assert_array_equal(hb[hdr_mis:hdr_mis + 32 * n], v[o[:, None] + R.HEADER_PERM[None, :]].reshape(-1))
    np.testing.assert_array_equal(hb[:hdr_mis], np.full(hdr_mis, 0xEE, np.uint8))
    np.testing.assert_array_equal(host(buf), a)
    return exp_ok


def ring(rng, n, slot, lens, mode, mis=0, valid_every=3):
    """Images at mis + k * slot, every valid_every-th one FILLed (as sent)."""
    from oracle import ref16 as R
    ln = np.asarray(lens, np.int64)
    off = np.arange(n, dtype=np.int64) * slot
    a = rng.integers(0, 256, n * slot + 64, dtype=np.uint8)
    v = a[mis:]
    for k in range(0, n, valid_every):
        R.fill_np(v[off[k]:off[k] + ln[k]], mode)
    return a, off, ln


def hints_for(ln, sorted_=True):
    return dict(total_bytes=int(ln.sum()), min_len=int(ln.min()), max_len=int(ln.max()), sorted=sorted_)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("mis", [0, 2, 6, 16])
@pytest.mark.parametrize("hdr_mis", [0, 4])
def test_combined_ring_head_boundary(ctx, mode, mis, hdr_mis):
    """Lengths around the 128-B head (32 .. 260 B) mixed with MSS images so the
    ring's typical image is above 256 B (the combined form), including runs of
    short images, in 2048-B slots."""
    rng = np.random.default_rng(100 * mode + 10 * mis + hdr_mis)
    n, slot = 30000, 2048
    pick = np.asarray([32, 34, 96, 126, 128, 130, 132, 142, 144, 160, 254, 256, 258, 1492, 1492, 1492, 1492, 1460, 2000])
    ln = pick[rng.integers(0, pick.size, n)]
    ln[100:140] = 96     # a run of short images (empty tails borrow the next tail's start)
    ln[5000:5300] = 128  # ... exactly at the head size
    a, off, ln = ring(rng, n, slot, ln, mode, mis)
    exp_ok = check(ctx, a, off, ln, mode, mis, hdr_mis, hints_for(ln))
    assert exp_ok.sum() >= n // 3


@pytest.mark.parametrize("mode", [0, 1])
def test_combined_ring_tail_end_short(ctx, mode):
    """Every image of some runs short, the batch ending in short images: empty
    tails with no longer image after them in their run sit at their own end."""
    rng = np.random.default_rng(7 + mode)
    n, slot = 4096, 1536
    ln = np.where(rng.random(n) < 0.5, 1492, 64)
    ln[-300:] = 64
    ln[:200] = 100
    a, off, ln = ring(rng, n, slot, ln, mode, valid_every=2)
    check(ctx, a, off, ln, mode, 0, 0, hints_for(ln))


@pytest.mark.parametrize("mode", [0, 1])
def test_combined_wrong_sorted_hint(ctx, mode):
    """A SORTED hint that is wrong (the images shuffled): still exact (the
    stream's per-image fallback sums the tails)."""
    rng = np.random.default_rng(11 + mode)
    n, slot = 8192, 2048
    ln = np.asarray((96, 608, 1492))[rng.integers(0, 3, n)]
    a, off, ln = ring(rng, n, slot, ln, mode)
    perm = rng.permutation(n)
    check(ctx, a, off[perm], ln[perm], mode, 0, 0, hints_for(ln))


@pytest.mark.parametrize("stride,length", [(2048, 1492), (1536, 1492), (4096, 3000), (528, 258), (16384, 9000)])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("mis", [0, 2])
def test_combined_fixed_slots(ctx, stride, length, mode, mis):
    """Fixed slots on the slot stream (stride a multiple of 16, images > 256 B):
    the tail stream on the arena shifted by 128 B."""
    rng = np.random.default_rng(stride + length + mode + mis)
    n = max(1, min(20000, (48 << 20) // stride))
    a, off, ln = ring(rng, n, stride, np.full(n, length), mode, mis)
    check(ctx, a, off, ln, mode, mis, 0, fixed=(stride, length))


@pytest.mark.parametrize("n", [1, 2, 63, 65, 129])
def test_combined_small_counts(ctx, n):
    rng = np.random.default_rng(n)
    a, off, ln = ring(rng, n, 2048, rng.choice([130, 608, 1492], n), 0)
    check(ctx, a, off, ln, 0, 0, 0, hints_for(ln))
    a, off, ln = ring(rng, n, 2048, np.full(n, 1492), 1)
    check(ctx, a, off, ln, 1, 0, 0, fixed=(2048, 1492))


def test_combined_past_scratch(ctx, oracle_c):
    """More datagrams than the scratch's 8M results: the combined form runs in
    chunks (8M + 4099 images of 258-320 B in 320-B slots, 2.7 GB)."""
    import tcpck
    from oracle import ref16 as R
    n, slot = (8 << 20) + 4099, 320
    rng = np.random.default_rng(5)
    ln = (rng.integers(129, 161, n) * 2).astype(np.uint32)
    off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    a = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
    tcpck.synth_var(a, dev(off), dev(ln), int(ln.max()), n, seed=9)
    bad = np.arange(3, n, 7919, dtype=np.int64)
    a[torch.from_numpy(bad * slot + 200).cuda()] ^= 0x20  # inside the tails of some images
    a[torch.from_numpy(bad[::2] * slot + 40).cuda()] ^= 0x01  # inside the heads of others
    h = host(a)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    hdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.batch_receive(a, n, ok, hdr, offsets=dev(off), lengths=dev(ln), **hints_for(ln))
    exp = oracle_c.batch(h, off, ln, threads=16)
    np.testing.assert_array_equal(host(ok), (exp == 0).astype(np.uint8))
    pick = np.unique(np.concatenate([np.arange(0, n, 100003), bad[:50], [n - 1]]))
    o = off.astype(np.int64)[pick]
    np.testing.assert_array_equal(host(hdr).reshape(n, 32)[pick], h[o[:, None] + R.HEADER_PERM[None, :]])
