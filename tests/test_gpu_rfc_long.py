"""RFC 1071 mode with an image of 128 KiB or more behind an understated hint.

The streaming kernels' RFC 1071 form takes image sums as differences of an
exact u32 word prefix, which is exact only while an image holds fewer than
2^16 words.  AUTO picks those kernels from the caller's layout hint
(tcpck_layout.max_len < 128 KiB), and tcpck.h promises that a wrong hint never
changes results: a run holding a longer image must leave for the exact
per-image pass on the device.  Images here are all-0xFF (the word sum of a
300000-B image is 150000 x 0xFFFF, past 2^32) next to ordinary ones.
Oracle: oracle_rfc1071 (oracle/ref16.c, our own RFC 1071 restatement -- not
reference parity)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LONG = 300000


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    from conftest import RoutedContext
    c = RoutedContext(0)  # libtcpck.so; measurement-only variants on libtcpck_probe.so
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def batch(n, small, where, gap, seed):
    """n images of `small` bytes (random), the ones at `where` LONG bytes of 0xFF;
    `gap` bytes between images (0: packed)."""
    rng = np.random.default_rng(seed)
    ln = np.full(n, small, np.uint32)
    ln[list(where)] = LONG
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gap)
    total = int(off[-1] + ln[-1]) + 64
    a = rng.integers(0, 256, total, dtype=np.uint8)
    for k in where:
        a[int(off[k]):int(off[k]) + LONG] = 0xFF
    return a, off, ln


CASES = [  # (n, small image, long images at, gap between images)
    (5000, 1492, (17, 4999), 0),           # packed: vvstream (AUTO's RFC 1071 packed choice)
    (5000, 608, (0, 2500), 0),
    (4 << 20, 32, (3 << 20,), 0),          # runs of ~500 32-B images: the long one in a later round
    (5000, 1492, (17, 4999), 556),         # in order with gaps, SORTED: sstream
    (20000, 96, (19000,), 160),
]


@pytest.mark.parametrize("n,small,where,gap", CASES)
@pytest.mark.parametrize("op", [0, 1, 2])
def test_rfc_long_image_understated_hint(ctx, oracle_c, n, small, where, gap, op):
    import tcpck
    from oracle import ref16 as R
    a, off, ln = batch(n, small, where, gap, seed=n + small + op)
    hint = dict(total_bytes=int(ln.astype(np.int64).sum()), min_len=small, max_len=1492,  # understated
                packed=gap == 0, sorted=gap != 0)
    if op == tcpck.OP_FILL and gap:
        hint["sorted"] = False  # FILL on offset lists stays on seg: nothing to check there
    d = dev(a)
    out = torch.zeros(n, dtype=torch.uint8 if op == tcpck.OP_VERIFY else torch.int16, device="cuda")
    ctx.batch_var(op, d, dev(off), dev(ln), n, out, mode=tcpck.MODE_RFC1071, **hint)
    if op == tcpck.OP_FILL:
        exp_a = a.copy()
        idx = np.unique(np.concatenate([np.arange(0, n, max(1, n // 3000)), list(where), [n - 1]]))
        want = np.array([R.fill_np(exp_a[int(off[k]):int(off[k]) + int(ln[k])], 1) for k in idx], np.uint16)
        np.testing.assert_array_equal(host(out).view(np.uint16)[idx], want)
        got_a = host(d)
        for k in idx:
            o, l = int(off[k]), int(ln[k])
            np.testing.assert_array_equal(got_a[o:o + l], exp_a[o:o + l], err_msg=f"image {k}")
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        ctx.batch_var(tcpck.OP_VERIFY, d, dev(off), dev(ln), n, ok, mode=tcpck.MODE_RFC1071, **hint)
        assert bool(host(ok)[idx].all())
        return
    exp = oracle_c.batch(a, off, ln, mode=1, threads=8)
    got = host(out)
    if op == tcpck.OP_VERIFY:
        np.testing.assert_array_equal(got, (exp == 0).astype(np.uint8))
    else:
        np.testing.assert_array_equal(got.view(np.uint16), exp)
        assert all(got.view(np.uint16)[k] == exp[k] for k in where)


@pytest.mark.parametrize("kernel,gap", [("VVSTREAM", 0), ("SSTREAM", 0), ("SSTREAM", 556)])
@pytest.mark.parametrize("op", [0, 2])
def test_rfc_long_image_explicit_kernel(ctx, oracle_c, kernel, gap, op):
    """The streaming kernel named through tcpck_batch_var_ex with mode RFC 1071 on
    an offset list holding long images: same results as the oracle."""
    import tcpck
    a, off, ln = batch(4000, 1492, (5, 3999), gap, seed=7 + gap)
    n = ln.size
    out = torch.zeros(n, dtype=torch.uint8 if op == tcpck.OP_VERIFY else torch.int16, device="cuda")
    ctx.batch_var_ex(op, dev(a), dev(off), dev(ln), n, out, getattr(tcpck, f"KERNEL_{kernel}"),
                     4 if kernel == "VVSTREAM" else 0,  # the policy variants (libtcpck.so)
                     mode=tcpck.MODE_RFC1071, total_bytes=int(ln.astype(np.int64).sum()), min_len=1492,
                     max_len=1492, packed=gap == 0, sorted=True)
    exp = oracle_c.batch(a, off, ln, mode=1, threads=8)
    got = host(out)
    if op == tcpck.OP_VERIFY:
        np.testing.assert_array_equal(got, (exp == 0).astype(np.uint8))
    else:
        np.testing.assert_array_equal(got.view(np.uint16), exp)
