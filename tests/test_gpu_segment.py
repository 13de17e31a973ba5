"""GPU parity of the batched segmentation op (tcpck_batch_segment,
tcpck_segment.hip): a device-resident send stream cut into checksummed images,
against the reference's own data-segment send path (tests/golden/
segment_golden.*, made by tests/golden/gen_segment.cc from tcp-buffer.h,
tcp-header.h) and the oracle restatement (oracle.ref16.segment_np) on random
streams: every image byte, the zeroed slot tails, the checksums, both modes,
misaligned payload pointers, 2-B stream tails, sequence-number wrap, and a
1.5 GB stream at full size."""
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


def align16(x):
    return (x + 15) // 16 * 16


def run(ctx, payload_np, seg, tmpl, seq0, stride, mis=0, mode=0, param=None):
    buf = torch.zeros(payload_np.size + 64, dtype=torch.uint8, device="cuda")
    buf[mis:mis + payload_np.size] = dev(payload_np)
    n = (payload_np.size + seg - 1) // seg
    images = torch.full((n * stride + 256,), 0xA5, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    got_n = ctx.batch_segment(buf.data_ptr() + mis, payload_np.size, seg, tmpl, seq0, images, stride, out,
                              mode=mode, param=param)
    assert got_n == n
    imgs = host(images)
    assert (imgs[n * stride:] == 0xA5).all(), "wrote past the last slot"
    return imgs[:n * stride], host(out).view(np.uint16)


@pytest.mark.parametrize("pad", [0, 48, 1024])
def test_segment_golden(ctx, segment_golden, pad):
    """Byte-exact against the reference's own send path, every fixture stream."""
    for c in segment_golden.cases:
        stride = align16(32 + c["seg"]) + pad
        imgs, cs = run(ctx, segment_golden.payload(c), c["seg"], segment_golden.template(c), c["seq0"], stride)
        ref = segment_golden.images(c)
        off = 0
        for k, n in enumerate(c["lengths"]):
            np.testing.assert_array_equal(imgs[k * stride:k * stride + n], ref[off:off + n], err_msg=f"{c['name']} {k}")
            assert not imgs[k * stride + n:(k + 1) * stride].any(), f"{c['name']} slot tail {k}"
            off += n
        assert list(cs) == c["checksums"], c["name"]


PARAMS = [None, 0, 1, 2, 3, 4, 5, 6, 7, 0x17, 0x27, 8, 0 | (1 << 16), 0 | (3 << 16), 0 | (48 << 16), 2 | (8 << 16),
          4 | (128 << 16), 7 | (2 << 16), 7 | (600 << 16)]


@pytest.mark.parametrize("param", PARAMS)
@pytest.mark.parametrize("seg,payload_bytes", [(4, 2), (4, 1002), (16, 16 * 1000 + 6), (100, 99998), (1024, 5000),
                                               (1024, 1024 * 3000), (1448, 1448 * 777 + 2), (1460, 1460 * 2001 + 2),
                                               (1460, 1460 * 64), (9000, 9000 * 150 + 14), (65532, 65532 * 30 + 4)])
@pytest.mark.parametrize("mode", [0, 1])
def test_segment_random_vs_oracle(ctx, param, seg, payload_bytes, mode):
    from oracle import ref16 as R
    rng = np.random.default_rng(seg * 7 + payload_bytes + mode + (param or 0))
    payload = rng.integers(0, 256, payload_bytes, dtype=np.uint8)
    tmpl = rng.integers(0, 256, 32, dtype=np.uint8)
    seq0 = int(rng.integers(0, 1 << 32))
    for stride, mis in ((align16(32 + seg), 0), (align16(32 + seg) + 16, 4), (align16(32 + seg) + 512, 12)):
        imgs, cs = run(ctx, payload, seg, tmpl, seq0, stride, mis=mis, mode=mode, param=param)
        exp, lens, exp_cs = R.segment_np(payload, seg, tmpl, seq0, stride=stride, mode=mode)
        np.testing.assert_array_equal(cs, exp_cs)
        np.testing.assert_array_equal(imgs, exp)


def test_segment_all_ff_and_zero_streams(ctx):
    from oracle import ref16 as R
    tmpl = np.zeros(32, np.uint8)
    for fill in (0x00, 0xFF):
        payload = np.full(1460 * 5000 + 2, fill, np.uint8)
        imgs, cs = run(ctx, payload, 1460, tmpl, 0xFFFFFFF0, 1504)
        exp, _, exp_cs = R.segment_np(payload, 1460, tmpl, 0xFFFFFFF0, stride=1504)
        np.testing.assert_array_equal(cs, exp_cs)
        np.testing.assert_array_equal(imgs, exp)


def test_segment_full_size_verifies(ctx, oracle_c):
    """A 1.5 GB send stream cut into 1460-B segments (1M + 1 images in 1504-B
    slots): every image verifies on the device (socket-manager.h:182) and
    under the oracle, every field holds the returned checksum, and sampled
    images equal the restatement byte for byte."""
    import tcpck
    from oracle import ref16 as R
    seg, stride = 1460, 1504
    P = seg * (1 << 20) + 2
    payload = torch.empty(P, dtype=torch.uint8, device="cuda")
    n = (P + seg - 1) // seg
    # the stream: a fixed-stride synthetic batch read as flat bytes
    tcpck.synth_fixed(payload, 1492, 1492, P // 1492, seed=11)
    tmpl = np.arange(32, dtype=np.uint8)
    images = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.batch_segment(payload, P, seg, tmpl, 12345, images, stride, out)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    ln = torch.full((n,), 32 + seg, dtype=torch.int32, device="cuda")
    ln[-1] = 32 + 2
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.batch_var(tcpck.OP_VERIFY, images, off, ln, n, ok, sorted=True)
    assert bool(ok.all().item())
    imgs = host(images)
    cs = host(out).view(np.uint16)
    # the oracle over the device's images: every filled image checks to 0
    assert not oracle_c.batch(imgs, off.cpu().numpy().astype(np.uint64), ln.cpu().numpy().astype(np.uint32),
                              threads=8).any()
    # every stored field holds its own checksum (raw u16 at 28-29)
    fields = imgs.reshape(n, stride)[:, 28:30].copy().view("<u2")[:, 0]
    np.testing.assert_array_equal(fields, cs)
    pay = host(payload)
    for k in (0, 1, 777, n // 2, n - 2, n - 1):
        sub = pay[k * seg:min(P, (k + 1) * seg)]
        exp, _, exp_cs = R.segment_np(sub, seg, tmpl, (12345 + k * seg) & 0xFFFFFFFF, stride=stride)
        np.testing.assert_array_equal(imgs[k * stride:(k + 1) * stride], exp)
        assert cs[k] == exp_cs[0]


def test_segment_stream_beyond_4gib(ctx):
    """A 4.5 GB send stream (3M + 1 MSS segments, 4.7 GB of slots): offsets
    and image indices past 2^32 bytes.  Every image verifies on the device,
    and 256 sampled images across the stream -- the last ones included --
    equal the restatement byte for byte (copied back one by one)."""
    import tcpck
    from oracle import ref16 as R
    seg, stride = 1460, 1504
    n_full = 3 << 20
    P = seg * n_full + 2
    assert P > (1 << 32)
    payload = torch.empty(P, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(payload, 1492, 1492, P // 1492, seed=5)
    n = (P + seg - 1) // seg
    images = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    tmpl = np.arange(32, dtype=np.uint8)[::-1].copy()
    ctx.batch_segment(payload, P, seg, tmpl, 0xFFFFF000, images, stride, out)
    ok = torch.empty(n - 1, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, images, stride, 32 + seg, n - 1, ok)
    assert bool(ok.all().item())
    last = torch.empty(1, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, images[(n - 1) * stride:], stride, 32 + 2, 1, last)
    assert int(last.item()) == 1
    rng = np.random.default_rng(1)
    picks = np.concatenate([rng.choice(n, 250, replace=False), [0, n // 2, n - 3, n - 2, n - 1, (1 << 32) // seg]])
    cs = host(out).view(np.uint16)
    for k in picks:
        k = int(k)
        sub = host(payload[k * seg:min(P, (k + 1) * seg)])
        exp, _, exp_cs = R.segment_np(sub, seg, tmpl, (0xFFFFF000 + k * seg) & 0xFFFFFFFF, stride=stride)
        np.testing.assert_array_equal(host(images[k * stride:(k + 1) * stride]), exp, err_msg=str(k))
        assert cs[k] == exp_cs[0], k
    del payload, images


def test_segment_argument_errors(ctx):
    import tcpck
    p = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    im = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    h = np.zeros(32, np.uint8)
    bad = [dict(payload_bytes=1001, seg=1024, stride=1056),      # odd stream
           dict(payload_bytes=1000, seg=1022, stride=1056),      # seg % 4
           dict(payload_bytes=1000, seg=1024, stride=1064),      # stride % 16
           dict(payload_bytes=1000, seg=1024, stride=1040),      # stride < 32 + seg
           dict(payload_bytes=1000, seg=65536, stride=65568),    # seg > 65532
           dict(payload_bytes=1000, seg=0, stride=64)]
    for b in bad:
        with pytest.raises(tcpck.TcpckError):
            ctx.batch_segment(p, b["payload_bytes"], b["seg"], h, 0, im, b["stride"])
    with pytest.raises(tcpck.TcpckError):  # images not 16-B aligned
        ctx.batch_segment(p, 1000, 1024, h, 0, im.data_ptr() + 8, 1056)
    with pytest.raises(tcpck.TcpckError):  # payload not 4-B aligned
        ctx.batch_segment(p.data_ptr() + 2, 1000, 1024, h, 0, im, 1056)
    with pytest.raises(ValueError):
        ctx.batch_segment(p, 1000, 1024, np.zeros(31, np.uint8), 0, im, 1056)
    assert ctx.batch_segment(p, 0, 1024, h, 0, im, 1056) == 0  # empty stream: nothing to do
