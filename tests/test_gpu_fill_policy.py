"""AUTO FILL on packed fixed images around round 4's policy edges: vvstream's
deferred form for 320 B - 1 KiB, gstream up to 256 B, rstream's deferred form
from 1 KiB (tcpck_api.hip pick_fixed / run_fixed_impl; measurements in
profiles/r04/fill_policy_sweep.log).

Every arena byte and result against the oracle's FILL (socket-manager.cc:9-10:
Checksum() = 0, then CalculateChecksum, include/tcp-header.h:252-263), with a
results buffer and without one (the context's scratch), misaligned arenas, both
modes, guard bytes around the arena untouched; and the kernels AUTO launched
at the band's edges (torch.profiler)."""
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


def expected_fill(a, length, count, mode):
    from oracle import ref16 as R
    exp = a.copy()
    v = exp[:count * length].reshape(count, length)
    v[:, 28:30] = 0
    off = np.arange(count, dtype=np.int64) * length
    want = R.ref16_batch_np(exp, off, np.full(count, length, np.int64), mode).astype(np.uint16)
    v[:, 28:30] = want.view(np.uint8).reshape(count, 2)
    return exp, want


@pytest.mark.parametrize("length", [254, 256, 300, 318, 320, 322, 384, 448, 450, 510, 512, 514, 640, 768, 1000,
                                    1022, 1024, 1026])
@pytest.mark.parametrize("mis", [0, 2, 6, 16])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("with_out", [True, False])
def test_auto_fill_policy_band(ctx, length, mis, mode, with_out):
    import tcpck
    rng = np.random.default_rng(length * 100 + mis * 4 + mode * 2 + with_out)
    pad = 64
    count = 3000 + (length % 97)
    a = rng.integers(0, 256, pad + mis + count * length + pad, dtype=np.uint8)
    buf = torch.from_numpy(a).cuda()
    out = torch.full((count,), 0x5A5A, dtype=torch.int16, device="cuda") if with_out else None
    ctx.batch_fixed(tcpck.OP_FILL, buf.data_ptr() + pad + mis, length, length, count, out, mode=mode)
    torch.cuda.synchronize()
    exp, want = expected_fill(a[pad + mis:], length, count, mode)
    got = buf.cpu().numpy()
    if with_out:
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), want)
    np.testing.assert_array_equal(got[:pad + mis], a[:pad + mis])
    np.testing.assert_array_equal(got[pad + mis:], exp)


def _kernel_names(fn):
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if "kernel" in e.name}
    return names or None


@pytest.mark.parametrize("length,stream_kernel,field_pass", [
    (256, "gstream_kernel", False),
    (320, "vvstream_kernel", True),
    (512, "vvstream_kernel", True),
    (1022, "vvstream_kernel", True),
    (1024, "rstream_kernel", True),
    (1492, "rstream_kernel", True),
])
def test_auto_fill_policy_kernels(ctx, length, stream_kernel, field_pass):
    """The kernels AUTO's FILL launches at the band's edges: the stream named,
    then (deferred forms) the write-through field pass."""
    import tcpck
    count = 20000
    a = torch.zeros(count * length, dtype=torch.uint8, device="cuda")
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    names = _kernel_names(lambda: ctx.batch_fixed(tcpck.OP_FILL, a, length, length, count, out))
    if names is None:
        pytest.skip("torch.profiler records no device kernels on this box")
    assert any(stream_kernel in k for k in names), names
    assert any("patch_fields_kernel" in k for k in names) == field_pass, names
