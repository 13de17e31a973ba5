"""GPU parity of the side-buffer FILL probe forms (rstream 33 / 34 + the side
copy, libtcpck_probe.so; round 6): the arena and the
results must be the reference's insert (socket-manager.cc:9-10: field zeroed,
CalculateChecksum of include/tcp-header.h:252-263, stored raw), checked against
the oracle -- including an arena that starts 2 bytes past a 64-B boundary, so
that the first image's field block begins before the arena (its field alone is
stored), the shortest stride the form takes (128 B) and strides that are not
multiples of 64."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_gpu_full_paths import expected_fill  # noqa: E402


@pytest.fixture(scope="module")
def pctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = tcpck.Context(0, probe=True)
    yield c
    c.close()


@pytest.mark.parametrize("variant", [33, 33 | 0x100, 34, 34 | 0x100], ids=["33", "33nt", "34", "34nt"])
@pytest.mark.parametrize("L,count,shift", [(1492, 200_003, 0), (1492, 70_001, 2), (128, 300_000, 0),
                                           (130, 99_999, 34), (4096, 20_000, 0), (610, 55_555, 62)])
def test_side_fill(pctx, oracle_c, variant, L, count, shift):
    import tcpck
    buf = torch.empty(count * L + 128, dtype=torch.uint8, device="cuda")
    base = (-buf.data_ptr()) % 64 + shift  # the arena starts `shift` bytes past a 64-B boundary
    a = buf[base:base + count * L]
    tcpck.synth_fixed(a, L, L, count, seed=L + shift)
    torch.cuda.synchronize()
    before = buf.cpu().numpy()
    want = expected_fill(a.cpu().numpy(), np.arange(count, dtype=np.int64) * L, np.full(count, L), oracle_c)
    out = torch.full((count,), -1, dtype=torch.int16, device="cuda")
    pctx.batch_fixed_ex(tcpck.OP_FILL, a, L, L, count, out, tcpck.KERNEL_RSTREAM, variant)
    torch.cuda.synchronize()
    after = buf.cpu().numpy()
    np.testing.assert_array_equal(after[base:base + count * L], want)
    # nothing outside the arena changed
    np.testing.assert_array_equal(after[:base], before[:base])
    np.testing.assert_array_equal(after[base + count * L:], before[base + count * L:])
    f = np.arange(count, dtype=np.int64) * L + 28
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16),
                                  want[f].astype(np.uint16) | (want[f + 1].astype(np.uint16) << 8))
