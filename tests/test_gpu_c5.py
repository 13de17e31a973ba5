"""BASELINE configs[4] (C5) at its sub-8-GPU shard sizes, on the HIP path.

C5 is 8M x 1492-B images split evenly into G contiguous shards (SURVEY.md
§8e, tcpck/shard.py).  At G = 1 / 2 / 4 a GPU holds 8M / 4M / 2M images =
12.5 / 6.3 / 3.1 GB, so AUTO's kernel for the layout (rstream) walks byte
offsets past 4, 8 and 12 GiB.  Reference anchor: the per-segment checksum
include/tcp-header.h:252-263, applied to independent segments.

* G = 1: CHECKSUM against the oracle on a sample that straddles the 4, 8 and
  12 GiB byte lines plus the batch end; the same launch through rstream's
  policy variant explicitly; FILL -> VERIFY over every image; single-byte
  corruption (including the bytes either side of each line) caught exactly
  where injected.
* G = 2, 4: every rank's shard generated on its own (first_index = the
  shard start, as bench.py and one process per GPU do) gives exactly the
  full batch's results for its index range -- all 8M results compared.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

COUNT, L = 8 << 20, 1492


@pytest.fixture(scope="module")
def ctx(built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    from conftest import RoutedContext
    c = RoutedContext(0)  # libtcpck.so; measurement-only variants on libtcpck_probe.so
    yield c
    c.close()


def host(t) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _synth(count, first_index):
    import tcpck
    a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, count, seed=42, first_index=first_index)
    return a


def _line_images(count):
    """Images holding the bytes either side of each 4 GiB multiple inside the batch."""
    edges = [(m << 32) // L for m in range(1, 4) if (m << 32) < count * L]
    return edges, np.unique(np.concatenate([np.arange(max(e - 40, 0), min(e + 40, count)) for e in edges]))


@pytest.fixture(scope="module")
def c5_full(ctx):
    """The whole 8M-image batch on one GPU (G = 1) and its CHECKSUM results."""
    import tcpck
    a = _synth(COUNT, 0)
    out = torch.empty(COUNT, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, COUNT, out)
    got = host(out).view(np.uint16).copy()
    yield a, got
    del a, out
    torch.cuda.empty_cache()


def test_c5_one_gpu_checksum_vs_oracle(ctx, oracle_c, c5_full):
    import tcpck
    a, got = c5_full
    edges, near = _line_images(COUNT)
    assert len(edges) == 2 and (3 << 32) > COUNT * L  # 12.5 GB: the 4 and 8 GiB lines (12 GiB is past the end)
    rng = np.random.default_rng(8)
    idx = np.unique(np.concatenate([rng.integers(0, COUNT, 20000), near, np.arange(COUNT - 70, COUNT),
                                    np.arange(0, 70)]))
    sample = host(a.view(COUNT, L)[torch.from_numpy(idx).cuda()]).reshape(-1)
    exp = oracle_c.batch(sample, stride=L, length=L, count=idx.size, threads=16)
    np.testing.assert_array_equal(got[idx], exp)
    # the layout's kernel named explicitly (rstream, the policy variant) gives every result identically
    out = torch.empty(COUNT, dtype=torch.int16, device="cuda")
    ctx.batch_fixed_ex(tcpck.OP_CHECKSUM, a, L, L, COUNT, out, tcpck.KERNEL_RSTREAM, 20)
    np.testing.assert_array_equal(host(out).view(np.uint16), got)


def test_c5_one_gpu_12gib_line(ctx, oracle_c):
    """A batch that crosses 12 GiB too: 9M images (13.4 GB), every result near the
    three lines against the oracle."""
    import tcpck
    count = 9 << 20
    a = _synth(count, 0)
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out)
    edges, near = _line_images(count)
    assert len(edges) == 3
    idx = np.unique(np.concatenate([near, np.arange(count - 70, count)]))
    sample = host(a.view(count, L)[torch.from_numpy(idx).cuda()]).reshape(-1)
    exp = oracle_c.batch(sample, stride=L, length=L, count=idx.size)
    np.testing.assert_array_equal(host(out).view(np.uint16)[idx], exp)
    del a, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world", [2, 4])
def test_c5_shards_equal_full_batch(ctx, c5_full, world):
    """Each rank's shard, generated alone from its first_index, checksums to the
    full batch's results over its whole range (4M / 2M images per shard)."""
    import tcpck
    from tcpck.shard import shard_range
    _, full = c5_full
    for rank in range(world):
        first, stop = shard_range(COUNT, world, rank)
        n = stop - first
        a = _synth(n, first)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, n, out)
        np.testing.assert_array_equal(host(out).view(np.uint16), full[first:stop], err_msg=f"rank {rank}/{world}")
        del a, out


def test_c5_one_gpu_fill_verify_corrupt(ctx, c5_full):
    """Send-side FILL over all 8M images, VERIFY all true, then single bytes
    flipped -- including the bytes at 4 GiB - 1, 4 GiB, 8 GiB - 1, 8 GiB and the
    batch's last byte -- are caught exactly in the images that hold them.
    (Runs last: it rewrites the shared arena.)"""
    import tcpck
    a, _ = c5_full
    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, COUNT, None)
    ok = torch.empty(COUNT, dtype=torch.uint8, device="cuda")
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, COUNT, ok)
    assert int(ok.sum(dtype=torch.int64).item()) == COUNT
    rng = np.random.default_rng(9)
    bad = np.unique(rng.integers(0, COUNT, 2000))
    pos = bad.astype(np.int64) * L + rng.integers(0, L, bad.size)
    keep = np.ones(bad.size, bool)
    lines = np.array([(1 << 32) - 1, 1 << 32, (2 << 32) - 1, 2 << 32, COUNT * L - 1], np.int64)
    for p in lines:  # drop random picks in the same images, then add the line bytes
        keep &= bad != p // L
    pos = np.concatenate([pos[keep], lines])
    a[torch.from_numpy(pos).cuda()] ^= 0x40
    ctx.batch_fixed(tcpck.OP_VERIFY, a, L, L, COUNT, ok)
    fails = np.nonzero(host(ok) == 0)[0]
    np.testing.assert_array_equal(fails, np.unique(pos // L))
