"""N>1 path on CPU: world_size-2 gloo process groups.

The multi-GPU design has no data-path collective: each rank generates and
checksums its own contiguous shard (tcpck.shard), and only the timing is
reduced (max over ranks).  These tests run that exact flow with the oracle in
place of the GPU kernel and check that the shards' results, concatenated by
index, equal the checksums of the whole batch -- for the fixed-stride strong
split (C5), the byte-balanced split of a mixed batch (C3), and the weak
per-rank batches bench.py uses (first_index = rank * count).
"""
import os
import socket

import numpy as np
import pytest

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.ref16 import ref16_batch_np
from synth_np import arena_fixed, image, mixed_layout
from tcpck.shard import gather_ranks, max_over_ranks, shard_by_bytes, shard_range

WORLD = 2


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        # C5-style strong split of one fixed-stride batch
        count, L = 37, 96
        a, b = shard_range(count, world, rank)
        arena = arena_fixed(42, b - a, L, L, first_index=a)
        res["fixed"] = ref16_batch_np(arena, np.arange(b - a) * L, np.full(b - a, L))
        # C3-style byte-balanced split of a mixed packed batch
        off, ln, total = mixed_layout(53, seed=5)
        a, b = shard_by_bytes(ln, world, rank)
        imgs = [image(42, k, int(ln[k])) for k in range(a, b)]
        shard = np.concatenate(imgs) if imgs else np.zeros(0, np.uint8)
        loff = np.concatenate([[0], np.cumsum(ln[a:b].astype(np.int64))[:-1]]) if b > a else np.zeros(0, np.int64)
        res["mixed"] = ref16_batch_np(shard, loff, ln[a:b])
        res["mixed_bytes"] = int(ln[a:b].astype(np.int64).sum())
        # weak: each rank its own batch of the same size, first_index = rank * count
        wc = 11
        warena = arena_fixed(42, wc, 608, 608, first_index=rank * wc)
        res["weak"] = ref16_batch_np(warena, np.arange(wc) * 608, np.full(wc, 608))
        # timing reduction: the job's time is the slowest rank's
        res["tmax"] = max_over_ranks(1.0 + rank)
        res["all"] = gather_ranks(0.25 * (rank + 1))  # per-GPU kernel times for per-GPU roofline fractions
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        if rank == 0:
            q.put(gathered)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def gathered():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_fixed_strong_split(gathered):
    whole = ref16_batch_np(arena_fixed(42, 37, 96, 96), np.arange(37) * 96, np.full(37, 96))
    np.testing.assert_array_equal(np.concatenate([g["fixed"] for g in gathered]), whole)


def test_mixed_byte_balanced_split(gathered):
    off, ln, total = mixed_layout(53, seed=5)
    arena = np.zeros(total, np.uint8)
    for k in range(53):
        arena[int(off[k]):int(off[k]) + int(ln[k])] = image(42, k, int(ln[k]))
    whole = ref16_batch_np(arena, off.astype(np.int64), ln)
    np.testing.assert_array_equal(np.concatenate([g["mixed"] for g in gathered]), whole)
    b = [g["mixed_bytes"] for g in gathered]
    assert abs(b[0] - b[1]) <= int(ln.max()), b


def test_weak_batches(gathered):
    for r, g in enumerate(gathered):
        a = arena_fixed(42, 11, 608, 608, first_index=r * 11)
        np.testing.assert_array_equal(g["weak"], ref16_batch_np(a, np.arange(11) * 608, np.full(11, 608)))
    assert not np.array_equal(gathered[0]["weak"], gathered[1]["weak"])


def test_max_over_ranks(gathered):
    assert [g["tmax"] for g in gathered] == [2.0, 2.0]


def test_gather_ranks(gathered):
    assert [g["all"] for g in gathered] == [[0.25, 0.5], [0.25, 0.5]]
    assert gather_ranks(3.0) == [3.0]  # no process group in this process


@pytest.mark.parametrize("count,world", [(0, 3), (1, 2), (7, 8), (8 << 20, 8), (1000003, 7)])
def test_shard_range_partitions(count, world):
    ranges = [shard_range(count, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == count
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    sizes = [b - a for a, b in ranges]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_by_bytes_partitions(world):
    _, ln, _ = mixed_layout(10007, seed=world)
    ranges = [shard_by_bytes(ln, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == ln.size
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    per = [int(ln[a:b].astype(np.int64).sum()) for a, b in ranges]
    assert max(per) - min(per) <= 2 * int(ln.max())
    with pytest.raises(ValueError):
        shard_by_bytes(ln, world, world)
