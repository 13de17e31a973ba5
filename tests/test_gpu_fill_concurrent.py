"""GPU parity: FILL without a results buffer from concurrent callers.

The reference inserts checksums from at least three threads at once -- the
timer worker under a socket mutex (include/socket-manager.h:255-260), the
app/reaction threads through SendPacket (src/socket-manager.cc:6-11) and the
receive thread (src/network-service.cc:55-56) -- each on its own packet.  The
batched equivalent is several host threads, each on its own stream and arena,
calling OP_FILL with out=None at once: AUTO's two-pass forms then write their
results into the context's scratch slots (tcpck.h), and two FILLs sharing a
slot without ordering would store each other's checksums.  Every arena is
compared byte-exact with the reference's insert (oracle/ref16.c restating
include/tcp-header.h:252-263, pinned by tests/golden).

Also: which out-less FILLs take a slot at all (only the forms
that read the results back), and that a FILL captured into a HIP graph takes
none and replays byte-exact.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_gpu_full_paths import expected_fill  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(scope="module", params=[False, True], ids=["libtcpck", "probe"])
def any_ctx(request, built_lib):
    import tcpck
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = tcpck.Context(0, probe=request.param)
    yield c
    c.close()


def _c2_arena(count, seed, oracle_c):
    import tcpck
    L = 1492
    a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
    tcpck.synth_fixed(a, L, L, count, seed=seed)
    want = expected_fill(host(a), np.arange(count, dtype=np.int64) * L, np.full(count, L), oracle_c)
    return a, want


def _c3_arena(count, seed, oracle_c):
    import tcpck
    import synth_np
    off, ln, total = synth_np.mixed_layout(count, seed=seed)
    a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_off, d_ln = dev(off), dev(ln)
    tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=seed)
    want = expected_fill(host(a), off, ln, oracle_c)
    hints = dict(total_bytes=int(ln.astype(np.int64).sum()), min_len=int(ln.min()), max_len=int(ln.max()),
                 packed=True)
    return a, want, d_off, d_ln, hints


@pytest.mark.parametrize("layout", ["c2", "c3"])
def test_fill_noout_four_threads_four_streams(any_ctx, oracle_c, layout):
    """4 host threads, each on its own stream and arena, 20 out-less FILLs each
    at once (FILL is idempotent: the field is zeroed before the sum), C2's
    fixed layout or C3's packed mix: every arena byte-exact."""
    import tcpck
    n_thr, reps = 4, 20
    jobs = []
    for t in range(n_thr):
        if layout == "c2":
            a, want = _c2_arena(1 << 17, 60 + t, oracle_c)
            jobs.append((a, want, None))
        else:
            a, want, d_off, d_ln, hints = _c3_arena(1 << 19, 70 + t, oracle_c)
            jobs.append((a, want, (d_off, d_ln, hints)))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(n_thr)]
    barrier = threading.Barrier(n_thr)
    errors = []

    def worker(i):
        try:
            a, _, var = jobs[i]
            s = streams[i]
            barrier.wait()
            for _ in range(reps):
                if var is None:
                    any_ctx.batch_fixed(tcpck.OP_FILL, a, 1492, 1492, a.numel() // 1492, None, stream=s)
                else:
                    d_off, d_ln, hints = var
                    any_ctx.batch_var(tcpck.OP_FILL, a, d_off, d_ln, d_off.numel(), None, stream=s, **hints)
            s.synchronize()
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n_thr)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for a, want, _ in jobs:
        np.testing.assert_array_equal(host(a), want)


def test_scratch_taken_only_by_forms_that_read_results(built_lib, oracle_c):
    """A fresh probe context: a 128-B out-less FILL (gstream, in-stream fields)
    and a 96-B one (vvstream in-stream) allocate no slot; C2's 1492-B
    out-less FILL (rstream's deferred fields) allocates the slots and uses one;
    the bytes are the reference's insert each time."""
    import tcpck
    c = tcpck.Context(0, probe=True)
    try:
        for L in (128, 96):
            count = 50000
            a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
            tcpck.synth_fixed(a, L, L, count, seed=L)
            want = expected_fill(host(a), np.arange(count, dtype=np.int64) * L, np.full(count, L), oracle_c)
            c.batch_fixed(tcpck.OP_FILL, a, L, L, count, None)
            np.testing.assert_array_equal(host(a), want)
            assert c.scratch_state() == (0, 0), L
        a, want = _c2_arena(1 << 16, 81, oracle_c)
        c.batch_fixed(tcpck.OP_FILL, a, 1492, 1492, 1 << 16, None)
        np.testing.assert_array_equal(host(a), want)
        alloc, used = c.scratch_state()
        assert alloc == 4 and bin(used).count("1") == 1
    finally:
        c.close()


def test_fill_noout_under_graph_capture(built_lib, oracle_c):
    """An out-less C2 FILL captured into a HIP graph (torch.cuda.graph) takes
    no scratch slot (its in-stream form runs instead) and the replayed graph
    stores the reference's fields."""
    import tcpck
    c = tcpck.Context(0, probe=True)
    try:
        count, L = 1 << 16, 1492
        a, want = _c2_arena(count, 82, oracle_c)
        before = c.scratch_state()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                c.batch_fixed(tcpck.OP_FILL, a, L, L, count, None, stream=torch.cuda.current_stream())
        assert c.scratch_state() == before
        tcpck.synth_fixed(a, L, L, count, seed=82)  # the capture ran nothing: restore the images anyway
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(host(a), want)
        assert c.scratch_state() == before
    finally:
        c.close()
