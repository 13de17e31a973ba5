"""CPU tests of the C-ABI library: it loads, exports every symbol include/tcpck.h
declares, and its host-side (single image) entry points match the golden
vectors.  No compute call here touches a GPU."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def declared_symbols(header="tcpck.h"):
    with open(os.path.join(ROOT, "include", header)) as f:
        text = f.read()
    decl = r"^(?:int|uint16_t|const char \*)\s*(tcpck_[a-z0-9_]+)\s*\("
    return sorted(set(re.findall(decl, text, flags=re.M)))


def test_header_and_binding_agree(built_lib):
    import tcpck
    assert declared_symbols() == sorted(tcpck.EXPORTS)
    assert declared_symbols("tcpck_tuning.h") == sorted(tcpck.TUNING_EXPORTS)
    assert declared_symbols("tcpck_probe.h") == sorted(tcpck.PROBE_EXPORTS)


def test_library_exports_every_declared_symbol(built_lib):
    for name in declared_symbols() + declared_symbols("tcpck_tuning.h"):
        assert hasattr(built_lib, name), name
    assert built_lib.tcpck_abi_version() == 1


def test_probe_symbols_only_in_probe_library(built_lib):
    """The measurement-only entry points (tcpck_probe.h) live in
    libtcpck_probe.so; libtcpck.so does not export them."""
    import ctypes
    import tcpck
    product = ctypes.CDLL(tcpck.LIB_PATH)
    probe = tcpck.probe_lib()
    for name in declared_symbols("tcpck_probe.h"):
        assert not hasattr(product, name), name
        assert hasattr(probe, name), name
    for name in declared_symbols() + declared_symbols("tcpck_tuning.h"):
        assert hasattr(probe, name), name


def _kernels(path):
    """{kernel name: {mangled template arguments}} of the code objects in a library."""
    import re
    with open(path, "rb") as f:
        blob = f.read()
    out = {}
    for k, args in re.findall(rb"_ZN5tcpck12_GLOBAL__N_1[0-9]+([a-z_]+_kernel)I([A-Za-z0-9_]*?)EEvN", blob):
        out.setdefault(k.decode(), set()).add(args.decode())
    return out


def test_product_library_holds_only_auto_kernels(built_lib):
    """libtcpck.so carries the kernels the AUTO policy can pick and nothing
    else (measurement-only code out of the product): rstream only
    as the policy's instantiation <U4, op, no stamps, no priority, flavour
    263 (7 + the first line only L2-kept, round 5), REF / RFC 1071>; no
    rvstream (a measured alternative, not AUTO's); no diag kernels; fewer
    instantiations than the probe build for every kernel that has
    measurement-only variants."""
    import tcpck
    prod, probe = _kernels(tcpck.LIB_PATH), _kernels(tcpck.PROBE_PATH)
    assert set(prod["rstream_kernel"]) == {f"Li4ELi{op}ELb0ELi0ELi263ELi{m}E" for op in range(3) for m in range(2)}
    assert "rvstream_kernel" not in prod and "rvstream_kernel" in probe
    blobs = [open(p, "rb").read() for p in (tcpck.LIB_PATH, tcpck.PROBE_PATH)]
    assert b"diag_stream_kernel" not in blobs[0] and b"diag_stream_kernel" in blobs[1]
    for k in ("rstream_kernel", "seg_kernel", "gstream_kernel", "sstream_kernel", "segment_kernel"):
        assert len(prod[k]) < len(probe[k]), k


def test_library_has_gfx950_code_object(built_lib):
    import tcpck
    with open(tcpck.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_host_checksum_matches_golden(golden, built_lib):
    import tcpck
    for c in golden.by_kind("checksum"):
        assert tcpck.checksum16(golden.image(c)) == c["expected"], c["name"]


def test_host_fill_matches_golden(golden, built_lib):
    import tcpck
    for c in golden.by_kind("fill"):
        img = golden.image(c)
        assert tcpck.fill16(img) == c["expected"]
        np.testing.assert_array_equal(img, golden.blob[c["fill_off"]:c["fill_off"] + c["len"]])


def test_host_rfc1071_mode(built_lib, oracle_c):
    import tcpck
    rng = np.random.default_rng(5)
    for n in (0, 2, 30, 32, 1492, 65536, 200000):
        img = rng.integers(0, 256, n, dtype=np.uint8)
        assert tcpck.checksum16(img, tcpck.MODE_RFC1071) == oracle_c.one(img, 1)
    ones = np.full(4096, 0xFF, np.uint8)
    assert tcpck.checksum16(ones, tcpck.MODE_RFC1071) == oracle_c.one(ones, 1)


def test_host_large_and_wrapping(built_lib, oracle_c):
    import tcpck
    ones = np.full(1 << 20, 0xFF, np.uint8)
    assert tcpck.checksum16(ones) == oracle_c.one(ones)
    rng = np.random.default_rng(9)
    for n in (6, 8, 10, 14, 262144 + 6, (1 << 18) - 2):
        img = rng.integers(0, 256, n, dtype=np.uint8)
        assert tcpck.checksum16(img) == oracle_c.one(img), n


def test_host_rejects_odd_and_null(built_lib):
    import tcpck
    with pytest.raises(tcpck.TcpckError) as e:
        tcpck.checksum16(np.zeros(59, np.uint8))
    assert e.value.status == tcpck.EINVAL
    with pytest.raises(tcpck.TcpckError):
        tcpck.fill16(np.zeros(28, np.uint8))  # no room for the checksum field


def test_fill_with_bad_mode_leaves_image_untouched(built_lib):
    """a rejected fill16 must not have zeroed bytes 28-29."""
    import tcpck
    img = np.arange(64, dtype=np.uint8)
    before = img.copy()
    with pytest.raises(tcpck.TcpckError) as e:
        tcpck.fill16(img, mode=7)
    assert e.value.status == tcpck.EINVAL
    np.testing.assert_array_equal(img, before)


@pytest.mark.parametrize("mode", [0, 1])
def test_incremental_update_matches_recompute(built_lib, oracle_c, mode):
    """Retransmit ACK rewrite (socket-internal.h:376-377) without a full pass."""
    import tcpck
    rng = np.random.default_rng(11 + mode)
    for _ in range(300):
        n = int(rng.integers(16, 400)) * 2
        img = rng.integers(0, 256, n, dtype=np.uint8)
        c0 = tcpck.fill16(img, mode)
        w = int(rng.integers(0, n // 2))
        if w == 14:  # the checksum field itself
            continue
        old = int(img[2 * w]) | int(img[2 * w + 1]) << 8
        new = int(rng.integers(0, 1 << 16))
        img[2 * w], img[2 * w + 1] = new & 0xFF, new >> 8
        c1 = tcpck.update16(c0, old, new, mode)
        img[28], img[29] = 0, 0
        assert c1 == oracle_c.one(img, mode)


def test_ctx_create_without_gpu_fails_cleanly(built_lib):
    import torch
    import tcpck
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(tcpck.TcpckError) as e:
        tcpck.Context(0)
    assert e.value.status in (tcpck.ENODEV,) or e.value.status <= tcpck.EHIP


def test_multi_ctx_rejects_bad_lists(built_lib):
    """tcpck_host_batch_*_multi validate the context list before any shard runs
    (no GPU needed): NULL list, zero contexts, a NULL entry."""
    import ctypes
    import tcpck
    L = tcpck.lib()
    img = np.zeros(1492 * 4, np.uint8)
    out = np.zeros(4, np.uint16)
    off = np.arange(4, dtype=np.uint64) * 1492
    ln = np.full(4, 1492, np.uint32)
    assert L.tcpck_host_batch_fixed_multi(None, 1, 0, 0, img.ctypes.data, 1492, 1492, 4, out.ctypes.data) == tcpck.EINVAL
    arr = (ctypes.c_void_p * 2)(None, None)
    p = ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p))
    assert L.tcpck_host_batch_fixed_multi(p, 0, 0, 0, img.ctypes.data, 1492, 1492, 4, out.ctypes.data) == tcpck.EINVAL
    assert L.tcpck_host_batch_fixed_multi(p, 2, 0, 0, img.ctypes.data, 1492, 1492, 4, out.ctypes.data) == tcpck.EINVAL
    assert L.tcpck_host_batch_var_multi(p, 2, 0, 0, img.ctypes.data, off.ctypes.data, ln.ctypes.data, 4,
                                        out.ctypes.data) == tcpck.EINVAL
