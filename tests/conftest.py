"""Test configuration: markers, import paths and shared fixtures.

`-m "not gpu"` runs the oracle-vs-golden, ABI/host-logic and multi-process
(gloo) tests on CPU; `-m gpu` runs the HIP parity tests through the C ABI.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tcp-stack_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libtcpck.so")


class Golden:
    """tests/golden/golden.{bin,json}: reference outputs from tests/golden/gen_golden.cc."""

    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
            meta = json.load(f)
        self.blob = np.fromfile(os.path.join(GOLDEN_DIR, meta["blob"]), dtype=np.uint8)
        assert self.blob.size == meta["blob_bytes"]
        self.cases = meta["cases"]

    def image(self, case, key="off"):
        o = case[key]
        return self.blob[o:o + case["len"]].copy()

    def by_kind(self, kind):
        return [c for c in self.cases if c["kind"] == kind]


@pytest.fixture(scope="session")
def golden():
    return Golden()


class SegmentGolden:
    """tests/golden/segment_golden.{bin,json}: the reference's data-segment send
    path (tcp-buffer.h:82-98 .. socket-manager.h:259-260) on known send streams,
    from tests/golden/gen_segment.cc."""

    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "segment_golden.json")) as f:
            meta = json.load(f)
        self.blob = np.fromfile(os.path.join(GOLDEN_DIR, meta["blob"]), dtype=np.uint8)
        assert self.blob.size == meta["blob_bytes"]
        self.cases = meta["cases"]

    def payload(self, c):
        return self.blob[c["payload_off"]:c["payload_off"] + c["payload_len"]].copy()

    def template(self, c):
        return self.blob[c["template_off"]:c["template_off"] + 32].copy()

    def images(self, c):
        """The reference's images, back to back."""
        return self.blob[c["images_off"]:c["images_off"] + sum(c["lengths"])].copy()


@pytest.fixture(scope="session")
def segment_golden():
    return SegmentGolden()


class ReceiveGolden:
    """tests/golden/receive_golden.{bin,json}: 96 wire images from the
    reference's send side (24 of them damaged) and the same arena after
    ReceivePacket's verdict + TcpHeaderN2H (socket-manager.h:181-184), with the
    host-order fields the accessors read, from tests/golden/gen_receive.cc."""

    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "receive_golden.json")) as f:
            meta = json.load(f)
        blob = np.fromfile(os.path.join(GOLDEN_DIR, meta["blob"]), dtype=np.uint8)
        assert blob.size == meta["blob_bytes"]
        n = meta["arena_bytes"]
        self.wire = blob[meta["wire_off"]:meta["wire_off"] + n].copy()
        self.host = blob[meta["host_off"]:meta["host_off"] + n].copy()
        self.offsets = np.asarray(meta["offsets"], np.uint64)
        self.lengths = np.asarray(meta["lengths"], np.uint32)
        self.ok = np.asarray(meta["ok"], np.uint8)
        self.damage = np.asarray(meta["damage"])
        self.fields = {k: np.asarray(v, np.uint64) for k, v in meta["fields"].items()}


@pytest.fixture(scope="session")
def receive_golden():
    return ReceiveGolden()


@pytest.fixture(scope="session")
def oracle_c():
    from oracle.ref16 import Ref16C
    return Ref16C(build=True)


@pytest.fixture(scope="session")
def built_lib():
    """libtcpck.so, built in-tree if missing (hipcc cross-compiles without a GPU)."""
    import tcpck
    if not os.path.exists(tcpck.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tcp-stack_amd"), "-j8"], check=True)
    return tcpck.lib()


# ---- the product library and the probe library -------------------------------
#
# libtcpck.so carries only the kernels the AUTO policy picks; its tuning entry
# points (batch_*_ex) accept those alone.  libtcpck_probe.so is the same
# sources with every measured variant.  Variant tests run each AUTO choice on
# libtcpck.so over their whole matrix, and each measurement-only variant once
# (one representative case) on libtcpck_probe.so.

class RoutedContext:
    """A libtcpck.so context that sends explicit-kernel calls the product
    library does not run to a libtcpck_probe.so context on the same device."""

    def __init__(self, device: int = 0):
        import tcpck
        self._tcpck = tcpck
        self.product = tcpck.Context(device)
        self.probe = tcpck.Context(device, probe=True)

    def _for(self, kernel, param, op=None):
        return self.product if self._tcpck.in_product(kernel, param, op) else self.probe

    def batch_fixed_ex(self, op, arena, stride, length, count, out, kernel, param=0, **kw):
        return self._for(kernel, param, op).batch_fixed_ex(op, arena, stride, length, count, out, kernel, param, **kw)

    def batch_var_ex(self, op, arena, offsets, lengths, count, out, kernel, param=0, **kw):
        return self._for(kernel, param, op).batch_var_ex(op, arena, offsets, lengths, count, out, kernel, param,
                                                         **kw)

    def batch_receive(self, *a, kernel=None, param=0, **kw):
        c = self.product if kernel is None else self._for(kernel, param & ~(1 << 30))
        return c.batch_receive(*a, kernel=kernel, param=param, **kw)

    def batch_segment(self, *a, param=None, **kw):
        c = self.product if param is None or self._tcpck.segment_in_product(param) else self.probe
        return c.batch_segment(*a, param=param, **kw)

    def __getattr__(self, name):
        return getattr(self.product, name)

    def close(self):
        self.product.close()
        self.probe.close()


def _variant_kernel(item):
    """(kernel, param) of a variant test item, or None when the item names no variant."""
    import tcpck
    cs = getattr(item, "callspec", None)
    if cs is None:
        return None
    p = cs.params
    name = item.originalname or item.name
    if "kernel" in p and ("param" in p or "variant" in p) and isinstance(p["kernel"], int):
        return p["kernel"], p.get("param", p.get("variant"))
    v = p.get("variant", p.get("param"))
    if not isinstance(v, int):
        return None
    if "segment" in item.module.__name__ and "param" in p:
        return ("segment", v)
    for key, k in (("rstream", tcpck.KERNEL_RSTREAM), ("vvstream", tcpck.KERNEL_VVSTREAM),
                   ("gstream", tcpck.KERNEL_GSTREAM), ("sstream", tcpck.KERNEL_SSTREAM),
                   ("fused_hdr", tcpck.KERNEL_SSTREAM)):
        if key in name or key in item.module.__name__:
            return k, v
    return None


def pytest_collection_modifyitems(config, items):
    """Measurement-only variants (libtcpck_probe.so) keep ONE representative
    case per test function -- the middle one of their matrix; AUTO's variants
    (libtcpck.so) keep every case.  TCPCK_ALL_VARIANTS=1 keeps every case of
    every variant (a full sweep of the probe library)."""
    import tcpck
    if os.environ.get("TCPCK_ALL_VARIANTS") == "1":
        return
    groups, keep, drop = {}, [], []
    for it in items:
        kv = _variant_kernel(it)
        if kv is None:
            keep.append(it)
            continue
        kernel, v = kv
        op = tcpck.OP_CHECKSUM if kernel == tcpck.KERNEL_GSTREAM and "fill" not in it.name else None
        prod = tcpck.segment_in_product(v) if kernel == "segment" else tcpck.in_product(kernel, v & ~(1 << 30), op)
        if prod:
            keep.append(it)
        else:
            groups.setdefault((it.module.__name__, it.originalname, kernel, v), []).append(it)
    chosen = {id(g[len(g) // 2]) for g in groups.values()}
    grouped = {id(x) for g in groups.values() for x in g}
    for it in items:
        if id(it) in chosen:
            keep.append(it)
        elif id(it) in grouped:
            drop.append(it)
    if drop:
        config.hook.pytest_deselected(items=drop)
        order = {id(it): i for i, it in enumerate(items)}
        items[:] = sorted(keep, key=lambda it: order[id(it)])
