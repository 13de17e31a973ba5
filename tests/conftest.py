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
