"""Drop-in C++ header (include/tcp_stack/tcp-header.h, packet-batch.h).

Compiles tests/cpp/drop_in_test.cc against the headers and libtcpck.so and
checks it against the reference's golden vectors (tests/golden, generated from
/root/reference/include/tcp-header.h by tests/golden/gen_golden.cc) and the
structured-header known answer (0x4ba4).  The CPU tests use
only the host single-image path (tcpck_checksum16); the batch test runs
PacketBatch on the GPU through tcpck_host_batch_var.
"""
import os
import subprocess

import pytest

from conftest import ROOT

BUILD = os.path.join(ROOT, "tests", "cpp", "build")
SRC = os.path.join(ROOT, "tests", "cpp", "drop_in_test.cc")
LIBDIR = os.path.join(ROOT, "tcp-stack_amd")


def build(variant: str) -> str:
    """variant: 'asan' (host sanitizers, CPU tests) or 'opt'."""
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, f"drop_in_test_{variant}")
    deps = [SRC] + [os.path.join(ROOT, "include", "tcp_stack", f) for f in ("tcp-header.h", "packet-batch.h")]
    if os.path.exists(exe) and all(os.path.getmtime(exe) >= os.path.getmtime(d) for d in deps):
        return exe
    tmp = f"{exe}.{os.getpid()}.tmp"
    flags = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"] if variant == "asan" else ["-O2"]
    cmd = (["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror"] + flags +
           ["-I", os.path.join(ROOT, "include"), SRC, "-o", tmp, "-L", LIBDIR, "-ltcpck",
            f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath-link,/opt/rocm/lib"])
    subprocess.run(cmd, check=True)
    os.replace(tmp, exe)  # atomic: a parallel test process never runs a half-written binary
    return exe


@pytest.fixture(scope="module")
def exe(built_lib):
    return build("asan")


def run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout.splitlines()


def test_golden_vectors(exe, golden, tmp_path):
    manifest = tmp_path / "manifest.txt"
    manifest.write_text("".join(f"{c['kind']} {c['off']} {c['len']}\n" for c in golden.cases))
    blob = os.path.join(ROOT, "tests", "golden", "golden.bin")
    lines = run(exe, "golden", blob, manifest)
    assert len(lines) == len(golden.cases)
    for c, line in zip(golden.cases, lines):
        vals = [int(v) for v in line.split()]
        if c["kind"] == "fill":
            assert vals == [c["expected"], 0], c["name"]
        else:
            assert vals[0] == c["expected"], c["name"]


def test_layout_and_known_answer(exe, golden):
    out = dict(line.split(" ", 1) for line in run(exe, "layout"))
    assert out["text"] == "Ack Syn 43981->10 S287454020 A1432778632 L4660"
    assert out["size"] == "32"
    img = bytes(int(b, 16) for b in out["bytes"].split())
    ref = [c for c in golden.cases if c["name"] == "struct_hdr/32" and c["kind"] == "checksum"][0]
    assert img == bytes(golden.image(ref)), "header bytes differ from the reference's struct_hdr image"
    assert int(out["checksum"]) == 0x4BA4
    assert out["reverify"] == "0"
    inc, full = out["update"].split()
    assert inc == full
    assert out["n2h"] == "7f000001 11223344 1024 1234"
    assert [out[f] for f in ("urg", "ack", "psh", "rst", "syn", "fin", "cleared")] == \
        ["04", "08", "10", "20", "40", "80", "00"]
    assert out["payload"] == "38 1 6"
    odd_sum, odd_verify = map(int, out["odd"].split())
    assert odd_verify == 0
    # odd rule: last byte is the low byte of a zero-padded word
    from oracle.ref16 import ref16_np
    import numpy as np
    img = bytearray(32) + bytes([9, 8, 7, 6, 5]) + b"\0"
    assert odd_sum == ref16_np(np.frombuffer(bytes(img), np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("ctxs", [1, 3])
def test_packet_batch_gpu(built_lib, ctxs):
    """PacketBatch over one context, or over three (tcpck_host_batch_var_multi;
    on a one-GPU box all on device 0): checksums, send-path fill and
    receive-path verdicts equal the per-packet reference calls."""
    exe = build("opt")
    lines = run(exe, "batch", 20000, 7, ctxs)
    assert lines[-1].endswith("mismatches=0"), lines
    assert "gpu_images=0" not in lines[-1]


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes,window", [(5000, 1024), (3 * 1460 + 2, 1460), (2 * 65532 + 8, 65532),
                                           (1_000_000, 1448), (40, 4), (2, 1024), (9000 * 40 + 6, 9000)])
def test_segment_cpp_gpu(built_lib, nbytes, window):
    """tcpck_batch_segment from C++, with the header template built through the
    drop-in exactly as INTEGRATION.md shows, against the per-packet send path
    (MakeTcpPacket, Estab's fields, TcpHeaderH2N, CalculateChecksum) built with
    the same drop-in: every image byte, checksum and zeroed slot tail."""
    exe = build("opt")
    lines = run(exe, "segment", nbytes, window, 11)
    assert lines[-1].endswith("mismatches=0"), lines


@pytest.mark.gpu
@pytest.mark.parametrize("n,slot", [(5000, 2048), (20000, 1536), (300, 9216), (1, 64), (4000, 48)])
def test_receive_cpp_gpu(built_lib, n, slot):
    """tcpck_batch_receive from C++ on a ring of datagram slots (INTEGRATION.md
    section 2), against ReceivePacket's front half per packet through the
    drop-in (MakeNetPacket, CalculateChecksum == 0, TcpHeaderN2H): verdicts,
    the header array, the ring untouched by it, then the in-place form."""
    exe = build("opt")
    lines = run(exe, "receive", n, slot, 5)
    assert lines[-1].endswith("mismatches=0"), lines


def _loopback_c1(n):
    import json
    exe = os.path.join(LIBDIR, "bin", "loopback_c1")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", LIBDIR], check=True)
    r = subprocess.run([exe, str(n), "1460"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["received"] == d["verified"] == n
    assert d["image_bytes"] == 1492
    return d


def test_loopback_c1(built_lib):
    """Config C1: segments over UDP loopback, filled and verified through the drop-in
    (socket-manager.cc:9-10 send insert, network-service.cc:49-56 receive buffer,
    socket-manager.h:182 verify)."""
    _loopback_c1(3000)


@pytest.mark.gpu
def test_loopback_c1_gpu_box(built_lib):
    """C1 again inside the `-m gpu` run, so the driver's GPU-box record holds it:
    the same prebuilt binary (host CPU only: one segment never goes to the GPU)
    with verified == received over 20000 segments."""
    d = _loopback_c1(20000)
    assert d["us_per_segment"] > 0


def _recv_burst(args, gpu):
    import json
    exe = os.path.join(LIBDIR, "bin", "recv_burst")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", LIBDIR], check=True)
    r = subprocess.run([exe] + [str(a) for a in args] + ([] if gpu else ["--cpu-only"]),
                       capture_output=True, text=True, timeout=120)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, (r.stderr, d)
    assert d["lost"] == 0 and d["truncated"] == 0 and d["mismatches"] == 0 and d["flagged_wrong"] == 0
    assert d["flagged"] == d["expected_flagged"]
    return d


@pytest.mark.parametrize("segments,payload,batch,every", [(20000, 1460, 4096, 97), (3000, 14, 700, 5),
                                                           (2000, 1461, 512, 11), (1000, 576, 1000, 0)])
def test_recv_burst_cpu(built_lib, segments, payload, batch, every):
    """SURVEY §8f rank 2 plumbing on CPU: recvmmsg bursts into an arena, verdicts
    per packet through the drop-in CalculateChecksum, corrupted segments flagged."""
    d = _recv_burst([segments, payload, batch, every], gpu=False)
    assert d["batches"] == -(-segments // batch)
    assert d["odd"] == (segments if payload % 2 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("segments,payload,batch,every", [(100000, 1460, 32768, 97), (20000, 64, 8192, 3),
                                                           (4000, 1461, 1024, 13)])
def test_recv_burst_gpu(built_lib, segments, payload, batch, every):
    """One tcpck_host_batch_var(VERIFY) per batch of received datagrams; every GPU
    verdict equals CalculateChecksum on the same bytes (odd lengths stay on the CPU)."""
    d = _recv_burst([segments, payload, batch, every], gpu=True)
    assert d["gpu"] is True and d["batches"] == -(-segments // batch)


@pytest.mark.skipif(not os.path.exists("/root/reference/src/socket-manager.cc"),
                    reason="the reference checkout exists only in the build container")
def test_reference_stack_compiles_against_drop_in(built_lib):
    """The reference's own translation units that use tcp-header.h compile
    unchanged with tcp-header.h resolved to include/tcp_stack/tcp-header.h, and
    link against libtcpck.so with nothing left undefined but TimeoutQueue::Worker
    (src/timeout-queue.cc, which g++ 11 rejects on the reference header too).
    CalculateChecksum at socket-manager.cc:10 / socket-manager.h:182,260 now
    calls tcpck_checksum16 (oracle/Makefile `dropin`)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "dropin"], check=True)
    d = os.path.join(ROOT, "oracle", "_ref", "dropin")
    unresolved = open(os.path.join(d, "unresolved.txt")).read().split("\n")
    assert [u for u in unresolved if u] == ["undefined reference to `TimeoutQueue::Worker()'"]
    assert open(os.path.join(d, "uses_tcpck.txt")).read().strip() == "1"
