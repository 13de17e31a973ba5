#!/usr/bin/env python3
"""bench.py -- device-resident batched TCP checksum on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|...]

A step = one pass of the hot path (one tcpck_batch_* CHECKSUM launch) over one
batch of synthetic segments already resident in HBM; consecutive steps take
--arenas (2) identical batches in turn, so no step reads lines the previous
step left in the 256-MB Infinity Cache.  Default workload (N=1)
is BASELINE.json configs[1] (C2): 1,048,576 segments with a 1460-B Ethernet-MSS
payload = 1492-B checksummed images (32-B pseudo+TCP header + payload,
SURVEY.md fact 3), fixed stride.  With N>1 GPUs (one process per GPU via
torch.distributed.run) every rank checksums its own 1M-image shard
(first_index = rank * count, shard-reproducible generator), no data-path
collective: weak scaling, so SCALE's N=1 line is BENCH's line.  Rank 0 prints
ONE JSON line with the driver's fields plus:

  roofline      dominant kernel vs the HBM-read roof (8.0 TB/s): achieved =
                algorithmic bytes per launch (sum of image bytes + 2 B written
                per image) / average launch time (HIP events on the launch
                stream around the K launches, / K); traffic = PMC HBM bytes
                per launch from the committed rocprofv3 passes
                (profiles/pmc_summary.json) when they were captured on the
                very libtcpck.so loaded (sha256 stamp), else null with the
                reason in traffic_source
  c3, c4        (default C2 run only) BASELINE configs[2] and [3] timed the same
                way in the same process, after C2: each rank its own batch
  fill,         (default C2 run only) the SURVEY §8f rows timed the same way:
  fill_noout,   send-side FILL on C2's layout with and without a results
  fill_c3,      buffer (the reference's call shape) and on C3's mix; C2 in
  c2_rfc,       RFC 1071 mode; VERIFY and RECEIVE (verdicts + host-order
  slots,        headers) on a 1M-slot receive ring, the send stream cut into
  receive,      checksummed MSS images; each with its own metric
  segment
  c5_strong     (default C2 run only) BASELINE configs[4]: ONE 8M x 1492-B batch
                split over the N ranks with shard_range (8M images on one GPU
                at N=1, 1M per GPU at N=8); value = all ranks' bytes / the
                slowest rank's wall time per step, kernel_GiBs = / the slowest
                rank's kernel time, per_gpu_frac = each GPU's roofline fraction
  cpu_baseline  the reference's own CalculateChecksum (oracle/_ref, built from
                /root/reference/include/tcp-header.h) on the host cores over the
                whole C2 arena (DRAM-sized: 6x the host L3), median of 7 passes
                with min / max (rank 0, N=1 only); falls back to the in-repo C
                restatement ("port") where oracle/_ref is absent.  The c3 key
                carries one over the whole C3 arena, c4 over C4's first 2 GiB,
                c2_rfc the RFC 1071 restatement ("port") over C2's arena
  e2e           host-memory rate incl. pinned hipMemcpyAsync H2D + D2H (not `value`)
  settle        untimed launches run before the W warm-up steps until --settle-ms
                has passed (the idle GPU's clock ramp, scripts/transient.py)
  devices       distinct GPUs the ranks ran on (a hash of each rank's PCI
                address, UUID and HIP bus id, gathered): fewer than the ranks
                exits 3, unless the one-GPU rehearsal knob TCPCK_BENCH_DEVICE
                is set, which marks the line `rehearsal`; every process group
                times out after 300 s (TCPCK_BENCH_PG_TIMEOUT)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tcp-stack_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "GiB/s device-resident TCP checksum over batched segments; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md (spec 8.0 TB/s)
GIB = float(1 << 30)

CONFIGS = {
    # name: (description, kind, count, image bytes)
    "c2": ("C2: 1M x 1460-B payload (1492-B images), fixed stride, device-resident", "fixed", 1 << 20, 1492),
    "c3": ("C3: 4M images, payload uniform over {64,576,1460} B (96/608/1492-B images), packed, u64 offsets",
           "mixed", 4 << 20, None),
    "c4": ("C4: 256K x 64-KiB jumbo images (payload 65504), fixed stride", "fixed", 256 << 10, 65536),
    # strong scaling: one 8M-image batch split evenly over the ranks (at N=8 each rank holds a C2)
    "c5": ("C5: 8M x 1460-B payload (1492-B images) sharded evenly across the GPUs, fixed stride",
           "fixed", 8 << 20, 1492),
}
STRONG = {"c5"}  # configs whose total work is fixed as N grows; the rest are per-GPU (weak)
# the other BASELINE configs, then the §8f ops, timed inside the default (C2) run, and their keys in its line
# (the big C3 / C4 arenas last: C5 timed after C3/C4 had allocated and freed 19 GB ran 2.5 % slower
# than in a process of its own -- 1.737 vs 1.695 ms, profiles/r03/c5_order_probe.log; in this order
# every config matches its own process within 1 %, profiles/r03/bench_order_probe.log)
EXTRAS = (("c5", "c5_strong"), ("fill", "fill"), ("fill_noout", "fill_noout"), ("c2_rfc", "c2_rfc"),
          ("slots", "slots"), ("receive", "receive"), ("segment", "segment"), ("c3", "c3"), ("fill_c3", "fill_c3"),
          ("c4", "c4"))
# round-2 ops (not BASELINE configs; same contract, their own metric):
EXTRA = {
    # the device-resident receive arena: 1M 2048-B slots, one datagram per slot
    "slots": ("receive slots: 1M x 2048-B slots, images of 96/608/1492 B (C3's mix), offset list, "
              "TCPCK_LAYOUT_SORTED, VERIFY", "slots", 1 << 20, 2048),
    # the receive path's front half on the same ring: verdicts + host-order headers into a dense array
    "receive": ("receive ring: 1M x 2048-B slots, images of 96/608/1492 B, offset list, TCPCK_LAYOUT_SORTED; "
                "tcpck_batch_receive: verdicts + TcpHeaderN2H into a 32-B-per-image header array",
                "receive", 1 << 20, 2048),
    # the send path's insert (socket-manager.cc:9-10) on C2's layout: zero, compute, store in place
    "fill": ("send-side FILL on C2's layout: 1M x 1492-B images, fixed stride, checksum field zeroed, computed "
             "and stored in place, results also to a u16 array", "fill", 1 << 20, 1492),
    # the same without a results buffer: the reference's call shape (socket-manager.cc:9-10 stores only into
    # the packet); the library keeps its two-pass form through the context's results scratch
    "fill_noout": ("send-side FILL on C2's layout without a results buffer (the reference's call shape): 1M x "
                   "1492-B images, checksum field zeroed, computed and stored in place", "fill", 1 << 20, 1492),
    # FILL on C3's mix (packed offsets): the send path's insert on variable-length segments
    "fill_c3": ("send-side FILL on C3's mix: 4M images of 96/608/1492 B, packed, u64 offsets, fields stored in "
                "place, results also to a u16 array", "fill_var", 4 << 20, None),
    # the opt-in RFC 1071 arithmetic (end-around carry) on C2's batch
    "c2_rfc": ("C2 in TCPCK_MODE_RFC1071 (opt-in one's-complement with end-around carry; not the reference's "
               "arithmetic): 1M x 1492-B images, fixed stride", "fixed", 1 << 20, 1492),
    # the send path's producer: a 1.5 GB send stream cut into MSS segments
    "segment": ("send stream 1.5 GiB -> 1460-B segments in 1504-B slots (header template + payload, "
                "checksum filled; tcpck_batch_segment)", "segment", (1460 << 20) + 2, 1460),
}


IMAGE_BYTES = {"slots": "96/608/1492 in 2048-B slots", "receive": "96/608/1492 in 2048-B slots",
               "segment": "32 + 1460 in 1504-B slots"}
MODES = {"c2_rfc": 1}  # TCPCK_MODE_RFC1071; every other config runs the reference arithmetic (0)
NO_RESULTS = {"fill_noout"}  # steps that write no results array (only the fields in place)
ARENAS = 2  # identical batches taken in turn by every step (Workload; --arenas)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS) + ["c1"] + sorted(EXTRA))
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget (7 passes)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="default run: skip the c3/c4/c5_strong keys")
    p.add_argument("--settle-ms", type=float, default=250.0,
                   help="untimed back-to-back launches before the warm-up steps (clock ramp)")
    p.add_argument("--arenas", type=int, default=ARENAS,
                   help="identical batches per config, taken in turn by the steps (no cross-step cache reuse)")
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks and print their layout only (no GPU; tests/test_bench_contract.py)")
    p.add_argument("--per-launch-events", action="store_true",
                   help="one HIP event pair per launch (adds ~10 us idle per step)")
    p.add_argument("--fail-rank", type=int, default=-1,
                   help="--launch-check only: this rank exits with status 3 after joining the process group "
                        "(tests/test_bench_contract.py: the job must fail, not hang)")
    return p.parse_args()


# A rank that stalls in the rendezvous, a barrier or a collective must not hold
# an 8-GPU lease silently for torch's default 10 minutes:
# every process group gets this timeout (TCPCK_BENCH_PG_TIMEOUT overrides it).
PG_TIMEOUT_S = 300.0


def init_group(backend: str, device=None) -> None:
    import datetime
    import torch.distributed as dist
    timeout = datetime.timedelta(seconds=float(os.environ.get("TCPCK_BENCH_PG_TIMEOUT", PG_TIMEOUT_S)))
    if device is not None:
        dist.init_process_group(backend, timeout=timeout, device_id=device)
    else:
        dist.init_process_group(backend, timeout=timeout)


def device_identity(dev_index: int) -> tuple[int, int]:
    """(PCI address as dom << 16 | bus << 8 | device, a 48-bit identity code)
    of the HIP device this rank runs on.  The code hashes the PCI address and
    the device UUID, so ranks on distinct GPUs get distinct codes; 0 when the
    runtime reports neither (then nothing can be concluded)."""
    import hashlib
    import torch
    p = torch.cuda.get_device_properties(dev_index)
    dom, bus, dv = int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)
    try:
        uuid = str(p.uuid).strip()
    except Exception:  # noqa: BLE001 -- an optional field
        uuid = ""
    bus_id = hip_pci_bus_id(dev_index)  # "dddd:bb:dd.f": the function too (partitioned GPUs)
    pci = (dom << 16) | (bus << 8) | dv
    if pci == 0 and uuid.strip("0-") in ("", "GPU") and not bus_id:
        return pci, 0
    code = int.from_bytes(hashlib.sha256(f"{pci:x}|{uuid}|{bus_id}".encode()).digest()[:6], "big") or 1
    return pci, code


def hip_pci_bus_id(dev_index: int) -> str:
    """hipDeviceGetPCIBusId of the HIP runtime this process already loaded
    (found in /proc/self/maps, never a second copy), or "" if unavailable."""
    import ctypes
    try:
        with open("/proc/self/maps") as f:
            paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
        if len(paths) != 1:
            return ""
        hip = ctypes.CDLL(paths.pop())
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(dev_index)) != 0:
            return ""
        return buf.value.decode(errors="replace")
    except Exception:  # noqa: BLE001 -- identity is best effort
        return ""


def check_devices(world: int, dev_index: int, coll_dev, rehearsal: bool) -> dict:
    """Every rank's device identity, gathered.  With fewer distinct devices
    than ranks the line would read as an N-GPU result it is not: an error (exit
    3 on every rank -- all of them see the same list), or, under the one-GPU
    rehearsal knob TCPCK_BENCH_DEVICE, a line marked as a rehearsal.  A rank
    whose runtime reports no identity makes the count unknown (null), never an
    error."""
    from tcpck.shard import gather_ranks
    pci, code = device_identity(dev_index)
    pcis = [int(x) for x in gather_ranks(float(pci), device=coll_dev)]
    codes = [int(x) for x in gather_ranks(float(code), device=coll_dev)]
    names = [f"{c >> 16:04x}:{(c >> 8) & 0xFF:02x}:{c & 0xFF:02x}" for c in pcis]
    if 0 in codes:
        log(f"warning: the runtime reports no device identity on some rank ({names}): devices unknown")
        return {"devices": None, "device_ids": names, "rehearsal": rehearsal}
    distinct = len(set(codes))
    if distinct < world:
        if not rehearsal:
            log(f"error: {world} ranks on {distinct} distinct device(s) {names}: not an {world}-GPU run")
            sys.exit(3)
        log(f"warning: rehearsal (TCPCK_BENCH_DEVICE set): {world} ranks on {distinct} device(s) {names}")
    return {"devices": distinct, "device_ids": names, "rehearsal": distinct < world}


def run_c1(n: int) -> dict:
    """C1 (BASELINE configs[0]): n single 1460-B segments over UDP loopback,
    CPU only -- send insert (socket-manager.cc:9-10), receive buffer
    (network-service.cc:49-56), verify (socket-manager.h:182).
    tcp-stack_amd/bin/loopback_c1 is the program compiled against the drop-in
    header (this library); oracle/_ref/loopback_c1_ref, where present, the same
    source compiled against the reference's own include/tcp-header.h is its
    cpu_baseline.  Both run on the host."""
    import subprocess

    def run(exe):
        r = subprocess.run([exe, str(n), "1460"], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise SystemExit(f"{exe} failed rc={r.returncode}: {r.stderr}")
        return json.loads(r.stdout.strip().splitlines()[-1])

    ours = run(os.path.join(ROOT, "tcp-stack_amd", "bin", "loopback_c1"))
    rec = {"value": round(ours["us_per_segment"], 3), "unit": "us/segment", "segments": n,
           "received": ours["received"], "verified": ours["verified"],
           "send_ck_ns": ours["send_checksum_ns"], "recv_ck_ns": ours["recv_checksum_ns"]}
    ref = os.path.join(ROOT, "oracle", "_ref", "loopback_c1_ref")
    if os.path.exists(ref):
        r = run(ref)
        rec["cpu_baseline"] = {"value": round(r["us_per_segment"], 3), "unit": "us/segment", "cores": 1,
                               "kind": "reference", "verified": r["verified"],
                               "send_ck_ns": r["send_checksum_ns"], "recv_ck_ns": r["recv_checksum_ns"]}
    return rec


def bench_c1(args):
    """--config c1: the C1 record as a line of its own."""
    n = max(1000, args.steps * 1000)
    r = run_c1(n)
    rec = {"metric": "C1 loopback send+fill+recv+verify latency per 1492-B segment (CPU, no GPU)",
           "value": r.pop("value"), "unit": r.pop("unit"), "n_gpus": 0, "steps": n, "warmup": 0,
           "ms_per_step": None, "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
           "data": "synthetic (fixed payload pattern)",
           "config": {"workload": "C1: single 1460-B segments over UDP 127.0.0.1, drop-in tcp_stack/tcp-header.h",
                      **{k: v for k, v in r.items() if k != "cpu_baseline"}}}
    rec["ms_per_step"] = round(rec["value"] / 1e3, 6)
    if "cpu_baseline" in r:
        rec["cpu_baseline"] = r["cpu_baseline"]
    print(json.dumps(rec), flush=True)


class Workload:
    """One config's device-resident batch on this rank and its step function."""

    def __init__(self, name, ctx, stream, rank, world, n_arenas=1):
        import torch
        import tcpck
        from tcpck.shard import shard_range
        desc, kind, count, L = CONFIGS[name] if name in CONFIGS else EXTRA[name]
        self.name, self.desc, self.kind, self.L = name, desc, kind, L
        self.strong = name in STRONG
        self.mode = MODES.get(name, 0)
        mode = self.mode
        if self.strong:
            first, stop = shard_range(count, world, rank)  # independent contiguous shard, no exchange
            count = stop - first
        else:
            first = rank * count  # weak: every rank checksums its own batch of the config's size
        self.extra_bytes = 0  # algorithmic bytes per launch beyond the image bytes read (+2 per result)
        self.layout = None
        self.arena = None
        # Every step reads one of n_arenas identical batches, taken in turn
        # (--arenas, default ARENAS): step k+1 never finds the lines step k left
        # in the 256-MB Infinity Cache -- a sender or receiver never sees the
        # same segments twice.  make() builds one batch, run(batch, out) is
        # one pass of the hot path over it.
        if kind in ("slots", "receive"):
            rng = np.random.default_rng(42 + rank)
            ln = (np.asarray((64, 576, 1460), np.uint32)[rng.integers(0, 3, count)] + 32).astype(np.uint32)
            off = np.arange(count, dtype=np.uint64) * np.uint64(L)
            d_off, d_ln = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
            img_bytes = int(ln.astype(np.int64).sum())
            lmin, lmax = int(ln.min()), int(ln.max())

            def make():
                a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
                tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42, first_index=first, stream=stream)
                return a

            if kind == "slots":
                def run(a, out):
                    ctx.batch_var(tcpck.OP_VERIFY, a, d_off, d_ln, count, out, total_bytes=img_bytes,
                                  min_len=lmin, max_len=lmax, sorted=True, stream=stream)
            else:
                hdr_out = torch.empty(count * 32, dtype=torch.uint8, device="cuda")
                self.extra_bytes = 32 * count  # the header array written

                def run(a, out):
                    ctx.batch_receive(a, count, out, hdr_out, offsets=d_off, lengths=d_ln,
                                      total_bytes=img_bytes, min_len=lmin, max_len=lmax, sorted=True,
                                      stream=stream)
        elif kind == "segment":
            P, seg, stride = count, L, 1504
            count = (P + seg - 1) // seg
            hdr = np.zeros(32, np.uint8)
            hdr[0:4], hdr[4:8], hdr[12:14], hdr[14:16] = [127, 0, 0, 1], [127, 0, 0, 1], [0x3C, 0x8C], [0x3C, 0x8D]
            hdr[20:24], hdr[25] = [0, 0, 0x1E, 0x61], 0x08  # ack 7777, ACK (state.cc:178-180)
            img_bytes = P  # the stream read
            self.extra_bytes = P + 32 * count  # the images written (header + payload; slot padding excluded)

            def make():
                payload = torch.empty(P, dtype=torch.uint8, device="cuda")
                tcpck.synth_fixed(payload, 1492, 1492, P // 1492, seed=42, first_index=first, stream=stream)
                return payload, torch.empty(count * stride, dtype=torch.uint8, device="cuda")

            def run(b, out):
                ctx.batch_segment(b[0], P, seg, hdr, 1001, b[1], stride, out, stream=stream)
        elif kind in ("fill", "fixed"):
            img_bytes = count * L

            def make():
                a = torch.empty(count * L, dtype=torch.uint8, device="cuda")
                tcpck.synth_fixed(a, L, L, count, seed=42, first_index=first, stream=stream)
                return a

            if kind == "fill":
                self.extra_bytes = 2 * count  # the fields written in place (+2 per result below)
                with_out = name not in NO_RESULTS

                def run(a, out):
                    ctx.batch_fixed(tcpck.OP_FILL, a, L, L, count, out if with_out else None, stream=stream)
            else:
                def run(a, out):
                    ctx.batch_fixed(tcpck.OP_CHECKSUM, a, L, L, count, out, mode=mode, stream=stream)
        else:
            from synth_np import mixed_layout
            off, ln, total = mixed_layout(count, seed=42 + rank)
            d_off = torch.from_numpy(off).cuda()
            d_ln = torch.from_numpy(ln).cuda()
            img_bytes = int(ln.astype(np.int64).sum())
            lmin, lmax = int(ln.min()), int(ln.max())  # host-side layout hint, computed once
            self.layout = (off, ln)

            def make():
                a = torch.empty(total, dtype=torch.uint8, device="cuda")
                tcpck.synth_var(a, d_off, d_ln, 1492, count, seed=42, first_index=first, stream=stream)
                return a

            op = tcpck.OP_FILL if kind == "fill_var" else tcpck.OP_CHECKSUM
            if kind == "fill_var":
                self.extra_bytes = 2 * count  # the fields written in place (+2 per result below)

            def run(a, out):
                ctx.batch_var(op, a, d_off, d_ln, count, out, total_bytes=img_bytes, min_len=lmin, max_len=lmax,
                              packed=True, stream=stream)
        self.bufs = [make() for _ in range(max(1, n_arenas))]
        self.n_arenas, self.turn = len(self.bufs), 0

        def step(out):
            run(self.bufs[self.turn % self.n_arenas], out)
            self.turn += 1
        arena = self.bufs[0]
        self.arena = arena if kind in ("fixed", "mixed", "fill", "fill_var", "slots", "receive") else None
        self.count, self.first, self.img_bytes = count, first, img_bytes
        self.verdicts = kind in ("slots", "receive")  # u8 results
        self.results_written = name not in NO_RESULTS
        self.out = torch.empty(count, dtype=torch.uint8 if self.verdicts else torch.int16, device="cuda")
        self._step = step
        torch.cuda.synchronize()

    def step(self):
        self._step(self.out)

    @property
    def algo_bytes(self) -> int:
        """Algorithmic bytes per launch: image bytes read + other bytes written + the results."""
        res = ((1 if self.verdicts else 2) * self.count) if self.results_written else 0
        return self.img_bytes + self.extra_bytes + res

    def results(self) -> np.ndarray:
        import torch
        res = self.out.cpu().numpy()
        return res.view(np.uint16) if self.out.dtype == torch.int16 else res


def measure(w: Workload, args, world, stream, coll_dev):
    """Settle, warm up, then time exactly K steps between barrier + synchronize
    brackets.  Returns (slowest rank's wall seconds, this rank's per-launch ms,
    every rank's per-launch ms, the bytes all ranks read per step, settle info)."""
    import torch
    import torch.distributed as dist
    from tcpck.shard import gather_ranks, max_over_ranks
    # Settle: an idle MI355X takes 10-50 ms of back-to-back HBM streaming to
    # reach its steady clocks (scripts/transient.py, profiles/r01/transient.log:
    # C3 launches run at 54-79% of the roof for the first ~50 ms, then 83-84%).
    # Untimed launches of the same step until settle_ms have passed, then the W
    # warm-up steps; neither is in the timed region.
    settled, t_set = 0, time.perf_counter()
    while (time.perf_counter() - t_set) * 1e3 < args.settle_ms:
        for _ in range(8):
            w.step()
        torch.cuda.synchronize()
        settled += 8
    settle_ms = (time.perf_counter() - t_set) * 1e3
    for _ in range(args.warmup):
        w.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the launch stream bracket the K launches.  An event recorded
    # between two launches costs ~10 us of idle GPU per step on ROCm (rocprof
    # trace: 0 us between back-to-back launches, 10-11 us with per-launch
    # events), so the per-launch average is the bracket / K; it includes the
    # (near-zero) kernel boundaries, so it can only under-state the kernel rate.
    # --per-launch-events restores one event pair per launch (diagnostics).
    n_ev = args.steps if args.per_launch_events else 1
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    t0 = time.perf_counter()
    if not args.per_launch_events:
        starts[0].record(stream)
    for i in range(args.steps):
        if args.per_launch_events:
            starts[i].record(stream)
        w.step()
        if args.per_launch_events:
            ends[i].record(stream)
    if not args.per_launch_events:
        ends[0].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    launch_ms = float(np.sum([s.elapsed_time(e) for s, e in zip(starts, ends)])) / args.steps
    tmax = max_over_ranks(elapsed, device=coll_dev)
    launch_ms_all = gather_ranks(launch_ms, device=coll_dev)  # per-GPU kernel time (ranks start together)
    shard_bytes = torch.tensor([w.img_bytes], dtype=torch.int64, device=coll_dev)
    if world > 1:
        dist.all_reduce(shard_bytes)  # bytes all ranks processed per step (shards may differ by one image)
    settle = {"ms": round(settle_ms, 1), "launches": settled}
    return tmax, launch_ms, launch_ms_all, int(shard_bytes.item()), settle


def roofline(w: Workload, launch_ms, launch_ms_all, traffic_key, world):
    algo = w.algo_bytes
    achieved = algo / (launch_ms * 1e-3) / 1e9
    traffic, note = pmc_traffic(traffic_key) if world == 1 else (None, "PMC passes are single-GPU runs")
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": note,
         "algorithmic_bytes_per_launch": algo, "avg_launch_ms": round(launch_ms, 5)}
    if world > 1:  # rank 0's kernel above; every GPU's fraction here (equal shards)
        r["per_gpu_frac"] = [round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for ms in launch_ms_all]
    return r


def extra_config(name, key, ctx, stream, rank, world, args, coll_dev):
    """Another BASELINE config timed in the default run; its record for rank 0's line."""
    import torch
    w = Workload(name, ctx, stream, rank, world, args.arenas)
    same_ring = None
    if w.n_arenas > 1 and w.kind in ("slots", "receive"):
        # first the same step on ONE ring, every step over the same datagrams:
        # what the Infinity Cache's cross-step reuse adds (never `value`; timed
        # first so that the key's own K launches are the last ones in a trace)
        rings, w.n_arenas = w.n_arenas, 1
        tmax1, launch1, _, step_bytes1, _ = measure(w, args, world, stream, coll_dev)
        same_ring = {"value": round(step_bytes1 * args.steps / tmax1 / GIB, 2),
                     "frac": round(w.algo_bytes / (launch1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        w.n_arenas = rings
    tmax, launch_ms, launch_ms_all, step_bytes, settle = measure(w, args, world, stream, coll_dev)
    rec = {"workload": w.desc, "metric": metric_for(w.kind, w.mode), "value": round(step_bytes * args.steps / tmax / GIB, 2),
           "unit": "GiB/s",
           "ms_per_step": round(tmax / args.steps * 1e3, 5), "scaling": "strong" if w.strong else "weak",
           "images_per_gpu": w.count, "bytes_per_gpu": w.img_bytes,
           "roofline": roofline(w, launch_ms, launch_ms_all, name, world), "settle": settle}
    if name in CPU_EXTRA and rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline_for(w, CPU_EXTRA[name][1])
    if w.strong:
        # the 8M-image batch's bytes over the slowest GPU's kernel time
        rec["kernel_GiBs"] = round(step_bytes / (max(launch_ms_all) * 1e-3) / GIB, 2)
        rec["images_total"] = CONFIGS[name][2]
        rec["parallelism"] = f"shard{world}: one batch split by tcpck.shard.shard_range, no collective"
    if same_ring is not None:
        rec["same_ring"] = same_ring
    del w
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return key, rec


def spawn_ranks(args) -> int | None:
    """`--gpus N` (N > 1) run bare, without a launcher: start the N ranks as a
    CHILD `torch.distributed.run` on this same command line (one process per
    GPU, rendezvous on 127.0.0.1) and return its exit code; rank 0's line
    reaches our stdout through the inherited descriptor.  Runs before anything
    touches the GPU, and never replaces this process (no exec).  None when
    there is nothing to spawn (N = 1, or already a rank of a launcher)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:  # a free rendezvous port
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"--gpus {args.gpus} without a launcher: spawning {' '.join(cmd[1:6])} ...")
    sys.stdout.flush()
    return subprocess.run(cmd).returncode


def launch_check(args) -> None:
    """--launch-check: the rank layout alone (no GPU): every rank joins the
    process group on TCPCK_BENCH_BACKEND (gloo here), rank 0 prints the world
    size and every rank's (rank, local rank).  Exercises spawn_ranks on CPU."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        init_group(os.environ.get("TCPCK_BENCH_BACKEND", "gloo"))
        if rank == args.fail_rank:
            log(f"rank {rank}: --fail-rank, exiting with status 3")
            sys.exit(3)
        t = torch.zeros(2 * world, dtype=torch.int64)
        t[2 * rank], t[2 * rank + 1] = rank, local
        dist.all_reduce(t)
        ranks = t.view(world, 2).tolist()
    else:
        ranks = [[rank, local]]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "gpus_arg": args.gpus, "ranks": ranks}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.config == "c1":
        return bench_c1(args)
    rc = spawn_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # one line per job: a launcher with another rank count than --gpus would
        # print an N-GPU line for a different N
        log(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE {world} ranks")
        sys.exit(2)
    if args.launch_check:
        return launch_check(args)
    import torch
    import torch.distributed as dist
    import tcpck

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): several ranks on one GPU with
    # gloo collectives, to exercise the N>1 path on a one-GPU box
    backend = os.environ.get("TCPCK_BENCH_BACKEND", "nccl")
    rehearsal = "TCPCK_BENCH_DEVICE" in os.environ
    dev_index = int(os.environ.get("TCPCK_BENCH_DEVICE", local))
    coll_dev = "cuda" if backend == "nccl" else "cpu"
    torch.cuda.set_device(dev_index)
    local = dev_index
    if world > 1:
        init_group(backend, torch.device("cuda", local) if backend == "nccl" else None)
    devices = check_devices(world, dev_index, coll_dev, rehearsal)

    from tcpck.shard import gather_ranks, max_over_ranks
    ctx = tcpck.Context(local)
    stream = torch.cuda.current_stream()
    w = Workload(args.config, ctx, stream, rank, world, args.arenas)
    one_arena = None
    if w.n_arenas > 1:
        # the same K steps on ONE batch re-read step after step, for reference:
        # the Infinity Cache then serves part of each step (never `value`; timed
        # first so that a kernel trace's last K launches are `value`'s)
        k, w.n_arenas = w.n_arenas, 1
        tmax1, launch1, _, step_bytes1, _ = measure(w, args, world, stream, coll_dev)
        one_arena = {"value": round(step_bytes1 * args.steps / tmax1 / GIB, 2),
                     "frac": round(w.algo_bytes / (launch1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        w.n_arenas = k
    tmax, launch_ms, launch_ms_all, step_bytes, settle = measure(w, args, world, stream, coll_dev)
    value = step_bytes * args.steps / tmax / GIB
    res = w.results()  # checksum results of this rank (the CPU baseline compares them)

    # End to end through PCIe (never `value`): every rank at once, so the
    # driver's N-GPU runs also record the host-memory path's aggregate rate
    e2e = None
    if not args.no_e2e and w.kind == "fixed" and not w.strong and w.mode == 0:
        if world > 1:
            dist.barrier()
        dt, ok = e2e_seconds(ctx, w.arena, res, w.count, w.L)
        dt_max = max_over_ranks(dt, device=coll_dev)
        ok_all = min(gather_ranks(1.0 if ok else 0.0, device=coll_dev)) > 0
        if np.isfinite(dt_max):
            e2e = {"value": round(world * w.count * w.L / dt_max / GIB, 2), "unit": "GiB/s", "match": ok_all,
                   "what": "pinned host arena -> 64 MiB chunks H2D on 2 streams -> kernel -> u16 results D2H, "
                           f"all {world} rank(s) at once, whole-job bytes / slowest rank; match: results == the "
                           "device path's"}

    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and w.kind in ("fixed", "mixed")
    cpu_rec = cpu_baseline_for(w, args.cpu_seconds) if want_cpu else None  # before the extras free the arena
    rec = {
        "metric": metric_for(w.kind, w.mode), "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(tmax / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if w.strong else "weak", "vs_baseline": None, "dtype": "u16",
        "data": "synthetic (device-generated: send-path headers + splitmix64 payloads, seed 42)",
        "config": {"workload": w.desc, "images_per_gpu": w.count,
                   "image_bytes": IMAGE_BYTES.get(w.kind, w.L if w.L else "96/608/1492"),
                   "bytes_per_gpu": w.img_bytes,
                   "parallelism": f"shard{world} (independent per-GPU batches, no collective)"},
        "roofline": roofline(w, launch_ms, launch_ms_all, args.config, world),
        "settle": settle,
        "devices": devices["devices"],
        "device_ids": devices["device_ids"],
    }
    if devices["rehearsal"]:
        rec["rehearsal"] = "TCPCK_BENCH_DEVICE: several ranks share a device; not an N-GPU measurement"
    if one_arena is not None:
        rec["one_arena"] = one_arena
    del w
    torch.cuda.empty_cache()

    # The other BASELINE configs, driver-timed in the same process (default run only)
    if args.config == "c2" and not args.no_extras:
        for name, key in EXTRAS:
            k, r = extra_config(name, key, ctx, stream, rank, world, args, coll_dev)
            rec[k] = r
    if cpu_rec is not None:
        rec["cpu_baseline"] = cpu_rec
    if e2e is not None:
        rec["e2e"] = e2e
    if rank == 0 and world == 1 and args.config == "c2" and not args.no_extras:
        rec["c1"] = run_c1(20000)  # BASELINE configs[0], host CPU only
    if rank == 0:
        line, detail = compact_line(rec)
        print(json.dumps(line, separators=(",", ":")), flush=True)
        write_detail(detail, args)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


def metric_for(kind, mode=0):
    if mode == 1:
        return ("GiB/s device-resident TCP checksum in RFC 1071 mode (opt-in end-around carry, not the reference's "
                "arithmetic) over batched segments; % HBM roofline")
    if kind == "slots":
        return "GiB/s device-resident TCP verify over a slotted receive arena (image bytes); % HBM roofline"
    if kind in ("fill", "fill_var"):
        return "GiB/s device-resident TCP send-side fill (zero, checksum, store in place) over batched segments; % HBM roofline"
    if kind == "receive":
        return ("GiB/s device-resident TCP receive (verify + TcpHeaderN2H into a header array) over a slotted "
                "receive arena (image bytes); % HBM roofline (read + write)")
    if kind == "segment":
        return "GiB/s of device-resident send stream segmented into checksummed images; % HBM roofline (read + write)"
    return METRIC


# ---- the printed line: numbers only, under LINE_LIMIT bytes ------------------
# The driver keeps only the tail of stdout (BENCH_r04 kept 8.3 KB of an 11.9-KB
# line, cutting four keys), so the line carries the numbers and every prose
# field goes to the detail record (stderr + gpurun_out/bench_detail_<config>_n<N>.json).
LINE_LIMIT = 6000
_TOP_CPU = ("value", "unit", "cores", "kind", "sample", "match", "min_GiBs", "max_GiBs", "one_thread_GiBs",
            "reference_O0_GiBs", "cpu_model")
_KEY_CPU = ("value", "cores", "kind", "match", "min_GiBs", "max_GiBs")


def _split(d: dict, keep) -> tuple[dict, dict]:
    return {k: v for k, v in d.items() if k in keep}, {k: v for k, v in d.items() if k not in keep}


def compact_line(rec: dict) -> tuple[dict, dict]:
    """(the printed line, the detail record) of a full bench record: prose,
    pass lists and per-key descriptions move to the detail."""
    line, detail = {}, {}
    for k, v in rec.items():
        if k in ("settle", "device_ids"):
            detail[k] = v
        elif k == "roofline":
            line[k], rest = _split(v, ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                       "algorithmic_bytes_per_launch", "avg_launch_ms", "per_gpu_frac"))
            detail[k] = rest
        elif k == "cpu_baseline":
            line[k], detail[k] = _split(v, _TOP_CPU)
        elif k == "e2e":
            line[k], detail[k] = _split(v, ("value", "unit", "match"))
        elif k == "c1":
            line[k] = v
        elif isinstance(v, dict) and "roofline" in v and k != "config":  # an extra key
            r = v["roofline"]
            key = {"value": v["value"], "ms_per_step": v["ms_per_step"],
                   "roofline": {"frac": r["frac"], "achieved": r["achieved"], "traffic": r["traffic"],
                                "algo_bytes": r["algorithmic_bytes_per_launch"], "launch_ms": r["avg_launch_ms"]}}
            if "per_gpu_frac" in r:
                key["roofline"]["per_gpu_frac"] = r["per_gpu_frac"]
            for extra in ("scaling", "kernel_GiBs", "images_total", "same_ring"):
                if extra in v and (extra != "scaling" or v[extra] != "weak"):
                    key[extra] = v[extra]
            d = {kk: vv for kk, vv in v.items() if kk not in key and kk not in ("roofline", "cpu_baseline")}
            d["traffic_source"] = r.get("traffic_source")
            if "cpu_baseline" in v:
                key["cpu_baseline"], d["cpu_baseline"] = _split(v["cpu_baseline"], _KEY_CPU)
            line[k], detail[k] = key, d
        else:
            line[k] = v
    line["detail"] = "stderr + gpurun_out/bench_detail_<config>_n<N>.json: per-key workload, metric, sample, settle"
    return line, detail


def write_detail(detail: dict, args) -> None:
    text = json.dumps(detail, separators=(",", ":"))
    log("bench detail: " + text)
    try:
        d = os.path.join(ROOT, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"bench_detail_{args.config}_n{args.gpus}.json"), "w") as f:
            f.write(text + "\n")
    except OSError as e:
        log(f"bench detail not written: {e}")


_LIB_SHA = None


def lib_sha256() -> str:
    """sha256 of the libtcpck.so this process loaded (the PMC stamps name it)."""
    global _LIB_SHA
    if _LIB_SHA is None:
        import hashlib
        import tcpck
        with open(tcpck.LIB_PATH, "rb") as f:
            _LIB_SHA = hashlib.sha256(f.read()).hexdigest()
    return _LIB_SHA


def pmc_traffic(config: str):
    """(HBM bytes per launch, note) from the committed rocprofv3 PMC passes
    (profiles/pmc_summary.json), or (None, why) when there is no pass for this
    config or it was captured on another build of libtcpck.so than the one
    loaded (each entry carries the library's sha256)."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            e = json.load(f)[config]
    except (OSError, KeyError, ValueError):
        return None, f"no PMC pass for {config} in profiles/pmc_summary.json"
    if e.get("lib_sha256") != lib_sha256():
        return None, (f"PMC pass captured on libtcpck.so sha256 {str(e.get('lib_sha256'))[:16]}, loaded "
                      f"{lib_sha256()[:16]}: not this build")
    return e["hbm_bytes_per_launch"], f"{e['source']} (libtcpck.so sha256 {lib_sha256()[:16]})"


def cpu_threads() -> tuple[int, dict]:
    """Threads for the CPU baseline: this process's CPU share.  The GPU box
    gives one GPU's job a 16-CPU share (OMP_NUM_THREADS=16 there; nproc and
    the affinity mask show the whole machine), so the baseline uses
    min(affinity, OMP_NUM_THREADS) threads and reports all three counts."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = min(aff, omp) if omp > 0 else aff
    return max(1, n), {"affinity_cpus": aff, "nproc": os.cpu_count(), "omp_num_threads": omp or None}


def cpu_baseline(host_arena, gpu_res, sargs, sbytes, sdesc, budget_s, mode=0, secondary_o0=False):
    """The reference's CalculateChecksum (oracle/_ref, tcp-header.h:252-263) on
    the host cores over `host_arena` (sargs: stride/length/count or
    offsets/lengths), every packet materialised once with MakeNetPacket:
    7 timed passes of ~budget_s / 7 each, median, with min / max and every
    pass.  RFC 1071 mode (not the reference's arithmetic) and a missing
    oracle/_ref use the in-repo C restatement (oracle/ref16.c, "port")."""
    from oracle import ref16 as R
    nthr, counts = cpu_threads()
    out = {"unit": "GiB/s", "cores": nthr, **counts}
    n = int(sargs["count"]) if "count" in sargs else int(np.asarray(sargs["offsets"]).size)

    def summary(rates):
        return {"value": round(statistics.median(rates), 2), "min_GiBs": round(min(rates), 2),
                "max_GiBs": round(max(rates), 2), "passes_GiBs": [round(r, 1) for r in rates]}

    if mode == 0 and R.RefLib.available("O3"):
        pk = R.RefLib("O3").packets(host_arena, **sargs)  # MakeNetPacket once, outside timing

        def passes(lib_pk, threads, n_pass, target_s):
            """GiB/s of n_pass timed passes of ~target_s each."""
            t1 = lib_pk.run_reps(threads, 1)
            reps = max(1, int(target_s / max(t1, 1e-6)))
            return [sbytes * reps / lib_pk.run_reps(threads, reps) / GIB for _ in range(n_pass)], reps

        got, _ = pk.run(nthr)
        match = bool(np.array_equal(got, gpu_res[:n]))
        rates, reps = passes(pk, nthr, 7, budget_s / 7)
        one, _ = passes(pk, 1, 1, 0.5)
        pk.close()
        out.update(summary(rates))
        out.update({"kind": "reference", "match": match, "one_thread_GiBs": round(one[0], 2),
                    "sample": sdesc,
                    "sample_detail": f"7 passes of {reps} sweeps on {nthr} threads (median; min/max beside it); "
                                     "CalculateChecksum (tcp-header.h:252-263) built -O3 -march=x86-64-v3; "
                                     "match: results == the GPU's"})
        if secondary_o0 and R.RefLib.available("O0"):
            # secondary: the reference as its makefile builds it (-O0 -g, makefile:2), same threads
            p0 = R.RefLib("O0").packets(host_arena, **sargs)
            rates0, _ = passes(p0, nthr, 5, 0.3)
            p0.close()
            out["reference_O0_GiBs"] = round(statistics.median(rates0), 2)
            out["reference_O0_note"] = f"-O0 -g build (makefile:2), median of 5 passes on {nthr} threads"
    else:
        c = R.Ref16C(build=False)
        got = c.batch(host_arena, mode=mode, threads=nthr, **sargs)
        t0 = time.perf_counter()
        c.batch(host_arena, mode=mode, threads=nthr, **sargs)
        t1 = max(time.perf_counter() - t0, 1e-6)
        reps = max(1, int(budget_s / 7 / t1))
        rates = []
        for _ in range(7):
            t0 = time.perf_counter()
            for _ in range(reps):
                c.batch(host_arena, mode=mode, threads=nthr, **sargs)
            rates.append(sbytes * reps / (time.perf_counter() - t0) / GIB)
        out.update(summary(rates))
        what = "RFC 1071 restatement (oracle/ref16.c oracle_rfc1071)" if mode else "oracle/ref16.c restatement"
        out.update({"kind": "port", "match": bool(np.array_equal(got, gpu_res[:n])), "sample": sdesc,
                    "sample_detail": f"{what}, 7 passes of {reps} sweeps on {nthr} threads (median; min/max beside "
                                     "it); match: results == the GPU's"})
    log(f"cpu baseline: {out['value']} GiB/s on {nthr} threads (min {out['min_GiBs']}, max {out['max_GiBs']})")
    try:
        out["cpu_model"] = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t")
    except Exception:
        pass
    return out


# CPU baselines beside the extra keys (rank 0, N = 1): (config -> images of the batch's head timed, seconds)
CPU_EXTRA = {"c3": (None, 6.0), "c4": (32768, 6.0), "c2_rfc": (None, 4.0)}


def cpu_baseline_for(w: "Workload", budget_s: float):
    """cpu_baseline over the same bytes as workload w (C4: its first 2 GiB)."""
    res = w.results()
    if w.kind == "mixed":
        off, ln = w.layout
        host_arena = w.arena.cpu().numpy()
        sbytes = int(ln.astype(np.int64).sum())
        return cpu_baseline(host_arena, res, dict(offsets=off, lengths=ln), sbytes,
                            f"all {w.count} images ({sbytes / 1e9:.2f} GB, host copy)", budget_s, w.mode)
    n = CPU_EXTRA.get(w.name, (None,))[0] or w.count
    host_arena = w.arena[:n * w.L].cpu().numpy()
    sbytes = n * w.L
    what = f"all {n} images" if n == w.count else f"the first {n} images"
    return cpu_baseline(host_arena, res, dict(stride=w.L, length=w.L, count=n), sbytes,
                        f"{what} ({sbytes / 1e9:.2f} GB, host copy)", budget_s, w.mode,
                        secondary_o0=w.name == "c2")


def e2e_seconds(ctx, arena, gpu_res, count, L):
    """Seconds per pass of host (pinned) -> GPU -> host over this rank's batch
    through tcpck_host_batch_fixed, and whether the results equal the device
    path's.  A failure (e.g. pinning refused) returns (inf, False) rather than
    leaving the other ranks waiting in the collectives that follow."""
    import torch
    import tcpck
    try:
        h = torch.empty(count * L, dtype=torch.uint8).pin_memory()
        h.copy_(arena.cpu())
        hout = torch.empty(count, dtype=torch.int16).pin_memory()
        ctx.set_chunk_bytes(64 << 20)
        ctx.host_batch_fixed(tcpck.OP_CHECKSUM, h, L, L, count, hout)  # warm (staging alloc)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.host_batch_fixed(tcpck.OP_CHECKSUM, h, L, L, count, hout)
        dt = (time.perf_counter() - t0) / reps
        return dt, bool(np.array_equal(hout.numpy().view(np.uint16), gpu_res))
    except Exception as e:  # noqa: BLE001 -- reported, never fatal to the bench line
        log(f"e2e leg failed: {e}")
        return float("inf"), False


if __name__ == "__main__":
    main()
