"""bench.py's configuration tables (CPU only, no GPU calls): every config the
default run times beside C2 exists, its key is unique, C5 is the strong split,
and the extras keep the order that made each match its own process
(profiles/r03/bench_order_probe.log: C5 first, the 19 GB of C3 / C4 last)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_extras_exist_and_keys_unique():
    names = [n for n, _ in bench.EXTRAS]
    keys = [k for _, k in bench.EXTRAS]
    assert len(set(keys)) == len(keys)
    for n in names:
        assert n in bench.CONFIGS or n in bench.EXTRA, n
    # every BASELINE config (C2 is `value`, C1 is the CPU loopback line) is timed in the default run
    assert {"c3", "c4", "c5"} <= set(names)


def test_c5_is_the_strong_split():
    assert bench.STRONG == {"c5"}
    assert dict(bench.EXTRAS)["c5"] == "c5_strong"
    _, kind, count, length = bench.CONFIGS["c5"]
    assert (kind, count, length) == ("fixed", 8 << 20, 1492)


def test_extras_order():
    names = [n for n, _ in bench.EXTRAS]
    assert names[0] == "c5"
    assert names[-3:] == ["c3", "fill_c3", "c4"]


def test_pmc_traffic_belongs_to_the_loaded_library(tmp_path, monkeypatch):
    """A PMC entry counts only when its sha256 stamp is the loaded libtcpck.so's
    (traffic from a kernel the product no longer ran)."""
    import json
    sha = bench.lib_sha256()
    entry = {"hbm_bytes_per_launch": 123, "source": "profiles/rX/pmc_c2_{fetch,write}.csv"}
    (tmp_path / "profiles").mkdir()
    for stamp, want in ((sha, 123), ("0" * 64, None), (None, None)):
        e = dict(entry, lib_sha256=stamp) if stamp else dict(entry)
        (tmp_path / "profiles" / "pmc_summary.json").write_text(json.dumps({"c2": e}))
        monkeypatch.setattr(bench, "ROOT", str(tmp_path))
        got, note = bench.pmc_traffic("c2")
        assert got == want, note
    got, note = bench.pmc_traffic("c9")
    assert got is None and "no PMC pass" in note


def test_metric_per_kind():
    for n, _ in bench.EXTRAS:
        kind = bench.CONFIGS[n][1] if n in bench.CONFIGS else bench.EXTRA[n][1]
        assert bench.metric_for(kind).startswith("GiB/s")


def _env_without_launcher():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["TCPCK_BENCH_BACKEND"] = "gloo"
    return env


def test_bare_gpus_n_spawns_n_ranks():
    """`python bench.py --gpus N` run bare (the driver's command
    has no launcher) must start N ranks, not print a 1-GPU line.  The launch
    check starts them through bench.py's own child torch.distributed.run and
    gathers every rank's (rank, local rank) over gloo -- no GPU."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=_env_without_launcher(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line == {"n_gpus": 2, "gpus_arg": 2, "ranks": [[0, 0], [1, 1]]}


@pytest.mark.parametrize("n", [4, 8])
def test_bare_gpus_4_and_8_spawn_their_ranks(n):
    """The driver's SCALE runs (N = 4, 8) through the same bare launch: N ranks,
    local ranks 0..N-1 (one device each on an 8-GPU node), over gloo on CPU."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, timeout=400, env=_env_without_launcher(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line == {"n_gpus": n, "gpus_arg": n, "ranks": [[i, i] for i in range(n)]}


def test_launcher_world_mismatch_fails():
    """A launcher that started another rank count than --gpus is an error (rc 2), not a silent N-line."""
    import subprocess
    env = _env_without_launcher()
    env.update(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120, env=env, cwd="/tmp")
    assert r.returncode == 2 and "WORLD_SIZE 3" in r.stderr


def test_failing_rank_fails_the_job():
    """a rank that dies must fail the job, not leave the
    others waiting in a collective for torch's default 10 minutes.  Bare
    `--gpus 2 --launch-check --fail-rank 1` over gloo: rank 1 exits 3 after
    joining the group, rank 0 waits in its all-reduce; the job must return
    non-zero well inside the process-group timeout (shortened to 60 s here)."""
    import subprocess
    import time
    env = _env_without_launcher()
    env["TCPCK_BENCH_PG_TIMEOUT"] = "60"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check",
                        "--fail-rank", "1"], capture_output=True, text=True, timeout=200, env=env, cwd="/tmp")
    assert r.returncode != 0, r.stdout
    assert time.monotonic() - t0 < 150
    assert "--fail-rank, exiting with status 3" in r.stderr


def test_device_check(monkeypatch):
    """The line proves its ranks sat on distinct devices:
    check_devices gathers every rank's device identity (PCI address + UUID);
    fewer distinct devices than ranks exits 3, unless the one-GPU rehearsal
    knob is set (then the line is marked a rehearsal); a rank whose runtime
    reports no identity makes the count unknown, never an error."""
    import pytest
    from tcpck import shard
    cases = (([(0x10300, 11), (0x10400, 12)], False, 2), ([(0x10300, 11), (0x10300, 11)], True, 1),
             ([(0x10300, 11), (0x10300, 11)], False, "exit"), ([(0, 0), (0, 0)], False, None))
    for ranks, rehearsal, want in cases:
        calls = []

        def gather(v, device=None, ranks=ranks, calls=calls):
            calls.append(v)  # first the PCI addresses, then the identity codes
            return [float(r[(len(calls) - 1) % 2]) for r in ranks]
        monkeypatch.setattr(bench, "device_identity", lambda i, r=ranks: r[0])
        monkeypatch.setattr(shard, "gather_ranks", gather)
        if want == "exit":
            with pytest.raises(SystemExit) as e:
                bench.check_devices(2, 0, "cpu", rehearsal)
            assert e.value.code == 3
            continue
        d = bench.check_devices(2, 0, "cpu", rehearsal)
        assert d["devices"] == want
        if want is not None:
            assert d["rehearsal"] == (want < 2) and d["device_ids"][0] == "0001:03:00"


def test_init_group_timeout(monkeypatch):
    """Every process group gets PG_TIMEOUT_S (or TCPCK_BENCH_PG_TIMEOUT), not torch's default."""
    import datetime
    import torch.distributed as dist
    seen = {}
    monkeypatch.setattr(dist, "init_process_group", lambda backend, **kw: seen.update(kw, backend=backend))
    monkeypatch.delenv("TCPCK_BENCH_PG_TIMEOUT", raising=False)
    bench.init_group("gloo")
    assert seen["timeout"] == datetime.timedelta(seconds=bench.PG_TIMEOUT_S) and "device_id" not in seen
    monkeypatch.setenv("TCPCK_BENCH_PG_TIMEOUT", "42")
    bench.init_group("nccl", "cuda:0")
    assert seen["timeout"] == datetime.timedelta(seconds=42) and seen["device_id"] == "cuda:0"


def _full_record(world=1):
    """A bench record as main() assembles it before compact_line, every prose
    field at its real length and every number at full width."""
    long = "x" * 240
    roof = {"bound": "hbm", "achieved": 7454.1234, "peak": 8000.0, "unit": "GB/s", "frac": 0.93181,
            "traffic": 1566653440, "traffic_source": long, "algorithmic_bytes_per_launch": 17180393472,
            "avg_launch_ms": 2.310341}
    if world > 1:
        roof["per_gpu_frac"] = [0.9318] * world
    cpu = {"unit": "GiB/s", "cores": 16, "affinity_cpus": 256, "nproc": 256, "omp_num_threads": 16,
           "value": 123.45, "min_GiBs": 120.01, "max_GiBs": 125.99, "passes_GiBs": [123.4] * 7, "kind": "reference",
           "match": True, "one_thread_GiBs": 9.87, "sample": "all 1048576 images (1.56 GB, host copy)",
           "sample_detail": long, "reference_O0_GiBs": 1.23, "reference_O0_note": long, "cpu_model": "A" * 48}
    rec = {"metric": bench.METRIC, "value": 6946.12, "unit": "GiB/s", "n_gpus": world, "steps": 20, "warmup": 5,
           "ms_per_step": 0.21199, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
           "data": "synthetic (device-generated: send-path headers + splitmix64 payloads, seed 42)",
           "config": {"workload": bench.CONFIGS["c2"][0], "images_per_gpu": 1 << 20, "image_bytes": 1492,
                      "bytes_per_gpu": 1564475392, "parallelism": "shard1 (independent per-GPU batches, no collective)"},
           "roofline": dict(roof), "settle": {"ms": 250.3, "launches": 1184},
           "devices": world, "device_ids": [f"0000:{0x11 + i:02x}:00" for i in range(world)],
           "one_arena": {"value": 6999.99, "frac": 0.9399}}
    for name, key in bench.EXTRAS:
        desc = bench.CONFIGS[name][0] if name in bench.CONFIGS else bench.EXTRA[name][0]
        kind = bench.CONFIGS[name][1] if name in bench.CONFIGS else bench.EXTRA[name][1]
        r = {"workload": desc, "metric": bench.metric_for(kind), "value": 6946.12, "unit": "GiB/s",
             "ms_per_step": 0.212345, "scaling": "strong" if name in bench.STRONG else "weak",
             "images_per_gpu": 4194304, "bytes_per_gpu": 3070000000, "roofline": dict(roof),
             "settle": {"ms": 250.3, "launches": 1184}}
        if name in bench.CPU_EXTRA:
            r["cpu_baseline"] = dict(cpu)
        if name in bench.STRONG:
            r.update(kernel_GiBs=6946.12, images_total=8 << 20, parallelism="shard8: " + long)
        if kind in ("slots", "receive"):
            r["same_ring"] = {"value": 5123.45, "frac": 0.7512}
        rec[key] = r
    rec["cpu_baseline"] = dict(cpu)
    rec["e2e"] = {"value": 49.19, "unit": "GiB/s", "match": True, "what": long}
    rec["c1"] = {"value": 2.812, "unit": "us/segment", "segments": 20000, "received": 20000, "verified": 20000,
                 "send_ck_ns": 123.4, "recv_ck_ns": 120.1,
                 "cpu_baseline": {"value": 2.9, "unit": "us/segment", "cores": 1, "kind": "reference",
                                  "verified": 20000, "send_ck_ns": 400.1, "recv_ck_ns": 390.2}}
    return rec


def test_line_fits_the_driver_tail():
    """the driver keeps ~8.3 KB of stdout; the line stays under
    bench.LINE_LIMIT (6 KB) with every key's numbers in it, at N=1 and N=8."""
    import json
    for world in (1, 8):
        line, detail = bench.compact_line(_full_record(world))
        text = json.dumps(line, separators=(",", ":"))
        assert len(text) < bench.LINE_LIMIT, len(text)
        for _, key in bench.EXTRAS:
            k = line[key]
            assert {"value", "ms_per_step", "roofline"} <= set(k), key
            assert {"frac", "achieved", "traffic", "algo_bytes", "launch_ms"} <= set(k["roofline"]), key
            assert "workload" in detail[key] and "metric" in detail[key]
        for key in ("c3", "c4", "c2_rfc"):
            assert {"value", "min_GiBs", "max_GiBs", "match", "kind", "cores"} <= set(line[key]["cpu_baseline"])
        # the contract's top-level fields
        for f in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "vs_baseline", "dtype", "data", "config"):
            assert f in line, f
        assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(line["roofline"])
        assert {"value", "unit", "cores", "kind", "sample"} <= set(line["cpu_baseline"])
        assert line["c1"]["verified"] == line["c1"]["segments"]
        assert line["receive"]["same_ring"]["frac"] > 0
        assert line["one_arena"]["frac"] > 0
        assert line["devices"] == world and len(detail["device_ids"]) == world
