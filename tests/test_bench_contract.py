"""bench.py's configuration tables (CPU only, no GPU calls): every config the
default run times beside C2 exists, its key is unique, C5 is the strong split,
and the extras keep the order that made each match its own process
(profiles/r03/bench_order_probe.log: C5 first, the 19 GB of C3 / C4 last)."""
import os
import sys

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
