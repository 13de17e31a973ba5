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
    assert names[-2:] == ["c3", "c4"]


def test_metric_per_kind():
    for n, _ in bench.EXTRAS:
        kind = bench.CONFIGS[n][1] if n in bench.CONFIGS else bench.EXTRA[n][1]
        assert bench.metric_for(kind).startswith("GiB/s")
