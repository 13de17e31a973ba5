#!/usr/bin/env python3
"""Tabulate a slot_probe.py log: one row per layout x op, one column per kernel
(% of the roof in image bytes).   python scripts/probe_table.py LOG"""
import re
import sys
from collections import OrderedDict

rows = OrderedDict()
cols = []
for line in open(sys.argv[1]):
    m = re.match(r"(.+?)\s+(checksum|verify|fill)\s+(\S+)\s+([\d.]+) us\s+image bytes\s+([\d.]+) %", line)
    if not m:
        continue
    name, op, k, _, pct = m.groups()
    rows.setdefault((name, op), {})[k] = pct
    if k not in cols:
        cols.append(k)
print(f"{'layout':40s} {'op':8s} " + " ".join(f"{c:>6s}" for c in cols))
for (name, op), d in rows.items():
    print(f"{name:40s} {op:8s} " + " ".join(f"{d.get(c, '-'):>6s}" for c in cols))
