#!/usr/bin/env python3
"""Cuts a kernel trace of scripts/fill_drain_probe.py into its phases (host
pauses > 20 ms) and prints, per phase, the mean duration of each kernel over
the phase's last K steps -- and, given a counter CSV, the mean counter value
per launch of each kernel in each phase.

    python scripts/fill_drain_summary.py TRACE.csv [--counters COUNTERS.csv] [--last 30]"""
import argparse
import csv
import re
import statistics


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--counters")
    ap.add_argument("--last", type=int, default=30)
    ap.add_argument("--names", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur, last_end = [], [], None
    for r in rows:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and st - last_end > 20_000_000:
            phases.append(cur)
            cur = []
        cur.append(r)
        last_end = en
    phases.append(cur)
    ctr = {}
    if a.counters:
        for r in csv.DictReader(open(a.counters)):
            ctr.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    names = a.names.split(",") if a.names else [f"phase{i}" for i in range(len(phases))]
    for i, ph in enumerate(phases):
        by = {}
        for r in ph:
            by.setdefault(short(r["Kernel_Name"]), []).append(r)
        label = names[i] if i < len(names) else f"phase{i}"
        parts = []
        for k, rs in by.items():
            tail = rs[-a.last:]
            d = statistics.mean((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tail)
            extra = ""
            if ctr:
                vals = {}
                for r in tail:
                    for cn, cv in ctr.get(int(r["Dispatch_Id"]), {}).items():
                        vals.setdefault(cn, []).append(cv)
                extra = " ".join(f"{cn}={statistics.mean(v):.0f}" for cn, v in vals.items())
            parts.append(f"{k} x{len(rs)} {d:.1f} us {extra}".rstrip())
        print(f"{label:16s} | " + " | ".join(parts))


if __name__ == "__main__":
    main()
