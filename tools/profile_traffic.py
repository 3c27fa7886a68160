#!/usr/bin/env python3
"""Fold rocprofv3 PMC runs into profiles/traffic.json (HBM bytes per launch).

Usage: profile_traffic.py KEY FETCH_DIR WRITE_DIR [--out profiles/traffic.json]

FETCH_DIR / WRITE_DIR are the output directories of two separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of the same command
(TCC has 4 counter slots: FETCH_SIZE costs 3, WRITE_SIZE 2 — they cannot
share a pass).  Both counters are in KiB.  Per MI355X_MICROARCH.md
("HBM"), gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads,
so traffic = 2 * FETCH_SIZE + WRITE_SIZE; the fetch half of that is an
upper bound for narrower accesses (the guide leaves them uncalibrated).
KEY names the workload as bench.py does: "<scene>:<W>x<H>:<method>[:P<launch>]".
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sqlite3


def short(name):
    m = re.search(r"orx::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def load(d, counter):
    """Per-kernel list of `counter` values from a rocprofv3 output directory
    (CSV output, or the rocpd SQLite database that ROCm 7.2 writes by default)."""
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        for name, value in con.execute("select kernel_name, value from counters_collection where counter_name = ?",
                                       (counter,)):
            per[short(name)].append(float(value))
        con.close()
    return per


def kernel_stats(d, out_csv):
    """rocprofv3 --stats summary (top_kernels view of the rocpd database; durations in us) -> CSV."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        rows += con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
        con.close()
    with open(out_csv, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 3), round(r[3], 3), round(r[4], 3)])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--trace-dir", help="kernel-trace run: also write kernel_stats.csv next to --out")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "traffic.json"))
    a = ap.parse_args()
    fetch, write = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    table = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        table[k] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                    "bytes_per_launch": int((2 * f + w) * 1024), "launches": len(fetch.get(k, []))}
    try:
        allt = json.load(open(a.out))
    except (OSError, ValueError):
        allt = {}
    allt[a.key] = table
    json.dump(allt, open(a.out, "w"), indent=1, sort_keys=True)
    if a.trace_dir:
        kernel_stats(a.trace_dir, os.path.join(os.path.dirname(a.out), "kernel_stats.csv"))
    for k, v in table.items():
        print(f"{k:24s} {v['bytes_per_launch'] / 1e6:10.1f} MB/launch  ({v['launches']} launches)")


if __name__ == "__main__":
    main()
