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
    """Kernel key: the name with its template arguments (k_ppm_direct_output<1> and <2> are
    different kernels and must not pool), without namespace and parameter list."""
    m = re.search(r"orx::(\w+(?:<[^>(]*>)?)", name)
    return m.group(1) if m else name.split("(")[0]


def load(d, counter):
    """Per-kernel list of `counter` values in dispatch order from a rocprofv3 output directory
    (CSV output, or the rocpd SQLite database that ROCm 7.2 writes by default)."""
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        for r in rows:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        q = ("select kernel_name, sum(value) from counters_collection where counter_name = ? "
             "group by dispatch_id order by dispatch_id")
        for name, value in con.execute(q, (counter,)):
            per[short(name)].append(float(value))
        con.close()
    return per


def durations_us(d):
    """Per-kernel list of dispatch durations (us) in start order from a --kernel-trace run."""
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        for name, dur in con.execute("select name, duration from kernels order by start"):
            per[short(name)].append(float(dur) * 1e-3)
        con.close()
    return per


def pmc_durations_us(d):
    """Per-kernel dispatch durations (us) in dispatch order from a PMC run: rocprofv3 serialises
    the dispatches while it collects counters, so these are the kernels' stand-alone times."""
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        q = "select kernel_name, max(duration) from counters_collection group by dispatch_id order by dispatch_id"
        for name, dur in con.execute(q):
            per[short(name)].append(float(dur) * 1e-3)
        con.close()
    return per


def windows(n, warmup, steps):
    """The bench's iteration windows over a kernel's n per-iteration dispatches: `timed` =
    the timed steps [warmup, warmup + steps); `serial` = the three measured iterations of the
    serial leg bench.py runs after a pipelined timed region (one untimed iteration first).
    Kernels whose dispatch count is not per-iteration (setup) get no window."""
    w = {}
    if n in (warmup + steps, warmup + steps + 4):
        w["timed"] = (warmup, warmup + steps)
    if n == warmup + steps + 4:
        w["serial"] = (warmup + steps + 1, warmup + steps + 4)
    return w


def window_mean(vals, win):
    a, b = win
    sel = vals[a:b]
    return sum(sel) / len(sel) if sel else None


def kernel_stats(d, out_csv, warmup=None, steps=None):
    """rocprofv3 --kernel-trace summary -> CSV: every kernel's calls and average duration, and,
    given the bench's warmup/steps, the averages over the timed iterations and over the serial
    leg (the windows bench.py's event times cover)."""
    per = durations_us(d)
    rows = []
    for k, v in per.items():
        row = [k, len(v), round(sum(v), 3), round(sum(v) / len(v), 3)]
        win = windows(len(v), warmup, steps) if warmup is not None else {}
        for name in ("timed", "serial"):
            if name in win:
                row += [win[name][1] - win[name][0], round(window_mean(v, win[name]), 3)]
            else:
                row += ["", ""]
        rows.append(row)
    rows.sort(key=lambda r: -r[2])
    with open(out_csv, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "TimedCalls", "TimedAverageUs", "SerialCalls",
                    "SerialAverageUs"])
        w.writerows(rows)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--trace-dir", help="kernel-trace run: also write kernel_stats.csv next to --out")
    ap.add_argument("--warmup", type=int, help="bench warmup iterations: per-launch figures over the timed window")
    ap.add_argument("--steps", type=int)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "traffic.json"))
    a = ap.parse_args()
    fetch, write = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    table = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        fv, wv = fetch.get(k, [0.0]), write.get(k, [0.0])
        win = windows(len(fv), a.warmup, a.steps).get("timed") if a.warmup is not None else None
        f = window_mean(fv, win) if win else sum(fv) / len(fv)
        w = (window_mean(wv, win) if win and len(wv) == len(fv) else sum(wv) / len(wv))
        table[k] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                    "bytes_per_launch": int((2 * f + w) * 1024), "launches": len(fv),
                    "window": "timed iterations" if win else "all launches"}
    try:
        allt = json.load(open(a.out))
    except (OSError, ValueError):
        allt = {}
    allt[a.key] = table
    json.dump(allt, open(a.out, "w"), indent=1, sort_keys=True)
    if a.trace_dir:
        kernel_stats(a.trace_dir, os.path.join(os.path.dirname(a.out), "kernel_stats.csv"), a.warmup, a.steps)
    for k, v in table.items():
        print(f"{k:32s} {v['bytes_per_launch'] / 1e6:10.1f} MB/launch  ({v['launches']} launches, {v['window']})")


if __name__ == "__main__":
    main()
