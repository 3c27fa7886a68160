#!/usr/bin/env python3
"""What bounds each kernel, from rocprofv3 PMC passes: profiles/bound.json.

Usage: pmc_bound.py KEY --sq SQ_DIR --ta TA_DIR --trace TRACE_DIR [--traffic profiles/traffic.json]
                        [--out profiles/bound.json]

SQ_DIR, TA_DIR: output directories of two separate `rocprofv3 --pmc` runs of the same
command (tools/profile_round.sh):
  SQ pass:  SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY
            SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  TA pass:  TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
TRACE_DIR: a --kernel-trace run (average duration per kernel, for the HBM fraction).
rocprofv3 serialises dispatches while it collects counters, so the figures describe each
kernel running alone (its stand-alone bound), not its overlapped schedule.

Per kernel (cycles = GRBM_GUI_ACTIVE / 8, the per-XCD busy cycles of the dispatch,
MI355X_MICROARCH.md "DVFS give-back"):
  valu_frac = SQ_INSTS_VALU x 2 / (1024 SIMDs x cycles)   a wave64 VALU instruction occupies its
                                                           SIMD-32 for 2 cycles (packed and
                                                           transcendental ones longer: a lower bound)
  ta_frac   = TA_TA_BUSY_sum / (256 CUs x cycles)          the vector-memory address unit
  hbm_frac  = (2 x FETCH_SIZE + WRITE_SIZE) / avg duration / 8 TB/s   (traffic.json, gfx950 correction)
  bound     = the largest of the three if it is >= 0.5, else "latency" (no unit near saturation:
              dependent memory latency and issue gaps dominate).
"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_traffic import load, short  # noqa: E402

import glob  # noqa: E402
import sqlite3  # noqa: E402

CUS, SIMDS, HBM_PEAK = 256, 1024, 8.0e12


def mean_counters(d, names):
    out = collections.defaultdict(dict)
    for n in names:
        for k, vals in load(d, n).items():
            out[k][n] = sum(vals) / len(vals)
    return out


def avg_durations_us(d):
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        for name, avg in con.execute("select name, average from top_kernels"):
            dur[short(name)] = float(avg)  # us (rocpd top_kernels)
        con.close()
    return dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("--sq", required=True)
    ap.add_argument("--ta", required=True)
    ap.add_argument("--trace", required=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--traffic", default=os.path.join(root, "profiles", "traffic.json"))
    ap.add_argument("--out", default=os.path.join(root, "profiles", "bound.json"))
    a = ap.parse_args()
    sq = mean_counters(a.sq, ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES",
                              "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"])
    ta = mean_counters(a.ta, ["TA_TA_BUSY_sum", "TA_BUFFER_READ_WAVEFRONTS_sum", "TCP_TOTAL_CACHE_ACCESSES_sum",
                              "GRBM_GUI_ACTIVE"])
    dur = avg_durations_us(a.trace)
    try:
        traffic = json.load(open(a.traffic)).get(a.key, {})
    except (OSError, ValueError):
        traffic = {}
    table = {}
    for k in sorted(set(sq) | set(ta)):
        if not k.startswith("k_"):
            continue
        s, t = sq.get(k, {}), ta.get(k, {})
        cyc_s = s.get("GRBM_GUI_ACTIVE", 0) / 8
        cyc_t = t.get("GRBM_GUI_ACTIVE", 0) / 8
        e = {}
        if cyc_s > 0 and "SQ_INSTS_VALU" in s:
            e["valu_frac"] = round(s["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc_s), 3)
            if s.get("SQ_WAVES"):
                e["valu_per_wave"] = round(s["SQ_INSTS_VALU"] / s["SQ_WAVES"], 1)
                e["vmem_rd_per_wave"] = round(s.get("SQ_INSTS_VMEM_RD", 0) / s["SQ_WAVES"], 1)
            if s.get("SQ_WAVE_CYCLES"):
                e["wait_frac"] = round(s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"], 3)
        if cyc_t > 0 and "TA_TA_BUSY_sum" in t:
            e["ta_frac"] = round(t["TA_TA_BUSY_sum"] / (CUS * cyc_t), 3)
            if t.get("TA_BUFFER_READ_WAVEFRONTS_sum"):
                e["ta_cycles_per_buffer_read"] = round(t["TA_TA_BUSY_sum"] / t["TA_BUFFER_READ_WAVEFRONTS_sum"], 1)
        if k in traffic and dur.get(k):
            e["hbm_frac"] = round(traffic[k]["bytes_per_launch"] / (dur[k] * 1e-6) / HBM_PEAK, 4)
        if dur.get(k):
            e["avg_us_profiled"] = round(dur[k], 2)
        units = {u: e[f"{u}_frac"] for u in ("valu", "ta", "hbm") if f"{u}_frac" in e}
        if units:
            top = max(units, key=units.get)
            e["bound"] = top if units[top] >= 0.5 else "latency"
            e["bound_source"] = "rocprofv3 PMC (stand-alone dispatch): " + ", ".join(
                f"{u} {v:.2f}" for u, v in units.items())
        table[k] = e
    try:
        allt = json.load(open(a.out))
    except (OSError, ValueError):
        allt = {}
    allt[a.key] = table
    json.dump(allt, open(a.out, "w"), indent=1, sort_keys=True)
    for k, v in table.items():
        print(f"{k:26s} {v.get('bound', '?'):8s} " + " ".join(f"{x}={v[x]}" for x in ("valu_frac", "ta_frac", "hbm_frac")
                                                          if x in v))


if __name__ == "__main__":
    main()
