#!/usr/bin/env python3
"""What bounds each kernel, from rocprofv3 PMC passes: profiles/bound.json.

Usage: pmc_bound.py KEY --sq SQ_DIR --valu VALU_DIR --ta TA_DIR --trace TRACE_DIR
                        [--warmup W --steps K] [--calib CALIB_JSON]
                        [--traffic profiles/traffic.json] [--out profiles/bound.json]

SQ_DIR, VALU_DIR, TA_DIR: output directories of separate `rocprofv3 --pmc` runs of the same
command (tools/profile_round.sh):
  SQ pass:    SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY
              SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  VALU pass:  SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32
              SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE
  TA pass:    TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
TRACE_DIR: a --kernel-trace run of the same command (its overlapped schedule; kept for reference).
The HBM and fp32 fractions use the SQ pass's own dispatch durations: rocprofv3 serialises the
dispatches while it collects counters, so they are the kernels' stand-alone times.
With --warmup/--steps every per-launch figure is the mean over the bench's timed iterations
(profile_traffic.windows); setup kernels use all their dispatches.  Kernels are keyed by name
with template arguments (k_ppm_direct_output<1> and <2> are separate entries).
rocprofv3 serialises dispatches while it collects counters, so the figures describe each
kernel running alone (its stand-alone bound), not its overlapped schedule.

Per kernel (cycles = GRBM_GUI_ACTIVE / 8, the per-XCD busy cycles of the dispatch,
MI355X_MICROARCH.md "DVFS give-back"):
  valu_frac       = SQ_INSTS_VALU x 2 / (1024 SIMDs x cycles): the round-2 figure, at 2 cycles
                    per wave64 VALU instruction (half the calibrated cost: kept for comparison)
  valu_issue_frac = SQ_INSTS_VALU x valu_cycles / (1024 x cycles), valu_cycles the calibrated
                    issue cost of a wave64 VALU instruction (tools/calib/valu_calib.hip,
                    CALIB_JSON: 4 cycles on a SIMD-32, plain and packed fp32 alike)
  fp32_tflops     = SQ_INSTS_VALU_FLOPS_FP32 x 64 / duration (the counter books FLOPs per
                    wave-instruction: v_fma_f32 2, v_pk_fma_f32 4), against the 157.3 TF fp32
                    vector peak: fp32_frac
  ta_frac         = TA_TA_BUSY_sum / (256 CUs x cycles)          the vector-memory address unit
  hbm_frac        = (2 x FETCH_SIZE + WRITE_SIZE) / avg duration / 8 TB/s   (traffic.json)
  bound           = the largest of valu(_issue), ta, hbm if it is >= 0.5, else "latency".
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_traffic import load, pmc_durations_us, window_mean, windows  # noqa: E402

CUS, SIMDS, HBM_PEAK, FP32_PEAK_TF = 256, 1024, 8.0e12, 157.3
SQ = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
      "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]
VALU = ["SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32",
        "SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE"]
TA = ["TA_TA_BUSY_sum", "TA_BUFFER_READ_WAVEFRONTS_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "GRBM_GUI_ACTIVE"]


def mean_counters(d, names, warmup=None, steps=None):
    """{kernel: {counter: mean per dispatch}} over the bench's timed window when given."""
    out = {}
    for n in names:
        for k, vals in load(d, n).items():
            win = windows(len(vals), warmup, steps).get("timed") if warmup is not None else None
            out.setdefault(k, {})[n] = window_mean(vals, win) if win else sum(vals) / len(vals)
    return out


def mean_durations(d, warmup=None, steps=None):
    """Stand-alone dispatch durations from a PMC pass (dispatches serialised)."""
    out = {}
    for k, vals in pmc_durations_us(d).items():
        win = windows(len(vals), warmup, steps).get("timed") if warmup is not None else None
        out[k] = window_mean(vals, win) if win else sum(vals) / len(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("--sq", required=True)
    ap.add_argument("--valu")
    ap.add_argument("--ta", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--warmup", type=int)
    ap.add_argument("--steps", type=int)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--calib", default=os.path.join(root, "profiles", "valu_calib.json"))
    ap.add_argument("--traffic", default=os.path.join(root, "profiles", "traffic.json"))
    ap.add_argument("--out", default=os.path.join(root, "profiles", "bound.json"))
    a = ap.parse_args()
    sq = mean_counters(a.sq, SQ, a.warmup, a.steps)
    vm = mean_counters(a.valu, VALU, a.warmup, a.steps) if a.valu else {}
    ta = mean_counters(a.ta, TA, a.warmup, a.steps)
    dur = mean_durations(a.sq, a.warmup, a.steps)
    try:
        calib = json.load(open(a.calib))
    except (OSError, ValueError):
        calib = {}
    try:
        traffic = json.load(open(a.traffic)).get(a.key, {})
    except (OSError, ValueError):
        traffic = {}
    table = {}
    for k in sorted(set(sq) | set(ta)):
        if not k.startswith("k_"):
            continue
        s, t, v = sq.get(k, {}), ta.get(k, {}), vm.get(k, {})
        cyc_s = s.get("GRBM_GUI_ACTIVE", 0) / 8
        cyc_t = t.get("GRBM_GUI_ACTIVE", 0) / 8
        cyc_v = v.get("GRBM_GUI_ACTIVE", 0) / 8
        e = {}
        if cyc_s > 0 and "SQ_INSTS_VALU" in s:
            e["valu_frac"] = round(s["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc_s), 3)
            if s.get("SQ_WAVES"):
                e["valu_per_wave"] = round(s["SQ_INSTS_VALU"] / s["SQ_WAVES"], 1)
                e["vmem_rd_per_wave"] = round(s.get("SQ_INSTS_VMEM_RD", 0) / s["SQ_WAVES"], 1)
            if s.get("SQ_WAVE_CYCLES"):
                e["wait_frac"] = round(s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"], 3)
        if cyc_s > 0 and calib.get("valu_cycles") and "SQ_INSTS_VALU" in s:
            e["valu_issue_frac"] = round(s["SQ_INSTS_VALU"] * calib["valu_cycles"] / (SIMDS * cyc_s), 3)
        if cyc_v > 0 and dur.get(k) and "SQ_INSTS_VALU_FLOPS_FP32" in v:
            tf = v["SQ_INSTS_VALU_FLOPS_FP32"] * 64 / (dur[k] * 1e-6) / 1e12
            e["fp32_tflops"] = round(tf, 2)
            e["fp32_frac"] = round(tf / FP32_PEAK_TF, 4)
        if cyc_t > 0 and "TA_TA_BUSY_sum" in t:
            e["ta_frac"] = round(t["TA_TA_BUSY_sum"] / (CUS * cyc_t), 3)
            if t.get("TA_BUFFER_READ_WAVEFRONTS_sum"):
                e["ta_cycles_per_buffer_read"] = round(t["TA_TA_BUSY_sum"] / t["TA_BUFFER_READ_WAVEFRONTS_sum"], 1)
        if k in traffic and dur.get(k):
            e["hbm_frac"] = round(traffic[k]["bytes_per_launch"] / (dur[k] * 1e-6) / HBM_PEAK, 4)
        if dur.get(k):
            e["avg_us_standalone"] = round(dur[k], 2)
        units = {}
        if "valu_issue_frac" in e:
            units["valu"] = e["valu_issue_frac"]
        elif "valu_frac" in e:
            units["valu"] = e["valu_frac"]
        for u in ("ta", "hbm"):
            if f"{u}_frac" in e:
                units[u] = e[f"{u}_frac"]
        if units:
            top = max(units, key=units.get)
            e["bound"] = top if units[top] >= 0.5 else "latency"
            e["bound_source"] = "rocprofv3 PMC (stand-alone dispatch, bench timed window): " + ", ".join(
                f"{u} {val:.2f}" for u, val in units.items())
        table[k] = e
    try:
        allt = json.load(open(a.out))
    except (OSError, ValueError):
        allt = {}
    allt[a.key] = table
    json.dump(allt, open(a.out, "w"), indent=1, sort_keys=True)
    for k, v in table.items():
        print(f"{k:34s} {v.get('bound', '?'):8s} " + " ".join(
            f"{x}={v[x]}" for x in ("valu_frac", "valu_issue_frac", "ta_frac", "hbm_frac") if x in v))


if __name__ == "__main__":
    main()
