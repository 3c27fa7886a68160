#!/usr/bin/env python3
"""Fold the VALU calibration runs (tools/calib/valu_calib.hip under the SQ and VALU-mix PMC
passes of tools/profile_round.sh) into profiles/valu_calib.json, the per-instruction costs
tools/pmc_bound.py prices VALU issue with.

usage: calib_fold.py SQ_DIR VALU_DIR [--out profiles/valu_calib.json]

Each calibration kernel is a dependency-free stream of one instruction kind at 8 waves per
SIMD, so the chip's SIMDs issue it back to back: cycles per wave-instruction per SIMD =
(GRBM_GUI_ACTIVE / 8) x 1024 / SQ_INSTS_VALU.  The packed kernels also say how the FLOPS
counter books a packed instruction: extra FLOPs per lane beyond the plain form the
instruction-kind counters (FMA/MUL) file it under."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pmc_bound import SQ, VALU, mean_counters  # noqa: E402

SIMDS = 1024
BLOCKS, WAVES_PER_BLOCK, ITERS, CHAINS = 256 * 8, 4, 2048, 8
STREAM = BLOCKS * WAVES_PER_BLOCK * ITERS * CHAINS  # wave-instructions of the measured kind


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq")
    ap.add_argument("valu")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), "profiles", "valu_calib.json"))
    a = ap.parse_args()
    sq, vm = mean_counters(a.sq, SQ), mean_counters(a.valu, VALU)
    res = {"source": "tools/calib/valu_calib.hip: dependency-free streams of one instruction kind, "
                     "8 waves/SIMD, rocprofv3 PMC (GRBM_GUI_ACTIVE, SQ_INSTS_VALU*, SQ_INSTS_VALU_FLOPS_FP32)"}
    per = {}
    for k in ("k_cal_fma", "k_cal_pk_fma", "k_cal_mul", "k_cal_pk_mul"):
        s, v = sq.get(k, {}), vm.get(k, {})
        if not s or not v:
            continue
        cyc = s["GRBM_GUI_ACTIVE"] / 8
        per[k] = {"cycles_per_wave_instruction": round(cyc * SIMDS / s["SQ_INSTS_VALU"], 3),
                  "insts_valu": s["SQ_INSTS_VALU"], "stream_instructions": STREAM,
                  "fma_f32": v.get("SQ_INSTS_VALU_FMA_F32"), "mul_f32": v.get("SQ_INSTS_VALU_MUL_F32"),
                  "add_f32": v.get("SQ_INSTS_VALU_ADD_F32"), "flops_fp32": v.get("SQ_INSTS_VALU_FLOPS_FP32"),
                  "active_inst_valu": s.get("SQ_ACTIVE_INST_VALU")}
    res["kernels"] = per
    if "k_cal_fma" in per:
        f = per["k_cal_fma"]
        # SQ_ACTIVE_INST_VALU counts quad-cycles: one per wave-instruction of the stream, i.e. a
        # wave64 VALU instruction holds its SIMD-32 for 4 cycles; the stream's wall cycles per
        # instruction (GRBM) agree up to the loop overhead
        res["valu_cycles"] = round(4.0 * (f["active_inst_valu"] or 0) / f["insts_valu"], 3)
        res["plain_cycles_measured"] = f["cycles_per_wave_instruction"]
    if "k_cal_pk_fma" in per:
        p = per["k_cal_pk_fma"]
        res["packed_cycles_measured"] = p["cycles_per_wave_instruction"]
        # the FLOPS counter books per wave-instruction (not per lane): v_fma_f32 2, v_pk_fma_f32 4
        plain = 2 * (p["fma_f32"] or 0) + (p["add_f32"] or 0) + (p["mul_f32"] or 0)
        res["packed_fma_extra_flops"] = round(((p["flops_fp32"] or 0) - plain) / STREAM, 3)
    if "k_cal_pk_mul" in per:
        p = per["k_cal_pk_mul"]
        res["packed_mul_cycles_measured"] = p["cycles_per_wave_instruction"]
        plain = 2 * (p["fma_f32"] or 0) + (p["add_f32"] or 0) + (p["mul_f32"] or 0)
        res["packed_mul_extra_flops"] = round(((p["flops_fp32"] or 0) - plain) / STREAM, 3)
    res["note"] = ("packed fp32 (v_pk_fma_f32, v_pk_mul_f32) issues at the cost of the plain instruction "
                   "(4 cycles per wave64 on a SIMD-32), so VALU issue = SQ_INSTS_VALU x valu_cycles; the fp32 "
                   "vector peak (157.3 TF) needs packed instructions")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
