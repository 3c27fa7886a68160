#!/bin/bash
# Profile one bench workload on the GPU box, in the bench's own iteration window.
# usage: tools/profile_round.sh TAG KEY [bench args...]
#   TAG  output directory gpurun_out/<TAG>;  KEY  the workload key bench.py looks up
#        ("<scene>:<W>x<H>:<method>[:P<launch>][:<photon map>]")
# Passes (each its own rocprofv3 run of the same bench command; gfx950 PMC slot limits, no PMC
# beside trace domains): FETCH_SIZE, WRITE_SIZE, SQ, VALU mix, TA.  Their per-launch figures are
# the means over the bench's timed iterations (tools/profile_traffic.py windows) and fold into
# profiles/traffic.json + profiles/bound.json; then a --kernel-trace --stats run of the same
# command prints the bench line (which reads those tables) and its kernel_stats.csv gives every
# kernel's average over the timed iterations and over the serial leg, the windows the line's
# event times cover.  The VALU calibration kernels (tools/calib) run under the SQ and VALU passes
# once per box when profiles/valu_calib.json is absent or CALIB=1.
set -eo pipefail
TAG=$1; KEY=$2; shift 2
ROOTD=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOTD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
WARMUP=${WARMUP:-4}; STEPS=${STEPS:-32}
ARGS="--steps $STEPS --warmup $WARMUP $*"
BENCH="$ROOTD/bench.py --no-cpu-baseline $ARGS"
SQC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
VALUC="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
TAC="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
cd /tmp
if [ ! -f "$ROOTD/profiles/valu_calib.json" ] || [ "${CALIB:-0}" = 1 ]; then
    CAL=$ROOTD/tools/calib/valu_calib
    timeout -k 10 60 "$CAL" > "$OUT/calib_time.txt"
    timeout -s KILL 60 rocprofv3 --pmc $SQC -d "$OUT/calib_sq" -o run -- "$CAL" > "$OUT/calib_sq.log" 2>&1
    timeout -s KILL 60 rocprofv3 --pmc $VALUC -d "$OUT/calib_valu" -o run -- "$CAL" > "$OUT/calib_valu.log" 2>&1
    (cd "$ROOTD" && python3 tools/calib/calib_fold.py "$OUT/calib_sq" "$OUT/calib_valu" > "$OUT/calib.txt")
fi
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc $SQC -d "$OUT/sq" -o run -- python3 $BENCH > "$OUT/sq.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc $VALUC -d "$OUT/valu" -o run -- python3 $BENCH > "$OUT/valu.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc $TAC -d "$OUT/ta" -o run -- python3 $BENCH > "$OUT/ta.log" 2>&1
cd "$ROOTD"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace0" -o run -- python3 $BENCH > /dev/null 2> "$OUT/trace0.log"
python3 tools/profile_traffic.py "$KEY" "$OUT/fetch" "$OUT/write" --trace-dir "$OUT/trace0" --warmup "$WARMUP" \
    --steps "$STEPS" > "$OUT/traffic.txt"
python3 tools/pmc_bound.py "$KEY" --sq "$OUT/sq" --valu "$OUT/valu" --ta "$OUT/ta" --trace "$OUT/trace0" \
    --warmup "$WARMUP" --steps "$STEPS" > "$OUT/bound.txt"
# the bench line and its kernel trace from one run (the line reads the tables just written);
# cpu_baseline rides along unless the caller passes --no-cpu-baseline
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$ROOTD/bench.py" $ARGS \
    > "$OUT/bench.json" 2> "$OUT/trace.log"
cd "$ROOTD"
python3 -c "import sys; sys.path.insert(0, 'tools'); import profile_traffic as p; p.kernel_stats('$OUT/trace', '$OUT/kernel_stats.csv', $WARMUP, $STEPS)"
rm -f profiles/kernel_stats.csv
tail -1 "$OUT/bench.json" | cut -c1-400
