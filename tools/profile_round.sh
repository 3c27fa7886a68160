#!/bin/bash
# Profile one bench workload on the GPU box: kernel trace + stats, the two PMC passes for
# HBM traffic, and the SQ / TA passes for the bound; each rocprofv3 pass is its own run
# (gfx950 slot limits; no PMC beside trace domains).  Summaries land in gpurun_out/<tag>/,
# profiles/traffic.json and profiles/bound.json get the workload's entry.
# (kernel_stats.csv: the bench's timed schedule; kernel_stats_serial.csv: ORX_PIPELINE=0, whose
# stand-alone durations the bound's HBM fraction uses)
# usage: tools/profile_round.sh TAG KEY [bench args...]
set -eo pipefail
TAG=$1; KEY=$2; shift 2
ROOTD=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOTD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$ROOTD/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-serial-pass-times $*"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.log" 2>&1
ORX_PIPELINE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_serial" -o run -- python3 $BENCH \
    > "$OUT/trace_serial.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/sq" -o run -- python3 $BENCH > "$OUT/sq.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    GRBM_GUI_ACTIVE -d "$OUT/ta" -o run -- python3 $BENCH > "$OUT/ta.log" 2>&1
cd "$ROOTD"
python3 tools/profile_traffic.py "$KEY" "$OUT/fetch" "$OUT/write" --trace-dir "$OUT/trace" > "$OUT/traffic.txt"
mv profiles/kernel_stats.csv "$OUT/kernel_stats.csv"
python3 -c "import sys; sys.path.insert(0, 'tools'); import profile_traffic as p; p.kernel_stats('$OUT/trace_serial', '$OUT/kernel_stats_serial.csv')"
python3 tools/pmc_bound.py "$KEY" --sq "$OUT/sq" --ta "$OUT/ta" --trace "$OUT/trace_serial" > "$OUT/bound.txt"
