#!/bin/bash
# Profile one bench workload on the GPU box: kernel trace + stats, then the
# two PMC passes for HBM traffic; summaries land in gpurun_out/<tag>/.
# usage: tools/profile_round.sh TAG KEY [bench args...]
set -eo pipefail
TAG=$1; KEY=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 8 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.log" 2>&1
python3 tools/profile_traffic.py "$KEY" "$OUT/fetch" "$OUT/write" --out "$OUT/traffic.json" --trace-dir "$OUT/trace" > "$OUT/traffic.txt"
