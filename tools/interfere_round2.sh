#!/bin/bash
# round 6: configs[4] N=8 per-rank frame with the collectives' local side (tools/shard_model.py --interfere),
# ShardedPPM's schedule (reduce-scatter behind the next all-gather, finish on its own stream: the default);
# fresh processes, then the in-process sweep at 8 and 16 hardware queues; outputs under gpurun_out/$TAG
set -o pipefail
TAG=${TAG:-r06_interfere2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { local n=$1; shift
  timeout -k 10 400 python -u tools/shard_model.py --pipelined --config 4 "$@" > $OUT/$n.txt 2>&1 || { tail -5 $OUT/$n.txt; exit 1; }
  grep -E "^N=|single" $OUT/$n.txt | cut -c1-330; }
run n8_defer_link1 --interfere 153 32 8
run n8_defer_link7 --interfere 1071 32 8
run sweep_defer_link1 --interfere 153 32 1 2 4 8
GPU_MAX_HW_QUEUES=16 run sweep_defer_link1_q16 --interfere 153 32 1 2 4 8
