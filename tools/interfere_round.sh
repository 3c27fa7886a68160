#!/bin/bash
# round 6: the configs[4] row-partition per-rank frame with the collectives' local side run (tools/shard_model.py
# --interfere), fresh processes per N plus an in-process sweep; outputs under gpurun_out/$TAG
set -o pipefail
TAG=${TAG:-r06_interfere}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u tools/shard_model.py --pipelined --config 4 "$@" > $OUT/$n.txt 2>&1 || { tail -5 $OUT/$n.txt; exit 1; }
  grep -E "^N=|single" $OUT/$n.txt | cut -c1-330
}
run n8_plain 8
MODEL_RS_DEFER=0 run n8_link1 --interfere 153 32 8
MODEL_RS_DEFER=0 run n8_link7 --interfere 1071 32 8
MODEL_RS_DEFER=0 run sweep_link1 --interfere 153 32 1 2 4 8
