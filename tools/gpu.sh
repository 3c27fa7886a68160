#!/bin/bash
# One parameterised recipe for every GPU-box run (replaces the per-round one-off launchers).
# Run from the repo root through gpurun, e.g.
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh suite'
# Every GPU step runs under its own time limit and the steps are chained: the first failure ends
# the call (no retries).  Outputs go under gpurun_out/<TAG> (TAG defaults to the subcommand).
#
#   suite [-k SEL]                 pytest -m gpu (optionally a -k selection), smoke, the default bench line
#   bench CONF...                  bench lines of BASELINE configs (0..4; 4 = --config 4, 8 steps), with cpu_baseline
#   ab-env VAR "V1 V2" [ARGS]      alternating bench runs per value of an environment switch (REPS, default 2)
#   ab-lib "LIB1 LIB2" [ARGS]      alternating bench runs per in-tree build (cur = liborx.so, x = liborx_x.so)
#   profile TAG KEY [ARGS]         tools/profile_round.sh: PMC passes + kernel trace + the bench line
#   shard-model [ARGS]             tools/shard_model.py (per-rank cost of the row partition), ARGS passed on
#   timeline [ARGS]                rocprofv3 --kernel-trace of the pipelined bench (concurrency, gaps)
#   trav [SCENE METHOD [WxHxP]]    tools/trav_stats.py (needs the `make stats` build)
set -o pipefail
cmd=${1:?subcommand}; shift
TAG=${TAG:-$cmd}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

bench_line() { # file: print value, ms and the passes' (ms, serial ms)
  python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) if isinstance(v, dict) else v
                                           for k, v in d['passes'].items()}, d.get('cpu_baseline', {}).get('value'))"
}

case "$cmd" in
suite)
  SEL=""; [ "$1" = -k ] && SEL=$2
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${SEL:+-k "$SEL"} \
      > $OUT/gputest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/gputest.log | tail -40; exit 1; }
  tail -3 $OUT/gputest.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
      || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
      || { tail -20 $OUT/bench_default.err; exit 1; }
  bench_line $OUT/bench_default.json default ;;
bench)
  for c in "$@"; do
    extra="--config $c"; [ "$c" = 4 ] && extra="--config 4 --steps 8 --warmup 2"
    timeout -k 10 400 python -u bench.py $extra $BENCH_ARGS > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err \
        || { tail -20 $OUT/bench_c$c.err; exit 1; }
    bench_line $OUT/bench_c$c.json "config $c"
  done ;;
ab-env)
  var=$1; vals=$2; shift 2
  for rep in $(seq 1 ${REPS:-2}); do for v in $vals; do
    env $var=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/${v}_$rep.json 2> $OUT/err.txt \
        || { tail -5 $OUT/err.txt; exit 1; }
    bench_line $OUT/${v}_$rep.json "$var=$v rep $rep"
  done; done ;;
ab-lib)
  libs=$1; shift
  for rep in $(seq 1 ${REPS:-2}); do for n in $libs; do
    if [ "$n" = cur ]; then L=$PWD/oppositerenderer_amd/liborx.so; else L=$PWD/oppositerenderer_amd/liborx_$n.so; fi
    ORX_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/${n}_$rep.json 2> $OUT/err.txt \
        || { tail -5 $OUT/err.txt; exit 1; }
    bench_line $OUT/${n}_$rep.json "$n rep $rep"
  done; done ;;
profile)
  bash tools/profile_round.sh "$@" ;;
shard-model)
  timeout -k 10 600 python -u tools/shard_model.py "$@" > $OUT/model.txt 2>&1 || { tail -20 $OUT/model.txt; exit 1; }
  grep -v amdgpu.ids $OUT/model.txt | cut -c1-600 ;;
timeline)
  R=$PWD
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d $R/$OUT/tr -o run -- python3 $R/bench.py --steps 12 --warmup 4 \
      --no-cpu-baseline --no-serial-pass-times "$@" > $R/$OUT/b.json 2> $R/$OUT/err.txt) || { tail -5 $OUT/err.txt; exit 1; }
  db=$(python3 -c "import glob; print(sorted(glob.glob('$OUT/tr/**/*.db', recursive=True))[0])") || exit 1
  python3 tools/timeline_summary.py "$db" > $OUT/timeline.txt && cat $OUT/timeline.txt ;;
trav)
  timeout -k 10 300 python -u tools/trav_stats.py "$@" > $OUT/trav.txt 2>&1 || { tail -5 $OUT/trav.txt; exit 1; }
  grep -v amdgpu.ids $OUT/trav.txt ;;
*)
  echo "unknown subcommand $cmd" >&2; exit 2 ;;
esac
