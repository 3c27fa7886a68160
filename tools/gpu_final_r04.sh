# round-4 final validation on one MI355X: GPU suite, smoke, the bench lines (configs[2] default, [3] VCM,
# [4] conference 4K, [1] Cornell 1024, [0] Cornell PT), then the PMC profile rounds (tools/profile_round.sh)
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gputest.log 2>&1 || { tail -40 gpurun_out/final/gputest.log; exit 1; }
tail -2 gpurun_out/final/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
for c in 2 3 4 1 0; do
  extra=""; [ $c = 3 ] && extra="--method vcm"; [ $c = 4 ] && extra="--config 4 --steps 12 --warmup 3"
  [ $c = 1 ] && extra="--config 1"; [ $c = 0 ] && extra="--config 0"; [ $c = 3 ] && extra="--config 3"
  timeout -k 10 400 python -u bench.py $extra > gpurun_out/final/bench_c$c.json 2> gpurun_out/final/bench_c$c.err || { tail -20 gpurun_out/final/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/final/bench_c$c.json'));print('config $c', d['value'], d['ms_per_step'], d.get('cpu_baseline', {}).get('value'))"
done
