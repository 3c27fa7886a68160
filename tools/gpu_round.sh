# final-tree check after the 7-wave gather: GPU suite, smoke, 4K profile round, shard model
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -1 gpurun_out/t/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 1; }
tail -1 gpurun_out/t/smoke.log
WARMUP=2 STEPS=8 timeout -k 10 900 bash tools/profile_round.sh r03j_conf4k SyntheticConference:3840x2160:ppm:P4096 --config 4 > gpurun_out/prof_4k.log 2>&1 || { tail -20 gpurun_out/prof_4k.log; exit 1; }
tail -1 gpurun_out/r03j_conf4k/bench.json | cut -c1-200
timeout -k 10 500 python -u tools/shard_model.py --config 4 > gpurun_out/t/sm_conf4k.txt 2>&1 || { tail -5 gpurun_out/t/sm_conf4k.txt; exit 1; }
grep "per-rank" gpurun_out/t/sm_conf4k.txt | cut -c1-120
timeout -k 10 400 python -u bench.py > gpurun_out/t/bench_default.json 2> gpurun_out/t/bench_default.err || { tail -20 gpurun_out/t/bench_default.err; exit 1; }
tail -1 gpurun_out/t/bench_default.json | cut -c1-200
