# GPU suite (optionally a -k selection: $1), then smoke and the default bench line
set -o pipefail
mkdir -p gpurun_out/t
SEL=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/t/gputest.log 2>&1 || { tail -40 gpurun_out/t/gputest.log; exit 1; }
tail -3 gpurun_out/t/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 1; }
tail -1 gpurun_out/t/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/t/bench_default.json 2> gpurun_out/t/bench_default.err || { tail -20 gpurun_out/t/bench_default.err; exit 1; }
tail -1 gpurun_out/t/bench_default.json | cut -c1-300
