set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a/gputest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02a/gputest.log; exit 1; }
tail -3 gpurun_out/r02a/gputest.log
timeout -k 10 300 python -u bench.py > gpurun_out/r02a/bench.log 2>&1 && tail -1 gpurun_out/r02a/bench.log
