# GPU suite, then an A/B of one switch on the default bench: tools/gpu_test_ab.sh VAR "v1 v2 ..." [pytest -k expr]
set -o pipefail
VAR=$1; VALS=$2; K=${3:-}
mkdir -p gpurun_out/t
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -2 gpurun_out/t/gputest.log
bash tools/gpu_ab.sh $VAR "$VALS"
