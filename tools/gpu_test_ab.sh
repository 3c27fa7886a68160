# full GPU suite on the current liborx.so, then an A/B of in-tree libs: tools/gpu_test_ab.sh "base cur" [bench args]
set -o pipefail
LIBS=$1; shift
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -2 gpurun_out/t/gputest.log
bash tools/gpu_lib_ab.sh "$LIBS" "$@"
