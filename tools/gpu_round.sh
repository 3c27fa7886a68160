set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -2 gpurun_out/t/gputest.log
bash tools/gpu_lib_ab.sh "base cur" --steps 24 --warmup 4 && bash tools/gpu_lib_ab.sh "base cur" --config 4 --steps 8 --warmup 2
