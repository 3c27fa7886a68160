set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_features.py -m gpu -x -q --timeout 200 --timeout-method thread -k "vcm or VCM" > gpurun_out/t/gt.log 2>&1 || { tail -30 gpurun_out/t/gt.log; exit 1; }
tail -2 gpurun_out/t/gt.log
bash tools/gpu_lib_ab.sh "base cur base cur" --method vcm --steps 16 --warmup 2
