set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -k "vcm" > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --method vcm > gpurun_out/q_vcm.json 2> gpurun_out/q_ppm.err || exit 1
