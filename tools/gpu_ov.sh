set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/ov_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ov_on.json 2> gpurun_out/ov_on.err || exit 1
ORX_OVERLAP_DIRECT=0 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ov_off.json 2> gpurun_out/ov_off.err || exit 1
