set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -k "ppm" > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/q_ppm.json 2> gpurun_out/q_ppm.err || exit 1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_hall3
timeout -k 10 600 rocprofv3 -i tools/pmc_passes.txt -d $OUT -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_hall3.log 2>&1
