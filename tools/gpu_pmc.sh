set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_hall2
timeout -k 10 600 rocprofv3 -i tools/pmc_passes.txt -d $OUT -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_hall2.log 2>&1
