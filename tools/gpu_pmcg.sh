# PMC passes over the hall PPM bench (load-path counters for the gather)
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_g
timeout -k 10 600 rocprofv3 -i tools/pmc_gather2.txt -d $OUT -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_g.log 2>&1
