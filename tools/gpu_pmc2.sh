# PMC passes over a short hall PPM + VCM bench (kernel counters for the traversal kernels)
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_r1b
timeout -k 10 600 rocprofv3 -i tools/pmc_photon.txt -d $OUT -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_r1b.log 2>&1
