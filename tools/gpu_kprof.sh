# kernel-trace profile of the default hall PPM bench -> gpurun_out/kprof
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${KPROF_NAME:-kprof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${KPROF_NAME:-kprof}.log 2>&1
