# kernel-trace profile of the wavefront photon pass (hall PPM)
set -o pipefail
export TMPDIR=/tmp
export ORX_PHOTON_WAVEFRONT=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/wfprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/wfprof.log 2>&1
