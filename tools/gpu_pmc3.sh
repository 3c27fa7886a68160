# PMC passes over the wavefront photon pass (hall PPM)
set -o pipefail
export TMPDIR=/tmp
export ORX_PHOTON_WAVEFRONT=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_wf
timeout -k 10 600 rocprofv3 -i tools/pmc_photon.txt -d $OUT -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_wf.log 2>&1
