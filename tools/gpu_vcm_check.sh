# VCM parity tests + the configs[3] bench line
set -o pipefail
mkdir -p gpurun_out/vcm
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "vcm or VCM" --timeout 300 --timeout-method thread > gpurun_out/vcm/test.log 2>&1 || { tail -40 gpurun_out/vcm/test.log; exit 1; }
tail -2 gpurun_out/vcm/test.log
timeout -k 10 300 python -u bench.py --method vcm --no-cpu-baseline > gpurun_out/vcm/bench.log 2>&1 && tail -1 gpurun_out/vcm/bench.log | cut -c1-900
# the roctx ranges of a short PPM run (marker trace beside the kernel trace)
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/vcm/markers -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-serial-pass-times > $GRAFT_REPO_ROOT/gpurun_out/vcm/markers.log 2>&1 && echo markers ok
