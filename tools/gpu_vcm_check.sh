# VCM parity tests + the configs[3] bench line
set -o pipefail
mkdir -p gpurun_out/vcm
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "vcm or VCM" --timeout 300 --timeout-method thread > gpurun_out/vcm/test.log 2>&1 || { tail -40 gpurun_out/vcm/test.log; exit 1; }
tail -2 gpurun_out/vcm/test.log
timeout -k 10 300 python -u bench.py --method vcm --no-cpu-baseline > gpurun_out/vcm/bench.log 2>&1 && tail -1 gpurun_out/vcm/bench.log | cut -c1-900
