set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/bs_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/bs_ppm.json 2> gpurun_out/bs_ppm.err || exit 1
ORX_GRID_ATOMIC=1 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/bs_ppm_atomic.json 2> gpurun_out/bs_ppm_atomic.err || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --scene Cornell --width 1024 --height 1024 --photon-launch 1024 > gpurun_out/bs_cornell.json 2> gpurun_out/bs_cornell.err
