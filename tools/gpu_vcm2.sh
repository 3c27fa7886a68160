set -o pipefail
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -k "vcm or texture" > gpurun_out/vcm2_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --method vcm > gpurun_out/vcm2.json 2> gpurun_out/vcm2.err || exit 1
timeout -k 10 300 python tools/trav_stats.py SyntheticHall vcm > gpurun_out/trav_vcm.txt 2>&1
