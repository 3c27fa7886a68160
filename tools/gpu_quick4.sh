set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_sharded.py -x -q -k "ppm or shard" > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/q_ppm.json 2> gpurun_out/q_ppm.err || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --scene Cornell --width 1024 --height 1024 --photon-launch 1024 > gpurun_out/q_cornell.json 2> gpurun_out/q_ppm.err || exit 1
