set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/bvh2_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/bvh2_dev.json 2> gpurun_out/bvh2_dev.err || exit 1
ORX_BVH_HOST=1 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/bvh2_host.json 2> gpurun_out/bvh2_host.err || exit 1
timeout -k 10 300 python tools/trav_stats.py SyntheticHall ppm > gpurun_out/trav_dev.txt 2>&1 || exit 1
ORX_BVH_HOST=1 timeout -k 10 300 python tools/trav_stats.py SyntheticHall ppm > gpurun_out/trav_host.txt 2>&1
