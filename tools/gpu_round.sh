set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
bash tools/profile_round.sh r01_hall_ppm "SyntheticHall:1920x1080:ppm:P2048" && \
bash tools/profile_round.sh r01_hall_vcm "SyntheticHall:1920x1080:vcm" --method vcm && \
timeout -k 10 600 python bench.py > gpurun_out/bench_hall_ppm.json 2> gpurun_out/bench_hall_ppm.err
