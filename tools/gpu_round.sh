# round record: GPU test suite, rocprof kernel stats + PMC traffic for the
mkdir -p gpurun_out
# hall PPM / VCM workloads and Cornell 1024^2 PPM, then the default bench line
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
bash tools/profile_round.sh r01_hall_ppm "SyntheticHall:1920x1080:ppm:P2048" && \
bash tools/profile_round.sh r01_hall_vcm "SyntheticHall:1920x1080:vcm" --method vcm && \
bash tools/profile_round.sh r01_cornell_ppm "Cornell:1024x1024:ppm:P1024" --scene Cornell --width 1024 --height 1024 --photon-launch 1024 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_hall_ppm.json 2> gpurun_out/bench_hall_ppm.err && \
timeout -k 10 300 python bench.py --method vcm --no-cpu-baseline > gpurun_out/bench_hall_vcm.json 2> gpurun_out/bench_hall_vcm.err
