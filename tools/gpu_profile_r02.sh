# r02 evidence: profiles of the hall PPM and VCM bench workloads + the configs[4] single-GPU line
set -eo pipefail
mkdir -p gpurun_out/r02b
bash tools/profile_round.sh r02_hall_ppm SyntheticHall:1920x1080:ppm:P2048
bash tools/profile_round.sh r02_hall_vcm SyntheticHall:1920x1080:vcm --method vcm
timeout -k 10 300 python -u bench.py --method vcm > gpurun_out/r02b/bench_vcm.log 2>&1
timeout -k 10 400 python -u bench.py --config 4 --steps 6 --warmup 2 > gpurun_out/r02b/bench_conf4k.log 2>&1
tail -1 gpurun_out/r02b/bench_vcm.log; tail -1 gpurun_out/r02b/bench_conf4k.log
