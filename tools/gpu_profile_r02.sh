# r02 evidence: profiles of the hall PPM and VCM bench workloads + the bench lines of configs[2]-[4]
set -eo pipefail
T=${1:-r02c}
mkdir -p gpurun_out/$T
bash tools/profile_round.sh ${T}_hall_ppm SyntheticHall:1920x1080:ppm:P2048
bash tools/profile_round.sh ${T}_hall_vcm SyntheticHall:1920x1080:vcm --method vcm
timeout -k 10 300 python -u bench.py > gpurun_out/$T/bench_ppm.log 2>&1
timeout -k 10 300 python -u bench.py --method vcm > gpurun_out/$T/bench_vcm.log 2>&1
timeout -k 10 400 python -u bench.py --config 4 --steps 6 --warmup 2 > gpurun_out/$T/bench_conf4k.log 2>&1
tail -1 gpurun_out/$T/bench_ppm.log | cut -c1-400; tail -1 gpurun_out/$T/bench_vcm.log | cut -c1-300; tail -1 gpurun_out/$T/bench_conf4k.log | cut -c1-300
