# round-4 profile refresh: PMC passes + kernel traces of the bench workloads (tools/profile_round.sh); the
# tables are folded locally from the merged gpurun_out/<tag> directories afterwards
set -eo pipefail
case "${1:-hall}" in
  hall) bash tools/profile_round.sh r04k_hall_ppm SyntheticHall:1920x1080:ppm:P2048
        bash tools/profile_round.sh r04k_hall_vcm SyntheticHall:1920x1080:vcm --method vcm --no-cpu-baseline ;;
  conf4k) STEPS=8 WARMUP=2 bash tools/profile_round.sh r04k_conf4k_ppm SyntheticConference:3840x2160:ppm:P4096 --config 4 --no-cpu-baseline ;;
esac
