# final-tree hall PPM profile round (bench line + rocprof + PMC)
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 900 bash tools/profile_round.sh r03j_hall_ppm SyntheticHall:1920x1080:ppm:P2048 > gpurun_out/prof_hall.log 2>&1 || { tail -20 gpurun_out/prof_hall.log; exit 1; }
tail -1 gpurun_out/r03j_hall_ppm/bench.json | cut -c1-200
