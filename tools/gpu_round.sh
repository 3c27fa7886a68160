set -o pipefail
timeout -k 10 900 bash tools/profile_round.sh r03f_hall SyntheticHall:1920x1080:ppm:P2048 > gpurun_out/prof_hall.log 2>&1 || { tail -20 gpurun_out/prof_hall.log; exit 1; }
tail -3 gpurun_out/prof_hall.log | cut -c1-300
