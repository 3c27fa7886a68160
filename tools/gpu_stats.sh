set -o pipefail
timeout -k 10 300 python tools/trav_stats.py SyntheticHall ppm > gpurun_out/trav_hall.txt 2>&1 && \
timeout -k 10 300 python tools/trav_stats.py SyntheticHall vcm > gpurun_out/trav_hall_vcm.txt 2>&1
