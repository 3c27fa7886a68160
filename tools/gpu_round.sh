# final-tree check: GPU suite, smoke, hall PPM profile round (bench line + rocprof + PMC)
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -1 gpurun_out/t/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 1; }
tail -2 gpurun_out/t/smoke.log
timeout -k 10 900 bash tools/profile_round.sh r03g_hall_ppm SyntheticHall:1920x1080:ppm:P2048 > gpurun_out/prof_hall.log 2>&1 || { tail -20 gpurun_out/prof_hall.log; exit 1; }
tail -1 gpurun_out/r03g_hall_ppm/bench.json | cut -c1-300
