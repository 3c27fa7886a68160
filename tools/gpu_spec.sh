set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/spec_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/spec_ppm.json 2> gpurun_out/spec_ppm.err || exit 1
ORX_PHOTON_WAVEFRONT=1 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/spec_ppm_wf.json 2> gpurun_out/spec_ppm_wf.err || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --method vcm > gpurun_out/spec_vcm.json 2> gpurun_out/spec_vcm.err || exit 1
timeout -k 10 300 python tools/trav_stats.py SyntheticHall ppm > gpurun_out/trav_hall.txt 2>&1
