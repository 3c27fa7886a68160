set -o pipefail
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err || exit 1
ORX_PHOTON_PERSISTENT=1 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ab_pers.json 2> gpurun_out/ab_pers.err || exit 1
ORX_PHOTON_WAVEFRONT=1 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ab_wf.json 2> gpurun_out/ab_wf.err || exit 1
