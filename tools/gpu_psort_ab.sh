# A/B: photon pass in launch order vs ordered by first-ray direction bins
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 32 --warmup 4 --no-cpu-baseline 2>>gpurun_out/psort_ab.err | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"; }
run ORX_PIPELINE=0 ORX_PHOTON_SORT=0 && run ORX_PIPELINE=0 ORX_PHOTON_SORT=1 && run ORX_PHOTON_SORT=0 && run ORX_PHOTON_SORT=1
