# A/B: one photon per lane vs persistent refill (photon pass)
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 16 --warmup 3 --no-cpu-baseline 2>>gpurun_out/photon_ab.err | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"; }
run ORX_PIPELINE=0 ORX_PHOTON_PERSISTENT=0 && run ORX_PIPELINE=0 ORX_PHOTON_PERSISTENT=1 && run ORX_PHOTON_PERSISTENT=1
