# A/B: cap the overlapped gather's blocks per CU with unused dynamic LDS
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 32 --warmup 4 --no-cpu-baseline 2>>gpurun_out/pad_ab.err | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"; }
run ORX_GATHER_LDS_PAD_KB=0 && run ORX_GATHER_LDS_PAD_KB=24 && run ORX_GATHER_LDS_PAD_KB=40 && run ORX_GATHER_LDS_PAD_KB=56 && run ORX_GATHER_LDS_PAD_KB=80
