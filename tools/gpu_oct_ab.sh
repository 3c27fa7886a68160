# A/B: octahedral normal-test prefilter in the grid gather (serial and pipelined)
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 32 --warmup 4 --no-cpu-baseline 2>>gpurun_out/oct_ab.err | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"; }
run ORX_PIPELINE=0 ORX_GATHER_OCT=0 && run ORX_PIPELINE=0 ORX_GATHER_OCT=1 && run ORX_GATHER_OCT=0 && run ORX_GATHER_OCT=1
