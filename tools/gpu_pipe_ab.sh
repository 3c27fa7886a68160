# A/B of the PPM pipelining and stream priorities on the hall bench
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 32 --warmup 4 --no-cpu-baseline 2>>gpurun_out/pipe_ab.err | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"; }
run ORX_PIPELINE=0 && run ORX_PIPELINE=1 ORX_GATHER_PRIORITY=0 && run ORX_PIPELINE=1 ORX_GATHER_PRIORITY=1 && \
run ORX_PIPELINE=1 ORX_GATHER_PRIORITY=1 ORX_MAIN_PRIORITY=1 && run ORX_PIPELINE=1 ORX_GATHER_PRIORITY=0 ORX_MAIN_PRIORITY=1
