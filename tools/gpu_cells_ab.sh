# A/B: k_bs_cells block size (co-scheduling beside the overlapped gather)
mkdir -p gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 32 --warmup 4 --no-cpu-baseline 2>>gpurun_out/cells_ab.err | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"; }
run ORX_BS_CELLS_THREADS=1024 && run ORX_BS_CELLS_THREADS=512 && run ORX_BS_CELLS_THREADS=256 && run ORX_PIPELINE=0 ORX_BS_CELLS_THREADS=256 && run ORX_PIPELINE=0 ORX_BS_CELLS_THREADS=1024
