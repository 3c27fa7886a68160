# round 4: gather tile order (ORX_GATHER_ORDER) at configs[4] and [2]: serial gather time + FETCH_SIZE;
# sharded-cell variants in the shard model
set -o pipefail
mkdir -p gpurun_out/ord
export TMPDIR=/tmp
R=$PWD
for o in 0 8 16; do
  ORX_GATHER_ORDER=$o timeout -k 10 200 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ord/c4_o$o.json 2> gpurun_out/ord/c4_o$o.err || { tail -5 gpurun_out/ord/c4_o$o.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ord/c4_o$o.json'));p=d['passes'];print('c4 order $o', d['value'], d['ms_per_step'], {k:(v['ms'],v.get('serial_ms')) for k,v in p.items()})"
  (cd /tmp && ORX_GATHER_ORDER=$o timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/ord/f_c4_o$o -o run -- python3 $R/bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-serial-pass-times > $R/gpurun_out/ord/f_c4_o$o.log 2>&1) || { tail -5 gpurun_out/ord/f_c4_o$o.log; exit 1; }
  python3 -c "
import sys; sys.path.insert(0,'tools'); import profile_traffic as p, statistics as s
per=p.load('gpurun_out/ord/f_c4_o$o','FETCH_SIZE')
for k,v in per.items():
    if 'gather' in k: print('  fetch', k, len(v), 'launches, mean', round(2*s.mean(v)*1024/1e9,2), 'GB (2xFETCH)')
"
done
for o in 0 8; do
  ORX_GATHER_ORDER=$o timeout -k 10 120 python -u bench.py --steps 16 --warmup 4 --no-cpu-baseline > gpurun_out/ord/c2_o$o.json 2> gpurun_out/ord/c2_o$o.err || { tail -5 gpurun_out/ord/c2_o$o.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ord/c2_o$o.json'));p=d['passes'];print('c2 order $o', d['value'], d['ms_per_step'], {k:(v['ms'],v.get('serial_ms')) for k,v in p.items()})"
done
MODEL_GATHER_VARIANT=2 timeout -k 10 200 python -u tools/shard_model.py --config 4 8 > gpurun_out/ord/sm_c4_scaled_sub.txt 2>&1 && grep N= gpurun_out/ord/sm_c4_scaled_sub.txt | cut -c1-330
ORX_SHARD_CELLS=1 MODEL_GATHER_VARIANT=2 timeout -k 10 200 python -u tools/shard_model.py --config 4 8 > gpurun_out/ord/sm_c4_unscaled_sub.txt 2>&1 && grep N= gpurun_out/ord/sm_c4_unscaled_sub.txt | cut -c1-330
ORX_SHARD_CELLS=1 timeout -k 10 200 python -u tools/shard_model.py --config 4 8 > gpurun_out/ord/sm_c4_unscaled.txt 2>&1 && grep N= gpurun_out/ord/sm_c4_unscaled.txt | cut -c1-330
MODEL_GATHER_VARIANT=2 timeout -k 10 200 python -u tools/shard_model.py 8 > gpurun_out/ord/sm_c2_scaled_sub.txt 2>&1 && grep N= gpurun_out/ord/sm_c2_scaled_sub.txt | cut -c1-330
