# A/B of the gather tile order on the pipelined benches (alternating runs)
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do for o in 0 8; do
  ORX_GATHER_ORDER=$o timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/ab/c2_o${o}_$rep.json 2> gpurun_out/ab/err.txt || { tail -5 gpurun_out/ab/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/c2_o${o}_$rep.json'));print('c2 order $o rep $rep', d['value'], d['ms_per_step'], 'gather serial', d['passes']['ppm_gather'].get('serial_ms'))"
done; done
for o in 0 8; do
  ORX_GATHER_ORDER=$o timeout -k 10 200 python -u bench.py --config 4 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab/c4_o$o.json 2> gpurun_out/ab/err.txt || { tail -5 gpurun_out/ab/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/c4_o$o.json'));print('c4 order $o', d['value'], d['ms_per_step'], 'gather serial', d['passes']['ppm_gather'].get('serial_ms'))"
done
