# A/B of two builds of liborx.so (ORX_LIB=oppositerenderer_amd/liborx_ab.so vs the tree's) on the hall PPM bench
# and configs[4]; alternating runs.  Usage: bash tools/gpu_ab_lib.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do for v in base new; do
  if [ $v = base ]; then export ORX_LIB=$PWD/oppositerenderer_amd/liborx_ab.so; else unset ORX_LIB; fi
  timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab/c2_${v}_$rep.json 2> gpurun_out/ab/err.txt || { tail -5 gpurun_out/ab/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/c2_${v}_$rep.json'));print('c2 $v(base=ab) rep $rep', d['value'], d['ms_per_step'], {k: v.get('serial_ms') for k, v in d['passes'].items()})"
done; done
for v in base new; do
  if [ $v = base ]; then export ORX_LIB=$PWD/oppositerenderer_amd/liborx_ab.so; else unset ORX_LIB; fi
  timeout -k 10 200 python -u bench.py --config 4 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab/c4_$v.json 2> gpurun_out/ab/err.txt || { tail -5 gpurun_out/ab/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/c4_$v.json'));print('c4 $v', d['value'], d['ms_per_step'], {k: v.get('serial_ms') for k, v in d['passes'].items()})"
done
