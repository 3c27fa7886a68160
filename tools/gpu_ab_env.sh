# A/B of an environment knob on the hall PPM bench (configs[2]) and configs[4], alternating runs.
# Usage: REPS=3 bash tools/gpu_ab_env.sh VAR VALUE_A VALUE_B [extra bench args]
set -o pipefail
var=$1; a=$2; b=$3; shift 3
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do for v in $a $b; do
  env $var=$v timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab/c2_${v}_$rep.json 2> gpurun_out/ab/err.txt || { tail -5 gpurun_out/ab/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/c2_${v}_$rep.json'));print('c2 $var=$v rep $rep', d['value'], d['ms_per_step'], {k: v.get('serial_ms') for k, v in d['passes'].items()})"
done; done
if [ -z "$NO_C4" ]; then for v in $a $b; do
  env $var=$v timeout -k 10 200 python -u bench.py --config 4 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab/c4_$v.json 2> gpurun_out/ab/err.txt || { tail -5 gpurun_out/ab/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/c4_$v.json'));print('c4 $var=$v', d['value'], d['ms_per_step'], {k: v.get('serial_ms') for k, v in d['passes'].items()})"
done; fi
