# A/B of an environment switch on the default bench workload: tools/gpu_ab.sh VAR "v1 v2 ..." [bench args]
set -o pipefail
VAR=$1; VALS=$2; shift 2
mkdir -p gpurun_out/ab
for v in $VALS; do
  LOG=gpurun_out/ab/$VAR-$(basename "$v").log
  env $VAR=$v timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 24 --warmup 4 "$@" > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$LOG').read().strip().splitlines()[-1])
print('$VAR=$v', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) for k, v in d['passes'].items()})"
done
