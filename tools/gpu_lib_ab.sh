# A/B of in-tree liborx builds on one bench workload: tools/gpu_lib_ab.sh "base noslp ..." [bench args]
# (name x = oppositerenderer_amd/liborx_x.so; "cur" = liborx.so)
set -o pipefail
LIBS=$1; shift
mkdir -p gpurun_out/ab
for n in $LIBS; do
  if [ "$n" = cur ]; then L=$PWD/oppositerenderer_amd/liborx.so; else L=$PWD/oppositerenderer_amd/liborx_$n.so; fi
  LOG=gpurun_out/ab/lib-$n-$(echo "$@" | tr -c 'a-zA-Z0-9' _).log
  ORX_LIB=$L timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
  python3 -c "
import json; d=json.loads(open('$LOG').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) for k, v in d['passes'].items()})"
done
