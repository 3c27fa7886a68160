#!/bin/bash
# round 6: the device builder's treelet sweeps + SAH-optimal collapse (default) against the round-5 tree
# (ORX_BVH_TREELET=0 ORX_BVH_COLLAPSE=0): BVH parity tests, traversal statistics, alternating bench runs.
set -o pipefail
TAG=${TAG:-r06k_bvhdev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "bvh or mesh or texture or hall or conference or vcm" > $OUT/parity.log 2>&1 \
    || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for v in old new; do
  if [ $v = old ]; then E="ORX_BVH_TREELET=0 ORX_BVH_COLLAPSE=0"; else E="ORX_BVH_TREELET=3"; fi
  env $E timeout -k 10 300 python -u tools/trav_stats.py SyntheticHall ppm 1920x1080x2048 > $OUT/trav_$v.txt 2>&1 \
      || { tail -5 $OUT/trav_$v.txt; exit 1; }
  grep -v amdgpu.ids $OUT/trav_$v.txt | grep -E "it2 (closest|any) |stack" | cut -c1-200
done
for rep in 1 2; do for v in old new; do for c in 2 3; do
  if [ $v = old ]; then E="ORX_BVH_TREELET=0 ORX_BVH_COLLAPSE=0"; else E="ORX_BVH_TREELET=3"; fi
  env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 > $OUT/${v}_c${c}_$rep.json 2> $OUT/err.txt \
      || { tail -5 $OUT/err.txt; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_c${c}_$rep.json').read().strip().splitlines()[-1])
print('$v c$c rep $rep', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) for k, v in d['passes'].items()})"
done; done; done
for v in old new; do
  if [ $v = old ]; then E="ORX_BVH_TREELET=0 ORX_BVH_COLLAPSE=0"; else E="ORX_BVH_TREELET=3"; fi
  env $E timeout -k 10 400 python -u bench.py --no-cpu-baseline --config 4 --steps 8 --warmup 2 > $OUT/${v}_c4.json 2> $OUT/err.txt \
      || { tail -5 $OUT/err.txt; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_c4.json').read().strip().splitlines()[-1])
print('$v c4', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) for k, v in d['passes'].items()})"
done
