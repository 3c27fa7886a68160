#!/bin/bash
# round 6: host-built BVH variants (ORX_BVH_HOST=1) on the GPU: parity of the treelet-restructured, SAH-collapsed
# tree against the oracle, traversal statistics, and alternating bench runs (PPM configs[2], VCM configs[3]).
# Variants: base = the shipped rules on the host; tre = ORX_BVH_TREELET=3 ORX_BVH_COLLAPSE=1.
set -o pipefail
TAG=${TAG:-r06j_bvh}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export ORX_BVH_HOST=1
ORX_BVH_TREELET=3 ORX_BVH_COLLAPSE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "mesh_bvh or vcm_mesh or texture" > $OUT/parity.log 2>&1 \
    || { tail -20 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for v in base tre; do
  if [ $v = tre ]; then E="ORX_BVH_TREELET=3 ORX_BVH_COLLAPSE=1"; else E="ORX_BVH_TREELET=0"; fi
  env $E timeout -k 10 300 python -u tools/trav_stats.py SyntheticHall ppm 1920x1080x2048 > $OUT/trav_$v.txt 2>&1 \
      || { tail -5 $OUT/trav_$v.txt; exit 1; }
  grep -v amdgpu.ids $OUT/trav_$v.txt | tail -4 | cut -c1-300
done
for rep in 1 2; do for v in base tre; do for c in 2 3; do
  if [ $v = tre ]; then E="ORX_BVH_TREELET=3 ORX_BVH_COLLAPSE=1"; else E="ORX_BVH_TREELET=0"; fi
  env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 > $OUT/${v}_c${c}_$rep.json 2> $OUT/err.txt \
      || { tail -5 $OUT/err.txt; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_c${c}_$rep.json').read().strip().splitlines()[-1])
print('$v c$c rep $rep', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) for k, v in d['passes'].items()})"
done; done; done
