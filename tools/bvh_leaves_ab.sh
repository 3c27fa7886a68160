#!/bin/bash
# round 6: 7- against 9-leaf treelets in the device builder: scene-init time, parity, traversal statistics, bench A/B
set -o pipefail
TAG=${TAG:-r06l_tl9}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for L in 7 9; do
  ORX_BVH_TREELET_LEAVES=$L timeout -k 10 300 python -u -c "
import time, sys
sys.path.insert(0, '.')
from oppositerenderer_amd import _abi, synthetic
from oppositerenderer_amd.renderer import OptixRenderer
for name, sc in (('hall', synthetic.synthetic_hall()), ('conference', synthetic.synthetic_conference())):
    r = OptixRenderer(_abi.default_config()); r.initialize(0)
    t0 = time.perf_counter(); r.initScene(sc); t1 = time.perf_counter()
    print('leaves $L', name, 'initScene %.3f s' % (t1 - t0), 'stack', r.stats().bvh_stack_entries)
    r.destroy()
" 2>&1 | grep leaves || exit 1
done
ORX_BVH_TREELET_LEAVES=9 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "bvh or mesh or texture" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for L in 7 9; do
  ORX_BVH_TREELET_LEAVES=$L timeout -k 10 300 python -u tools/trav_stats.py SyntheticHall ppm 1920x1080x2048 > $OUT/trav_$L.txt 2>&1 \
      || { tail -5 $OUT/trav_$L.txt; exit 1; }
  grep -v amdgpu.ids $OUT/trav_$L.txt | grep -E "it2 (closest|any) |stack" | cut -c1-200
done
for rep in 1 2; do for L in 7 9; do for c in 2 3; do
  ORX_BVH_TREELET_LEAVES=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 > $OUT/${L}_c${c}_$rep.json 2> $OUT/err.txt \
      || { tail -5 $OUT/err.txt; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/${L}_c${c}_$rep.json').read().strip().splitlines()[-1])
print('leaves $L c$c rep $rep', d['value'], d['ms_per_step'], {k: (v['ms'], v.get('serial_ms')) for k, v in d['passes'].items()})"
done; done; done
