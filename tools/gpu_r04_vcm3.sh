# per-kernel times of the deferred VCM camera pass
set -o pipefail
mkdir -p gpurun_out/vcm3
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/vcm3/tr -o run -- python3 $R/bench.py --method vcm --steps 8 --warmup 2 --no-cpu-baseline > $R/gpurun_out/vcm3/b.json 2> $R/gpurun_out/vcm3/err.txt || { tail -5 $R/gpurun_out/vcm3/err.txt; exit 1; }
cd $R
f=$(find gpurun_out/vcm3/tr -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 $f | head -14
python3 -c "
import sys; sys.path.insert(0,'.')
from oppositerenderer_amd import _abi, synthetic
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius
import numpy as np
sc=synthetic.synthetic_hall(); W,H=1920,1080
r=OptixRenderer(_abi.default_config(seed=1645301512, photon_launch_width=64, photon_launch_height=64)); r.initialize(0); r.initScene(sc)
det=RenderRequestDetails(sc.default_camera.set_aspect_ratio(W/H), sc.name, _abi.VCM_BIDIRECTIONAL_PATH_TRACING, W, H)
rad=sc.initial_ppm_radius()
for it in range(3):
    r.renderNextIteration(it,it,rad,False,det); rad=next_ppm_radius(rad,it)
    st=r.stats(); print('it',it,'shadow rays',st.vcm_shadow_rays, 'per px', st.vcm_shadow_rays/(W*H), 'overflow', st.vcm_shadow_overflow)
"
