"""Debug helper: first differences between the device and the oracle on the media path."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import oracle_lib
from oppositerenderer_amd import _abi, scenes
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails

SEED = 1645301512
W = H = 64
P = int(sys.argv[1]) if len(sys.argv) > 1 else 128
sc = scenes.cornell_medium(sigma_s=0.001)
c = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P, enable_media=1, max_photon_trace_depth=15)
gpu = OptixRenderer(c)
gpu.initialize(0)
gpu.initScene(sc)
ora = oracle_lib.OracleRenderer(c)
ora.init_scene(sc)
cam = sc.default_camera.set_aspect_ratio(1.0)
det = RenderRequestDetails(cam, sc.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
r = sc.initial_ppm_radius()
gpu.renderNextIteration(0, 0, r, True, det)
ora.render_next_iteration(0, 0, r, det.to_abi())
g = gpu.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 4, 9) if False else gpu.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9)
o = ora.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9)
D = 4
diff = np.nonzero((g != o).any(1))[0]
print("slots differ", len(diff), "of", len(g))
paths = np.unique(diff // D)
print("paths differ", len(paths), "first", paths[:10])
for p in paths[:6]:
    print("path", p)
    for k in range(D):
        print("  gpu", np.round(g[p * D + k], 4))
        print("  ora", np.round(o[p * D + k], 4))
gt = gpu.read_buffer(_abi.BUF_VOLUMETRIC_PHOTONS).reshape(-1, 7)
ot = ora.read_buffer(_abi.BUF_VOLUMETRIC_PHOTONS).reshape(-1, 7)
print("vol table rows differ", int((gt != ot).any(1).sum()), "nonempty gpu", int((gt[:, 6] != 0).sum()), "ora", int((ot[:, 6] != 0).sum()))
