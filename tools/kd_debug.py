"""Dump the device and oracle kd-trees of one Cornell PPM iteration (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402
from oppositerenderer_amd import _abi, scenes  # noqa: E402
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails  # noqa: E402

W, H, P = 64, 48, 64
scene = scenes.cornell()
cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P, photon_map=2)
gpu = OptixRenderer(cfg)
gpu.initialize(0)
gpu.initScene(scene)
ora = oracle_lib.OracleRenderer(_abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P,
                                                    photon_map=2))
ora.init_scene(scene)
cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
r = scene.initial_ppm_radius()
gpu.renderNextIteration(0, 0, r, True, det)
ora.render_next_iteration(0, 0, r, det.to_abi())
out = {}
for name, x in (("g", gpu), ("o", ora)):
    out[name + "_tree"] = x.read_buffer(_abi.BUF_KD_TREE)
    out[name + "_dbg"] = x.read_buffer(_abi.BUF_DEBUG_VISITED, np.uint32)
    out[name + "_ind"] = x.read_buffer(_abi.BUF_INDIRECT)
    out[name + "_slots"] = x.read_buffer(_abi.BUF_PHOTON_SLOTS)
out["hp"] = ora.read_buffer(_abi.BUF_HITPOINTS)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "kd_dbg.npz"), **out)
print("saved", gpu.stats().valid_photons, ora.stats().valid_photons)
