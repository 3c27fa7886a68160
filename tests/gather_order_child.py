"""Child process of tests/test_gpu_parity.py::test_gather_tile_order (TEST INFRASTRUCTURE; needs a
GPU).  ORX_GATHER_ORDER (the gather's tile order, orx_capi.hip gather_order) is read once per
process, so each order runs in a process of its own.

With the order in the environment: a single renderer (the local gather, gather_tile's super-tile
walk over the image) and three row shards on the one device (the external gather over the
segment-major hit points, tests/shard_emul.py) render Cornell at 200 x 150 — 13 x 10 tiles of
16 x 16 pixels, neither a multiple of 8 nor of 3, so the super-tile order pads and drops tiles on
both edges — and are compared with the CPU oracle.  A tile skipped leaves its pixels' indirect at
zero; one taken twice by different blocks races.  Prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import oracle_lib  # noqa: E402
import shard_emul  # noqa: E402
from oppositerenderer_amd import _abi, scenes  # noqa: E402
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius  # noqa: E402

SEED = 1645301512
W, H, P, ITERS = 200, 150, 64, 2


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).sum()) / max(np.sqrt((b * b).sum()), 1e-30))


def main():
    scene = scenes.cornell()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = det.to_abi()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
    gpu = OptixRenderer(cfg)
    gpu.initialize(0)
    gpu.initScene(scene)
    ora = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
    ora.init_scene(scene)
    radius = scene.initial_ppm_radius()
    res = {"order": os.environ.get("ORX_GATHER_ORDER")}
    worst_ind = 0.0
    for it in range(ITERS):
        gpu.renderNextIteration(it, it, radius, False, det)
        ora.render_next_iteration(it, it, radius, req)
        gi = gpu.read_buffer(_abi.BUF_INDIRECT).reshape(H, W, 3)
        oi = ora.read_buffer(_abi.BUF_INDIRECT).reshape(H, W, 3)
        worst_ind = max(worst_ind, rel_l2(gi, oi))
        # a skipped tile: pixels the oracle lights and the GPU leaves at zero
        res.setdefault("dark_pixels", 0)
        res["dark_pixels"] += int(((oi.sum(-1) > 0) & (gi.sum(-1) == 0)).sum())
        radius = next_ppm_radius(radius, it)
    res["local_indirect_rel_l2"] = worst_ind
    ref = ora.output()
    res["local_output_rel_l2"] = rel_l2(gpu.getOutputBuffer().reshape(ref.shape), ref)
    res["lit_pixels"] = int((ref.reshape(H, W, 3).sum(-1) > 0).sum())
    gpu.destroy()
    shards = shard_emul.make_shards(scene, 3, P, P)
    got, _ = shard_emul.run_iterations(shards, scene, W, H, req, ITERS)
    res["rows3_output_rel_l2"] = rel_l2(got, ref.reshape(H, W, 3))
    for b in shards:
        b.r.destroy()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
