"""Two RCCL ranks on one GPU running the pipelined ShardedPPM (the bench's N>1 path) against a
single-GPU render of the same union photon launch.  Debug aid for a 1-GPU box:
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_two_rank_check.py"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oppositerenderer_amd import _abi, multigpu, scenes  # noqa: E402
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
W, H, P, iters = 96, 64, 64, 4
scene = scenes.cornell()
cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
req = det.to_abi()
r = OptixRenderer(_abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P * world))
r.initialize(0)
r.set_shard(rank, world)
r.initScene(scene)
b = multigpu.DeviceShard(r, torch, torch.device("cuda", 0))
sh = multigpu.ShardedPPM(b, dist, world, rank, W, H, pipeline=os.environ.get("ORX_PIPELINE", "1") != "0")
radius = scene.initial_ppm_radius()
for it in range(iters):
    sh.iteration(it, it, radius, req)
    radius = next_ppm_radius(radius, it)
img = sh.image()
if rank == 0:
    single = OptixRenderer(_abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P * world))
    single.initialize(0)
    single.initScene(scene)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        single.renderNextIteration(it, it, radius, True, det)
        radius = next_ppm_radius(radius, it)
    ref = single.getOutputBuffer()
    err = float(np.sqrt(((img.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum()))
    print(json.dumps({"pipelined": sh.pipe, "rel_l2": err}), flush=True)
dist.barrier()
dist.destroy_process_group()
