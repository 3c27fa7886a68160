"""Child process of tests/test_gpu_steady_state.py::test_rccl_world1_sharded_paths_match_oracle
(TEST INFRASTRUCTURE; needs a GPU).

Runs the multi-GPU bench's orchestration (oppositerenderer_amd/multigpu.py) over a real
torch.distributed "nccl" (= RCCL) process group of world size 1 — the only RCCL world a one-GPU
box can host — through the product backend (multigpu.device_shard_factory: liborx.so on HIP),
and compares each variant's image with the CPU oracle's single renderer:

  ppm_rows_pipelined  all_gather_into_tensor(async) + work.wait() on the side stream +
                      reduce_scatter_tensor there (bench.py's default schedule)
  ppm_rows_serial     the same with ORX_PIPELINE=0 semantics (pipeline=False)
  ppm_slab_pipelined  + the histogram all-gather, the slab plan and all_to_all_single of the photons
  ppm_slab_serial
  vcm                 reduce_scatter_tensor of the light-tracing splats (ShardedVCM)
  pt                  no per-iteration exchange (ShardedPT), bit-exact
Every variant ends with ShardedPPM.image()'s all_gather.  Prints one JSON line.

The rendezvous is a FileStore (argv[1]): no TCP port to race for."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle_lib  # noqa: E402
from oppositerenderer_amd import _abi, multigpu, synthetic  # noqa: E402
from oppositerenderer_amd.renderer import RenderRequestDetails, next_ppm_radius  # noqa: E402

SEED = 1645301512
W, H, P, ITERS = 480, 270, 256, 3


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).sum()) / max(np.sqrt((b * b).sum()), 1e-30))


def oracle_image(scene, method, req):
    ora = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
    ora.init_scene(scene)
    radius = scene.initial_ppm_radius()
    for it in range(ITERS):
        ora.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    out = ora.output().copy()
    ora.close()
    return out


def main():
    torch.cuda.set_device(0)
    store = dist.FileStore(sys.argv[1], 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    scene = synthetic.synthetic_hall()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    refs = {}
    res = {"backend": dist.get_backend(), "variants": {}}
    variants = [("ppm_rows_pipelined", "ppm", True, False), ("ppm_rows_serial", "ppm", False, False),
                ("ppm_slab_pipelined", "ppm", True, True), ("ppm_slab_serial", "ppm", False, True),
                ("vcm", "vcm", False, False), ("pt", "pt", False, False)]
    for name, method, pipeline, slab in variants:
        mcode = {"ppm": _abi.PROGRESSIVE_PHOTON_MAPPING, "vcm": _abi.VCM_BIDIRECTIONAL_PATH_TRACING,
                 "pt": _abi.PATH_TRACING}[method]
        req = RenderRequestDetails(cam, scene.name, mcode, W, H).to_abi()
        cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
        backend = multigpu.device_shard_factory(cfg, 0, 1, 0, scene)
        if method == "ppm":
            sh = multigpu.ShardedPPM(backend, dist, 1, 0, W, H, pipeline=pipeline, slab=slab)
        elif method == "vcm":
            sh = multigpu.ShardedVCM(backend, dist, 1, 0, W, H)
        else:
            sh = multigpu.ShardedPT(backend, dist, 1, 0, W, H)
        radius = scene.initial_ppm_radius()
        for it in range(ITERS):
            sh.iteration(it, it, radius, req)
            radius = next_ppm_radius(radius, it)
        pipelined = bool(backend.r.pipelined())
        img = sh.image()
        if method not in refs:
            refs[method] = oracle_image(scene, mcode, req)
        ref = refs[method]
        entry = {"rel_l2": rel_l2(img, ref), "mean": float(img.mean()), "pipelined": pipelined,
                 "expect_pipelined": bool(pipeline and method == "ppm"),
                 "bit_exact": bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)))}
        if slab:
            axis, bin_dest, counts = sh.last_plan
            entry["slab_photons"] = int(counts.sum())
        res["variants"][name] = entry
        backend.r.destroy()
        torch.cuda.synchronize()
        print(name, entry, file=sys.stderr, flush=True)
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
