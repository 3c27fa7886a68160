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
  {ppm,vcm,pt}_batch  the photon-batch partition (bench.py's default multi-GPU mode, BatchSharded over
                      multigpu.device_batch_factory): the single-device path, reduce of the radiance
  ppm_batch2_emulated two photon-batch ranks' renderers on the one GPU (seeds batch_seed(SEED, 0/1),
                      global iterations dealt round-robin), their radiance summed, against the oracle's
                      two renderers
Every rows/slab variant ends with ShardedPPM.image()'s all_gather.  Prints one JSON line.

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


def oracle_image(scene, method, req, world=1):
    """world > 1: the photon-batch partition's sum of `world` renderers (multigpu.batch_seed, global
    iterations g, g + world, ...)"""
    radii = multigpu.radius_sequence(scene.initial_ppm_radius(), ITERS * world)
    out = None
    for g in range(world):
        cfg = _abi.default_config(seed=multigpu.batch_seed(SEED, g), photon_launch_width=P, photon_launch_height=P)
        ora = oracle_lib.OracleRenderer(cfg)
        ora.init_scene(scene)
        for i in range(ITERS):
            it = multigpu.batch_iteration(i, g, world)
            ora.render_next_iteration(it, i, radii[it], req)
        o = ora.output().astype(np.float64)
        out = o if out is None else out + o
        ora.close()
    return out.astype(np.float32) if world == 1 else out


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
    for name, method in (("ppm_batch", "ppm"), ("vcm_batch", "vcm"), ("pt_batch", "pt")):
        mcode = {"ppm": _abi.PROGRESSIVE_PHOTON_MAPPING, "vcm": _abi.VCM_BIDIRECTIONAL_PATH_TRACING,
                 "pt": _abi.PATH_TRACING}[method]
        req = RenderRequestDetails(cam, scene.name, mcode, W, H).to_abi()
        cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
        backend = multigpu.device_batch_factory(cfg, 0, 1, 0, scene)
        sh = multigpu.BatchSharded(backend, dist, 1, 0, W, H, reduce_every=2)
        radii = multigpu.radius_sequence(scene.initial_ppm_radius(), ITERS)
        for i in range(ITERS):
            sh.iteration(multigpu.batch_iteration(i, 0, 1), i, radii[i], req)
        pipelined = bool(backend.r.pipelined())
        img = sh.image()
        ref = refs[method]
        entry = {"rel_l2": rel_l2(img, ref), "mean": float(img.mean()), "pipelined": pipelined,
                 "expect_pipelined": method == "ppm",
                 "bit_exact": bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)))}
        res["variants"][name] = entry
        backend.r.destroy()
        torch.cuda.synchronize()
        print(name, entry, file=sys.stderr, flush=True)
    # two photon-batch ranks emulated on the one GPU (the collective is the sum below)
    mcode = _abi.PROGRESSIVE_PHOTON_MAPPING
    req = RenderRequestDetails(cam, scene.name, mcode, W, H).to_abi()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
    radii = multigpu.radius_sequence(scene.initial_ppm_radius(), ITERS * 2)
    acc = None
    for g in range(2):
        backend = multigpu.device_batch_factory(cfg, g, 2, 0, scene)
        for i in range(ITERS):
            it = multigpu.batch_iteration(i, g, 2)
            backend.render_next(it, i, radii[it], req)
        t = backend.output_local_tensor(H)
        torch.cuda.synchronize()
        o = t.cpu().numpy().astype(np.float64).reshape(H, W, 3)
        acc = o if acc is None else acc + o
        backend.r.destroy()
    ref2 = oracle_image(scene, mcode, req, world=2)
    entry = {"rel_l2": rel_l2(acc, ref2), "mean": float(acc.mean()),
             "rank_images_differ": bool(rel_l2(acc, 2 * refs["ppm"]) > 1e-3)}
    res["variants"]["ppm_batch2_emulated"] = entry
    print("ppm_batch2_emulated", entry, file=sys.stderr, flush=True)
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
