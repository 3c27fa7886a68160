#!/usr/bin/env python3
"""Headline benchmark: progressive photon mapping throughput (Mpaths/s) and
ms/frame on MI355X, with a live HBM-roofline figure for the dominant kernel and
the CPU oracle timed on the host cores beside it.

Workload (BASELINE.json configs[1]): Cornell box 1024x1024, PPM, 1,048,576
emitted photons per iteration (1024x1024 photon launch, <= 4 deposits each),
r0 = IScene::getSceneInitialPPMRadiusEstimate, alpha = 2/3, seed 1645301512.
paths/iteration = W*H eye paths + emitted photon paths.

Single GPU:  python bench.py [--steps K --warmup W]
Multi GPU:   torchrun --nproc-per-node N bench.py --gpus N   (one rank per GPU;
             see DESIGN.md "Multi-GPU" for the sharding and the RCCL exchange)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--width", type=int, default=1024)
    p.add_argument("--height", type=int, default=1024)
    p.add_argument("--photon-launch", type=int, default=1024)
    p.add_argument("--scene", default="Cornell")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=20.0)
    p.add_argument("--gather-variant", type=int, default=0)
    p.add_argument("--force-sharded", action="store_true",
                   help="run the torch.distributed/RCCL sharded path even with one rank (tests the N>1 code)")
    return p.parse_args()


def gather_bytes_per_launch(W, H, valid_photons, num_cells):
    """Algorithmic HBM bytes of one gather launch (DESIGN.md 'Roofline'):
    every hitpoint read once (40 B: pos+flags 16, normal+atten.x 16, atten.yz 8),
    the indirect result written once (12 B), every grid-resident photon read
    once (36 B), the offset table read once (4 B per cell)."""
    return W * H * (40 + 12) + valid_photons * 36 + (num_cells + 1) * 4


def cpu_baseline(scene, args, W, H, P, seconds):
    """Oracle (oracle/liborx_oracle.so, OpenMP, the CPU restatement of the
    reference passes) on the host cores: the same scene, resolution, photon
    count and seed as the GPU line; one warm-up iteration, then timed
    iterations until `seconds` of CPU wall time or 8 iterations."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from oppositerenderer_amd import _abi
    from oppositerenderer_amd.renderer import next_ppm_radius

    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    lib = oracle_lib.load()
    lib.orc_set_threads(cores)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    req = _abi.OrxRequest()
    req.camera = cam.to_abi()
    req.method = _abi.PROGRESSIVE_PHOTON_MAPPING
    req.width, req.height, req.ppm_alpha = W, H, 2.0 / 3.0
    cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P)
    r = oracle_lib.OracleRenderer(cfg)
    r.init_scene(scene)
    radius = scene.initial_ppm_radius()
    r.render_next_iteration(0, 0, radius, req)  # warm-up: allocation + RNG init
    radius = next_ppm_radius(radius, 0)
    times = []
    t_start = time.perf_counter()
    it = 1
    while it <= 8 and (time.perf_counter() - t_start) < seconds:
        t0 = time.perf_counter()
        r.render_next_iteration(it, it, radius, req)
        times.append(time.perf_counter() - t0)
        radius = next_ppm_radius(radius, it)
        it += 1
    r.close()
    t = float(np.median(times))
    paths = W * H + P * P
    return {"value": round(paths / t / 1e6, 3), "unit": "Mpaths/s", "cores": cores, "kind": "port",
            "ms_per_step": round(t * 1e3, 2),
            "sample": f"oracle (C/OpenMP restatement) full {scene.name} {W}x{H} PPM, {P * P} photons/iter, "
                      f"median of {len(times)} iterations after 1 warm-up"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 or world > 1 or args.force_sharded:
        from oppositerenderer_amd import multigpu
        return multigpu.bench_main(args, METRIC)

    from oppositerenderer_amd import _abi, scenes
    from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

    W, H, P = args.width, args.height, args.photon_launch
    scene = scenes.scene_by_name(args.scene)
    cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P,
                              gather_variant=args.gather_variant)
    r = OptixRenderer(cfg)
    r.initialize(local_rank)
    r.initScene(scene)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    radius = scene.initial_ppm_radius()
    it = 0
    for _ in range(args.warmup):
        r.renderNextIteration(it, it, radius, False, det)
        radius = next_ppm_radius(radius, it)
        it += 1
    r.stats()  # synchronises the renderer's stream
    r.reset_timing()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r.renderNextIteration(it, it, radius, False, det)
        radius = next_ppm_radius(radius, it)
        it += 1
    st = r.stats()  # synchronises
    t1 = time.perf_counter()
    wall = t1 - t0
    ms_per_step = wall * 1e3 / args.steps
    paths = W * H + P * P
    value = paths * args.steps / wall / 1e6

    per_pass = {name: st.pass_ms[i] / max(1, st.timed_iterations) for i, name in enumerate(_abi.PASS_NAMES)}
    dominant = max(per_pass, key=per_pass.get)
    valid_avg = st.valid_photons_total / max(1, st.timed_iterations)
    gms = per_pass["ppm_gather"]
    gbytes = gather_bytes_per_launch(W, H, valid_avg, st.num_cells)
    achieved = gbytes / (gms * 1e-3) / 1e9 if gms > 0 else 0.0
    visited_avg = st.photons_visited_total / max(1, st.timed_iterations)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "gather_traffic_bytes.json")
    if os.path.exists(tfile):
        try:
            traffic = json.load(open(tfile)).get("bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (built-in Cornell scene, seeded XORWOW streams)",
        "config": {"workload": f"{scene.name} {W}x{H} PPM, {P * P} photons/iter (BASELINE configs[1])",
                   "scene": scene.name, "width": W, "height": H, "photons_per_iteration": P * P,
                   "paths_per_iteration": paths, "parallelism": "single GPU"},
        "roofline": {"kernel": "k_ppm_gather", "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "bytes_per_launch": int(gbytes), "avg_launch_ms": round(gms, 4),
                     "photons_visited_per_launch": int(visited_avg),
                     "photons_staged_per_launch": int(st.gather_staged_total / max(1, st.timed_iterations)),
                     "visited_photon_GBps": round(visited_avg * 36 / (gms * 1e-3) / 1e9, 1) if gms > 0 else None},
        "passes_ms": {k: round(v, 4) for k, v in per_pass.items() if v > 0},
        "dominant_pass": dominant,
    }
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(scene, args, W, H, P, args.cpu_seconds)
        except Exception as e:  # the baseline must never hide the GPU line
            out["cpu_baseline"] = {"error": repr(e)}
    r.destroy()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
