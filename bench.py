#!/usr/bin/env python3
"""Headline benchmark: progressive photon mapping throughput (Mpaths/s) and
ms/frame on MI355X, with a live HBM-roofline figure for the dominant kernel and
the CPU oracle timed on the host cores beside it.

Workload: the metric's own configuration, "1080p Sponza PPM" (BASELINE.json
configs[2]): the seeded synthetic Sponza-class hall
(oppositerenderer_amd/synthetic.py, 261,120 triangles, one quad area light),
1920x1080, PPM with a 2048x2048 photon launch (4,194,304 emitted photons,
<= 4 deposits each), r0 = IScene::getSceneInitialPPMRadiusEstimate,
alpha = 2/3, seed 1645301512.  paths/iteration = W*H eye paths + emitted
photon paths.  --scene Cornell --width 1024 --height 1024
--photon-launch 1024 gives configs[1]; --method vcm gives configs[3].

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



def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--photon-launch", type=int, default=2048)
    p.add_argument("--scene", default="SyntheticHall")
    p.add_argument("--method", choices=["ppm", "vcm", "pt"], default="ppm")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=20.0)
    p.add_argument("--gather-variant", type=int, default=0)
    p.add_argument("--photon-map", choices=["grid", "hash", "kd"], default="grid",
                   help="uniform grid (the reference's shipped configuration), stochastic hash (single GPU) "
                        "or kd-tree (ACCELERATION_STRUCTURE_KD_TREE_CPU, built on the device)")
    p.add_argument("--force-sharded", action="store_true",
                   help="run the torch.distributed/RCCL sharded path even with one rank (tests the N>1 code)")
    return p.parse_args()


METHODS = {"ppm": 2, "vcm": 1, "pt": 0}  # orx_method (include/orx.h)


def traffic_lookup(key, kernels):
    """PMC-measured HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md) recorded by tools/profile_traffic.py for
    this exact workload, or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        table = json.load(open(path)).get(key, {})
    except (OSError, ValueError):
        return None
    vals = [table[k]["bytes_per_launch"] for k in kernels if k in table]
    return int(sum(vals)) if vals else None


PHOTON_MAPS = {"grid": 0, "hash": 1, "kd": 2}  # orx_config.photon_map


def cpu_baseline(scene, method, W, H, P, seconds, photon_map=0):
    """Oracle (oracle/liborx_oracle.so: the C/OpenMP restatement of the
    reference passes) on the host cores, same scene, resolution, photon count
    and seed as the GPU line: one untimed warm-up iteration (allocation, RNG
    init, VCM estimate launch), then timed iterations until `seconds` of CPU
    wall time are spent (at least one, at most 8); median."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from oppositerenderer_amd import _abi, roofline
    from oppositerenderer_amd.renderer import next_ppm_radius

    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    lib = oracle_lib.load()
    lib.orc_set_threads(cores)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    req = _abi.OrxRequest()
    req.camera = cam.to_abi()
    req.method = method
    req.width, req.height, req.ppm_alpha = W, H, 2.0 / 3.0
    cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P, photon_map=photon_map)
    r = oracle_lib.OracleRenderer(cfg)
    r.init_scene(scene)
    radius = scene.initial_ppm_radius()
    r.render_next_iteration(0, 0, radius, req)
    radius = next_ppm_radius(radius, 0)
    times = []
    t_start = time.perf_counter()
    it = 1
    while it <= 8 and (it == 1 or (time.perf_counter() - t_start) < seconds):
        t0 = time.perf_counter()
        r.render_next_iteration(it, it, radius, req)
        times.append(time.perf_counter() - t0)
        radius = next_ppm_radius(radius, it)
        it += 1
    r.close()
    t = float(np.median(times))
    paths = roofline.paths_per_iteration(method, W, H, P * P)
    return {"value": round(paths / t / 1e6, 3), "unit": "Mpaths/s", "cores": cores, "kind": "port",
            "ms_per_step": round(t * 1e3, 2),
            "sample": f"oracle (C/OpenMP restatement, {cores} threads) on the full workload: {scene.name} {W}x{H} "
                      f"{_METHOD_NAME[method]}" + (f", {P * P} photons/iter" if method == 2 else "") +
                      f"; median of {len(times)} iteration(s) after 1 warm-up"}


_METHOD_NAME = {0: "PT", 1: "VCM", 2: "PPM"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 or world > 1 or args.force_sharded:
        from oppositerenderer_amd import multigpu
        return multigpu.bench_main(args, METRIC)

    from oppositerenderer_amd import _abi, roofline, scenes
    from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

    method = METHODS[args.method]
    W, H, P = args.width, args.height, args.photon_launch
    scene = scenes.scene_by_name(args.scene)
    cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P,
                              gather_variant=args.gather_variant,
                              photon_map=PHOTON_MAPS[args.photon_map])
    r = OptixRenderer(cfg)
    r.initialize(local_rank)
    r.initScene(scene)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, method, W, H)
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
    wall = time.perf_counter() - t0
    ms_per_step = wall * 1e3 / args.steps
    paths = roofline.paths_per_iteration(method, W, H, P * P)
    value = paths * args.steps / wall / 1e6

    n_it = max(1, st.timed_iterations)
    per_pass = {name: st.pass_ms[i] / n_it for i, name in enumerate(_abi.PASS_NAMES)}
    per_pass = {k: v for k, v in per_pass.items() if v > 0}
    # pipelined PPM: the gather and output run on a side stream beside the next iteration's
    # passes, so their times are overlapped wall time; the roofline names the longest pass on
    # the critical chain (eye -> photon -> grid)
    pipelined = method == _abi.PROGRESSIVE_PHOTON_MAPPING and r.pipelined()
    overlapped = ["ppm_gather", "ppm_direct_output"] if pipelined else []
    critical = {k: v for k, v in per_pass.items() if k not in overlapped} or per_pass
    dominant = max(critical, key=critical.get)
    valid_avg = st.valid_photons_total / n_it
    light_vertices = 0
    if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING:
        light_vertices = int(np.minimum(r.read_buffer(_abi.BUF_VCM_VERTEX_COUNT, np.uint32), 9).sum())
    pmap = PHOTON_MAPS[args.photon_map]
    pbytes = roofline.pass_bytes(method, W, H, P * P, valid_avg, st.num_cells, light_vertices, photon_map=pmap)
    key = (f"{scene.name}:{W}x{H}:{args.method}" + (f":P{P}" if method == 2 else "")
           + (f":{args.photon_map}" if pmap else ""))
    traffic = traffic_lookup(key, roofline.kernels_of(dominant, pmap))
    roof = roofline.roofline(dominant, pbytes[dominant], per_pass[dominant], traffic, photon_map=pmap)
    passes = {k: {"ms": round(v, 4), "algorithmic_GBps": round(pbytes.get(k, 0) / (v * 1e-3) / 1e9, 1)}
              for k, v in per_pass.items()}
    if method == _abi.PROGRESSIVE_PHOTON_MAPPING:
        gms = per_pass.get("ppm_gather", 0.0)
        visited = st.photons_visited_total / n_it
        roof["gather_visited_photons_per_launch"] = int(visited)
        roof["gather_visited_photon_GBps"] = round(visited * 36 / (gms * 1e-3) / 1e9, 1) if gms > 0 else None
    data = ("synthetic: seeded procedural scene (" + scene.name + "), XORWOW streams seeded 1645301512; "
            "no assets or checkpoints")
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": data,
        "config": {"workload": f"{scene.name} {W}x{H} {_METHOD_NAME[method]}"
                               + (f", {P * P} photons/iter" if method == 2 else ""),
                   "scene": scene.name, "width": W, "height": H, "method": _METHOD_NAME[method],
                   "photons_per_iteration": P * P if method == 2 else 0, "paths_per_iteration": paths,
                   "photon_map": {"grid": "uniform grid", "hash": "stochastic hash", "kd": "kd-tree"}[args.photon_map],
                   "parallelism": "single GPU"},
        "roofline": roof,
        "passes": passes,
        "dominant_pass": dominant,
        "overlapped_passes": overlapped,
    }
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(scene, method, W, H, P, args.cpu_seconds,
                                               photon_map=PHOTON_MAPS[args.photon_map])
        except Exception as e:  # the baseline must never hide the GPU line
            out["cpu_baseline"] = {"error": repr(e)}
    r.destroy()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
