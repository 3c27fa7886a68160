#!/usr/bin/env python3
"""Headline benchmark: progressive photon mapping throughput (Mpaths/s) and
ms/frame on MI355X, with a live HBM-roofline figure for the dominant kernel and
the CPU oracle timed on the host cores beside it.

Workloads (--config, BASELINE.json "configs"; SURVEY 8(d) C1-C5, synthetic
stand-ins for the absent Sponza/Conference assets):
  0  Cornell 256x256, PT, 1 spp
  1  Cornell 1024x1024, PPM, 1024^2 = 1,048,576 photons/iter
  2  SyntheticHall 1920x1080, PPM, 2048^2 = 4,194,304 photons/iter   <- default: the metric's
     "1080p Sponza PPM" (261,120 triangles, one quad area light)
  3  SyntheticHall 1920x1080, VCM
  4  SyntheticConference 3840x2160, PPM, 4096^2 = 16,777,216 photons/iter
PPM: r0 = IScene::getSceneInitialPPMRadiusEstimate, alpha = 2/3, seed
1645301512; paths/iteration = W*H eye paths + emitted photon paths.
--scene/--width/--height/--photon-launch/--method override the config's values.

Single GPU:  python bench.py [--config C] [--steps K --warmup W]
Multi GPU:   python bench.py --gpus N   (bench.py starts N rank processes itself, one per GPU,
             RCCL over xGMI), or under a launcher that sets WORLD_SIZE/RANK/LOCAL_RANK
             (torchrun --nproc-per-node N bench.py --gpus N).
             Default --partition batch (the reference's distributed mode): every
             rank renders its own whole iterations of the workload and the accumulated
             radiance is reduced over RCCL (weak scaling).  --partition rows (the default for
             --config 4, BASELINE's "pixel-tile shard over 8xMI355X"): one frame split by rows
             over the ranks (strong scaling; --scaling weak gives every rank a full photon
             launch).  See DESIGN.md "Multi-GPU".
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]

CONFIGS = {
    0: dict(scene="Cornell", width=256, height=256, method="pt", photon_launch=1024),
    1: dict(scene="Cornell", width=1024, height=1024, method="ppm", photon_launch=1024),
    2: dict(scene="SyntheticHall", width=1920, height=1080, method="ppm", photon_launch=2048),
    3: dict(scene="SyntheticHall", width=1920, height=1080, method="vcm", photon_launch=2048),
    4: dict(scene="SyntheticConference", width=3840, height=2160, method="ppm", photon_launch=4096),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--config", type=int, choices=sorted(CONFIGS), default=2,
                   help="BASELINE.json configs[i] (2 = the metric's 1080p Sponza-class PPM)")
    p.add_argument("--width", type=int)
    p.add_argument("--height", type=int)
    p.add_argument("--photon-launch", type=int)
    p.add_argument("--scene")
    p.add_argument("--method", choices=["ppm", "vcm", "pt"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=20.0)
    p.add_argument("--gather-variant", type=int, default=0)
    p.add_argument("--photon-map", choices=["grid", "hash", "kd"], default="grid",
                   help="uniform grid (the reference's shipped configuration), stochastic hash (single GPU) "
                        "or kd-tree (ACCELERATION_STRUCTURE_KD_TREE_CPU, built on the device)")
    p.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                   help="multi-GPU PPM: strong = fixed global photon launch split by rows over the ranks "
                        "(the default); weak = a full photon launch per rank")
    p.add_argument("--partition", choices=["batch", "rows", "slab"], default=None,
                   help="multi-GPU: batch = photon-batch (iteration) partition, the reference's distributed mode "
                        "and the default except for --config 4: every rank renders its own whole iterations "
                        "(global iteration numbers dealt round-robin, its own RNG streams) and the accumulated "
                        "radiance is summed by an RCCL reduce every --reduce-every iterations (weak scaling); "
                        "rows = one frame split by row-interleaved RNG/pixel/photon ownership, every rank "
                        "gathers all hit points against its own photons (strong scaling, equal to one device up "
                        "to fp32 order) -- the default for --config 4, whose BASELINE entry is a pixel-tile "
                        "shard over 8 GPUs; slab = rows with the gather partitioned by spatial photon slabs "
                        "(all-to-all of the photons; PPM only)")
    p.add_argument("--reduce-every", type=int, default=8,
                   help="photon-batch partition: local iterations between two reduces of the radiance buffers")
    p.add_argument("--force-sharded", action="store_true",
                   help="run the torch.distributed/RCCL sharded path even with one rank (tests the N>1 code)")
    p.add_argument("--no-serial-pass-times", action="store_true",
                   help="skip the few serial (unpipelined) iterations after the timed region that give each "
                        "pass's stand-alone time")
    a = p.parse_args(argv)
    requested = a.config
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.config = matching_config(a)
    if a.partition is None:
        # BASELINE.json configs[4] is "pixel-tile shard over 8xMI355X + RCCL radiance reduce": one frame
        # split over the GPUs (strong scaling); the other configs keep the reference's own distributed
        # mode, whole iterations per GPU (weak)
        a.partition = "rows" if requested == 4 and a.method == "ppm" else "batch"
    return a


def matching_config(a):
    """The BASELINE configs[] entry the resolved workload is (e.g. --method vcm on the default
    config is configs[3]); None for a workload that is none of them."""
    for i, cfg in CONFIGS.items():
        if all(getattr(a, k) == v for k, v in cfg.items() if not (k == "photon_launch" and cfg["method"] != "ppm")):
            return i
    return None


METHODS = {"ppm": 2, "vcm": 1, "pt": 0}  # orx_method (include/orx.h)
PHOTON_MAPS = {"grid": 0, "hash": 1, "kd": 2}  # orx_config.photon_map
_METHOD_NAME = {0: "PT", 1: "VCM", 2: "PPM"}


def _table(name, key):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name))).get(key, {})
    except (OSError, ValueError):
        return {}


def table_entries(table, kernels):
    """The entries of a per-kernel profile table (keys: kernel names with template arguments,
    tools/profile_traffic.short) that belong to the pass's kernels (base names, `k_kd_*` prefixes)."""
    out = {}
    for k, v in table.items():
        base = k.split("<")[0]
        if any(base == w or (w.endswith("*") and base.startswith(w[:-1])) for w in kernels):
            out[k] = v
    return out


def traffic_lookup(key, kernels):
    """PMC-measured HBM bytes per launch of the pass (2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md; mean over the bench's timed iterations) recorded by
    tools/profile_traffic.py for this exact workload, or None."""
    vals = [v["bytes_per_launch"] for v in table_entries(_table("traffic.json", key), kernels).values()]
    return int(sum(vals)) if vals else None


def profiled_kernels(key, kernels):
    """The pass's kernels (with template arguments) the committed PMC profile of this workload saw
    dispatched (None: no profile)."""
    return sorted(table_entries(_table("traffic.json", key), kernels)) or None


def bound_lookup(key, kernels):
    """What bounds the pass's longest kernel, from the committed PMC passes (profiles/bound.json,
    tools/pmc_bound.py): VALU issue, the vector-memory address path (TA) or HBM."""
    ent = table_entries(_table("bound.json", key), kernels)
    if not ent:
        return None
    k = max(ent, key=lambda n: ent[n].get("avg_us_standalone", ent[n].get("avg_us_profiled", 0.0)))
    return dict(ent[k], bound_kernel=k)


def host_cpu():
    """Threads the CPU baseline may use on this host and what they are: the process's CPU
    affinity, capped by a cgroup CPU quota and by OMP_NUM_THREADS when either is set (on the
    GPU box the harness grants one GPU's share of the node's cores and says so through
    OMP_NUM_THREADS)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    threads = aff
    if quota:
        threads = min(threads, max(1, int(math.floor(quota))))
    if omp:
        threads = min(threads, omp)
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp,
                     "node_cpus": os.cpu_count(), "model": model}


def cpu_baseline(scene, method, W, H, P, seconds, photon_map=0):
    """Oracle (oracle/liborx_oracle.so: the C/OpenMP restatement of the reference
    passes) on the host cores, same scene, resolution, photon count and seed as
    the GPU line.  Iteration 0 runs untimed; iterations 1, 2, ... are timed until
    `seconds` of CPU wall time are spent (at least one, at most 8); median."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from oppositerenderer_amd import _abi, roofline
    from oppositerenderer_amd.renderer import next_ppm_radius

    cores, info = host_cpu()
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
    # iteration 0 carries the buffer allocation, the RNG initialisation and (VCM) the light-vertex
    # estimate launch: untimed, like the GPU line's warmup
    r.render_next_iteration(0, 0, radius, req)
    radius = next_ppm_radius(radius, 0)
    times = []
    t_start = time.perf_counter()
    it = 1
    while it < 9 and (it == 1 or (time.perf_counter() - t_start) < seconds):
        t0 = time.perf_counter()
        r.render_next_iteration(it, it, radius, req)
        times.append(time.perf_counter() - t0)
        radius = next_ppm_radius(radius, it)
        it += 1
    r.close()
    t = float(np.median(times))
    paths = roofline.paths_per_iteration(method, W, H, P * P)
    return {"value": round(paths / t / 1e6, 3), "unit": "Mpaths/s", "cores": cores, "kind": "port",
            "ms_per_step": round(t * 1e3, 2), "value_per_core": round(paths / t / 1e6 / cores, 4),
            "host": info,
            "sample": f"oracle (C/OpenMP restatement of the reference passes, {cores} threads) on the full "
                      f"workload: {scene.name} {W}x{H} {_METHOD_NAME[method]}"
                      + (f", {P * P} photons/iter" if method == 2 else "") +
                      f"; median of {len(times)} iteration(s) after one untimed iteration"}


def roofline_block(pass_ms, pbytes, key, photon_map, serial_ms=None, overlapped=()):
    """The roofline entry for the kernel with the largest measured time per launch in the timed
    schedule (what rocprofv3 --stats shows dominant), with its stand-alone (serial) time when the
    schedule overlaps it with other passes."""
    from oppositerenderer_amd import roofline
    dominant = max(pass_ms, key=pass_ms.get)
    kernels = roofline.kernels_of(dominant, photon_map)
    seen = profiled_kernels(key, kernels)
    roof = roofline.roofline(dominant, pbytes[dominant], pass_ms[dominant], traffic_lookup(key, kernels),
                             photon_map=photon_map, kernels=seen)
    b = bound_lookup(key, kernels)
    if b:
        roof["bound"] = b.get("bound", "unmeasured")
        roof["bound_source"] = b.get("bound_source")
        # the compute roofline beside the HBM one: VALU issue slots of the chip's 1024 SIMD-32s
        # (calibrated cost per instruction, profiles/valu_calib.json), achieved fp32 FLOP/s, the
        # vector-memory address unit, and the fraction of wave time spent waiting
        roof["compute"] = {k: b[k] for k in ("valu_issue_frac", "fp32_tflops", "fp32_frac", "ta_frac", "wait_frac",
                                              "hbm_frac", "avg_us_standalone", "bound_kernel") if k in b}
        roof["compute"]["peak"] = ("VALU issue: 1024 SIMD-32 x clock at 4 cycles per wave64 instruction "
                                   "(profiles/valu_calib.json); fp32: 157.3 TFLOP/s; TA: 256 CUs x clock")
    else:
        roof["bound"] = "unmeasured"
    roof["overlapped"] = dominant in overlapped
    if serial_ms and dominant in serial_ms:
        roof["serial_ms"] = round(serial_ms[dominant], 4)
        roof["serial_achieved"] = round(pbytes[dominant] / (serial_ms[dominant] * 1e-3) / 1e9, 1)
        roof["serial_frac"] = round(roof["serial_achieved"] / roofline.HBM_PEAK_GBS, 5)
    return dominant, roof


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (RANK = LOCAL_RANK =
    0..N-1, rendezvous on 127.0.0.1) and wait for them.  This process never touches the GPU
    (nothing here initialises HIP), so the ranks are children, never an exec of this process.
    Rank 0 prints the JSON line on the inherited stdout.  If a rank fails, the others are
    stopped (they would wait in a collective forever) and the exit code is the failure's."""
    import socket
    import subprocess

    port = os.environ.get("MASTER_PORT")  # a caller-chosen port avoids the probe below
    if not port:
        # probe a free port (another process could take it before rank 0 binds it: set
        # MASTER_PORT to pin one where that matters)
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    procs = []
    for rank in range(n):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
                for q in procs:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                procs = []
                break
        time.sleep(0.05)
    return rc


def hw_queues():
    """HIP hardware queues for the multi-GPU paths, before the first HIP call: the pipelined row partition keeps
    torch's compute stream, the renderer's aux stream, the gather side stream, the finish stream and RCCL's busy at
    once; with HIP's default of 4 queues the side stream could share the compute stream's queue and the two
    serialise (configs[4] N=8 per-rank frame 8.05 against 6.56 ms with 8 queues, tools/shard_model.py --pipelined).
    Below 8 (or unset) it is raised to 16 (the pool allows 32) with a note on stderr -- the GPU boxes export 4 --
    unless ORX_KEEP_HW_QUEUES=1 keeps the caller's value; the bench line records the inherited and the used value
    (config.hw_queues)."""
    v = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["ORX_INHERITED_HW_QUEUES"] = v if v is not None else "unset"
    if os.environ.get("ORX_KEEP_HW_QUEUES", "0") == "1":
        return
    if v is None or int(v or 0) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"
        print(f"bench.py: GPU_MAX_HW_QUEUES {v if v is not None else 'unset'} -> 16 for the multi-GPU schedule "
              "(ORX_KEEP_HW_QUEUES=1 keeps it)", file=sys.stderr)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        hw_queues()  # inherited by the ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 or world > 1 or args.force_sharded:
        hw_queues()  # before the first HIP call
        from oppositerenderer_amd import multigpu
        return multigpu.bench_main(args, METRIC, cpu_baseline=None if args.no_cpu_baseline else cpu_baseline)

    from oppositerenderer_amd import _abi, roofline, scenes
    from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

    method = METHODS[args.method]
    W, H, P = args.width, args.height, args.photon_launch
    scene = scenes.scene_by_name(args.scene)
    pmap = PHOTON_MAPS[args.photon_map]
    cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P,
                              gather_variant=args.gather_variant, photon_map=pmap)
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
    st = r.stats()  # synchronises (the last iteration's deferred gather included)
    wall = time.perf_counter() - t0
    ms_per_step = wall * 1e3 / args.steps
    paths = roofline.paths_per_iteration(method, W, H, P * P)
    value = paths * args.steps / wall / 1e6

    n_it = max(1, st.timed_iterations)
    per_pass = {name: st.pass_ms[i] / n_it for i, name in enumerate(_abi.PASS_NAMES)}
    per_pass = {k: v for k, v in per_pass.items() if v > 0}
    # pipelined PPM: the gather and output run on a side stream beside the next iteration's
    # passes, so every pass time is wall time under interference; a few serial iterations after
    # the timed region give each pass's stand-alone time
    pipelined = r.pipelined()
    # the pipelined PPM grid build's schedule, chosen by the renderer from its first pipelined iteration
    # (orx.h orx_ppm_grid_schedule); read before the serial legs below
    gsched, gprobe = r.grid_schedule() if method == _abi.PROGRESSIVE_PHOTON_MAPPING else (0, (0.0, 0.0))
    # pipelined (single device): gather + output of iteration i beside iteration i+1's passes, the
    # direct pass beside the grid build, and the eye pass of i+1 on the direct pass's stream beside
    # the grid build of i, so the chain per frame is photon pass + grid build
    # VCM: the deferred shadow rays and colours of iteration i beside the light pass and camera
    # subpaths of i+1
    overlapped = ([] if not pipelined else ["ppm_eye", "ppm_gather", "ppm_direct_output"]
                  if method == _abi.PROGRESSIVE_PHOTON_MAPPING else ["vcm_shadow"])
    serial = None
    if pipelined and not args.no_serial_pass_times:
        r.set_iteration_pipelining(0)
        for k in range(4):
            if k == 1:
                r.stats()
                r.reset_timing()
            r.renderNextIteration(it, it, radius, False, det)
            radius = next_ppm_radius(radius, it)
            it += 1
        ss = r.stats()
        sn = max(1, ss.timed_iterations)
        serial = {name: ss.pass_ms[i] / sn for i, name in enumerate(_abi.PASS_NAMES) if ss.pass_ms[i] > 0}
        r.set_iteration_pipelining(-1)
    valid_avg = st.valid_photons_total / n_it
    light_vertices = 0
    if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING:
        light_vertices = int(np.minimum(r.read_buffer(_abi.BUF_VCM_VERTEX_COUNT, np.uint32), 9).sum())
    pbytes = roofline.pass_bytes(method, W, H, P * P, valid_avg, st.num_cells, light_vertices, photon_map=pmap,
                                 vcm_entries=st.vcm_shadow_rays if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING else 0,
                                 vcm_light_entries=st.vcm_light_connections
                                 if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING else 0)
    key = (f"{scene.name}:{W}x{H}:{args.method}" + (f":P{P}" if method == 2 else "")
           + (f":{args.photon_map}" if pmap else ""))
    dominant, roof = roofline_block(per_pass, pbytes, key, pmap, serial, overlapped)
    if pipelined:
        chain = {k: round(v, 4) for k, v in per_pass.items() if k not in overlapped}
        roof["critical_chain_ms"] = chain
    passes = {k: {"ms": round(v, 4), "algorithmic_GBps": round(pbytes.get(k, 0) / (v * 1e-3) / 1e9, 1)}
              for k, v in per_pass.items()}
    if serial:
        for k, v in serial.items():
            if k in passes:
                passes[k]["serial_ms"] = round(v, 4)
    if method == _abi.PROGRESSIVE_PHOTON_MAPPING and dominant == "ppm_gather":
        # SURVEY 8(d) prices the gather as N*(64+12) + Z*8 + V*36 with V the photons in the
        # reference's search windows; those window photons are re-read from L1/LDS, not HBM
        # (each grid photon is loaded once per 8x8 wave tile), so the algorithmic bytes here
        # charge each grid photon once
        visited = st.photons_visited_total / n_it
        roof["bytes_model"] = ("hit points 40 B + indirect 12 B per pixel, each grid photon once (36 B), "
                               "offsets once; departs from SURVEY 8(d)'s V x 36 B per window photon")
        roof["window_photons_per_launch"] = int(visited)
    data = ("synthetic: seeded procedural scene (" + scene.name + "), XORWOW streams seeded 1645301512; "
            "no assets or checkpoints")
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        # one GPU: the per-GPU work of the default multi-GPU partition (batch: whole iterations per GPU)
        "scaling": "weak" if args.partition == "batch" else "strong",
        "vs_baseline": None, "dtype": "f32", "data": data,
        "config": {"workload": f"{scene.name} {W}x{H} {_METHOD_NAME[method]}"
                               + (f", {P * P} photons/iter" if method == 2 else ""),
                   "baseline_config": args.config,
                   "scene": scene.name, "width": W, "height": H, "method": _METHOD_NAME[method],
                   "photons_per_iteration": P * P if method == 2 else 0, "paths_per_iteration": paths,
                   "photon_map": {"grid": "uniform grid", "hash": "stochastic hash", "kd": "kd-tree"}[args.photon_map],
                   "pipelined": bool(pipelined), "parallelism": "single GPU"},
        "roofline": roof,
        "passes": passes,
        "dominant_pass": dominant,
        "overlapped_passes": overlapped,
    }
    if pipelined and method == _abi.PROGRESSIVE_PHOTON_MAPPING:
        out["config"]["grid_build"] = {-1: "not chosen", 0: "synchronous", 1: "asynchronous"}.get(gsched, "n/a")
        out["config"]["grid_build_measured_ms"] = {"photon_and_grid": round(gprobe[0], 4),
                                                   "gather": round(gprobe[1], 4)}
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(scene, method, W, H, P, args.cpu_seconds, photon_map=pmap)
        except Exception as e:  # the baseline must never hide the GPU line
            out["cpu_baseline"] = {"error": repr(e)}
    r.destroy()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
