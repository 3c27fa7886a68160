#!/usr/bin/env python3
"""Traversal statistics on the GPU (build: make -C oppositerenderer_amd/csrc stats).
Prints per-iteration rays / inner nodes / leaves / triangle tests for closest-hit
and any-hit traversals of one bench workload."""
import ctypes as C
import os
import sys

import numpy as np
import torch  # noqa: F401  (torch's HIP runtime before liborx's first HIP call, as tests/conftest.py)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oppositerenderer_amd import _abi, renderer, scenes  # noqa: E402

lib = renderer.load_library(os.environ.get("ORX_STATS_LIB") or os.path.join(ROOT, "oppositerenderer_amd", "liborx_stats.so"))
SHARD = 0
if "--shard" in sys.argv:  # the row partition's gather of rank 0 of N (all W*H hit points, its own photons)
    k = sys.argv.index("--shard")
    SHARD = int(sys.argv[k + 1])
    del sys.argv[k:k + 2]
GV = 0
if "--variant" in sys.argv:  # orx_config.gather_variant: 1 cell order, 2 sub-rows (0: the renderer's choice)
    k = sys.argv.index("--variant")
    GV = int(sys.argv[k + 1])
    del sys.argv[k:k + 2]
lib.orx_trav_stats_read.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
scene_name = sys.argv[1] if len(sys.argv) > 1 else "SyntheticHall"
method = {"ppm": 2, "vcm": 1, "pt": 0}[sys.argv[2] if len(sys.argv) > 2 else "ppm"]
W, H, P = (1920, 1080, 2048) if scene_name.startswith("Synthetic") else (1024, 1024, 1024)
if len(sys.argv) > 3:  # WxHxP
    W, H, P = (int(v) for v in sys.argv[3].split("x"))
sc = scenes.scene_by_name(scene_name)
if SHARD:
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import shard_model
    from oppositerenderer_amd import multigpu
    dev = torch.device("cuda", 0)
    req = renderer.RenderRequestDetails(sc.default_camera.set_aspect_ratio(W / H), sc.name, 2, W, H).to_abi()
    its = 6
    hps = shard_model.full_hitpoints(sc, W, H, SHARD, its, dev, req)
    r = renderer.OptixRenderer(_abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P,
                                                   gather_variant=GV))
    r.initialize(0)
    r.set_shard(0, SHARD)
    r.initScene(sc)
    b = multigpu.DeviceShard(r, torch, dev)
    mr = (H + SHARD - 1) // SHARD
    part = b.alloc(SHARD * mr * W * 3)
    buf = (C.c_ulonglong * 21)()
    radii = multigpu.radius_sequence(sc.initial_ppm_radius(), its)
    waves = SHARD * mr * W / 64
    for it in range(its):
        b.local_passes(it, it, radii[it], req)
        assert lib.orx_trav_stats_read(r._h, buf, 1) == 0  # drop the local passes' counts
        b.gather_external(hps[it], SHARD, part)
        torch.cuda.synchronize()
        assert lib.orx_trav_stats_read(r._h, buf, 1) == 0
        v = list(buf)
        lc, up, nr, wr = v[12], v[13], v[14], v[15]
        print(f"it{it} shard 0/{SHARD} gather: lane candidates/px {lc / (W * H):8.2f}  union photons/wave {up / waves:8.1f}"
              f"  union factor {64 * up / max(1, lc):5.2f}  lane sub-rows/px {nr / (W * H):6.2f}"
              f"  wave sub-rows/wave {wr / waves:6.2f} (with photons {v[16] / waves:6.2f})"
              f"  union photons per non-empty wave sub-row {up / max(1, v[16]):6.1f}", flush=True)
    sys.exit(0)
r = renderer.OptixRenderer(_abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P))
r.initialize(0)
r.initScene(sc)
det = renderer.RenderRequestDetails(sc.default_camera.set_aspect_ratio(W / H), sc.name, method, W, H)
buf = (C.c_ulonglong * 21)()
radius = sc.initial_ppm_radius()
for it in range(3):
    r.renderNextIteration(it, it, radius, False, det)
    radius = renderer.next_ppm_radius(radius, it)
    assert lib.orx_trav_stats_read(r._h, buf, 1) == 0
    v = list(buf)
    for name, b in (("closest", 0), ("any", 4)):
        rays = max(1, v[b])
        wn, wl = v[8 + b // 2], v[9 + b // 2]
        print(f"it{it} {name:8s} rays {v[b]:12d}  nodes/ray {v[b + 1] / rays:6.2f}  leaves/ray {v[b + 2] / rays:6.2f}"
              f"  tris/ray {v[b + 3] / rays:6.2f}  SIMT node {v[b + 1] / max(1, 64 * wn):5.3f}"
              f"  leaf {v[b + 2] / max(1, 64 * wl):5.3f}")
    print(f"it{it} closest node visits in the top BVH4 levels (index < 21/85/341/1365): "
          + " ".join(f"{v[17 + q] / max(1, v[1]):5.3f}" for q in range(4)))
    if method == 2:  # the union gather (single device)
        lc, up, nr = v[12], v[13], v[14]
        waves = W * H / 64
        print(f"it{it} union    lane candidates/px {lc / (W * H):8.1f}  union photons/px {64 * up / (W * H):8.1f}"
              f"  union factor {64 * up / max(1, lc):5.2f}  lane sub-rows/px {nr / (W * H):6.1f}"
              f"  wave sub-rows/wave {v[15] / waves:6.2f} (with photons {v[16] / waves:6.2f})")
print("bvh stack entries", r.stats().bvh_stack_entries)
