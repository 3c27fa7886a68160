"""GPU parity at the BASELINE workloads' full sizes (BASELINE.json configs[0]-[3]).

The parity tests in test_gpu_parity.py run toy sizes (<= 96x80 pixels, <= 128^2
photons).  These run the bench's own workloads through liborx.so and the CPU
oracle on the same seeds, so the multi-chunk bucket sort, the full 1e6-cell
grid, the 2M-pixel gather and the full light-vertex cache are compared at the
sizes bench.py times:

  configs[0]  Cornell 256x256 PT, 1 spp                 output + RNG bit-exact
  configs[1]  Cornell 1024x1024 PPM, 1024^2 photons      two iterations (radius update)
  configs[2]  hall 1920x1080 PPM, 2048^2 photons         two iterations
  configs[3]  hall 1920x1080 VCM                         two iterations (the first runs the LVC estimate
                                                         launch; the second is the bench's steady state)
  configs[4]  conference 3840x2160 PPM, 4096^2 photons   one iteration on one device, and the same frame
                                                         through eight row-interleaved shards (strong
                                                         scaling, the 8-GPU bench's partition)

Bars (north_star; same as check_ppm_iteration / check_vcm_iteration): RNG,
hit points, grid offsets, per-cell photon multisets, direct light, visit
counters, VCM vertex counts / light vertices / camera colours bit-exact;
indirect and splats rel-L2 <= 1e-5 (summation order); output rel-L2 <= 1e-4.
The oracle runs on the box's host cores (OMP_NUM_THREADS).
"""
import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes, synthetic
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

pytestmark = pytest.mark.gpu
SEED = 1645301512


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).sum()) / max(np.sqrt((b * b).sum()), 1e-30))


def cell_sorted_photons(photons, offsets):
    """Grid-ordered photons [n, 9] with each cell's rows put in a canonical
    order (by a 64-bit hash of the row): equal arrays <=> every cell holds the
    same multiset of photons (two different rows of one cell with equal hashes
    would only make equal multisets compare unequal, never the reverse)."""
    rows = np.ascontiguousarray(photons.view(np.uint32).reshape(-1, 9))
    off = offsets.astype(np.int64)
    n = int(off[-1] - off[0])
    assert rows.shape[0] == n, (rows.shape, n)
    cell = np.repeat(np.arange(len(off) - 1, dtype=np.int32), np.diff(off))
    h = np.zeros(n, np.uint64)
    with np.errstate(over="ignore"):
        for k in range(9):
            h = (h * np.uint64(0x100000001B3)) ^ rows[:, k].astype(np.uint64)
    order = np.lexsort((h, cell))
    return rows[order]


def assert_same(gpu, ora, buf, what=None):
    g, o = gpu.read_buffer(buf, np.uint32), ora.read_buffer(buf, np.uint32)
    assert g.shape == o.shape, (what or buf, g.shape, o.shape)
    mism = np.count_nonzero(g != o)
    assert mism == 0, f"{what or buf}: {mism} of {g.size} words differ"


def check_ppm_full(gpu, ora):
    for buf, name in ((_abi.BUF_RNG, "rng"), (_abi.BUF_HITPOINTS, "hitpoints"), (_abi.BUF_GRID_OFFSETS, "offsets"),
                      (_abi.BUF_DIRECT, "direct"), (_abi.BUF_DEBUG_VISITED, "visit counters")):
        assert_same(gpu, ora, buf, name)
    gs, os_ = gpu.stats(), ora.stats()
    assert list(gs.grid_size) == list(os_.grid_size)
    assert np.float32(gs.cell_size) == np.float32(os_.cell_size)
    assert gs.valid_photons == os_.valid_photons
    assert gs.photons_visited == os_.photons_visited
    off = gpu.read_buffer(_abi.BUF_GRID_OFFSETS, np.uint32)
    gp = cell_sorted_photons(gpu.read_buffer(_abi.BUF_PHOTONS), off)
    op = cell_sorted_photons(ora.read_buffer(_abi.BUF_PHOTONS), off)
    assert np.array_equal(gp, op), "per-cell photon multisets differ"
    gi, oi = gpu.read_buffer(_abi.BUF_INDIRECT), ora.read_buffer(_abi.BUF_INDIRECT)
    assert rel_l2(gi, oi) < 1e-5, rel_l2(gi, oi)
    np.testing.assert_allclose(gi, oi, rtol=1e-4, atol=1e-6)


def pair(scene, W, H, P, method):
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
    gpu = OptixRenderer(cfg)
    gpu.initialize(0)
    gpu.initScene(scene)
    ora = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
    ora.init_scene(scene)
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    return gpu, ora, RenderRequestDetails(cam, scene.name, method, W, H)


def test_configs0_cornell256_pt():
    scene = scenes.cornell()
    gpu, ora, det = pair(scene, 256, 256, 1024, _abi.PATH_TRACING)
    for it in range(2):
        gpu.renderNextIteration(it, it, 1.0, True, det)
        ora.render_next_iteration(it, it, 1.0, det.to_abi())
        assert_same(gpu, ora, _abi.BUF_RNG, "rng")
    g, o = gpu.getOutputBuffer(), ora.output()
    assert g.mean() > 0
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32)), rel_l2(g, o)
    gpu.destroy()
    ora.close()


@pytest.mark.parametrize("which", ["configs1_cornell1024_ppm", "configs2_hall1080p_ppm"])
def test_full_size_ppm(which):
    if which.startswith("configs1"):
        scene, W, H, P = scenes.cornell(), 1024, 1024, 1024
    else:
        scene, W, H, P = synthetic.synthetic_hall(), 1920, 1080, 2048
    gpu, ora, det = pair(scene, W, H, P, _abi.PROGRESSIVE_PHOTON_MAPPING)
    radius = scene.initial_ppm_radius()
    for it in range(2):
        gpu.renderNextIteration(it, it, radius, True, det)
        ora.render_next_iteration(it, it, radius, det.to_abi())
        check_ppm_full(gpu, ora)
        radius = next_ppm_radius(radius, it)
    g, o = gpu.getOutputBuffer(), ora.output()
    assert g.mean() > 0
    assert rel_l2(g, o) < 1e-4, rel_l2(g, o)
    gpu.destroy()
    ora.close()


def check_vcm_full(gpu, ora, W, H):
    for buf, name in ((_abi.BUF_RNG, "rng"), (_abi.BUF_VCM_VERTEX_COUNT, "vertex counts"),
                      (_abi.BUF_VCM_CAMERA, "camera colours")):
        assert_same(gpu, ora, buf, name)
    cnt = np.minimum(gpu.read_buffer(_abi.BUF_VCM_VERTEX_COUNT, np.uint32), 9)
    assert cnt.sum() > W * H // 2
    gv = gpu.read_buffer(_abi.BUF_VCM_VERTICES, np.uint32).reshape(9, -1, 16)  # 9 x W*H x 64 B
    ov = ora.read_buffer(_abi.BUF_VCM_VERTICES, np.uint32).reshape(9, -1, 16)
    for k in range(9):  # one vertex level at a time: only stored vertices are defined
        sel = cnt > k
        assert np.array_equal(gv[k][sel], ov[k][sel]), f"light vertices of level {k} differ"
    del gv, ov
    gs, os_ = gpu.read_buffer(_abi.BUF_VCM_SPLAT), ora.read_buffer(_abi.BUF_VCM_SPLAT)
    assert rel_l2(gs, os_) < 1e-5, rel_l2(gs, os_)


def test_configs3_hall1080p_vcm():
    """Iteration 0 (with the light-vertex-count estimate launch, OptixRenderer.cpp:699-773) and
    iteration 1, the steady state bench.py times: the camera pass continues each slot's RNG
    stream from the light pass of the same iteration (VCMLightPass.cu:88, VCMCameraPass.cu:79,
    112) and the vertex cache is rewritten."""
    scene = synthetic.synthetic_hall()
    W, H = 1920, 1080
    gpu, ora, det = pair(scene, W, H, 64, _abi.VCM_BIDIRECTIONAL_PATH_TRACING)
    radius = scene.initial_ppm_radius()
    for it in range(2):
        gpu.renderNextIteration(it, it, radius, True, det)
        ora.render_next_iteration(it, it, radius, det.to_abi())
        check_vcm_full(gpu, ora, W, H)
        radius = next_ppm_radius(radius, it)
    g, o = gpu.getOutputBuffer(), ora.output()
    assert np.isfinite(g).all() and g.mean() > 0
    assert rel_l2(g, o) < 1e-4, rel_l2(g, o)
    gpu.destroy()
    ora.close()


def test_configs4_conference4k_ppm_single_and_8_shards():
    """configs[4] (IndirectRadianceEstimation.cu:69-227, OptixRenderer.cpp:569-673) at full size:
    conference 3840x2160, 4096^2 = 16,777,216 emitted photons, one iteration.

    1. One device against the oracle with check_ppm_full's bars (RNG, hit points, offsets,
       per-cell photon multisets, direct, visit counters bit-exact; indirect rel-L2 <= 1e-5).
    2. The same frame through eight row-interleaved shards in the 8-GPU bench's strong-scaling
       partition (each shard: 1/8 of the pixel rows, photon launch rows and RNG rows; cell-order
       photon layout and the gather that world >= 8 selects), exchanging hit points, photons
       (slab mode) and partial indirect through torch ops (tests/shard_emul.py), against the
       oracle's output: rel-L2 <= 1e-5, with spatial photon slabs and with the row partition
       (the bench's default, `bench.py --partition rows`)."""
    import torch

    from oppositerenderer_amd import multigpu

    scene = synthetic.synthetic_conference()
    W, H, P = 3840, 2160, 4096
    gpu, ora, det = pair(scene, W, H, P, _abi.PROGRESSIVE_PHOTON_MAPPING)
    radius = scene.initial_ppm_radius()
    gpu.renderNextIteration(0, 0, radius, True, det)
    ora.render_next_iteration(0, 0, radius, det.to_abi())
    check_ppm_full(gpu, ora)
    assert gpu.stats().valid_photons > P * P // 2
    g, o = gpu.getOutputBuffer(), ora.output()
    assert g.mean() > 0
    assert rel_l2(g, o) < 1e-4, rel_l2(g, o)
    gpu.destroy()
    ora.close()
    del g
    torch.cuda.empty_cache()

    import shard_emul

    world = 8
    req = det.to_abi()
    for slab in (True, False):  # spatial slabs, and the row partition (the bench default)
        shards = shard_emul.make_shards(scene, world, P, P, slab=slab)
        got, plans = shard_emul.run_iterations(shards, scene, W, H, req, 1, slab=slab)
        assert np.isfinite(got).all()
        assert rel_l2(got, o) < 1e-5, (slab, rel_l2(got, o))
        for b in shards:
            b.r.destroy()
        del shards, got
        torch.cuda.empty_cache()
