"""Stochastic-hash photon map (orx_config.photon_map = 1) on the oracle: the restatement of
ACCELERATION_STRUCTURE_STOCHASTIC_HASH (OptixRenderer_SpatialHash.cu:286-302, store_photon.h,
IndirectRadianceEstimation.cu:131-162) keeps its invariants.  GPU parity: test_gpu_parity.py."""
import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes
from oppositerenderer_amd.renderer import next_ppm_radius

SEED = 1645301512


def render(photon_map, W=40, H=32, P=32, iters=2):
    scene = scenes.cornell()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P, photon_map=photon_map)
    r = oracle_lib.OracleRenderer(cfg)
    oracle_lib.load().orc_set_threads(4)
    r.init_scene(scene)
    req = _abi.OrxRequest()
    req.camera = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H))).to_abi()
    req.method, req.width, req.height, req.ppm_alpha = _abi.PROGRESSIVE_PHOTON_MAPPING, W, H, 2.0 / 3.0
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        r.render_next_iteration(it, it, radius, req)
        last = radius
        radius = next_ppm_radius(radius, it)
    return r, last, scene


def test_hash_table_invariants():
    r, radius, scene = render(_abi.PHOTON_MAP_STOCHASTIC_HASH)
    counts = r.read_buffer(_abi.BUF_GRID_OFFSETS, np.uint32)
    table = r.read_buffer(_abi.BUF_PHOTONS).reshape(-1, 9)
    st = r.stats()
    assert counts.size == 32 * 32 * 4 and st.num_cells == counts.size
    assert counts.sum() == st.valid_photons > 0
    # an entry holds a photon iff its count is nonzero; that photon hashes to the entry
    assert np.all((np.abs(table).sum(1) > 0) <= (counts > 0))
    o = np.array(st.world_origin, np.float32)
    inv = np.float32(1.0) / np.float32(st.cell_size)
    occupied = np.nonzero(counts)[0]
    pos = table[occupied, 3:6].astype(np.float32)
    c = np.floor((pos - o) * inv).astype(np.int64)
    gx, gy = st.grid_size[0], st.grid_size[1]
    h = (c[:, 0] + c[:, 1] * gx + c[:, 2] * gx * gy) & (counts.size - 1)
    assert np.array_equal(h, occupied)
    # the hash grid: cell = r, origin = scene AABB min - (r + 1e-4)
    assert st.cell_size == np.float32(radius)
    assert np.allclose(o, np.array([-5, -5, -5], np.float32) - (radius + 1e-4), atol=1e-4)
    # 27 cells per non-specular hit point
    dbg = r.read_buffer(_abi.BUF_DEBUG_VISITED, np.uint32).reshape(-1, 2)
    assert set(np.unique(dbg[:, 0])) <= {0, 27} and np.array_equal(dbg[:, 0], dbg[:, 1])


def test_hash_deposits_are_uncapped():
    """store_photon.h's hash STORE_PHOTON never counts, so paths deposit past max_photon_deposits."""
    r, _, _ = render(_abi.PHOTON_MAP_STOCHASTIC_HASH)
    g, _, _ = render(_abi.PHOTON_MAP_UNIFORM_GRID)
    assert r.stats().valid_photons > g.stats().valid_photons


def test_hash_estimate_is_close_to_grid():
    """Both are consistent estimators of the same indirect light: images agree to a loose tolerance."""
    r, _, _ = render(_abi.PHOTON_MAP_STOCHASTIC_HASH, W=32, H=32, P=64, iters=3)
    g, _, _ = render(_abi.PHOTON_MAP_UNIFORM_GRID, W=32, H=32, P=64, iters=3)
    a, b = r.output().mean(), g.output().mean()
    assert a > 0 and b > 0 and abs(a - b) / b < 0.5


def test_hash_config_rejected_when_not_power_of_two():
    from oppositerenderer_amd import renderer
    import ctypes as C
    lib = renderer.load_library()
    h = C.c_void_p()
    cfg = _abi.default_config(photon_launch_width=48, photon_launch_height=32, photon_map=1)
    st = lib.orx_create(0, C.byref(cfg), C.byref(h))
    assert st == _abi.ORX_ERR_INVALID_ARGUMENT and not h.value
