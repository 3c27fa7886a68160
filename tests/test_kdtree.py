"""kd-tree photon map (orx_config.photon_map = 2) on the oracle: the restatement of
ACCELERATION_STRUCTURE_KD_TREE_CPU (OptixRenderer_CPUKdTree.cpp:27-127 with select.h, and the
traversal of IndirectRadianceEstimation.cu:164-209) keeps the tree's invariants and gathers the
same photons a brute-force radius search finds.  GPU parity: test_gpu_parity.py."""
import numpy as np
import pytest

import oracle_lib
from oppositerenderer_amd import _abi, scenes
from oppositerenderer_amd.renderer import next_ppm_radius

SEED = 1645301512
PPM_X, PPM_Y, PPM_Z, PPM_LEAF, PPM_NULL = 1, 2, 4, 8, 16


def render(photon_map, W=40, H=32, P=32, iters=2, scene=None):
    scene = scene or scenes.cornell()
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


def read_tree(r):
    t = r.read_buffer(_abi.BUF_KD_TREE).reshape(-1, 10)
    return t[:, :9].copy(), t[:, 9].copy().view(np.uint32)


def walk(photons, axis, root=0):
    """Reachable nodes of the implicit tree: (index, depth) in DFS order."""
    out, stack = [], [(root, 0)]
    while stack:
        i, d = stack.pop()
        out.append((i, d))
        a = axis[i]
        if a & (PPM_NULL | PPM_LEAF):
            continue
        stack.append((2 * i + 2, d + 1))
        stack.append((2 * i + 1, d + 1))
    return out


def check_tree(photons, axis, valid_slots):
    """The invariants every correct build of the reference's tree keeps, however its median
    selection breaks ties: node sizes follow median = (start+end)/2, every split node's left
    subtree lies at or below its coordinate and the right at or above, and the tree holds
    exactly the valid photons.  Vectorised level by level; returns the reachable nodes."""
    T = axis.size
    L = int(np.log2(T + 1))
    reach = np.zeros(T, bool)
    reach[0] = True
    split = lambda i: (axis[i] & (PPM_NULL | PPM_LEAF)) == 0
    for l in range(L - 1):
        lv = np.arange(2 ** l - 1, 2 ** (l + 1) - 1)
        sp = lv[reach[lv] & split(lv)]
        assert np.all(np.isin(axis[sp], (PPM_X, PPM_Y, PPM_Z)))
        reach[2 * sp + 1] = True
        reach[2 * sp + 2] = True
    last = np.arange(2 ** (L - 1) - 1, T)
    assert not np.any(reach[last] & split(last))  # the deepest level holds leaves and NULL nodes only
    held = reach & ((axis & PPM_NULL) == 0)
    # multiset of the photons held == the valid slots
    a = np.sort(photons[held].view(np.uint32).view([("", np.uint32)] * 9).ravel())
    b = np.sort(valid_slots.view(np.uint32).view([("", np.uint32)] * 9).ravel())
    assert a.size == b.size and np.array_equal(a, b)
    # bottom-up subtree sizes and coordinate ranges
    size = held.astype(np.int64)
    lo = np.where(held[:, None], photons[:, 3:6], np.inf)
    hi = np.where(held[:, None], photons[:, 3:6], -np.inf)
    for l in range(L - 2, -1, -1):
        lv = np.arange(2 ** l - 1, 2 ** (l + 1) - 1)
        sp = lv[reach[lv] & split(lv)]
        cl, cr = 2 * sp + 1, 2 * sp + 2
        k = np.log2(axis[sp]).astype(np.int64)
        v = photons[sp, 3 + k]
        assert np.all(hi[cl, k] <= v) and np.all(lo[cr, k] >= v)
        n = 1 + size[cl] + size[cr]
        assert np.array_equal(size[cl], n // 2) and np.array_equal(size[cr], n - n // 2 - 1)
        size[sp] = n
        lo[sp] = np.minimum(lo[sp], np.minimum(lo[cl], lo[cr]))
        hi[sp] = np.maximum(hi[sp], np.maximum(hi[cl], hi[cr]))
    return np.nonzero(reach)[0]


def test_kdtree_invariants():
    r, radius, scene = render(_abi.PHOTON_MAP_KD_TREE)
    photons, axis = read_tree(r)
    st = r.stats()
    S = 32 * 32 * 4
    assert photons.shape[0] == st.num_cells == 2 ** int(np.ceil(np.log2(S + 1))) - 1  # pow2roundup(S+1)-1
    slots = r.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9)
    valid = slots[slots[:, 0:3].max(1) > 0]
    assert st.valid_photons == valid.shape[0] > 0
    nodes = check_tree(photons, axis, valid)
    assert np.array_equal(nodes, sorted(i for i, _ in walk(photons, axis)))
    # balanced: depth = ceil(log2(n + 1)) levels
    assert int(np.log2(nodes.max() + 1)) + 1 == int(np.ceil(np.log2(valid.shape[0] + 1)))


def test_kdtree_gather_matches_brute_force():
    """The traversal finds every photon within the radius: the indirect estimate equals a
    brute-force sum over all valid photons (float64, so within fp32 summation order)."""
    r, radius, _ = render(_abi.PHOTON_MAP_KD_TREE, iters=1)
    hp = r.read_buffer(_abi.BUF_HITPOINTS).reshape(-1, 13)
    flags = hp[:, 12].copy().view(np.uint32)
    slots = r.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9).astype(np.float64)
    valid = slots[slots[:, 0:3].max(1) > 0]
    ind = r.read_buffer(_abi.BUF_INDIRECT).reshape(-1, 3)
    r2 = np.float64(np.float32(radius) * np.float32(radius))
    P = 32 * 32
    ns = np.nonzero(flags & _abi.PRD_HIT_NON_SPECULAR)[0]
    assert ns.size > 0
    ref = np.zeros((hp.shape[0], 3))
    for i in ns:
        d = hp[i, 0:3].astype(np.float64) - valid[:, 3:6]
        d2 = (d * d).sum(1)
        ok = (d2 <= r2) & ((-valid[:, 6:9] * hp[i, 3:6]).sum(1) >= 0)
        w = 1.818 * (1 - (1 - np.exp(-1.953 * d2[ok] / (2 * r2))) / (1 - 0.141847))
        ref[i] = (valid[ok, 0:3] * w[:, None]).sum(0) * hp[i, 6:9] / (np.pi * r2) / P
    err = np.sqrt(((ind - ref) ** 2).sum() / (ref ** 2).sum())
    assert err < 2e-5, err


def test_kdtree_and_grid_gather_the_same_photons():
    """Same photons, hit points and RNG streams as the uniform grid: the two photon maps'
    indirect estimates differ only by fp32 summation order."""
    k, _, _ = render(_abi.PHOTON_MAP_KD_TREE)
    g, _, _ = render(_abi.PHOTON_MAP_UNIFORM_GRID)
    assert np.array_equal(k.read_buffer(_abi.BUF_HITPOINTS), g.read_buffer(_abi.BUF_HITPOINTS))
    # cleared slots keep a stale direction (PhotonGenerator.cu:111-118 zeroes power and position only)
    ks, gs = (x.read_buffer(_abi.BUF_PHOTON_SLOTS).reshape(-1, 9) for x in (k, g))
    assert np.array_equal(ks[:, :6], gs[:, :6])
    v = ks[:, 0:3].max(1) > 0
    assert np.array_equal(ks[v], gs[v])
    a, b = k.read_buffer(_abi.BUF_INDIRECT), g.read_buffer(_abi.BUF_INDIRECT)
    err = np.sqrt(((a - b) ** 2).sum() / (b ** 2).sum())
    assert err < 1e-5, err
    dbg = k.read_buffer(_abi.BUF_DEBUG_VISITED, np.uint32).reshape(-1, 2)
    assert np.all(dbg[:, 0] == 0) and dbg[:, 1].sum() == k.stats().photons_visited > 0


def test_kdtree_empty_photon_map():
    """No valid photons (every surface a mirror: mirrors never store, Mirror.cu:65-77): the root
    is a NULL node, the gather visits it once per non-specular hit point and adds nothing."""
    scene = scenes.cornell()
    for i, m in enumerate(scene.materials):
        if m.type == _abi.MAT_DIFFUSE:
            scene.materials[i] = scenes.Mirror((0.5, 0.5, 0.5))
    r, _, _ = render(_abi.PHOTON_MAP_KD_TREE, W=16, H=16, P=16, iters=1, scene=scene)
    photons, axis = read_tree(r)
    assert r.stats().valid_photons == 0
    assert axis[0] == PPM_NULL
    assert np.all(r.read_buffer(_abi.BUF_INDIRECT) == 0)
