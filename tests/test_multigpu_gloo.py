"""N>1 path on CPU: the sharded PPM iteration of oppositerenderer_amd.multigpu,
run by 2 (and 3) gloo ranks over the oracle backend, must equal one renderer
tracing the union photon launch (up to fp32 summation order in the gather).

This exercises the same orchestration code the RCCL bench path uses
(row-interleaved ownership, hitpoint all-gather, indirect reduce-scatter,
row reassembly)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib
from oppositerenderer_amd import _abi, multigpu, scenes
from oppositerenderer_amd.renderer import next_ppm_radius

SEED = 1645301512


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def request(scene, W, H, method=_abi.PROGRESSIVE_PHOTON_MAPPING):
    req = _abi.OrxRequest()
    req.camera = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H))).to_abi()
    req.method = method
    req.width, req.height, req.ppm_alpha = W, H, 2.0 / 3.0
    return req


def worker(rank, world, port, out_path, W, H, P, iters, method=_abi.PROGRESSIVE_PHOTON_MAPPING, photon_map=0,
           PH=None, slab=False):
    """PH: global photon launch height (default P * world: every rank a full P x P batch)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = scenes.cornell()
    PH = P * world if PH is None else PH
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=PH, photon_map=photon_map)
    r = oracle_lib.OracleRenderer(cfg)
    oracle_lib.load().orc_set_threads(2)
    r.init_scene(scene)
    b = oracle_lib.OracleShard(r, torch)
    b.set_shard(rank, world)
    cls = {_abi.VCM_BIDIRECTIONAL_PATH_TRACING: multigpu.ShardedVCM,
           _abi.PATH_TRACING: multigpu.ShardedPT}.get(method, multigpu.ShardedPPM)
    sh = cls(b, dist, world, rank, W, H, slab=slab) if slab else cls(b, dist, world, rank, W, H)
    req = request(scene, W, H, method)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        sh.iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    img = sh.image()
    if rank == 0:
        np.save(out_path, img)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,photon_map,scaling", [(2, 48, 40, 0, "weak"), (3, 40, 37, 0, "weak"),
                                                            (2, 48, 40, 2, "weak"), (2, 48, 40, 0, "strong"),
                                                            (3, 40, 37, 0, "strong"), (2, 48, 40, 2, "strong"),
                                                            (3, 41, 37, 0, "strong")])
def test_sharded_ppm_matches_single(world, W, H, photon_map, scaling):
    """photon_map 2: each rank builds a kd-tree over its own photons and gathers every rank's
    hit points against it (the gather is linear in the photon set, like the grid's).
    strong: a fixed 48 x 41 global photon launch (the bench's default multi-GPU mode) whose
    rows are dealt to the ranks (41 rows: uneven shares); weak: a full 32 x 32 batch per rank.
    41 x 37 over 3 ranks: 13 x 41 = 533 pixels per segment, an odd count (the export planes are
    padded to a multiple of 4 pixels, so every segment stays 16-B aligned)."""
    P, iters = (32, 2) if scaling == "weak" else (48, 2)
    PH = P * world if scaling == "weak" else 41
    out = os.path.join(tempfile.mkdtemp(), "img.npy")
    mp.spawn(worker, args=(world, free_port(), out, W, H, P, iters, _abi.PROGRESSIVE_PHOTON_MAPPING, photon_map, PH),
             nprocs=world, join=True)
    got = np.load(out)
    scene = scenes.cornell()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=PH, photon_map=photon_map)
    r = oracle_lib.OracleRenderer(cfg)
    r.init_scene(scene)
    req = request(scene, W, H)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        r.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    ref = r.output()
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert err < 1e-5, err
    assert got.mean() > 0


@pytest.mark.parametrize("world,W,H,PH", [(2, 48, 40, 41), (3, 40, 37, 48), (4, 40, 37, 41)])
def test_sharded_ppm_slab_partition_matches_single(world, W, H, PH):
    """Slab mode (include/orx.h orx_set_slab_partition): every rank traces its launch rows, the
    photons are redistributed by a spatial slab of one scene axis (histograms all-gathered, the
    plan of multigpu.slab_plan, photon records all-to-all), each rank grids its slab's photons
    and gathers every hit point against them; the sum is the single renderer's image."""
    P, iters = 48, 2
    out = os.path.join(tempfile.mkdtemp(), "img.npy")
    mp.spawn(worker, args=(world, free_port(), out, W, H, P, iters, _abi.PROGRESSIVE_PHOTON_MAPPING, 0, PH, True),
             nprocs=world, join=True)
    got = np.load(out)
    scene = scenes.cornell()
    r = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=PH))
    r.init_scene(scene)
    req = request(scene, W, H)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        r.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    ref = r.output()
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert err < 1e-5, err
    assert got.mean() > 0


def test_slab_plan_properties():
    """slab_plan: contiguous ascending slabs, identical on every rank, counts = the photon bins
    each rank sends, and the chosen axis balances the cost better than the others."""
    rng = np.random.default_rng(7)
    world, nb = 4, 64
    hists = rng.integers(0, 50, size=(world, 2, 3, nb)).astype(np.uint32)
    hists[:, :, 1, :] = 0
    hists[:, :, 1, 10] = 1000  # axis 1: everything in one bin, a poor axis to split
    axis, dest, counts = multigpu.slab_plan(hists, world)
    assert axis != 1
    assert np.all(np.diff(dest.astype(int)) >= 0) and dest.max() < world
    for src in range(world):
        for d in range(world):
            assert counts[src, d] == hists[src, 0, axis][dest == d].sum()
    a2, d2, c2 = multigpu.slab_plan(hists.copy(), world)
    assert a2 == axis and np.array_equal(d2, dest) and np.array_equal(c2, counts)
    empty = np.zeros((2, 2, 3, 8), np.uint32)
    a0, d0, c0 = multigpu.slab_plan(empty, 2)
    assert c0.sum() == 0 and d0.max() < 2


def test_slab_plan_voxel_weights():
    """With voxel counts the gather term weighs a hit point by the photons of its voxel: hit points
    spread evenly along x, photons all in the voxel layer of the first x-quarter -> the first rank
    gets a thin slab of that layer, and the split follows the voxel cost, not the hit-point count."""
    V, nb, world = multigpu.SLAB_VOXELS, 256, 4
    hists = np.zeros((world, 2, 3, nb), np.uint32)
    vox = np.zeros((world, 2, V, V, V), np.uint32)  # [z][y][x]
    hists[:, 1, 0, :] = 10                           # hit points: uniform in x
    hists[:, 1, 1, nb // 2] = 10 * nb                # ... all in one y and one z bin
    hists[:, 1, 2, nb // 2] = 10 * nb
    vox[:, 1, V // 2, V // 2, :] = 10 * (nb // V)
    hists[:, 0, 0, 0:nb // V] = 100                  # photons in the first x voxel layer
    hists[:, 0, 1, nb // 2] = 100 * (nb // V)
    hists[:, 0, 2, nb // 2] = 100 * (nb // V)
    vox[:, 0, V // 2, V // 2, 0] = 100 * (nb // V)
    axis, dest, counts = multigpu.slab_plan(hists, world, vox.reshape(world, 2, -1))
    assert axis == 0
    assert np.all(np.diff(dest.astype(int)) >= 0)
    # the first layer's bins (the whole gather cost) are split over the ranks, not one rank's
    assert len(set(dest[:nb // V].tolist())) >= 3
    w = multigpu.slab_hist_words(nb)
    words = np.arange(world * w, dtype=np.uint32).reshape(world, w)
    h2, v2, box = multigpu.split_slab_hists(words.view(np.int32), world, nb)
    assert h2.shape == (world, 2, 3, nb) and v2.shape == (world, 2, V ** 3)
    assert box[0] == words[:, 6 * nb].min() and box[5] == words[:, 6 * nb + 5].max()


@pytest.mark.parametrize("world,W,H", [(2, 40, 32), (3, 36, 29)])
def test_sharded_vcm_matches_single(world, W, H):
    """VCM row sharding: own-row light + camera subpaths, splats reduce-scattered."""
    iters = 2
    out = os.path.join(tempfile.mkdtemp(), "img.npy")
    vcm = _abi.VCM_BIDIRECTIONAL_PATH_TRACING
    mp.spawn(worker, args=(world, free_port(), out, W, H, 32, iters, vcm), nprocs=world, join=True)
    got = np.load(out)
    scene = scenes.cornell()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32 * world)
    r = oracle_lib.OracleRenderer(cfg)
    r.init_scene(scene)
    req = request(scene, W, H, vcm)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        r.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    ref = r.output()
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert err < 1e-5, err
    assert got.mean() > 0


@pytest.mark.parametrize("world,W,H", [(2, 40, 32), (3, 36, 29)])
def test_sharded_pt_matches_single_bitexact(world, W, H):
    """PT row sharding: no exchange; every pixel's path is the single-renderer one."""
    out = os.path.join(tempfile.mkdtemp(), "img.npy")
    pt = _abi.PATH_TRACING
    mp.spawn(worker, args=(world, free_port(), out, W, H, 32, 2, pt), nprocs=world, join=True)
    got = np.load(out)
    scene = scenes.cornell()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32 * world)
    r = oracle_lib.OracleRenderer(cfg)
    r.init_scene(scene)
    req = request(scene, W, H, pt)
    for it in range(2):
        r.render_next_iteration(it, it, 1.0, req)
    assert np.array_equal(got.view(np.uint32), r.output().view(np.uint32))
    assert got.mean() > 0


def test_assemble_rows_roundtrip():
    W, H, world = 5, 11, 4
    img = np.arange(H * W * 3, dtype=np.float32).reshape(H, W, 3)
    mr = (H + world - 1) // world
    blocks = []
    for g in range(world):
        b = np.zeros((mr, W, 3), np.float32)
        rows = img[g::world]
        b[:len(rows)] = rows
        blocks.append(b)
    assert np.array_equal(multigpu.assemble_rows(blocks, W, H, world), img)


def batch_worker(rank, world, port, out_path, W, H, P, iters, method, reduce_every):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import shard_backends

    scene = scenes.cornell()
    cfg = _abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P)
    b = shard_backends.oracle_batch(cfg, rank, world, rank, scene)
    sh = multigpu.BatchSharded(b, dist, world, rank, W, H, reduce_every=reduce_every)
    req = request(scene, W, H, method)
    radii = multigpu.radius_sequence(scene.initial_ppm_radius(), iters * world)
    for i in range(iters):
        it = multigpu.batch_iteration(i, rank, world)
        sh.iteration(it, i, radii[it], req)
    img = sh.image()
    if rank == 0:
        np.save(out_path, img)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,method,reduce_every", [(2, _abi.PROGRESSIVE_PHOTON_MAPPING, 1),
                                                       (3, _abi.PROGRESSIVE_PHOTON_MAPPING, 2),
                                                       (4, _abi.PROGRESSIVE_PHOTON_MAPPING, 8),
                                                       (2, _abi.VCM_BIDIRECTIONAL_PATH_TRACING, 0),
                                                       (2, _abi.PATH_TRACING, 1)])
def test_batch_partition_is_the_sum_of_independent_renderers(world, method, reduce_every):
    """Photon-batch partition (the bench's default multi-GPU mode, the reference's client/server
    iteration dealing): the reduced radiance equals the sum of `world` independent renderers, rank
    g seeded batch_seed(SEED, g) rendering global iterations g, g + N, ... with the global radius
    sequence; rank 0 alone is the single-device run's seed."""
    W, H, P, iters = 40, 32, 24, 3
    out = os.path.join(tempfile.mkdtemp(), "img.npy")
    mp.spawn(batch_worker, args=(world, free_port(), out, W, H, P, iters, method, reduce_every), nprocs=world,
             join=True)
    got = np.load(out)
    scene = scenes.cornell()
    radii = multigpu.radius_sequence(scene.initial_ppm_radius(), iters * world)
    ref = np.zeros((H, W, 3), np.float64)
    for g in range(world):
        cfg = _abi.default_config(seed=multigpu.batch_seed(SEED, g), photon_launch_width=P, photon_launch_height=P)
        r = oracle_lib.OracleRenderer(cfg)
        r.init_scene(scene)
        req = request(scene, W, H, method)
        for i in range(iters):
            it = multigpu.batch_iteration(i, g, world)
            r.render_next_iteration(it, i, radii[it], req)
        ref += r.output().astype(np.float64)
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref ** 2).sum())
    assert err < 1e-6, err
    assert got.mean() > 0


def test_batch_seeds_and_iterations():
    assert multigpu.batch_seed(SEED, 0) == SEED
    seeds = {multigpu.batch_seed(SEED, g) for g in range(64)}
    assert len(seeds) == 64 and 0 not in seeds
    # seed 0 (the reference's clock seed): rank 0 keeps it; the other ranks get a clock-derived seed
    # with the rank mixed in, so ranks started in the same second still draw different streams
    assert multigpu.batch_seed(0, 0) == 0
    clock = {multigpu.batch_seed(0, g) for g in range(1, 64)}
    assert len(clock) == 63 and 0 not in clock
    assert sorted(multigpu.batch_iteration(i, g, 4) for i in range(3) for g in range(4)) == list(range(12))
    r = multigpu.radius_sequence(1.0, 5)
    x = 1.0
    for k in range(4):
        x = next_ppm_radius(x, k)
        assert r[k + 1] == x
