"""Device-side sharded PPM (orx_ppm_local_passes / _export_hitpoints /
_gather_external / _finish): two row-interleaved shards on one MI355X with the
collectives done by plain torch ops must equal one renderer tracing the union
photon launch (up to fp32 summation order in the gather)."""
import numpy as np
import pytest
import torch

from oppositerenderer_amd import _abi, multigpu, scenes
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius

pytestmark = pytest.mark.gpu
SEED = 1645301512


@pytest.mark.parametrize("world,W,H,P,photon_map", [(2, 64, 48, 64, 0), (3, 50, 41, 48, 0), (2, 64, 48, 64, 2)])
def test_sharded_device_path_matches_single(world, W, H, P, photon_map):
    dev = torch.device("cuda", 0)
    scene = scenes.cornell()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = det.to_abi()
    shards = []
    for rank in range(world):
        r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P * world,
                                              photon_map=photon_map))
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        shards.append(multigpu.DeviceShard(r, torch, dev))
    mr = (H + world - 1) // world
    radius = scene.initial_ppm_radius()
    for it in range(3):
        for b in shards:
            b.local_passes(it, it, radius, req)
        hps = []
        for b in shards:
            t = b.alloc(multigpu.hp_export_floats(mr, W))
            b.export_hitpoints(t)
            hps.append(t)
        hp_all = torch.cat(hps)
        total = None
        for b in shards:
            part = b.alloc(world * mr * W * 3)
            b.gather_external(hp_all, world, part)
            total = part if total is None else total + part
        blk = mr * W * 3
        for k, b in enumerate(shards):
            b.finish(total[k * blk:(k + 1) * blk].contiguous())
        radius = next_ppm_radius(radius, it)
    torch.cuda.synchronize()
    blocks = [b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards]
    got = multigpu.assemble_rows(blocks, W, H, world)
    single = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P * world,
                                               photon_map=photon_map))
    single.initialize(0)
    single.initScene(scene)
    radius = scene.initial_ppm_radius()
    for it in range(3):
        single.renderNextIteration(it, it, radius, True, det)
        radius = next_ppm_radius(radius, it)
    ref = single.getOutputBuffer()
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert err < 1e-5, err
    for b in shards:
        b.r.destroy()
    single.destroy()


@pytest.mark.parametrize("world,W,H", [(2, 64, 48), (3, 50, 41)])
def test_sharded_device_vcm_matches_single(world, W, H):
    """Device-side sharded VCM (orx_vcm_local_light / _export_vcm_splats /
    _vcm_finish): own-row subpaths, splat buffers summed by torch ops (the
    reduce-scatter), must equal the single-device VCM iteration."""
    dev = torch.device("cuda", 0)
    scene = scenes.cornell()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.VCM_BIDIRECTIONAL_PATH_TRACING, W, H)
    req = det.to_abi()
    cfg = lambda: _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32)
    shards = []
    for rank in range(world):
        r = OptixRenderer(cfg())
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        shards.append(multigpu.DeviceShard(r, torch, dev))
    mr = (H + world - 1) // world
    blk = mr * W * 3
    radius = scene.initial_ppm_radius()
    for it in range(3):
        total = None
        for b in shards:
            b.vcm_local_light(it, it, radius, req)
            t = b.alloc(world * blk)
            b.export_vcm_splats(t)
            total = t if total is None else total + t
        for k, b in enumerate(shards):
            b.vcm_finish(total[k * blk:(k + 1) * blk].contiguous())
        radius = next_ppm_radius(radius, it)
    torch.cuda.synchronize()
    blocks = [b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards]
    got = multigpu.assemble_rows(blocks, W, H, world)
    single = OptixRenderer(cfg())
    single.initialize(0)
    single.initScene(scene)
    radius = scene.initial_ppm_radius()
    for it in range(3):
        single.renderNextIteration(it, it, radius, True, det)
        radius = next_ppm_radius(radius, it)
    ref = single.getOutputBuffer()
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert err < 1e-5, err
    assert got.mean() > 0
    for b in shards:
        b.r.destroy()
    single.destroy()


@pytest.mark.parametrize("world,W,H", [(2, 64, 48), (3, 50, 41)])
def test_sharded_device_pt_matches_single(world, W, H):
    """Device-side PT row shards (no exchange): bit-identical to one device."""
    dev = torch.device("cuda", 0)
    scene = scenes.scene_by_name("CornellSmallSmallSpheres")
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PATH_TRACING, W, H)
    req = det.to_abi()
    cfg = lambda: _abi.default_config(seed=SEED, photon_launch_width=32, photon_launch_height=32)
    shards = []
    for rank in range(world):
        r = OptixRenderer(cfg())
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        shards.append(multigpu.DeviceShard(r, torch, dev))
    for it in range(3):
        for b in shards:
            b.render_next(it, it, 1.0, req)
    torch.cuda.synchronize()
    mr = (H + world - 1) // world
    got = multigpu.assemble_rows([b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards], W, H, world)
    single = OptixRenderer(cfg())
    single.initialize(0)
    single.initScene(scene)
    for it in range(3):
        single.renderNextIteration(it, it, 1.0, True, det)
    ref = single.getOutputBuffer()
    assert np.array_equal(got.reshape(-1).view(np.uint32), ref.reshape(-1).view(np.uint32))
    for b in shards:
        b.r.destroy()
    single.destroy()


@pytest.mark.parametrize("world,W,H,P", [(2, 64, 48, 64), (3, 50, 41, 48)])
def test_sharded_device_pipelined_matches_single(world, W, H, P):
    """orx_set_ppm_pipeline: gather + finish of iteration i on a side stream while iteration i+1's
    eye/photon/grid passes run, issued back to back with no host synchronisation; the image equals
    the single-GPU one (fp32 summation order)."""
    dev = torch.device("cuda", 0)
    scene = scenes.cornell()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = det.to_abi()
    side = torch.cuda.Stream(dev)
    shards = []
    for rank in range(world):
        r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P * world))
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        b = multigpu.DeviceShard(r, torch, dev)
        b.enable_pipeline(side)
        shards.append(b)
    main = torch.cuda.current_stream(dev)
    mr = (H + world - 1) // world
    sets = [([b.alloc(multigpu.hp_export_floats(mr, W)) for b in shards], shards[0].alloc(world * multigpu.hp_export_floats(mr, W)),
             [b.alloc(world * mr * W * 3) for b in shards], shards[0].alloc(world * mr * W * 3)) for _ in range(2)]
    radius = scene.initial_ppm_radius()
    iters = 5
    for it in range(iters):
        hp_loc, hp_all, parts, total = sets[it % 2]
        for b, t in zip(shards, hp_loc):
            b.local_eye(it, it, radius, req)
            b.export_hitpoints(t)
        hp_all.copy_(torch.cat(hp_loc))  # the all-gather, on the compute stream
        hp_ready = torch.cuda.Event()  # its completion is all the side stream waits for (work.wait())
        hp_ready.record(main)
        for b in shards:
            b.local_photons()
        with torch.cuda.stream(side):
            side.wait_event(hp_ready)
            for b, part in zip(shards, parts):
                b.gather_external(hp_all, world, part)
            total.copy_(torch.stack(parts).sum(0))  # the reduce-scatter, on the side stream
            blk = mr * W * 3
            for k, b in enumerate(shards):
                b.finish(total[k * blk:(k + 1) * blk].contiguous())
        radius = next_ppm_radius(radius, it)
    torch.cuda.synchronize()
    blocks = [b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards]
    got = multigpu.assemble_rows(blocks, W, H, world)
    single = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P * world))
    single.initialize(0)
    single.initScene(scene)
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        single.renderNextIteration(it, it, radius, True, det)
        radius = next_ppm_radius(radius, it)
    ref = single.getOutputBuffer()
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert err < 1e-5, err
    assert all(b.r.pipelined() for b in shards)
    for b in shards:
        b.r.destroy()
    single.destroy()


@pytest.mark.slow
def test_full_size_conference_sharded_equals_single():
    """configs[4] at full size on one GPU, in the bench's default multi-GPU mode (strong scaling:
    the 4096^2 = 16,777,216 photons/iter and 3840x2160 pixels are fixed and split over the
    shards): two row-interleaved shards (each half of the photon launch rows, RNG rows and pixel
    rows, exchanging hit points and partial indirect through torch ops) reproduce the
    single-renderer image — the size-independent property behind the 8-GPU pixel/photon
    sharding (the oracle would need minutes at this size)."""
    dev = torch.device("cuda", 0)
    scene = scenes.scene_by_name("SyntheticConference")
    W, H, P, world = 3840, 2160, 4096, 2
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = det.to_abi()
    radius = scene.initial_ppm_radius()
    single = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
    single.initialize(0)
    single.initScene(scene)
    single.renderNextIteration(0, 0, radius, True, det)
    ref = single.getOutputBuffer()
    st = single.stats()
    assert st.valid_photons > P * P // 2
    single.destroy()
    torch.cuda.empty_cache()
    shards = []
    for rank in range(world):
        r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        shards.append(multigpu.DeviceShard(r, torch, dev))
    mr = (H + world - 1) // world
    for b in shards:
        b.local_passes(0, 0, radius, req)
    hps = []
    for b in shards:
        t = b.alloc(multigpu.hp_export_floats(mr, W))
        b.export_hitpoints(t)
        hps.append(t)
    hp_all = torch.cat(hps)
    total = None
    for b in shards:
        part = b.alloc(world * mr * W * 3)
        b.gather_external(hp_all, world, part)
        total = part if total is None else total + part
    blk = mr * W * 3
    for k, b in enumerate(shards):
        b.finish(total[k * blk:(k + 1) * blk].contiguous())
    torch.cuda.synchronize()
    blocks = [b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards]
    got = multigpu.assemble_rows(blocks, W, H, world)
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert np.isfinite(got).all() and ref.mean() > 0
    assert err < 1e-5, err
    for b in shards:
        b.r.destroy()


def _oracle_ppm(scene, W, H, P, PH, iters, photon_map=0):
    import oracle_lib

    ora = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=PH,
                                                        photon_map=photon_map))
    ora.init_scene(scene)
    req = RenderRequestDetails(scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H))),
                               scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H).to_abi()
    radius = scene.initial_ppm_radius()
    for it in range(iters):
        ora.render_next_iteration(it, it, radius, req)
        radius = next_ppm_radius(radius, it)
    out = ora.output().copy()
    ora.close()
    return out


@pytest.mark.parametrize("world,W,H,P,PH,photon_map,pipelined",
                         [(4, 96, 80, 128, 128, 0, False), (8, 96, 80, 128, 128, 0, False),
                          (8, 100, 75, 96, 101, 0, False), (4, 96, 80, 128, 128, 0, True),
                          (8, 96, 80, 128, 128, 0, True), (4, 96, 80, 128, 128, 2, False),
                          (8, 96, 80, 128, 128, 2, True)])
def test_sharded_world4_world8_match_oracle(world, W, H, P, PH, photon_map, pipelined):
    """The 4- and 8-GPU partitions of the multi-GPU bench (strong scaling: a fixed P x PH global
    photon launch and W x H pixels dealt to the ranks by rows; PH = 101 gives uneven shares),
    on one device with the collectives done by torch ops, against the ORACLE's single renderer
    (OptixRenderer.cpp:569-673; the gather is linear in the photon set, so the union of the
    shards is the reference frame up to fp32 summation order).  Covers what world >= 4 selects:
    cell-order photon layout, the per-lane gather at eight segments, the kd-tree shard, and the
    pipelined side-stream schedule (orx_set_ppm_pipeline)."""
    dev = torch.device("cuda", 0)
    scene = scenes.cornell()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = det.to_abi()
    side = torch.cuda.Stream(dev) if pipelined else None
    shards = []
    for rank in range(world):
        r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=PH,
                                              photon_map=photon_map))
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        b = multigpu.DeviceShard(r, torch, dev)
        if pipelined:
            b.enable_pipeline(side)
        shards.append(b)
    main = torch.cuda.current_stream(dev)
    mr = (H + world - 1) // world
    blk = mr * W * 3
    nsets = 2 if pipelined else 1
    sets = [([b.alloc(multigpu.hp_export_floats(mr, W)) for b in shards], shards[0].alloc(world * multigpu.hp_export_floats(mr, W)),
             [b.alloc(world * blk) for b in shards], shards[0].alloc(world * blk)) for _ in range(nsets)]
    radius = scene.initial_ppm_radius()
    iters = 3
    for it in range(iters):
        hp_loc, hp_all, parts, total = sets[it % nsets]
        if pipelined:
            for b, t in zip(shards, hp_loc):
                b.local_eye(it, it, radius, req)
                b.export_hitpoints(t)
            hp_all.copy_(torch.cat(hp_loc))
            hp_ready = torch.cuda.Event()  # the all-gather's completion only, as work.wait()
            hp_ready.record(main)
            for b in shards:
                b.local_photons()
            with torch.cuda.stream(side):
                side.wait_event(hp_ready)
                for b, part in zip(shards, parts):
                    b.gather_external(hp_all, world, part)
                total.copy_(torch.stack(parts).sum(0))
                for k, b in enumerate(shards):
                    b.finish(total[k * blk:(k + 1) * blk].contiguous())
        else:
            for b, t in zip(shards, hp_loc):
                b.local_passes(it, it, radius, req)
                b.export_hitpoints(t)
            hp_all.copy_(torch.cat(hp_loc))
            for b, part in zip(shards, parts):
                b.gather_external(hp_all, world, part)
            total.copy_(torch.stack(parts).sum(0))
            for k, b in enumerate(shards):
                b.finish(total[k * blk:(k + 1) * blk].contiguous())
        radius = next_ppm_radius(radius, it)
    torch.cuda.synchronize()
    got = multigpu.assemble_rows([b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards],
                                 W, H, world)
    ref = _oracle_ppm(scene, W, H, P, PH, iters, photon_map)
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert ref.mean() > 0 and np.isfinite(got).all()
    assert err < 1e-5, err
    if pipelined:
        assert all(b.r.pipelined() for b in shards)
    for b in shards:
        b.r.destroy()


@pytest.mark.parametrize("world,W,H,P,PH,pipelined", [(2, 96, 80, 128, 128, False), (4, 96, 80, 128, 128, False),
                                                       (8, 100, 75, 96, 101, False), (4, 96, 80, 128, 128, True),
                                                       (8, 96, 80, 128, 128, True)])
def test_sharded_slab_partition_matches_oracle(world, W, H, P, PH, pipelined):
    """Slab mode on the device (include/orx.h orx_set_slab_partition: k_slab_hist, k_slab_pack,
    k_slab_import, the culled gather), N shards on one GPU with the all-gathers and the photon
    all-to-all done by torch ops, against the ORACLE's single renderer (the gather is linear in the
    photon set; every photon lands in exactly one rank's grid): rel-L2 <= 1e-5."""
    import shard_emul

    dev = torch.device("cuda", 0)
    scene = scenes.cornell()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    req = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H).to_abi()
    side = torch.cuda.Stream(dev) if pipelined else None
    shards = shard_emul.make_shards(scene, world, P, PH, slab=True, pipelined=pipelined, side=side)
    got, plans = shard_emul.run_iterations(shards, scene, W, H, req, 3, slab=True, pipelined=pipelined, side=side)
    ref = _oracle_ppm(scene, W, H, P, PH, 3)
    err = np.sqrt(((got.astype(np.float64) - ref) ** 2).sum() / (ref.astype(np.float64) ** 2).sum())
    assert ref.mean() > 0 and np.isfinite(got).all()
    assert err < 1e-5, err
    axis, counts = plans[-1]
    assert counts.sum() > 0 and (counts.sum(0) > 0).sum() >= 2  # photons really moved between slabs
    for b in shards:
        b.r.destroy()
