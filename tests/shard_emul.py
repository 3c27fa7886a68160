"""World-N sharded PPM on ONE device (TEST INFRASTRUCTURE): N row-interleaved DeviceShards whose
collectives are done by plain torch ops, in the bench's orchestration (multigpu.ShardedPPM):
  rows  the hit-point all-gather, every shard gathers all hit points, reduce-scatter (sum);
  slab  additionally the histogram all-gather, multigpu.slab_plan, per-shard pack, the photon
        all-to-all (each destination's records concatenated in source-rank order) and import.
Two RCCL ranks cannot share one GPU, so this is how the N > 1 device code runs on a 1-GPU box."""
import numpy as np
import torch

from oppositerenderer_amd import _abi, multigpu
from oppositerenderer_amd.renderer import OptixRenderer, next_ppm_radius

SEED = 1645301512


def make_shards(scene, world, P, PH, slab=False, pipelined=False, photon_map=0, side=None, dev=None):
    dev = dev or torch.device("cuda", 0)
    shards = []
    for rank in range(world):
        r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=PH,
                                              photon_map=photon_map))
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        b = multigpu.DeviceShard(r, torch, dev, (rank, world))
        if pipelined:
            b.enable_pipeline(side)
        if slab:
            b.enable_slab()
        shards.append(b)
    return shards


def slab_exchange(shards, world, radius, nb=multigpu.SLAB_BINS):
    hists = []
    for b in shards:
        h = b.alloc_i32(multigpu.slab_hist_words(nb))
        b.slab_histogram(h, nb)
        hists.append(h)
    H, vox, box = multigpu.split_slab_hists(torch.stack(hists).cpu().numpy(), world, nb)
    halo = [shards[0].slab_halo(nb, a, radius) for a in range(3)]
    axis, bin_dest, counts = multigpu.slab_plan(H, world, vox, halo)
    sends = []
    for rank, b in enumerate(shards):
        n = counts[rank]
        base = np.concatenate([[0], np.cumsum(n)[:-1]]).astype(np.uint32)
        send = b.alloc(9 * int(n.sum()) + 9)
        b.slab_pack(bin_dest, nb, axis, halo[axis], base, int(n.sum()), send)
        sends.append((send, base, n))
    for d, b in enumerate(shards):
        parts = [s[9 * int(base[d]):9 * int(base[d] + n[d])] for s, base, n in sends]
        recv = torch.cat(parts) if parts else b.alloc(0)
        nr = int(counts[:, d].sum())
        b.slab_import(recv.contiguous(), nr, box, axis, nb, multigpu.slab_owned(bin_dest, d))
    return axis, counts


def run_iterations(shards, scene, W, H, req, iters, slab=False, pipelined=False, side=None):
    world = len(shards)
    mr = (H + world - 1) // world
    blk = mr * W * 3
    nsets = 2 if pipelined else 1
    sets = [([b.alloc(multigpu.hp_export_floats(mr, W)) for b in shards], shards[0].alloc(world * multigpu.hp_export_floats(mr, W)),
             [b.alloc(world * blk) for b in shards], shards[0].alloc(world * blk)) for _ in range(nsets)]
    main = torch.cuda.current_stream()
    radius = scene.initial_ppm_radius()
    plans = []
    for it in range(iters):
        hp_loc, hp_all, parts, total = sets[it % nsets]
        for b, t in zip(shards, hp_loc):
            if pipelined:
                b.local_eye(it, it, radius, req)
            elif slab:
                b.local_trace(it, it, radius, req)
            else:
                b.local_passes(it, it, radius, req)
            b.export_hitpoints(t)
        hp_all.copy_(torch.cat(hp_loc))
        # the all-gather's completion: the side stream waits for this and nothing else, as
        # ShardedPPM's work.wait() does, so the gather relies on the library's own events for the
        # grid, the slab import and the direct pass (orx_capi.hip ev_grid_done / ev_direct_done)
        hp_ready = torch.cuda.Event()
        hp_ready.record(main)
        if pipelined:
            for b in shards:
                if slab:
                    b.local_photon_trace()
                else:
                    b.local_photons()
        if slab:
            plans.append(slab_exchange(shards, world, radius))
        ctx = torch.cuda.stream(side) if pipelined else torch.cuda.stream(main)
        with ctx:
            if pipelined:
                side.wait_event(hp_ready)
            for b, part in zip(shards, parts):
                b.gather_external(hp_all, world, part)
            total.copy_(torch.stack(parts).sum(0))
            for k, b in enumerate(shards):
                b.finish(total[k * blk:(k + 1) * blk].contiguous())
        radius = next_ppm_radius(radius, it)
    torch.cuda.synchronize()
    blocks = [b.output_local_tensor(mr).cpu().numpy().reshape(mr, W, 3) for b in shards]
    return multigpu.assemble_rows(blocks, W, H, world), plans
