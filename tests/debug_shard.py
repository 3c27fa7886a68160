"""Debug helper: device shard vs oracle shard, buffer by buffer (not collected by pytest)."""
import sys
import numpy as np
import torch
import oracle_lib
from oppositerenderer_amd import _abi, multigpu, scenes
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails

SEED = 1645301512
world, W, H, P = 2, 64, 48, 64
dev = torch.device("cuda", 0)
scene = scenes.cornell()
cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
req = det.to_abi()
mr = (H + world - 1) // world
dsh, osh = [], []
for rank in range(world):
    r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P * world))
    r.initialize(0); r.set_shard(rank, world); r.initScene(scene)
    dsh.append(multigpu.DeviceShard(r, torch, dev))
    o = oracle_lib.OracleRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P * world))
    o.init_scene(scene)
    ob = oracle_lib.OracleShard(o, torch); ob.set_shard(rank, world)
    osh.append(ob)
radius = scene.initial_ppm_radius()
for k in range(world):
    dsh[k].local_passes(0, 0, radius, req)
    osh[k].local_passes(0, 0, radius, req)
torch.cuda.synchronize()
for k in range(world):
    for buf, name in ((_abi.BUF_RNG, "rng"), (_abi.BUF_HITPOINTS, "hp"), (_abi.BUF_GRID_OFFSETS, "off")):
        g = dsh[k].r.read_buffer(buf, np.uint32); o = osh[k].r.read_buffer(buf, np.uint32)
        print(k, name, g.shape, o.shape, "mismatch", np.count_nonzero(g[:min(len(g),len(o))] != o[:min(len(g),len(o))]))
    gs, os_ = dsh[k].r.stats(), osh[k].r.stats()
    print(k, "valid", gs.valid_photons, os_.valid_photons, list(gs.grid_size), list(os_.grid_size))
hd, ho = [], []
for k in range(world):
    t = dsh[k].alloc(mr * W * 10); dsh[k].export_hitpoints(t); hd.append(t)
    t2 = osh[k].alloc(mr * W * 10); osh[k].export_hitpoints(t2); ho.append(t2)
torch.cuda.synchronize()
for k in range(world):
    a = hd[k].cpu().numpy().view(np.uint32); b = ho[k].numpy().view(np.uint32)
    print(k, "export mismatch", np.count_nonzero(a != b), "of", a.size)
hpd = torch.cat(hd); hpo = torch.cat(ho)
for k in range(world):
    pd = dsh[k].alloc(world * mr * W * 3); dsh[k].gather_external(hpd, world, pd)
    po = osh[k].alloc(world * mr * W * 3); osh[k].gather_external(hpo, world, po)
    torch.cuda.synchronize()
    a = pd.cpu().numpy(); b = po.numpy()
    print(k, "partial rel", np.abs(a - b).sum() / max(1e-30, np.abs(b).sum()), a.sum(), b.sum())
