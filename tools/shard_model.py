#!/usr/bin/env python3
"""Per-rank cost of the strong-scaling sharded PPM at world size N, measured on one GPU.

A renderer is set up as rank 0 of N (own pixel rows y = 0 mod N, own photon-launch rows
of the fixed global launch), and its phases are run and timed one after the other with
torch events: local passes (eye, photon, grid, direct), hit-point export, the gather of ALL
W*H hit points against the local photons, and the finish (direct + output of the own rows).
The full-image hit points come from a second, unsharded renderer's eye pass on the
same camera and radius, rearranged into the ranks' row-interleaved segments (what the
all-gather delivers).  The collectives are not run; their volumes are printed so the exchange
over xGMI can be added by hand.  Usage: shard_model.py [--config 2|4] [N ...]  (default 1 2 4 8):
configs[2] hall 1080p with a 2048^2 photon launch (default), configs[4] conference 3840x2160
with 4096^2."""
import os
import sys
import time

# the pipelined schedule runs five streams at once (compute, the renderer's aux stream, the gather side
# stream, and in the bench RCCL's): with HIP's default of 4 hardware queues the gather shared the compute
# stream's queue and the per-rank frame serialised (configs[4] N=8: 8.05 against 6.56 ms with 8 queues)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:  # before torch loads HIP (the boxes export 4)
    os.environ["GPU_MAX_HW_QUEUES"] = "8"


import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oppositerenderer_amd import _abi, multigpu, synthetic  # noqa: E402
from oppositerenderer_amd.renderer import OptixRenderer, RenderRequestDetails, next_ppm_radius  # noqa: E402

SEED = 1645301512
XGMI_LINK_GBS = 153.0  # one xGMI link per direction (MI355X: 7 links per GPU)


def collectives_ms(ag_mb, rs_mb, world):
    """The exchange per iteration and rank over xGMI, two bounds: every rank receives (N-1)/N of
    the all-gather and of the reduce-scatter.  'one link': a single ring (each step one link,
    153 GB/s); 'all links': the N-1 peer links of a fully connected node used at once."""
    if world == 1:
        return 0.0, 0.0
    recv_mb = (ag_mb + rs_mb) * (world - 1) / world
    one = recv_mb * 1e6 / (XGMI_LINK_GBS * 1e9) * 1e3
    return one, one / (world - 1)


def run(world, W=1920, H=1080, P=2048, iters=6, warm=2, scene=None):
    dev = torch.device("cuda", 0)
    scene = scene or synthetic.synthetic_hall()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    req = det.to_abi()
    gv = int(os.environ.get("MODEL_GATHER_VARIANT", "0"))  # 1: whole cell rows (no sub-rows)
    # MODEL_GMAX_DIV=1: the rank's grid gets PHOTON_GRID_MAX_SIZE / N cells (1/N of the photons)
    gmax = 1000000 // world if os.environ.get("MODEL_GMAX_DIV", "0") != "0" else 1000000
    r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P, gather_variant=gv,
                                          photon_grid_max_size=gmax))
    r.initialize(0)
    r.set_shard(0, world)
    r.initScene(scene)
    b = multigpu.DeviceShard(r, torch, dev)
    full = OptixRenderer(_abi.default_config(seed=SEED + 1, photon_launch_width=16, photon_launch_height=16))
    full.initialize(0)
    full.initScene(scene)
    fb = multigpu.DeviceShard(full, torch, dev)
    fhp = fb.alloc(multigpu.hp_export_floats(H, W))
    mr = (H + world - 1) // world
    hp = b.alloc(multigpu.hp_export_floats(mr, W))

    def segments(t):
        """[H][W] planes A (4), N (3) -> N segments of mr rows, rows y = s + lj*N (planes padded to
        a multiple of 4 pixels, multigpu.hp_export_floats)"""
        P1 = multigpu.hp_export_floats(H, W) // 7
        A = t[:H * W * 4].view(H, W, 4)
        Nn = t[P1 * 4:P1 * 4 + H * W * 3].view(H, W, 3)
        Pm = multigpu.hp_export_floats(mr, W) // 7
        out = []
        for s_ in range(world):
            for P_, k in ((A, 4), (Nn, 3)):
                blk = torch.zeros(Pm * k, device=dev)
                rows = P_[s_::world]
                blk[:rows.shape[0] * W * k] = rows.reshape(-1)
                out.append(blk)
        return torch.cat(out)

    part = b.alloc(world * mr * W * 3)
    radius = scene.initial_ppm_radius()
    names = ("local", "export", "gather", "finish")
    tot = dict.fromkeys(names, 0.0)
    for it in range(iters):
        if it == warm:
            r.reset_timing()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        b.local_passes(it, it, radius, req)
        ev[1].record()
        b.export_hitpoints(hp)
        ev[2].record()
        fb.local_passes(it, it, radius, req)
        hp_all = segments(fhp) if fb.export_hitpoints(fhp) is None else None
        ev[3].record()
        b.gather_external(hp_all, world, part)
        ev[4].record()
        b.finish(part[:mr * W * 3].contiguous())
        ev[5].record()
        torch.cuda.synchronize()
        if it >= warm:
            tot["local"] += ev[0].elapsed_time(ev[1])
            tot["export"] += ev[1].elapsed_time(ev[2])
            tot["gather"] += ev[3].elapsed_time(ev[4])
            tot["finish"] += ev[4].elapsed_time(ev[5])
        radius = next_ppm_radius(radius, it)
    n = iters - warm
    ms = {k: round(v / n, 3) for k, v in tot.items()}
    st = r.stats()
    ni = max(1, st.timed_iterations)
    passes = {name: round(st.pass_ms[i] / ni, 3) for i, name in enumerate(_abi.PASS_NAMES) if st.pass_ms[i] > 0}
    allgather_mb = world * 4 * multigpu.hp_export_floats(mr, W) / 1e6
    rs_mb = world * mr * W * 12 / 1e6
    r.destroy()
    full.destroy()
    return ms, passes, allgather_mb, rs_mb


def run_slab(world, W=1920, H=1080, P=2048, iters=6, warm=2, scene=None, nb=multigpu.SLAB_BINS):
    """Slab mode (orx_set_slab_partition): all N shards on the one GPU, each phase of each rank
    timed on its own (the shards run one after another), the collectives by torch ops and not
    timed (their volumes are returned).  Per-rank serial time = the slowest rank's sum of phases."""
    dev = torch.device("cuda", 0)
    scene = scene or synthetic.synthetic_hall()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    req = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H).to_abi()
    shards = []
    for rank in range(world):
        r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
        r.initialize(0)
        r.set_shard(rank, world)
        r.initScene(scene)
        b = multigpu.DeviceShard(r, torch, dev, (rank, world))
        b.enable_slab()
        shards.append(b)
    mr = (H + world - 1) // world
    hps = [b.alloc(multigpu.hp_export_floats(mr, W)) for b in shards]
    hp_all = shards[0].alloc(world * multigpu.hp_export_floats(mr, W))
    part = shards[0].alloc(world * mr * W * 3)
    names = ("local", "hist_pack", "import_grid", "gather", "finish")
    tot = [dict.fromkeys(names, 0.0) for _ in range(world)]
    a2a_mb = 0.0
    radius = scene.initial_ppm_radius()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    diag = []
    for it in range(iters):
        ms = [dict.fromkeys(names, 0.0) for _ in range(world)]
        hists = []
        for k, b in enumerate(shards):
            ms[k]["local"] += timed(lambda: (b.local_trace(it, it, radius, req), b.export_hitpoints(hps[k])))
            h = b.alloc_i32(multigpu.slab_hist_words(nb))
            ms[k]["hist_pack"] += timed(lambda: b.slab_histogram(h, nb))
            hists.append(h)
        hp_all.copy_(torch.cat(hps))
        Hh, vox, box = multigpu.split_slab_hists(torch.stack(hists).cpu().numpy(), world, nb)
        halo = [shards[0].slab_halo(nb, a, radius) for a in range(3)]
        axis, bin_dest, counts = multigpu.slab_plan(Hh, world, vox, halo)
        sends = []
        for k, b in enumerate(shards):
            n = counts[k]
            base = np.concatenate([[0], np.cumsum(n)[:-1]]).astype(np.uint32)
            send = b.alloc(9 * int(n.sum()) + 9)
            ms[k]["hist_pack"] += timed(lambda: b.slab_pack(bin_dest, nb, axis, halo[axis], base, int(n.sum()), send))
            sends.append((send, base, n))
        for d, b in enumerate(shards):
            recv = torch.cat([s_[9 * int(bs[d]):9 * int(bs[d] + n_[d])] for s_, bs, n_ in sends]).contiguous()
            ms[d]["import_grid"] += timed(lambda: b.slab_import(recv, int(counts[:, d].sum()), box, axis, nb,
                                                                multigpu.slab_owned(bin_dest, d)))
            ms[d]["gather"] += timed(lambda: b.gather_external(hp_all, world, part))
            if it == iters - 1:
                # diagnostic: the non-specular hit points whose sphere reaches this rank's photons
                pr = recv.view(-1, 9)[:, :3]
                if pr.shape[0] == 0:
                    diag.append((d, 0, 0, 0))
                else:
                    lo, hi = pr.min(0).values, pr.max(0).values
                    A = hp_all.view(world, -1)[:, :mr * W * 4].reshape(-1, 4)
                    ns = (A[:, 3].view(torch.int32) & (1 << 27)) != 0
                    q = A[:, :3]
                    # owned hit points: bin of the slab axis in this rank's range (float32 as the device)
                    alo, ahi = np.float32(scene.aabb_min[axis]), np.float32(scene.aabb_max[axis])
                    inv = np.float32(nb) / (ahi - alo)
                    v = q[:, axis].cpu().numpy().astype(np.float32)
                    bins = np.clip(np.floor((v - alo) * inv), 0, nb - 1).astype(np.int64)
                    o0, o1 = multigpu.slab_owned(bin_dest, d)
                    own = ns.cpu().numpy() & (bins >= o0) & (bins <= o1)
                    diag.append((d, int(ns.sum()), int(own.sum()), int(pr.shape[0])))
            ms[d]["finish"] += timed(lambda: b.finish(part[:mr * W * 3].contiguous()))
        if it >= warm:
            for k in range(world):
                for n_ in names:
                    tot[k][n_] += ms[k][n_]
            a2a_mb = (counts.sum() - np.trace(counts)) * 36 / 1e6
        radius = next_ppm_radius(radius, it)
    n = iters - warm
    per_rank = [{k: round(v / n, 3) for k, v in t.items()} for t in tot]
    slowest = max(range(world), key=lambda k: sum(per_rank[k].values()))
    for b in shards:
        b.r.destroy()
    print("  (rank, NS hit points, owned, photons received):", diag, flush=True)
    return per_rank, slowest, a2a_mb, int(axis), counts


def full_hitpoints(scene, W, H, world, n_iters, dev, req):
    """The full image's exported hit points of iterations 0 .. n_iters-1 (an unsharded renderer's eye
    pass, its radius sequence), each rearranged into the N ranks' row-interleaved segments: what the
    all-gather delivers to every rank.  Computed before any timing."""
    full = OptixRenderer(_abi.default_config(seed=SEED + 1, photon_launch_width=16, photon_launch_height=16))
    full.initialize(0)
    full.initScene(scene)
    fb = multigpu.DeviceShard(full, torch, dev)
    fhp = fb.alloc(multigpu.hp_export_floats(H, W))
    mr = (H + world - 1) // world
    P1, Pm = multigpu.hp_export_floats(H, W) // 7, multigpu.hp_export_floats(mr, W) // 7
    out = []
    radius = scene.initial_ppm_radius()
    for it in range(n_iters):
        fb.local_passes(it, it, radius, req)
        fb.export_hitpoints(fhp)
        A = fhp[:H * W * 4].view(H, W, 4)
        Nn = fhp[P1 * 4:P1 * 4 + H * W * 3].view(H, W, 3)
        seg = []
        for s_ in range(world):
            for P_, k in ((A, 4), (Nn, 3)):
                blk = torch.zeros(Pm * k, device=dev)
                rows = P_[s_::world]
                blk[:rows.shape[0] * W * k] = rows.reshape(-1)
                seg.append(blk)
        out.append(torch.cat(seg))
        radius = next_ppm_radius(radius, it)
    torch.cuda.synchronize()
    full.destroy()
    return out


_EMUL = None


def xgmi_emul():
    """tools/libxgmi_emul.so (built by __graft_entry__.build()): a paced copy / add kernel with an RCCL
    collective's footprint (tools/xgmi_emul.hip)."""
    global _EMUL
    if _EMUL is None:
        import ctypes as C
        _EMUL = C.CDLL(os.path.join(ROOT, "tools", "libxgmi_emul.so"))
        _EMUL.xgmi_emul.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_double, C.c_int, C.c_int, C.c_void_p]
        _EMUL.xgmi_emul.restype = C.c_int
    return _EMUL


def run_pipelined(world, W=1920, H=1080, P=2048, warm=4, steps=32, scene=None, interfere=None):
    """Rank 0 of N in the pipelined row-partition schedule ShardedPPM(pipeline=True) runs
    (multigpu.py): per iteration the local eye pass and hit-point export on the compute stream, an
    event standing for the all-gather's completion (work.wait()), the local photon pass + grid
    build (+ the own rows' direct pass on the renderer's aux stream), and on the side stream the
    gather of ALL W*H hit points (the full image's, precomputed per iteration) against the local
    photons, the own block's copy (the reduce-scatter's place) and the finish -- so the gather of
    iteration i runs beside iteration i+1's local passes, as on the real ranks.  The iteration
    window is the bench's (warmup `warm`, `steps` timed iterations, the global radius sequence), and
    the wall time between two synchronisations gives the per-rank frame without the collectives.

    interfere = (link GB/s, workgroups): the collectives' local side is run too, on a stream of its own
    at the points RCCL runs them -- the all-gather after the export, the side stream's gather waiting for
    it (work.wait()), the reduce-scatter after the gather, the finish waiting for it -- as paced kernels
    (tools/xgmi_emul.hip) that hold `workgroups` workgroups for the link time of the bytes a rank receives
    ((N-1)/N of each collective) and move those bytes through HBM (all-gather: a copy; reduce-scatter: an
    add of the received chunk into the local one)."""
    dev = torch.device("cuda", 0)
    scene = scene or synthetic.synthetic_hall()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    req = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H).to_abi()
    n = warm + steps
    hps = full_hitpoints(scene, W, H, world, n, dev, req)
    radii = multigpu.radius_sequence(scene.initial_ppm_radius(), n)
    gv = int(os.environ.get("MODEL_GATHER_VARIANT", "0"))  # 1: cell order, 2: sub-rows (0: the renderer's choice)
    r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P, gather_variant=gv))
    r.initialize(0)
    r.set_shard(0, world)
    r.initScene(scene)
    b = multigpu.DeviceShard(r, torch, dev)
    side = torch.cuda.Stream(dev)
    b.enable_pipeline(side)
    main = torch.cuda.current_stream(dev)
    mr = (H + world - 1) // world
    sets = [(b.alloc(multigpu.hp_export_floats(mr, W)), b.alloc(world * mr * W * 3), b.alloc(mr * W * 3))
            for _ in range(2)]
    ag_bytes = world * 4 * multigpu.hp_export_floats(mr, W) * (world - 1) // world // 16 * 16
    rs_bytes = world * mr * W * 12 * (world - 1) // world // 16 * 16
    if interfere and world > 1:
        link_gbs, wgs = interfere
        rccl = torch.cuda.Stream(dev)
        ag_src = torch.zeros(ag_bytes // 4, device=dev)
        ag_dst = [torch.zeros(ag_bytes // 4, device=dev) for _ in range(2)]
        rs_in = torch.zeros(rs_bytes // 4, device=dev)
        rs_acc = [torch.zeros(rs_bytes // 4, device=dev) for _ in range(2)]
        ag_ns, rs_ns = ag_bytes / link_gbs, rs_bytes / link_gbs  # bytes / (GB/s) = ns

    # ShardedPPM's schedule (MODEL_RS_DEFER=1, the default): the reduce-scatter of iteration i is issued after
    # the all-gather of i+1 (so that one does not queue behind the gather of i on RCCL's in-order stream), and
    # the finish (orx_ppm_finish_on) waits for it on a stream of its own, so that the side stream goes on to the
    # next gather; MODEL_RS_DEFER=0: the round-5 schedule (reduce-scatter and finish on the side stream)
    rs_defer = interfere and world > 1 and os.environ.get("MODEL_RS_DEFER", "1") == "1"
    if rs_defer:
        fin = torch.cuda.Stream(dev)
    pending = []

    def issue_rs(j, gdone):
        _, part_j, own_j = sets[j % 2]
        rccl.wait_event(gdone)
        xgmi_emul().xgmi_emul(rs_in.data_ptr(), rs_acc[j % 2].data_ptr(), rs_bytes, rs_ns, 1, wgs, rccl.cuda_stream)
        rdone = torch.cuda.Event()
        rdone.record(rccl)
        fin.wait_event(rdone)
        with torch.cuda.stream(fin):
            own_j.copy_(part_j[:mr * W * 3])
            b.finish_on(own_j, fin)

    def step(it):
        hp_loc, part, own = sets[it % 2]
        b.local_eye(it, it, radii[it], req)
        b.export_hitpoints(hp_loc)
        ready = torch.cuda.Event()
        ready.record(main)
        if rs_defer:
            rccl.wait_event(ready)
            xgmi_emul().xgmi_emul(ag_src.data_ptr(), ag_dst[it % 2].data_ptr(), ag_bytes, ag_ns, 0, wgs,
                                  rccl.cuda_stream)
            ag_done = torch.cuda.Event()
            ag_done.record(rccl)
            if pending:
                issue_rs(*pending.pop())
            b.local_photons()
            with torch.cuda.stream(side):
                side.wait_event(ag_done)
                b.gather_external(hps[it], world, part)
                gdone = torch.cuda.Event()
                gdone.record(side)
            pending.append((it, gdone))
            return
        if interfere and world > 1:  # the all-gather on RCCL's stream, beside the photon pass + grid build
            rccl.wait_event(ready)
            xgmi_emul().xgmi_emul(ag_src.data_ptr(), ag_dst[it % 2].data_ptr(), ag_bytes, ag_ns, 0, wgs,
                                  rccl.cuda_stream)
            ready = torch.cuda.Event()
            ready.record(rccl)
        b.local_photons()
        with torch.cuda.stream(side):
            side.wait_event(ready)
            b.gather_external(hps[it], world, part)
            if interfere and world > 1:  # the reduce-scatter after the gather, the finish waits for it
                gdone = torch.cuda.Event()
                gdone.record(side)
                rccl.wait_event(gdone)
                xgmi_emul().xgmi_emul(rs_in.data_ptr(), rs_acc[it % 2].data_ptr(), rs_bytes, rs_ns, 1, wgs,
                                      rccl.cuda_stream)
                rdone = torch.cuda.Event()
                rdone.record(rccl)
                side.wait_event(rdone)
            own.copy_(part[:mr * W * 3])
            b.finish(own)

    for it in range(warm):
        step(it)
    if pending:
        issue_rs(*pending.pop())
    torch.cuda.synchronize()
    r.reset_timing()
    t0 = time.perf_counter()
    for it in range(warm, n):
        step(it)
    if pending:
        issue_rs(*pending.pop())
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    st = r.stats()
    ni = max(1, st.timed_iterations)
    passes = {name: round(st.pass_ms[i] / ni, 3) for i, name in enumerate(_abi.PASS_NAMES) if st.pass_ms[i] > 0}
    allgather_mb = world * 4 * multigpu.hp_export_floats(mr, W) / 1e6
    rs_mb = world * mr * W * 12 / 1e6
    r.destroy()
    del hps
    torch.cuda.empty_cache()
    return ms, passes, allgather_mb, rs_mb


def run_single_pipelined(W=1920, H=1080, P=2048, warm=4, steps=32, scene=None):
    """The single-device frame the bench ships (bench.py's schedule: renderNextIteration pipelined,
    same iteration window): the reference point of the strong-scaling speed-up."""
    scene = scene or synthetic.synthetic_hall()
    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    det = RenderRequestDetails(cam, scene.name, _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    r = OptixRenderer(_abi.default_config(seed=SEED, photon_launch_width=P, photon_launch_height=P))
    r.initialize(0)
    r.initScene(scene)
    radii = multigpu.radius_sequence(scene.initial_ppm_radius(), warm + steps)
    for it in range(warm):
        r.renderNextIteration(it, it, radii[it], False, det)
    r.stats()
    t0 = time.perf_counter()
    for it in range(warm, warm + steps):
        r.renderNextIteration(it, it, radii[it], False, det)
    r.stats()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    r.destroy()
    return ms


if __name__ == "__main__":
    if "--pipelined" in sys.argv:
        # pipelined per-rank schedule against the single-device pipelined frame (bench iteration window)
        args = [a for a in sys.argv[1:] if a != "--pipelined"]
        interfere = None
        if "--interfere" in args:  # --interfere LINK_GBS WORKGROUPS: the collectives' local side run too
            i = args.index("--interfere")
            interfere = (float(args[i + 1]), int(args[i + 2]))
            args = args[:i] + args[i + 3:]
        conf = 2
        if args[:1] == ["--config"]:
            conf, args = int(args[1]), args[2:]
        worlds = [int(v) for v in args] or [1, 2, 4, 8]
        kw = (dict(W=3840, H=2160, P=4096, warm=2, steps=8, scene=synthetic.synthetic_conference()) if conf == 4
              else dict(warm=4, steps=32))
        print(f"configs[{conf}] pipelined, iterations {kw['warm']}..{kw['warm'] + kw['steps'] - 1} (the bench's window)",
              flush=True)
        single = run_single_pipelined(**kw)
        print(f"single device, bench schedule: {single:.3f} ms/frame", flush=True)
        for n in worlds:
            ms, passes, ag, rs = run_pipelined(n, interfere=interfere, **kw)
            one, alll = collectives_ms(ag, rs, n)
            # overlap-aware: the all-gather of iteration i runs beside its photon pass + grid build, the
            # reduce-scatter (side stream, after the gather) beside the next iteration's eye + photon
            # passes; only what outlasts those windows is exposed.  One link (a single ring), the slowest case.
            ag1 = ag * (n - 1) / n * 1e6 / (XGMI_LINK_GBS * 1e9) * 1e3 if n > 1 else 0.0
            rs1 = rs * (n - 1) / n * 1e6 / (XGMI_LINK_GBS * 1e9) * 1e3 if n > 1 else 0.0
            grid = sum(passes.get(k, 0.0) for k in ("grid_hash", "grid_scan", "grid_scatter"))
            win_ag = passes.get("ppm_photon", 0.0) + grid
            win_rs = passes.get("ppm_eye", 0.0) + passes.get("ppm_photon", 0.0)
            exposed = max(0.0, ag1 - win_ag) + max(0.0, rs1 - win_rs)
            ov = ms + exposed
            lo, hi = max(ms, alll), ms + one
            if interfere and n > 1:
                print(f"N={n}: per-rank pipelined frame {ms:.3f} ms WITH the collectives' local side run (paced at "
                      f"{interfere[0]:.0f} GB/s on {interfere[1]} workgroups: all-gather {ag1 * 153.0 / interfere[0]:.3f} ms, "
                      f"reduce-scatter {rs1 * 153.0 / interfere[0]:.3f} ms) = {single / ms:.2f}x the single-device frame "
                      f"| passes {passes}", flush=True)
                continue
            print(f"N={n}: per-rank pipelined frame {ms:.3f} ms (collectives not run) | all-gather {ag:.0f} MB, "
                  f"reduce-scatter {rs:.0f} MB; one link: all-gather {ag1:.3f} ms beside photon+grid {win_ag:.3f} ms, "
                  f"reduce-scatter {rs1:.3f} ms beside eye+photon {win_rs:.3f} ms -> exposed {exposed:.3f} ms; "
                  f"projected frame {ov:.3f} ms overlapped on one link = {single / ov:.2f}x the single-device frame "
                  f"(bounds: {lo:.3f} ms all {max(1, n - 1)} links hidden, {hi:.3f} ms one link nothing overlapped = "
                  f"{single / hi:.2f}-{single / lo:.2f}x) | passes {passes}", flush=True)
        sys.exit(0)

    args = sys.argv[1:]
    conf = 2
    slab = "--slab" in args
    args = [a for a in args if a not in ("--slab", "--slab1")]
    if args[:1] == ["--config"]:
        conf, args = int(args[1]), args[2:]
    worlds = [int(v) for v in args] or [1, 2, 4, 8]
    kw = (dict(W=3840, H=2160, P=4096, iters=4, warm=1, scene=synthetic.synthetic_conference()) if conf == 4
          else {})
    print(f"configs[{conf}]: " + ("conference 3840x2160, 4096^2 photons" if conf == 4 else "hall 1920x1080, 2048^2"))
    if slab:
        for n in worlds:
            if n == 1 and "--slab1" not in sys.argv:
                ms, passes, ag, rs = run(1, **kw)
                print(f"N=1: per-rank serial {sum(ms.values()):.3f} ms {ms}", flush=True)
                continue
            per_rank, slowest, a2a, axis, counts = run_slab(n, **kw)
            pr = per_rank[slowest]
            print(f"N={n} slab: per-rank serial {sum(pr.values()):.3f} ms (slowest rank {slowest}: {pr}) | "
                  f"rank sums {[round(sum(p.values()), 3) for p in per_rank]} | axis {axis}, photons per rank "
                  f"{counts.sum(0).tolist()}, all-to-all {a2a:.0f} MB", flush=True)
        sys.exit(0)
    base = None
    for n in worlds:
        ms, passes, ag, rs = run(n, **kw)
        comp = sum(ms.values())
        one, alll = collectives_ms(ag, rs, n)
        base = comp if n == 1 else base
        # projected frame: the all-gather overlaps the photon pass and the reduce-scatter the next
        # iteration's local passes in the pipelined schedule ('hidden': max(compute, exchange));
        # 'exposed': compute + exchange (nothing overlapped)
        proj = (f" | exchange {one:.3f} ms on one link, {alll:.3f} ms over {n - 1} links; projected frame "
                f"{max(comp, alll):.3f}-{comp + one:.3f} ms" + (f" ({base / (comp + one):.1f}-{base / max(comp, alll):.1f}x"
                                                                f" of N=1)" if base else "")) if n > 1 else ""
        print(f"N={n}: per-rank serial {comp:.3f} ms {ms} | all-gather {ag:.0f} MB, "
              f"reduce-scatter {rs:.0f} MB{proj} | passes {passes}", flush=True)
