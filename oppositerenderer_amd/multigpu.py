"""Multi-GPU progressive photon mapping: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests).

Two partitions.  The photon-batch partition (BatchSharded, bench.py's default) is the
reference's own distributed mode: every rank renders whole iterations (global iteration
numbers dealt round-robin, the global radius sequence, its own RNG streams) and the
accumulated radiance buffers are summed by one reduce every few iterations.  The row
partition (ShardedPPM / ShardedVCM / ShardedPT) splits one frame over the ranks:

Sharding (option A) — rank g of N owns every RNG-slot row
y with y % N == g, i.e. its pixel rows AND its photon-launch rows (photon
thread (x,y) aliases RNG slot (x,y), OptixRenderer_SpatialHash.cu:310-334),
so RNG state never crosses GPUs.  Per PPM iteration:

  1. local passes   eye rays for own pixel rows, own photon batch, photon grid over own photons
  2. all-gather     compact hitpoints (28 B/pixel) of every rank           (RCCL all_gather)
  3. gather         ALL pixels against the own photon grid -> partial indirect radiance
  4. reduce-scatter partial indirect, summed, to the row owners            (RCCL reduce_scatter)
  5. finish         own hit points' attenuation, direct light + running-sum output on own rows

The gather is linear in the photon set and normalises by the global emitted
count, so the result equals one GPU running the union photon launch, up to
fp32 summation order.  The photon launch is global: rank g traces the launch
rows y % N == g, so a fixed photon_launch_width x photon_launch_height
workload is split over the ranks (strong scaling, the bench default);
bench_main's weak mode instead sets the global launch height to N x the
per-rank height.

Backends: `DeviceShard` drives liborx.so with torch device tensors on the
renderer's (= torch's current) stream; tests drive the CPU oracle through
the same phase API with gloo (tests/test_multigpu_gloo.py).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import time

import numpy as np


HP_EXPORT_FLOATS = 7  # orx_export_hitpoints: 28 B per pixel (position|flags float4, normal float3)


def hp_export_floats(max_rows, W):
    """float32 words of one rank's orx_export_hitpoints buffer (orx_hitpoint_export_bytes / 4): two
    planes of max_rows * W pixels rounded up to a multiple of 4 (16-B aligned segments)"""
    return HP_EXPORT_FLOATS * ((max_rows * W + 3) // 4 * 4)


def local_rows(H, rank, world):
    return (H - rank + world - 1) // world if H > rank else 0


SLAB_BINS = 1024
SLAB_VOXELS = 32  # ORX_SLAB_VOXELS (include/orx.h)


def slab_hist_words(nb):
    """uint32 words of one rank's orx_ppm_slab_histogram output (orx_slab_histogram_words):
    [2][3][nb] counts, the AABB of its photons, [2][V^3] voxel counts"""
    return 6 * nb + 6 + 2 * SLAB_VOXELS ** 3


def split_slab_hists(words, world, nb):
    """all-gathered histogram words -> (counts uint32[world][2][3][nb], voxel counts
    uint32[world][2][V^3] (photons, hit points; voxel x + V (y + V z)), the AABB of every rank's
    photons: uint32[6] ordered words, include/orx.h orx_ppm_slab_import's photon_box)"""
    w = np.ascontiguousarray(words).view(np.uint32).reshape(world, slab_hist_words(nb))
    box = np.concatenate([w[:, 6 * nb:6 * nb + 3].min(0), w[:, 6 * nb + 3:6 * nb + 6].max(0)]).astype(np.uint32)
    vox = w[:, 6 * nb + 6:].reshape(world, 2, SLAB_VOXELS ** 3)
    return w[:, :6 * nb].reshape(world, 2, 3, nb), vox, box


def slab_plan(hists, world, vox=None, halo=0, w_gather=0.8, w_photon=0.15, w_pixel=0.05):
    """The slab partition of one iteration (include/orx.h orx_set_slab_partition), computed on
    every rank from the all-gathered histograms, identically (float64 numpy on identical inputs).

    hists: [world][2][3][nb] counts (uint32): each rank's valid deposits and own non-specular hit
    points per bin of each axis of the scene AABB; vox: [world][2][V^3] the same over V^3 voxels.
    A bin's cost mixes the gather (its hit points, each weighted by the photon count of its voxel:
    a hit point gathers the photons near it; spread over the bins of a voxel layer by their hit
    points), the import and grid build (photons) and the per-pixel work (hit points), each
    normalised to sum 1.  Without vox the gather term is photons x hit points per bin.  On each
    axis every bin goes to the rank whose share of the cumulative cost holds the bin's midpoint
    (contiguous slabs, ascending ranks); the axis with the smallest largest-slab cost wins (ties:
    the lower axis).  halo: bins (one int, or one per axis, include/orx.h orx_ppm_slab_halo): a
    photon in bin b also goes to the ranks of bins b - halo .. b + halo.
    Returns (axis, bin_dest uint8[nb], counts int64[world][world]: photons rank s sends to rank d)."""
    h = np.asarray(hists, dtype=np.float64).reshape(world, 2, 3, -1)
    nb = h.shape[-1]
    ph, hp = h[:, 0].sum(0), h[:, 1].sum(0)
    if vox is not None:
        V = SLAB_VOXELS
        v = np.asarray(vox, dtype=np.float64).reshape(world, 2, V, V, V).sum(0)  # [2][z][y][x]
        cost = v[0] * v[1]  # hit points x photons in the same voxel
        layer = nb // V
    best = None
    for a in range(3):
        if vox is not None:
            ax = (2, 1, 0)[a]  # numpy axis of voxel coordinate a
            other = tuple(k for k in range(3) if k != ax)
            lc, lh = cost.sum(axis=other), v[1].sum(axis=other)  # per voxel layer
            per_hp = np.divide(lc, lh, out=np.zeros_like(lc), where=lh > 0)
            g = hp[a] * np.repeat(per_hp, layer)
        else:
            g = ph[a] * hp[a]
        w = np.zeros(nb)
        for part, weight in ((g, w_gather), (ph[a], w_photon), (hp[a], w_pixel)):
            tot = part.sum()
            if tot > 0:
                w += weight * part / tot
        total = w.sum()
        if total > 0:
            mid = np.cumsum(w) - 0.5 * w
            dest = np.minimum(np.floor(mid * world / total), world - 1).astype(np.int64)
        else:
            dest = np.minimum(np.arange(nb) * world // nb, world - 1)
        cost_a = np.bincount(dest, weights=w, minlength=world).max() if total > 0 else 0.0
        if best is None or cost_a < best[0]:
            best = (cost_a, a, dest)
    _, axis, dest = best
    return axis, dest.astype(np.uint8), slab_counts(h[:, 0, axis], dest, world, halo_of(halo, axis))


def halo_of(halo, axis):
    return int(halo[axis]) if np.ndim(halo) else int(halo)


def slab_counts(ph, dest, world, halo):
    """photons rank s sends to rank d (orx_ppm_slab_pack): ph[s][b] photon counts per bin, a photon
    in bin b going to every rank from dest[b - halo] to dest[b + halo] (clamped; dest ascending)"""
    ph = np.asarray(ph, dtype=np.float64)
    nb = len(dest)
    b = np.arange(nb)
    d0 = np.asarray(dest)[np.maximum(b - halo, 0)]
    d1 = np.asarray(dest)[np.minimum(b + halo, nb - 1)]
    r = np.arange(world)
    m = ((r[None, :] >= d0[:, None]) & (r[None, :] <= d1[:, None])).astype(np.float64)  # [nb][world]
    return np.rint(ph @ m).astype(np.int64)


def slab_owned(dest, rank):
    """(own_lo, own_hi): the bins rank owns (own_lo > own_hi: none), include/orx.h orx_ppm_slab_import"""
    idx = np.nonzero(np.asarray(dest) == rank)[0]
    return (int(idx[0]), int(idx[-1])) if len(idx) else (1, 0)


def assemble_rows(blocks, W, H, world):
    """blocks[g]: [max_rows, W, 3] of rank g (local row j = global row g + j*world)."""
    img = np.zeros((H, W, 3), np.float32)
    for g, b in enumerate(blocks):
        n = local_rows(H, g, world)
        img[g::world] = b[:n]
    return img


def batch_seed(seed, rank, clock_ns=None):
    """Rank g's RNG seed in the photon-batch partition.  Rank 0 keeps the configured seed, so a
    one-rank job renders exactly the single-device sequence; the others get their own XORWOW
    streams, as the reference's render servers each seed from their own clock
    (OptixRenderer_SpatialHash.cu:319-334).  Seed 0 (the renderer seeds from clock()/time(NULL)):
    rank 0 keeps 0; every other rank gets a seed from this process's nanosecond clock with the rank
    mixed in, since ranks started in the same second would otherwise share time(NULL) and draw
    correlated streams."""
    if rank == 0:
        return seed
    if seed == 0:
        t = time.time_ns() if clock_ns is None else int(clock_ns)
        seed = (t ^ (t >> 32)) & 0xFFFFFFFF
    return ((seed + 0x9E3779B9 * rank) & 0xFFFFFFFF) or 1


def batch_iteration(i, rank, world):
    """Global iteration number of rank's i-th local iteration: the reference's client deals
    consecutive iteration numbers round-robin to its render servers (DistributedApplication.cpp:96-122)."""
    return i * world + rank


def radius_sequence(r0, n, alpha=2.0 / 3.0):
    """PPM radii of global iterations 0..n-1 (the client's host-computed sequence, StandaloneRenderManager.cpp:105-107)."""
    from .renderer import next_ppm_radius

    out = [float(r0)]
    for k in range(n - 1):
        out.append(next_ppm_radius(out[-1], k, alpha))
    return out


class BatchSharded:
    """Photon-batch partition, the reference's own multi-GPU mode: its client deals consecutive
    iteration numbers with the host-computed radius sequence to the render servers
    (DistributedApplication.cpp:96-122) and merges their running-sum buffers
    (RenderResultPacketReceiver.cpp:63-190).  Rank g renders global iterations g, g + N, g + 2N, ...
    of the whole frame with a full photon launch and its own RNG streams (batch_seed) on the
    single-device path (pipelined PPM, VCM, PT), so an iteration needs no exchange at all; the
    accumulated radiance buffers are summed by one reduce to rank 0 (RCCL over xGMI) every
    `reduce_every` local iterations and on image().  The merged buffer is the sum of the ranks'
    running sums: divide by the total iteration count to display, as for one device.

    Backends expose render_next / output_local_tensor(rows)."""

    def __init__(self, backend, dist, world, rank, W, H, reduce_every=8):
        self.b, self.dist, self.world, self.rank, self.W, self.H = backend, dist, world, rank, W, H
        self.reduce_every = int(reduce_every)
        self.n = 0
        self.merged = None

    def iteration(self, it, local_it, radius, request):
        """`it` is the global iteration number (batch_iteration), `local_it` the rank's own count."""
        self.b.render_next(it, local_it, radius, request)
        self.n += 1
        if self.reduce_every > 0 and self.n % self.reduce_every == 0:
            self.reduce()

    def reduce(self):
        """Sum of every rank's running-sum radiance buffer, on rank 0 (collective)."""
        t = self.b.output_local_tensor(self.H)
        self.dist.reduce(t, dst=0)
        self.merged = t

    def image(self):
        """The merged running sum on rank 0 (None elsewhere; collective)."""
        self.reduce()
        if self.rank != 0:
            return None
        return self.merged.detach().cpu().numpy().reshape(self.H, self.W, 3).copy()


class ShardedPPM:
    """Runs the 5-step sharded iteration for any backend exposing
    local_passes / export_hitpoints / gather_external / finish / alloc."""

    def __init__(self, backend, dist, world, rank, W, H, pipeline=False, slab=False):
        self.b, self.dist, self.world, self.rank, self.W, self.H = backend, dist, world, rank, W, H
        self.max_rows = (H + world - 1) // world
        self.gloo = dist.get_backend() == "gloo"
        self.pipe = pipeline and not self.gloo and hasattr(backend, "enable_pipeline")
        self.slab = slab
        if slab:
            # spatial photon partition: each rank gathers against the photons of its slab
            backend.enable_slab()
            s_local, s_global = backend.slot_capacity()
            self.nb = SLAB_BINS
            self.hist = backend.alloc_i32(slab_hist_words(self.nb))
            self.hists = backend.alloc_i32(world * slab_hist_words(self.nb))
            self.send = backend.alloc(9 * s_local + 9)
            self.recv = backend.alloc(9 * s_global + 9)
            self.last_plan = None
        nsets = 2 if self.pipe else 1
        hpf = hp_export_floats(self.max_rows, W)
        self.sets = [(backend.alloc(hpf),                                # own hitpoints, 28 B/px as float32
                      backend.alloc(world * hpf),                        # all hitpoints
                      backend.alloc(world * self.max_rows * W * 3),      # partial indirect, all pixels
                      backend.alloc(self.max_rows * W * 3))              # summed indirect, own rows
                     for _ in range(nsets)]
        self.hp_local, self.hp_all, self.ind_partial, self.ind_local = self.sets[0]
        self.k = 0
        self.pending = None  # pipelined: the last gather's (partial, summed indirect, done event), not yet reduced
        if self.pipe:
            backend.enable_pipeline()
            # the reduce-scatter + finish of iteration i run here, issued after iteration i+1's all-gather:
            # RCCL runs one communicator's collectives in issue order, so a reduce-scatter issued right
            # after the gather of i would hold the all-gather of i+1 until that gather ends, and the side
            # stream would wait for it before the next gather (tools/shard_model.py --interfere: configs[4]
            # N=8 per-rank frame 7.96 -> 6.74 ms with the collectives' local side emulated)
            self.fin = backend.torch.cuda.Stream(backend.device)

    def slab_exchange(self, radius):
        """histograms -> plan (host) -> pack -> all-to-all of the photon records -> import + grid"""
        b, d, world, rank = self.b, self.dist, self.world, self.rank
        b.slab_histogram(self.hist, self.nb)
        if self.gloo:
            d.all_gather(list(self.hists.chunk(world)), self.hist)
        else:
            d.all_gather_into_tensor(self.hists, self.hist)
        hists, vox, box = split_slab_hists(self.hists.cpu().numpy(), world, self.nb)
        halo = [b.slab_halo(self.nb, a, radius) for a in range(3)]
        axis, bin_dest, counts = slab_plan(hists, world, vox, halo)
        send_n, recv_n = counts[rank], counts[:, rank]
        base = np.concatenate([[0], np.cumsum(send_n)[:-1]]).astype(np.uint32)
        ns, nr = int(send_n.sum()), int(recv_n.sum())
        if 9 * ns + 9 > self.send.numel():  # halo copies: more records than own photons
            self.send = b.alloc(9 * ns + 9)
        b.slab_pack(bin_dest, self.nb, axis, halo[axis], base, ns, self.send)
        recv = self.recv[:9 * nr]
        d.all_to_all_single(recv, self.send[:9 * ns], (9 * recv_n).tolist(), (9 * send_n).tolist())
        own = slab_owned(bin_dest, rank)
        b.slab_import(recv, nr, box, axis, self.nb, own)
        self.last_plan = (axis, bin_dest, counts)

    def _gather_async(self, work, hp_all, ind_partial, ind_local):
        """pipelined: the gather of this iteration on the side stream once its all-gather is in; its
        reduce-scatter + finish wait for the next iteration's all-gather to be issued (drain)"""
        torch = self.b.torch
        with torch.cuda.stream(self.b.side):
            work.wait()
            self.b.gather_external(hp_all, self.world, ind_partial)
            done = torch.cuda.Event()
            done.record(self.b.side)
        self.pending = (ind_partial, ind_local, done)

    def drain(self):
        """Issue the outstanding reduce-scatter + finish (pipelined schedule; a no-op otherwise): called by
        the next iteration right after its all-gather, and before anything reads the output."""
        if self.pending is None:
            return
        ind_partial, ind_local, done = self.pending
        self.pending = None
        torch = self.b.torch
        with torch.cuda.stream(self.fin):
            self.fin.wait_event(done)
            self.dist.reduce_scatter_tensor(ind_local, ind_partial)
            self.b.finish_on(ind_local, self.fin)

    def iteration(self, it, local_it, radius, request):
        d = self.dist
        if self.slab:
            return self._iteration_slab(it, local_it, radius, request)
        if self.pipe:
            # iteration i's gather on the side stream and its reduce-scatter + output on the finish stream
            # while the next iteration's eye, photon and grid passes run on the compute stream (buffer sets
            # alternate; the renderer orders the RNG chain and the buffer reuse with events)
            hp_local, hp_all, ind_partial, ind_local = self.sets[self.k]
            self.k ^= 1
            self.b.local_eye(it, local_it, radius, request)
            self.b.export_hitpoints(hp_local)
            work = d.all_gather_into_tensor(hp_all, hp_local, async_op=True)
            self.drain()  # the previous iteration's reduce-scatter + finish, behind this all-gather
            self.b.local_photons()
            self._gather_async(work, hp_all, ind_partial, ind_local)
            return
        if self.gloo or not hasattr(self.b, "local_eye"):
            self.b.local_passes(it, local_it, radius, request)
            self.b.export_hitpoints(self.hp_local)
            if self.gloo:
                parts = list(self.hp_all.chunk(self.world))
                d.all_gather(parts, self.hp_local)
            else:
                d.all_gather_into_tensor(self.hp_all, self.hp_local)
        else:
            # eye pass, then the hitpoint all-gather on RCCL's stream overlaps
            # the photon pass + grid build on the compute stream
            self.b.local_eye(it, local_it, radius, request)
            self.b.export_hitpoints(self.hp_local)
            work = d.all_gather_into_tensor(self.hp_all, self.hp_local, async_op=True)
            self.b.local_photons()
            work.wait()
        self.b.gather_external(self.hp_all, self.world, self.ind_partial)
        if self.gloo:  # gloo has no reduce_scatter: all_reduce + own block
            d.all_reduce(self.ind_partial)
            blk = self.max_rows * self.W * 3
            self.ind_local.copy_(self.ind_partial[self.rank * blk:(self.rank + 1) * blk])
        else:
            d.reduce_scatter_tensor(self.ind_local, self.ind_partial)
        self.b.finish(self.ind_local)

    def _iteration_slab(self, it, local_it, radius, request):
        d = self.dist
        if self.pipe:
            hp_local, hp_all, ind_partial, ind_local = self.sets[self.k]
            self.k ^= 1
            self.b.local_eye(it, local_it, radius, request)
            self.b.export_hitpoints(hp_local)
            work = d.all_gather_into_tensor(hp_all, hp_local, async_op=True)
            self.drain()
            self.b.local_photon_trace()
            self.slab_exchange(radius)
            self._gather_async(work, hp_all, ind_partial, ind_local)
            return
        self.b.local_trace(it, local_it, radius, request)
        self.b.export_hitpoints(self.hp_local)
        if self.gloo:
            d.all_gather(list(self.hp_all.chunk(self.world)), self.hp_local)
        else:
            d.all_gather_into_tensor(self.hp_all, self.hp_local)
        self.slab_exchange(radius)
        self.b.gather_external(self.hp_all, self.world, self.ind_partial)
        if self.gloo:
            d.all_reduce(self.ind_partial)
            blk = self.max_rows * self.W * 3
            self.ind_local.copy_(self.ind_partial[self.rank * blk:(self.rank + 1) * blk])
        else:
            d.reduce_scatter_tensor(self.ind_local, self.ind_partial)
        self.b.finish(self.ind_local)

    def image(self):
        """Full running-sum image on every rank (collective)."""
        if hasattr(self, "drain"):
            self.drain()
        out = self.b.output_local_tensor(self.max_rows)
        parts = [out.clone() for _ in range(self.world)]
        self.dist.all_gather(parts, out)
        blocks = [p.detach().cpu().numpy().reshape(self.max_rows, self.W, 3) for p in parts]
        return assemble_rows(blocks, self.W, self.H, self.world)


class ShardedVCM:
    """Sharded VCM iteration (include/orx.h orx_vcm_*): light + camera subpaths
    of the own rows; the light pass's connectCameraT1 splats (vcm.h:311-384)
    are the only cross-rank data, summed with one reduce-scatter of the
    owner-block splat buffers [world][max_rows][W][3] before the camera pass.

    Backends expose vcm_local_light / export_vcm_splats / vcm_finish / alloc."""

    def __init__(self, backend, dist, world, rank, W, H):
        self.b, self.dist, self.world, self.rank, self.W, self.H = backend, dist, world, rank, W, H
        self.max_rows = (H + world - 1) // world
        self.rows = local_rows(H, rank, world)
        self.blk = self.max_rows * W * 3
        self.splat_all = backend.alloc(world * self.blk)
        self.splat_own = backend.alloc(self.blk)
        self.gloo = dist.get_backend() == "gloo"

    def iteration(self, it, local_it, radius, request):
        self.b.vcm_local_light(it, local_it, radius, request)
        self.b.export_vcm_splats(self.splat_all)
        if self.gloo:  # gloo has no reduce_scatter: all_reduce + own block
            self.dist.all_reduce(self.splat_all)
            self.splat_own.copy_(self.splat_all[self.rank * self.blk:(self.rank + 1) * self.blk])
        else:
            self.dist.reduce_scatter_tensor(self.splat_own, self.splat_all)
        self.b.vcm_finish(self.splat_own)

    image = ShardedPPM.image


class ShardedPT:
    """Path tracing shards by pixel rows with no per-iteration exchange
    (SURVEY 8(e)): each rank runs RayGeneratorPT over its own rows
    (orx_render_next_iteration on a sharded renderer); only the image is
    gathered, on request."""

    def __init__(self, backend, dist, world, rank, W, H):
        self.b, self.dist, self.world, self.rank, self.W, self.H = backend, dist, world, rank, W, H
        self.max_rows = (H + world - 1) // world

    def iteration(self, it, local_it, radius, request):
        self.b.render_next(it, local_it, radius, request)

    image = ShardedPPM.image


class DeviceShard:
    """liborx.so backend: buffers are torch device tensors, kernels run on torch's current stream."""

    def __init__(self, renderer, torch, device, rank_world=(0, 1)):
        self.r, self.torch, self.device = renderer, torch, device
        self.rank_world = rank_world
        lib = renderer._lib
        for name, args, res in (
            ("orx_set_stream", [C.c_void_p, C.c_void_p, C.c_int], C.c_int),
            ("orx_ppm_local_passes", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orx_ppm_local_eye", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orx_ppm_local_photons", [C.c_void_p], C.c_int),
            ("orx_export_hitpoints", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orx_ppm_gather_external", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t], C.c_int),
            ("orx_ppm_finish", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orx_ppm_finish_on", [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p], C.c_int),
            ("orx_set_ppm_pipeline", [C.c_void_p, C.c_void_p, C.c_int], C.c_int),
            ("orx_vcm_local_light", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orx_export_vcm_splats", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orx_vcm_finish", [C.c_void_p, C.c_void_p, C.c_size_t], C.c_int),
            ("orx_set_slab_partition", [C.c_void_p, C.c_int], C.c_int),
            ("orx_ppm_local_trace", [C.c_void_p, C.c_uint64, C.c_uint64, C.c_float, C.c_void_p], C.c_int),
            ("orx_ppm_local_photon_trace", [C.c_void_p], C.c_int),
            ("orx_ppm_slab_histogram", [C.c_void_p, C.c_void_p, C.c_uint32], C.c_int),
            ("orx_ppm_slab_pack", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                   C.c_uint64, C.c_void_p], C.c_int),
            ("orx_ppm_slab_import", [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_uint32,
                                     C.c_uint32, C.c_uint32], C.c_int),
            ("orx_ppm_slab_halo", [C.c_void_p, C.c_uint32, C.c_uint32, C.c_float], C.c_uint32),
        ):
            f = getattr(lib, name)
            f.argtypes, f.restype = args, res
        self.lib = lib
        # one non-blocking stream shared by the renderer, torch ops and the
        # RCCL collectives (which order themselves after torch's current stream)
        cur = torch.cuda.current_stream(device)
        if cur.cuda_stream == 0:
            torch.cuda.set_stream(torch.cuda.Stream(device))
            cur = torch.cuda.current_stream(device)
        self.stream = cur
        self.side = None
        renderer._check(lib.orx_set_stream(renderer._h, C.c_void_p(cur.cuda_stream), 1))

    def enable_pipeline(self, side=None):
        """Gather + finish of iteration i on a side stream, overlapping iteration i+1's local
        passes (orx_set_ppm_pipeline; before the first iteration)."""
        self.side = side if side is not None else self.torch.cuda.Stream(self.device)
        self.r._check(self.lib.orx_set_ppm_pipeline(self.r._h, C.c_void_p(self.side.cuda_stream), 1))

    def alloc(self, nfloat):
        return self.torch.zeros(nfloat, dtype=self.torch.float32, device=self.device)

    def alloc_i32(self, n):
        return self.torch.zeros(n, dtype=self.torch.int32, device=self.device)

    def local_passes(self, it, local_it, radius, request):
        self.r._check(self.lib.orx_ppm_local_passes(self.r._h, it, local_it, radius, C.byref(request)))

    # -- slab mode (orx_set_slab_partition) --
    def enable_slab(self):
        self.r._check(self.lib.orx_set_slab_partition(self.r._h, 1))

    def slot_capacity(self):
        """(own deposit slots, global deposit slots): the send and receive capacities in photons"""
        cfg = self.r._cfg
        rank, world = self.rank_world
        prows = local_rows(cfg.photon_launch_height, rank, world)
        return (cfg.photon_launch_width * prows * cfg.max_photon_deposits,
                cfg.photon_launch_width * cfg.photon_launch_height * cfg.max_photon_deposits)

    def local_trace(self, it, local_it, radius, request):
        self.r._check(self.lib.orx_ppm_local_trace(self.r._h, it, local_it, radius, C.byref(request)))

    def local_photon_trace(self):
        self.r._check(self.lib.orx_ppm_local_photon_trace(self.r._h))

    def slab_histogram(self, hist, nb):
        self.r._check(self.lib.orx_ppm_slab_histogram(self.r._h, C.c_void_p(hist.data_ptr()), nb))

    def slab_halo(self, nb, axis, radius):
        return int(self.lib.orx_ppm_slab_halo(self.r._h, nb, axis, radius))

    def slab_pack(self, bin_dest, nb, axis, halo, base, n_records, send):
        bd = np.ascontiguousarray(bin_dest, np.uint8)
        bs = np.ascontiguousarray(base, np.uint32)
        self.r._check(self.lib.orx_ppm_slab_pack(self.r._h, bd.ctypes.data, nb, axis, halo, bs.ctypes.data,
                                                 n_records, C.c_void_p(send.data_ptr())))

    def slab_import(self, recv, n_records, box, axis, nb, own):
        bx = None if box is None else np.ascontiguousarray(box, np.uint32)
        self.r._check(self.lib.orx_ppm_slab_import(self.r._h, C.c_void_p(recv.data_ptr()), n_records,
                                                   None if bx is None else bx.ctypes.data, axis, nb, own[0],
                                                   own[1]))

    def local_eye(self, it, local_it, radius, request):
        self.r._check(self.lib.orx_ppm_local_eye(self.r._h, it, local_it, radius, C.byref(request)))

    def local_photons(self):
        self.r._check(self.lib.orx_ppm_local_photons(self.r._h))

    def export_hitpoints(self, t):
        self.r._check(self.lib.orx_export_hitpoints(self.r._h, C.c_void_p(t.data_ptr()), t.numel() * 4))

    def gather_external(self, hp_all, segments, out):
        self.r._check(self.lib.orx_ppm_gather_external(self.r._h, C.c_void_p(hp_all.data_ptr()), segments,
                                                       C.c_void_p(out.data_ptr()), out.numel() * 4))

    def finish(self, ind_local):
        self.r._check(self.lib.orx_ppm_finish(self.r._h, C.c_void_p(ind_local.data_ptr()), ind_local.numel() * 4))

    def finish_on(self, ind_local, stream):
        """orx_ppm_finish_on: the oldest outstanding pipelined iteration's finish, on `stream`"""
        self.r._check(self.lib.orx_ppm_finish_on(self.r._h, C.c_void_p(ind_local.data_ptr()), ind_local.numel() * 4,
                                                 C.c_void_p(stream.cuda_stream)))

    def render_next(self, it, local_it, radius, request):
        self.r._check(self.lib.orx_render_next_iteration(self.r._h, it, local_it, radius, 1, C.byref(request)))

    def vcm_local_light(self, it, local_it, radius, request):
        self.r._check(self.lib.orx_vcm_local_light(self.r._h, it, local_it, radius, C.byref(request)))

    def export_vcm_splats(self, t):
        self.r._check(self.lib.orx_export_vcm_splats(self.r._h, C.c_void_p(t.data_ptr()), t.numel() * 4))

    def vcm_finish(self, splat_own):
        self.r._check(self.lib.orx_vcm_finish(self.r._h, C.c_void_p(splat_own.data_ptr()), splat_own.numel() * 4))

    def output_local_tensor(self, max_rows):
        t = self.alloc(max_rows * self.r.getWidth() * 3)
        self.r.getOutputBufferDevice(t.data_ptr(), t.numel() * 4)
        return t


class DeviceBatch:
    """liborx.so backend of the photon-batch partition: a whole-frame renderer on its own streams
    (the single-device pipelined path); the radiance buffer is copied out on the renderer's stream
    and handed to torch's stream for the collective."""

    def __init__(self, renderer, torch, device):
        self.r, self.torch, self.device = renderer, torch, device
        self.ext = None

    def render_next(self, it, local_it, radius, request):
        self.r._check(self.r._lib.orx_render_next_iteration(self.r._h, it, local_it, radius, 1, C.byref(request)))

    def alloc(self, nfloat):
        return self.torch.zeros(nfloat, dtype=self.torch.float32, device=self.device)

    def output_local_tensor(self, rows):
        torch = self.torch
        if self.ext is None:
            self.ext = torch.cuda.ExternalStream(self.r.stream_handle(), device=self.device)
        cur = torch.cuda.current_stream(self.device)
        t = torch.empty(rows * self.r.getWidth() * 3, dtype=torch.float32, device=self.device)
        self.ext.wait_stream(cur)  # t's block may have been read by the last collective on cur
        self.r.getOutputBufferDevice(t.data_ptr(), t.numel() * 4)  # after the pipelined output pass
        cur.wait_stream(self.ext)
        return t


def device_batch_factory(cfg, rank, world, local_rank, scene):
    """The photon-batch backend on HIP device `local_rank`: rank's seed (batch_seed), whole frame,
    full photon launch (raises without a GPU or without liborx.so; no CPU fallback)."""
    import torch

    from .renderer import OptixRenderer

    torch.cuda.set_device(local_rank)
    c = type(cfg).from_buffer_copy(cfg)
    c.seed = batch_seed(cfg.seed, rank)
    r = OptixRenderer(c)
    r.initialize(local_rank)
    r.initScene(scene)
    return DeviceBatch(r, torch, torch.device("cuda", local_rank))


def device_shard_factory(cfg, rank, world, local_rank, scene):
    """The product backend of the multi-GPU bench: liborx.so on HIP device `local_rank`
    (raises without a GPU or without liborx.so; there is no CPU fallback)."""
    import torch

    from .renderer import OptixRenderer

    torch.cuda.set_device(local_rank)
    r = OptixRenderer(cfg)
    r.initialize(local_rank)
    r.set_shard(rank, world)
    r.initScene(scene)
    return DeviceShard(r, torch, torch.device("cuda", local_rank), (rank, world))


def _resolve_factory(batch=False):
    """ORX_SHARD_BACKEND=module:function swaps the shard backend (ORX_BATCH_BACKEND for the
    photon-batch partition); only the CPU launcher test (tests/test_bench_launch.py) sets them, to
    run the orchestration under gloo on the oracle."""
    spec = os.environ.get("ORX_BATCH_BACKEND" if batch else "ORX_SHARD_BACKEND")
    if not spec:
        return (device_batch_factory if batch else device_shard_factory), "hip"
    import importlib

    mod, fn = spec.split(":")
    return getattr(importlib.import_module(mod), fn), spec


_METHOD = {0: "PT", 1: "VCM", 2: "PPM"}  # orx_method (include/orx.h)


def bench_main(args, metric, cpu_baseline=None):
    """bench.py --gpus N, one rank per GPU (bench.py starts the ranks itself when no launcher
    set WORLD_SIZE).  PPM: strong scaling by default (the global photon launch P x P and the
    W x H pixels are fixed and dealt to the ranks by rows); args.scaling == "weak" gives every
    rank a full P x P photon launch.  cpu_baseline: bench.py's oracle timing, run on rank 0 when
    there is one rank."""
    import torch
    import torch.distributed as dist

    from . import _abi, scenes
    from .renderer import RenderRequestDetails

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    method = getattr(args, "method", "ppm")
    if method not in ("ppm", "vcm", "pt"):
        raise SystemExit("the sharded bench runs ppm, vcm or pt")
    vcm = method == "vcm"
    pt = method == "pt"
    partition = getattr(args, "partition", "batch")
    batch = partition == "batch"
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    factory, backend_name = _resolve_factory(batch)
    on_gpu = backend_name == "hip"
    # RCCL prints its version banner on fd 1: keep stdout for the one JSON line
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    W, H, P = args.width, args.height, args.photon_launch
    scene = scenes.scene_by_name(args.scene)
    weak = getattr(args, "scaling", "strong") == "weak" and not batch
    PH = P * world if weak else P  # global photon launch height (batch: every rank's own launch)
    cfg = _abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=PH,
                              gather_variant=args.gather_variant)
    # the renderer (and its streams) before the process group: RCCL's streams then take the
    # hardware queues after the renderer's three
    if on_gpu:
        torch.cuda.set_device(local_rank)
    backend = factory(cfg, rank, world, local_rank, scene)
    r = backend.r
    if on_gpu:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group("gloo")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    cam = scene.default_camera.set_aspect_ratio(float(np.float32(W) / np.float32(H)))
    mcode = (_abi.VCM_BIDIRECTIONAL_PATH_TRACING if vcm else _abi.PATH_TRACING if pt
             else _abi.PROGRESSIVE_PHOTON_MAPPING)
    det = RenderRequestDetails(cam, scene.name, mcode, W, H)
    req = det.to_abi()
    n_total = max(1, args.warmup) + args.steps
    radii = radius_sequence(scene.initial_ppm_radius(), n_total * (world if batch else 1))
    if batch:
        sharded = BatchSharded(backend, dist, world, rank, W, H, reduce_every=getattr(args, "reduce_every", 8))
    elif vcm or pt:
        sharded = (ShardedVCM if vcm else ShardedPT)(backend, dist, world, rank, W, H)
    else:
        slab = partition == "slab" and world > 1
        sharded = ShardedPPM(backend, dist, world, rank, W, H, pipeline=os.environ.get("ORX_PIPELINE", "1") != "0",
                             slab=slab)

    def step(i):
        """local iteration i: the rank's global iteration number (batch: dealt round-robin) and its radius"""
        it = batch_iteration(i, rank, world) if batch else i
        sharded.iteration(it, i, radii[it], req)

    drain = getattr(sharded, "drain", lambda: None)  # pipelined rows/slab: the last reduce-scatter + finish
    i = 0
    for _ in range(max(1, args.warmup)):
        step(i)
        i += 1
    drain()
    sync()
    dist.barrier()
    if hasattr(r, "reset_timing"):
        r.reset_timing()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(i)
        i += 1
    if batch and sharded.reduce_every > 0 and sharded.n % sharded.reduce_every:
        sharded.reduce()  # the timed job ends with its radiance merged on rank 0
    drain()  # the timed job ends with the last iteration's reduce-scatter and output
    sync()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local_rank) if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())
    world_size = dist.get_world_size()
    st = r.stats()
    if rank == 0:
        from . import roofline
        # PPM: the global launch P x PH (PH = P strong, P * world weak); VCM: the W*H light +
        # W*H camera subpaths are split over the ranks (strong scaling)
        paths = 2 * W * H if vcm else W * H if pt else W * H + P * PH
        if batch:  # every rank renders whole iterations: W*H eye (+ W*H light) paths and P x P photons each
            paths *= world
        n_it = max(1, st.timed_iterations)
        per_pass = {name: st.pass_ms[i] / n_it for i, name in enumerate(_abi.PASS_NAMES)}
        per_pass = {k: v for k, v in per_pass.items() if v > 0}
        # pipelined PPM: gather and output overlap the next iteration (side stream)
        overlapped = (["ppm_gather", "ppm_direct_output"]
                      if getattr(sharded, "pipe", False) or (batch and getattr(r, "pipelined", lambda: False)()) else [])
        critical = {k: v for k, v in per_pass.items() if k not in overlapped} or per_pass
        dominant = max(critical, key=critical.get) if critical else None
        valid_avg = st.valid_photons_total / n_it
        rows0 = H if batch else local_rows(H, 0, world)
        if batch:  # rank 0's passes are the single-device passes
            pb = roofline.pass_bytes(mcode, W, H, P * P, valid_avg, st.num_cells,
                                     **({"light_vertices": int(np.minimum(r.read_buffer(
                                         _abi.BUF_VCM_VERTEX_COUNT, np.uint32), 9).sum())} if vcm else {}))
        elif pt:
            pb = roofline.pass_bytes(mcode, W, rows0, 0)
        elif vcm:  # rank 0 traces its own rows' subpaths; light vertices counted in the stats
            lv = int(np.minimum(r.read_buffer(_abi.BUF_VCM_VERTEX_COUNT, np.uint32), 9).sum())
            pb = roofline.pass_bytes(mcode, W, rows0, 0, light_vertices=lv)
        else:
            # rank 0's passes: its own photon rows, its pixel rows (eye/direct), all pixels (gather)
            pb = roofline.pass_bytes(mcode, W, H, P * local_rows(PH, 0, world), valid_avg, st.num_cells)
            for k in ("ppm_eye", "ppm_direct_output"):
                pb[k] = pb[k] * rows0 / H
        roof = roofline.roofline(dominant, pb[dominant], per_pass[dominant], None) if dominant else None
        out = {
            "metric": metric, "value": round(paths * args.steps / t_max / 1e6, 3), "unit": "Mpaths/s",
            "n_gpus": world_size, "world_size": world_size, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t_max * 1e3 / args.steps, 4), "higher_is_better": True,
            "scaling": "weak" if (batch or (weak and not (vcm or pt))) else "strong",
            "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic: seeded procedural scene ({scene.name}), XORWOW streams seeded 1645301512",
            "config": ({"workload": (f"{scene.name} {W}x{H} {_METHOD[mcode]}"
                                     + (f", {P * P:,} photons/iter" if not (vcm or pt) else "")
                                     + f" per GPU, photon-batch partition: each of {world} GPUs renders its own "
                                       "iterations (weak scaling)"),
                        "baseline_config": getattr(args, "config", None),
                        "hw_queues": {"used": os.environ.get("GPU_MAX_HW_QUEUES"),
                                      "inherited": os.environ.get("ORX_INHERITED_HW_QUEUES")},
                        "scene": scene.name, "width": W, "height": H, "method": _METHOD[mcode],
                        "photons_per_iteration": 0 if (vcm or pt) else P * P,
                        "paths_per_iteration": paths,
                        "parallelism": f"photon-batch (iteration) partition x{world}: global iterations dealt "
                                       f"round-robin, per-rank RNG streams, RCCL reduce of the accumulated radiance "
                                       f"every {sharded.reduce_every} iterations and at the end"}
                       if batch else
                       {"workload": f"{scene.name} {W}x{H} PT, 1 spp/iter (strong scaling)",
                        "scene": scene.name, "width": W, "height": H, "method": "PT",
                        "paths_per_iteration": paths,
                        "parallelism": f"row-interleaved RNG/pixel ownership x{world}, no per-iteration exchange"}
                       if pt else
                       {"workload": f"{scene.name} {W}x{H} VCM, {W * H} light subpaths/iter (strong scaling)",
                        "scene": scene.name, "width": W, "height": H, "method": "VCM",
                        "paths_per_iteration": paths,
                        "parallelism": f"row-interleaved RNG/pixel ownership x{world}, "
                                       "RCCL reduce_scatter(light-tracing splats)"} if vcm else
                       {"workload": (f"{scene.name} {W}x{H} PPM, {P * P:,} photons/iter per GPU (weak scaling)" if weak
                                     else f"{scene.name} {W}x{H} PPM, {P * PH:,} photons/iter total (strong scaling)"),
                        "baseline_config": getattr(args, "config", None),
                        "hw_queues": {"used": os.environ.get("GPU_MAX_HW_QUEUES"),
                                      "inherited": os.environ.get("ORX_INHERITED_HW_QUEUES")},
                        "scene": scene.name, "width": W, "height": H, "photons_per_iteration": P * PH,
                        "paths_per_iteration": paths,
                        "parallelism": (f"row-interleaved RNG/pixel/photon ownership x{world}; "
                                        + ("spatial photon slabs: RCCL all_gather(hitpoints, histograms) + "
                                           "all_to_all(photons) + reduce_scatter(indirect)"
                                           if getattr(sharded, "slab", False) else
                                           "RCCL all_gather(hitpoints) + reduce_scatter(indirect)"))}),
            "roofline": roof,
            "passes": {k: round(v, 4) for k, v in per_pass.items()},
            "dominant_pass": dominant,
            "overlapped_passes": overlapped,
        }
        if not on_gpu:
            out["backend"] = f"{backend_name} (launcher test, not a measurement)"
        if cpu_baseline is not None and world == 1:  # the oracle on the host cores, N = 1 only
            try:
                out["cpu_baseline"] = cpu_baseline(scene, mcode, W, H, P, getattr(args, "cpu_seconds", 20.0))
            except Exception as e:  # the baseline must never hide the GPU line
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), file=json_out, flush=True)
    if hasattr(r, "destroy"):
        r.destroy()
    elif hasattr(r, "close"):
        r.close()
    dist.barrier()
    dist.destroy_process_group()
