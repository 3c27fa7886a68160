/*
 * orx_kdtree.hip — kd-tree photon map (orx_config.photon_map = 2), gfx950.
 *
 * The reference's ACCELERATION_STRUCTURE_KD_TREE_CPU maps the photon buffer to
 * the host every iteration and builds a balanced kd-tree there
 * (createPhotonKdTreeOnCPU / buildKDTree, OptixRenderer_CPUKdTree.cpp:27-127,
 * quickselect from the OptiX SDK's select.h), then the gather walks it
 * (IndirectRadianceEstimation.cu:164-209).  Here the same tree is built on the
 * device, level by level, with no host round trip:
 *
 *   k_kd_vcount / k_kd_vwrite   valid slots (vmask) in slot order        -> ids
 *   k_kd_keys, k_rs_count, k_rs_scatter (x4 digits)  stable LSD radix sort of
 *                               the ids by each axis' coordinate         -> one list per axis
 *   k_kd_root                   root box = photon AABB (the photon pass's
 *                               fused bbox replicas), root segment [0, n)
 *   per level l:
 *     k_kd_nodes                node = its segment's median along the
 *                               box's longest axis (max_component), children
 *                               segments and boxes; NULL / LEAF nodes
 *     k_kd_pcount, scan, k_kd_pmove   stable partition of all three lists
 *                               into [left | median | right]
 *   k_kd_subtree                once segments hold <= KD_CAP photons: one
 *                               block per subtree, the same levels in LDS
 *
 * Each segment of every list stays sorted by its axis' (ordered key, slot), so
 * the median of a segment is read directly at (start+end)/2, and an element's
 * side follows from comparing its own (key, slot) on the split axis with the
 * median's: list entries carry the photon position and slot (16 B), so the
 * partition passes stream the lists with no random reads.  The tree's shape,
 * axes and split coordinates depend only on the photon multiset, so they equal
 * the reference's; which of several photons with the same split coordinate
 * becomes the node is the one freedom (select.h breaks such ties by its
 * partition order), and it only permutes the gather's summation.
 *
 * Node record: three float4 — A pos.xyz | axis bits, B power.xyz | dir.x,
 * C dir.yz — so the traversal loads 16 B per node and the rest only for
 * photons inside the radius.
 */
#include <cfloat>

#include "orx_kernels.h"

namespace orx {

constexpr uint32_t KD_NONE = 0xffffffffu;
constexpr uint32_t KD_PPM_X = 1u, KD_PPM_Y = 2u, KD_PPM_Z = 4u, KD_PPM_LEAF = 8u, KD_PPM_NULL = 16u; /* config.h:12-16 */
static_assert(KD_PPM_Z == KD_PPM_X << 2, "split flags are PPM_X << axis");

__device__ __forceinline__ uint32_t kd_f2ord(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kd_ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ float kd_comp(const float4& p, uint32_t a) { return a == 0 ? p.x : a == 1 ? p.y : p.z; }

/* node record: A plane pos.xyz | axis bits (all the traversal reads), BC plane power.xyz | dir.x,
 * dir.yz (read for photons within the radius) */
__device__ __forceinline__ void kd_put_node(const PhotonBufs& pb, const KdBufs& kd, size_t node, uint32_t flag,
                                            uint32_t slot) {
    const float4* sl = pb.slots + 4 * (size_t)slot;
    const float4 a = sl[0], b = sl[1], c = sl[2];
    kd.tree[node] = make_float4(a.x, a.y, a.z, __uint_as_float(flag));
    kd.tree_bc[2 * node] = make_float4(a.w, b.w, c.x, b.x);
    kd.tree_bc[2 * node + 1] = make_float4(b.y, b.z, 0.f, 0.f);
}
/* NULL node: buildKDTree writes axis and power only (OptixRenderer_CPUKdTree.cpp:31-34) */
__device__ __forceinline__ void kd_put_null(const KdBufs& kd, size_t node) {
    kd.tree[node].w = __uint_as_float(KD_PPM_NULL);
    const float4 b = kd.tree_bc[2 * node];
    kd.tree_bc[2 * node] = make_float4(0.f, 0.f, 0.f, b.w);
}

/* exclusive scan of one uint32 per thread over a 256-thread block (4 waves) */
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* lds4, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) lds4[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t t = lds4[k];
        if (k < w) base += t;
        tot += t;
    }
    __syncthreads();
    if (total) *total = tot;
    return base + inc - v;
}

/* ------------------------------------------------------------------ */
/* generic exclusive scan of m uint32 (in place): block sums, one-block */
/* scan of the sums, apply                                              */
/* ------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_kd_scan_reduce(const uint32_t* a, uint32_t m, uint32_t* part) {
    __shared__ uint32_t l4[4];
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x * 4;
    uint32_t s = 0;
    for (int k = 0; k < 4; k++)
        if (base + k < m) s += a[base + k];
    uint32_t tot;
    block_excl_scan256(s, l4, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
__global__ __launch_bounds__(1024) void k_kd_scan_top(uint32_t* part, uint32_t np, uint32_t* grand) {
    __shared__ uint32_t wsum[16];
    const uint32_t chunk = (np + 1023) / 1024;
    const uint32_t b = threadIdx.x * chunk;
    uint32_t s = 0;
    for (uint32_t k = 0; k < chunk; k++)
        if (b + k < np) s += part[b + k];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t k = 0; k < 16; k++) {
        if (k < w) base += wsum[k];
        tot += wsum[k];
    }
    uint32_t run = base + inc - s;
    for (uint32_t k = 0; k < chunk; k++)
        if (b + k < np) {
            const uint32_t t = part[b + k];
            part[b + k] = run;
            run += t;
        }
    if (threadIdx.x == 0 && grand) *grand = tot;
}
__global__ __launch_bounds__(256) void k_kd_scan_apply(uint32_t* a, uint32_t m, const uint32_t* part) {
    __shared__ uint32_t l4[4];
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x * 4;
    uint32_t v[4], s = 0;
    for (int k = 0; k < 4; k++) {
        v[k] = base + k < m ? a[base + k] : 0u;
        s += v[k];
    }
    uint32_t run = part[blockIdx.x] + block_excl_scan256(s, l4, nullptr);
    for (int k = 0; k < 4; k++)
        if (base + k < m) {
            a[base + k] = run;
            run += v[k];
        }
}
static void kd_scan(hipStream_t st, uint32_t* a, uint32_t m, uint32_t* part, uint32_t* grand) {
    const uint32_t nb = (m + 1023) / 1024;
    hipLaunchKernelGGL(k_kd_scan_reduce, dim3(nb), dim3(256), 0, st, a, m, part);
    hipLaunchKernelGGL(k_kd_scan_top, dim3(1), dim3(1024), 0, st, part, nb, grand);
    hipLaunchKernelGGL(k_kd_scan_apply, dim3(nb), dim3(256), 0, st, a, m, part);
}

/* ------------------------------------------------------------------ */
/* valid photons in slot order (the reference's numValidPhotons loop,  */
/* OptixRenderer_CPUKdTree.cpp:98-110, keeps the same set)             */
/* ------------------------------------------------------------------ */
__device__ __forceinline__ bool kd_slot_valid(const PhotonBufs& pb, uint32_t s) {
    return s < pb.S && ((pb.vmask[s / pb.D] >> (s % pb.D)) & 1u);
}
__global__ __launch_bounds__(256) void k_kd_vcount(PhotonBufs pb, KdBufs kd) {
    __shared__ uint32_t l4[4];
    const uint32_t base = blockIdx.x * 1024 + threadIdx.x * 4;
    uint32_t s = 0;
    for (int k = 0; k < 4; k++) s += kd_slot_valid(pb, base + k) ? 1u : 0u;
    uint32_t tot;
    block_excl_scan256(s, l4, &tot);
    if (threadIdx.x == 0) kd.vpart[blockIdx.x] = tot;
}
__global__ __launch_bounds__(256) void k_kd_vwrite(PhotonBufs pb, KdBufs kd) {
    __shared__ uint32_t l4[4];
    const uint32_t base = blockIdx.x * 1024 + threadIdx.x * 4;
    bool v[4];
    uint32_t s = 0;
    for (int k = 0; k < 4; k++) {
        v[k] = kd_slot_valid(pb, base + k);
        s += v[k] ? 1u : 0u;
    }
    uint32_t run = kd.vpart[blockIdx.x] + block_excl_scan256(s, l4, nullptr);
    for (int k = 0; k < 4; k++)
        if (v[k]) kd.ids[1][0][run++] = base + k;
}

/* ------------------------------------------------------------------ */
/* stable LSD radix sort of (key, slot) by 8-bit digits                */
/* ------------------------------------------------------------------ */
constexpr uint32_t RS_ITEMS = 16, RS_TILE = 256 * RS_ITEMS;

__global__ __launch_bounds__(256) void k_kd_keys(PhotonBufs pb, KdBufs kd, uint32_t axis) {
    const uint32_t n = kd.count[0];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = kd.ids[1][0][i];
    kd.keys[0][i] = kd_f2ord(kd_comp(pb.pos4[s], axis));
    kd.ids[0][axis][i] = s;
}
/* sorted slots -> list records (position, slot) */
__global__ __launch_bounds__(256) void k_kd_lists(PhotonBufs pb, KdBufs kd, uint32_t axis) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= kd.count[0]) return;
    const uint32_t s = kd.ids[0][axis][i];
    const float4 a = pb.pos4[s];
    kd.lst[0][axis][i] = make_float4(a.x, a.y, a.z, __uint_as_float(s));
}
/* histogram of one digit per tile -> table[digit][tile] */
__global__ __launch_bounds__(256) void k_rs_count(const uint32_t* keys, const uint32_t* count, uint32_t shift,
                                                  uint32_t* table, uint32_t ntiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t n = *count;
    const uint32_t t0 = blockIdx.x * RS_TILE;
    for (uint32_t j = 0; j < RS_ITEMS; j++) {
        const uint32_t i = t0 + j * 256 + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    table[threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}
/* stable scatter: within a tile, element order = (round j, thread); ranks of equal
 * digits inside a wave from eight ballots, across waves from LDS counts */
__global__ __launch_bounds__(256) void k_rs_scatter(const uint32_t* keys, const uint32_t* vals, const uint32_t* count,
                                                    uint32_t shift, const uint32_t* table, uint32_t ntiles,
                                                    uint32_t* okeys, uint32_t* ovals) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wc[4][256];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    run[tid] = table[tid * ntiles + blockIdx.x];
    const uint32_t n = *count;
    const uint32_t t0 = blockIdx.x * RS_TILE;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t j = 0; j < RS_ITEMS; j++) {
        if (t0 + j * 256 >= n) break; /* uniform across the block */
        wc[0][tid] = 0;
        wc[1][tid] = 0;
        wc[2][tid] = 0;
        wc[3][tid] = 0;
        const uint32_t i = t0 + j * 256 + tid;
        const bool ok = i < n;
        const uint32_t key = ok ? keys[i] : 0u;
        const uint32_t val = ok ? vals[i] : 0u;
        const uint32_t d = (key >> shift) & 255u;
        uint64_t peers = __ballot(ok);
        for (int b = 0; b < 8; b++) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        __syncthreads(); /* wc zeroed */
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (ok && rank == 0) wc[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (ok) {
            uint32_t off = run[d] + rank;
            for (uint32_t k = 0; k < w; k++) off += wc[k][d];
            okeys[off] = key;
            ovals[off] = val;
        }
        __syncthreads();
        run[tid] += wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
        __syncthreads();
    }
}

/* ------------------------------------------------------------------ */
/* root: the photon AABB (fminf/fmaxf over valid positions,            */
/* OptixRenderer_CPUKdTree.cpp:112-124) from the photon pass's fused   */
/* replicas, which are reset for the next iteration                    */
/* ------------------------------------------------------------------ */
__global__ void k_kd_root(PhotonBufs pb, KdBufs kd) {
    __shared__ uint32_t red[6];
    const uint32_t lane = threadIdx.x;
    for (int k = 0; k < 6; k++) {
        uint32_t v = pb.bbox[k * BBOX_REPLICAS + lane];
        for (int o = 32; o > 0; o >>= 1) {
            uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
            v = k < 3 ? min(v, w) : max(v, w);
        }
        if (lane == 0) red[k] = v;
        pb.bbox[k * BBOX_REPLICAS + lane] = k < 3 ? 0xffffffffu : 0u;
    }
    __syncthreads();
    if (lane != 0) return;
    const uint32_t n = kd.count[0];
    for (int k = 0; k < 3; k++) {
        kd.box[k] = n ? kd_ord2f(red[k]) : FLT_MAX;
        kd.box[3 + k] = n ? kd_ord2f(red[3 + k]) : -FLT_MAX;
    }
    kd.seg[0] = make_uint2(0u, n);
    GridParams* g = pb.grid;
    g->ox = g->oy = g->oz = 0.f;
    g->cell = 0.f;
    g->gx = g->gy = g->gz = 0;
    g->G = kd.tree_size;
    g->valid = n;
    g->error = 0;
    g->any_valid = n ? 1u : 0u;
    g->photons_visited = 0;
    g->cells_visited = 0;
    g->valid_total += n;
}

/* ------------------------------------------------------------------ */
/* levels                                                              */
/* ------------------------------------------------------------------ */
/* one thread per node of level l: buildKDTree's body (OptixRenderer_CPUKdTree.cpp:27-88) */
__global__ __launch_bounds__(256) void k_kd_nodes(PhotonBufs pb, KdBufs kd, uint32_t level, uint32_t src) {
    const uint32_t first = (1u << level) - 1u;
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= (1u << level)) return;
    const uint32_t node = first + k;
    const uint2 se = kd.seg[node];
    const uint32_t c0 = 2 * node + 1;
    const bool has_children = c0 + 1 < kd.tree_size;
    uint32_t info = KD_NONE;
    if (se.x != KD_NONE) {
        const uint32_t size = se.y - se.x;
        if (size == 0) { /* NULL node: axis and power */
            kd_put_null(kd, node);
        } else {
            uint32_t axis = 0, med = se.x;
            if (size > 1) {
                const float* bx = kd.box + 6 * (size_t)node;
                const float dx = bx[3] - bx[0], dy = bx[4] - bx[1], dz = bx[5] - bx[2];
                axis = (dx > dy && dx > dz) ? 0u : (dy > dz ? 1u : 2u); /* max_component :14-25 */
                med = (se.x + se.y) / 2;
            }
            const float4 e = kd.lst[src][axis][med];
            const uint32_t s = __float_as_uint(e.w);
            kd_put_node(pb, kd, node, size == 1 ? KD_PPM_LEAF : (KD_PPM_X << axis), s);
            const float4 a = pb.pos4[s];
            if (size > 1) {
                info = (med << 2) | axis;
                kd.nkey[node] = make_uint2(kd_f2ord(kd_comp(e, axis)), s);
                if (has_children) {
                    const float* bx = kd.box + 6 * (size_t)node;
                    const float split = kd_comp(make_float4(a.x, a.y, a.z, 0.f), axis);
                    float* lb = kd.box + 6 * (size_t)c0;
                    float* rb = lb + 6;
                    for (int q = 0; q < 6; q++) {
                        lb[q] = bx[q];
                        rb[q] = bx[q];
                    }
                    lb[3 + axis] = split; /* leftMax */
                    rb[axis] = split;     /* rightMin */
                    kd.seg[c0] = make_uint2(se.x, med);
                    kd.seg[c0 + 1] = make_uint2(med + 1, se.y);
                }
            }
        }
    }
    kd.ninfo[node] = info;
    if (info == KD_NONE && has_children) {
        kd.seg[c0] = make_uint2(KD_NONE, KD_NONE);
        kd.seg[c0 + 1] = make_uint2(KD_NONE, KD_NONE);
    }
}

/* side of a list element in its split segment: (key, slot) on the split axis against the median's */
__device__ __forceinline__ uint32_t kd_side(const float4& e, uint32_t axis, uint2 mk) {
    const uint32_t k = kd_f2ord(kd_comp(e, axis)), sl = __float_as_uint(e.w);
    if (k != mk.x) return k < mk.x ? 0u : 1u;
    if (sl != mk.y) return sl < mk.y ? 0u : 1u;
    return 2u;
}
/* per position: (left, median) indicators of the three lists, packed left | median << 16 */
__device__ __forceinline__ void kd_pos_bits(const KdBufs& kd, uint32_t src, uint32_t p, uint32_t n, uint32_t v[3]) {
    v[0] = v[1] = v[2] = 0;
    if (p >= n) return;
    const uint32_t node = kd.nodepos[p];
    if (node == KD_NONE) return;
    const uint32_t info = kd.ninfo[node];
    if (info == KD_NONE) return;
    const uint2 mk = kd.nkey[node];
    for (int b = 0; b < 3; b++) {
        const uint32_t sd = kd_side(kd.lst[src][b][p], info & 3u, mk);
        v[b] = sd == 0 ? 1u : (sd == 2 ? 0x10000u : 0u);
    }
}
/* Positions go 1024 per block in four coalesced rounds of 256 (position = block*1024 +
 * round*256 + thread).  Pass 1 (k_kd_pcount): per block and list the left and median counts ->
 * ppart, and for every segment that starts in the block the in-block exclusive prefix at its
 * start -> nodeP.  After the scan of ppart, pass 2 (k_kd_pmove) recomputes the in-block prefix of
 * each position, so the count of left (median) elements before position p within its segment
 * [s, e) is  ppart[blk(p)] + inblock(p) - ppart[blk(s)] - nodeP. */
__global__ __launch_bounds__(256) void k_kd_pcount(KdBufs kd, uint32_t src, uint32_t nblk) {
    __shared__ uint32_t l4[4];
    const uint32_t n = kd.count[0];
    uint32_t carry[3] = {0, 0, 0};
    for (int k = 0; k < 4; k++) {
        const uint32_t p = blockIdx.x * 1024 + k * 256 + threadIdx.x;
        uint32_t v[3];
        kd_pos_bits(kd, src, p, n, v);
        uint32_t ex[3];
        for (int b = 0; b < 3; b++) {
            uint32_t tot;
            ex[b] = carry[b] + block_excl_scan256(v[b], l4, &tot);
            carry[b] += tot;
        }
        if (p < n) {
            const uint32_t node = kd.nodepos[p];
            if (node != KD_NONE && kd.ninfo[node] != KD_NONE && kd.seg[node].x == p)
                for (int b = 0; b < 3; b++) kd.nodeP[3 * (size_t)node + b] = ex[b];
        }
    }
    if (threadIdx.x == 0)
        for (int b = 0; b < 3; b++) {
            kd.ppart[(2 * b) * nblk + blockIdx.x] = carry[b] & 0xffffu;
            kd.ppart[(2 * b + 1) * nblk + blockIdx.x] = carry[b] >> 16;
        }
}
/* stable partition of the three lists of every split segment into [left | median | right]
 * (the median leaves the lists: it is the node), and the positions' next-level nodes */
__global__ __launch_bounds__(256) void k_kd_pmove(KdBufs kd, uint32_t src, uint32_t nblk) {
    __shared__ uint32_t l4[4];
    const uint32_t n = kd.count[0];
    uint32_t carry[3] = {0, 0, 0};
    for (int k = 0; k < 4; k++) {
        const uint32_t p = blockIdx.x * 1024 + k * 256 + threadIdx.x;
        uint32_t v[3];
        kd_pos_bits(kd, src, p, n, v);
        uint32_t ex[3];
        for (int b = 0; b < 3; b++) {
            uint32_t tot;
            ex[b] = carry[b] + block_excl_scan256(v[b], l4, &tot);
            carry[b] += tot;
        }
        if (p >= n) continue;
        const uint32_t node = kd.nodepos[p];
        if (node == KD_NONE) continue;
        const uint32_t info = kd.ninfo[node];
        if (info == KD_NONE) { /* a leaf: its element is the node */
            kd.nodepos[p] = KD_NONE;
            continue;
        }
        const uint32_t m = info >> 2;
        const uint32_t s = kd.seg[node].x;
        const uint32_t sblk = s / 1024;
        for (int b = 0; b < 3; b++) {
            if (v[b] & 0x10000u) continue; /* the median */
            const uint32_t np = kd.nodeP[3 * (size_t)node + b];
            const uint32_t L = kd.ppart[(2 * b) * nblk + blockIdx.x] + (ex[b] & 0xffffu) -
                               kd.ppart[(2 * b) * nblk + sblk] - (np & 0xffffu);
            const uint32_t M = kd.ppart[(2 * b + 1) * nblk + blockIdx.x] + (ex[b] >> 16) -
                               kd.ppart[(2 * b + 1) * nblk + sblk] - (np >> 16);
            const uint32_t dst = (v[b] & 1u) ? s + L : m + 1 + (p - s) - L - M;
            kd.lst[src ^ 1][b][dst] = kd.lst[src][b][p];
        }
        kd.nodepos[p] = p < m ? 2 * node + 1 : (p > m ? 2 * node + 2 : KD_NONE);
    }
}
__global__ __launch_bounds__(256) void k_kd_pos_init(KdBufs kd) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p < kd.S) kd.nodepos[p] = p < kd.count[0] ? 0u : KD_NONE;
}

/* ------------------------------------------------------------------ */
/* subtrees of at most KD_CAP photons, one block each, entirely in LDS  */
/* ------------------------------------------------------------------ */
/* Once every segment of a level holds at most KD_CAP photons, one 256-thread block takes a
 * segment and builds its whole subtree: the same per-level median / stable three-list partition
 * as the global levels, on 16-bit indices into an LDS copy of the segment's list records. */
constexpr uint32_t KD_CAP = 512;
constexpr uint32_t KD_HASH = 1024;
constexpr uint16_t KD_NONE16 = 0xffffu;


__global__ __launch_bounds__(256) void k_kd_subtree(PhotonBufs pb, KdBufs kd, uint32_t level0, uint32_t src) {
    __shared__ float4 E[KD_CAP];
    __shared__ uint16_t L[2][3][KD_CAP];
    __shared__ uint32_t Pp[3][KD_CAP];          /* exclusive (left | median << 16) prefix per list */
    __shared__ uint16_t pnode[KD_CAP];          /* node (offset within its level) of each position */
    __shared__ uint32_t hkey[KD_HASH];
    __shared__ uint16_t hval[KD_HASH];
    __shared__ uint16_t cs[2][KD_CAP], ce[2][KD_CAP]; /* segments of the current / next level */
    __shared__ float cb[2][KD_CAP / 2][6];            /* boxes of split candidates (size >= 2) */
    __shared__ uint32_t sinfo[KD_CAP / 2][3];         /* split nodes: m | axis << 16, median key, median slot */
    __shared__ uint32_t l4[4];
    __shared__ uint32_t any_split;
    const uint32_t tid = threadIdx.x;
    const size_t root = ((size_t)1 << level0) - 1 + blockIdx.x;
    const uint2 se = kd.seg[root];
    if (se.x == KD_NONE) return; /* uniform */
    const uint32_t n0 = se.y - se.x;
    for (uint32_t h = tid; h < KD_HASH; h += 256) hkey[h] = KD_NONE;
    __syncthreads();
    for (uint32_t i = tid; i < n0; i += 256) {
        const float4 e = kd.lst[src][0][se.x + i];
        E[i] = e;
        L[0][0][i] = (uint16_t)i;
        uint32_t h = (__float_as_uint(e.w) * 2654435761u) >> 22;
        while (atomicCAS(&hkey[h], KD_NONE, __float_as_uint(e.w)) != KD_NONE) h = (h + 1) & (KD_HASH - 1);
        hval[h] = (uint16_t)i;
        pnode[i] = 0;
    }
    __syncthreads();
    for (uint32_t i = tid; i < n0; i += 256)
        for (int b = 1; b < 3; b++) {
            const uint32_t sl = __float_as_uint(kd.lst[src][b][se.x + i].w);
            uint32_t h = (sl * 2654435761u) >> 22;
            while (hkey[h] != sl) h = (h + 1) & (KD_HASH - 1);
            L[0][b][i] = hval[h];
        }
    if (tid == 0) {
        cs[0][0] = 0;
        ce[0][0] = (uint16_t)n0;
        for (int q = 0; q < 6; q++) cb[0][0][q] = kd.box[6 * root + q];
    }
    __syncthreads();
    uint32_t cur = 0, lv = 0;
    for (uint32_t d = 0;; d++) {
        /* nodes of depth d below the subtree root: buildKDTree's body */
        const uint32_t count = 1u << d;
        const size_t first = (root + 1) * ((size_t)1 << d) - 1;
        if (tid == 0) any_split = 0;
        __syncthreads();
        for (uint32_t k = tid; k < count && k < KD_CAP; k += 256) {
            const uint32_t s = cs[lv][k], e = ce[lv][k];
            const size_t node = first + k;
            const size_t c0 = 2 * node + 1;
            const bool has_children = c0 + 1 < kd.tree_size && 2 * k + 1 < KD_CAP;
            bool split = false;
            if (s != KD_NONE16) {
                const uint32_t size = e - s;
                if (size == 0) {
                    kd_put_null(kd, node);
                } else if (size == 1) {
                    kd_put_node(pb, kd, node, KD_PPM_LEAF, __float_as_uint(E[L[cur][0][s]].w));
                } else {
                    split = true; /* only depths <= 8 hold such nodes: k < KD_CAP / 2 */
                }
            }
            if (split) {
                const float* bx = cb[lv][k];
                const float dx = bx[3] - bx[0], dy = bx[4] - bx[1], dz = bx[5] - bx[2];
                const uint32_t axis = (dx > dy && dx > dz) ? 0u : (dy > dz ? 1u : 2u); /* max_component */
                const uint32_t m = (s + e) / 2;
                const float4 med = E[L[cur][axis][m]];
                const uint32_t slot = __float_as_uint(med.w);
                kd_put_node(pb, kd, node, KD_PPM_X << axis, slot);
                sinfo[k][0] = m | (axis << 16);
                sinfo[k][1] = kd_f2ord(kd_comp(med, axis));
                sinfo[k][2] = slot;
                any_split = 1;
                if (has_children) {
                    const float split_v = kd_comp(med, axis);
                    const uint32_t nl = lv ^ 1u;
                    cs[nl][2 * k] = (uint16_t)s;
                    ce[nl][2 * k] = (uint16_t)m;
                    cs[nl][2 * k + 1] = (uint16_t)(m + 1);
                    ce[nl][2 * k + 1] = (uint16_t)e;
                    /* children with >= 2 photons split again: hand down the cut boxes */
                    if (m - s >= 2 && 2 * k < KD_CAP / 2)
                        for (int q = 0; q < 6; q++) cb[nl][2 * k][q] = q == 3 + (int)axis ? split_v : bx[q];
                    if (e - m - 1 >= 2 && 2 * k + 1 < KD_CAP / 2)
                        for (int q = 0; q < 6; q++) cb[nl][2 * k + 1][q] = q == (int)axis ? split_v : bx[q];
                }
            } else if (2 * k + 1 < KD_CAP) {
                cs[lv ^ 1u][2 * k] = KD_NONE16;
                cs[lv ^ 1u][2 * k + 1] = KD_NONE16;
            }
        }
        __syncthreads();
        if (!any_split) break; /* uniform */
        /* stable partition of the three lists around each split node's median */
        const uint32_t p0 = 2 * tid, p1 = 2 * tid + 1;
        uint32_t v[2][3];
        for (int q = 0; q < 2; q++) {
            const uint32_t p = q ? p1 : p0;
            v[q][0] = v[q][1] = v[q][2] = 0;
            if (p < n0 && pnode[p] != KD_NONE16 && cs[lv][pnode[p]] != KD_NONE16 &&
                ce[lv][pnode[p]] - cs[lv][pnode[p]] >= 2) {
                const uint32_t k = pnode[p];
                const uint32_t axis = sinfo[k][0] >> 16;
                const uint2 mk = make_uint2(sinfo[k][1], sinfo[k][2]);
                for (int b = 0; b < 3; b++) {
                    const uint32_t sd = kd_side(E[L[cur][b][p]], axis, mk);
                    v[q][b] = sd == 0 ? 1u : (sd == 2 ? 0x10000u : 0u);
                }
            }
        }
        for (int b = 0; b < 3; b++) {
            const uint32_t ex = block_excl_scan256(v[0][b] + v[1][b], l4, nullptr);
            if (p0 < n0) Pp[b][p0] = ex;
            if (p1 < n0) Pp[b][p1] = ex + v[0][b];
        }
        __syncthreads();
        for (int q = 0; q < 2; q++) {
            const uint32_t p = q ? p1 : p0;
            if (p >= n0 || pnode[p] == KD_NONE16) continue;
            const uint32_t k = pnode[p];
            const uint32_t s = cs[lv][k], e = ce[lv][k];
            if (s == KD_NONE16 || e - s < 2) { /* a leaf: its element is the node */
                pnode[p] = KD_NONE16;
                continue;
            }
            const uint32_t m = sinfo[k][0] & 0xffffu;
            for (int b = 0; b < 3; b++) {
                if (v[q][b] & 0x10000u) continue; /* the median */
                const uint32_t Lc = (Pp[b][p] & 0xffffu) - (Pp[b][s] & 0xffffu);
                const uint32_t Mc = (Pp[b][p] >> 16) - (Pp[b][s] >> 16);
                const uint32_t dst = (v[q][b] & 1u) ? s + Lc : m + 1 + (p - s) - Lc - Mc;
                L[cur ^ 1u][b][dst] = L[cur][b][p];
            }
            pnode[p] = p < m ? (uint16_t)(2 * k) : (p > m ? (uint16_t)(2 * k + 1) : KD_NONE16);
        }
        __syncthreads();
        cur ^= 1u;
        lv ^= 1u;
    }
}

void launch_kd_build(hipStream_t st, const PhotonBufs& pb, const KdBufs& kd) {
    const uint32_t S = kd.S;
    const uint32_t nb1024 = (S + 1023) / 1024;
    const uint32_t nb256 = (S + 255) / 256;
    /* valid slots in slot order -> ids[1][0], count[0] = n */
    hipLaunchKernelGGL(k_kd_vcount, dim3(nb1024), dim3(256), 0, st, pb, kd);
    hipLaunchKernelGGL(k_kd_scan_top, dim3(1), dim3(1024), 0, st, kd.vpart, nb1024, kd.count);
    hipLaunchKernelGGL(k_kd_vwrite, dim3(nb1024), dim3(256), 0, st, pb, kd);
    /* one stably sorted list per axis -> ids[0][axis] */
    for (uint32_t axis = 0; axis < 3; axis++) {
        hipLaunchKernelGGL(k_kd_keys, dim3(nb256), dim3(256), 0, st, pb, kd, axis);
        uint32_t* k0 = kd.keys[0];
        uint32_t* k1 = kd.keys[1];
        uint32_t* v0 = kd.ids[0][axis];
        uint32_t* v1 = kd.ids[1][1]; /* scratch list during the sorts */
        for (uint32_t pass = 0; pass < 4; pass++) {
            hipLaunchKernelGGL(k_rs_count, dim3(kd.ntiles), dim3(256), 0, st, k0, kd.count, 8 * pass, kd.table,
                               kd.ntiles);
            kd_scan(st, kd.table, 256 * kd.ntiles, kd.tpart, nullptr);
            hipLaunchKernelGGL(k_rs_scatter, dim3(kd.ntiles), dim3(256), 0, st, k0, v0, kd.count, 8 * pass, kd.table,
                               kd.ntiles, k1, v1);
            std::swap(k0, k1);
            std::swap(v0, v1);
        }
        /* four passes: the result is back in (keys[0], ids[0][axis]) */
        hipLaunchKernelGGL(k_kd_lists, dim3(nb256), dim3(256), 0, st, pb, kd, axis);
    }
    hipLaunchKernelGGL(k_kd_root, dim3(1), dim3(64), 0, st, pb, kd);
    hipLaunchKernelGGL(k_kd_pos_init, dim3(nb256), dim3(256), 0, st, kd);
    const uint32_t nblk = nb1024;
    /* global levels until every segment holds at most KD_CAP photons (a level-l segment holds at
     * most floor(n / 2^l) <= S >> l), then one LDS block per subtree */
    uint32_t lg = 0;
    while ((S >> lg) > KD_CAP) lg++;
    uint32_t src = 0;
    for (uint32_t level = 0; level < kd.levels; level++) {
        const uint32_t nodes = 1u << level;
        if (level == lg) {
            hipLaunchKernelGGL(k_kd_subtree, dim3(nodes), dim3(256), 0, st, pb, kd, level, src);
            break;
        }
        hipLaunchKernelGGL(k_kd_nodes, dim3((nodes + 255) / 256), dim3(256), 0, st, pb, kd, level, src);
        if (level + 1 == kd.levels) break; /* the last level holds leaves and NULL nodes only */
        hipLaunchKernelGGL(k_kd_pcount, dim3(nblk), dim3(256), 0, st, kd, src, nblk);
        kd_scan(st, kd.ppart, 6 * nblk, kd.tpart, nullptr);
        hipLaunchKernelGGL(k_kd_pmove, dim3(nblk), dim3(256), 0, st, kd, src, nblk);
        src ^= 1;
    }
}

/* ------------------------------------------------------------------ */
/* gather (IndirectRadianceEstimation.cu:164-209 + :211-221)           */
/* ------------------------------------------------------------------ */
/* The reference's stack walk (select.h / IndirectRadianceEstimation.cu:164-209), wave-cooperative:
 * the wave walks the union of its lanes' traversals once, with a
 * 64-bit mask of the lanes that visit each node.  A lane is active at a child iff it was active at
 * the parent and the child is its near child or the split plane lies within its radius — exactly
 * the reference's per-lane descend/push rule — so every lane visits, counts and accepts the same
 * nodes as a per-lane walk; only the order of its sum changes (children are taken left first).
 * Node loads are wave-uniform (one address per wave), the control flow is uniform (a per-lane
 * walk measured 12.9 ms against 8.3 on the hall, 4M photons). */
__global__ __launch_bounds__(64) void k_ppm_gather_kd_wave(GatherIn gi, PhotonBufs pb, KdBufs kd, Consts c) {
    extern __shared__ uint32_t kd_wstack[]; /* [entries][3]: node, mask lo, mask hi */
    const uint32_t lane = threadIdx.x;
    const uint32_t x = blockIdx.x * 8 + (lane & 7);
    const uint32_t y = blockIdx.y * 8 + (lane >> 3);
    const uint32_t j = gather_row(gi, y);
    const bool inimg = x < gi.W && y < gi.segments * gi.seg_rows;
    const size_t i = (size_t)j * gi.W + x;
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    float2 Cc = make_float2(0.f, 0.f);
    if (inimg) hp_load(gi, j, x, A, B, Cc);
    const uint32_t flags = __float_as_uint(A.w);
    const bool gathers = inimg && (flags & PRD_HIT_NON_SPECULAR);
    f3 acc = mk1(0.0f);
    uint32_t dP = 0;
    const f3 pos = mk(A.x, A.y, A.z), nrm = mk(B.x, B.y, B.z);
    const float radius2 = c.ppm_radius2;
    const float alpha = 1.818f, beta = 1.953f, expNegativeBeta = 0.141847f;
    const float inv2r2 = 1.0f / (2 * radius2);
    const float invDen = 1.0f / (1 - expNegativeBeta);
    uint64_t mask = __ballot(gathers);
    uint32_t node = 0, sc = 0;
    const uint32_t max_sc = kd.levels + 2;
    while (mask) {
        node = __builtin_amdgcn_readfirstlane(node);
        const float4 a = kd.tree[node];
        const bool act = (mask >> lane) & 1ull;
        const uint32_t axis = __float_as_uint(a.w);
        dP += act ? 1u : 0u;
        uint64_t lm = 0, rm = 0;
        if (!(axis & KD_PPM_NULL)) {
            const f3 diff = pos - mk(a.x, a.y, a.z);
            const float distance2 = dot(diff, diff);
            const bool in = act && distance2 <= radius2;
            if (__ballot(in)) {
                const float4 b = kd.tree_bc[2 * (size_t)node];
                const float4 cc = kd.tree_bc[2 * (size_t)node + 1];
                if (in && dot(-mk(b.w, cc.x, cc.y), nrm) >= 0) {
                    const float e = orx_expf_unit((-beta * distance2) * inv2r2);
                    const float wgt = alpha * (1 - (1 - e) * invDen);
                    acc = acc + mk(b.x, b.y, b.z) * wgt;
                }
            }
            if (!(axis & KD_PPM_LEAF)) {
                const float d = (axis & KD_PPM_X) ? diff.x : (axis & KD_PPM_Y) ? diff.y : diff.z;
                const bool near_left = d < 0.0f, cross = d * d < radius2;
                lm = __ballot(act && (near_left || cross));
                rm = __ballot(act && (!near_left || cross));
            }
        }
        if (lm) {
            if (rm && sc < max_sc) {
                if (lane == 0) {
                    kd_wstack[3 * sc] = 2 * node + 2;
                    kd_wstack[3 * sc + 1] = (uint32_t)rm;
                    kd_wstack[3 * sc + 2] = (uint32_t)(rm >> 32);
                }
                sc++;
            }
            node = 2 * node + 1;
            mask = lm;
        } else if (rm) {
            node = 2 * node + 2;
            mask = rm;
        } else if (sc) {
            sc--;
            node = kd_wstack[3 * sc];
            mask = (uint64_t)kd_wstack[3 * sc + 1] | ((uint64_t)kd_wstack[3 * sc + 2] << 32);
        } else {
            mask = 0;
        }
        if (node >= kd.tree_size) mask = 0; /* unreachable on a well-formed tree */
    }
    if (inimg) {
        const f3 att = mk(B.w, Cc.x, Cc.y);
        const float s1 = 1.0f / (ORX_PI_F * c.ppm_radius2);
        const float s2 = 1.0f / c.emitted_f;
        const f3 ind = ((acc * att) * s1) * s2;
        gi.indirect[3 * i + 0] = ind.x;
        gi.indirect[3 * i + 1] = ind.y;
        gi.indirect[3 * i + 2] = ind.z;
        if (gi.dbg) {
            gi.dbg[2 * i] = 0;
            gi.dbg[2 * i + 1] = gathers ? dP : 0u;
        }
    }
    uint64_t sp = gathers ? dP : 0u;
    for (int o = 32; o > 0; o >>= 1) sp += __shfl_xor(sp, o, 64);
    if (lane == 0 && sp) {
        atomicAdd((unsigned long long*)&pb.grid->photons_visited, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->photons_visited_total, (unsigned long long)sp);
    }
}
void launch_ppm_gather_kd(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const KdBufs& kd, const Consts& c) {
    const uint32_t rows = gi.segments * gi.seg_rows;
    dim3 grid((gi.W + 7) / 8, (rows + 7) / 8);
    hipLaunchKernelGGL(k_ppm_gather_kd_wave, grid, dim3(64), (size_t)(kd.levels + 2) * 12, s, gi, pb, kd, c);
}

} // namespace orx
