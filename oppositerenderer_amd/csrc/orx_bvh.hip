/*
 * orx_bvh.hip — on-device BVH build for the triangle meshes of orx_init_scene.
 *
 * The reference hands the meshes to OptiX's `Trbvh` builder (scene/Scene.cpp:353,
 * :513, :547), which runs on the GPU.  Here the build is a level-synchronous
 * binned-SAH construction followed by a collapse to the 64-byte quantised
 * four-wide nodes the traversal kernels read (DevBvh4, orx_device.h), all in
 * HIP kernels; the host only loops over tree levels (one small read-back of
 * the next level's size per level) and receives the leaf order of the
 * triangles to lay out their attribute arrays.
 *
 * Binary build (one 64-lane wave per node of the current level):
 *   bounds and centroid bounds of the node's primitives (wave reductions);
 *   32-bin SAH per axis, bins filled with LDS atomics (bounds as ordered ints);
 *   the same decisions as the host builder (BvhBuilder, orx_capi.hip): SAH leaf
 *   test up to leaf_max triangles, object-median fallback near the depth cap;
 *   stable partition of the node's range with ballots; children appended to
 *   the next level through two global counters (nodes, tasks).
 * Collapse (one lane per BVH4 node of the current level): open the
 * largest-area inner children until four, quantise the child boxes outward on
 * 8 bits per axis against the node origin, allocate the inner children's
 * slots; then a reverse pass over the levels computes the traversal-stack
 * bound (k - 1 pushes at a node with k children hit, plus the deepest child).
 *
 * Boxes are expanded by a relative 1e-6 exactly as the host builder does, so the
 * conservativeness argument of the traversal is unchanged; the closest hit
 * never depends on the tree (exact triangle tests + the lowest-id tie rule).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "orx_device.h"
#include "orx_kernels.h"

namespace orx {

struct BvhTask {
    uint32_t node, first, count, depth;
};

__device__ __forceinline__ uint32_t ford(float f) { /* order-preserving float -> uint */
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fdec(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ float wmin(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wmax(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float box_area(float lx, float ly, float lz, float hx, float hy, float hz) {
    const float dx = fmaxf(0.f, hx - lx), dy = fmaxf(0.f, hy - ly), dz = fmaxf(0.f, hz - lz);
    return dx * dy + dy * dz + dz * dx;
}

/* per-triangle box and centroid (BuildTri) from the original-order vertices */
__global__ void k_bvh_tris(const float* __restrict__ V, const uint32_t* __restrict__ I, uint32_t nt, float* tb) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int v = 0; v < 3; v++) {
        const float* p = V + 3 * (size_t)I[3 * (size_t)i + v];
        for (int k = 0; k < 3; k++) {
            lo[k] = fminf(lo[k], p[k]);
            hi[k] = fmaxf(hi[k], p[k]);
        }
    }
    for (int k = 0; k < 3; k++) {
        tb[(size_t)k * nt + i] = lo[k];
        tb[(size_t)(3 + k) * nt + i] = hi[k];
        tb[(size_t)(6 + k) * nt + i] = 0.5f * (lo[k] + hi[k]);
    }
}

struct BvhBuildBufs {
    const float* tb;       /* [9][nt]: lo xyz, hi xyz, centroid xyz */
    uint32_t nt;
    uint32_t* prims;       /* [nt] permutation (leaf order at the end) */
    uint32_t* tmp;         /* [nt] partition scratch */
    DevBvhNode* nodes;     /* binary nodes */
    uint32_t* ctl;         /* [0] node count, [1] next task count, [2] max depth, [3] error */
    int bins;
    uint32_t leaf_max;
    float leaf_sah;
};

constexpr int BVH_NB = 32;
constexpr int BVH_WAVES = 4; /* waves (tasks) per 256-thread block */

__global__ __launch_bounds__(256) void k_bvh_level(BvhBuildBufs B, const BvhTask* __restrict__ tasks, uint32_t ntasks,
                                                   BvhTask* __restrict__ next) {
    __shared__ uint32_t s_cnt[BVH_WAVES][3][BVH_NB];
    __shared__ uint32_t s_lo[BVH_WAVES][3][BVH_NB][3];
    __shared__ uint32_t s_hi[BVH_WAVES][3][BVH_NB][3];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t ti = blockIdx.x * BVH_WAVES + wv;
    if (ti >= ntasks) return; /* whole wave leaves: no block barrier below */
    const BvhTask T = tasks[ti];
    const uint32_t nt = B.nt;
    const float* tb = B.tb;
    /* bounds and centroid bounds */
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = lane; i < T.count; i += 64) {
        const uint32_t p = B.prims[T.first + i];
        for (int k = 0; k < 3; k++) {
            lo[k] = fminf(lo[k], tb[(size_t)k * nt + p]);
            hi[k] = fmaxf(hi[k], tb[(size_t)(3 + k) * nt + p]);
            const float c = tb[(size_t)(6 + k) * nt + p];
            clo[k] = fminf(clo[k], c);
            chi[k] = fmaxf(chi[k], c);
        }
    }
    for (int k = 0; k < 3; k++) {
        lo[k] = wmin(lo[k]);
        hi[k] = wmax(hi[k]);
        clo[k] = wmin(clo[k]);
        chi[k] = wmax(chi[k]);
    }
    DevBvhNode& N = B.nodes[T.node];
    if (lane == 0) {
        for (int k = 0; k < 3; k++) {
            const float m = fmaxf(fabsf(lo[k]), fabsf(hi[k]));
            const float e = m * 1e-6f + 1e-20f;
            N.lo[k] = lo[k] - e;
            N.hi[k] = hi[k] + e;
        }
        atomicMax(&B.ctl[2], T.depth);
    }
    auto make_leaf = [&]() {
        if (lane == 0) {
            N.left_or_first = T.first;
            N.count_or_right = 0x80000000u | T.count;
        }
    };
    if (T.count <= 1 || (T.count <= B.leaf_max && B.leaf_sah == 0.f)) {
        make_leaf();
        return;
    }
    uint32_t lg = 0;
    while ((1u << lg) < (T.count + 3) / 4) lg++;
    const bool median = T.depth + lg + 2 >= ORX_BVH_STACK;
    const int NB = B.bins;
    /* binning: all three axes at once */
    for (uint32_t i = lane; i < 3 * BVH_NB; i += 64) {
        const uint32_t ax = i / BVH_NB, b = i % BVH_NB;
        s_cnt[wv][ax][b] = 0;
        for (int k = 0; k < 3; k++) {
            s_lo[wv][ax][b][k] = 0xffffffffu;
            s_hi[wv][ax][b][k] = 0u;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float ext[3];
    for (int k = 0; k < 3; k++) ext[k] = chi[k] - clo[k];
    int axis_sel = -1;        /* median mode: widest centroid axis */
    if (median) {
        axis_sel = 0;
        for (int a = 1; a < 3; a++)
            if (ext[a] > ext[axis_sel]) axis_sel = a;
    }
    for (uint32_t i = lane; i < T.count; i += 64) {
        const uint32_t p = B.prims[T.first + i];
        float pl[3], ph[3];
        for (int k = 0; k < 3; k++) {
            pl[k] = tb[(size_t)k * nt + p];
            ph[k] = tb[(size_t)(3 + k) * nt + p];
        }
        for (int ax = 0; ax < 3; ax++) {
            if (!(ext[ax] > 0)) continue;
            if (median && ax != axis_sel) continue;
            const float c = tb[(size_t)(6 + ax) * nt + p];
            const int b = min(NB - 1, (int)((c - clo[ax]) / ext[ax] * NB));
            atomicAdd(&s_cnt[wv][ax][b], 1u);
            for (int k = 0; k < 3; k++) {
                atomicMin(&s_lo[wv][ax][b][k], ford(pl[k]));
                atomicMax(&s_hi[wv][ax][b][k], ford(ph[k]));
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    /* SAH sweep: lane ax evaluates axis ax (the host's order and strict < ties) */
    float bcost = INFINITY;
    int bbin = 0;
    if (lane < 3 && !median && ext[lane] > 0) {
        const int ax = (int)lane;
        float rl[BVH_NB], rc[BVH_NB];
        float al[3] = {INFINITY, INFINITY, INFINITY}, ah[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t acc = 0;
        for (int b = NB - 1; b > 0; b--) {
            acc += s_cnt[wv][ax][b];
            for (int k = 0; k < 3; k++) {
                al[k] = fminf(al[k], fdec(s_lo[wv][ax][b][k]));
                ah[k] = fmaxf(ah[k], fdec(s_hi[wv][ax][b][k]));
            }
            rl[b] = box_area(al[0], al[1], al[2], ah[0], ah[1], ah[2]);
            rc[b] = (float)acc;
        }
        float ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t lc = 0;
        for (int b = 0; b < NB - 1; b++) {
            lc += s_cnt[wv][ax][b];
            for (int k = 0; k < 3; k++) {
                ll[k] = fminf(ll[k], fdec(s_lo[wv][ax][b][k]));
                lh[k] = fmaxf(lh[k], fdec(s_hi[wv][ax][b][k]));
            }
            const float cost = box_area(ll[0], ll[1], ll[2], lh[0], lh[1], lh[2]) * (float)lc + rl[b + 1] * rc[b + 1];
            if (lc > 0 && lc < T.count && cost < bcost) {
                bcost = cost;
                bbin = b;
            }
        }
    }
    float best_cost = INFINITY;
    int best_axis = -1, best_split = 0;
    for (int ax = 0; ax < 3; ax++) {
        const float c = __shfl(bcost, ax, 64);
        const int b = __shfl(bbin, ax, 64);
        if (c < best_cost) {
            best_cost = c;
            best_axis = ax;
            best_split = b;
        }
    }
    if (T.count <= B.leaf_max) {
        const float A = box_area(lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]);
        if (best_axis < 0 || !(A > 0) || B.leaf_sah + best_cost / A >= (float)T.count) {
            make_leaf();
            return;
        }
    }
    /* split predicate: bin <= split on the SAH axis; median mode: the bin holding
     * the median on the widest axis (then the range is cut at count / 2, which
     * keeps the depth bound); no usable axis: cut at count / 2 in place */
    int pax = best_axis, psplit = best_split;
    if (median && axis_sel >= 0 && ext[axis_sel] > 0) {
        pax = axis_sel;
        uint32_t acc = 0;
        psplit = NB - 1;
        for (int b = 0; b < NB; b++) {
            acc += s_cnt[wv][pax][b];
            if (acc >= T.count / 2) {
                psplit = b;
                break;
            }
        }
    } else if (median) {
        pax = -1;
    }
    uint32_t nl = 0;
    if (pax >= 0) {
        /* stable partition through tmp: left in order, then right in order */
        uint32_t left_total = 0;
        for (uint32_t i0 = 0; i0 < T.count; i0 += 64) {
            const uint32_t i = i0 + lane;
            bool left = false;
            if (i < T.count) {
                const uint32_t p = B.prims[T.first + i];
                const float c = tb[(size_t)(6 + pax) * nt + p];
                left = min(NB - 1, (int)((c - clo[pax]) / ext[pax] * NB)) <= psplit;
            }
            left_total += (uint32_t)__popcll(__ballot(left));
        }
        uint32_t lpos = 0, rpos = left_total;
        for (uint32_t i0 = 0; i0 < T.count; i0 += 64) {
            const uint32_t i = i0 + lane;
            bool left = false, valid = i < T.count;
            uint32_t p = 0;
            if (valid) {
                p = B.prims[T.first + i];
                const float c = tb[(size_t)(6 + pax) * nt + p];
                left = min(NB - 1, (int)((c - clo[pax]) / ext[pax] * NB)) <= psplit;
            }
            const uint64_t ml = __ballot(valid && left), mr = __ballot(valid && !left);
            const uint64_t below = (1ull << lane) - 1ull;
            if (valid) {
                const uint32_t o = left ? lpos + (uint32_t)__popcll(ml & below) : rpos + (uint32_t)__popcll(mr & below);
                B.tmp[T.first + o] = p;
            }
            lpos += (uint32_t)__popcll(ml);
            rpos += (uint32_t)__popcll(mr);
        }
        __threadfence(); /* the lanes' tmp stores complete before any lane reads them back */
        for (uint32_t i = lane; i < T.count; i += 64) B.prims[T.first + i] = B.tmp[T.first + i];
        nl = left_total;
        if (median || nl == 0 || nl == T.count) nl = T.count / 2;
    } else {
        nl = T.count / 2;
    }
    if (lane == 0) {
        const uint32_t base = atomicAdd(&B.ctl[0], 2u);
        N.left_or_first = base;
        N.count_or_right = base + 1;
        const uint32_t t = atomicAdd(&B.ctl[1], 2u);
        next[t] = BvhTask{base, T.first, nl, T.depth + 1};
        next[t + 1] = BvhTask{base + 1, T.first + nl, T.count - nl, T.depth + 1};
    }
}

/* ---- treelet restructuring of the binary tree (the refinement of OptiX's Trbvh: Karras & Aila 2013) ----
 * Per inner node, bottom up, the treelet of the NL (9; Karras & Aila use 7) largest-area subtrees below it
 * (largest-area expansion from the node) is rebuilt as the SAH-optimal binary tree over them: a dynamic
 * programme over the 2^NL - 1 subsets
 * (node cost ci x area, leaf cost area x triangles), the partition of each subset scanned once; the rebuilt
 * treelet reuses its six inner nodes, the treelet root keeps its index.  One thread per node of a level (the
 * nodes of a level have disjoint subtrees); the levels come from a top-down pass over the current tree before
 * each bottom-up sweep.  Boxes become the unions of the children's (already conservatively expanded) boxes.
 * Hall: photon-path node steps 17.71 -> 17.21 (7 leaves) -> 16.91 (9) per ray, hall PPM 1018 -> 1033 -> 1043
 * Mpaths/s, VCM 561 -> 572 -> 576 (profiles/r06j_bvh_treelet_ab.txt; priced in tools/bvh_quality.cpp, where 11
 * leaves gain nothing more); scene init 0.1 -> 0.2 s on the hall. */
__device__ __forceinline__ float nd_area(const DevBvhNode& n) {
    return box_area(n.lo[0], n.lo[1], n.lo[2], n.hi[0], n.hi[1], n.hi[2]);
}
__device__ __forceinline__ bool nd_leaf(const DevBvhNode& n) { return (n.count_or_right & 0x80000000u) != 0; }
struct TreeletBufs {
    DevBvhNode* nodes;
    float* cost; /* [nodes] SAH cost of the subtree (area-weighted) */
    float ci;    /* inner-node cost relative to one triangle test (the build's leaf SAH) */
};
__device__ void tl_refresh(const TreeletBufs& T, uint32_t n) {
    DevBvhNode& x = T.nodes[n];
    if (nd_leaf(x)) {
        T.cost[n] = nd_area(x) * (float)(x.count_or_right & 0x7fffffffu);
        return;
    }
    const DevBvhNode l = T.nodes[x.left_or_first], r = T.nodes[x.count_or_right];
    for (int k = 0; k < 3; k++) x.lo[k] = fminf(l.lo[k], r.lo[k]), x.hi[k] = fmaxf(l.hi[k], r.hi[k]);
    T.cost[n] = T.ci * nd_area(x) + T.cost[x.left_or_first] + T.cost[x.count_or_right];
}
template <uint32_t NL> /* treelet leaves */
__global__ __launch_bounds__(64) void k_bvh_treelet(TreeletBufs T, const uint32_t* __restrict__ list, uint32_t n,
                                                    int restructure) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t nd = list[t];
    tl_refresh(T, nd);
    if (!restructure || nd_leaf(T.nodes[nd])) return;
    uint32_t lv[NL], inner[NL - 1];
    uint32_t m = 2, ni = 1;
    lv[0] = T.nodes[nd].left_or_first;
    lv[1] = T.nodes[nd].count_or_right;
    inner[0] = nd;
    while (m < NL) {
        int bi = -1;
        float ba = -1.f;
        for (uint32_t i = 0; i < m; i++) {
            const DevBvhNode& c = T.nodes[lv[i]];
            if (!nd_leaf(c) && nd_area(c) > ba) ba = nd_area(c), bi = (int)i;
        }
        if (bi < 0) break;
        const uint32_t c = lv[bi];
        inner[ni++] = c;
        lv[bi] = T.nodes[c].left_or_first;
        lv[m++] = T.nodes[c].count_or_right;
    }
    if (m < 3) return;
    const uint32_t full = (1u << m) - 1u;
    float copt[1u << NL], ar[1u << NL];
    uint16_t split[1u << NL];
    for (uint32_t S = 1; S <= full; S++) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = 0; i < m; i++)
            if (S >> i & 1u) {
                const DevBvhNode& c = T.nodes[lv[i]];
                for (int k = 0; k < 3; k++) lo[k] = fminf(lo[k], c.lo[k]), hi[k] = fmaxf(hi[k], c.hi[k]);
            }
        ar[S] = box_area(lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]);
    }
    for (uint32_t S = 1; S <= full; S++) {
        if ((S & (S - 1u)) == 0) {
            copt[S] = T.cost[lv[__builtin_ctz(S)]];
            split[S] = 0;
            continue;
        }
        float best = INFINITY;
        uint32_t bp = 0;
        const uint32_t low = S & (0u - S); /* the part holding the lowest member: each partition once */
        for (uint32_t P = (S - 1u) & S; P; P = (P - 1u) & S) {
            if (!(P & low)) continue;
            const float c = copt[P] + copt[S ^ P];
            if (c < best) best = c, bp = P;
        }
        copt[S] = T.ci * ar[S] + best;
        split[S] = (uint16_t)bp;
    }
    if (!(copt[full] < T.cost[nd] * (1.f - 1e-6f))) return;
    /* the optimal shape, top down (inner node k takes subset sub[k]), then boxes and costs bottom up */
    uint32_t sub[NL - 1], id[NL - 1], cnt = 1, next = 1;
    sub[0] = full;
    id[0] = nd;
    for (uint32_t k = 0; k < cnt; k++) {
        const uint32_t S = sub[k], P = split[S], Q = S ^ P;
        uint32_t ch[2];
        const uint32_t parts[2] = {P, Q};
        for (int h = 0; h < 2; h++) {
            const uint32_t X = parts[h];
            if ((X & (X - 1u)) == 0) {
                ch[h] = lv[__builtin_ctz(X)];
            } else {
                ch[h] = inner[next++];
                sub[cnt] = X;
                id[cnt++] = ch[h];
            }
        }
        T.nodes[id[k]].left_or_first = ch[0];
        T.nodes[id[k]].count_or_right = ch[1];
    }
    for (uint32_t k = cnt; k-- > 0;) tl_refresh(T, id[k]);
}
/* the current tree's levels, top down: the inner nodes of `cur` append their two children to `next` */
__global__ void k_bvh_bfs(const DevBvhNode* __restrict__ nodes, const uint32_t* __restrict__ cur, uint32_t n,
                          uint32_t* __restrict__ next, uint32_t* ctl) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const DevBvhNode x = nodes[cur[t]];
    if (nd_leaf(x)) return;
    const uint32_t o = atomicAdd(&ctl[1], 2u);
    next[o] = x.left_or_first;
    next[o + 1] = x.count_or_right;
}
/* SAH-optimal collapse to four-wide nodes (Ylitie et al. 2017), bottom up: F[n] = the cheapest cover of n's
 * subtree by at most 1..4 roots (a four-wide node visit costs 2.5 triangle tests x area, a leaf area x
 * triangles), K[n] = the roots given to the left child for each budget (0: n itself is the one root; for
 * budget 1, the distribution inside n's own node).  Priced -0.8..-2.0 % photon-ray node steps on its own. */
__global__ void k_bvh_sahdp(const DevBvhNode* __restrict__ nodes, float4* __restrict__ F, uchar4* __restrict__ K,
                            const uint32_t* __restrict__ list, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t nd = list[t];
    const DevBvhNode x = nodes[nd];
    const float a = nd_area(x);
    if (nd_leaf(x)) {
        const float c = a * (float)(x.count_or_right & 0x7fffffffu);
        F[nd] = make_float4(c, c, c, c);
        K[nd] = make_uchar4(0, 0, 0, 0);
        return;
    }
    const float4 fl = F[x.left_or_first], fr = F[x.count_or_right];
    const float L[5] = {0.f, fl.x, fl.y, fl.z, fl.w}, R[5] = {0.f, fr.x, fr.y, fr.z, fr.w};
    float f[5];
    uint8_t kk[5];
    auto G = [&](int i, uint8_t& kb) {
        float best = INFINITY;
        for (int k = 1; k < i; k++)
            if (L[k] + R[i - k] < best) best = L[k] + R[i - k], kb = (uint8_t)k;
        return best;
    };
    uint8_t k = 1;
    f[1] = 2.5f * a + G(4, k);
    kk[1] = k;
    for (int i = 2; i <= 4; i++) {
        const float g = G(i, k);
        if (g < f[1]) f[i] = g, kk[i] = k;
        else f[i] = f[1], kk[i] = 0;
    }
    F[nd] = make_float4(f[1], f[2], f[3], f[4]);
    K[nd] = make_uchar4(kk[1], kk[2], kk[3], kk[4]);
}
__device__ __forceinline__ uint8_t kget(const uchar4 k, int i) { return i == 1 ? k.x : i == 2 ? k.y : i == 3 ? k.z : k.w; }

/* ---- collapse to quantised BVH4 ---- */
struct CollapseItem {
    uint32_t n2, out;
};
struct CollapseBufs {
    const DevBvhNode* b2;
    const uchar4* K;       /* SAH-optimal collapse decisions (k_bvh_sahdp), or NULL: largest-area opening */
    DevBvh4* out;
    uint8_t* nch;          /* [out] children per BVH4 node */
    uint32_t* ctl;         /* [0] BVH4 node count, [1] next item count, [3] error */
    uint32_t cap;
};
__device__ __forceinline__ bool b2leaf(const DevBvhNode& n) { return (n.count_or_right & 0x80000000u) != 0; }
__device__ __forceinline__ float b2area(const DevBvhNode& n) {
    const float dx = n.hi[0] - n.lo[0], dy = n.hi[1] - n.lo[1], dz = n.hi[2] - n.lo[2];
    return dx * dy + dy * dz + dz * dx;
}
/* outward 8-bit quantisation of [clo, chi] on origin + q * 2^e (Bvh4Builder::quantise) */
__device__ bool quantise8(float origin, int e, float clo, float chi, uint32_t& qlo, uint32_t& qhi) {
    const float sc = ldexpf(1.0f, e);
    const double fl = floor(((double)clo - origin) / sc), ch = ceil(((double)chi - origin) / sc);
    qlo = (uint32_t)fmin(255.0, fmax(0.0, fl));
    qhi = (uint32_t)fmin(255.0, fmax(0.0, ch));
    while (qlo > 0 && origin + (float)qlo * sc > clo) qlo--;
    if (origin + (float)qlo * sc > clo) return false;
    while (qhi < 255 && origin + (float)qhi * sc < chi) qhi++;
    return origin + (float)qhi * sc >= chi;
}
__global__ void k_bvh_collapse(CollapseBufs C, const CollapseItem* __restrict__ items, uint32_t n,
                               CollapseItem* __restrict__ next) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const CollapseItem it = items[t];
    const DevBvhNode* B = C.b2;
    uint32_t ch[4];
    uint32_t nc = 0;
    if (b2leaf(B[it.n2])) {
        ch[nc++] = it.n2;
    } else if (C.K) { /* the roots of the cheapest cover: budget K[n].x to the left child, the rest to the right */
        uint32_t sn[4], sb[4], sp = 0;
        const uint8_t k1 = C.K[it.n2].x;
        sn[sp] = B[it.n2].count_or_right, sb[sp++] = 4u - k1;
        sn[sp] = B[it.n2].left_or_first, sb[sp++] = k1;
        while (sp) {
            const uint32_t n = sn[--sp], b = sb[sp];
            const uint8_t kb = b > 1 && !b2leaf(B[n]) ? kget(C.K[n], (int)b) : (uint8_t)0;
            if (kb == 0) {
                ch[nc++] = n;
            } else {
                sn[sp] = B[n].count_or_right, sb[sp++] = b - kb;
                sn[sp] = B[n].left_or_first, sb[sp++] = kb;
            }
        }
    } else {
        ch[nc++] = B[it.n2].left_or_first;
        ch[nc++] = B[it.n2].count_or_right;
        while (nc < 4) {
            int bi = -1;
            float ba = -1.f;
            for (uint32_t i = 0; i < nc; i++)
                if (!b2leaf(B[ch[i]]) && b2area(B[ch[i]]) > ba) ba = b2area(B[ch[i]]), bi = (int)i;
            if (bi < 0) break;
            const uint32_t c = ch[bi];
            ch[bi] = B[c].left_or_first;
            ch[nc++] = B[c].count_or_right;
        }
    }
    DevBvh4 nd;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < nc; i++)
        for (int k = 0; k < 3; k++) lo[k] = fminf(lo[k], B[ch[i]].lo[k]), hi[k] = fmaxf(hi[k], B[ch[i]].hi[k]);
    nd.ox = lo[0];
    nd.oy = lo[1];
    nd.oz = lo[2];
    nd.sx = nd.sy = nd.sz = 1.f;
    bool ok = true;
    for (int k = 0; k < 3; k++) {
        nd.qlo[k] = nd.qhi[k] = 0;
        const float ext = hi[k] - lo[k];
        int e = -126;
        if (ext > 0) {
            int ee;
            frexpf(ext / 255.0f, &ee);
            e = max(-126, ee - 1);
        }
        for (;; e++) {
            if (e > 127) {
                ok = false;
                break;
            }
            bool good = true;
            uint32_t ql[4] = {0, 0, 0, 0}, qh[4] = {0, 0, 0, 0};
            for (uint32_t i = 0; i < nc && good; i++) good = quantise8(lo[k], e, B[ch[i]].lo[k], B[ch[i]].hi[k], ql[i], qh[i]);
            if (!good) continue;
            uint32_t wl = 0, wh = 0;
            /* an empty slot gets the empty box lo = 255 > hi = 0: every ray misses it */
            for (int i = 0; i < 4; i++) wl |= ((uint32_t)i < nc ? ql[i] : 255u) << (8 * i), wh |= qh[i] << (8 * i);
            nd.qlo[k] = wl;
            nd.qhi[k] = wh;
            (k == 0 ? nd.sx : k == 1 ? nd.sy : nd.sz) = ldexpf(1.0f, e); /* 2^e, exact for e in [-126, 127] */
            break;
        }
    }
    uint32_t ninner = 0;
    for (uint32_t i = 0; i < nc; i++) ninner += b2leaf(B[ch[i]]) ? 0u : 1u;
    uint32_t base = ninner ? atomicAdd(&C.ctl[0], ninner) : 0u;
    uint32_t slot = ninner ? atomicAdd(&C.ctl[1], ninner) : 0u;
    for (int i = 0; i < 4; i++) nd.child[i] = ORX_EMPTY;
    for (uint32_t i = 0; i < nc; i++) {
        const DevBvhNode& c = B[ch[i]];
        if (b2leaf(c)) {
            const uint32_t cnt = c.count_or_right & 0x7fffffffu;
            if (cnt == 0 || cnt > 8 || c.left_or_first >= (1u << 28)) ok = false;
            nd.child[i] = ORX_LEAF | (c.left_or_first << 3) | (cnt - 1u);
        } else {
            if (base >= C.cap) ok = false;
            nd.child[i] = base;
            next[slot++] = CollapseItem{ch[i], base};
            base++;
        }
    }
    if (!ok) C.ctl[3] = 1;
    if (it.out < C.cap) {
        C.out[it.out] = nd;
        C.nch[it.out] = (uint8_t)nc;
    }
}
/* traversal-stack bound, bottom-up over the collapse levels: k - 1 pushes at a
 * node with k children plus the largest bound among its inner children */
__global__ void k_bvh_bound(const DevBvh4* __restrict__ out, const uint8_t* __restrict__ nch,
                            const CollapseItem* __restrict__ items, uint32_t n, uint32_t* bound) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t o = items[t].out;
    uint32_t sub = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t c = out[o].child[i];
        if (c != ORX_EMPTY && !(c & ORX_LEAF)) sub = max(sub, bound[c]);
    }
    bound[o] = (uint32_t)nch[o] - 1u + sub;
}

/* Host driver.  V/I: device copies of the mesh's vertices (float3) and indices.
 * Outputs: out4[cap4] BVH4 nodes, leaf_order[nt] (position k holds the
 * original id of the k-th triangle in leaf order). */
hipError_t device_build_bvh4(hipStream_t s, const float* V, const uint32_t* I, uint32_t nt, int bins, uint32_t leaf_max,
                             float leaf_sah, int treelet_passes, int treelet_leaves, bool sah_collapse, DevBvh4* out4,
                             uint32_t cap4,
                             uint32_t* leaf_order, uint32_t* nodes4, uint32_t* stack_bound, uint32_t* max_depth,
                             bool* ok) {
    *ok = false;
    if (nt == 0) return hipSuccess;
    hipError_t e;
    auto chk = [&](hipError_t x) { return (e = x) == hipSuccess; };
    float* tb = nullptr;
    uint32_t *tmp = nullptr, *ctl = nullptr, *bound = nullptr;
    DevBvhNode* nodes = nullptr;
    BvhTask *ta = nullptr, *tn = nullptr;
    CollapseItem* citems = nullptr;
    uint8_t* nch = nullptr;
    const size_t cap2 = 2 * (size_t)nt + 1;
    bool good = chk(hipMalloc(&tb, 9 * (size_t)nt * 4)) && chk(hipMalloc(&tmp, (size_t)nt * 4)) &&
                chk(hipMalloc(&ctl, 64)) && chk(hipMalloc(&nodes, cap2 * sizeof(DevBvhNode))) &&
                chk(hipMalloc(&ta, (size_t)nt * sizeof(BvhTask))) && chk(hipMalloc(&tn, (size_t)nt * sizeof(BvhTask))) &&
                chk(hipMalloc(&citems, (size_t)cap4 * sizeof(CollapseItem))) && chk(hipMalloc(&nch, cap4)) &&
                chk(hipMalloc(&bound, (size_t)cap4 * 4));
    std::vector<uint32_t> ident(nt);
    for (uint32_t i = 0; i < nt; i++) ident[i] = i;
    uint32_t hctl[16] = {1, 0, 0, 0};
    std::vector<uint32_t> level_off, level_cnt;
    if (good) {
        hipLaunchKernelGGL(k_bvh_tris, dim3((nt + 255) / 256), dim3(256), 0, s, V, I, nt, tb);
        good = chk(hipMemcpyAsync(leaf_order, ident.data(), (size_t)nt * 4, hipMemcpyHostToDevice, s)) &&
               chk(hipMemcpyAsync(ctl, hctl, 64, hipMemcpyHostToDevice, s));
        BvhTask root{0, 0, nt, 0};
        good = good && chk(hipMemcpyAsync(ta, &root, sizeof root, hipMemcpyHostToDevice, s));
    }
    BvhBuildBufs BB{tb, nt, leaf_order, tmp, nodes, ctl, std::min(bins, BVH_NB), leaf_max, leaf_sah};
    uint32_t ntasks = 1;
    while (good && ntasks) {
        const uint32_t zero = 0;
        good = chk(hipMemcpyAsync(ctl + 1, &zero, 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_bvh_level, dim3((ntasks + BVH_WAVES - 1) / BVH_WAVES), dim3(256), 0, s, BB, ta, ntasks, tn);
        good = good && chk(hipMemcpyAsync(hctl, ctl, 16, hipMemcpyDeviceToHost, s)) && chk(hipStreamSynchronize(s));
        ntasks = hctl[1];
        std::swap(ta, tn);
    }
    *max_depth = hctl[2];
    /* treelet restructuring sweeps and the SAH-optimal collapse's covers, each over the current tree's levels */
    float* cost = nullptr;
    float4* F = nullptr;
    uchar4* K = nullptr;
    uint32_t* lvl = nullptr;
    if (good && (treelet_passes > 0 || sah_collapse)) {
        good = chk(hipMalloc(&cost, cap2 * 4)) && chk(hipMalloc(&F, cap2 * sizeof(float4))) &&
               chk(hipMalloc(&K, cap2 * sizeof(uchar4))) && chk(hipMalloc(&lvl, cap2 * 4));
        std::vector<uint32_t> off;
        auto levels = [&]() { /* lvl = the nodes by depth, off[d] .. off[d + 1] */
            const uint32_t zero = 0;
            off.assign({0u, 1u});
            bool g = chk(hipMemcpyAsync(lvl, &zero, 4, hipMemcpyHostToDevice, s));
            uint32_t cur = 0, n = 1;
            while (g && n) {
                g = chk(hipMemcpyAsync(ctl + 1, &zero, 4, hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL(k_bvh_bfs, dim3((n + 255) / 256), dim3(256), 0, s, nodes, lvl + cur, n, lvl + cur + n,
                                   ctl);
                g = g && chk(hipMemcpyAsync(hctl, ctl, 16, hipMemcpyDeviceToHost, s)) && chk(hipStreamSynchronize(s));
                cur += n;
                n = hctl[1];
                if (n) off.push_back(cur + n);
                if (cur + n > cap2) g = false;
            }
            return g;
        };
        const TreeletBufs T{nodes, cost, leaf_sah > 0.f ? leaf_sah : 0.6f};
        for (int p = 0; good && p < treelet_passes; p++) {
            good = levels();
            for (size_t d = off.size() - 1; good && d-- > 0;) {
                const uint32_t n = off[d + 1] - off[d];
                if (treelet_leaves == 9)
                    hipLaunchKernelGGL(k_bvh_treelet<9>, dim3((n + 63) / 64), dim3(64), 0, s, T, lvl + off[d], n, 1);
                else
                    hipLaunchKernelGGL(k_bvh_treelet<7>, dim3((n + 63) / 64), dim3(64), 0, s, T, lvl + off[d], n, 1);
            }
        }
        if (good && sah_collapse) {
            good = levels();
            for (size_t d = off.size() - 1; good && d-- > 0;) {
                const uint32_t n = off[d + 1] - off[d];
                hipLaunchKernelGGL(k_bvh_sahdp, dim3((n + 255) / 256), dim3(256), 0, s, nodes, F, K, lvl + off[d], n);
            }
        }
        if (good && treelet_passes > 0) {
            if (!sah_collapse) good = levels();
            *max_depth = (uint32_t)off.size() - 2u; /* the restructured tree's depth */
        }
    }
    /* collapse, level by level from the root */
    uint32_t nitems = 1;
    if (good) {
        const uint32_t c0[4] = {1, 0, 0, 0};
        CollapseItem root{0, 0};
        good = chk(hipMemcpyAsync(ctl, c0, 16, hipMemcpyHostToDevice, s)) &&
               chk(hipMemcpyAsync(citems, &root, sizeof root, hipMemcpyHostToDevice, s));
    }
    CollapseBufs CB{nodes, sah_collapse ? K : nullptr, out4, nch, ctl, cap4};
    uint32_t off = 0;
    while (good && nitems) {
        if (off + nitems > cap4) {
            good = false;
            break;
        }
        level_off.push_back(off);
        level_cnt.push_back(nitems);
        const uint32_t zero = 0;
        good = chk(hipMemcpyAsync(ctl + 1, &zero, 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_bvh_collapse, dim3((nitems + 63) / 64), dim3(64), 0, s, CB, citems + off, nitems,
                           citems + off + nitems);
        good = good && chk(hipMemcpyAsync(hctl, ctl, 16, hipMemcpyDeviceToHost, s)) && chk(hipStreamSynchronize(s));
        off += nitems;
        nitems = hctl[1];
    }
    const uint32_t total4 = hctl[0];
    const bool collapse_ok = good && hctl[3] == 0 && total4 <= cap4;
    if (collapse_ok) {
        for (size_t l = level_off.size(); l-- > 0;)
            hipLaunchKernelGGL(k_bvh_bound, dim3((level_cnt[l] + 255) / 256), dim3(256), 0, s, out4, nch,
                               citems + level_off[l], level_cnt[l], bound);
        uint32_t b0 = 0;
        good = chk(hipMemcpyAsync(&b0, bound, 4, hipMemcpyDeviceToHost, s)) && chk(hipStreamSynchronize(s));
        *stack_bound = b0;
        *nodes4 = total4;
        *ok = good;
    }
    hipFree(tb);
    hipFree(tmp);
    hipFree(ctl);
    hipFree(nodes);
    hipFree(ta);
    hipFree(tn);
    hipFree(citems);
    hipFree(nch);
    hipFree(bound);
    hipFree(cost);
    hipFree(F);
    hipFree(K);
    hipFree(lvl);
    return good ? hipSuccess : (e != hipSuccess ? e : hipErrorUnknown);
}

}  // namespace orx
