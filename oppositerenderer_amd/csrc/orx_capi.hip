/*
 * orx_capi.hip — host side of liborx.so: the OptixRenderer replacement.
 *
 * Owns the device buffers and sequences the passes of one progressive
 * iteration exactly as OptixRenderer::renderNextIteration does
 * (RenderEngine/renderer/OptixRenderer.cpp:507-821), but as plain HIP
 * launches on one stream: no OptiX context, no per-launch validation, no
 * debug-buffer maps (the reference maps ~36 MB of debug counters to the
 * host every PPM iteration, OptixRenderer.cpp:620/:872-953; here they stay
 * on the device and are summed in-kernel).
 */
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <new>
#include <string>
#include <vector>

#include "orx.h"
#include "orx_kernels.h"

using namespace orx;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        release();
        if (n == 0) n = 16;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

/* host-side BVH over triangles: binned SAH, conservative boxes */
struct BuildTri {
    float lo[3], hi[3], c[3];
};

struct BvhBuilder {
    std::vector<DevBvhNode> nodes;
    std::vector<uint32_t> prims;
    const std::vector<BuildTri>* tris = nullptr;

    static void grow(float* lo, float* hi, const float* l2, const float* h2) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], l2[k]);
            hi[k] = std::max(hi[k], h2[k]);
        }
    }
    static float area(const float* lo, const float* hi) {
        float dx = std::max(0.f, hi[0] - lo[0]), dy = std::max(0.f, hi[1] - lo[1]), dz = std::max(0.f, hi[2] - lo[2]);
        return dx * dy + dy * dz + dz * dx;
    }
    uint32_t max_depth = 0;
    /* defaults measured on the 1080p hall (tools/trav_stats.py): SAH leaf
     * test up to 8 triangles cuts triangle tests/ray 5.9 -> 3.2 */
    int bins = 32;          /* SAH bins per axis (ORX_BVH_BINS) */
    uint32_t leaf_max = 8;  /* largest leaf (ORX_BVH_LEAF_MAX, <= 8) */
    float leaf_sah = 0.6f;  /* node traversal cost relative to a triangle test (ORX_BVH_LEAF_SAH); 0 = leaves of <= leaf_max, no test */
    static uint32_t ceil_log2(uint32_t v) {
        uint32_t l = 0;
        while ((1u << l) < v) l++;
        return l;
    }
    uint32_t build(uint32_t first, uint32_t count, uint32_t depth = 0) {
        if (depth > max_depth) max_depth = depth;
        uint32_t idx = (uint32_t)nodes.size();
        nodes.push_back(DevBvhNode{});
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = first; i < first + count; i++) {
            const BuildTri& t = (*tris)[prims[i]];
            grow(lo, hi, t.lo, t.hi);
            grow(clo, chi, t.c, t.c);
        }
        /* conservative expansion so that rounding in the slab test can never
         * cull a primitive the exact test would hit */
        for (int k = 0; k < 3; k++) {
            float m = std::max(std::fabs(lo[k]), std::fabs(hi[k]));
            float e = m * 1e-6f + 1e-20f;
            nodes[idx].lo[k] = lo[k] - e;
            nodes[idx].hi[k] = hi[k] + e;
        }
        if (count <= 1 || (count <= leaf_max && leaf_sah == 0.f)) {
            nodes[idx].left_or_first = first;
            nodes[idx].count_or_right = 0x80000000u | count;
            return idx;
        }
        /* binned SAH on the centroid extent; object-median split once the
         * depth budget (ORX_BVH_STACK) would otherwise be at risk */
        const int NB = bins;
        int best_axis = -1, best_split = 0;
        float best_cost = INFINITY;
        const bool median = depth + ceil_log2((count + 3) / 4) + 2 >= ORX_BVH_STACK;
        for (int ax = 0; ax < 3 && !median; ax++) {
            float ext = chi[ax] - clo[ax];
            if (!(ext > 0)) continue;
            uint32_t cnt[64] = {0};
            float blo[64][3], bhi[64][3];
            for (int b = 0; b < NB; b++)
                for (int k = 0; k < 3; k++) blo[b][k] = INFINITY, bhi[b][k] = -INFINITY;
            for (uint32_t i = first; i < first + count; i++) {
                const BuildTri& t = (*tris)[prims[i]];
                int b = std::min(NB - 1, (int)((t.c[ax] - clo[ax]) / ext * NB));
                cnt[b]++;
                grow(blo[b], bhi[b], t.lo, t.hi);
            }
            float rl[64], rcount[64];
            float alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t acc = 0;
            for (int b = NB - 1; b > 0; b--) {
                acc += cnt[b];
                grow(alo, ahi, blo[b], bhi[b]);
                rl[b] = area(alo, ahi);
                rcount[b] = (float)acc;
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t lc = 0;
            for (int b = 0; b < NB - 1; b++) {
                lc += cnt[b];
                grow(llo, lhi, blo[b], bhi[b]);
                float cost = area(llo, lhi) * (float)lc + rl[b + 1] * rcount[b + 1];
                if (lc > 0 && lc < count && cost < best_cost) {
                    best_cost = cost;
                    best_axis = ax;
                    best_split = b;
                }
            }
        }
        if (count <= leaf_max) {
            /* SAH leaf test: split cost Ct + (A_L N_L + A_R N_R)/A vs leaf cost N (Ci = 1) */
            const float A = area(lo, hi);
            if (best_axis < 0 || !(A > 0) || leaf_sah + best_cost / A >= (float)count) {
                nodes[idx].left_or_first = first;
                nodes[idx].count_or_right = 0x80000000u | count;
                return idx;
            }
        }
        uint32_t mid;
        if (best_axis < 0) {
            /* object median along the widest centroid axis */
            int ax = 0;
            for (int a = 1; a < 3; a++)
                if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
            mid = first + count / 2;
            std::nth_element(prims.begin() + first, prims.begin() + mid, prims.begin() + first + count,
                             [&](uint32_t p, uint32_t q) { return (*tris)[p].c[ax] < (*tris)[q].c[ax]; });
        } else {
            float ext = chi[best_axis] - clo[best_axis];
            auto it = std::partition(prims.begin() + first, prims.begin() + first + count, [&](uint32_t p) {
                const BuildTri& t = (*tris)[p];
                int b = std::min(NB - 1, (int)((t.c[best_axis] - clo[best_axis]) / ext * NB));
                return b <= best_split;
            });
            mid = (uint32_t)(it - prims.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        uint32_t l = build(first, mid - first, depth + 1);
        uint32_t r = build(mid, first + count - mid, depth + 1);
        nodes[idx].left_or_first = l;
        nodes[idx].count_or_right = r;
        return idx;
    }
};

/* Treelet restructuring of the binary tree (Karras & Aila 2013, the refinement of OptiX's Trbvh; the host
 * counterpart of the device builder's k_bvh_treelet, priced in tools/bvh_quality.cpp): per inner node, bottom
 * up, the treelet of its 7 largest-area descendants' subtrees is rebuilt as the SAH-optimal binary tree over
 * them (dynamic programme over the 127 subsets; node cost leaf_sah x area, leaf cost area x triangles), reusing
 * the treelet's inner nodes.  Boxes are unions of the children's (already conservatively expanded) boxes. */
struct TreeletOpt {
    std::vector<DevBvhNode>& B;
    float ci;
    size_t nl = 7; /* treelet leaves */
    std::vector<double> cost;
    explicit TreeletOpt(std::vector<DevBvhNode>& b, float c) : B(b), ci(c), cost(b.size(), 0.0) {}
    static bool leaf(const DevBvhNode& n) { return (n.count_or_right & 0x80000000u) != 0; }
    static float area(const float* lo, const float* hi) {
        float dx = std::max(0.f, hi[0] - lo[0]), dy = std::max(0.f, hi[1] - lo[1]), dz = std::max(0.f, hi[2] - lo[2]);
        return dx * dy + dy * dz + dz * dx;
    }
    void refresh(uint32_t n) {
        DevBvhNode& x = B[n];
        if (leaf(x)) {
            cost[n] = (double)area(x.lo, x.hi) * (double)(x.count_or_right & 0x7fffffffu);
            return;
        }
        const DevBvhNode &l = B[x.left_or_first], &r = B[x.count_or_right];
        for (int k = 0; k < 3; k++) x.lo[k] = std::min(l.lo[k], r.lo[k]), x.hi[k] = std::max(l.hi[k], r.hi[k]);
        cost[n] = (double)ci * area(x.lo, x.hi) + cost[x.left_or_first] + cost[x.count_or_right];
    }
    uint32_t emit(int S, uint32_t hint, const std::vector<uint32_t>& inner, size_t& next, const std::vector<int>& split,
                  const std::vector<uint32_t>& lv) {
        if ((S & (S - 1)) == 0) return lv[__builtin_ctz(S)];
        const uint32_t id = hint != 0xffffffffu ? hint : inner[next++];
        const uint32_t l = emit(split[S], 0xffffffffu, inner, next, split, lv);
        const uint32_t r = emit(S ^ split[S], 0xffffffffu, inner, next, split, lv);
        B[id].left_or_first = l;
        B[id].count_or_right = r;
        refresh(id);
        return id;
    }
    bool restructure(uint32_t n) {
        if (leaf(B[n])) return false;
        std::vector<uint32_t> lv = {B[n].left_or_first, B[n].count_or_right}, inner = {n};
        while (lv.size() < nl) {
            int bi = -1;
            float ba = -1.f;
            for (size_t i = 0; i < lv.size(); i++)
                if (!leaf(B[lv[i]]) && area(B[lv[i]].lo, B[lv[i]].hi) > ba) ba = area(B[lv[i]].lo, B[lv[i]].hi), bi = (int)i;
            if (bi < 0) break;
            const uint32_t c = lv[bi];
            inner.push_back(c);
            lv[bi] = B[c].left_or_first;
            lv.push_back(B[c].count_or_right);
        }
        const int m = (int)lv.size();
        if (m < 3) return false;
        const int full = (1 << m) - 1;
        std::vector<double> copt(1 << m, 0.0);
        std::vector<float> ar(1 << m, 0.f);
        std::vector<int> split(1 << m, 0);
        for (int S = 1; S <= full; S++) {
            float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = 0; i < m; i++)
                if (S >> i & 1)
                    for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], B[lv[i]].lo[k]), hi[k] = std::max(hi[k], B[lv[i]].hi[k]);
            ar[S] = area(lo, hi);
        }
        for (int S = 1; S <= full; S++) {
            if ((S & (S - 1)) == 0) {
                copt[S] = cost[lv[__builtin_ctz(S)]];
                continue;
            }
            double best = INFINITY;
            int bp = 0;
            const int low = S & -S;
            for (int P = (S - 1) & S; P; P = (P - 1) & S) {
                if (!(P & low)) continue;
                const double c = copt[P] + copt[S ^ P];
                if (c < best) best = c, bp = P;
            }
            copt[S] = (double)ci * ar[S] + best;
            split[S] = bp;
        }
        if (!(copt[full] < cost[n] * (1.0 - 1e-6))) return false;
        size_t next = 1;
        emit(full, n, inner, next, split, lv);
        return true;
    }
    uint32_t pass() {
        std::vector<uint32_t> order, st = {0u};
        while (!st.empty()) {
            const uint32_t n = st.back();
            st.pop_back();
            order.push_back(n);
            if (!leaf(B[n])) st.push_back(B[n].left_or_first), st.push_back(B[n].count_or_right);
        }
        uint32_t changed = 0;
        for (auto it = order.rbegin(); it != order.rend(); ++it) {
            refresh(*it);
            changed += restructure(*it);
        }
        return changed;
    }
    uint32_t depth(uint32_t n) const {
        return leaf(B[n]) ? 0u : 1u + std::max(depth(B[n].left_or_first), depth(B[n].count_or_right));
    }
};

/* Collapse the binary SAH tree into the four-wide quantised BVH the kernels
 * traverse (DevBvh4).  Each node opens its largest-area inner children until
 * it has four; child boxes are quantised outward on an 8-bit grid per axis.
 * `bound` = the most stack entries a traversal can hold: at a node with k
 * children hit, k-1 are pushed before descending. */
struct Bvh4Builder {
    const std::vector<DevBvhNode>* b2 = nullptr;
    std::vector<DevBvh4> out;
    std::vector<DevBvh4F> outf; /* same topology, fp32 child boxes */
    bool ok = true;
    /* the SAH-optimal collapse (Ylitie et al. 2017; the device builder's k_bvh_sahdp): F[n][i], the cheapest cover of n's
     * subtree by at most i roots (a four-wide node visit costing 2.5 triangle tests x area, a leaf area x
     * triangles), and K[n][i] the roots given to the left child (0: n is one root) */
    std::vector<std::array<double, 5>> F;
    std::vector<std::array<uint8_t, 5>> K;
    void dp(uint32_t n) {
        const std::vector<DevBvhNode>& B = *b2;
        if (F.empty()) F.assign(B.size(), {}), K.assign(B.size(), {});
        const float a = area(B[n]);
        if (leaf(B[n])) {
            for (int i = 1; i <= 4; i++) F[n][i] = (double)a * (double)(B[n].count_or_right & 0x7fffffffu), K[n][i] = 0;
            return;
        }
        const uint32_t l = B[n].left_or_first, r = B[n].count_or_right;
        dp(l);
        dp(r);
        auto G = [&](int i, int& kb) {
            double best = INFINITY;
            for (int k = 1; k < i; k++)
                if (F[l][k] + F[r][i - k] < best) best = F[l][k] + F[r][i - k], kb = k;
            return best;
        };
        int k = 1;
        F[n][1] = 2.5 * (double)a + G(4, k);
        K[n][1] = (uint8_t)k; /* the distribution inside n's own node */
        for (int i = 2; i <= 4; i++) {
            const double g = G(i, k);
            if (g < F[n][1]) F[n][i] = g, K[n][i] = (uint8_t)k;
            else F[n][i] = F[n][1], K[n][i] = 0;
        }
    }
    void roots(uint32_t n, int i, std::vector<uint32_t>& out_) const {
        const std::vector<DevBvhNode>& B = *b2;
        if (i == 1 || leaf(B[n]) || K[n][i] == 0) {
            out_.push_back(n);
            return;
        }
        roots(B[n].left_or_first, K[n][i], out_);
        roots(B[n].count_or_right, i - K[n][i], out_);
    }

    static bool leaf(const DevBvhNode& n) { return (n.count_or_right & 0x80000000u) != 0; }
    static float area(const DevBvhNode& n) {
        float dx = n.hi[0] - n.lo[0], dy = n.hi[1] - n.lo[1], dz = n.hi[2] - n.lo[2];
        return dx * dy + dy * dz + dz * dx;
    }
    /* outward 8-bit quantisation of [clo, chi] on origin + q * 2^e */
    static bool quantise(float origin, int e, float clo, float chi, uint32_t& qlo, uint32_t& qhi) {
        const float sc = std::ldexp(1.0f, e);
        auto dec = [&](uint32_t q) { return origin + (float)q * sc; };
        double fl = std::floor(((double)clo - origin) / sc), ch = std::ceil(((double)chi - origin) / sc);
        qlo = (uint32_t)std::min(255.0, std::max(0.0, fl));
        qhi = (uint32_t)std::min(255.0, std::max(0.0, ch));
        while (qlo > 0 && dec(qlo) > clo) qlo--;
        if (dec(qlo) > clo) return false;
        while (qhi < 255 && dec(qhi) < chi) qhi++;
        return dec(qhi) >= chi;
    }
    uint32_t build(uint32_t n2, uint32_t& bound) {
        const std::vector<DevBvhNode>& B = *b2;
        std::vector<uint32_t> ch;
        if (leaf(B[n2])) {
            ch.push_back(n2);
        } else if (!F.empty()) {
            roots(B[n2].left_or_first, K[n2][1], ch);
            roots(B[n2].count_or_right, 4 - K[n2][1], ch);
        } else {
            ch = {B[n2].left_or_first, B[n2].count_or_right};
            while (ch.size() < 4) {
                int bi = -1;
                float ba = -1.f;
                for (size_t i = 0; i < ch.size(); i++)
                    if (!leaf(B[ch[i]]) && area(B[ch[i]]) > ba) ba = area(B[ch[i]]), bi = (int)i;
                if (bi < 0) break;
                const uint32_t c = ch[bi];
                ch[bi] = B[c].left_or_first;
                ch.push_back(B[c].count_or_right);
            }
        }
        DevBvh4 nd;
        std::memset(&nd, 0, sizeof nd);
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t c : ch)
            for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], B[c].lo[k]), hi[k] = std::max(hi[k], B[c].hi[k]);
        nd.ox = lo[0];
        nd.oy = lo[1];
        nd.oz = lo[2];
        for (int k = 0; k < 3; k++) {
            const float ext = hi[k] - lo[k];
            int e = -126;
            if (ext > 0) {
                int ee;
                std::frexp(ext / 255.0f, &ee);
                e = std::max(-126, ee - 1);
            }
            for (;; e++) {
                if (e > 127) { ok = false; break; }
                bool good = true;
                uint32_t ql[4] = {0, 0, 0, 0}, qh[4] = {0, 0, 0, 0};
                for (size_t i = 0; i < ch.size() && good; i++)
                    good = quantise(lo[k], e, B[ch[i]].lo[k], B[ch[i]].hi[k], ql[i], qh[i]);
                if (!good) continue;
                uint32_t wl = 0, wh = 0;
                /* an empty slot gets the empty box lo = 255 > hi = 0: every ray misses it */
                for (int i = 0; i < 4; i++) wl |= ((size_t)i < ch.size() ? ql[i] : 255u) << (8 * i), wh |= qh[i] << (8 * i);
                nd.qlo[k] = wl;
                nd.qhi[k] = wh;
                (k == 0 ? nd.sx : k == 1 ? nd.sy : nd.sz) = ldexpf(1.0f, e); /* 2^e, exact for e in [-126, 127] */
                break;
            }
        }
        const uint32_t idx = (uint32_t)out.size();
        out.push_back(nd);
        DevBvh4F nf;
        std::memset(&nf, 0, sizeof nf);
        for (int i = 0; i < 4; i++) {
            const bool has = (size_t)i < ch.size();
            for (int k = 0; k < 3; k++) {
                nf.b[2 * k][i] = has ? B[ch[i]].lo[k] : INFINITY;
                nf.b[2 * k + 1][i] = has ? B[ch[i]].hi[k] : -INFINITY;
            }
        }
        outf.push_back(nf);
        uint32_t sub = 0;
        uint32_t refs[4] = {ORX_EMPTY, ORX_EMPTY, ORX_EMPTY, ORX_EMPTY};
        for (size_t i = 0; i < ch.size(); i++) {
            const DevBvhNode& c = B[ch[i]];
            if (leaf(c)) {
                const uint32_t cnt = c.count_or_right & 0x7fffffffu;
                if (cnt == 0 || cnt > 8 || c.left_or_first >= (1u << 28)) ok = false;
                refs[i] = ORX_LEAF | (c.left_or_first << 3) | (cnt - 1u);
            } else {
                uint32_t b = 0;
                refs[i] = build(ch[i], b);
                sub = std::max(sub, b);
            }
        }
        for (int i = 0; i < 4; i++) out[idx].child[i] = outf[idx].child[i] = refs[i];
        bound = (uint32_t)ch.size() - 1u + sub;
        return idx;
    }
};

/* host float3 with the same OptiX semantics as the device (f3 is __host__) */
f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

DevLight make_light(const orx_light& L) {
    /* Light ctors (renderer/Light.cpp:14-49) */
    DevLight l;
    std::memset(&l, 0, sizeof l);
    l.type = L.type;
    l.power = ld3(L.power);
    l.position = ld3(L.position);
    if (L.type == ORX_LIGHT_AREA) {
        l.v1 = ld3(L.v1);
        l.v2 = ld3(L.v2);
        f3 c = cross(l.v1, l.v2);
        l.normal = normalize(c);
        l.area = length(c);
        l.inverseArea = 1.0f / l.area;
        l.Lemit = (l.power * l.inverseArea) * ORX_1_PI_F;
    } else if (L.type == ORX_LIGHT_POINT) {
        l.Lemit = (l.power * 0.25f) * ORX_1_PI_F;
    } else {
        l.direction = ld3(L.direction); /* ctor normalises its by-value parameter only (Light.cpp:41) */
        l.normal = l.direction;
        l.angle = L.angle;
        float angleFactor = 1.0f / (1.0f - cosf(l.angle * 180 * ORX_1_PI_F));
        l.Lemit = ((l.power * 0.25f) * ORX_1_PI_F) * angleFactor;
    }
    return l;
}

float dtor(float d) { return d * ((float)M_PI / 180.f); } /* Camera.cpp:87-90 */

DevCamera camera_setup(const orx_camera& c, float* ulen_out = nullptr, float* vlen_out = nullptr) {
    /* Camera::setup (renderer/Camera.cpp:333-345) */
    DevCamera k;
    f3 eye = ld3(c.eye), lookat = ld3(c.lookat), up = ld3(c.up);
    k.eye = eye;
    k.lookdir = lookat - eye;
    float lookdir_len = length(k.lookdir);
    up = normalize(up);
    f3 cu = normalize(cross(k.lookdir, up));
    f3 cv = normalize(cross(cu, k.lookdir));
    float ulen = lookdir_len * tanf(dtor(c.hfov * 0.5f));
    k.u = cu * ulen;
    float vlen = lookdir_len * tanf(dtor(c.vfov * 0.5f));
    k.v = cv * vlen;
    k.aperture = c.aperture;
    if (ulen_out) *ulen_out = ulen;
    if (vlen_out) *vlen_out = vlen;
    return k;
}

enum PassId { P_EYE = 0, P_PHOTON, P_SETUP_HASH, P_SCAN, P_SCATTER, P_GATHER, P_DIRECT, P_PT, P_VCM_LIGHT, P_VCM_CAMERA,
              P_VCM_SHADOW, P_COUNT };
constexpr int EV_POOL = 1024; /* timed launches kept per pass between resets */

}  // namespace

struct orx_renderer {
    int device = 0;
    orx_config cfg{};
    hipStream_t stream = nullptr;
    hipStream_t aux = nullptr;   /* PPM direct pass, overlapped with the grid build and gather */
    hipEvent_t ev_photon_done = nullptr, ev_direct_done = nullptr;
    bool overlap_direct = false;
    /* one device, three buffer sets, uniform grid: the grid build of iteration i on a stream of its own (gridq)
     * beside the photon pass of i + 1, the photon pass's outputs (deposit records, positions, validity bits,
     * AABB replicas) alternating between two sets (d_slotsB ...; po: the set the last photon pass wrote);
     * ev_gsrc[set]: the last grid build that read that set */
    bool async_grid = false;
    uint32_t po = 0;
    hipStream_t gridq = nullptr;
    hipEvent_t ev_gsrc[2] = {nullptr, nullptr};
    DevBuf d_slotsB, d_vmaskB, d_bboxB, d_pos4B;
    bool out_b = false; /* set B allocated: the asynchronous build may run */
    /* the schedule chosen from the workload (ORX_GRID_ASYNC unset): the first pipelined iteration after a
     * resize times its photon pass + grid build on the renderer's stream and its gather, the next one's
     * photon pass waits for that gather (so nothing overlaps it), and the iteration after that picks the
     * asynchronous build if photon + grid take more than GRID_CHAIN_RATIO x the gather (the chain, not the
     * gather, then sets the frame).  probe_stage: 0 decided, 1 measure, 2 isolate, 3 decide */
    uint32_t probe_stage = 0, probe_k = 0;
    float probe_ms[2] = {0.f, 0.f}; /* photon + grid, gather of the measured iteration */
    hipEvent_t ev_pm[4] = {};
    /* pipelined PPM: the eye pass of iteration i+1 runs on aux right behind the direct pass of i
     * (the RNG chain), beside the grid build of i; ev_eye_done orders the photon pass after it.
     * eye_chain: aux is already ordered after every earlier renderer-stream write the eye pass
     * reads (the previous call was a pipelined iteration, nothing else enqueued since) */
    hipEvent_t ev_eye_done = nullptr, ev_main = nullptr;
    bool eye_chain = false;
    /* PPM iteration pipelining (world 1, uniform grid, own stream): the gather and output of
     * iteration i run on gstream beside the eye/photon/grid passes of iteration i+1, each
     * iteration on one of two buffer sets (hitpoints, direct, grid-ordered photons, offsets,
     * grid parameters); ev_gdone[k] marks the end of the last gather+output on set k */
    hipStream_t gstream = nullptr;
    hipEvent_t ev_grid_done = nullptr, ev_gdone[3] = {nullptr, nullptr, nullptr};
    /* buffer sets the pipeline cycles through: 3 on one device (the eye pass of i + 1 then waits for the gather
     * of i - 2, not of i - 1), 2 for the sharded pipeline; set_id: the physical set each view slot holds */
    uint32_t nsets = 2, set_id[3] = {0, 1, 2};
    bool pipe_bufs = false, pend = false, last_pipelined = false;
    /* sharded PPM pipelining (orx_set_ppm_pipeline): gather + finish on the caller's side stream */
    bool shard_pipe = false;
    /* its finishes (orx_ppm_finish / _on): fin_due, the current iteration's is outstanding; fin_snap, the
     * previous iteration's is, its pixel buffers, constants and buffer set held here (the caller may issue
     * it after the next iteration's eye pass, behind that iteration's hit-point all-gather) */
    bool fin_due = false, fin_snap = false;
    PixelBufs fin_px{};
    Consts fin_consts{};
    uint32_t fin_pp = 0;
    /* slab mode (orx_set_slab_partition): photon buffers sized for the imported slab photons */
    bool slab = false;
    size_t S_cap = 0;
    DevBuf d_slabtab, d_slabcur;
    DevBuf d_tiles; /* slab gather: tile list, count, flags */
    uint32_t own_axis = 0, own_nb = 0, own_lo = 1, own_hi = 0; /* slab gather: the bins this rank owns */
    int pipe_mode = -1; /* orx_set_iteration_pipelining: -1 = ORX_PIPELINE env */
    hipStream_t side = nullptr;
    uint32_t pp = 0;
    std::string err;
    bool scene_ready = false;
    /* scene */
    DevBuf d_quads, d_qmat, d_spheres, d_smat, d_triv, d_trin, d_tmat, d_mats, d_lights, d_bvh, d_bvhprims;
    DevBuf d_triuv, d_trit, d_tribt, d_texels, d_texdesc; /* Texture material attributes and images */
    bool has_tex = false;
    DevScene scene{};
    /* frame */
    uint32_t W = 10, H = 10, RW = 0, RH = 0;
    uint32_t rank = 0, world = 1;
    uint32_t rows = 0, max_rows = 0, rng_rows = 0, prows = 0;
    bool rng_ready = false;
    hipStream_t ext_stream = nullptr; /* caller-provided stream (orx_set_stream) */
    bool use_ext = false;
    DevBuf d_rng, d_hp, d_ind, d_dir, d_out, d_dbg;
    DevBuf d_slots, d_vmask, d_sorted, d_perm, d_keys;
    DevBuf d_offsets, d_bbox, d_grid;
    DevBuf d_pos4, d_bstable, d_bspartials, d_bspairs, d_subofs;  /* bucket-sort grid build */
    DevBuf d_hcount, d_hwin;  /* stochastic hash table */
    DevBuf d_ptrav;           /* photon pass: the deep traversal-stack entries */
    DevBuf d_hp2, d_dir2, d_sorted2, d_subofs2, d_offsets2, d_grid2; /* second buffer set (pipelining) */
    DevBuf d_kdtree2; /* kd-tree photon map: the second tree */
    DevBuf d_slots2, d_hcount2, d_hwin2; /* stochastic hash: second deposit records and table */
    DevBuf d_hp3, d_dir3, d_sorted3, d_subofs3, d_offsets3, d_grid3, d_kdtree3, d_slots3, d_hcount3, d_hwin3; /* third */
    /* kd-tree photon map (photon_map = 2, orx_kdtree.hip) */
    DevBuf d_kdtree, d_kdids, d_kdlst, d_kdnkey, d_kdkeys, d_kdnodepos, d_kdseg, d_kdbox, d_kdninfo, d_kdP, d_kdppart,
        d_kdtable, d_kdtpart, d_kdvpart, d_kdcount;
    KdBufs kd{};
    f3 aabb_lo{}, aabb_hi{};  /* IScene::getSceneAABB (the stochastic hash grid's bounds) */
    PixelBufs px{};
    PhotonBufs pb{};
    /* timing: event pairs per pass since the last orx_reset_timing */
    std::vector<hipEvent_t> ev[P_COUNT];
    int ev_n[P_COUNT]{};
    uint32_t timed_iterations = 0;
    bool timing = true;
    uint64_t last_method = 0;
    Consts last_consts{};
    /* VCM: pixelSizeFactor (OptixRenderer.cpp:306, :846), LVC estimate flag (:83, :461, :847) */
    float psf_x = 1.0f, psf_y = 1.0f;
    bool vcm_estimated = false;
    size_t vcm_npx = 0;  /* own-row subpaths W*rows the VCM buffers are sized for */
    size_t vcm_spx = 0;  /* owner-block splat pixels W*max_rows*world */
    bool vcm_pending = false; /* light pass done, camera pass (orx_vcm_finish) outstanding */
    bool vcm_kd = false;      /* d_vkd sized for the current vcm_npx */
    VcmBufs vcm_vb{};
    VcmConsts vcm_c{};
    DevBuf d_vcount, d_vverts, d_vsplat, d_vcam, d_vkd, d_vshq, d_vwork, d_vconst, d_tstats;
    DevBuf d_vdq, d_vdpx, d_vrngsave, d_vshstk; /* VCM camera pass: deferred shadow-ray entries, per-pixel list heads, RNG copy, deep stack */
    /* VCM overlap (single device, deferred shadow rays): the camera pass's resolve (shadow rays,
     * colours) of iteration i runs on aux beside the light pass and walk of i+1; the light images and
     * the entry lists with their control words alternate (d_vsplat2, d_vdq2, d_vdpx2, vcm_dpar),
     * ev_vcam ends the walk, ev_vacc the resolve, vcm_pend: one in flight */
    DevBuf d_vsplat2, d_vdq2, d_vdpx2, d_vlcq, d_vlcq2; /* d_vlcq: the light pass's deferred camera connections */
    /* the other set of what the resolve's in-place rerun reads while the next iteration runs: light
     * vertices, their counts and texel colours, the walk's RNG start words */
    DevBuf d_vverts2, d_vcount2, d_vkd2, d_vrngsave2;
    uint32_t vcm_dpar = 0;
    bool last_vcm_overlap = false;
    size_t vcm_dqcap = 0; /* entries per list (ORX_VCM_DEFER per own pixel) */
    hipEvent_t ev_vcam = nullptr, ev_vacc = nullptr;
    bool vcm_pend = false;
    std::vector<DevLight> host_lights;
    /* participating medium (cfg.enable_media with a medium box): the box, this frame's per-pixel
     * volumetricRadiance and per-photon last events, the volumetric table of the last photon pass */
    bool media = false;
    VolMap vm{};
    DevBuf d_volR, d_ev_a, d_ev_b;
    DevBuf d_vcnt, d_vwin, d_vA, d_vB, d_vkeys, d_vvals, d_vkeys2, d_vvals2, d_vsort, d_vstart, d_vrec;
};

static orx_status set_err(orx_renderer* r, orx_status s, const std::string& m) {
    if (r) r->err = m;
    return s;
}
#define HIPCHK(r, x)                                                                                      \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess)                                                                             \
            return set_err(r, e_ == hipErrorOutOfMemory ? ORX_ERR_OUT_OF_MEMORY : ORX_ERR_DEVICE,          \
                           std::string("HIP error in ") + #x + ": " + hipGetErrorString(e_));           \
    } while (0)

static orx_status sync_all(orx_renderer* r);
static orx_status photon_stack_ensure(orx_renderer* r);

extern "C" {

#ifdef ORX_TRAV_STATS
/* stats build only: [closest: rays, nodes, leaves, tris, any: rays, nodes, leaves, tris]; reset = 1 zeroes */
int orx_trav_stats_read(orx_renderer* r, unsigned long long* out, int reset) {
    if (!r || !r->scene.trav_stats || hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpy(out, r->scene.trav_stats, 96, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    /* [16]: gather photons accepted (out must hold 21 values) */
    if (r->pb.grid && hipMemcpy(out + 16, &r->pb.grid->st_accepted, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    /* [17..20]: closest-hit node visits to BVH4 nodes with index < 21, 85, 341, 1365 (the top 2..5 levels) */
    if (hipMemcpy(out + 17, r->scene.trav_stats + 16, 32, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    if (reset && hipMemset(r->scene.trav_stats, 0, 256) != hipSuccess) return 1;
    /* [12..15]: gather lane batches, wave batches, lane rows, wave rows */
    if (r->pb.grid) {
        if (hipMemcpy(out + 12, &r->pb.grid->st_lane_batches, 32, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        if (reset && hipMemset(&r->pb.grid->st_lane_batches, 0, 40) != hipSuccess) return 1;
    } else {
        for (int k = 12; k < 16; k++) out[k] = 0;
    }
    return 0;
}
#endif

void orx_default_config(orx_config* c) {
    std::memset(c, 0, sizeof *c);
    c->photon_launch_width = 1024;
    c->photon_launch_height = 1024;
    c->max_photon_deposits = 4;
    c->photon_grid_max_size = 100 * 100 * 100;
    c->max_photon_trace_depth = 7;
    c->max_radiance_trace_depth = 9;
    c->vcm_max_path_length = 10;
    c->seed = 0;
    c->debug_counters = 1;
    c->volumetric_photons = 200000; /* NUM_VOLUMETRIC_PHOTONS (config.h:35) */
}

/* stochastic hash: photonsSize = NUM_PHOTONS must be a power of two (getHashValue masks with
 * photonsSize - 1; OptixRenderer.cpp:46 "Ensure that NUM PHOTONS are a power of 2"), and a path's
 * deposits (one per non-specular hit at depth >= 1, never capped) fit the 8-bit deposit mask */
static bool hash_config_ok(const orx_config& c) {
    const uint64_t n = (uint64_t)c.photon_launch_width * c.photon_launch_height * c.max_photon_deposits;
    return n && n <= (1ull << 31) && (n & (n - 1)) == 0 && c.max_photon_trace_depth <= 9;
}

/* the deferred gather yields to the next iteration's passes (lowest priority; measured equal
 * to normal priority on the hall) */
/* The deferred gather's stream at the highest priority (ORX_GATHER_PRIO=0: the lowest): at configs[4] (4K) the
 * gather stream is the frame's long pole (gather 23.7 ms serial, ~42 ms beside the next iteration's eye, photon
 * and grid passes, which need ~20 ms), and dispatching its workgroups first gains 1.8 % (552 -> 562 Mpaths/s,
 * 45.4 -> 44.6 ms); on the 1080p hall the frame is unchanged (1014 / 1014 Mpaths/s)
 * (profiles/r06i_gather_priority_ab.txt) */
static int gather_stream_priority() {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
    static const bool high = [] {
        const char* e = getenv("ORX_GATHER_PRIO");
        return !(e && atoi(e) == 0);
    }();
    return high ? greatest : least;
}

/* the asynchronous grid build's stream: the gather's priority, or the least (ORX_GRIDQ_PRIO=0) */
static int grid_stream_priority() {
    static const bool low = [] {
        const char* e = getenv("ORX_GRIDQ_PRIO");
        return e && atoi(e) == 0;
    }();
    int least = 0, greatest = 0;
    if (low && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess) return least;
    return gather_stream_priority();
}

orx_status orx_create(int hip_device, const orx_config* cfg, orx_renderer** out) {
    if (!out) return ORX_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    orx_config c;
    if (cfg) c = *cfg;
    else orx_default_config(&c);
    if (c.max_photon_deposits == 0 || c.max_photon_deposits > 8 || c.photon_launch_width == 0 ||
        c.photon_launch_height == 0 || c.photon_grid_max_size == 0 || c.photon_grid_max_size > (1u << 26) ||
        c.gather_variant > 2 || c.photon_map > 2 || (c.photon_map == 1 && !hash_config_ok(c)) ||
        (c.photon_map == 2 && (uint64_t)c.photon_launch_width * c.photon_launch_height * c.max_photon_deposits >
                                  (1ull << 28)))
        return ORX_ERR_INVALID_ARGUMENT;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORX_ERR_DEVICE;
    if (hip_device < 0 || hip_device >= n) return ORX_ERR_INVALID_ARGUMENT;
    orx_renderer* r = new (std::nothrow) orx_renderer();
    if (!r) return ORX_ERR_OUT_OF_MEMORY;
    r->device = hip_device;
    r->cfg = c;
    if (hipSetDevice(hip_device) != hipSuccess ||
        hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&r->aux, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&r->gstream, hipStreamNonBlocking, gather_stream_priority()) != hipSuccess ||
        hipStreamCreateWithPriority(&r->gridq, hipStreamNonBlocking, grid_stream_priority()) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_gsrc[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_gsrc[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_grid_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_gdone[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_gdone[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_gdone[2], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_photon_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_direct_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_eye_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_vcam, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_vacc, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->ev_main, hipEventDisableTiming) != hipSuccess) {
        delete r;
        return ORX_ERR_DEVICE;
    }
    *out = r;
    return ORX_OK;
}

void orx_destroy(orx_renderer* r) {
    if (!r) return;
    hipSetDevice(r->device);
    /* every stream first: the pass timing events are recorded on all of them */
    if (r->stream) hipStreamSynchronize(r->stream);
    if (r->aux) hipStreamSynchronize(r->aux);
    if (r->gstream) hipStreamSynchronize(r->gstream);
    for (int p = 0; p < P_COUNT; p++)
        for (hipEvent_t e : r->ev[p]) hipEventDestroy(e);
    for (hipEvent_t e : {r->ev_grid_done, r->ev_gdone[0], r->ev_gdone[1], r->ev_gdone[2]})
        if (e) hipEventDestroy(e);
    if (r->gridq) hipStreamSynchronize(r->gridq);
    if (r->gstream) hipStreamDestroy(r->gstream);
    if (r->gridq) hipStreamDestroy(r->gridq);
    for (hipEvent_t e : {r->ev_gsrc[0], r->ev_gsrc[1]})
        if (e) hipEventDestroy(e);
    for (hipEvent_t e : r->ev_pm)
        if (e) hipEventDestroy(e);
    if (r->ev_photon_done) hipEventDestroy(r->ev_photon_done);
    if (r->ev_direct_done) hipEventDestroy(r->ev_direct_done);
    if (r->ev_eye_done) hipEventDestroy(r->ev_eye_done);
    if (r->ev_vcam) hipEventDestroy(r->ev_vcam);
    if (r->ev_vacc) hipEventDestroy(r->ev_vacc);
    if (r->ev_main) hipEventDestroy(r->ev_main);
    if (r->aux) hipStreamDestroy(r->aux);
    if (r->stream) hipStreamDestroy(r->stream);
    delete r;
}

const char* orx_last_error(const orx_renderer* r) { return r ? r->err.c_str() : "null renderer"; }
void* orx_stream(orx_renderer* r) { return r ? (void*)r->stream : nullptr; }

orx_status orx_set_shard(orx_renderer* r, uint32_t rank, uint32_t world) {
    if (!r || world == 0 || rank >= world) return ORX_ERR_INVALID_ARGUMENT;
    if (world > 1 && r->cfg.enable_media)
        return set_err(r, ORX_ERR_UNSUPPORTED, "participating media are single-device");
    if (world > 1 && r->cfg.photon_map == 1)
        return set_err(r, ORX_ERR_UNSUPPORTED, "the stochastic hash photon map is single-device (one table per iteration)");
    r->rank = rank;
    r->world = world;
    r->rng_ready = false; /* force re-allocation of the local rows */
    return ORX_OK;
}

orx_status orx_init_scene(orx_renderer* r, const orx_scene* s) {
    if (!r || !s) return ORX_ERR_INVALID_ARGUMENT;
    if (s->n_lights == 0 || !s->lights) return set_err(r, ORX_ERR_NO_LIGHTS, "No lights exists in this scene.");
    if (s->n_materials == 0 || !s->materials) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "scene has no materials");
    HIPCHK(r, hipSetDevice(r->device));
    {
        orx_status s0 = sync_all(r); /* in-flight passes read the scene being replaced */
        if (s0 != ORX_OK) return s0;
    }
    const uint32_t nq = s->n_quads, ns = s->n_spheres, nt = s->n_triangles, nm = s->n_materials;
    /* the traversal addresses triangles (48 B) and BVH4 nodes (64 B, fewer than triangles) with
     * 32-bit byte offsets */
    if (nt >= (1u << 26)) return set_err(r, ORX_ERR_UNSUPPORTED, "more than 2^26 triangles");
    /* validate material indices and triangle vertex indices */
    for (uint32_t i = 0; i < nq; i++)
        if (s->quad_material[i] >= nm) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "quad material out of range");
    for (uint32_t i = 0; i < ns; i++)
        if (s->sphere_material[i] >= nm) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "sphere material out of range");
    for (uint32_t i = 0; i < s->n_textures; i++) {
        const orx_texture& t = s->textures[i];
        if (!t.rgba || !t.width || !t.height || (t.normal_rgba && (!t.normal_width || !t.normal_height)))
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "texture image without texels");
    }
    for (uint32_t i = 0; i < nm; i++)
        if (s->materials[i].type == ORX_MAT_TEXTURE &&
            (s->materials[i].texture < 0 || (uint32_t)s->materials[i].texture >= s->n_textures))
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "Texture material without a texture image");
    const bool media = r->cfg.enable_media && s->n_media;
    if (media) {
        if (s->n_media != 1 || !s->media)
            return set_err(r, ORX_ERR_UNSUPPORTED, "participating media: one medium box per scene");
        const float* m = s->media;
        if (!(m[0] < m[3] && m[1] < m[4] && m[2] < m[5]) || !(m[6] >= 0 && m[7] >= 0 && m[6] + m[7] > 0))
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "medium box: min < max and sigma_s + sigma_a > 0");
        if (r->cfg.volumetric_photons == 0)
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "volumetric_photons must be > 0 with media");
        if (r->world > 1) return set_err(r, ORX_ERR_UNSUPPORTED, "participating media are single-device");
    }
    r->media = media;
    r->vm = VolMap{};
    if (media) {
        r->vm.on = 1;
        r->vm.lo = mk(s->media[0], s->media[1], s->media[2]);
        r->vm.hi = mk(s->media[3], s->media[4], s->media[5]);
        r->vm.sig_s = s->media[6];
        r->vm.sig_a = s->media[7];
        const uint32_t NV = r->cfg.volumetric_photons;
        HIPCHK(r, r->d_vcnt.ensure((size_t)NV * 4));
        HIPCHK(r, r->d_vwin.ensure((size_t)NV * 4));
        HIPCHK(r, r->d_vA.ensure((size_t)NV * 16));
        HIPCHK(r, r->d_vB.ensure((size_t)NV * 16));
        HIPCHK(r, r->d_vkeys.ensure((size_t)NV * 4));
        HIPCHK(r, r->d_vvals.ensure((size_t)NV * 4));
        HIPCHK(r, r->d_vkeys2.ensure((size_t)NV * 4));
        HIPCHK(r, r->d_vvals2.ensure((size_t)NV * 4));
        HIPCHK(r, r->d_vsort.ensure(vol_sort_tmp_bytes(NV) + 256));
        HIPCHK(r, r->d_vrec.ensure((size_t)NV * 32 + 32));
    }
    for (uint32_t i = 0; i < nt; i++) {
        if (s->triangle_material[i] >= nm) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "triangle material out of range");
        for (int k = 0; k < 3; k++)
            if (s->triangles[3 * (size_t)i + k] >= s->n_vertices)
                return set_err(r, ORX_ERR_INVALID_ARGUMENT, "triangle vertex index out of range");
    }
    /* Cornell::createParallelogram (scene/Cornell.cpp:33-64) */
    std::vector<DevQuad> quads(nq);
    for (uint32_t i = 0; i < nq; i++) {
        f3 anchor = ld3(s->quads + 9 * i), o1 = ld3(s->quads + 9 * i + 3), o2 = ld3(s->quads + 9 * i + 6);
        f3 normal = normalize(cross(o1, o2));
        float d = dot(normal, anchor);
        f3 v1 = o1 / dot(o1, o1), v2 = o2 / dot(o2, o2);
        quads[i] = DevQuad{normal.x, normal.y, normal.z, d, anchor.x, anchor.y, anchor.z, v1.x,
                           v1.y, v1.z, v2.x, v2.y, v2.z, 0, 0, 0};
    }
    std::vector<DevSphere> sph(ns);
    for (uint32_t i = 0; i < ns; i++)
        sph[i] = DevSphere{s->spheres[4 * i], s->spheres[4 * i + 1], s->spheres[4 * i + 2], s->spheres[4 * i + 3]};
    std::vector<DevMaterial> mats(nm);
    for (uint32_t i = 0; i < nm; i++) {
        const orx_material& m = s->materials[i];
        DevMaterial d;
        std::memset(&d, 0, sizeof d);
        d.type = m.type;
        d.Kd = ld3(m.Kd);
        d.Ks = ld3(m.Ks);
        d.Kr = ld3(m.Kr);
        d.Kt = ld3(m.Kt);
        d.ior = m.ior;
        d.exponent = m.exponent;
        d.tex = m.texture;
        if (m.type == ORX_MAT_DIFFUSE_EMITTER) {
            /* DiffuseEmitter.cpp:17-25, :48-62 */
            f3 power = ld3(m.power) * d.Kd;
            d.inverseArea = m.inverse_area;
            d.powerPerArea = power * m.inverse_area;
            d.Lemit = (power * m.inverse_area) * ORX_1_PI_F;
        } else if (m.type == ORX_MAT_GLOSSY) {
            /* Glossy.cpp:16-30 */
            f3 sumK = d.Kd + d.Ks;
            float sumScale = 1.f / maxf(maxf(sumK.x, sumK.y), sumK.z);
            if (sumScale < 1.f) {
                d.Kd = d.Kd * sumScale;
                d.Ks = d.Ks * sumScale;
            }
        } else if (m.type < 0 || m.type > ORX_MAT_TEXTURE) {
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "unknown material type");
        }
        mats[i] = d;
    }
    std::vector<DevLight> lights(s->n_lights);
    for (uint32_t i = 0; i < s->n_lights; i++) lights[i] = make_light(s->lights[i]);
    r->host_lights = lights;
    /* triangles: BVH over triangle boxes, then vertex / normal / material
     * arrays rewritten in leaf order (tri_v[3k].w carries the original id) */
    std::vector<BuildTri> bt(nt);
    for (uint32_t i = 0; i < nt; i++) {
        BuildTri& b = bt[i];
        for (int k = 0; k < 3; k++) b.lo[k] = INFINITY, b.hi[k] = -INFINITY;
        for (int v = 0; v < 3; v++) {
            const float* p = s->vertices + 3 * (size_t)s->triangles[3 * (size_t)i + v];
            for (int k = 0; k < 3; k++) {
                b.lo[k] = std::min(b.lo[k], p[k]);
                b.hi[k] = std::max(b.hi[k], p[k]);
            }
        }
        for (int k = 0; k < 3; k++) b.c[k] = 0.5f * (b.lo[k] + b.hi[k]);
    }
    /* BVH: built on the device (orx_bvh.hip) by default; the host builder
     * below is the reference implementation (ORX_BVH_HOST=1) and the only
     * one for the fp32-box variant */
    int bins = 32;
    uint32_t leaf_max = 8;
    float leaf_sah = 0.6f;
    if (const char* e = getenv("ORX_BVH_BINS")) bins = std::max(2, std::min(32, atoi(e)));
    if (const char* e = getenv("ORX_BVH_LEAF_MAX")) leaf_max = (uint32_t)std::max(1, std::min(8, atoi(e)));
    if (const char* e = getenv("ORX_BVH_LEAF_SAH")) leaf_sah = (float)atof(e);
    /* treelet restructuring sweeps of the binary tree and the SAH-optimal four-wide collapse (the refinement
     * OptiX's Trbvh does, Scene.cpp:353): hall photon-path node steps 17.71 -> 16.91 per ray, PPM frame +2.5 %,
     * VCM +2.6 % (profiles/r06j_bvh_treelet_ab.txt); ORX_BVH_TREELET=0 / ORX_BVH_COLLAPSE=0: the round-5 tree */
    int treelet_passes = 3;
    bool sah_collapse = true;
    if (const char* e = getenv("ORX_BVH_TREELET")) treelet_passes = std::max(0, std::min(8, atoi(e)));
    if (const char* e = getenv("ORX_BVH_COLLAPSE")) sah_collapse = atoi(e) != 0;
    int treelet_leaves = 9; /* ORX_BVH_TREELET_LEAVES: 9 or 7 (9: hall PPM +0.9 %, VCM +0.6 % over 7; 11 priced: no further gain) */
    if (const char* e = getenv("ORX_BVH_TREELET_LEAVES")) treelet_leaves = atoi(e) == 7 ? 7 : 9;
#ifdef ORX_BVH_FP32
    const bool device_bvh = false;
#else
    const char* host_env = getenv("ORX_BVH_HOST");
    const bool device_bvh = !(host_env && atoi(host_env));
#endif
    std::vector<uint32_t> leaf_order;
    uint32_t stack_bound = 0, nodes4 = 0;
    BvhBuilder bb;
    Bvh4Builder b4;
    if (nt && device_bvh) {
        DevBuf dV, dI;
        HIPCHK(r, dV.ensure((size_t)s->n_vertices * 12));
        HIPCHK(r, dI.ensure((size_t)nt * 12));
        HIPCHK(r, hipMemcpy(dV.p, s->vertices, (size_t)s->n_vertices * 12, hipMemcpyHostToDevice));
        HIPCHK(r, hipMemcpy(dI.p, s->triangles, (size_t)nt * 12, hipMemcpyHostToDevice));
        HIPCHK(r, r->d_bvh.ensure((size_t)nt * sizeof(DevBvh4) + 64));
        HIPCHK(r, r->d_bvhprims.ensure((size_t)nt * 4));
        uint32_t depth = 0;
        bool ok = false;
        HIPCHK(r, device_build_bvh4(r->stream, dV.as<float>(), dI.as<uint32_t>(), nt, bins, leaf_max, leaf_sah,
                                    treelet_passes, treelet_leaves, sah_collapse,
                                    r->d_bvh.as<DevBvh4>(), nt, r->d_bvhprims.as<uint32_t>(), &nodes4, &stack_bound,
                                    &depth, &ok));
        if (!ok) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "device BVH build failed (quantisation or capacity)");
        if (depth >= ORX_BVH_STACK) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "BVH deeper than the traversal stack");
        leaf_order.resize(nt);
        HIPCHK(r, hipMemcpy(leaf_order.data(), r->d_bvhprims.p, (size_t)nt * 4, hipMemcpyDeviceToHost));
    } else if (nt) {
        bb.tris = &bt;
        bb.bins = bins;
        bb.leaf_max = leaf_max;
        bb.leaf_sah = leaf_sah;
        bb.prims.resize(nt);
        for (uint32_t i = 0; i < nt; i++) bb.prims[i] = i;
        bb.nodes.reserve(2 * (size_t)nt / 2 + 1);
        bb.build(0, nt);
        if (treelet_passes > 0) { /* the device builder's sweeps, on the host tree (TreeletOpt) */
            TreeletOpt to(bb.nodes, leaf_sah > 0.f ? leaf_sah : 0.6f);
            to.nl = (size_t)treelet_leaves;
            for (int p = 0; p < treelet_passes; p++) to.pass();
            bb.max_depth = to.depth(0);
        }
        if (bb.max_depth >= ORX_BVH_STACK)
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "BVH deeper than the traversal stack");
        b4.b2 = &bb.nodes;
        b4.out.reserve(bb.nodes.size() / 2 + 1);
        if (sah_collapse) b4.dp(0);
        b4.build(0, stack_bound);
        if (!b4.ok) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "BVH4 quantisation failed");
        leaf_order = bb.prims;
        nodes4 = (uint32_t)b4.out.size();
    }
    if (stack_bound > 96) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "BVH4 traversal stack bound above 96");
    std::vector<float4> tv((size_t)nt * 3), tn, tt, tbt;
    std::vector<float2> tuv;
    std::vector<uint32_t> tmat_leaf(nt);
    const bool has_tb = s->normals && s->tangents && s->bitangents; /* TriangleMesh.cu:56-70 */
    if (s->normals) tn.resize((size_t)nt * 3);
    if (s->texcoords) tuv.resize((size_t)nt * 3);
    if (has_tb) tt.resize((size_t)nt * 3), tbt.resize((size_t)nt * 3);
    for (uint32_t k = 0; k < nt; k++) {
        const uint32_t i = leaf_order[k];
        tmat_leaf[k] = s->triangle_material[i];
        for (int v = 0; v < 3; v++) {
            uint32_t vi = s->triangles[3 * (size_t)i + v];
            const float* p = s->vertices + 3 * (size_t)vi;
            float w = 0.f;
            if (v == 0) std::memcpy(&w, &i, 4);
            tv[3 * (size_t)k + v] = make_float4(p[0], p[1], p[2], w);
            if (s->normals) {
                const float* n = s->normals + 3 * (size_t)vi;
                tn[3 * (size_t)k + v] = make_float4(n[0], n[1], n[2], 0.f);
            }
            if (s->texcoords) tuv[3 * (size_t)k + v] = make_float2(s->texcoords[2 * (size_t)vi], s->texcoords[2 * (size_t)vi + 1]);
            if (has_tb) {
                const float* t = s->tangents + 3 * (size_t)vi;
                const float* b = s->bitangents + 3 * (size_t)vi;
                tt[3 * (size_t)k + v] = make_float4(t[0], t[1], t[2], 0.f);
                tbt[3 * (size_t)k + v] = make_float4(b[0], b[1], b[2], 0.f);
            }
        }
    }
    auto up = [&](DevBuf& b, const void* src, size_t bytes) -> hipError_t {
        hipError_t e = b.ensure(bytes);
        if (e != hipSuccess) return e;
        if (bytes) return hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice);
        return hipSuccess;
    };
    HIPCHK(r, up(r->d_quads, quads.data(), quads.size() * sizeof(DevQuad)));
    HIPCHK(r, up(r->d_qmat, s->quad_material, (size_t)nq * 4));
    HIPCHK(r, up(r->d_spheres, sph.data(), sph.size() * sizeof(DevSphere)));
    HIPCHK(r, up(r->d_smat, s->spheres ? s->sphere_material : nullptr, (size_t)ns * 4));
    HIPCHK(r, up(r->d_triv, tv.data(), tv.size() * sizeof(float4)));
    HIPCHK(r, up(r->d_trin, tn.data(), tn.size() * sizeof(float4)));
    HIPCHK(r, up(r->d_tmat, tmat_leaf.data(), (size_t)nt * 4));
    HIPCHK(r, up(r->d_mats, mats.data(), mats.size() * sizeof(DevMaterial)));
    HIPCHK(r, up(r->d_triuv, tuv.data(), tuv.size() * sizeof(float2)));
    HIPCHK(r, up(r->d_trit, tt.data(), tt.size() * sizeof(float4)));
    HIPCHK(r, up(r->d_tribt, tbt.data(), tbt.size() * sizeof(float4)));
    /* texture images back to back (256-B aligned), descriptors with device pointers */
    std::vector<DevTexture> texd(s->n_textures);
    {
        size_t total = 0;
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        for (uint32_t i = 0; i < s->n_textures; i++) {
            const orx_texture& t = s->textures[i];
            total += al((size_t)t.width * t.height * 4);
            if (t.normal_rgba) total += al((size_t)t.normal_width * t.normal_height * 4);
        }
        HIPCHK(r, r->d_texels.ensure(total));
        size_t off = 0;
        uint8_t* base = r->d_texels.as<uint8_t>();
        for (uint32_t i = 0; i < s->n_textures; i++) {
            const orx_texture& t = s->textures[i];
            DevTexture& d = texd[i];
            std::memset(&d, 0, sizeof d);
            d.w = t.width;
            d.h = t.height;
            d.rgba = base + off;
            HIPCHK(r, hipMemcpy(base + off, t.rgba, (size_t)t.width * t.height * 4, hipMemcpyHostToDevice));
            off += al((size_t)t.width * t.height * 4);
            if (t.normal_rgba) {
                d.nw = t.normal_width;
                d.nh = t.normal_height;
                d.nrgba = base + off;
                HIPCHK(r, hipMemcpy(base + off, t.normal_rgba, (size_t)t.normal_width * t.normal_height * 4,
                                    hipMemcpyHostToDevice));
                off += al((size_t)t.normal_width * t.normal_height * 4);
            }
        }
    }
    HIPCHK(r, up(r->d_texdesc, texd.data(), texd.size() * sizeof(DevTexture)));
    r->has_tex = false;
    for (const DevMaterial& m : mats) r->has_tex |= m.type == ORX_MAT_TEXTURE;
    HIPCHK(r, up(r->d_lights, lights.data(), lights.size() * sizeof(DevLight)));
#ifdef ORX_BVH_FP32
    HIPCHK(r, up(r->d_bvh, b4.outf.data(), b4.outf.size() * sizeof(DevBvh4F)));
#else
    if (!device_bvh) HIPCHK(r, up(r->d_bvh, b4.out.data(), b4.out.size() * sizeof(DevBvh4)));
#endif
    DevScene& S = r->scene;
    S.nq = nq;
    S.ns = ns;
    S.nt = nt;
    S.quads = r->d_quads.as<DevQuad>();
    S.qmat = r->d_qmat.as<uint32_t>();
    S.spheres = r->d_spheres.as<DevSphere>();
    S.smat = r->d_smat.as<uint32_t>();
    S.tri_v = r->d_triv.as<float4>();
    S.tri_n = s->normals ? r->d_trin.as<float4>() : nullptr;
    S.tmat = r->d_tmat.as<uint32_t>();
    S.tri_uv = s->texcoords && nt ? r->d_triuv.as<float2>() : nullptr;
    S.tri_t = has_tb && nt ? r->d_trit.as<float4>() : nullptr;
    S.tri_bt = has_tb && nt ? r->d_tribt.as<float4>() : nullptr;
    S.tex = r->d_texdesc.as<DevTexture>();
    S.ntex = s->n_textures;
    S.mats = r->d_mats.as<DevMaterial>();
    S.lights = r->d_lights.as<DevLight>();
    S.nl = s->n_lights;
    S.bvh4 = r->d_bvh.as<DevNode4>();
    S.bvh_nodes = nodes4;
    S.stack_entries = nt ? stack_bound + 1 : 0;
#ifdef ORX_TRAV_STATS
    HIPCHK(r, r->d_tstats.ensure(256));
    HIPCHK(r, hipMemset(r->d_tstats.p, 0, 256));
    S.trav_stats = r->d_tstats.as<unsigned long long>();
#else
    S.trav_stats = nullptr;
#endif
    /* AAB::getBoundingSphere (math/AAB.cpp:26-33) with Vector3::length's
     * dot bug a.z*b.x (math/Vector3.cpp:27-30) */
    f3 lo = ld3(s->aabb_min), hi = ld3(s->aabb_max);
    r->aabb_lo = lo;
    r->aabb_hi = hi;
    f3 center = (lo + hi) * 0.5f;
    f3 e = hi - center;
    S.bs_cx = center.x;
    S.bs_cy = center.y;
    S.bs_cz = center.z;
    S.bs_r = sqrtf(e.x * e.x + e.y * e.y + e.z * e.x);
    r->vcm_estimated = false;
    r->scene_ready = true;
    return photon_stack_ensure(r);
}

/* the photon pass's deep traversal-stack entries: (stack bound + 2 - its LDS entries) per photon of
 * the device (1.4 GB for 4096^2 photons on the conference room; touched only by paths whose stack
 * outgrows LDS); sized again whenever a scene or a resize comes in */
static orx_status photon_stack_ensure(orx_renderer* r) {
    const size_t lanes = ((size_t)r->pb.prows * r->pb.PW + 63) / 64 * 64;
    const uint32_t deep = photon_stack_deep(r->scene.stack_entries);
    HIPCHK(r, r->d_ptrav.ensure(256 + (size_t)deep * lanes * 4));
    r->pb.tstk = r->d_ptrav.as<uint32_t>();
    r->pb.tlanes = (uint32_t)lanes;
    r->pb.tdeep = deep;
    return ORX_OK;
}
static orx_status resize(orx_renderer* r, uint32_t W, uint32_t H) {
    const uint32_t PW = r->cfg.photon_launch_width, PH = r->cfg.photon_launch_height;
    const bool hash = r->cfg.photon_map == 1;
    /* slots per emitted photon: the deposit limit (uniform grid), or room for every non-specular
     * hit at depth 1..max depth - 1 (stochastic hash: store_photon.h never counts deposits) */
    const uint32_t D = hash ? std::min(r->cfg.max_photon_trace_depth, 8u) : r->cfg.max_photon_deposits;
    r->fin_due = r->fin_snap = false; /* a finish held back across a resize is dropped with its buffers */
    r->W = W;
    r->H = H;
    r->RW = std::max(PW, W);
    r->RH = std::max(PH, H);
    auto local_rows = [&](uint32_t n) { return n > r->rank ? (n - r->rank + r->world - 1) / r->world : 0u; };
    r->rows = local_rows(H);
    r->rng_rows = local_rows(r->RH);
    r->prows = local_rows(PH);
    r->max_rows = (H + r->world - 1) / r->world;
    const size_t nhp = (size_t)r->max_rows * W; /* hitpoint planes padded to max_rows */
    const size_t nslot_rng = (size_t)r->rng_rows * r->RW;
    const size_t nphot = (size_t)r->prows * PW;
    const size_t S = nphot * D;
    /* slab mode: room for every deposit slot of the global launch (the photons this rank imports) */
    const size_t S_cap = r->slab ? std::max(S, (size_t)PW * PH * D) : S;
    r->S_cap = S_cap;
    const size_t G2 = (size_t)r->cfg.photon_grid_max_size + 2;
    HIPCHK(r, r->d_rng.ensure(nslot_rng * 24));
    HIPCHK(r, r->d_hp.ensure(nhp * 40));
    HIPCHK(r, r->d_ind.ensure(nhp * 12));
    HIPCHK(r, r->d_dir.ensure(nhp * 12));
    HIPCHK(r, r->d_out.ensure(nhp * 12));
    HIPCHK(r, r->d_dbg.ensure(nhp * 8));
    if (r->media) { /* volumetricRadiance per pixel, last volumetric event per photon */
        HIPCHK(r, r->d_volR.ensure(nhp * 12));
        HIPCHK(r, r->d_ev_a.ensure(nphot * 16 + 16));
        HIPCHK(r, r->d_ev_b.ensure(nphot * 16 + 16));
        HIPCHK(r, hipMemsetAsync(r->d_volR.p, 0, nhp * 12, r->stream));
        r->vm.valid = 0;
    }
    HIPCHK(r, r->d_slots.ensure(S_cap * 64));
    HIPCHK(r, r->d_vmask.ensure(S_cap / D + 1));
    /* 64 photons of tail padding per plane: the union gather loads whole 64-photon chunks, up to
     * index U1 + 63 of the last plane */
    const size_t splane = ((S_cap + 64) + 3) & ~(size_t)3;
    if ((size_t)SP_PLANES * splane * 4 > 0xffffff00ull) /* the gather addresses the planes with 32-bit buffer offsets */
        return set_err(r, ORX_ERR_UNSUPPORTED, "photon slots per device exceed the 4 GiB sorted-photon window");
    HIPCHK(r, r->d_sorted.ensure(SP_PLANES * splane * 4));
    HIPCHK(r, r->d_perm.ensure(S_cap * 4 + 16));
    HIPCHK(r, hipMemsetAsync(r->d_sorted.p, 0, SP_PLANES * splane * 4, r->stream)); /* tail reads stay finite */
    HIPCHK(r, r->d_keys.ensure(S_cap * 4));
    HIPCHK(r, r->d_offsets.ensure(G2 * 4));
    HIPCHK(r, r->d_bbox.ensure(6 * BBOX_REPLICAS * 4));
    HIPCHK(r, r->d_grid.ensure(sizeof(GridParams)));
    /* bucket-sort grid build: at most 2048 buckets of 2^bshift virtual cells
     * (nsub sub-rows per cell row, k_bs_count) */
    /* sub-row layout on one device; a row-partition shard of world >= 2 gathers all W*H hit points
     * against 1/N of the photons and runs faster on whole cell rows (tools/shard_model.py, hall
     * 1080p: per-rank gather N=2 1.40 -> 1.32 ms, N=8 0.96 -> 0.90 ms, grid build shorter too);
     * a slab shard holds the single-device photon density in its cells: sub-rows (configs[4]
     * N=2 rank 0: 47 ms gather in cell order) */
    const bool cell_order =
        r->cfg.gather_variant == 1 || (r->cfg.gather_variant == 0 && r->world >= 2 && !r->slab);
    const uint32_t nsub = cell_order ? 1u : SUBR * SUBR;
    const size_t vmax = (size_t)r->cfg.photon_grid_max_size * nsub;
    uint32_t bshift = 10;
    while (((vmax + (1u << bshift) - 1) >> bshift) > 2048) bshift++;
    const size_t bs_nchunk = (S + 16383) / 16384;
    const size_t bs_nchunk_cap = (S_cap + 16383) / 16384;
    const size_t bs_nbmax = (vmax + (1u << bshift) - 1) >> bshift;
    const size_t bs_nscan = (bs_nbmax * bs_nchunk_cap + 1023) / 1024;
    HIPCHK(r, r->d_pos4.ensure(S_cap * 16 + 16));
    HIPCHK(r, r->d_bstable.ensure(bs_nbmax * bs_nchunk_cap * 4 + 16));
    HIPCHK(r, r->d_bspartials.ensure((bs_nscan + 2) * 4));
    HIPCHK(r, r->d_bspairs.ensure(S_cap * 8 + 16));
    HIPCHK(r, r->d_subofs.ensure(G2 * 4 * SUBX * nsub + 16));
    /* the second buffer set of PPM pipelining is allocated on the first pipelined iteration
     * (ensure_second_set); the sharded pipeline (orx_set_ppm_pipeline) wants it at once */
    r->pipe_bufs = false;
    r->pend = false;
    HIPCHK(r, hipMemsetAsync(r->d_offsets.p, 0, G2 * 4, r->stream));
    HIPCHK(r, hipMemsetAsync(r->d_vmask.p, 0, S_cap / D + 1, r->stream));
    HIPCHK(r, hipMemsetAsync(r->d_grid.p, 0, sizeof(GridParams), r->stream));
    HIPCHK(r, hipMemsetAsync(r->d_out.p, 0, nhp * 12, r->stream));
    HIPCHK(r, hipMemsetAsync(r->d_hp.p, 0, nhp * 40, r->stream)); /* pad rows: flags 0 */
    HIPCHK(r, hipMemsetAsync(r->d_bbox.p, 0xff, 3 * BBOX_REPLICAS * 4, r->stream));
    HIPCHK(r, hipMemsetAsync(r->d_bbox.as<uint32_t>() + 3 * BBOX_REPLICAS, 0, 3 * BBOX_REPLICAS * 4, r->stream));

    PixelBufs& px = r->px;
    px.W = W;
    px.H = H;
    px.rank = r->rank;
    px.world = r->world;
    px.rows = r->rows;
    px.RW = r->RW;
    for (int k = 0; k < 6; k++) px.rng.p[k] = r->d_rng.as<uint32_t>() + k * nslot_rng;
    px.hpA = r->d_hp.as<float4>();
    px.hpB = r->d_hp.as<float4>() + nhp;
    px.hpC = (float2*)(r->d_hp.as<float4>() + 2 * nhp);
    px.seg_rows = r->max_rows;
    px.indirect = r->d_ind.as<float>();
    px.direct = r->d_dir.as<float>();
    px.output = r->d_out.as<float>();
    px.dbg = r->cfg.debug_counters ? r->d_dbg.as<uint32_t>() : nullptr;
    PhotonBufs& pb = r->pb;
    pb.PW = PW;
    pb.PH = PH;
    pb.prows = r->prows;
    pb.D = D;
    pb.S = (uint32_t)S;
    pb.hash = hash ? 1u : 0u;
    pb.Dlim = hash ? 0xffffffffu : D;
    pb.hnum = 0;
    pb.hcount = pb.hwin = nullptr;
    if (hash) {
        const size_t hnum = (size_t)PW * PH * r->cfg.max_photon_deposits; /* NUM_PHOTONS */
        HIPCHK(r, r->d_hcount.ensure(hnum * 4));
        HIPCHK(r, r->d_hwin.ensure(hnum * 4));
        pb.hnum = (uint32_t)hnum;
        pb.hcount = r->d_hcount.as<uint32_t>();
        pb.hwin = r->d_hwin.as<uint32_t>();
    }
    {
        const orx_status st = photon_stack_ensure(r);
        if (st != ORX_OK) return st;
    }
    if (r->cfg.photon_map == 2) {
        /* m_photonKdTreeSize = pow2roundup(NUM_PHOTONS + 1) - 1 (OptixRenderer.cpp:65-74, :207) */
        uint32_t t = (uint32_t)S;
        t |= t >> 1;
        t |= t >> 2;
        t |= t >> 4;
        t |= t >> 8;
        t |= t >> 16;
        const size_t tree = (size_t)t; /* pow2roundup(S + 1) - 1 */
        uint32_t levels = 0;
        while (((size_t)1 << levels) - 1 < tree) levels++;
        const size_t nblk = (S + 1023) / 1024;
        const size_t ntiles = (S + 4095) / 4096;
        const size_t tp = std::max((256 * ntiles + 1023) / 1024, (6 * nblk + 1023) / 1024) + 16;
        HIPCHK(r, r->d_kdtree.ensure(tree * 48 + 48));
        HIPCHK(r, r->d_kdids.ensure(6 * S * 4 + 64));
        HIPCHK(r, r->d_kdkeys.ensure(2 * S * 4 + 64));
        HIPCHK(r, r->d_kdnodepos.ensure(S * 4 + 16));
        HIPCHK(r, r->d_kdlst.ensure(6 * S * 16 + 64));
        HIPCHK(r, r->d_kdnkey.ensure(tree * 8 + 16));
        HIPCHK(r, r->d_kdseg.ensure(tree * 8 + 16));
        HIPCHK(r, r->d_kdbox.ensure(tree * 24 + 24));
        HIPCHK(r, r->d_kdninfo.ensure(tree * 4 + 16));
        HIPCHK(r, r->d_kdP.ensure(tree * 12 + 64));
        HIPCHK(r, r->d_kdppart.ensure(6 * nblk * 4 + 64));
        HIPCHK(r, r->d_kdtable.ensure(256 * ntiles * 4 + 64));
        HIPCHK(r, r->d_kdtpart.ensure(tp * 4));
        HIPCHK(r, r->d_kdvpart.ensure(nblk * 4 + 64));
        HIPCHK(r, r->d_kdcount.ensure(64));
        HIPCHK(r, hipMemsetAsync(r->d_kdtree.p, 0, tree * 48 + 48, r->stream));
        KdBufs& kd = r->kd;
        kd.S = (uint32_t)S;
        kd.tree_size = (uint32_t)tree;
        kd.levels = levels;
        kd.ntiles = (uint32_t)ntiles;
        kd.tree = r->d_kdtree.as<float4>();
        kd.tree_bc = kd.tree + tree + 1;
        for (int q = 0; q < 2; q++)
            for (int a = 0; a < 3; a++) {
                kd.ids[q][a] = r->d_kdids.as<uint32_t>() + (size_t)(3 * q + a) * S;
                kd.lst[q][a] = r->d_kdlst.as<float4>() + (size_t)(3 * q + a) * S;
            }
        kd.keys[0] = r->d_kdkeys.as<uint32_t>();
        kd.keys[1] = kd.keys[0] + S;
        kd.nodepos = r->d_kdnodepos.as<uint32_t>();
        kd.nkey = r->d_kdnkey.as<uint2>();
        kd.seg = r->d_kdseg.as<uint2>();
        kd.box = r->d_kdbox.as<float>();
        kd.ninfo = r->d_kdninfo.as<uint32_t>();
        kd.nodeP = r->d_kdP.as<uint32_t>();
        kd.ppart = r->d_kdppart.as<uint32_t>();
        kd.table = r->d_kdtable.as<uint32_t>();
        kd.tpart = r->d_kdtpart.as<uint32_t>();
        kd.vpart = r->d_kdvpart.as<uint32_t>();
        kd.count = r->d_kdcount.as<uint32_t>();
        HIPCHK(r, hipMemsetAsync(r->d_kdcount.p, 0, 64, r->stream));
    }
    pb.gmax = r->cfg.photon_grid_max_size;
    /* ORX_SHARD_CELLS=2: a row shard of world N sizes its cells for gmax / N cells (N times the
     * single-device volume, the single-device photons per cell; the accepted set does not depend on
     * the cell size).  Measured slower (tools/shard_model.py, N = 8: configs[4] per-rank gather
     * 5.96 -> 8.43 ms in cell order, 5.82 -> 6.24 ms on sub-rows; hall 0.42 ms either way): a
     * window of radius r ~ one single-device cell then walks 2^3 cells of twice the edge, about 2.4x
     * the volume of the 3^3 it walks otherwise, so the default keeps single-device cells */
    {
        static const int scaled = [] {
            const char* e = getenv("ORX_SHARD_CELLS");
            return e && atoi(e) == 2 ? 1 : 0;
        }();
        pb.gcells = (r->world >= 2 && !r->slab && scaled) ? std::max(1u, pb.gmax / r->world) : pb.gmax;
    }
    pb.slots = r->d_slots.as<float4>();
    pb.vmask = r->d_vmask.as<uint8_t>();
    pb.sorted = r->d_sorted.as<float>();
    pb.splane = (uint32_t)splane;
    pb.perm = r->d_perm.as<uint32_t>();
    pb.keys = r->d_keys.as<uint32_t>();
    pb.offsets = r->d_offsets.as<uint32_t>();
    pb.bbox = r->d_bbox.as<uint32_t>();
    pb.grid = r->d_grid.as<GridParams>();
    pb.pos4 = r->d_pos4.as<float4>();
    pb.bshift = bshift;
    pb.nsub = nsub;
    pb.bs_nchunk = (uint32_t)bs_nchunk;
    pb.bs_table = r->d_bstable.as<uint32_t>();
    pb.bs_partials = r->d_bspartials.as<uint32_t>();
    pb.bs_pairs = r->d_bspairs.as<uint2>();
    pb.subofs = r->d_subofs.as<uint32_t>();

    /* initializeRandomStates (OptixRenderer_SpatialHash.cu:310-347) */
    uint32_t seed = r->cfg.seed;
    if (seed == 0) seed = 574133u * (uint32_t)clock() + (uint32_t)(47844152748ull * (uint32_t)time(NULL));
    launch_rng_init(r->stream, px.rng, r->RW, r->rng_rows, r->rank, r->world, seed);
    HIPCHK(r, hipGetLastError());
    r->rng_ready = true;
    return ORX_OK;
}

/* roctx ranges around every pass (the role of the reference's NVTX ranges,
 * renderer/helpers/nsight.h:17-199): visible in `rocprofv3 --marker-trace`;
 * they span the host-side enqueue, the HIP events above time the device work */
static const char* const PASS_NAME[P_COUNT] = {
    "OptixEntryPoint::RAYTRACE_PASS (ppm_eye)",   "OptixEntryPoint::PHOTON_PASS (ppm_photon)",
    "Creating photon map (grid_hash)",            "Creating photon map (grid_scan)",
    "Creating photon map (grid_scatter)",         "OptixEntryPoint::INDIRECT_RADIANCE_ESTIMATION (ppm_gather)",
    "OptixEntryPoint::PPM_DIRECT_RADIANCE_ESTIMATION_PASS (ppm_direct_output)",
    "OptixEntryPoint::PT_RAYTRACE_PASS (pt)",     "OptixEntryPoint::VCM_LIGHT_PASS (vcm_light)",
    "OptixEntryPoint::VCM_CAMERA_PASS (vcm_camera)", "OptixEntryPoint::VCM_CAMERA_PASS (vcm_shadow)"};
static inline void ev_begin(orx_renderer* r, int p) {
    roctxRangePushA(PASS_NAME[p]);
    if (!r->timing || r->ev_n[p] >= EV_POOL) return;
    auto& v = r->ev[p];
    size_t need = 2 * (size_t)r->ev_n[p] + 2;
    while (v.size() < need) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        v.push_back(e);
    }
    hipEventRecord(v[2 * r->ev_n[p]], r->use_ext ? r->ext_stream : r->stream);
}
static inline void ev_end(orx_renderer* r, int p) {
    roctxRangePop();
    if (!r->timing || r->ev_n[p] >= EV_POOL || r->ev[p].size() < 2 * (size_t)r->ev_n[p] + 2) return;
    hipEventRecord(r->ev[p][2 * r->ev_n[p] + 1], r->use_ext ? r->ext_stream : r->stream);
    r->ev_n[p]++;
}
/* the same on an explicit stream (the overlapped direct pass) */
static inline void ev_begin_on(orx_renderer* r, int p, hipStream_t st) {
    roctxRangePushA(PASS_NAME[p]);
    if (!r->timing || r->ev_n[p] >= EV_POOL) return;
    auto& v = r->ev[p];
    while (v.size() < 2 * (size_t)r->ev_n[p] + 2) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        v.push_back(e);
    }
    hipEventRecord(v[2 * r->ev_n[p]], st);
}
static inline void ev_end_on(orx_renderer* r, int p, hipStream_t st) {
    roctxRangePop();
    if (!r->timing || r->ev_n[p] >= EV_POOL || r->ev[p].size() < 2 * (size_t)r->ev_n[p] + 2) return;
    hipEventRecord(r->ev[p][2 * r->ev_n[p] + 1], st);
    r->ev_n[p]++;
}

static inline hipStream_t cur_stream(orx_renderer* r) { return r->use_ext ? r->ext_stream : r->stream; }
/* the stream the deferred gather + output run on */
static inline hipStream_t gather_stream(orx_renderer* r) { return r->shard_pipe ? r->side : r->gstream; }

/* order everything later on the renderer's stream (and the gather stream) after a VCM camera
 * pass's resolve half still running on aux */
static void flush_vcm(orx_renderer* r) {
    if (!r->vcm_pend) return;
    hipStreamWaitEvent(cur_stream(r), r->ev_vacc, 0);
    if (r->gstream) hipStreamWaitEvent(r->gstream, r->ev_vacc, 0);
    r->vcm_pend = false;
}
/* order everything later on the renderer's stream after a deferred gather + output */
static void flush_pipeline(orx_renderer* r) {
    flush_vcm(r);
    r->eye_chain = false;
    if (!r->pend) return;
    hipStreamWaitEvent(cur_stream(r), r->ev_gdone[r->pp], 0);
    r->pend = false;
}

static orx_status sync_all(orx_renderer* r) {
    flush_pipeline(r);
    HIPCHK(r, hipStreamSynchronize(r->stream));
    HIPCHK(r, hipStreamSynchronize(r->aux));
    if (r->use_ext) HIPCHK(r, hipStreamSynchronize(r->ext_stream));
    if (r->gstream) HIPCHK(r, hipStreamSynchronize(r->gstream));
    if (r->gridq) HIPCHK(r, hipStreamSynchronize(r->gridq));
    if (r->shard_pipe) HIPCHK(r, hipStreamSynchronize(r->side));
    return ORX_OK;
}

/* The second buffer set of PPM pipelining: only what the photon map of the renderer
 * alternates between consecutive iterations (the buffers the deferred gather of iteration i
 * reads while iteration i+1 writes its own): hit points, direct light, grid parameters, and
 * the uniform grid's sorted photons and offsets, or the hash's deposit records and table, or
 * the kd-tree.  Allocated on the first pipelined iteration after a resize, so PT/VCM-only
 * renderers and the serial schedule never hold it. */
/* one extra set: the views of set `n` (2 or 3) */
struct SetBufs {
    DevBuf *hp, *dir, *grid, *sorted, *subofs, *offsets, *hcount, *hwin, *slots, *kdtree;
};
static SetBufs set_bufs(orx_renderer* r, int n) {
    if (n == 2)
        return SetBufs{&r->d_hp2, &r->d_dir2, &r->d_grid2, &r->d_sorted2, &r->d_subofs2, &r->d_offsets2,
                       &r->d_hcount2, &r->d_hwin2, &r->d_slots2, &r->d_kdtree2};
    return SetBufs{&r->d_hp3, &r->d_dir3, &r->d_grid3, &r->d_sorted3, &r->d_subofs3, &r->d_offsets3,
                   &r->d_hcount3, &r->d_hwin3, &r->d_slots3, &r->d_kdtree3};
}
static orx_status ensure_set(orx_renderer* r, const SetBufs& b) {
    const size_t nhp = (size_t)r->max_rows * r->W;
    HIPCHK(r, b.hp->ensure(nhp * 40));
    HIPCHK(r, hipMemsetAsync(b.hp->p, 0, nhp * 40, r->stream));
    HIPCHK(r, b.dir->ensure(nhp * 12));
    HIPCHK(r, b.grid->ensure(sizeof(GridParams)));
    HIPCHK(r, hipMemsetAsync(b.grid->p, 0, sizeof(GridParams), r->stream));
    const size_t G2 = (size_t)r->cfg.photon_grid_max_size + 2;
    if (r->cfg.photon_map == 0) {
        const size_t bytes = (size_t)SP_PLANES * r->pb.splane * 4;
        HIPCHK(r, b.sorted->ensure(bytes));
        HIPCHK(r, hipMemsetAsync(b.sorted->p, 0, bytes, r->stream)); /* tail reads stay finite */
        HIPCHK(r, b.subofs->ensure(r->d_subofs.bytes));
        HIPCHK(r, b.offsets->ensure(G2 * 4));
        HIPCHK(r, hipMemsetAsync(b.offsets->p, 0, G2 * 4, r->stream));
    } else if (r->cfg.photon_map == 1) {
        HIPCHK(r, b.hcount->ensure((size_t)r->pb.hnum * 4));
        HIPCHK(r, b.hwin->ensure((size_t)r->pb.hnum * 4));
        HIPCHK(r, b.slots->ensure((size_t)r->pb.S * 64));
    } else {
        const size_t bytes = (size_t)r->kd.tree_size * 48 + 48;
        HIPCHK(r, b.kdtree->ensure(bytes));
        HIPCHK(r, hipMemsetAsync(b.kdtree->p, 0, bytes, r->stream));
    }
    return ORX_OK;
}
/* The further buffer sets of PPM pipelining: only what the photon map of the renderer
 * alternates between iterations (the buffers the deferred gather of iteration i reads while the
 * next iterations write their own): hit points, direct light, grid parameters, and the uniform
 * grid's sorted photons and offsets, or the hash's deposit records and table, or the kd-tree.
 * Allocated on the first pipelined iteration after a resize, so PT/VCM-only renderers and the
 * serial schedule never hold them.  One device takes three sets (ORX_PIPE_SETS=2: two): with two,
 * the eye pass of iteration i + 1 waited for the gather and output of i - 1, which on the hall ran
 * until the grid build of i had ended, and the photon pass of i + 1 then waited ~1 ms per frame for
 * that eye pass (kernel trace gpurun_out/r06n_tl); the sharded pipeline keeps two (its finish may
 * be held back one iteration, orx_ppm_finish_on). */
static orx_status ensure_second_set(orx_renderer* r) {
    if (r->pipe_bufs) return ORX_OK;
    static const uint32_t sets_env = [] {
        const char* e = getenv("ORX_PIPE_SETS");
        return e && atoi(e) == 2 ? 2u : 3u;
    }();
    r->nsets = r->shard_pipe ? 2u : sets_env;
    for (uint32_t n = 2; n <= r->nsets; n++) {
        const orx_status s0 = ensure_set(r, set_bufs(r, (int)n));
        if (s0 != ORX_OK) return s0;
    }
    /* The asynchronous grid build (ORX_GRID_ASYNC=1) pays where the chain eye -> photon -> grid -> next
     * photon sets the frame (hall: 1059 -> 1071 Mpaths/s); where the gather does it only reorders a
     * throughput-bound frame and costs 1-2 % (Cornell 2056 -> 2012, conference 4K 585 -> 578;
     * profiles/r06p_grid_async_ab.txt), so it is off by default. */
    static const int async_env = [] {
        const char* e = getenv("ORX_GRID_ASYNC");
        return e ? atoi(e) : -1;
    }();
    const bool eligible = r->nsets == 3 && r->cfg.photon_map == 0 && !r->media;
    r->async_grid = eligible && async_env > 0;
    r->probe_stage = eligible && async_env < 0 ? 1u : 0u;
    r->probe_ms[0] = r->probe_ms[1] = 0.f;
    r->out_b = eligible && async_env != 0;
    if (r->out_b) { /* the photon pass's second output set (the first is resize's) */
        HIPCHK(r, r->d_slotsB.ensure(r->d_slots.bytes));
        HIPCHK(r, r->d_vmaskB.ensure(r->d_vmask.bytes));
        HIPCHK(r, hipMemsetAsync(r->d_vmaskB.p, 0, r->d_vmaskB.bytes, r->stream));
        HIPCHK(r, r->d_pos4B.ensure(r->d_pos4.bytes));
        HIPCHK(r, r->d_bboxB.ensure(r->d_bbox.bytes));
        HIPCHK(r, hipMemsetAsync(r->d_bboxB.p, 0xff, 3 * BBOX_REPLICAS * 4, r->stream));
        HIPCHK(r, hipMemsetAsync(r->d_bboxB.as<uint32_t>() + 3 * BBOX_REPLICAS, 0, 3 * BBOX_REPLICAS * 4, r->stream));
        /* both sets' last-reader events exist from here on, so a wait on either is valid */
        HIPCHK(r, hipEventRecord(r->ev_gsrc[0], r->stream));
        HIPCHK(r, hipEventRecord(r->ev_gsrc[1], r->stream));
        for (hipEvent_t& e : r->ev_pm)
            if (!e) HIPCHK(r, hipEventCreate(&e));
    }
    r->set_id[0] = 0;
    r->set_id[1] = 1;
    r->set_id[2] = 2;
    r->pp = 0;
    /* the zero-fills above ran on the own stream; on a caller stream (the sharded pipeline) the
     * eye pass and grid build of this iteration write these buffers right after swap_sets */
    if (r->use_ext) HIPCHK(r, hipStreamSynchronize(r->stream));
    r->pipe_bufs = true;
    return ORX_OK;
}

static inline void swap_buf(DevBuf& a, DevBuf& b) {
    std::swap(a.p, b.p);
    std::swap(a.bytes, b.bytes);
}
/* the current view slot takes the next buffer set: with two sets the other one, with three the least recently
 * used ((cur, prev, prev2) -> (prev2, cur, prev)); then point the kernels' views at it */
static void cycle(orx_renderer* r, DevBuf& a, DevBuf& b, DevBuf& c) {
    if (r->nsets == 3) {
        swap_buf(a, c); /* (c, b, a) */
        swap_buf(b, c); /* (c, a, b) */
    } else {
        swap_buf(a, b);
    }
}
static void swap_sets(orx_renderer* r) {
    cycle(r, r->d_hp, r->d_hp2, r->d_hp3);
    cycle(r, r->d_dir, r->d_dir2, r->d_dir3);
    cycle(r, r->d_grid, r->d_grid2, r->d_grid3);
    if (r->cfg.photon_map == 0) {
        cycle(r, r->d_sorted, r->d_sorted2, r->d_sorted3);
        cycle(r, r->d_subofs, r->d_subofs2, r->d_subofs3);
        cycle(r, r->d_offsets, r->d_offsets2, r->d_offsets3);
    }
    if (r->cfg.photon_map == 1) { /* the hash gather reads the deposit records and the table */
        cycle(r, r->d_slots, r->d_slots2, r->d_slots3);
        cycle(r, r->d_hcount, r->d_hcount2, r->d_hcount3);
        cycle(r, r->d_hwin, r->d_hwin2, r->d_hwin3);
        r->pb.slots = r->d_slots.as<float4>();
        r->pb.hcount = r->d_hcount.as<uint32_t>();
        r->pb.hwin = r->d_hwin.as<uint32_t>();
    }
    if (r->cfg.photon_map == 2) {
        cycle(r, r->d_kdtree, r->d_kdtree2, r->d_kdtree3);
        r->kd.tree = r->d_kdtree.as<float4>();
        r->kd.tree_bc = r->kd.tree + r->kd.tree_size + 1;
    }
    const size_t nhp = (size_t)r->max_rows * r->W;
    r->px.hpA = r->d_hp.as<float4>();
    r->px.hpB = r->d_hp.as<float4>() + nhp;
    r->px.hpC = (float2*)(r->d_hp.as<float4>() + 2 * nhp);
    r->px.direct = r->d_dir.as<float>();
    r->pb.sorted = r->d_sorted.as<float>();
    if (r->pb.subofs) r->pb.subofs = r->d_subofs.as<uint32_t>();
    r->pb.offsets = r->d_offsets.as<uint32_t>();
    r->pb.grid = r->d_grid.as<GridParams>();
    if (r->nsets == 3) {
        const uint32_t t = r->set_id[2];
        r->set_id[2] = r->set_id[1];
        r->set_id[1] = r->set_id[0];
        r->set_id[0] = t;
    } else {
        std::swap(r->set_id[0], r->set_id[1]);
    }
    r->pp = r->set_id[0];
}

static Consts make_consts(orx_renderer* r, float ppm_radius, uint64_t local_iteration_number) {
    Consts c;
    c.max_photon_depth = r->cfg.max_photon_trace_depth;
    c.max_radiance_depth = r->cfg.max_radiance_trace_depth;
    c.ppm_radius = ppm_radius;
    c.ppm_radius2 = ppm_radius * ppm_radius;
    /* emittedPhotonsPerIterationFloat: global launch (all ranks) */
    c.emitted_f = (float)(r->cfg.photon_launch_width * r->cfg.photon_launch_height);
    c.local_iteration = (uint32_t)(local_iteration_number != 0);
    c.media = r->media ? 1u : 0u;
    return c;
}

/* The volumetric table's grid for radius R (host): the box padded by 2R, cells >= 1.01 R and at
 * least the cube root of (volume / table slots), at most 1024 per axis (orx_device.h VolMap) */
static void vol_grid(orx_renderer* r, float R) {
    VolMap& vm = r->vm;
    vm.R = R;
    const f3 pad = mk1(2.f * R);
    vm.glo = vm.lo - pad;
    const f3 ext = (vm.hi + pad) - vm.glo;
    double cell = std::max((double)R * 1.01, std::cbrt((double)ext.x * ext.y * ext.z / (double)r->cfg.volumetric_photons));
    cell = std::max(cell, (double)std::max(ext.x, std::max(ext.y, ext.z)) / 1024.0);
    vm.cell = (float)cell * 1.0001f;
    const float e[3] = {ext.x, ext.y, ext.z};
    for (int k = 0; k < 3; k++) vm.n[k] = std::min(1024u, std::max(1u, (uint32_t)std::ceil(e[k] / vm.cell)));
    vm.G = vm.n[0] * vm.n[1] * vm.n[2];
    vm.ilo = vm.lo - mk1(R);
    vm.ihi = vm.hi + mk1(R);
}
static MediaBufs media_bufs(orx_renderer* r) {
    MediaBufs mb;
    mb.vm = r->vm;
    mb.vm.start = r->d_vstart.as<uint32_t>();
    mb.vm.rec = r->d_vrec.as<float4>();
    mb.volR = r->d_volR.as<float>();
    mb.ev_a = r->d_ev_a.as<float4>();
    mb.ev_b = r->d_ev_b.as<float4>();
    return mb;
}
/* after the photon pass: this pass's volumetric table, gathered by the next eye pass with this
 * iteration's radius (volumetricRadius = PPMRadius after the eye pass, OptixRenderer.cpp:592-593) */
static orx_status vol_build(orx_renderer* r, hipStream_t st, float R) {
    vol_grid(r, R);
    HIPCHK(r, r->d_vstart.ensure(((size_t)r->vm.G + 2) * 4));
    VolBuild vb;
    vb.ev_a = r->d_ev_a.as<float4>();
    vb.ev_b = r->d_ev_b.as<float4>();
    vb.nphot = r->prows * r->cfg.photon_launch_width;
    vb.D = r->cfg.max_photon_deposits;
    vb.NV = r->cfg.volumetric_photons;
    vb.vcnt = r->d_vcnt.as<uint32_t>();
    vb.vwin = r->d_vwin.as<uint32_t>();
    vb.vA = r->d_vA.as<float4>();
    vb.vB = r->d_vB.as<float4>();
    vb.keys = r->d_vkeys.as<uint32_t>();
    vb.vals = r->d_vvals.as<uint32_t>();
    vb.keys_sorted = r->d_vkeys2.as<uint32_t>();
    vb.vals_sorted = r->d_vvals2.as<uint32_t>();
    vb.sort_tmp = r->d_vsort.p;
    vb.sort_tmp_bytes = vol_sort_tmp_bytes(vb.NV);
    vb.start = r->d_vstart.as<uint32_t>();
    vb.rec = r->d_vrec.as<float4>();
    launch_vol_build(st, vb, r->vm);
    r->vm.valid = 1;
    return ORX_OK;
}

/* resize / RNG init / output clear common to every method (OptixRenderer.cpp:531-557) */
static orx_status begin_iteration(orx_renderer* r, uint64_t local_iteration_number, const orx_request* det,
                                  bool pipelined = false, bool vcm_overlap = false) {
    if (!r->scene_ready) return set_err(r, ORX_ERR_STATE, "Traced before OptixRenderer was initialized.");
    if (det->width == 0 || det->height == 0) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "zero-sized request");
    HIPCHK(r, hipSetDevice(r->device));
    if (det->width != r->W || det->height != r->H) { /* resizeBuffers (OptixRenderer.cpp:826-848) */
        r->psf_x = 1.0f / (float)det->width;
        r->psf_y = 1.0f / (float)det->height;
        r->vcm_estimated = false;
    }
    if (det->width != r->W || det->height != r->H || !r->rng_ready) {
        orx_status s0 = sync_all(r); /* nothing in flight may touch the buffers being replaced */
        if (s0 != ORX_OK) return s0;
        orx_status st = resize(r, det->width, det->height);
        if (st != ORX_OK) return st;
        if (r->use_ext) HIPCHK(r, hipStreamSynchronize(r->stream)); /* resize work ran on the own stream */
    }
    /* an overlapped VCM iteration leaves the last resolve running: its light pass may start beside it */
    if (!(vcm_overlap && local_iteration_number != 0)) flush_vcm(r);
    if (!pipelined) {
        if (vcm_overlap) {
            r->eye_chain = false;
            if (r->pend) HIPCHK(r, hipStreamWaitEvent(cur_stream(r), r->ev_gdone[r->pp], 0));
            r->pend = false;
        } else {
            flush_pipeline(r);
        }
    }
    r->timed_iterations++;
    /* the output accumulates on the gather stream when pipelined (after the previous output) */
    if (local_iteration_number == 0)
        HIPCHK(r, hipMemsetAsync(r->d_out.p, 0, (size_t)r->max_rows * r->W * 12, pipelined ? gather_stream(r) : cur_stream(r)));
    return ORX_OK;
}

/* The gather's tile order (GatherIn.order) for an image of `px` pixels: super-tiles of 8 x 8 tiles
 * (128 x 128 pixels) from 4M pixels up, image bands per XCD below.  At configs[4] the super-tiles
 * halve the union gather's fetches from beyond L2 (2 x FETCH_SIZE 22.3 -> 11.8 GB per launch;
 * 16 x 16: 10.4 GB) and the frame gains 2.8 % (serial gather 24.1 -> 23.1 ms); on the 1080p hall
 * the serial gather gains too (1.37 -> 1.21 ms) but the pipelined frame, where the gather overlaps
 * the next iteration's passes, does not (977 / 971 Mpaths/s, two runs each;
 * profiles/r04b_gather_order_ab.txt).  ORX_GATHER_ORDER=S forces S (0: bands). */
static uint32_t gather_order(size_t px) {
    static const int o = [] {
        const char* e = getenv("ORX_GATHER_ORDER");
        return e ? std::max(0, std::min(64, atoi(e))) : -1;
    }();
    return o >= 0 ? (uint32_t)o : (px >= (4u << 20) ? 8u : 0u);
}

static GatherIn local_gather_in(orx_renderer* r) {
    GatherIn gi;
    gi.base = (const uint8_t*)r->d_hp.p;
    gi.seg_bytes = (size_t)r->max_rows * r->W * 40;
    gi.segments = 1;
    gi.seg_rows = r->max_rows;
    gi.W = r->W;
    gi.indirect = r->d_ind.as<float>();
    gi.dbg = r->cfg.debug_counters ? r->d_dbg.as<uint32_t>() : nullptr;
    gi.cull = 0;
    gi.visits = 1;
    gi.order = gather_order((size_t)r->W * r->H);
    return gi;
}

static void ppm_eye(orx_renderer* r, const DevCamera& cam, const Consts& c) {
    ev_begin(r, P_EYE);
    if (r->media) {
        const MediaBufs mb = media_bufs(r);
        launch_ppm_eye(cur_stream(r), r->scene, cam, r->px, c, &mb);
    } else {
        launch_ppm_eye(cur_stream(r), r->scene, cam, r->px, c);
    }
    ev_end(r, P_EYE);
}
/* initializeStochasticHashPhotonMap (OptixRenderer_SpatialHash.cu:286-302): the scene AABB padded
 * by r + 0.0001 (AAB::addPadding, the sum in double as written), cell = r, grid = max(1, ceil(extent/r))
 * with OptiX's float3/float (multiplication by the reciprocal, calculateGridSize :42-50) */
static HashParams hash_params(const orx_renderer* r, float ppm_radius) {
    const float a = (float)((double)ppm_radius + 0.0001);
    const f3 lo = r->aabb_lo - mk1(a), hi = r->aabb_hi + mk1(a);
    const f3 f = (hi - lo) * (1.0f / ppm_radius);
    HashParams hp;
    hp.ox = lo.x;
    hp.oy = lo.y;
    hp.oz = lo.z;
    hp.cell = ppm_radius;
    hp.gx = std::max(1u, orx_f2u_sat(orx_ceilf(f.x)));
    hp.gy = std::max(1u, orx_f2u_sat(orx_ceilf(f.y)));
    hp.gz = std::max(1u, orx_f2u_sat(orx_ceilf(f.z)));
    hp.mask = r->pb.hnum - 1u;
    return hp;
}
static void ppm_grid_build(orx_renderer* r, const PhotonBufs& pb, const GridBox& gb = GridBox{}, hipStream_t on = nullptr);
/* photon pass (+ the overlapped direct pass), then the photon map (build_map: false in slab
 * mode, whose grid is built over the imported photons by orx_ppm_slab_import) */
static orx_status ppm_photons_grid(orx_renderer* r, const Consts& c, bool build_map = true) {
    hipStream_t st = cur_stream(r);
    ev_begin(r, P_PHOTON);
    r->eye_chain = false;
    MediaBufs mb{};
    if (r->media) mb = media_bufs(r);
    if (!launch_ppm_photon(st, r->scene, r->px, r->pb, c, r->media ? &mb : nullptr)) {
        ev_end(r, P_PHOTON);
        return set_err(r, ORX_ERR_STATE, "photon pass larger than its traversal-stack buffer (photon_stack_ensure)");
    }
    if (r->media) vol_build(r, st, c.ppm_radius);
    ev_end(r, P_PHOTON);
    if (r->overlap_direct) {
        /* the direct pass needs the hitpoints and the RNG states the photon pass
         * left (slot (x,y) is shared, Appendix A.2); nothing after it reads
         * either until the output pass, so it runs beside the grid build and
         * the gather */
        hipEventRecord(r->ev_photon_done, st);
        hipStreamWaitEvent(r->aux, r->ev_photon_done, 0);
        ev_begin_on(r, P_DIRECT, r->aux);
        launch_ppm_direct_output(r->aux, r->scene, r->px, c, 1);
        ev_end_on(r, P_DIRECT, r->aux);
        hipEventRecord(r->ev_direct_done, r->aux);
    }
    if (!build_map) return ORX_OK;
    if (r->pb.hash) {
        ev_begin(r, P_SETUP_HASH);
        launch_hash_build(st, r->pb, hash_params(r, c.ppm_radius));
        ev_end(r, P_SETUP_HASH);
        return ORX_OK;
    }
    if (r->cfg.photon_map == 2) { /* createPhotonKdTreeOnCPU, on the device */
        ev_begin(r, P_SETUP_HASH);
        launch_kd_build(st, r->pb, r->kd);
        ev_end(r, P_SETUP_HASH);
        return ORX_OK;
    }
    ppm_grid_build(r, r->pb);
    return ORX_OK;
}
/* grid build: the atomic-free bucket sort (an atomic-rank counting sort measured slower:
 * one device-scope atomic per photon into a 4 MB histogram); on `on`, or the
 * renderer's stream */
static void ppm_grid_build(orx_renderer* r, const PhotonBufs& pb, const GridBox& gb, hipStream_t on) {
    hipStream_t st = on ? on : cur_stream(r);
    ev_begin_on(r, P_SETUP_HASH, st);
    launch_grid_setup(st, pb, gb);
    launch_grid_bucket_count(st, pb);
    ev_end_on(r, P_SETUP_HASH, st);
    ev_begin_on(r, P_SCAN, st);
    launch_grid_bucket_scan(st, pb);
    ev_end_on(r, P_SCAN, st);
    ev_begin_on(r, P_SCATTER, st);
    launch_grid_bucket_place(st, pb);
    ev_end_on(r, P_SCATTER, st);
}
/* async grid build: the photon pass writes the other output set */
static void swap_photon_out(orx_renderer* r) {
    swap_buf(r->d_slots, r->d_slotsB);
    swap_buf(r->d_vmask, r->d_vmaskB);
    swap_buf(r->d_pos4, r->d_pos4B);
    swap_buf(r->d_bbox, r->d_bboxB);
    r->pb.slots = r->d_slots.as<float4>();
    r->pb.vmask = r->d_vmask.as<uint8_t>();
    r->pb.pos4 = r->d_pos4.as<float4>();
    r->pb.bbox = r->d_bbox.as<uint32_t>();
    r->po ^= 1u;
}
static orx_status ppm_local_passes(orx_renderer* r, const DevCamera& cam, const Consts& c) {
    ppm_eye(r, cam, c);
    return ppm_photons_grid(r, c);
}

/* VCM_BIDIRECTIONAL_PATH_TRACING branch of renderNextIteration (OptixRenderer.cpp:675-795) */
/* Row-sharded layout: rank r owns image rows y = rank + j*world (j < rows);
 * light subpath i pairs with own pixel i, so vertex counts, light vertices,
 * camera colours and the output hold own rows only.  The light pass's
 * connectCameraT1 splats land anywhere on the image: they are accumulated in
 * an owner-block buffer [world][max_rows][W][3] that a sharded run sums
 * across ranks (reduce-scatter) before the camera pass. */
static orx_status vcm_prepare(orx_renderer* r, const orx_request* det, float ppm_radius) {
    const size_t lpx = (size_t)r->W * r->rows;
    const size_t spx = (size_t)r->W * r->max_rows * r->world;
    if (r->vcm_npx != lpx || r->vcm_spx != spx) {
        HIPCHK(r, r->d_vcount.ensure(lpx * 4 + 4));
        HIPCHK(r, r->d_vverts.ensure(lpx * VCM_MAX_VERTS * 64 + 64));
        HIPCHK(r, r->d_vsplat.ensure(spx * 12 + 12));
        HIPCHK(r, r->d_vcam.ensure(lpx * 12 + 12));
        HIPCHK(r, hipMemsetAsync(r->d_vcount.p, 0, lpx * 4, cur_stream(r)));
        HIPCHK(r, hipMemsetAsync(r->d_vcam.p, 0, lpx * 12, cur_stream(r)));
        r->vcm_npx = lpx;
        r->vcm_kd = false;
        r->vcm_spx = spx;
    }
    VcmBufs& vb = r->vcm_vb;
    vb.RW = r->RW;
    vb.lcq = nullptr; /* the light pass traces its camera connections itself unless vcm_iteration defers them */
    vb.lctl = nullptr;
    vb.lcap = 0;
    vb.rng = r->px.rng;
    vb.vcount = r->d_vcount.as<uint32_t>();
    const size_t plane = lpx * VCM_MAX_VERTS;
    vb.vA = r->d_vverts.as<float4>();
    vb.vB = vb.vA + plane;
    vb.vC = vb.vB + plane;
    vb.vD = vb.vC + plane;
    if (r->has_tex && !r->vcm_kd) {
        HIPCHK(r, r->d_vkd.ensure(lpx * VCM_MAX_VERTS * 16 + 16));
        r->vcm_kd = true;
    }
    vb.vE = r->has_tex ? r->d_vkd.as<float4>() : nullptr;
    vb.splat = r->d_vsplat.as<float>();
    vb.splat_in = vb.splat + (size_t)r->rank * r->max_rows * r->W * 3;
    vb.splat_n = (uint32_t)std::min<size_t>(spx * 3, 0xffffffffu);
    {
        const size_t waves = std::max(vcm_camera_waves(((r->W + 7) / 8) * ((r->rows + 7) / 8)),
                                      vcm_light_waves((uint32_t)((lpx + 63) / 64)));
        /* [waves] queues for the light pass and walk, [waves] for the resolve's rerun beside them */
        HIPCHK(r, r->d_vshq.ensure(2 * waves * VCM_SHQ_PER_WAVE * 16 + 16));
        vb.shq = r->d_vshq.as<float4>();
        vb.shq_rerun = vb.shq + waves * VCM_SHQ_PER_WAVE;
        HIPCHK(r, r->d_vwork.ensure(64)); /* [0..1] work counters, [4..7] / [8..11] entry-list control words */
        vb.work = r->d_vwork.as<uint32_t>();
        HIPCHK(r, r->d_vconst.ensure(3 * sizeof(VcmConsts))); /* [0] the launches', [1 + set] the resolve's */
        vb.consts = r->d_vconst.as<VcmConsts>();
        vb.consts_keep = vb.consts + 1 + r->vcm_dpar;
    }
    vb.cam = r->d_vcam.as<float>();
    vb.output = r->d_out.as<float>();
    {
        /* The camera pass defers its connection shadow rays to k_vcm_shadow through an entry list of
         * ORX_VCM_DEFER = N per own pixel (default 16; the hall averages 6.5; a list that overflows makes
         * the pass rerun in place, small N exercises that, tests/test_gpu_parity.py); 0 traces them in
         * place inside the camera kernel.  Hall camera pass 6.21 -> 5.74 ms (473 -> 500 Mpaths/s): the
         * shadow kernel (61 VGPRs) runs at 8 waves per SIMD with a 16-entry LDS stack continued in
         * global memory, against the camera kernel's 3 (profiles/r04g_vcm_shadow_short_stack.txt) */
        static const uint32_t per_px = [] {
            const char* e = getenv("ORX_VCM_DEFER");
            return e ? (uint32_t)std::max(0, atoi(e)) : 16u;
        }();
        if (per_px) {
            const size_t cap = lpx * per_px;
            const size_t nslot = (size_t)r->rows * r->RW;
            HIPCHK(r, r->d_vdq.ensure(cap * 49 + 64));
            HIPCHK(r, r->d_vdpx.ensure(lpx * 20 + 64));
            HIPCHK(r, r->d_vrngsave.ensure(nslot * 24 + 16));
            r->vcm_dqcap = cap;
            vb.dq0 = r->d_vdq.as<float4>();
            vb.dq1 = vb.dq0 + cap;
            vb.dq2 = vb.dq1 + cap;
            vb.docc = (uint8_t*)(vb.dq2 + cap);
            vb.demis = r->d_vdpx.as<float4>();
            vb.dhead = (uint32_t*)(vb.demis + lpx);
            vb.dctl = vb.work + 4; /* d_vwork: [0..1] work counters, [4..7] the deferred-entry control words */
            vb.dcap = (uint32_t)std::min<size_t>(cap, 0xfffffff0u);
            for (int k = 0; k < 6; k++) vb.rsave.p[k] = r->d_vrngsave.as<uint32_t>() + (size_t)k * nslot;
            /* the shadow kernel's deep stack entries: (stack bound + 2 - 16) per lane of the largest grid */
            int dev = 0, cus = 256;
            hipGetDevice(&dev);
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            const size_t lanes = (size_t)cus * 32 * 64;
            const uint32_t deep = vcm_shadow_stack_deep(r->scene.stack_entries);
            HIPCHK(r, r->d_vshstk.ensure((size_t)deep * lanes * 4 + 64));
            vb.shstk = r->d_vshstk.as<uint32_t>();
            vb.shstk_lanes = (uint32_t)lanes;
            vb.shdeep = deep;
        } else {
            vb.dq0 = nullptr;
        }
    }
    VcmConsts& c = r->vcm_c;
    float ulen = 0.f, vlen = 0.f;
    DevCamera cam = camera_setup(det->camera, &ulen, &vlen);
    c.eye = cam.eye;
    c.lookdir = cam.lookdir;
    c.u = cam.u;
    c.v = cam.v;
    c.unitU = normalize(cam.u);
    c.unitV = normalize(cam.v);
    c.lookdirN = normalize(cam.lookdir);
    c.lookdirLen = length(cam.lookdir);
    c.ipsx = 2.0f * ulen;
    c.ipsy = 2.0f * vlen;
    c.psfx = r->psf_x;
    c.psfy = r->psf_y;
    c.W = r->W;
    c.H = r->H;
    c.count = r->W * r->H;
    c.rank = r->rank;
    c.world = r->world;
    c.rows = r->rows;
    c.max_rows = r->max_rows;
    c.lcount = r->W * r->rows;
    c.maxPathLen = r->cfg.vcm_max_path_length;
    /* etaVCM = (nVM / nVC) * PI * r^2 with nVC = 1, nVM = lightSubPathCount */
    const float ppmRadiusSquared = ppm_radius * ppm_radius;
    const float etaVCM = ((float)c.count / (float)1u) * ORX_PI_F * ppmRadiusSquared;
    c.misVm = 0.f;
    c.misVc = 1.f / etaVCM;
    return ORX_OK;
}

static orx_status vcm_light(orx_renderer* r) {
    hipStream_t st = cur_stream(r);
    ev_begin(r, P_VCM_LIGHT);
    if (!r->vcm_estimated) { /* subpath length estimate launch: advances the RNG, stores nothing */
        launch_vcm_light(st, r->scene, r->vcm_vb, r->vcm_c, true);
        r->vcm_estimated = true;
    }
    HIPCHK(r, hipMemsetAsync(r->vcm_vb.splat, 0, r->vcm_spx * 12, st));
    launch_vcm_light(st, r->scene, r->vcm_vb, r->vcm_c, false);
    ev_end(r, P_VCM_LIGHT);
    return ORX_OK;
}

static orx_status vcm_camera(orx_renderer* r, bool overlap = false) {
    if (!overlap) {
        hipStream_t st = cur_stream(r);
        ev_begin(r, P_VCM_CAMERA);
        launch_vcm_camera_walk(st, r->scene, r->vcm_vb, r->vcm_c);
        ev_end(r, P_VCM_CAMERA);
        ev_begin(r, P_VCM_SHADOW);
        launch_vcm_camera_resolve(st, r->scene, r->vcm_vb, r->vcm_c);
        ev_end(r, P_VCM_SHADOW);
        return ORX_OK;
    }
    /* the walk on the renderer's stream, the resolve (with the rerun an overflow needs) on aux beside the
     * next iteration's light pass and walk (the pass interval ends with the resolve); the stream then
     * waits for the previous iteration's resolve, since the next light pass and walk write the set it
     * reads (light image, light vertices, entry list, RNG start words, constants copy) */
    hipStream_t st = cur_stream(r);
    ev_begin(r, P_VCM_CAMERA);
    launch_vcm_camera_walk(st, r->scene, r->vcm_vb, r->vcm_c);
    ev_end(r, P_VCM_CAMERA);
    HIPCHK(r, hipEventRecord(r->ev_vcam, st));
    if (r->vcm_pend) HIPCHK(r, hipStreamWaitEvent(st, r->ev_vacc, 0));
    HIPCHK(r, hipStreamWaitEvent(r->aux, r->ev_vcam, 0));
    ev_begin_on(r, P_VCM_SHADOW, r->aux);
    launch_vcm_camera_resolve(r->aux, r->scene, r->vcm_vb, r->vcm_c);
    ev_end_on(r, P_VCM_SHADOW, r->aux);
    HIPCHK(r, hipEventRecord(r->ev_vacc, r->aux));
    r->vcm_pend = true;
    return ORX_OK;
}

static orx_status vcm_check_lights(orx_renderer* r) {
    for (const DevLight& l : r->host_lights)
        if (l.type == LIGHT_SPOT)
            return set_err(r, ORX_ERR_UNSUPPORTED, "VCM: spot lights are not emitted by lightEmit (helpers/light.h:130)");
    return ORX_OK;
}

static orx_status vcm_iteration(orx_renderer* r, const orx_request* det, float ppm_radius, bool overlap = false) {
    orx_status s = vcm_prepare(r, det, ppm_radius);
    if (s != ORX_OK) return s;
    overlap = overlap && r->vcm_vb.dq0;
    if (overlap) { /* this iteration's light image and entry list: the ones the last resolve does not read */
        HIPCHK(r, r->d_vsplat2.ensure(r->d_vsplat.bytes));
        HIPCHK(r, r->d_vdq2.ensure(r->d_vdq.bytes));
        HIPCHK(r, r->d_vdpx2.ensure(r->d_vdpx.bytes));
        swap_buf(r->d_vsplat, r->d_vsplat2);
        swap_buf(r->d_vdq, r->d_vdq2);
        swap_buf(r->d_vdpx, r->d_vdpx2);
        r->vcm_dpar ^= 1u;
        VcmBufs& vb = r->vcm_vb;
        vb.splat = r->d_vsplat.as<float>();
        vb.splat_in = vb.splat + (size_t)r->rank * r->max_rows * r->W * 3;
        const size_t cap = r->vcm_dqcap;
        vb.dq0 = r->d_vdq.as<float4>();
        vb.dq1 = vb.dq0 + cap;
        vb.dq2 = vb.dq1 + cap;
        vb.docc = (uint8_t*)(vb.dq2 + cap);
        vb.demis = r->d_vdpx.as<float4>();
        vb.dhead = (uint32_t*)(vb.demis + (size_t)r->W * r->rows);
        vb.dctl = vb.work + (r->vcm_dpar ? 8 : 4);
        vb.consts_keep = vb.consts + 1 + r->vcm_dpar;
        /* the light vertices (with counts and texel colours) and the walk's RNG start words: the resolve's
         * in-place rerun after an overflow reads this iteration's while the next one writes the other set */
        HIPCHK(r, r->d_vverts2.ensure(r->d_vverts.bytes));
        HIPCHK(r, r->d_vcount2.ensure(r->d_vcount.bytes));
        HIPCHK(r, r->d_vrngsave2.ensure(r->d_vrngsave.bytes));
        swap_buf(r->d_vverts, r->d_vverts2);
        swap_buf(r->d_vcount, r->d_vcount2);
        swap_buf(r->d_vrngsave, r->d_vrngsave2);
        const size_t lpx = (size_t)r->W * r->rows, plane = lpx * VCM_MAX_VERTS, nslot = (size_t)r->rows * r->RW;
        vb.vcount = r->d_vcount.as<uint32_t>();
        vb.vA = r->d_vverts.as<float4>();
        vb.vB = vb.vA + plane;
        vb.vC = vb.vB + plane;
        vb.vD = vb.vC + plane;
        if (vb.vE) {
            HIPCHK(r, r->d_vkd2.ensure(r->d_vkd.bytes));
            swap_buf(r->d_vkd, r->d_vkd2);
            vb.vE = r->d_vkd.as<float4>();
        }
        for (int k = 0; k < 6; k++) vb.rsave.p[k] = r->d_vrngsave.as<uint32_t>() + (size_t)k * nslot;
        /* the light pass's camera connections go with the resolve too (hall 536 -> 568 Mpaths/s,
         * profiles/r05r_vcm_light_defer_ab.txt): room for 4 per own subpath, against the hall's ~3 stored
         * light vertices per subpath with at most one connection each (a wave whose queue does not fit
         * traces it in place; ORX_VCM_LIGHT_DEFER=0: all in place) */
        static const uint32_t lper = [] {
            const char* e = getenv("ORX_VCM_LIGHT_DEFER");
            return e ? (uint32_t)std::max(0, atoi(e)) : 4u;
        }();
        if (lper) {
            const size_t lcap = std::min<size_t>((size_t)r->W * r->rows * lper, 0x0ffffff0u);
            HIPCHK(r, r->d_vlcq.ensure(lcap * 48 + 64));
            HIPCHK(r, r->d_vlcq2.ensure(lcap * 48 + 64));
            swap_buf(r->d_vlcq, r->d_vlcq2);
            vb.lcq = r->d_vlcq.as<float4>();
            vb.lcap = (uint32_t)lcap;
            vb.lctl = vb.work + (r->vcm_dpar ? 14 : 12);
        }
    }
    if ((s = vcm_light(r)) != ORX_OK) return s;
    r->last_vcm_overlap = overlap;
    return vcm_camera(r, overlap);
}

/* the asynchronous grid build when the measured photon pass + grid build exceed this multiple of the gather.
 * Measured on the first pipelined iteration (its radius is the largest, so its gather the dearest): hall
 * 5.59 / 3.44 ms = 1.62 (the asynchronous build gains 1.2-1.8 % there), Cornell 0.79 / 0.98 = 0.81 and
 * conference 4K 19.2 / 51.0 = 0.38 (it loses 1-2 %); the threshold sits at their geometric middle
 * (profiles/r06p_grid_async_ab.txt, r06zh_grid_schedule_choice.txt) */
constexpr float GRID_CHAIN_RATIO = 1.15f;

/* One PPM iteration whose gather and output are left running on gstream, overlapping the next
 * iteration's eye, photon and grid passes (orx_render_next_iteration, single device).  Every
 * kernel and its inputs are those of the serial schedule; only the buffer set alternates. */
static orx_status ppm_pipelined_iteration(orx_renderer* r, const orx_request* det, float ppm_radius,
                                          uint64_t local_iteration_number) {
    const DevCamera cam = camera_setup(det->camera);
    const Consts c = make_consts(r, ppm_radius, local_iteration_number);
    hipStream_t st = r->stream;
    swap_sets(r);
    const uint32_t k = r->pp;
    const bool measure = r->probe_stage == 1;
    if (r->probe_stage == 2) { /* after the measured iteration: this photon pass waits for its gather */
        HIPCHK(r, hipStreamWaitEvent(st, r->ev_gdone[r->probe_k], 0));
        r->probe_stage = 3;
    } else if (r->probe_stage == 3) { /* the device still holds the previous iteration: no bubble */
        HIPCHK(r, hipEventSynchronize(r->ev_pm[3]));
        HIPCHK(r, hipEventElapsedTime(&r->probe_ms[0], r->ev_pm[0], r->ev_pm[1]));
        HIPCHK(r, hipEventElapsedTime(&r->probe_ms[1], r->ev_pm[2], r->ev_pm[3]));
        r->async_grid = r->probe_ms[0] > GRID_CHAIN_RATIO * r->probe_ms[1];
        r->probe_stage = 0;
    }
    /* asynchronous build: the photon pass writes the other output set, whose last reader is the grid build
     * two iterations back; synchronous after asynchronous iterations: the current set, last read by the
     * previous iteration's build on gridq (else an event long complete) */
    if (r->async_grid) swap_photon_out(r);
    if (r->out_b) HIPCHK(r, hipStreamWaitEvent(st, r->ev_gsrc[r->po], 0));
    /* the set's previous gather + output (two iterations back) and, through the RNG chain
     * (slot (x,y) is advanced by eye, photon and direct in turn), the last direct pass */
    HIPCHK(r, hipStreamWaitEvent(st, r->ev_gdone[k], 0));
    HIPCHK(r, hipStreamWaitEvent(r->aux, r->ev_gdone[k], 0)); /* eye and direct write this set */
    /* The eye pass needs the RNG slots after the direct pass of i (aux, stream order) and this
     * set free (above); not the grid build of i, which is still running on st.  So it runs on
     * aux beside that grid build, and the photon pass waits for it (RNG chain) and, in stream
     * order, for the grid build (the deposit records it reads).  Without an unbroken chain of
     * pipelined iterations aux first waits for everything enqueued on st. */
    if (!r->eye_chain) {
        HIPCHK(r, hipEventRecord(r->ev_main, st));
        HIPCHK(r, hipStreamWaitEvent(r->aux, r->ev_main, 0));
    }
    ev_begin_on(r, P_EYE, r->aux);
    launch_ppm_eye(r->aux, r->scene, cam, r->px, c);
    ev_end_on(r, P_EYE, r->aux);
    HIPCHK(r, hipEventRecord(r->ev_eye_done, r->aux));
    HIPCHK(r, hipStreamWaitEvent(st, r->ev_eye_done, 0));
    r->overlap_direct = true;
    if (measure) HIPCHK(r, hipEventRecord(r->ev_pm[0], st));
    const orx_status sp = ppm_photons_grid(r, c, !r->async_grid); /* photon, direct (aux), grid */
    if (measure) HIPCHK(r, hipEventRecord(r->ev_pm[1], st));
    r->overlap_direct = false;
    if (sp != ORX_OK) return sp;
    if (r->async_grid) {
        /* the grid build on its own stream: the photon pass of i + 1 waits only for the RNG chain (eye of i + 1
         * after the direct pass of i) and for this build's end of reading the output set two iterations on */
        HIPCHK(r, hipStreamWaitEvent(r->gridq, r->ev_photon_done, 0));
        ppm_grid_build(r, r->pb, GridBox{}, r->gridq);
        HIPCHK(r, hipEventRecord(r->ev_gsrc[r->po], r->gridq));
        HIPCHK(r, hipEventRecord(r->ev_grid_done, r->gridq));
    } else {
        HIPCHK(r, hipEventRecord(r->ev_grid_done, st));
    }
    hipStream_t g = r->gstream;
    HIPCHK(r, hipStreamWaitEvent(g, r->ev_grid_done, 0));
    ev_begin_on(r, P_GATHER, g);
    if (measure) HIPCHK(r, hipEventRecord(r->ev_pm[2], g));
    if (r->cfg.photon_map == 2) launch_ppm_gather_kd(g, local_gather_in(r), r->pb, r->kd, c);
    else if (r->pb.hash) launch_ppm_gather_hash(g, local_gather_in(r), r->pb, hash_params(r, c.ppm_radius), c);
    else launch_ppm_gather(g, local_gather_in(r), r->pb, c);
    if (measure) {
        HIPCHK(r, hipEventRecord(r->ev_pm[3], g));
        r->probe_stage = 2;
        r->probe_k = k;
    }
    ev_end_on(r, P_GATHER, g);
    HIPCHK(r, hipStreamWaitEvent(g, r->ev_direct_done, 0));
    ev_begin_on(r, P_DIRECT, g);
    launch_ppm_direct_output(g, r->scene, r->px, c, 2);
    ev_end_on(r, P_DIRECT, g);
    HIPCHK(r, hipEventRecord(r->ev_gdone[k], g));
    r->pend = true;
    r->eye_chain = true;
    HIPCHK(r, hipGetLastError());
    r->last_method = (uint64_t)det->method;
    r->last_consts = c;
    return ORX_OK;
}

static orx_status render_next_iteration(orx_renderer* r, uint64_t local_iteration_number, float ppm_radius,
                                        const orx_request* det);
orx_status orx_render_next_iteration(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                                     float ppm_radius, int create_output, const orx_request* det) {
    (void)create_output; /* ignored by the reference engine too */
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    char range[48]; /* OptixRenderer.cpp:518-520 */
    snprintf(range, sizeof range, "OptixRenderer::Trace Iteration %llu", (unsigned long long)iteration_number);
    roctxRangePushA(range);
    const orx_status st = render_next_iteration(r, local_iteration_number, ppm_radius, det);
    roctxRangePop();
    return st;
}
static orx_status render_next_iteration(orx_renderer* r, uint64_t local_iteration_number, float ppm_radius,
                                        const orx_request* det) {
    if (det->method != ORX_METHOD_PATH_TRACING && det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING &&
        det->method != ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING)
        return set_err(r, ORX_ERR_UNSUPPORTED, "render method not supported by this build");
    if (det->method == ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING && r->world > 1)
        return set_err(r, ORX_ERR_STATE, "sharded VCM runs through orx_vcm_local_light/orx_export_vcm_splats/orx_vcm_finish");
    if (det->method == ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING && vcm_check_lights(r) != ORX_OK)
        return ORX_ERR_UNSUPPORTED;
    if (det->method == ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING && r->world > 1)
        return set_err(r, ORX_ERR_STATE, "sharded PPM runs through orx_ppm_local_passes/_gather_external/_finish");
    if (r->media && det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING)
        return set_err(r, ORX_ERR_UNSUPPORTED, "participating media: progressive photon mapping only");
    if (r->media && r->cfg.photon_map == 1)
        return set_err(r, ORX_ERR_UNSUPPORTED, "participating media: uniform grid or kd-tree photon map");
    static const int pipeline_env = [] {
        const char* e = getenv("ORX_PIPELINE");
        return e ? atoi(e) : 1;
    }();
    const int pipe_on = r->pipe_mode >= 0 ? r->pipe_mode : pipeline_env;
    const bool pipelined = pipe_on && det->method == ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING && r->world == 1 &&
                           !r->use_ext && !r->media;
    /* VCM: the camera pass's resolve half beside the next light pass (ORX_VCM_OVERLAP=0: serial) */
    static const int vcm_overlap_env = [] {
        const char* e = getenv("ORX_VCM_OVERLAP");
        return e ? atoi(e) : 1;
    }();
    const bool vcm_overlap = pipe_on && vcm_overlap_env && det->method == ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING &&
                             r->world == 1 && !r->use_ext;
    orx_status s0 = begin_iteration(r, local_iteration_number, det, pipelined, vcm_overlap);
    r->last_vcm_overlap = false;
    if (s0 != ORX_OK) return s0;
    if (pipelined && (s0 = ensure_second_set(r)) != ORX_OK) return s0;
    r->last_pipelined = pipelined && r->pipe_bufs;
    if (r->last_pipelined) return ppm_pipelined_iteration(r, det, ppm_radius, local_iteration_number);
    if (pipelined) flush_pipeline(r);
    DevCamera cam = camera_setup(det->camera);
    Consts c = make_consts(r, ppm_radius, local_iteration_number);
    hipStream_t st = cur_stream(r);
    if (det->method == ORX_METHOD_PATH_TRACING) {
        ev_begin(r, P_PT);
        launch_pt(st, r->scene, cam, r->px, c);
        ev_end(r, P_PT);
    } else if (det->method == ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING) {
        orx_status sv = vcm_iteration(r, det, ppm_radius, vcm_overlap);
        if (sv != ORX_OK) return sv;
    } else {
        /* the direct pass on the aux stream beside the grid build and the gather; the output
         * accumulation after both */
        r->overlap_direct = true;
        const orx_status sp = ppm_local_passes(r, cam, c);
        if (sp != ORX_OK) {
            r->overlap_direct = false;
            return sp;
        }
        ev_begin(r, P_GATHER);
        if (r->pb.hash) launch_ppm_gather_hash(st, local_gather_in(r), r->pb, hash_params(r, c.ppm_radius), c);
        else if (r->cfg.photon_map == 2) launch_ppm_gather_kd(st, local_gather_in(r), r->pb, r->kd, c);
        else launch_ppm_gather(st, local_gather_in(r), r->pb, c);
        if (r->media) launch_vol_indirect(st, r->px, r->d_volR.as<float>(), c.emitted_f);
        ev_end(r, P_GATHER);
        ev_begin(r, P_DIRECT);
        HIPCHK(r, hipStreamWaitEvent(st, r->ev_direct_done, 0));
        launch_ppm_direct_output(st, r->scene, r->px, c, 2);
        ev_end(r, P_DIRECT);
        r->overlap_direct = false;
    }
    HIPCHK(r, hipGetLastError());
    r->last_method = (uint64_t)det->method;
    r->last_consts = c;
    return ORX_OK;
}

orx_status orx_ppm_local_passes(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                                float ppm_radius, const orx_request* det) {
    (void)iteration_number;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    if (r->media) return set_err(r, ORX_ERR_UNSUPPORTED, "participating media run through orx_render_next_iteration");
    if (det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING)
        return set_err(r, ORX_ERR_INVALID_ARGUMENT, "orx_ppm_local_passes needs a PPM request");
    r->last_pipelined = false;
    orx_status s0 = begin_iteration(r, local_iteration_number, det);
    if (s0 != ORX_OK) return s0;
    DevCamera cam = camera_setup(det->camera);
    Consts c = make_consts(r, ppm_radius, local_iteration_number);
    const orx_status sp = ppm_local_passes(r, cam, c);
    if (sp != ORX_OK) return sp;
    HIPCHK(r, hipGetLastError());
    r->last_method = (uint64_t)det->method;
    r->last_consts = c;
    return ORX_OK;
}

orx_status orx_ppm_local_eye(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                             float ppm_radius, const orx_request* det) {
    (void)iteration_number;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    if (r->media) return set_err(r, ORX_ERR_UNSUPPORTED, "participating media run through orx_render_next_iteration");
    if (det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING)
        return set_err(r, ORX_ERR_INVALID_ARGUMENT, "orx_ppm_local_eye needs a PPM request");
    orx_status s0 = begin_iteration(r, local_iteration_number, det, r->shard_pipe);
    if (s0 != ORX_OK) return s0;
    if (r->shard_pipe && (s0 = ensure_second_set(r)) != ORX_OK) return s0;
    DevCamera cam = camera_setup(det->camera);
    Consts c = make_consts(r, ppm_radius, local_iteration_number);
    r->last_pipelined = r->shard_pipe && r->pipe_bufs;
    if (r->last_pipelined) {
        if (r->fin_due) { /* the previous iteration's finish comes later: hold its set */
            if (r->fin_snap) return set_err(r, ORX_ERR_STATE, "two sharded PPM finishes outstanding");
            r->fin_px = r->px;
            r->fin_consts = r->last_consts;
            r->fin_pp = r->pp;
            r->fin_snap = true;
        }
        r->fin_due = true;
        /* the other buffer set; its last gather + finish (two iterations back) and, through the
         * RNG chain, the last direct pass precede this eye pass */
        swap_sets(r);
        HIPCHK(r, hipStreamWaitEvent(cur_stream(r), r->ev_gdone[r->pp], 0));
        HIPCHK(r, hipStreamWaitEvent(cur_stream(r), r->ev_direct_done, 0));
        HIPCHK(r, hipStreamWaitEvent(r->aux, r->ev_gdone[r->pp], 0));
    } else if (r->shard_pipe) {
        flush_pipeline(r);
    }
    ppm_eye(r, cam, c);
    HIPCHK(r, hipGetLastError());
    r->last_method = (uint64_t)det->method;
    r->last_consts = c;
    return ORX_OK;
}

orx_status orx_ppm_local_photons(orx_renderer* r) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->rng_ready) return set_err(r, ORX_ERR_STATE, "orx_ppm_local_eye first");
    HIPCHK(r, hipSetDevice(r->device));
    r->overlap_direct = r->last_pipelined; /* direct pass on the aux stream right after the photons */
    const orx_status sp = ppm_photons_grid(r, r->last_consts);
    r->overlap_direct = false;
    if (sp != ORX_OK) return sp;
    if (r->last_pipelined) HIPCHK(r, hipEventRecord(r->ev_grid_done, cur_stream(r)));
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

orx_status orx_set_slab_partition(orx_renderer* r, int enable) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    if (enable && r->cfg.photon_map != 0)
        return set_err(r, ORX_ERR_UNSUPPORTED, "the slab partition needs the uniform-grid photon map");
    HIPCHK(r, hipSetDevice(r->device));
    orx_status s0 = sync_all(r);
    if (s0 != ORX_OK) return s0;
    r->slab = enable != 0;
    r->rng_ready = false; /* re-allocate the photon buffers for the imported photons */
    return ORX_OK;
}

orx_status orx_ppm_local_trace(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                               float ppm_radius, const orx_request* det) {
    (void)iteration_number;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    if (r->media) return set_err(r, ORX_ERR_UNSUPPORTED, "participating media run through orx_render_next_iteration");
    if (det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING)
        return set_err(r, ORX_ERR_INVALID_ARGUMENT, "orx_ppm_local_trace needs a PPM request");
    if (!r->slab) return set_err(r, ORX_ERR_STATE, "orx_ppm_local_trace is the slab mode's first phase");
    r->last_pipelined = false;
    orx_status s0 = begin_iteration(r, local_iteration_number, det);
    if (s0 != ORX_OK) return s0;
    DevCamera cam = camera_setup(det->camera);
    Consts c = make_consts(r, ppm_radius, local_iteration_number);
    ppm_eye(r, cam, c);
    const orx_status sp = ppm_photons_grid(r, c, false);
    if (sp != ORX_OK) return sp;
    HIPCHK(r, hipGetLastError());
    r->last_method = (uint64_t)det->method;
    r->last_consts = c;
    return ORX_OK;
}

orx_status orx_ppm_local_photon_trace(orx_renderer* r) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->rng_ready) return set_err(r, ORX_ERR_STATE, "orx_ppm_local_eye first");
    if (!r->slab) return set_err(r, ORX_ERR_STATE, "orx_ppm_local_photon_trace is a slab-mode phase");
    HIPCHK(r, hipSetDevice(r->device));
    r->overlap_direct = r->last_pipelined; /* direct pass on the aux stream right after the photons */
    const orx_status sp = ppm_photons_grid(r, r->last_consts, false);
    r->overlap_direct = false;
    if (sp != ORX_OK) return sp;
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

static_assert(SLAB_VOX == ORX_SLAB_VOXELS, "slab voxel grid: kernels and ABI disagree");
size_t orx_slab_histogram_words(uint32_t nb) {
    return (size_t)6 * nb + 6 + (size_t)2 * ORX_SLAB_VOXELS * ORX_SLAB_VOXELS * ORX_SLAB_VOXELS;
}
static SlabBins slab_bins(const orx_renderer* r, uint32_t nb) {
    SlabBins sb;
    const float lo[3] = {r->aabb_lo.x, r->aabb_lo.y, r->aabb_lo.z}, hi[3] = {r->aabb_hi.x, r->aabb_hi.y, r->aabb_hi.z};
    for (int a = 0; a < 3; a++) {
        const float ext = hi[a] - lo[a];
        sb.lo[a] = lo[a];
        sb.inv[a] = ext > 0.f ? (float)nb / ext : 0.f;
    }
    sb.nb = nb;
    return sb;
}

uint32_t orx_ppm_slab_halo(const orx_renderer* r, uint32_t nb, uint32_t axis, float radius) {
    if (!r || axis > 2 || nb == 0) return 2u;
    const SlabBins sb = slab_bins(r, nb);
    const float h = orx_floorf(radius * sb.inv[axis]);
    return (h >= 0.f && h < 1e6f ? (uint32_t)h : 0u) + 2u;
}
orx_status orx_ppm_slab_histogram(orx_renderer* r, uint32_t* hist, uint32_t nb) {
    if (!r || !hist || nb < ORX_SLAB_VOXELS || nb > 1024 || nb % ORX_SLAB_VOXELS) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->slab || !r->rng_ready) return set_err(r, ORX_ERR_STATE, "orx_ppm_slab_histogram: slab mode, after the photon pass");
    HIPCHK(r, hipSetDevice(r->device));
    hipStream_t st = cur_stream(r);
    HIPCHK(r, hipMemsetAsync(hist, 0, orx_slab_histogram_words(nb) * 4, st));
    launch_slab_hist(st, r->pb, r->px, slab_bins(r, nb), slab_bins(r, ORX_SLAB_VOXELS), hist);
    launch_slab_bbox(st, r->pb, hist + 6 * (size_t)nb);
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

orx_status orx_ppm_slab_pack(orx_renderer* r, const uint8_t* bin_dest, uint32_t nb, uint32_t axis, uint32_t halo_bins,
                             const uint32_t* dest_base, uint64_t send_records, void* send) {
    if (!r || !bin_dest || !dest_base || !send || nb == 0 || nb > 1024 || axis > 2) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->slab || !r->rng_ready) return set_err(r, ORX_ERR_STATE, "orx_ppm_slab_pack: slab mode, after the photon pass");
    if (r->world > 64) return set_err(r, ORX_ERR_UNSUPPORTED, "slab mode supports at most 64 ranks");
    for (uint32_t b = 0; b < nb; b++)
        if (bin_dest[b] >= r->world || (b && bin_dest[b] < bin_dest[b - 1]))
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "bin_dest must be ascending ranks < world");
    /* the run of each rank must lie inside the send buffer; the plan's counts come from the
     * histogram of the same photons, so the runs are exactly filled */
    for (uint32_t d = 0; d < r->world; d++)
        if (dest_base[d] > send_records || (d && dest_base[d] < dest_base[d - 1]))
            return set_err(r, ORX_ERR_INVALID_ARGUMENT, "dest_base must be ascending and inside the send buffer");
    if (send_records > 0xffffffffull) return set_err(r, ORX_ERR_UNSUPPORTED, "send buffer beyond 2^32 records");
    HIPCHK(r, hipSetDevice(r->device));
    hipStream_t st = cur_stream(r);
    HIPCHK(r, r->d_slabtab.ensure(8192));
    HIPCHK(r, r->d_slabcur.ensure(64 * 4));
    HIPCHK(r, hipMemcpyAsync(r->d_slabtab.p, bin_dest, nb, hipMemcpyHostToDevice, st));
    HIPCHK(r, hipMemcpyAsync(r->d_slabcur.p, dest_base, (size_t)r->world * 4, hipMemcpyHostToDevice, st));
    launch_slab_pack(st, r->pb, slab_bins(r, nb), axis, halo_bins, r->d_slabtab.as<uint8_t>(), r->world,
                     r->d_slabcur.as<uint32_t>(), (uint32_t)send_records, (float*)send);
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

orx_status orx_ppm_slab_import(orx_renderer* r, const void* recv, uint64_t n, const uint32_t* photon_box,
                               uint32_t axis, uint32_t nb, uint32_t own_lo, uint32_t own_hi) {
    if (!r || (!recv && n) || axis > 2 || nb == 0 || nb > 1024) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->slab || !r->rng_ready) return set_err(r, ORX_ERR_STATE, "orx_ppm_slab_import: slab mode, after the photon pass");
    if (n > r->S_cap) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "more photons than the slab import capacity");
    HIPCHK(r, hipSetDevice(r->device));
    hipStream_t st = cur_stream(r);
    /* the photon AABB replicas hold the own photon pass's deposits: reset, then the imported ones */
    HIPCHK(r, hipMemsetAsync(r->d_bbox.p, 0xff, 3 * BBOX_REPLICAS * 4, st));
    HIPCHK(r, hipMemsetAsync(r->d_bbox.as<uint32_t>() + 3 * BBOX_REPLICAS, 0, 3 * BBOX_REPLICAS * 4, st));
    PhotonBufs pbi = r->pb;
    const size_t groups = n ? (n + pbi.D - 1) / pbi.D : 1; /* an empty import: one group with no deposit */
    pbi.S = (uint32_t)(groups * pbi.D);
    pbi.bs_nchunk = (pbi.S + 16383) / 16384;
    if (n == 0) HIPCHK(r, hipMemsetAsync(r->d_vmask.p, 0, 1, st));
    else launch_slab_import(st, pbi, (const float*)recv, (uint32_t)n);
    GridBox gb{};
    if (photon_box) {
        gb.on = 1;
        for (int k = 0; k < 6; k++) gb.b[k] = photon_box[k];
    }
    ppm_grid_build(r, pbi, gb);
    r->own_axis = axis;
    r->own_nb = nb;
    r->own_lo = own_lo;
    r->own_hi = own_hi;
    if (r->last_pipelined) HIPCHK(r, hipEventRecord(r->ev_grid_done, st));
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

orx_status orx_debug_limit_photon_stack(orx_renderer* r, uint32_t lanes) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    if (lanes < r->pb.tlanes) r->pb.tlanes = lanes;
    return ORX_OK;
}

/* test hook: drive the last VCM iteration's resolve again with stale list state -- the entry count
 * past the capacity, every odd own pixel's list head past the entries, and 64 light-connection entries
 * appended whose pixel offsets lie past the light image -- as a walk or light pass that did not write
 * this set's control words would leave them (vcm.h:315-400 / :43-58 have no such state: the device-side
 * bounds in k_vcm_accum and k_vcm_light_shadow are ours).  Synchronous; the colours land in
 * ORX_BUF_VCM_CAMERA (the output is accumulated once more: not a render) */
orx_status orx_debug_vcm_stale_resolve(orx_renderer* r) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    const VcmBufs& vb = r->vcm_vb;
    if (!vb.dq0 || !r->vcm_npx) return set_err(r, ORX_ERR_STATE, "no VCM iteration with deferred lists");
    HIPCHK(r, hipSetDevice(r->device));
    flush_pipeline(r);
    HIPCHK(r, hipStreamSynchronize(cur_stream(r)));
    HIPCHK(r, hipDeviceSynchronize());
    const size_t lpx = r->vcm_npx;
    std::vector<uint32_t> head(lpx);
    HIPCHK(r, hipMemcpy(head.data(), vb.dhead, lpx * 4, hipMemcpyDeviceToHost));
    for (size_t p = 1; p < lpx; p += 2) head[p] = vb.dcap + (uint32_t)p;
    HIPCHK(r, hipMemcpy(vb.dhead, head.data(), lpx * 4, hipMemcpyHostToDevice));
    const uint32_t stale = 0xfffffff0u;
    HIPCHK(r, hipMemcpy(vb.dctl, &stale, 4, hipMemcpyHostToDevice));
    if (vb.lcq && vb.lcap >= 64) {
        uint32_t lc[2] = {0, 0};
        HIPCHK(r, hipMemcpy(lc, vb.lctl, 8, hipMemcpyDeviceToHost));
        const uint32_t base = std::min(lc[0], vb.lcap - 64);
        std::vector<float4> e(3 * 64);
        for (uint32_t k = 0; k < 64; k++) {
            const uint32_t at = vb.splat_n + 3 * k; /* past the light image */
            float w;
            memcpy(&w, &at, 4);
            e[3 * k + 0] = make_float4(0.f, 0.f, 0.f, 0.f); /* distance 0: unoccluded without a walk */
            e[3 * k + 1] = make_float4(0.f, 0.f, 1.f, w);
            e[3 * k + 2] = make_float4(1.f, 1.f, 1.f, 0.f);
        }
        HIPCHK(r, hipMemcpy(vb.lcq + 3 * (size_t)base, e.data(), e.size() * 16, hipMemcpyHostToDevice));
        lc[0] = base + 64;
        HIPCHK(r, hipMemcpy(vb.lctl, lc, 4, hipMemcpyHostToDevice));
    }
    launch_vcm_camera_resolve(cur_stream(r), r->scene, vb, r->vcm_c);
    HIPCHK(r, hipGetLastError());
    HIPCHK(r, hipStreamSynchronize(cur_stream(r)));
    return ORX_OK;
}

orx_status orx_export_hitpoints(orx_renderer* r, void* dst, size_t bytes) {
    if (!r || !dst) return ORX_ERR_INVALID_ARGUMENT;
    const size_t npx = (size_t)r->max_rows * r->W, need = hp_export_plane(npx) * 28;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "destination too small");
    HIPCHK(r, hipSetDevice(r->device));
    launch_export_hp(cur_stream(r), r->px, (uint32_t)npx, (float*)dst);
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

orx_status orx_ppm_gather_external(orx_renderer* r, const void* hp, uint32_t segments, void* indirect, size_t bytes) {
    if (!r || !hp || !indirect || segments == 0) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->rng_ready) return set_err(r, ORX_ERR_STATE, "no local passes yet");
    if (r->pb.hash) return set_err(r, ORX_ERR_UNSUPPORTED, "the stochastic hash photon map is single-device");
    size_t need = (size_t)segments * r->max_rows * r->W * 12;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "indirect buffer too small");
    HIPCHK(r, hipSetDevice(r->device));
    GatherIn gi;
    gi.base = (const uint8_t*)hp;
    gi.seg_bytes = hp_export_plane((size_t)r->max_rows * r->W) * 28;
    gi.raw = 1;
    gi.segments = segments;
    gi.seg_rows = r->max_rows;
    gi.W = r->W;
    gi.indirect = (float*)indirect;
    gi.dbg = nullptr;
    gi.cull = r->slab ? 2u : 0u;
    gi.own_axis = r->own_axis;
    gi.own_lo = r->own_lo;
    gi.own_hi = r->own_hi;
    if (r->slab) gi.own_sb = slab_bins(r, r->own_nb);
    gi.visits = 0; /* rank-local counts are not the reference's; no per-pixel debug buffers here */
    gi.order = gather_order((size_t)r->W * r->H);
    hipStream_t st = cur_stream(r);
    if (r->last_pipelined) { /* on the side stream, after the grid build */
        st = gather_stream(r);
        HIPCHK(r, hipStreamWaitEvent(st, r->ev_grid_done, 0));
    }
    ev_begin_on(r, P_GATHER, st);
    if (r->slab && r->cfg.photon_map == 0) { /* the tiles with hit points that reach this rank's photons */
        const size_t ntiles = (size_t)((r->W + 15) / 16) * ((segments * r->max_rows + 15) / 16);
        HIPCHK(r, r->d_tiles.ensure(ntiles * 5 + 64));
        uint32_t* list = r->d_tiles.as<uint32_t>();
        uint32_t* count = list + ntiles;
        uint8_t* flags = (uint8_t*)(count + 4);
        launch_gather_tiles(st, gi, r->pb, r->last_consts, flags, list, count);
        gi.tile_list = list;
        gi.tile_count = count;
    }
    if (r->cfg.photon_map == 2) launch_ppm_gather_kd(st, gi, r->pb, r->kd, r->last_consts);
    else launch_ppm_gather(st, gi, r->pb, r->last_consts);
    ev_end_on(r, P_GATHER, st);
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}

orx_status orx_ppm_finish_on(orx_renderer* r, const void* indirect, size_t bytes, void* stream) {
    if (!r || !indirect) return ORX_ERR_INVALID_ARGUMENT;
    size_t need = (size_t)r->max_rows * r->W * 12;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "indirect buffer too small");
    HIPCHK(r, hipSetDevice(r->device));
    if (r->last_pipelined) {
        /* output only (direct ran beside the grid build), on `stream` (NULL: the side stream): the oldest
         * outstanding iteration, i.e. the one before the last eye pass if its finish was held back */
        if (!r->fin_snap && !r->fin_due) return set_err(r, ORX_ERR_STATE, "no sharded PPM iteration to finish");
        const bool prev = r->fin_snap;
        const PixelBufs px = prev ? r->fin_px : r->px;
        const Consts c = prev ? r->fin_consts : r->last_consts;
        const uint32_t k = prev ? r->fin_pp : r->pp;
        hipStream_t g = stream ? (hipStream_t)stream : gather_stream(r);
        launch_indirect_atten(g, px, (uint32_t)(need / 12), (const float*)indirect);
        /* the direct pass of that iteration: not yet overwritten, since the next one's photon pass (which
         * records the event again) is issued after this finish */
        HIPCHK(r, hipStreamWaitEvent(g, r->ev_direct_done, 0));
        ev_begin_on(r, P_DIRECT, g);
        launch_ppm_direct_output(g, r->scene, px, c, 2);
        ev_end_on(r, P_DIRECT, g);
        HIPCHK(r, hipEventRecord(r->ev_gdone[k], g));
        if (prev) r->fin_snap = false;
        else r->fin_due = false;
        r->pend = true;
        HIPCHK(r, hipGetLastError());
        return ORX_OK;
    }
    hipStream_t st = stream ? (hipStream_t)stream : cur_stream(r);
    launch_indirect_atten(st, r->px, (uint32_t)(need / 12), (const float*)indirect);
    ev_begin_on(r, P_DIRECT, st);
    launch_ppm_direct_output(st, r->scene, r->px, r->last_consts);
    ev_end_on(r, P_DIRECT, st);
    HIPCHK(r, hipGetLastError());
    return ORX_OK;
}
orx_status orx_ppm_finish(orx_renderer* r, const void* indirect, size_t bytes) {
    return orx_ppm_finish_on(r, indirect, bytes, nullptr);
}

orx_status orx_set_ppm_pipeline(orx_renderer* r, void* side_stream, int enable) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    if (enable && r->cfg.photon_map == 1)
        return set_err(r, ORX_ERR_UNSUPPORTED, "sharded PPM pipelining needs the uniform grid or kd-tree photon map");
    HIPCHK(r, hipSetDevice(r->device));
    orx_status s0 = sync_all(r);
    if (s0 != ORX_OK) return s0;
    r->shard_pipe = enable != 0;
    r->side = enable ? (hipStream_t)side_stream : nullptr;
    r->fin_due = r->fin_snap = false;
    r->rng_ready = false; /* re-allocate the frame with the second buffer set (as orx_set_shard) */
    return ORX_OK;
}

size_t orx_vcm_splat_bytes(const orx_renderer* r) { return r ? (size_t)r->W * r->max_rows * r->world * 12 : 0; }

orx_status orx_vcm_local_light(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                               float ppm_radius, const orx_request* det) {
    (void)iteration_number;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    if (det->method != ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING)
        return set_err(r, ORX_ERR_INVALID_ARGUMENT, "orx_vcm_local_light needs a VCM request");
    if (vcm_check_lights(r) != ORX_OK) return ORX_ERR_UNSUPPORTED;
    orx_status s = begin_iteration(r, local_iteration_number, det);
    if (s != ORX_OK) return s;
    if ((s = vcm_prepare(r, det, ppm_radius)) != ORX_OK) return s;
    if ((s = vcm_light(r)) != ORX_OK) return s;
    HIPCHK(r, hipGetLastError());
    r->vcm_pending = true;
    r->last_method = (uint64_t)det->method;
    r->last_consts = make_consts(r, ppm_radius, local_iteration_number);
    return ORX_OK;
}

orx_status orx_export_vcm_splats(orx_renderer* r, void* dst, size_t bytes) {
    if (!r || !dst) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->vcm_pending) return set_err(r, ORX_ERR_STATE, "no VCM light pass to export");
    const size_t need = orx_vcm_splat_bytes(r);
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "destination too small");
    HIPCHK(r, hipSetDevice(r->device));
    HIPCHK(r, hipMemcpyAsync(dst, r->d_vsplat.p, need, hipMemcpyDeviceToDevice, cur_stream(r)));
    return ORX_OK;
}

orx_status orx_vcm_finish(orx_renderer* r, const void* splat_own_rows, size_t bytes) {
    if (!r || !splat_own_rows) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->vcm_pending) return set_err(r, ORX_ERR_STATE, "orx_vcm_finish without a light pass");
    const size_t need = (size_t)r->W * r->rows * 12;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "splat buffer too small");
    HIPCHK(r, hipSetDevice(r->device));
    /* the summed own-row splats replace the local ones (readable as ORX_BUF_VCM_SPLAT) */
    float* own = r->d_vsplat.as<float>() + (size_t)r->rank * r->max_rows * r->W * 3;
    if ((const void*)own != splat_own_rows)
        HIPCHK(r, hipMemcpyAsync(own, splat_own_rows, need, hipMemcpyDeviceToDevice, cur_stream(r)));
    orx_status s = vcm_camera(r);
    if (s != ORX_OK) return s;
    HIPCHK(r, hipGetLastError());
    r->vcm_pending = false;
    return ORX_OK;
}

orx_status orx_set_stream(orx_renderer* r, void* stream, int use_external) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    HIPCHK(r, hipSetDevice(r->device));
    orx_status s0 = sync_all(r);
    if (s0 != ORX_OK) return s0;
    r->use_ext = use_external != 0;
    r->ext_stream = (hipStream_t)stream;
    return ORX_OK;
}
uint32_t orx_local_rows(const orx_renderer* r) { return r ? r->rows : 0; }
uint32_t orx_max_local_rows(const orx_renderer* r) { return r ? (r->H + r->world - 1) / r->world : 0; }
size_t orx_hitpoint_export_bytes(const orx_renderer* r) {
    return r ? hp_export_plane((size_t)((r->H + r->world - 1) / r->world) * r->W) * 28 : 0;
}

static orx_status check_grid_error(orx_renderer* r) {
    if (r->last_method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING || !r->d_grid.p) return ORX_OK;
    GridParams g;
    orx_status s0 = sync_all(r);
    if (s0 != ORX_OK) return s0;
    HIPCHK(r, hipMemcpy(&g, r->d_grid.p, sizeof g, hipMemcpyDeviceToHost));
    if (g.error)
        return set_err(r, ORX_ERR_GRID_TOO_LARGE, "Too many cells in SpatialHash.cu, over defined PHOTON_GRID_MAX_SIZE.");
    return ORX_OK;
}

orx_status orx_get_output(orx_renderer* r, float* dst, size_t bytes) {
    if (!r || !dst) return ORX_ERR_INVALID_ARGUMENT;
    size_t need = (size_t)r->rows * r->W * 12;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "destination too small");
    if (!r->d_out.p) return set_err(r, ORX_ERR_STATE, "no frame rendered yet");
    HIPCHK(r, hipSetDevice(r->device));
    orx_status s0 = sync_all(r);
    if (s0 != ORX_OK) return s0;
    HIPCHK(r, hipMemcpy(dst, r->d_out.p, need, hipMemcpyDeviceToHost));
    return check_grid_error(r);
}

orx_status orx_get_output_device(orx_renderer* r, void* dst, size_t bytes) {
    if (!r || !dst) return ORX_ERR_INVALID_ARGUMENT;
    size_t need = (size_t)r->rows * r->W * 12;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "destination too small");
    if (!r->d_out.p) return set_err(r, ORX_ERR_STATE, "no frame rendered yet");
    HIPCHK(r, hipSetDevice(r->device));
    /* after the last pipelined output pass; the pipeline itself stays unbroken (the copy only
     * reads the running sum, which the next output pass, on the gather stream after the grid
     * build that follows this copy on the main stream, writes) */
    if (r->pend) HIPCHK(r, hipStreamWaitEvent(cur_stream(r), r->ev_gdone[r->pp], 0));
    HIPCHK(r, hipMemcpyAsync(dst, r->d_out.p, need, hipMemcpyDeviceToDevice, cur_stream(r)));
    return ORX_OK;
}

uint32_t orx_width(const orx_renderer* r) { return r ? r->W : 0; }
uint32_t orx_height(const orx_renderer* r) { return r ? r->H : 0; }
size_t orx_output_bytes(const orx_renderer* r) { return r ? (size_t)r->W * r->H * 12 : 0; }
uint32_t orx_emitted_photons_per_iteration(const orx_renderer* r) {
    return r ? r->cfg.photon_launch_width * r->cfg.photon_launch_height : 0;
}

orx_status orx_read_buffer(orx_renderer* r, int32_t id, void* dst, size_t bytes, size_t* out_bytes) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    if (!r->rng_ready) return set_err(r, ORX_ERR_STATE, "no frame rendered yet");
    HIPCHK(r, hipSetDevice(r->device));
    {
        orx_status s0 = sync_all(r);
        if (s0 != ORX_OK) return s0;
    }
    GridParams g{};
    HIPCHK(r, hipMemcpy(&g, r->d_grid.p, sizeof g, hipMemcpyDeviceToHost));
    const size_t npx = (size_t)r->rows * r->W;
    const size_t nslot = (size_t)r->rng_rows * r->RW;
    size_t need = 0;
    switch (id) {
    case ORX_BUF_RNG: need = nslot * 24; break;
    case ORX_BUF_HITPOINTS: need = npx * 13 * 4; break;
    case ORX_BUF_PHOTONS: need = (r->pb.hash ? (size_t)r->pb.hnum : (size_t)g.valid) * 36; break;
    case ORX_BUF_GRID_OFFSETS: need = (r->pb.hash ? (size_t)r->pb.hnum : (size_t)g.G + 1) * 4; break;
    case ORX_BUF_INDIRECT: case ORX_BUF_DIRECT: case ORX_BUF_OUTPUT: need = npx * 12; break;
    case ORX_BUF_PHOTON_SLOTS: need = (size_t)r->pb.S * 36; break;
    case ORX_BUF_KD_TREE: need = r->cfg.photon_map == 2 ? (size_t)r->kd.tree_size * 40 : 0; break;
    case ORX_BUF_DEBUG_VISITED: need = npx * 8; break;
    case ORX_BUF_VCM_VERTEX_COUNT: need = r->vcm_npx * 4; break;
    case ORX_BUF_VCM_VERTICES: need = r->vcm_npx * VCM_MAX_VERTS * 64; break;
    case ORX_BUF_VCM_SPLAT: case ORX_BUF_VCM_CAMERA: need = r->vcm_npx * 12; break;
    case ORX_BUF_VOLUMETRIC: need = r->media ? npx * 12 : 0; break;
    case ORX_BUF_VOLUMETRIC_PHOTONS: need = r->media ? (size_t)r->cfg.volumetric_photons * 28 : 0; break;
    default: return set_err(r, ORX_ERR_INVALID_ARGUMENT, "unknown buffer id");
    }
    if (out_bytes) *out_bytes = need;
    if (!dst) return ORX_OK;
    if (bytes < need) return set_err(r, ORX_ERR_INVALID_ARGUMENT, "destination too small");
    auto d2h = [&](void* h, const void* d, size_t n) { return hipMemcpy(h, d, n, hipMemcpyDeviceToHost); };
    switch (id) {
    case ORX_BUF_RNG: {
        std::vector<uint32_t> planes(nslot * 6);
        HIPCHK(r, d2h(planes.data(), r->d_rng.p, nslot * 24));
        uint32_t* o = (uint32_t*)dst;
        for (size_t i = 0; i < nslot; i++)
            for (int k = 0; k < 6; k++) o[6 * i + k] = planes[k * nslot + i];
        break;
    }
    case ORX_BUF_HITPOINTS: {
        const size_t nhp = (size_t)r->max_rows * r->W;
        std::vector<float4> A(npx), B(npx);
        std::vector<float2> Cc(npx);
        HIPCHK(r, d2h(A.data(), r->d_hp.p, npx * 16));
        HIPCHK(r, d2h(B.data(), r->d_hp.as<float4>() + nhp, npx * 16));
        HIPCHK(r, d2h(Cc.data(), r->d_hp.as<float4>() + 2 * nhp, npx * 8));
        float* o = (float*)dst;
        for (size_t i = 0; i < npx; i++) {
            uint32_t flags;
            std::memcpy(&flags, &A[i].w, 4);
            bool ns = (flags & PRD_HIT_NON_SPECULAR) != 0;
            float v[13] = {A[i].x, A[i].y, A[i].z,
                           ns ? B[i].x : 0.f, ns ? B[i].y : 0.f, ns ? B[i].z : 0.f,
                           B[i].w, Cc[i].x, Cc[i].y,
                           ns ? 0.f : B[i].x, ns ? 0.f : B[i].y, ns ? 0.f : B[i].z, A[i].w};
            std::memcpy(o + 13 * i, v, sizeof v);
        }
        break;
    }
    case ORX_BUF_PHOTONS: {
        if (r->pb.hash) { /* the table: each entry's photon (its winning slot), zeros when empty */
            const size_t hn = r->pb.hnum, ns = (size_t)r->pb.S;
            std::vector<uint32_t> cnt(hn), win(hn);
            std::vector<float4> R(4 * ns);
            HIPCHK(r, d2h(cnt.data(), r->pb.hcount, hn * 4));
            HIPCHK(r, d2h(win.data(), r->pb.hwin, hn * 4));
            if (ns) HIPCHK(r, d2h(R.data(), r->d_slots.p, ns * 64));
            float* o = (float*)dst;
            for (size_t h = 0; h < hn; h++) {
                float v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                if (cnt[h] && win[h] && win[h] <= ns) {
                    const float4 a = R[4 * (win[h] - 1)], b = R[4 * (win[h] - 1) + 1], c = R[4 * (win[h] - 1) + 2];
                    const float t[9] = {a.w, b.w, c.x, a.x, a.y, a.z, b.x, b.y, b.z};
                    std::memcpy(v, t, sizeof v);
                }
                std::memcpy(o + 9 * h, v, sizeof v);
            }
            break;
        }
        /* nine SoA planes -> [n][power3 position3 direction3] (Photon.h:10-33 order) */
        const size_t n = g.valid, P = r->pb.splane;
        std::vector<float> pl(9 * n);
        static const uint32_t order[9] = {SP_PX, SP_PY, SP_PZ, SP_X, SP_Y, SP_Z, SP_DX, SP_DY, SP_DZ};
        for (int q = 0; q < 9 && n; q++)
            HIPCHK(r, d2h(pl.data() + q * n, r->d_sorted.as<float>() + order[q] * P, n * 4));
        /* sub-row layout: present the reference's cell order (each cell = its
         * nsub sub-row pieces, k_bs_count); within a cell the order is free */
        std::vector<uint32_t> idx;
        if (r->pb.subofs && r->pb.nsub > 1 && n) {
            const size_t rowlen = (size_t)g.gx * SUBX, nso = (size_t)g.G * r->pb.nsub * SUBX + 1;
            std::vector<uint32_t> so(nso);
            HIPCHK(r, d2h(so.data(), r->pb.subofs, nso * 4));
            idx.reserve(n);
            for (size_t c = 0; c < g.G; c++) {
                const size_t row = c / g.gx, x = c % g.gx;
                for (uint32_t sr = 0; sr < r->pb.nsub; sr++) {
                    const size_t b = (row * r->pb.nsub + sr) * rowlen + x * SUBX;
                    for (uint32_t k = so[b]; k < so[b + SUBX]; k++) idx.push_back(k);
                }
            }
            if (idx.size() != n) return set_err(r, ORX_ERR_STATE, "sub-row offsets do not cover the valid photons");
        }
        float* o = (float*)dst;
        for (size_t i = 0; i < n; i++) {
            const size_t src = idx.empty() ? i : idx[i];
            for (int k = 0; k < 9; k++) o[9 * i + k] = pl[k * n + src];
        }
        break;
    }
    case ORX_BUF_PHOTON_SLOTS: {
        const size_t n = (size_t)r->pb.S;
        std::vector<float4> R(4 * n);
        std::vector<uint8_t> vm((size_t)r->prows * r->cfg.photon_launch_width);
        if (n) HIPCHK(r, d2h(R.data(), r->d_slots.p, n * 64));
        if (!vm.empty()) HIPCHK(r, d2h(vm.data(), r->d_vmask.p, vm.size()));
        float* o = (float*)dst;
        const uint32_t D = r->pb.D; /* slots per emitted photon */
        for (size_t i = 0; i < n; i++) {
            const bool valid = (vm[i / D] >> (i % D)) & 1u;
            const float4 a = R[4 * i], b = R[4 * i + 1], c = R[4 * i + 2];
            float v[9] = {a.w, b.w, c.x, a.x, a.y, a.z, b.x, b.y, b.z};
            if (!valid) std::memset(v, 0, sizeof v);
            std::memcpy(o + 9 * i, v, sizeof v);
        }
        break;
    }
    case ORX_BUF_KD_TREE: { /* [tree_size][power3 position3 direction3 axis] */
        const size_t n = r->kd.tree_size;
        std::vector<float4> T(3 * n);
        if (n) HIPCHK(r, d2h(T.data(), r->kd.tree, n * 16));
        if (n) HIPCHK(r, d2h(T.data() + n, r->kd.tree_bc, n * 32));
        float* o = (float*)dst;
        for (size_t i = 0; i < n; i++) {
            const float4 a = T[i], b = T[n + 2 * i], c = T[n + 2 * i + 1];
            const float v[10] = {b.x, b.y, b.z, a.x, a.y, a.z, b.w, c.x, c.y, a.w};
            std::memcpy(o + 10 * i, v, sizeof v);
        }
        break;
    }
    case ORX_BUF_GRID_OFFSETS: HIPCHK(r, d2h(dst, r->pb.hash ? r->d_hcount.p : r->d_offsets.p, need)); break;
    case ORX_BUF_INDIRECT: HIPCHK(r, d2h(dst, r->d_ind.p, need)); break;
    case ORX_BUF_VOLUMETRIC: if (need) HIPCHK(r, d2h(dst, r->d_volR.p, need)); break;
    case ORX_BUF_VOLUMETRIC_PHOTONS: {
        if (!need) break;
        const size_t NV = r->cfg.volumetric_photons;
        std::vector<uint32_t> cnt(NV);
        std::vector<float4> A(NV), B(NV);
        HIPCHK(r, d2h(cnt.data(), r->d_vcnt.p, NV * 4));
        HIPCHK(r, d2h(A.data(), r->d_vA.p, NV * 16));
        HIPCHK(r, d2h(B.data(), r->d_vB.p, NV * 16));
        float* o = (float*)dst;
        for (size_t i = 0; i < NV; i++) {
            const bool on = r->vm.valid && cnt[i];
            float v[7] = {on ? B[i].x : 0.f, on ? B[i].y : 0.f, on ? B[i].z : 0.f,
                          on ? A[i].x : 0.f, on ? A[i].y : 0.f, on ? A[i].z : 0.f, 0.f};
            const uint32_t c = on ? cnt[i] : 0u;
            std::memcpy(&v[6], &c, 4);
            std::memcpy(o + 7 * i, v, sizeof v);
        }
        break;
    }
    case ORX_BUF_DIRECT: HIPCHK(r, d2h(dst, r->d_dir.p, need)); break;
    case ORX_BUF_OUTPUT: HIPCHK(r, d2h(dst, r->d_out.p, need)); break;
    case ORX_BUF_DEBUG_VISITED: HIPCHK(r, d2h(dst, r->d_dbg.p, need)); break;
    case ORX_BUF_VCM_VERTEX_COUNT: HIPCHK(r, d2h(dst, r->d_vcount.p, need)); break;
    case ORX_BUF_VCM_SPLAT: /* own rows of the owner-block buffer */
        HIPCHK(r, d2h(dst, r->d_vsplat.as<float>() + (size_t)r->rank * r->max_rows * r->W * 3, need));
        break;
    case ORX_BUF_VCM_CAMERA: HIPCHK(r, d2h(dst, r->d_vcam.p, need)); break;
    case ORX_BUF_VCM_VERTICES: { /* four float4 planes [9][npx] -> [9][npx][16] */
        const size_t plane = r->vcm_npx * VCM_MAX_VERTS;
        std::vector<float4> P(4 * plane);
        HIPCHK(r, d2h(P.data(), r->d_vverts.p, 4 * plane * 16));
        float* o = (float*)dst;
        for (size_t i = 0; i < plane; i++)
            for (int k = 0; k < 4; k++) std::memcpy(o + 16 * i + 4 * k, &P[k * plane + i], 16);
        break;
    }
    }
    return ORX_OK;
}

orx_status orx_get_stats(orx_renderer* r, orx_stats* out) {
    if (!r || !out) return ORX_ERR_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof *out);
    HIPCHK(r, hipSetDevice(r->device));
    {
        orx_status s0 = sync_all(r);
        if (s0 != ORX_OK) return s0;
    }
    if (r->d_grid.p) {
        GridParams g;
        HIPCHK(r, hipMemcpy(&g, r->d_grid.p, sizeof g, hipMemcpyDeviceToHost));
        out->grid_size[0] = g.gx;
        out->grid_size[1] = g.gy;
        out->grid_size[2] = g.gz;
        out->cell_size = g.cell;
        out->world_origin[0] = g.ox;
        out->world_origin[1] = g.oy;
        out->world_origin[2] = g.oz;
        out->valid_photons = g.valid;
        out->num_cells = g.G;
        out->photons_visited = g.photons_visited;
        out->cells_visited = g.cells_visited;
        out->photons_visited_total = g.photons_visited_total;
        out->cells_visited_total = g.cells_visited_total;
        out->valid_photons_total = g.valid_total;
        for (const DevBuf* b : {&r->d_grid2, &r->d_grid3}) { /* the other buffer sets' share of the totals */
            if (!r->pipe_bufs || !b->p || (b == &r->d_grid3 && r->nsets < 3)) continue;
            GridParams g2;
            HIPCHK(r, hipMemcpy(&g2, b->p, sizeof g2, hipMemcpyDeviceToHost));
            out->photons_visited_total += g2.photons_visited_total;
            out->cells_visited_total += g2.cells_visited_total;
            out->valid_photons_total += g2.valid_total;
        }
    }
    if (r->vcm_vb.dq0 && r->vcm_npx) { /* the last VCM camera pass's deferred connection shadow rays */
        uint32_t ctl[2] = {0, 0};
        HIPCHK(r, hipMemcpy(ctl, r->vcm_vb.dctl, 8, hipMemcpyDeviceToHost));
        out->vcm_shadow_rays = ctl[0];
        out->vcm_shadow_overflow = ctl[1];
    }
    if (r->vcm_vb.lcq && r->vcm_vb.lctl) { /* the last light pass's deferred camera connections */
        uint32_t ctl[2] = {0, 0};
        HIPCHK(r, hipMemcpy(ctl, r->vcm_vb.lctl, 8, hipMemcpyDeviceToHost));
        /* entries reserved minus those a wave could not fit and traced in place (their reserved range
         * below lcap holds inert placeholders): the connections the resolve traced */
        out->vcm_light_connections = ctl[0] - std::min(ctl[0], ctl[1]);
        out->vcm_light_inplace = ctl[1];
    }
    for (int p = 0; p < P_COUNT; p++) {
        double tot = 0.0;
        for (int k = 0; k < r->ev_n[p]; k++) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, r->ev[p][2 * k], r->ev[p][2 * k + 1]) == hipSuccess) tot += ms;
        }
        out->pass_ms[p] = (float)tot;
    }
    out->timed_iterations = r->timed_iterations;
    out->bvh_stack_entries = r->scene.stack_entries;
    return check_grid_error(r);
}

int orx_ppm_pipelined(const orx_renderer* r) { return r && (r->last_pipelined || r->last_vcm_overlap) ? 1 : 0; }
int orx_ppm_grid_schedule(const orx_renderer* r, float* probe_ms) {
    if (!r) return -2;
    if (probe_ms) {
        probe_ms[0] = r->probe_ms[0];
        probe_ms[1] = r->probe_ms[1];
    }
    return r->probe_stage ? -1 : r->async_grid ? 1 : 0;
}
orx_status orx_set_iteration_pipelining(orx_renderer* r, int mode) {
    if (!r || mode < -1 || mode > 1) return ORX_ERR_INVALID_ARGUMENT;
    r->pipe_mode = mode;
    return ORX_OK;
}

orx_status orx_reset_timing(orx_renderer* r) {
    if (!r) return ORX_ERR_INVALID_ARGUMENT;
    HIPCHK(r, hipSetDevice(r->device));
    {
        orx_status s0 = sync_all(r);
        if (s0 != ORX_OK) return s0;
    }
    for (int p = 0; p < P_COUNT; p++) r->ev_n[p] = 0;
    r->timed_iterations = 0;
    for (DevBuf* b : {&r->d_grid, &r->d_grid2, &r->d_grid3}) {
        if (!b->p || (b != &r->d_grid && !r->pipe_bufs) || (b == &r->d_grid3 && r->nsets < 3)) continue;
        GridParams g;
        HIPCHK(r, hipMemcpy(&g, b->p, sizeof g, hipMemcpyDeviceToHost));
        g.photons_visited_total = 0;
        g.cells_visited_total = 0;
        g.valid_total = 0;
        g.union_photons_total = 0;
        HIPCHK(r, hipMemcpy(b->p, &g, sizeof g, hipMemcpyHostToDevice));
    }
    return ORX_OK;
}

}  // extern "C"
