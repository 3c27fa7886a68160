// CPU pricing of BVH builder quality (design tool, not product).
// The shipped tree: binary binned SAH (32 bins, SAH leaf test with traversal cost ORX_BVH_LEAF_SAH = 0.6
// relative to a triangle test, leaves of at most 8) collapsed to a 4-wide BVH by opening the largest-area
// inner child, 8-bit outward-quantised child boxes.  Variants priced against it, at the same node format:
//   collapse  sah      SAH-optimal binary -> 4-wide collapse (the dynamic programme of Ylitie et al. 2017:
//                      F(n, i) = cheapest cover of n's subtree by at most i roots)
//   treelet            treelet restructuring of the binary tree (Karras & Aila 2013, the restructuring OptiX's
//                      Trbvh builder does): per node, the 7-leaf treelet of largest-area expansions is rebuilt
//                      as the SAH-optimal binary tree over those 7 subtrees (DP over subsets), bottom-up,
//                      three passes
//   presplit           early split clipping (Ernst & Greiner 2007), a form of spatial splits: triangle
//                      references whose bounding box wastes the most area are split at the middle of their
//                      box's longest axis, each half's box the bounds of the triangle clipped to it, until
//                      the reference count reaches the budget (x1.1, x1.25); leaves then hold references
// Per ray of photon paths (area light, cosine emission, up to five diffuse bounces, closest hit, hit children
// visited near-first) and per any-hit segment between photon hit points (children in slot order): node
// visits, child box tests, leaves, triangle tests.
//   g++ -O2 -std=c++17 tools/bvh_quality.cpp -o scratch/bvh_quality
//   scratch/bvh_quality scratch/hall.bin [photon paths]      (python tools/dump_scene_bin.py writes the .bin)
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

struct V3 {
    float x, y, z;
};
static V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V3 norm(V3 a) { return a * (1.f / std::sqrt(dot(a, a))); }
static float comp(V3 a, int k) { return k == 0 ? a.x : k == 1 ? a.y : a.z; }

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], b.lo[k]), hi[k] = std::max(hi[k], b.hi[k]);
    }
    void grow(V3 p) {
        for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], comp(p, k)), hi[k] = std::max(hi[k], comp(p, k));
    }
    float area() const {
        float dx = std::max(0.f, hi[0] - lo[0]), dy = std::max(0.f, hi[1] - lo[1]), dz = std::max(0.f, hi[2] - lo[2]);
        return dx * dy + dy * dz + dz * dx;
    }
    float c(int k) const { return 0.5f * (lo[k] + hi[k]); }
};
struct Ref {
    uint32_t tri;
    Box b;
};
struct N2 {
    Box b;
    int l = -1, r = -1, parent = -1;
    uint32_t first = 0, count = 0; /* leaves: reference range */
    uint32_t nprim = 0;            /* references in the subtree */
    double cost = 0;               /* SAH cost of the subtree (area-weighted) */
};

std::vector<V3> P;
std::vector<uint32_t> I;
std::vector<Ref> refs;
std::vector<N2> b2;
int LEAF_MAX = 8;
float LEAF_SAH = 0.6f; /* binary traversal step relative to one triangle test */
int QBITS = 8;
int NBINS = 32;
int TL_LEAVES = 7;   /* treelet size */
float TL_CI = -1.f;  /* treelet inner cost (< 0: LEAF_SAH) */
static double CI() { return TL_CI < 0.f ? (double)LEAF_SAH : (double)TL_CI; }

static Box tri_box(uint32_t t) {
    Box b;
    for (int v = 0; v < 3; v++) b.grow(P[I[3 * t + v]]);
    return b;
}

/* ---- binary binned SAH (the shipped builder's rules, on references) ---- */
static int build(uint32_t first, uint32_t count) {
    int idx = (int)b2.size();
    b2.push_back(N2{});
    Box bb, cb;
    for (uint32_t i = first; i < first + count; i++) {
        bb.grow(refs[i].b);
        cb.grow(V3{refs[i].b.c(0), refs[i].b.c(1), refs[i].b.c(2)});
    }
    b2[idx].b = bb;
    b2[idx].first = first;
    b2[idx].count = count;
    if (count <= 1) return idx;
    constexpr int NBMAX = 256;
    const int NB = NBINS;
    int ba = -1, bs = 0;
    float bc = INFINITY;
    for (int ax = 0; ax < 3; ax++) {
        float ext = cb.hi[ax] - cb.lo[ax];
        if (!(ext > 0)) continue;
        uint32_t cnt[NBMAX] = {0};
        Box bin[NBMAX];
        for (uint32_t i = first; i < first + count; i++) {
            int b = std::min(NB - 1, (int)((refs[i].b.c(ax) - cb.lo[ax]) / ext * NB));
            cnt[b]++;
            bin[b].grow(refs[i].b);
        }
        float rl[NBMAX], rc[NBMAX];
        Box acc;
        uint32_t n = 0;
        for (int b = NB - 1; b > 0; b--) {
            n += cnt[b];
            acc.grow(bin[b]);
            rl[b] = acc.area();
            rc[b] = (float)n;
        }
        Box la;
        uint32_t lc = 0;
        for (int b = 0; b < NB - 1; b++) {
            lc += cnt[b];
            la.grow(bin[b]);
            float cost = la.area() * lc + rl[b + 1] * rc[b + 1];
            if (lc > 0 && lc < count && cost < bc) bc = cost, ba = ax, bs = b;
        }
    }
    if ((int)count <= LEAF_MAX) {
        float A = bb.area();
        if (ba < 0 || !(A > 0) || LEAF_SAH + bc / A >= (float)count) return idx;
    }
    uint32_t mid;
    if (ba < 0) {
        mid = first + count / 2;
    } else {
        float ext = cb.hi[ba] - cb.lo[ba];
        auto it = std::stable_partition(refs.begin() + first, refs.begin() + first + count, [&](const Ref& r) {
            return std::min(NB - 1, (int)((r.b.c(ba) - cb.lo[ba]) / ext * NB)) <= bs;
        });
        mid = (uint32_t)(it - refs.begin());
        if (mid == first || mid == first + count) mid = first + count / 2;
    }
    int l = build(first, mid - first);
    int r = build(mid, first + count - mid);
    b2[idx].l = l;
    b2[idx].r = r;
    return idx;
}

/* subtree costs (SAH, traversal step LEAF_SAH, triangle test 1), parents, primitive counts */
static void annotate(int n, int parent) {
    N2& x = b2[n];
    x.parent = parent;
    if (x.l < 0) {
        x.nprim = x.count;
        x.cost = (double)x.b.area() * x.count;
        return;
    }
    annotate(x.l, n);
    annotate(x.r, n);
    N2& y = b2[n];
    y.nprim = b2[y.l].nprim + b2[y.r].nprim;
    y.cost = CI() * y.b.area() + b2[y.l].cost + b2[y.r].cost;
}

/* ---- treelet restructuring (Karras & Aila 2013) ---- */
static bool restructure(int n) {
    if (b2[n].l < 0) return false;
    std::vector<int> leaves = {b2[n].l, b2[n].r}, inner = {n};
    while ((int)leaves.size() < TL_LEAVES) {
        int bi = -1;
        float ba = -1;
        for (size_t i = 0; i < leaves.size(); i++)
            if (b2[leaves[i]].l >= 0 && b2[leaves[i]].b.area() > ba) ba = b2[leaves[i]].b.area(), bi = (int)i;
        if (bi < 0) break;
        int c = leaves[bi];
        inner.push_back(c);
        leaves[bi] = b2[c].l;
        leaves.push_back(b2[c].r);
    }
    const int m = (int)leaves.size();
    if (m < 3) return false;
    const int full = (1 << m) - 1;
    std::vector<double> copt(1 << m, 0), area(1 << m, 0);
    std::vector<int> split(1 << m, 0);
    for (int S = 1; S <= full; S++) {
        Box b;
        for (int i = 0; i < m; i++)
            if (S >> i & 1) b.grow(b2[leaves[i]].b);
        area[S] = b.area();
    }
    for (int S = 1; S <= full; S++) {
        if ((S & (S - 1)) == 0) {
            copt[S] = b2[leaves[__builtin_ctz(S)]].cost;
            continue;
        }
        double best = INFINITY;
        int bp = 0;
        const int low = S & -S; /* the partition containing the lowest member: each split once */
        for (int Pp = (S - 1) & S; Pp; Pp = (Pp - 1) & S) {
            if (!(Pp & low)) continue;
            double c = copt[Pp] + copt[S ^ Pp];
            if (c < best) best = c, bp = Pp;
        }
        copt[S] = CI() * area[S] + best;
        split[S] = bp;
    }
    if (!(copt[full] < b2[n].cost * (1 - 1e-6))) return false;
    /* rebuild with the treelet's inner nodes (inner[0] = n keeps its place and parent) */
    size_t next = 1;
    const int parent_n = b2[n].parent;
    struct Rec {
        static int go(int S, int node_hint, std::vector<int>& inner, size_t& next, const std::vector<int>& split,
                      const std::vector<int>& leaves, int parent) {
            if ((S & (S - 1)) == 0) {
                int lf = leaves[__builtin_ctz(S)];
                b2[lf].parent = parent;
                return lf;
            }
            int id = node_hint >= 0 ? node_hint : inner[next++];
            int Pp = split[S];
            int l = go(Pp, -1, inner, next, split, leaves, id);
            int r = go(S ^ Pp, -1, inner, next, split, leaves, id);
            N2& x = b2[id];
            x.l = l;
            x.r = r;
            x.parent = parent;
            x.b = b2[l].b;
            x.b.grow(b2[r].b);
            x.nprim = b2[l].nprim + b2[r].nprim;
            x.cost = CI() * x.b.area() + b2[l].cost + b2[r].cost;
            return id;
        }
    };
    Rec::go(full, n, inner, next, split, leaves, parent_n);
    return true;
}
static int treelet_pass(int root) {
    /* post-order over the current tree */
    std::vector<int> order, st = {root};
    while (!st.empty()) {
        int n = st.back();
        st.pop_back();
        order.push_back(n);
        if (b2[n].l >= 0) st.push_back(b2[n].l), st.push_back(b2[n].r);
    }
    int changed = 0;
    for (auto it = order.rbegin(); it != order.rend(); ++it) {
        int n = *it;
        if (b2[n].l < 0) continue;
        /* children may have changed: refresh this node's box and cost first */
        N2& x = b2[n];
        x.b = b2[x.l].b;
        x.b.grow(b2[x.r].b);
        x.nprim = b2[x.l].nprim + b2[x.r].nprim;
        x.cost = CI() * x.b.area() + b2[x.l].cost + b2[x.r].cost;
        changed += restructure(n);
    }
    return changed;
}

/* ---- 4-wide collapse ---- */
struct WNode {
    int n = 0;
    float lo[8][3], hi[8][3];
    int child[8]; /* >= 0 wide node, < 0: binary leaf ~idx, INT32_MIN empty */
};
std::vector<WNode> wn;
static void set_child(WNode& w, int s, const std::vector<int>& ch, int c, int ref) {
    for (int k = 0; k < 3; k++) {
        float lo = b2[c].b.lo[k], hi = b2[c].b.hi[k];
        const float mm = std::max(std::fabs(lo), std::fabs(hi)), e = mm * 1e-6f + 1e-20f;
        lo -= e;
        hi += e;
        if (QBITS) {
            float nlo = INFINITY, nhi = -INFINITY;
            for (int j : ch) {
                const float m2 = std::max(std::fabs(b2[j].b.lo[k]), std::fabs(b2[j].b.hi[k])), e2 = m2 * 1e-6f + 1e-20f;
                nlo = std::min(nlo, b2[j].b.lo[k] - e2), nhi = std::max(nhi, b2[j].b.hi[k] + e2);
            }
            const float steps = (float)((1 << QBITS) - 1);
            int ee;
            std::frexp((nhi - nlo) / steps, &ee);
            const float sc = std::ldexp(1.0f, ee);
            lo = nlo + std::floor((lo - nlo) / sc) * sc;
            hi = nlo + std::ceil((hi - nlo) / sc) * sc;
        }
        w.lo[s][k] = lo, w.hi[s][k] = hi;
    }
    w.child[s] = ref;
}
static int collapse_area(int n2, int W) {
    std::vector<int> ch;
    if (b2[n2].l < 0) ch.push_back(n2);
    else {
        ch = {b2[n2].l, b2[n2].r};
        while ((int)ch.size() < W) {
            int bi = -1;
            float bar = -1;
            for (size_t i = 0; i < ch.size(); i++)
                if (b2[ch[i]].l >= 0 && b2[ch[i]].b.area() > bar) bar = b2[ch[i]].b.area(), bi = (int)i;
            if (bi < 0) break;
            int c = ch[bi];
            ch[bi] = b2[c].l;
            ch.push_back(b2[c].r);
        }
    }
    int idx = (int)wn.size();
    wn.push_back(WNode{});
    wn[idx].n = W;
    for (int s = 0; s < 8; s++) wn[idx].child[s] = INT32_MIN;
    for (size_t i = 0; i < ch.size(); i++) {
        int c = ch[i];
        int ref = b2[c].l < 0 ? ~c : collapse_area(c, W);
        set_child(wn[idx], (int)i, ch, c, ref);
    }
    return idx;
}
/* SAH-optimal collapse: F[n][i] for i = 1..W, C_NODE per wide-node visit, 1 per triangle test */
float C_NODE = 2.5f;
std::vector<std::array<double, 9>> F;
std::vector<std::array<int, 9>> Fk; /* i >= 2: 0 = one root, k = k roots to the left child */
static void dp(int n, int W) {
    N2& x = b2[n];
    auto& f = F[n];
    auto& fk = Fk[n];
    if (x.l < 0) {
        for (int i = 1; i <= W; i++) f[i] = (double)x.b.area() * x.count, fk[i] = 0;
        return;
    }
    dp(x.l, W);
    dp(x.r, W);
    auto G = [&](int i, int& kbest) {
        double best = INFINITY;
        for (int k = 1; k < i; k++) {
            double c = F[x.l][k] + F[x.r][i - k];
            if (c < best) best = c, kbest = k;
        }
        return best;
    };
    int k;
    f[1] = (double)C_NODE * x.b.area() + G(W, k);
    fk[1] = k; /* the children distribution of this node's own wide node */
    for (int i = 2; i <= W; i++) {
        double g = G(i, k);
        if (g < f[1]) f[i] = g, fk[i] = k;
        else f[i] = f[1], fk[i] = 0;
    }
}
static void roots(int n, int i, std::vector<int>& out) {
    if (i == 1 || b2[n].l < 0 || Fk[n][i] == 0) {
        out.push_back(n);
        return;
    }
    roots(b2[n].l, Fk[n][i], out);
    roots(b2[n].r, i - Fk[n][i], out);
}
static int collapse_sah(int n2, int W) {
    std::vector<int> ch;
    if (b2[n2].l < 0) ch.push_back(n2);
    else {
        const int k = Fk[n2][1];
        roots(b2[n2].l, k, ch);
        roots(b2[n2].r, W - k, ch);
    }
    int idx = (int)wn.size();
    wn.push_back(WNode{});
    wn[idx].n = W;
    for (int s = 0; s < 8; s++) wn[idx].child[s] = INT32_MIN;
    for (size_t i = 0; i < ch.size(); i++) {
        int c = ch[i];
        int ref = b2[c].l < 0 ? ~c : collapse_sah(c, W);
        set_child(wn[idx], (int)i, ch, c, ref);
    }
    return idx;
}

/* ---- traversal model ---- */
struct Stats {
    double rays = 0, nodes = 0, boxes = 0, leaves = 0, tris = 0;
    double deep = 0, maxd = 0; /* pushes past the 16 LDS stack entries (the global column), deepest stack */
};
static bool isect_tri(uint32_t t, V3 o, V3 d, float tmax, float& tout) {
    V3 p0 = P[I[3 * t]], p1 = P[I[3 * t + 1]], p2 = P[I[3 * t + 2]];
    V3 e0 = p1 - p0, e1 = p0 - p2, n = cross(e1, e0);
    V3 e2 = (p0 - o) * (1.0f / dot(n, d));
    V3 i = cross(d, e2);
    float beta = dot(i, e1), gamma = dot(i, e0), tt = dot(n, e2);
    if (tt < tmax && tt > 1e-4f && beta >= 0 && gamma >= 0 && beta + gamma <= 1) {
        tout = tt;
        return true;
    }
    return false;
}
static bool slab(const WNode& n, int s, V3 o, V3 inv, float tmax, float& t0) {
    float a0 = 1e-4f, t1 = tmax;
    for (int k = 0; k < 3; k++) {
        float a = (n.lo[s][k] - comp(o, k)) * comp(inv, k), b = (n.hi[s][k] - comp(o, k)) * comp(inv, k);
        a0 = std::max(a0, std::min(a, b));
        t1 = std::min(t1, std::max(a, b));
    }
    t0 = a0;
    return a0 <= t1;
}
static bool trace(int root, V3 o, V3 d, float& best, uint32_t& bt, Stats& st) {
    V3 inv = {1.f / d.x, 1.f / d.y, 1.f / d.z};
    std::vector<int> stk;
    stk.reserve(64);
    int cur = root;
    bool hit = false;
    st.rays++;
    for (;;) {
        if (cur >= 0) {
            const WNode& n = wn[cur];
            st.nodes++;
            float te[8];
            int ci[8], nh = 0;
            for (int s = 0; s < n.n; s++) {
                if (n.child[s] == INT32_MIN) continue;
                st.boxes++;
                float t0;
                if (slab(n, s, o, inv, best, t0)) te[nh] = t0, ci[nh++] = n.child[s];
            }
            for (int a = 1; a < nh; a++)
                for (int b = a; b > 0 && te[b] < te[b - 1]; b--) std::swap(te[b], te[b - 1]), std::swap(ci[b], ci[b - 1]);
            for (int a = nh - 1; a >= 1; a--) {
                stk.push_back(ci[a]);
                if (stk.size() > 16) st.deep++;
                st.maxd = std::max(st.maxd, (double)stk.size());
            }
            if (nh) {
                cur = ci[0];
                continue;
            }
        } else {
            const N2& l = b2[~cur];
            st.leaves++;
            for (uint32_t k = l.first; k < l.first + l.count; k++) {
                st.tris++;
                float t;
                if (isect_tri(refs[k].tri, o, d, best, t)) best = t, bt = refs[k].tri, hit = true;
            }
        }
        if (stk.empty()) break;
        cur = stk.back();
        stk.pop_back();
    }
    return hit;
}
static bool trace_any(int root, V3 o, V3 d, float tmax, Stats& st) {
    V3 inv = {1.f / d.x, 1.f / d.y, 1.f / d.z};
    std::vector<int> stk;
    stk.reserve(64);
    int cur = root;
    st.rays++;
    for (;;) {
        if (cur >= 0) {
            const WNode& n = wn[cur];
            st.nodes++;
            for (int s = 0; s < n.n; s++) {
                if (n.child[s] == INT32_MIN) continue;
                st.boxes++;
                float t0;
                if (slab(n, s, o, inv, tmax, t0)) stk.push_back(n.child[s]);
            }
        } else {
            const N2& l = b2[~cur];
            st.leaves++;
            for (uint32_t k = l.first; k < l.first + l.count; k++) {
                st.tris++;
                float t;
                if (isect_tri(refs[k].tri, o, d, tmax, t)) return true;
            }
        }
        if (stk.empty()) return false;
        cur = stk.back();
        stk.pop_back();
    }
}

/* ---- early split clipping ---- */
static void clip_poly(std::vector<V3>& poly, int ax, float v, bool keep_below) {
    std::vector<V3> out;
    for (size_t i = 0; i < poly.size(); i++) {
        V3 a = poly[i], b = poly[(i + 1) % poly.size()];
        float da = comp(a, ax) - v, db = comp(b, ax) - v;
        if (!keep_below) da = -da, db = -db;
        if (da <= 0) out.push_back(a);
        if ((da < 0 && db > 0) || (da > 0 && db < 0)) out.push_back(a + (b - a) * (da / (da - db)));
    }
    poly.swap(out);
}
static Box clip_box(uint32_t t, const Box& cell) {
    std::vector<V3> poly = {P[I[3 * t]], P[I[3 * t + 1]], P[I[3 * t + 2]]};
    for (int k = 0; k < 3 && !poly.empty(); k++) {
        clip_poly(poly, k, cell.lo[k], false);
        if (!poly.empty()) clip_poly(poly, k, cell.hi[k], true);
    }
    Box b;
    for (V3 p : poly) b.grow(p);
    for (int k = 0; k < 3; k++) /* rounding of the clip: stay inside the cell */
        b.lo[k] = std::max(b.lo[k], cell.lo[k]), b.hi[k] = std::min(b.hi[k], cell.hi[k]);
    return b;
}
static float tri_area(uint32_t t) {
    V3 c = cross(P[I[3 * t + 1]] - P[I[3 * t]], P[I[3 * t + 2]] - P[I[3 * t]]);
    return 0.5f * std::sqrt(dot(c, c));
}
static void presplit(uint32_t nt, double budget) {
    refs.clear();
    struct Item {
        double waste;
        uint32_t tri;
        Box b;
        bool operator<(const Item& o) const { return waste < o.waste; }
    };
    std::vector<Item> heap;
    for (uint32_t t = 0; t < nt; t++) {
        Box b = tri_box(t);
        heap.push_back({b.area() - 2.0 * tri_area(t), t, b});
    }
    std::make_heap(heap.begin(), heap.end());
    size_t total = nt, limit = (size_t)(budget * nt);
    while (total < limit && !heap.empty()) {
        Item it = heap.front();
        std::pop_heap(heap.begin(), heap.end());
        heap.pop_back();
        int ax = 0;
        for (int k = 1; k < 3; k++)
            if (it.b.hi[k] - it.b.lo[k] > it.b.hi[ax] - it.b.lo[ax]) ax = k;
        const float mid = it.b.c(ax);
        Box c0 = it.b, c1 = it.b;
        c0.hi[ax] = mid;
        c1.lo[ax] = mid;
        Box b0 = clip_box(it.tri, c0), b1 = clip_box(it.tri, c1);
        bool e0 = !(b0.lo[0] <= b0.hi[0]), e1 = !(b1.lo[0] <= b1.hi[0]);
        if (e0 || e1) { /* degenerate: keep whole */
            refs.push_back({it.tri, it.b});
            continue;
        }
        /* the halves' waste: their boxes' area minus their share of the triangle's (by box area) */
        const double share = 2.0 * tri_area(it.tri) / std::max(1e-30, (double)b0.area() + b1.area());
        heap.push_back({b0.area() * (1 - share), it.tri, b0});
        std::push_heap(heap.begin(), heap.end());
        heap.push_back({b1.area() * (1 - share), it.tri, b1});
        std::push_heap(heap.begin(), heap.end());
        total++;
    }
    for (auto& it : heap) refs.push_back({it.tri, it.b});
}

int main(int argc, char** argv) {
    FILE* f = std::fopen(argc > 1 ? argv[1] : "scratch/hall.bin", "rb");
    uint32_t nv, nt;
    if (!f || std::fread(&nv, 4, 1, f) != 1 || std::fread(&nt, 4, 1, f) != 1) return 1;
    P.resize(nv);
    I.resize(3 * (size_t)nt);
    float L[9];
    if (std::fread(P.data(), 12, nv, f) != nv || std::fread(I.data(), 4, 3 * (size_t)nt, f) != 3 * (size_t)nt ||
        std::fread(L, 4, 9, f) != 9)
        return 1;
    const int npaths = argc > 2 ? std::atoi(argv[2]) : 100000;
    V3 Lp = {L[0], L[1], L[2]}, L1 = {L[3], L[4], L[5]}, L2 = {L[6], L[7], L[8]};
    V3 Ln = norm(cross(L1, L2));
    /* the light faces into the scene: flip if most first rays miss */
    struct Var {
        const char* name;
        double split_budget; /* 1: no pre-splitting */
        int treelet_passes;
        int collapse; /* 0 largest area, 1 SAH DP */
        float c_node;
        int bins = 32;
        int tl_leaves = 7;
        float tl_ci = -1.f;
        float leaf_sah = 0.6f;
        int leaf_max = 8;
    };
    std::vector<Var> vars = {
        {"shipped r5 (area collapse)", 1.0, 0, 0, 0},
        {"r6: treelet x3, sah cn=2.5", 1.0, 3, 1, 2.5f},
        {"treelet x6, sah", 1.0, 6, 1, 2.5f},
        {"treelet9 x3, sah", 1.0, 3, 1, 2.5f, 32, 9},
        {"treelet x3 ci=1.2, sah", 1.0, 3, 1, 2.5f, 32, 7, 1.2f},
        {"treelet x3 ci=0.3, sah", 1.0, 3, 1, 2.5f, 32, 7, 0.3f},
        {"treelet9 x6 ci=1.2, sah", 1.0, 6, 1, 2.5f, 32, 9, 1.2f},
        {"t9 sah leafsah 0.4", 1.0, 3, 1, 2.5f, 32, 9, -1.f, 0.4f},
        {"t9 sah leafsah 0.9", 1.0, 3, 1, 2.5f, 32, 9, -1.f, 0.9f},
        {"t9 sah leafsah 1.3", 1.0, 3, 1, 2.5f, 32, 9, -1.f, 1.3f},
        {"t9 sah leafmax 4", 1.0, 3, 1, 2.5f, 32, 9, -1.f, 0.6f, 4},
    };
    if (getenv("BVHQ_ALL")) vars.insert(vars.end(), {
        {"sah collapse cn=2.5", 1.0, 0, 1, 2.5f},
        {"treelet x3, area collapse", 1.0, 3, 0, 0},
        {"presplit 1.10, area", 1.10, 0, 0, 0},
        {"presplit 1.25, area", 1.25, 0, 0, 0},
        {"presplit 1.25 + treelet + sah", 1.25, 3, 1, 2.5f},
        {"256 bins, area", 1.0, 0, 0, 0, 256},
        {"256 bins + treelet x3 + sah", 1.0, 3, 1, 2.5f, 256},
    });
    double base_nodes = 0, base_anodes = 0, base_tris = 0;
    for (const Var& v : vars) {
        if (v.split_budget > 1.0) presplit(nt, v.split_budget);
        else {
            refs.resize(nt);
            for (uint32_t t = 0; t < nt; t++) refs[t] = {t, tri_box(t)};
        }
        b2.clear();
        NBINS = v.bins;
        TL_LEAVES = v.tl_leaves;
        TL_CI = v.tl_ci;
        LEAF_SAH = v.leaf_sah;
        LEAF_MAX = v.leaf_max;
        build(0, (uint32_t)refs.size());
        annotate(0, -1);
        const double sah0 = b2[0].cost / b2[0].b.area();
        int changed = 0;
        for (int p = 0; p < v.treelet_passes; p++) changed += treelet_pass(0);
        annotate(0, -1);
        const double sah1 = b2[0].cost / b2[0].b.area();
        wn.clear();
        int root;
        if (v.collapse == 0) root = collapse_area(0, 4);
        else {
            C_NODE = v.c_node;
            F.assign(b2.size(), {});
            Fk.assign(b2.size(), {});
            dp(0, 4);
            root = collapse_sah(0, 4);
        }
        Stats st, sa;
        std::mt19937 rng(7);
        std::uniform_real_distribution<float> U(0.f, 1.f);
        std::vector<V3> pts;
        for (int r = 0; r < npaths; r++) {
            V3 o = Lp + L1 * U(rng) + L2 * U(rng);
            V3 n = Ln;
            for (int b = 0; b < 5; b++) {
                float u1 = U(rng), u2 = U(rng), rr = std::sqrt(u1), ph = 6.2831853f * u2;
                V3 a = std::fabs(n.x) > 0.5f ? V3{0, 1, 0} : V3{1, 0, 0};
                V3 t1 = norm(cross(a, n)), t2 = cross(n, t1);
                V3 d = norm(t1 * (rr * std::cos(ph)) + t2 * (rr * std::sin(ph)) + n * std::sqrt(std::max(0.f, 1 - u1)));
                float best = 1e27f;
                uint32_t bt = 0;
                if (!trace(root, o, d, best, bt, st)) break;
                o = o + d * best;
                if (pts.size() < 60000) pts.push_back(o - d * (best * 0.001f));
                V3 p0 = P[I[3 * bt]], p1 = P[I[3 * bt + 1]], p2 = P[I[3 * bt + 2]];
                n = norm(cross(p1 - p0, p2 - p0));
                if (dot(n, d) > 0) n = n * -1.f;
                if (U(rng) > 0.6f) break;
            }
        }
        for (size_t i = 0; i + 1 < pts.size(); i += 2) {
            V3 d = pts[i + 1] - pts[i];
            float len = std::sqrt(dot(d, d));
            if (!(len > 1e-3f)) continue;
            d = d * (1.f / len);
            trace_any(root, pts[i], d, len * 0.999f, sa);
        }
        const double nodes = st.nodes / st.rays, an = sa.nodes / sa.rays, tr = st.tris / st.rays;
        if (base_nodes == 0) base_nodes = nodes, base_anodes = an, base_tris = tr;
        std::printf("%-30s refs %7zu  SAH %.1f -> %.1f (%d restructured)  wide nodes %6zu\n", v.name, refs.size(), sah0, sah1,
                    changed, wn.size());
        std::printf("    photon rays %.0f: nodes %.2f (%+.1f%%) boxes %.1f leaves %.2f tris %.2f (%+.1f%%)  pushes past 16: %.3f/ray, max depth %.0f\n",
                    st.rays, nodes, 100 * (nodes / base_nodes - 1), st.boxes / st.rays, st.leaves / st.rays, tr,
                    100 * (tr / base_tris - 1), st.deep / st.rays, st.maxd);
        std::printf("    any-hit segments %.0f: nodes %.2f (%+.1f%%) boxes %.1f leaves %.2f tris %.2f\n", sa.rays, an,
                    100 * (an / base_anodes - 1), sa.boxes / sa.rays, sa.leaves / sa.rays, sa.tris / sa.rays);
        std::fflush(stdout);
    }
    return 0;
}
