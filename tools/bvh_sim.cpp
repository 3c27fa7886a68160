// CPU model of the traversal cost of BVH layouts on photon-like rays (design tool, not product).
// Binary binned-SAH build (the orx builder's rules: 32 bins, SAH leaf test with leaf cost
// ORX_BVH_LEAF_SAH, leaf cap), collapse to width 4 or 8 by opening the largest-area inner
// child, then per-ray counts of node visits, child box tests, leaves and triangle tests for
//   w4-sort   four-wide, hit children sorted by entry distance (the shipped traversal)
//   w8-sort   eight-wide, same order
//   w8-oct    eight-wide, children visited in the order slot ^ octant(ray) with slots assigned
//             at build time (Ylitie et al. 2017), no sort
// Rays: photon paths of the synthetic hall (area light, cosine emission, up to 4 diffuse
// bounces, closest hit).  Input: scratch/hall.bin written by a few lines of numpy.
//   g++ -O2 -std=c++17 tools/bvh_sim.cpp -o scratch/bvh_sim && scratch/bvh_sim scratch/hall.bin
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
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

struct Tri {
    float lo[3], hi[3], c[3];
};
struct N2 {
    float lo[3], hi[3];
    int l = -1, r = -1;
    uint32_t first = 0, count = 0;
};
std::vector<V3> P;
std::vector<uint32_t> I;
std::vector<Tri> tris;
std::vector<uint32_t> prims;
std::vector<N2> b2;
int LEAF_MAX = 8;
int QBITS = 0;
float LEAF_SAH = 0.6f;

static float area(const float* lo, const float* hi) {
    float dx = std::max(0.f, hi[0] - lo[0]), dy = std::max(0.f, hi[1] - lo[1]), dz = std::max(0.f, hi[2] - lo[2]);
    return dx * dy + dy * dz + dz * dx;
}
int build(uint32_t first, uint32_t count) {
    int idx = (int)b2.size();
    b2.push_back(N2{});
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = first; i < first + count; i++) {
        const Tri& t = tris[prims[i]];
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], t.lo[k]);
            hi[k] = std::max(hi[k], t.hi[k]);
            clo[k] = std::min(clo[k], t.c[k]);
            chi[k] = std::max(chi[k], t.c[k]);
        }
    }
    for (int k = 0; k < 3; k++) b2[idx].lo[k] = lo[k], b2[idx].hi[k] = hi[k];
    b2[idx].first = first;
    b2[idx].count = count;
    if (count <= 1) return idx;
    const int NB = 32;
    int ba = -1, bs = 0;
    float bc = INFINITY;
    for (int ax = 0; ax < 3; ax++) {
        float ext = chi[ax] - clo[ax];
        if (!(ext > 0)) continue;
        uint32_t cnt[NB] = {0};
        float blo[NB][3], bhi[NB][3];
        for (int b = 0; b < NB; b++)
            for (int k = 0; k < 3; k++) blo[b][k] = INFINITY, bhi[b][k] = -INFINITY;
        for (uint32_t i = first; i < first + count; i++) {
            const Tri& t = tris[prims[i]];
            int b = std::min(NB - 1, (int)((t.c[ax] - clo[ax]) / ext * NB));
            cnt[b]++;
            for (int k = 0; k < 3; k++) blo[b][k] = std::min(blo[b][k], t.lo[k]), bhi[b][k] = std::max(bhi[b][k], t.hi[k]);
        }
        float rl[NB], rc[NB], alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t acc = 0;
        for (int b = NB - 1; b > 0; b--) {
            acc += cnt[b];
            for (int k = 0; k < 3; k++) alo[k] = std::min(alo[k], blo[b][k]), ahi[k] = std::max(ahi[k], bhi[b][k]);
            rl[b] = area(alo, ahi);
            rc[b] = (float)acc;
        }
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t lc = 0;
        for (int b = 0; b < NB - 1; b++) {
            lc += cnt[b];
            for (int k = 0; k < 3; k++) llo[k] = std::min(llo[k], blo[b][k]), lhi[k] = std::max(lhi[k], bhi[b][k]);
            float cost = area(llo, lhi) * lc + rl[b + 1] * rc[b + 1];
            if (lc > 0 && lc < count && cost < bc) bc = cost, ba = ax, bs = b;
        }
    }
    if ((int)count <= LEAF_MAX) {
        float A = area(lo, hi);
        if (ba < 0 || !(A > 0) || LEAF_SAH + bc / A >= (float)count) return idx;
    }
    uint32_t mid;
    if (ba < 0) {
        mid = first + count / 2;
    } else {
        float ext = chi[ba] - clo[ba];
        auto it = std::stable_partition(prims.begin() + first, prims.begin() + first + count, [&](uint32_t p) {
            return std::min(NB - 1, (int)((tris[p].c[ba] - clo[ba]) / ext * NB)) <= bs;
        });
        mid = (uint32_t)(it - prims.begin());
        if (mid == first || mid == first + count) mid = first + count / 2;
    }
    int l = build(first, mid - first);
    int r = build(mid, first + count - mid);
    b2[idx].l = l;
    b2[idx].r = r;
    return idx;
}

struct WNode {
    int n = 0;
    float lo[8][3], hi[8][3];
    int child[8];      /* >= 0 inner node index, < 0: leaf binary node ~idx */
    /* treelet of the opened binary nodes: entry e < 0 -> slot ~e; tl[i] = {axis, a, b}: a is the
     * child with the lower centroid on axis */
    int ntl = 0, tl[7][3];
};
std::vector<WNode> wn;
static float b2area(int i) { return area(b2[i].lo, b2[i].hi); }
static int split_axis(int a, int b) {
    float best = -1;
    int ax = 0;
    for (int k = 0; k < 3; k++) {
        float d = std::fabs((b2[b].lo[k] + b2[b].hi[k]) - (b2[a].lo[k] + b2[a].hi[k]));
        if (d > best) best = d, ax = k;
    }
    return ax;
}
int collapse(int n2, int W, bool octant) {
    std::vector<int> ch;
    /* treelet: owner[i] = treelet entry the list position i came from */
    std::vector<std::array<int, 3>> tl;
    std::vector<int> pos_tl;  /* for each list position: (treelet index, side) encoded tl*2+side, -1 root */
    if (b2[n2].l < 0) ch.push_back(n2);
    else {
        ch = {b2[n2].l, b2[n2].r};
        tl.push_back({split_axis(b2[n2].l, b2[n2].r), 0, 0});
        pos_tl = {0, 1};
        while ((int)ch.size() < W) {
            int bi = -1;
            float bar = -1;
            for (size_t i = 0; i < ch.size(); i++)
                if (b2[ch[i]].l >= 0 && b2area(ch[i]) > bar) bar = b2area(ch[i]), bi = (int)i;
            if (bi < 0) break;
            int c = ch[bi];
            int t = (int)tl.size();
            tl.push_back({split_axis(b2[c].l, b2[c].r), 0, 0});
            /* the parent's reference to position bi now points at treelet t */
            int pt = pos_tl[bi];
            tl[pt / 2][1 + pt % 2] = t + 1000;
            ch[bi] = b2[c].l;
            ch.push_back(b2[c].r);
            pos_tl[bi] = 2 * t;
            pos_tl.push_back(2 * t + 1);
        }
        for (size_t i = 0; i < ch.size(); i++) tl[pos_tl[i] / 2][1 + pos_tl[i] % 2] = ~(int)i;  /* position -> slot below */
    }
    int idx = (int)wn.size();
    wn.push_back(WNode{});
    std::vector<int> slot_of(ch.size(), -1);
    if (octant && W == 8) {
        /* greedy slot assignment: slot s is visited first by rays of octant s (direction signs
         * s&1 -> -x, s&2 -> -y, s&4 -> -z); cost of child c in slot s = its centroid projected on
         * the octant's diagonal (smaller = nearer for those rays); take the globally cheapest
         * (child, slot) pair repeatedly */
        float pc[3] = {0, 0, 0};
        std::vector<V3> cc(ch.size());
        for (size_t i = 0; i < ch.size(); i++) {
            for (int k = 0; k < 3; k++) pc[k] += 0.5f * (b2[ch[i]].lo[k] + b2[ch[i]].hi[k]) / ch.size();
        }
        for (size_t i = 0; i < ch.size(); i++)
            cc[i] = {0.5f * (b2[ch[i]].lo[0] + b2[ch[i]].hi[0]) - pc[0], 0.5f * (b2[ch[i]].lo[1] + b2[ch[i]].hi[1]) - pc[1],
                     0.5f * (b2[ch[i]].lo[2] + b2[ch[i]].hi[2]) - pc[2]};
        std::vector<bool> used_s(8, false);
        for (size_t done = 0; done < ch.size(); done++) {
            float best = INFINITY;
            int bi = -1, bsl = -1;
            for (size_t i = 0; i < ch.size(); i++) {
                if (slot_of[i] >= 0) continue;
                for (int s = 0; s < 8; s++) {
                    if (used_s[s]) continue;
                    V3 d = {(s & 1) ? -1.f : 1.f, (s & 2) ? -1.f : 1.f, (s & 4) ? -1.f : 1.f};
                    float c = dot(cc[i], d);
                    if (c < best) best = c, bi = (int)i, bsl = s;
                }
            }
            slot_of[bi] = bsl;
            used_s[bsl] = true;
        }
    } else {
        for (size_t i = 0; i < ch.size(); i++) slot_of[i] = (int)i;
    }
    wn[idx].n = W;
    for (int s = 0; s < 8; s++) wn[idx].child[s] = INT32_MIN, wn[idx].lo[s][0] = INFINITY;
    wn[idx].ntl = (int)tl.size();
    for (size_t t = 0; t < tl.size(); t++) {
        wn[idx].tl[t][0] = tl[t][0];
        for (int e = 1; e < 3; e++) {
            int v = tl[t][e];
            wn[idx].tl[t][e] = v >= 1000 ? v - 1000 : ~slot_of[~v];
        }
    }
    for (size_t i = 0; i < ch.size(); i++) {
        int s = slot_of[i];
        for (int k = 0; k < 3; k++) {
            float lo = b2[ch[i]].lo[k], hi = b2[ch[i]].hi[k];
            /* the builder's conservative 1e-6 expansion, then outward quantisation on QBITS bits
             * against the node box (QBITS 0: exact) */
            const float m = std::max(std::fabs(lo), std::fabs(hi)), e = m * 1e-6f + 1e-20f;
            lo -= e;
            hi += e;
            if (QBITS) {
                float nlo = INFINITY, nhi = -INFINITY;
                for (size_t j = 0; j < ch.size(); j++) nlo = std::min(nlo, b2[ch[j]].lo[k] - e), nhi = std::max(nhi, b2[ch[j]].hi[k] + e);
                const float steps = (float)((1 << QBITS) - 1);
                int ee;
                std::frexp((nhi - nlo) / steps, &ee);
                const float sc = std::ldexp(1.0f, ee);  /* power-of-two step >= extent/steps */
                lo = nlo + std::floor((lo - nlo) / sc) * sc;
                hi = nlo + std::ceil((hi - nlo) / sc) * sc;
            }
            wn[idx].lo[s][k] = lo, wn[idx].hi[s][k] = hi;
        }
        int c = ch[i];
        int ref = b2[c].l < 0 ? ~c : collapse(c, W, octant);
        wn[idx].child[s] = ref;
    }
    return idx;
}

struct Stats {
    double rays = 0, nodes = 0, boxes = 0, leaves = 0, tris = 0, pushes = 0;
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
/* mode 0: sort by entry; mode 1: octant order */
static bool trace(int root, V3 o, V3 d, float& best, uint32_t& bt, int mode, Stats& st) {
    V3 inv = {1.f / d.x, 1.f / d.y, 1.f / d.z};
    int oct = (d.x < 0) | ((d.y < 0) << 1) | ((d.z < 0) << 2);
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
            for (int s0 = 0; s0 < n.n; s0++) {
                int s = mode == 1 ? (s0 ^ oct) : s0;
                if (n.child[s] == INT32_MIN) continue;
                st.boxes++;
                float t0 = 1e-4f, t1 = best;
                for (int k = 0; k < 3; k++) {
                    float a = (n.lo[s][k] - comp(o, k)) * comp(inv, k), b = (n.hi[s][k] - comp(o, k)) * comp(inv, k);
                    t0 = std::max(t0, std::min(a, b));
                    t1 = std::min(t1, std::max(a, b));
                }
                if (t0 <= t1) te[nh] = t0, ci[nh++] = n.child[s];
            }
            if (mode == 2 && n.ntl) { /* treelet order: at each opened node the child nearer along its
                                       * split axis (by the ray's direction sign) first */
                float pri[8];
                for (int s = 0; s < 8; s++) pri[s] = 0;
                /* DFS assigning visit ranks */
                int rank = 0;
                std::vector<int> st2 = {0};
                while (!st2.empty()) {
                    int e = st2.back();
                    st2.pop_back();
                    if (e < 0) {
                        pri[~e] = (float)rank++;
                        continue;
                    }
                    const int* t = n.tl[e];
                    /* which side has the lower centroid along the axis: side a (index 1) was built
                     * as the binary left child; compare with the recorded boxes is not stored, so
                     * use the split-axis convention: left = lower coordinates */
                    bool neg = comp(d, t[0]) < 0;
                    int first = neg ? t[2] : t[1], second = neg ? t[1] : t[2];
                    st2.push_back(second);
                    st2.push_back(first);
                }
                int idx8[8];
                int m = 0;
                for (int s0 = 0; s0 < n.n; s0++) {
                    int s = s0;
                    if (n.child[s] == INT32_MIN) continue;
                    idx8[m++] = s;
                }
                (void)idx8;
                /* reorder the hit list by pri of the slot the child came from: recompute */
                float tp[8];
                int cp[8], k2 = 0;
                for (int s = 0; s < n.n; s++) {
                    if (n.child[s] == INT32_MIN) continue;
                    for (int h = 0; h < nh; h++)
                        if (ci[h] == n.child[s]) tp[k2] = pri[s], cp[k2++] = ci[h];
                }
                for (int a = 1; a < k2; a++)
                    for (int b = a; b > 0 && tp[b] < tp[b - 1]; b--) std::swap(tp[b], tp[b - 1]), std::swap(cp[b], cp[b - 1]);
                for (int h = 0; h < k2; h++) ci[h] = cp[h];
                nh = k2;
            }
            if (mode == 0) { /* insertion sort by entry */
                for (int a = 1; a < nh; a++)
                    for (int b = a; b > 0 && te[b] < te[b - 1]; b--) std::swap(te[b], te[b - 1]), std::swap(ci[b], ci[b - 1]);
            }
            for (int a = nh - 1; a >= 1; a--) stk.push_back(ci[a]), st.pushes++;
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
                if (isect_tri(prims[k], o, d, best, t)) best = t, bt = prims[k], hit = true;
            }
        }
        if (stk.empty()) break;
        cur = stk.back();
        stk.pop_back();
    }
    return hit;
}

/* any hit in (1e-4, tmax): children in slot order, all hits pushed */
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
                float t0 = 1e-4f, t1 = tmax;
                for (int k = 0; k < 3; k++) {
                    float a = (n.lo[s][k] - comp(o, k)) * comp(inv, k), b = (n.hi[s][k] - comp(o, k)) * comp(inv, k);
                    t0 = std::max(t0, std::min(a, b));
                    t1 = std::min(t1, std::max(a, b));
                }
                if (t0 <= t1) stk.push_back(n.child[s]), st.pushes++;
            }
        } else {
            const N2& l = b2[~cur];
            st.leaves++;
            for (uint32_t k = l.first; k < l.first + l.count; k++) {
                st.tris++;
                float t;
                if (isect_tri(prims[k], o, d, tmax, t)) return true;
            }
        }
        if (stk.empty()) return false;
        cur = stk.back();
        stk.pop_back();
    }
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
    int nrays = argc > 2 ? std::atoi(argv[2]) : 200000;
    if (argc > 3) QBITS = std::atoi(argv[3]);
    tris.resize(nt);
    for (uint32_t t = 0; t < nt; t++) {
        for (int k = 0; k < 3; k++) tris[t].lo[k] = INFINITY, tris[t].hi[k] = -INFINITY;
        for (int v = 0; v < 3; v++)
            for (int k = 0; k < 3; k++) {
                float x = comp(P[I[3 * t + v]], k);
                tris[t].lo[k] = std::min(tris[t].lo[k], x);
                tris[t].hi[k] = std::max(tris[t].hi[k], x);
            }
        for (int k = 0; k < 3; k++) tris[t].c[k] = 0.5f * (tris[t].lo[k] + tris[t].hi[k]);
    }
    prims.resize(nt);
    for (uint32_t i = 0; i < nt; i++) prims[i] = i;
    build(0, nt);
    struct Var {
        const char* name;
        int W;
        bool oct;
        int mode;
    } vars[] = {{"w4-sort", 4, false, 0}, {"w8-sort", 8, false, 0}, {"w8-oct", 8, true, 1}, {"w8-oct-sorted", 8, true, 0}, {"w4-treelet", 4, false, 2}, {"w8-treelet", 8, false, 2}, {"w4-none", 4, false, 3}, {"w8-none", 8, false, 3}};
    V3 Lp = {L[0], L[1], L[2]}, L1 = {L[3], L[4], L[5]}, L2 = {L[6], L[7], L[8]};
    V3 Ln = norm(cross(L1, L2));
    for (auto& v : vars) {
        wn.clear();
        int root = collapse(0, v.W, v.oct);
        Stats st;
        std::mt19937 rng(7);
        std::uniform_real_distribution<float> U(0.f, 1.f);
        for (int r = 0; r < nrays; r++) {
            V3 o = Lp + L1 * U(rng) + L2 * U(rng);
            V3 n = Ln;
            for (int b = 0; b < 5; b++) {
                /* cosine hemisphere about n */
                float u1 = U(rng), u2 = U(rng), rr = std::sqrt(u1), ph = 6.2831853f * u2;
                V3 a = std::fabs(n.x) > 0.5f ? V3{0, 1, 0} : V3{1, 0, 0};
                V3 t1 = norm(cross(a, n)), t2 = cross(n, t1);
                V3 d = norm(t1 * (rr * std::cos(ph)) + t2 * (rr * std::sin(ph)) + n * std::sqrt(std::max(0.f, 1 - u1)));
                float best = 1e27f;
                uint32_t bt = 0;
                if (!trace(root, o, d, best, bt, v.mode, st)) break;
                o = o + d * best;
                V3 p0 = P[I[3 * bt]], p1 = P[I[3 * bt + 1]], p2 = P[I[3 * bt + 2]];
                n = norm(cross(p1 - p0, p2 - p0));
                if (dot(n, d) > 0) n = n * -1.f;
                if (U(rng) > 0.6f) break;
            }
        }
        std::printf("%-14s nodes %zu  per ray: nodes %.2f boxes %.1f pushes %.2f leaves %.2f tris %.2f  (rays %.0f)\n",
                    v.name, wn.size(), st.nodes / st.rays, st.boxes / st.rays, st.pushes / st.rays, st.leaves / st.rays,
                    st.tris / st.rays, st.rays);
        if (v.mode == 0 || v.mode == 3) {
            /* shadow segments between two photon-path hit points (VCM connections) */
            Stats sa;
            std::mt19937 rng2(11);
            std::vector<V3> pts;
            for (int r = 0; r < nrays && (int)pts.size() < 60000; r++) {
                V3 o = Lp + L1 * U(rng2) + L2 * U(rng2);
                float u1 = U(rng2), u2 = U(rng2), rr = std::sqrt(u1), ph = 6.2831853f * u2;
                V3 a = std::fabs(Ln.x) > 0.5f ? V3{0, 1, 0} : V3{1, 0, 0};
                V3 t1 = norm(cross(a, Ln)), t2 = cross(Ln, t1);
                V3 d = norm(t1 * (rr * std::cos(ph)) + t2 * (rr * std::sin(ph)) + Ln * std::sqrt(std::max(0.f, 1 - u1)));
                float best = 1e27f;
                uint32_t bt = 0;
                Stats dummy;
                if (trace(root, o, d, best, bt, 0, dummy)) pts.push_back(o + d * (best * 0.999f));
            }
            int occl = 0;
            for (size_t i = 0; i + 1 < pts.size(); i += 2) {
                V3 d = pts[i + 1] - pts[i];
                float len = std::sqrt(dot(d, d));
                d = d * (1.f / len);
                occl += trace_any(root, pts[i], d, len * 0.999f, sa);
            }
            std::printf("   any-hit segments: nodes %.2f boxes %.1f leaves %.2f tris %.2f (segments %.0f, occluded %d)\n",
                        sa.nodes / sa.rays, sa.boxes / sa.rays, sa.leaves / sa.rays, sa.tris / sa.rays, sa.rays, occl);
        }
    }
    return 0;
}
