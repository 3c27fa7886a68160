/*
 * orx_oracle.c — plain-C restatement of OppositeRenderer's progressive photon
 * mapping (PPM) and path tracing (PT) passes.  TEST INFRASTRUCTURE ONLY (see
 * orx_oracle.h).  Every function cites the reference file:line it follows;
 * float expressions keep the reference's operand order because the build
 * runs with -ffp-contract=off and the GPU kernels evaluate the same order.
 *
 * OptiX vector semantics used throughout (optixu_math_namespace.h, OptiX 3.x):
 *   dot(a,b) = a.x*b.x + a.y*b.y + a.z*b.z
 *   normalize(v) = v * (1.0f / sqrtf(dot(v,v)))
 *   float3 / float  = float3 * (1.0f / s)
 *   reflect(i,n) = i - 2*n*dot(n,i)
 * CUDA fast-math transcendentals are replaced by orx_detmath.h (see there).
 */
#include "orx_oracle.h"
#include "orx_detmath.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* float3                                                              */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 mk1(float a) { return mk(a, a, a); }
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 sub_s(v3 a, float s) { return mk(a.x - s, a.y - s, a.z - s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 divs(v3 a, float s) { float inv = 1.0f / s; return scl(a, inv); }
static inline v3 divv(v3 a, v3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float length(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 normalize(v3 a) { float inv = 1.0f / sqrtf(dot(a, a)); return scl(a, inv); }
static inline float maxf(float a, float b) { return a > b ? a : b; } /* helpers.h:143-146 */
static inline float fmax3(v3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
static inline v3 vmin(v3 a, v3 b) { return mk(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
static inline v3 vmax(v3 a, v3 b) { return mk(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
static inline float favgf(v3 v) { return (v.x + v.y + v.z) * 0.3333333333f; } /* helpers.h:163-166 */
static inline v3 reflect(v3 i, v3 n) { return sub(i, scl(scl(n, 2.0f), dot(n, i))); }
static inline int isnan3(v3 v) { return v.x != v.x || v.y != v.y || v.z != v.z; }

/* OptiX refract (optixu_math_namespace.h) */
static int refract(v3* r, v3 i, v3 n, float ior) {
    v3 nn = n;
    float negNdotV = dot(i, nn);
    float eta;
    if (negNdotV > 0.0f) {
        eta = ior;
        nn = neg(n);
        negNdotV = -negNdotV;
    } else {
        eta = 1.f / ior;
    }
    const float k = 1.f - eta * eta * (1.f - negNdotV * negNdotV);
    if (k < 0.0f) {
        *r = mk1(0.f);
        return 0;
    }
    *r = normalize(sub(scl(i, eta), scl(nn, eta * negNdotV + sqrtf(k))));
    return 1;
}

/* ------------------------------------------------------------------ */
/* cuRAND XORWOW (curand_kernel.h, CUDA 5.5) and helpers/random.h      */
/* ------------------------------------------------------------------ */
void orc_xorwow_init(uint64_t seed, uint32_t st[6]) {
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    st[5] = 6615241u + t1 + t0;
    st[0] = 123456789u + t0;
    st[1] = 362436069u ^ t0;
    st[2] = 521288629u + t1;
    st[3] = 88675123u ^ t1;
    st[4] = 5783321u + t0;
}
uint32_t orc_xorwow_next(uint32_t st[6]) {
    uint32_t t = st[0] ^ (st[0] >> 2);
    st[0] = st[1];
    st[1] = st[2];
    st[2] = st[3];
    st[3] = st[4];
    st[4] = (st[4] ^ (st[4] << 4)) ^ (t ^ (t << 1));
    st[5] += 362437u;
    return st[4] + st[5];
}
/* getRandomUniformFloat: max(curand_uniform - FLT_EPSILON, 0) (helpers/random.h:65-69);
 * curand_uniform = x*2^-32 + 2^-33, contracted to one FMA by nvcc. */
float orc_uniform(uint32_t st[6]) {
    uint32_t x = orc_xorwow_next(st);
    float u = fmaf((float)x, 2.3283064e-10f, 2.3283064e-10f / 2.0f);
    return maxf(u - ORX_FLT_EPSILON, 0.0f);
}

/* ------------------------------------------------------------------ */
/* samplers (helpers/samplers.h, helpers/helpers.h)                    */
/* ------------------------------------------------------------------ */
static void create_coordinate_system(v3 N, v3* U, v3* V) { /* helpers.h:119-134 */
    if (fabsf(N.x) > fabsf(N.y)) {
        float invLength = 1.f / sqrtf(N.x * N.x + N.z * N.z);
        *U = mk(-N.z * invLength, 0.f, N.x * invLength);
    } else {
        float invLength = 1.f / sqrtf(N.y * N.y + N.z * N.z);
        *U = mk(0.f, N.z * invLength, -N.y * invLength);
    }
    *V = cross(N, *U);
}
/* samplers.h:24-43 (no pdf outputs, no bias) */
static v3 sample_hemisphere_cos(v3 normal, float sx, float sy) {
    float theta = orx_acosf(sqrtf(sx));
    float phi = 2.0f * ORX_PI_F * sy;
    float st = orx_sinf(theta);
    float xs = st * orx_cosf(phi);
    float ys = orx_cosf(theta);
    float zs = st * orx_sinf(phi);
    v3 U, V;
    create_coordinate_system(normal, &U, &V);
    return normalize(add(add(scl(U, xs), scl(normal, ys)), scl(V, zs)));
}
/* samplers.h:46-57 */
static v3 sample_hemisphere(v3 normal, float sx, float sy) {
    v3 U, V;
    create_coordinate_system(normal, &U, &V);
    float phi = 2.0f * ORX_PI_F * sx;
    float r = sqrtf(sy);
    float x = r * orx_cosf(phi);
    float y = r * orx_sinf(phi);
    float z = 1.0f - x * x - y * y;
    z = z > 0.0f ? sqrtf(z) : 0.0f;
    return normalize(add(add(scl(U, x), scl(V, y)), scl(normal, z)));
}
/* samplers.h:59-72 */
static v3 sample_unit_sphere(float sx, float sy) {
    v3 v;
    v.z = 1.f - 2.f * sx;
    float phi = 2 * ORX_PI_F * sy;
    float r = sqrtf(1.f - v.z * v.z);
    v.x = r * orx_cosf(phi);
    v.y = r * orx_sinf(phi);
    return v;
}
/* samplers.h:74-93 */
static v3 sample_disc(float sx, float sy, v3 center, float radius, v3 normal) {
    v3 U, V;
    create_coordinate_system(normal, &U, &V);
    float r = sqrtf(sx);
    float theta = 2.f * ORX_PI_F * sy;
    float x = r * orx_cosf(theta);
    float y = r * orx_sinf(theta);
    return add(center, scl(add(scl(U, x), scl(V, y)), radius));
}

void orc_sample_unit_hemisphere_cos(const float n[3], float u1, float u2, float out[3]) {
    v3 r = sample_hemisphere_cos(ld3(n), u1, u2);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void orc_sample_unit_hemisphere(const float n[3], float u1, float u2, float out[3]) {
    v3 r = sample_hemisphere(ld3(n), u1, u2);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ------------------------------------------------------------------ */
/* scene                                                               */
/* ------------------------------------------------------------------ */
#define ORC_RT_DEFAULT_MAX 1.e27f /* optix_device.h RT_DEFAULT_MAX */
#define PRD_HIT_EMITTER (1u << 31)
#define PRD_ERROR (1u << 30)
#define PRD_MISS (1u << 29)
#define PRD_HIT_SPECULAR (1u << 28)
#define PRD_HIT_NON_SPECULAR (1u << 27)
#define PRD_PATH_TRACING (1u << 26)

typedef struct {
    int type;
    v3 Kd, Ks, Kr, Kt;
    float ior, exponent;
    v3 powerPerArea, Lemit;
    float inverseArea;
    int tex; /* Texture: index into the scene's textures */
} mat_t;

/* Texture images (material/Texture.cpp:83-107): diffuse map + optional normal map */
typedef struct { uint32_t w, h, nw, nh; uint8_t* rgba; uint8_t* nrgba; } tex_t;

typedef struct {
    int type;
    v3 power, position, v1, v2, normal, Lemit; /* Lemit doubles as intensity (Light.h union) */
    v3 direction;
    float area, inverseArea, angle;
} light_t;

typedef struct { v3 n; float d; v3 anchor, v1, v2; } quadp_t;
typedef struct { v3 c; float r; } sphere_t;

typedef struct { v3 position, normal, attenuation, radiance; uint32_t flags; } hitpoint_t;
typedef struct { v3 power, position, direction; } photon_t; /* Photon.h:10-33 */
typedef struct kdphoton { photon_t p; uint32_t axis; } kdphoton_t; /* KD_TREE_CPU adds `axis` (Photon.h:27-29) */

struct orc_renderer {
    orx_config cfg;
    char err[512];
    int scene_ready;
    /* scene */
    uint32_t nq, ns, nt, nv, nm, nl;
    quadp_t* quads; uint32_t* qmat;
    sphere_t* sph; uint32_t* smat;
    v3* verts; v3* vnorm; int has_normals;
    uint32_t* tris; uint32_t* tmat;
    float* uv; v3* tang; v3* btan; /* texCoordBuffer, tangentBuffer, bitangentBuffer (or NULL) */
    tex_t* tex; uint32_t ntex; int has_tex;
    /* triangle BVH: node i = {lo[3], hi[3], left|first, right|count|leafbit} */
    float* bvh_box; uint32_t* bvh_a; uint32_t* bvh_b; uint32_t* bvh_prims; uint32_t bvh_n;
    mat_t* mats;
    light_t* lights;
    v3 aabb_min, aabb_max;
    v3 bs_center; float bs_radius;
    /* frame; sharding: this renderer owns RNG/pixel/photon rows y % world == rank */
    uint32_t W, H, RW, RH;
    uint32_t rank, world, rows, max_rows, prows;
    float last_radius, last_radius2;
    uint64_t last_local;
    int rng_ready;
    uint32_t* rng; /* [RW*RH][6] */
    hitpoint_t* hp;
    photon_t* photons; uint32_t* keys; photon_t* sort_tmp;
    uint32_t* offsets; uint32_t* hist;
    v3* indirect; v3* direct; v3* output;
    uint32_t* dbg; /* [W*H][2] */
    /* grid state */
    uint32_t gsize[3]; float cell; v3 origo; uint32_t ncells; uint32_t valid;
    /* stochastic hash (cfg.photon_map == 1): dslot slots per emitted photon, deposits per photon,
     * photonsHashTableCount and the slot + 1 each entry keeps */
    uint32_t dslot; uint8_t* ndep; uint32_t* hcount; uint32_t* hwin; size_t hnum;
    /* kd-tree photon map (cfg.photon_map == 2): Photon records with their `axis` (Photon.h:27-29),
     * the working copy of the slots and the implicit tree of kdsize nodes */
    struct kdphoton* kdwork; struct kdphoton* kdtree; size_t kdsize; uint32_t kddepth;
    uint64_t sum_photons_visited, sum_cells_visited;
    /* VCM: pixelSizeFactor (OptixRenderer.cpp:306, :846), LVC-estimated flag (:83, :461, :847) */
    float psf_x, psf_y;
    int vcm_estimated, vcm_pending;
    /* slab mode: the bins on own_axis whose hit points this rank gathers (orc_ppm_slab_import) */
    int own_on;
    uint32_t own_axis, own_nb, own_lo, own_hi;
    size_t vcm_npx, vcm_spx;
    uint32_t* vcount; float* vverts; v3* vsplat; v3* vcam;
    v3* vkd; /* [9][lpx] texel colour of Texture light vertices */
    void* vcm_ctx; /* vcm_ctx_t of the pending sharded light pass */
    /* participating medium (cfg.enable_media, ENABLE_PARTICIPATING_MEDIA): one box
     * (geometry_instance/AAB.cu) with ParticipatingMedium's programs; the volumetric photon
     * table (NUM_VOLUMETRIC_PHOTONS slots: power, position, numDeposits) of the last photon pass,
     * gathered by the next eye pass with that iteration's radius */
    int med_on;
    v3 med_lo, med_hi;
    float sig_s, sig_a;
    uint32_t nvol;
    v3* vpow; v3* vpos; uint32_t* vcnt;
    int vol_ready;
    float vol_R;
    uint32_t* ev_n; v3* ev_pos; v3* ev_pow; /* per emitted photon: scatter events, the last one */
    v3* volR;                               /* per pixel: Hitpoint::volumetricRadiance */
};

static orx_status fail(orc_renderer* r, orx_status s, const char* msg) {
    if (r) snprintf(r->err, sizeof r->err, "%s", msg);
    return s;
}

const char* orc_last_error(const orc_renderer* r) { return r ? r->err : "null renderer"; }

void orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

orx_status orc_create(const orx_config* cfg, orc_renderer** out) {
    if (!out) return ORX_ERR_INVALID_ARGUMENT;
    orc_renderer* r = (orc_renderer*)calloc(1, sizeof *r);
    if (!r) return ORX_ERR_OUT_OF_MEMORY;
    if (cfg) r->cfg = *cfg;
    else orc_default_config(&r->cfg);
    r->W = 10; r->H = 10; /* OptixRenderer ctor m_width(10), m_height(10) */
    r->psf_x = 1.0f; r->psf_y = 1.0f;
    r->world = 1;
    *out = r;
    return ORX_OK;
}

static void free_scene(orc_renderer* r) {
    free(r->bvh_box); free(r->bvh_a); free(r->bvh_b); free(r->bvh_prims);
    r->bvh_box = NULL; r->bvh_a = NULL; r->bvh_b = NULL; r->bvh_prims = NULL; r->bvh_n = 0;
    free(r->quads); free(r->qmat); free(r->sph); free(r->smat);
    free(r->verts); free(r->vnorm); free(r->tris); free(r->tmat);
    free(r->mats); free(r->lights);
    for (uint32_t i = 0; i < r->ntex; i++) { free(r->tex[i].rgba); free(r->tex[i].nrgba); }
    free(r->tex); free(r->uv); free(r->tang); free(r->btan);
    r->tex = NULL; r->ntex = 0; r->has_tex = 0; r->uv = NULL; r->tang = NULL; r->btan = NULL;
    r->quads = NULL; r->qmat = NULL; r->sph = NULL; r->smat = NULL; r->verts = NULL;
    r->vnorm = NULL; r->tris = NULL; r->tmat = NULL; r->mats = NULL; r->lights = NULL;
    free(r->vpow); free(r->vpos); free(r->vcnt);
    r->vpow = NULL; r->vpos = NULL; r->vcnt = NULL; r->med_on = 0; r->vol_ready = 0;
}
static void free_frame(orc_renderer* r) {
    free(r->rng); free(r->hp); free(r->photons); free(r->keys); free(r->sort_tmp);
    free(r->offsets); free(r->hist); free(r->indirect); free(r->direct); free(r->output); free(r->dbg);
    r->rng = NULL; r->hp = NULL; r->photons = NULL; r->keys = NULL; r->sort_tmp = NULL;
    r->offsets = NULL; r->hist = NULL; r->indirect = NULL; r->direct = NULL; r->output = NULL; r->dbg = NULL;
    free(r->vcount); free(r->vverts); free(r->vsplat); free(r->vcam); free(r->vkd);
    r->vkd = NULL;
    r->vcount = NULL; r->vverts = NULL; r->vsplat = NULL; r->vcam = NULL; r->vcm_npx = 0; r->vcm_spx = 0;
    free(r->ndep); free(r->hcount); free(r->hwin);
    r->ndep = NULL; r->hcount = NULL; r->hwin = NULL;
    free(r->kdwork); free(r->kdtree);
    r->kdwork = NULL; r->kdtree = NULL; r->kdsize = 0;
    free(r->ev_n); free(r->ev_pos); free(r->ev_pow); free(r->volR);
    r->ev_n = NULL; r->ev_pos = NULL; r->ev_pow = NULL; r->volR = NULL;
    r->vol_ready = 0;
}
void orc_destroy(orc_renderer* r) {
    if (!r) return;
    free(r->vcm_ctx);
    free_scene(r);
    free_frame(r);
    free(r);
}

/* Light ctors (renderer/Light.cpp:14-49) */
static light_t make_light(const orx_light* L) {
    light_t l;
    memset(&l, 0, sizeof l);
    l.type = L->type;
    l.power = ld3(L->power);
    l.position = ld3(L->position);
    if (L->type == ORX_LIGHT_AREA) {
        l.v1 = ld3(L->v1);
        l.v2 = ld3(L->v2);
        v3 c = cross(l.v1, l.v2);
        l.normal = normalize(c);
        l.area = length(c);
        l.inverseArea = 1.0f / l.area;
        l.Lemit = scl(scl(l.power, l.inverseArea), ORX_1_PI_F);
    } else if (L->type == ORX_LIGHT_POINT) {
        l.Lemit = scl(scl(l.power, 0.25f), ORX_1_PI_F); /* intensity */
    } else {
        /* SPOT: the ctor normalises its by-value parameter, not the member (Light.cpp:41) */
        l.direction = ld3(L->direction);
        l.normal = l.direction;
        l.angle = L->angle;
        float angleFactor = 1.0f / (1.0f - cosf(l.angle * 180 * ORX_1_PI_F));
        l.Lemit = scl(scl(scl(l.power, 0.25f), ORX_1_PI_F), angleFactor);
    }
    return l;
}

/* Vector3::length with the reference's dot bug a.z*b.x (math/Vector3.cpp:27-30) */
static float vector3_buggy_length(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.x); }

/* ---- triangle BVH (median split on the widest centroid axis) ---- */
typedef struct { float c; uint32_t i; } cent_t;
static int cent_cmp(const void* a, const void* b) {
    float x = ((const cent_t*)a)->c, y = ((const cent_t*)b)->c;
    if (x < y) return -1;
    if (x > y) return 1;
    uint32_t i = ((const cent_t*)a)->i, j = ((const cent_t*)b)->i;
    return i < j ? -1 : (i > j);
}
static uint32_t bvh_build(orc_renderer* r, const float* tlo, const float* thi, uint32_t first, uint32_t count,
                          cent_t* scratch) {
    uint32_t idx = r->bvh_n++;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t k = first; k < first + count; k++) {
        uint32_t t = r->bvh_prims[k];
        for (int a = 0; a < 3; a++) {
            float l = tlo[3 * t + a], h = thi[3 * t + a], c = 0.5f * (l + h);
            if (l < lo[a]) lo[a] = l;
            if (h > hi[a]) hi[a] = h;
            if (c < clo[a]) clo[a] = c;
            if (c > chi[a]) chi[a] = c;
        }
    }
    for (int a = 0; a < 3; a++) { /* conservative box */
        float m = fmaxf(fabsf(lo[a]), fabsf(hi[a]));
        float e = m * 2e-6f + 1e-20f;
        r->bvh_box[6 * idx + a] = lo[a] - e;
        r->bvh_box[6 * idx + 3 + a] = hi[a] + e;
    }
    if (count <= 4) {
        r->bvh_a[idx] = first;
        r->bvh_b[idx] = 0x80000000u | count;
        return idx;
    }
    int ax = 0;
    for (int a = 1; a < 3; a++)
        if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
    for (uint32_t k = 0; k < count; k++) {
        uint32_t t = r->bvh_prims[first + k];
        scratch[k].c = 0.5f * (tlo[3 * t + ax] + thi[3 * t + ax]);
        scratch[k].i = t;
    }
    qsort(scratch, count, sizeof(cent_t), cent_cmp);
    for (uint32_t k = 0; k < count; k++) r->bvh_prims[first + k] = scratch[k].i;
    uint32_t half = count / 2;
    uint32_t l = bvh_build(r, tlo, thi, first, half, scratch);
    uint32_t rr = bvh_build(r, tlo, thi, first + half, count - half, scratch);
    r->bvh_a[idx] = l;
    r->bvh_b[idx] = rr;
    return idx;
}
static void build_tri_bvh(orc_renderer* r) {
    uint32_t nt = r->nt;
    float* tlo = (float*)malloc(12 * (size_t)nt);
    float* thi = (float*)malloc(12 * (size_t)nt);
    for (uint32_t t = 0; t < nt; t++) {
        for (int a = 0; a < 3; a++) {
            float v0 = (&r->verts[r->tris[3 * t]].x)[a], v1 = (&r->verts[r->tris[3 * t + 1]].x)[a],
                  v2 = (&r->verts[r->tris[3 * t + 2]].x)[a];
            tlo[3 * t + a] = fminf(fminf(v0, v1), v2);
            thi[3 * t + a] = fmaxf(fmaxf(v0, v1), v2);
        }
    }
    size_t cap = 2 * (size_t)nt + 1;
    r->bvh_box = (float*)malloc(24 * cap);
    r->bvh_a = (uint32_t*)malloc(4 * cap);
    r->bvh_b = (uint32_t*)malloc(4 * cap);
    r->bvh_prims = (uint32_t*)malloc(4 * (size_t)nt);
    for (uint32_t t = 0; t < nt; t++) r->bvh_prims[t] = t;
    cent_t* scratch = (cent_t*)malloc(sizeof(cent_t) * nt);
    r->bvh_n = 0;
    bvh_build(r, tlo, thi, 0, nt, scratch);
    free(scratch);
    free(tlo);
    free(thi);
}

orx_status orc_init_scene(orc_renderer* r, const orx_scene* s) {
    if (!r || !s) return ORX_ERR_INVALID_ARGUMENT;
    if (s->n_lights == 0) return fail(r, ORX_ERR_NO_LIGHTS, "No lights exists in this scene.");
    for (uint32_t i = 0; i < s->n_textures; i++) {
        const orx_texture* t = &s->textures[i];
        if (!t->rgba || !t->width || !t->height || (t->normal_rgba && (!t->normal_width || !t->normal_height)))
            return fail(r, ORX_ERR_INVALID_ARGUMENT, "texture image without texels");
    }
    for (uint32_t i = 0; i < s->n_materials; i++)
        if (s->materials[i].type == ORX_MAT_TEXTURE &&
            (s->materials[i].texture < 0 || (uint32_t)s->materials[i].texture >= s->n_textures))
            return fail(r, ORX_ERR_INVALID_ARGUMENT, "Texture material without a texture image");
    const int med = r->cfg.enable_media && s->n_media;
    if (med) {
        if (s->n_media != 1 || !s->media)
            return fail(r, ORX_ERR_UNSUPPORTED, "participating media: one medium box per scene");
        const float* m = s->media;
        if (!(m[0] < m[3] && m[1] < m[4] && m[2] < m[5]) || !(m[6] >= 0 && m[7] >= 0 && m[6] + m[7] > 0))
            return fail(r, ORX_ERR_INVALID_ARGUMENT, "medium box: min < max and sigma_s + sigma_a > 0");
        if (r->cfg.volumetric_photons == 0)
            return fail(r, ORX_ERR_INVALID_ARGUMENT, "volumetric_photons must be > 0 with media");
    }
    free_scene(r);
    if (med) {
        r->med_lo = ld3(s->media);
        r->med_hi = ld3(s->media + 3);
        r->sig_s = s->media[6];
        r->sig_a = s->media[7];
        r->nvol = r->cfg.volumetric_photons;
        r->vpow = (v3*)calloc(r->nvol, sizeof(v3));
        r->vpos = (v3*)calloc(r->nvol, sizeof(v3));
        r->vcnt = (uint32_t*)calloc(r->nvol, 4);
        if (!r->vpow || !r->vpos || !r->vcnt) return fail(r, ORX_ERR_OUT_OF_MEMORY, "oracle: out of memory");
        r->med_on = 1;
    }
    r->nq = s->n_quads; r->ns = s->n_spheres; r->nt = s->n_triangles; r->nv = s->n_vertices;
    r->nm = s->n_materials; r->nl = s->n_lights;
    r->quads = (quadp_t*)calloc(r->nq + 1, sizeof(quadp_t));
    r->qmat = (uint32_t*)calloc(r->nq + 1, 4);
    for (uint32_t i = 0; i < r->nq; i++) {
        /* Cornell::createParallelogram (scene/Cornell.cpp:33-64) */
        v3 anchor = ld3(s->quads + 9 * i), o1 = ld3(s->quads + 9 * i + 3), o2 = ld3(s->quads + 9 * i + 6);
        v3 normal = normalize(cross(o1, o2));
        r->quads[i].n = normal;
        r->quads[i].d = dot(normal, anchor);
        r->quads[i].anchor = anchor;
        r->quads[i].v1 = divs(o1, dot(o1, o1));
        r->quads[i].v2 = divs(o2, dot(o2, o2));
        r->qmat[i] = s->quad_material[i];
    }
    r->sph = (sphere_t*)calloc(r->ns + 1, sizeof(sphere_t));
    r->smat = (uint32_t*)calloc(r->ns + 1, 4);
    for (uint32_t i = 0; i < r->ns; i++) {
        r->sph[i].c = ld3(s->spheres + 4 * i);
        r->sph[i].r = s->spheres[4 * i + 3];
        r->smat[i] = s->sphere_material[i];
    }
    r->verts = (v3*)calloc(r->nv + 1, sizeof(v3));
    r->vnorm = (v3*)calloc(r->nv + 1, sizeof(v3));
    r->has_normals = s->normals != NULL;
    for (uint32_t i = 0; i < r->nv; i++) {
        r->verts[i] = ld3(s->vertices + 3 * i);
        if (s->normals) r->vnorm[i] = ld3(s->normals + 3 * i);
    }
    if (s->texcoords) {
        r->uv = (float*)malloc(8 * (size_t)r->nv + 8);
        memcpy(r->uv, s->texcoords, 8 * (size_t)r->nv);
    }
    if (s->tangents && s->bitangents) { /* hasTangentsAndBitangents */
        r->tang = (v3*)calloc(r->nv + 1, sizeof(v3));
        r->btan = (v3*)calloc(r->nv + 1, sizeof(v3));
        for (uint32_t i = 0; i < r->nv; i++) {
            r->tang[i] = ld3(s->tangents + 3 * i);
            r->btan[i] = ld3(s->bitangents + 3 * i);
        }
    }
    r->ntex = s->n_textures;
    r->tex = (tex_t*)calloc(r->ntex + 1, sizeof(tex_t));
    for (uint32_t i = 0; i < r->ntex; i++) {
        const orx_texture* t = &s->textures[i];
        tex_t* d = &r->tex[i];
        d->w = t->width; d->h = t->height;
        d->rgba = (uint8_t*)malloc(4 * (size_t)d->w * d->h);
        memcpy(d->rgba, t->rgba, 4 * (size_t)d->w * d->h);
        if (t->normal_rgba) {
            d->nw = t->normal_width; d->nh = t->normal_height;
            d->nrgba = (uint8_t*)malloc(4 * (size_t)d->nw * d->nh);
            memcpy(d->nrgba, t->normal_rgba, 4 * (size_t)d->nw * d->nh);
        }
    }
    r->tris = (uint32_t*)calloc(3 * (size_t)r->nt + 3, 4);
    r->tmat = (uint32_t*)calloc(r->nt + 1, 4);
    if (r->nt) {
        memcpy(r->tris, s->triangles, 12 * (size_t)r->nt);
        memcpy(r->tmat, s->triangle_material, 4 * (size_t)r->nt);
    }
    if (r->nt) build_tri_bvh(r);
    r->mats = (mat_t*)calloc(r->nm + 1, sizeof(mat_t));
    for (uint32_t i = 0; i < r->nm; i++) {
        const orx_material* m = &s->materials[i];
        mat_t* d = &r->mats[i];
        d->type = m->type;
        d->Kd = ld3(m->Kd); d->Ks = ld3(m->Ks); d->Kr = ld3(m->Kr); d->Kt = ld3(m->Kt);
        d->ior = m->ior; d->exponent = m->exponent;
        d->tex = m->texture;
        if (m->type == ORX_MAT_TEXTURE) r->has_tex = 1;
        if (m->type == ORX_MAT_DIFFUSE_EMITTER) {
            /* DiffuseEmitter.cpp:17-25, :48-62 */
            v3 power = mul(ld3(m->power), d->Kd);
            d->inverseArea = m->inverse_area;
            d->powerPerArea = scl(power, m->inverse_area);
            d->Lemit = scl(scl(power, m->inverse_area), ORX_1_PI_F);
        }
        if (m->type == ORX_MAT_GLOSSY) {
            /* Glossy.cpp:16-30 energy clamp */
            v3 sumK = add(d->Kd, d->Ks);
            float sumScale = 1.f / maxf(maxf(sumK.x, sumK.y), sumK.z);
            if (sumScale < 1.f) { d->Kd = scl(d->Kd, sumScale); d->Ks = scl(d->Ks, sumScale); }
        }
    }
    r->lights = (light_t*)calloc(r->nl + 1, sizeof(light_t));
    for (uint32_t i = 0; i < r->nl; i++) r->lights[i] = make_light(&s->lights[i]);
    r->aabb_min = ld3(s->aabb_min);
    r->aabb_max = ld3(s->aabb_max);
    /* AAB::getBoundingSphere (math/AAB.cpp:26-33) */
    v3 center = scl(add(r->aabb_min, r->aabb_max), 0.5f);
    r->bs_center = center;
    r->bs_radius = vector3_buggy_length(sub(r->aabb_max, center));
    r->vcm_estimated = 0;
    r->scene_ready = 1;
    return ORX_OK;
}

/* ------------------------------------------------------------------ */
/* ray casting (geometry_instance: parallelogram, Sphere, TriangleMesh) */
/* ------------------------------------------------------------------ */
typedef struct {
    float t;
    int32_t prim; /* global id: quads, spheres, triangles */
    v3 gn, sn;    /* geometricNormal / shadingNormal attributes */
    float b, g;   /* triangle barycentrics (beta, gamma) */
} hit_t;

/* parallelogram.cu:49-76 */
static inline int isect_quad(const quadp_t* q, v3 o, v3 d, float tmin, float tmax, float* tout) {
    v3 n = q->n;
    float dt = dot(d, n);
    float t = (q->d - dot(n, o)) / dt;
    if (t > tmin && t < tmax) {
        v3 p = add(o, scl(d, t));
        v3 vi = sub(p, q->anchor);
        float a1 = dot(q->v1, vi);
        if (a1 >= 0 && a1 <= 1) {
            float a2 = dot(q->v2, vi);
            if (a2 >= 0 && a2 <= 1) { *tout = t; return 1; }
        }
    }
    return 0;
}
/* Sphere.cu:32-56 — returns the reported root, normal through *n */
static inline int isect_sphere(const sphere_t* s, v3 o, v3 d, float tmin, float tmax, float* tout, v3* nout) {
    v3 O = sub(o, s->c);
    float b = dot(O, d);
    float c = dot(O, O) - s->r * s->r;
    float disc = b * b - c;
    if (disc > 0.0f) {
        float sdisc = sqrtf(disc);
        float root1 = (-b - sdisc);
        if (root1 > tmin && root1 < tmax) {
            *tout = root1;
            *nout = divs(add(O, scl(d, root1)), s->r);
            return 1;
        }
        float root2 = (-b + sdisc);
        if (root2 > tmin && root2 < tmax) {
            *tout = root2;
            *nout = divs(add(O, scl(d, root2)), s->r);
            return 1;
        }
    }
    return 0;
}
/* OptiX intersect_triangle_branchless (optixu_math_namespace.h), TriangleMesh.cu:35-54 */
static inline int isect_tri(v3 p0, v3 p1, v3 p2, v3 o, v3 d, float tmin, float tmax, float* tout, v3* nout,
                            float* bout, float* gout) {
    v3 e0 = sub(p1, p0);
    v3 e1 = sub(p0, p2);
    v3 n = cross(e1, e0);
    v3 e2 = scl(sub(p0, o), 1.0f / dot(n, d));
    v3 i = cross(d, e2);
    float beta = dot(i, e1);
    float gamma = dot(i, e0);
    float t = dot(n, e2);
    if ((t < tmax) & (t > tmin) & (beta >= 0.0f) & (gamma >= 0.0f) & (beta + gamma <= 1)) {
        *tout = t; *nout = n; *bout = beta; *gout = gamma;
        return 1;
    }
    return 0;
}

static inline int bvh_box_hit(const float* bx, v3 o, v3 inv, float tmin, float tmax) {
    float tx0 = (bx[0] - o.x) * inv.x, tx1 = (bx[3] - o.x) * inv.x;
    float ty0 = (bx[1] - o.y) * inv.y, ty1 = (bx[4] - o.y) * inv.y;
    float tz0 = (bx[2] - o.z) * inv.z, tz1 = (bx[5] - o.z) * inv.z;
    float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    return t0 <= t1;
}

/* closest hit; equal t -> lowest primitive id (NoAccel child order, Cornell.cpp:183-189) */
static int trace_closest(const orc_renderer* r, v3 o, v3 d, float tmin, float tmax, hit_t* h) {
    float best = tmax;
    int32_t bp = -1;
    float t;
    for (uint32_t i = 0; i < r->nq; i++)
        if (isect_quad(&r->quads[i], o, d, tmin, best, &t)) { best = t; bp = (int32_t)i; }
    v3 sn_s = mk1(0);
    for (uint32_t i = 0; i < r->ns; i++) {
        v3 n;
        if (isect_sphere(&r->sph[i], o, d, tmin, best, &t, &n)) { best = t; bp = (int32_t)(r->nq + i); sn_s = n; }
    }
    float tb = 0, tg = 0;
    v3 tn = mk1(0);
    if (r->nt) {
        const uint32_t base = r->nq + r->ns;
        v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        uint32_t stack[64];
        int sp = 0;
        uint32_t node = 0;
        for (;;) {
            const float* bx = r->bvh_box + 6 * node;
            if (bvh_box_hit(bx, o, inv, tmin, best)) {
                if (r->bvh_b[node] & 0x80000000u) {
                    uint32_t first = r->bvh_a[node], cnt = r->bvh_b[node] & 0x7fffffffu;
                    for (uint32_t k = 0; k < cnt; k++) {
                        uint32_t i = r->bvh_prims[first + k];
                        const uint32_t* ix = r->tris + 3 * (size_t)i;
                        v3 n; float b, g;
                        /* closest t; equal t -> lower primitive id (brute-force order) */
                        float lim = bp >= 0 ? nextafterf(best, INFINITY) : best;
                        if (isect_tri(r->verts[ix[0]], r->verts[ix[1]], r->verts[ix[2]], o, d, tmin, lim, &t, &n, &b, &g) &&
                            (t < best || (int32_t)(base + i) < bp)) {
                            best = t; bp = (int32_t)(base + i); tn = n; tb = b; tg = g;
                        }
                    }
                } else {
                    stack[sp++] = r->bvh_b[node];
                    node = r->bvh_a[node];
                    continue;
                }
            }
            if (sp == 0) break;
            node = stack[--sp];
        }
    }
    if (bp < 0) return 0;
    h->t = best;
    h->prim = bp;
    h->b = tb;
    h->g = tg;
    if ((uint32_t)bp < r->nq) {
        h->gn = h->sn = r->quads[bp].n;
    } else if ((uint32_t)bp < r->nq + r->ns) {
        h->gn = h->sn = sn_s;
    } else {
        uint32_t ti = (uint32_t)bp - r->nq - r->ns;
        const uint32_t* ix = r->tris + 3 * (size_t)ti;
        if (r->has_normals) {
            v3 n0 = r->vnorm[ix[0]], n1 = r->vnorm[ix[1]], n2 = r->vnorm[ix[2]];
            h->sn = normalize(add(add(scl(n1, tb), scl(n2, tg)), scl(n0, 1.0f - tb - tg)));
        } else {
            h->sn = normalize(tn);
        }
        h->gn = normalize(tn);
    }
    return 1;
}
static uint32_t prim_material(const orc_renderer* r, int32_t p) {
    if ((uint32_t)p < r->nq) return r->qmat[p];
    if ((uint32_t)p < r->nq + r->ns) return r->smat[p - r->nq];
    return r->tmat[p - r->nq - r->ns];
}
/* Texture attributes (TriangleMesh.cu:61-84; quads and spheres write no
 * textureCoordinate/tangent attributes: (0,0) and no normal mapping here). */
static void hit_texcoord(const orc_renderer* r, const hit_t* h, float* u, float* v) {
    *u = 0.f; *v = 0.f;
    if ((uint32_t)h->prim < r->nq + r->ns || !r->uv) return;
    const uint32_t* ix = r->tris + 3 * (size_t)((uint32_t)h->prim - r->nq - r->ns);
    const float w0 = 1.0f - h->b - h->g;
    *u = (r->uv[2 * ix[1]] * h->b + r->uv[2 * ix[2]] * h->g) + r->uv[2 * ix[0]] * w0;
    *v = (r->uv[2 * ix[1] + 1] * h->b + r->uv[2 * ix[2] + 1] * h->g) + r->uv[2 * ix[0] + 1] * w0;
}
/* tex2D(diffuseSampler, textureCoordinate).xyz (Texture.cu:107-109) */
static v3 tex_color(const orc_renderer* r, const mat_t* m, const hit_t* h) {
    const tex_t* t = &r->tex[m->tex];
    float u, v, c[4];
    hit_texcoord(r, h, &u, &v);
    orx_tex2d_linear(t->rgba, t->w, t->h, u, v, c);
    return mk(c[0], c[1], c[2]);
}
/* the radiance program's normal: getNormalMappedNormal when hasNormals
 * (Texture.cu:69-77, :88-95).  The reference reads the tangent attributes only
 * a mesh with vertex normals and tangents sets (TriangleMesh.cu:56-70); other
 * primitives keep the shading normal here. */
static v3 tex_normal(const orc_renderer* r, const mat_t* m, const hit_t* h, v3 wsn) {
    const tex_t* t = &r->tex[m->tex];
    if (!t->nrgba || !r->has_normals || !r->tang || (uint32_t)h->prim < r->nq + r->ns) return wsn;
    const uint32_t* ix = r->tris + 3 * (size_t)((uint32_t)h->prim - r->nq - r->ns);
    const float w0 = 1.0f - h->b - h->g;
    v3 T = normalize(add(add(scl(r->tang[ix[1]], h->b), scl(r->tang[ix[2]], h->g)), scl(r->tang[ix[0]], w0)));
    v3 B = normalize(add(add(scl(r->btan[ix[1]], h->b), scl(r->btan[ix[2]], h->g)), scl(r->btan[ix[0]], w0)));
    T = normalize(T);
    B = normalize(B);
    float u, v, c[4];
    hit_texcoord(r, h, &u, &v);
    orx_tex2d_linear(t->nrgba, t->nw, t->nh, u, v, c);
    const float nx = 2.f * c[0] - 1.f, ny = 2.f * c[1] - 1.f, nz = 2.f * c[2] - 1.f;
    v3 N = mk(nx * T.x + ny * B.x + nz * wsn.x, nx * T.y + ny * B.y + nz * wsn.y, nx * T.z + ny * B.z + nz * wsn.z);
    return normalize(N);
}

/* shadow ray: any hit in (tmin, tmax) occludes (every material carries
 * gatherAnyHitOnNonEmitter for RayType::SHADOW, Material.cpp:18-26, which
 * DiffuseEmitter.cpp:33 installs last and so overrides gatherAnyHitOnEmitter) */
static int trace_any(const orc_renderer* r, v3 o, v3 d, float tmin, float tmax) {
    float t;
    for (uint32_t i = 0; i < r->nq; i++)
        if (isect_quad(&r->quads[i], o, d, tmin, tmax, &t)) return 1;
    for (uint32_t i = 0; i < r->ns; i++) {
        v3 n;
        if (isect_sphere(&r->sph[i], o, d, tmin, tmax, &t, &n)) return 1;
    }
    if (r->nt) {
        v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        uint32_t stack[64];
        int sp = 0;
        uint32_t node = 0;
        for (;;) {
            const float* bx = r->bvh_box + 6 * node;
            if (bvh_box_hit(bx, o, inv, tmin, tmax)) {
                if (r->bvh_b[node] & 0x80000000u) {
                    uint32_t first = r->bvh_a[node], cnt = r->bvh_b[node] & 0x7fffffffu;
                    for (uint32_t k = 0; k < cnt; k++) {
                        const uint32_t* ix = r->tris + 3 * (size_t)r->bvh_prims[first + k];
                        v3 n; float b, g;
                        if (isect_tri(r->verts[ix[0]], r->verts[ix[1]], r->verts[ix[2]], o, d, tmin, tmax, &t, &n, &b, &g))
                            return 1;
                    }
                } else {
                    stack[sp++] = r->bvh_b[node];
                    node = r->bvh_a[node];
                    continue;
                }
            }
            if (sp == 0) break;
            node = stack[--sp];
        }
    }
    return 0;
}

/* The medium box (geometry_instance/AAB.cu:24-157): slab test with the near and far axes; a ray
 * starting inside (tNear < 0.01, tFar > 0) reports t = 0.000115 on the far axis with the normal
 * against the ray for RADIANCE/PHOTON rays (so the medium program starts its walk right there),
 * and the exit t = tFar with the normal along the ray for the IN_PARTICIPATING_MEDIUM types. */
#define MED_PRIM 0x7ffffff0
static inline int isect_medium(const orc_renderer* r, v3 o, v3 d, float tmin, float tmax, int in_medium, float* tout,
                               v3* nout) {
    int axn = 0, axf = 0;
    float tn, tf;
    const float divx = 1 / d.x;
    if (divx >= 0) { tn = (r->med_lo.x - o.x) * divx; tf = (r->med_hi.x - o.x) * divx; }
    else { tn = (r->med_hi.x - o.x) * divx; tf = (r->med_lo.x - o.x) * divx; }
    if (tf < tn) return 0;
    const float divy = 1 / d.y;
    float tyn, tyf;
    if (divy >= 0) { tyn = (r->med_lo.y - o.y) * divy; tyf = (r->med_hi.y - o.y) * divy; }
    else { tyn = (r->med_hi.y - o.y) * divy; tyf = (r->med_lo.y - o.y) * divy; }
    if (tyn > tn) { tn = tyn; axn = 1; }
    if (tyf < tf) { tf = tyf; axf = 1; }
    if (tf < tn) return 0;
    const float divz = 1 / d.z;
    float tzn, tzf;
    if (divz >= 0) { tzn = (r->med_lo.z - o.z) * divz; tzf = (r->med_hi.z - o.z) * divz; }
    else { tzn = (r->med_hi.z - o.z) * divz; tzf = (r->med_lo.z - o.z) * divz; }
    if (tzn > tn) { tn = tzn; axn = 2; }
    if (tzf < tf) { tf = tzf; axf = 2; }
    if (tf < tn) return 0;
    float t = tn, nvr = -1;
    int ax = axn;
    if (tn < 0.01f && tf > 0.0f) {
        ax = axf;
        if (!in_medium) t = (float)0.000115;
        else { t = tf; nvr = 1; }
    }
    if (!(t > tmin && t < tmax)) return 0;
    const float dc = ax == 0 ? d.x : ax == 1 ? d.y : d.z;
    const float nc = dc >= 0 ? nvr : -nvr;
    *nout = mk(ax == 0 ? nc : 0.f, ax == 1 ? nc : 0.f, ax == 2 ? nc : 0.f);
    *tout = t;
    return 1;
}
/* closest hit with the medium as the last primitive (a surface at the same t wins) */
static int trace_closest_m(const orc_renderer* r, v3 o, v3 d, float tmin, float tmax, int in_medium, hit_t* h) {
    const int hit = trace_closest(r, o, d, tmin, tmax, h);
    if (!r->med_on) return hit;
    float t;
    v3 n;
    if (isect_medium(r, o, d, tmin, hit ? h->t : tmax, in_medium, &t, &n)) {
        h->t = t;
        h->prim = MED_PRIM;
        h->gn = h->sn = n;
        h->b = h->g = 0.f;
        return 1;
    }
    return hit;
}
/* VolumetricPhotonSphere.cu:24-59 + VolumetricPhotonSphereRadiance.cu:24-34 over the table in
 * slot order: each root of the photon's sphere inside (tmin, tmax) reports an intersection whose
 * any-hit adds the photon when its projection on the ray is inside (tmin, tmax) and then ignores
 * it, so a photon with both roots inside counts twice */
static v3 vol_gather(const orc_renderer* r, v3 o, v3 d, float tmin, float tmax, float sig_t) {
    v3 acc = mk1(0.f);
    if (!r->vol_ready) return acc;
    const float R = r->vol_R, R2 = R * R;
    const float coef = 1 / (ORX_PI_F * R * R), k4 = 1.f / (4.f * ORX_PI_F);
    for (uint32_t s = 0; s < r->nvol; s++) {
        if (!r->vcnt[s] || !(fmax3(r->vpow[s]) > 0)) continue;
        const v3 pos = r->vpos[s];
        const v3 O = sub(o, pos);
        const float b = dot(O, d), c = dot(O, O) - R2, disc = b * b - c;
        if (!(disc > 0.0f)) continue;
        const float sd = sqrtf(disc), r1 = -b - sd, r2 = -b + sd;
        const float t = dot(sub(pos, o), d);
        if (!(t < tmax && t > tmin)) continue;
        const v3 pw = scl(r->vpow[s], (float)r->vcnt[s]);
        const v3 add1 = scl(scl(scl(pw, coef), orx_expf(-sig_t * t)), k4);
        if (r1 > tmin && r1 < tmax) acc = add(acc, add1);
        if (r2 > tmin && r2 < tmax) acc = add(acc, add1);
    }
    return acc;
}

int32_t orc_trace_closest(orc_renderer* r, const float o[3], const float d[3], float tmin, float tmax, float* t_out) {
    hit_t h;
    if (!trace_closest(r, ld3(o), ld3(d), tmin, tmax, &h)) return -1;
    if (t_out) *t_out = h.t;
    return h.prim;
}
int32_t orc_trace_any(orc_renderer* r, const float o[3], const float d[3], float tmin, float tmax) {
    return trace_any(r, ld3(o), ld3(d), tmin, tmax);
}

/* ------------------------------------------------------------------ */
/* camera (renderer/Camera.cpp:333-345)                                */
/* ------------------------------------------------------------------ */
typedef struct { v3 eye, lookdir, u, v; float aperture, ulen, vlen; } cam_t;

static float dtor(float d) { return d * ((float)M_PI / 180.f); } /* Camera.cpp:87-90 */

static cam_t camera_setup(const orx_camera* c) {
    cam_t k;
    v3 eye = ld3(c->eye), lookat = ld3(c->lookat), up = ld3(c->up);
    k.eye = eye;
    k.lookdir = sub(lookat, eye);
    float lookdir_len = length(k.lookdir);
    up = normalize(up);
    v3 cu = normalize(cross(k.lookdir, up));
    v3 cv = normalize(cross(cu, k.lookdir));
    float ulen = lookdir_len * tanf(dtor(c->hfov * 0.5f));
    k.u = scl(cu, ulen);
    float vlen = lookdir_len * tanf(dtor(c->vfov * 0.5f));
    k.v = scl(cv, vlen);
    k.aperture = c->aperture;
    k.ulen = ulen; /* imagePlaneSize = 2 * (ulen, vlen), Camera.cpp:344 */
    k.vlen = vlen;
    return k;
}
void orc_tex2d(const uint8_t* rgba, uint32_t w, uint32_t h, float u, float v, float out[4]) {
    orx_tex2d_linear(rgba, w, h, u, v, out);
}
void orc_camera_setup(const orx_camera* cam, float lookdir[3], float u[3], float v[3]) {
    cam_t k = camera_setup(cam);
    lookdir[0] = k.lookdir.x; lookdir[1] = k.lookdir.y; lookdir[2] = k.lookdir.z;
    u[0] = k.u.x; u[1] = k.u.y; u[2] = k.u.z;
    v[0] = k.v.x; v[1] = k.v.y; v[2] = k.v.z;
}

/* RayGeneratorPPM.cu:40-48 / RayGeneratorPT.cu:53-61 + helpers/camera.h:11-27 */
static void primary_ray(const cam_t* cam, uint32_t x, uint32_t y, uint32_t W, uint32_t H, uint32_t* rs, v3* o, v3* d) {
    float sx = orc_uniform(rs);
    float sy = orc_uniform(rs);
    float dx = ((float)x + sx) / (float)W * 2.0f - 1.0f;
    float dy = ((float)y + sy) / (float)H * 2.0f - 1.0f;
    v3 origin = cam->eye;
    v3 dir = normalize(add(add(scl(cam->u, dx), scl(cam->v, dy)), cam->lookdir));
    if (cam->aperture > 0) {
        v3 focal = add(cam->eye, cam->lookdir);
        v3 camLookDir = normalize(cam->lookdir);
        float focalPlaneT = (dot(camLookDir, focal) - dot(camLookDir, cam->eye)) / dot(camLookDir, dir);
        v3 lookAt = add(origin, scl(dir, focalPlaneT));
        float ux = orc_uniform(rs);
        float uy = orc_uniform(rs);
        float rr = sqrtf(ux);
        float th = 2.f * ORX_PI_F * uy;
        float discx = rr * orx_cosf(th);
        float discy = rr * orx_sinf(th);
        origin = add(origin, add(scl(scl(cam->u, discx), cam->aperture), scl(scl(cam->v, discy), cam->aperture)));
        dir = normalize(sub(lookAt, origin));
    }
    *o = origin;
    *d = dir;
}

/* ------------------------------------------------------------------ */
/* radiance rays: RadiancePRD + material closest-hit programs          */
/* ------------------------------------------------------------------ */
typedef struct {
    v3 attenuation, radiance;
    uint32_t depth;
    v3 position, normal;
    uint32_t flags;
    v3 newdir; /* randomNewDirection / Le union */
    uint32_t* rs;
} rprd_t;

/* Iterative form of the recursive rtTrace(RADIANCE) chain: Mirror/Glass
 * closest-hit programs tail-recurse (Mirror.cu:50-63, Glass.cu:90-143).
 *
 * With a medium (volR != NULL): ParticipatingMedium.cu:53-104.  A RADIANCE ray that enters the
 * box opens a frame: attenSaved = (attenuation + 0.1f) - 0.1f, then the rest of the path runs on
 * an IN_PARTICIPATING_MEDIUM ray from the entry point (tmin 0.01); when it returns, the frame's
 * distance is the radiancePrd.lastTHit left by that ray's first hit (every closest-hit program
 * writes its own tHit after its recursion; a miss and a back-facing emitter write nothing, so the
 * value is the PRD's initial one, 0 here; the medium program's own write goes through double,
 * tHit + 0.1 - 0.1), T = exp(-distance sigma_t), V = the volumetric gather on (entry, tmin 1e-7,
 * tmax distance), and volumetricRadiance = volumetricRadiance*T + attenSaved*V,
 * attenuation *= T.  Frames nest along the path; unrolled, the path's
 *   volumetricRadiance = sum_k attenSaved_k V_k prod_{j<k} T_j,  attenuation = (...) prod_k T_k,
 * accumulated here in path order (the nested evaluation's fp32 rounding order differs).  A ray
 * hitting the box from inside (leaving it) continues as RADIANCE from the exit point (tmin 0.01).
 * Glass rays travelling inside the glass are IN_PARTICIPATING_MEDIUM rays (Glass.cu:126-131). */
static void trace_radiance(const orc_renderer* r, v3 o, v3 d, float tmin, rprd_t* prd, v3* volR) {
    const uint32_t maxd = r->cfg.max_radiance_trace_depth;
    const int med = r->med_on && volR;
    const float sig_t = r->sig_a + r->sig_s;
    int inmed = 0, frame = 0;
    v3 fa = mk1(0.f), fh = mk1(0.f), fd = mk1(0.f);
    float P = 1.f;
    for (;;) {
        hit_t h;
        const int hit = med ? trace_closest_m(r, o, d, tmin, ORC_RT_DEFAULT_MAX, inmed, &h)
                            : trace_closest(r, o, d, tmin, ORC_RT_DEFAULT_MAX, &h);
        if (frame) { /* the open frame's inner ray has its first hit: close the frame */
            frame = 0;
            float dist = 0.f;
            if (hit) {
                if (h.prim == MED_PRIM) {
                    dist = (float)(((double)h.t + 0.1) - 0.1);
                } else {
                    const mat_t* fm = &r->mats[prim_material(r, h.prim)];
                    if (fm->type != ORX_MAT_DIFFUSE_EMITTER || !(dot(normalize(h.sn), neg(d)) < 0.f)) dist = h.t;
                }
            }
            const float T = orx_expf(-dist * sig_t);
            const v3 V = vol_gather(r, fh, fd, (float)0.0000001, dist, sig_t);
            *volR = add(*volR, scl(mul(fa, V), P));
            P = P * T;
        }
        if (!hit) {
            /* miss (RayGeneratorPPM.cu:72-77, RayGeneratorPT.cu:144-150) */
            prd->flags = PRD_MISS;
            prd->attenuation = mk1(0.f);
            prd->radiance = mk1(0.f);
            break;
        }
        v3 hitPoint = add(o, scl(d, h.t));
        if (h.prim == MED_PRIM) {
            const v3 N = normalize(h.sn);
            if (dot(N, d) < 0) { /* entering: open a frame */
                frame = 1;
                fa = sub_s(add(prd->attenuation, mk1(0.1f)), 0.1f);
                fh = hitPoint;
                fd = d;
                inmed = 1;
            } else {
                inmed = 0;
            }
            o = hitPoint;
            tmin = 0.01f;
            continue;
        }
        const mat_t* m = &r->mats[prim_material(r, h.prim)];
        if (m->type == ORX_MAT_DIFFUSE || m->type == ORX_MAT_GLOSSY) {
            /* Diffuse.cu:71-87, Glossy.cu:74-90 */
            v3 N = normalize(h.sn);
            prd->flags |= PRD_HIT_NON_SPECULAR;
            prd->attenuation = mul(prd->attenuation, m->Kd);
            prd->normal = N;
            prd->position = hitPoint;
            prd->depth++;
            if (prd->flags & PRD_PATH_TRACING) {
                float s0 = orc_uniform(prd->rs);
                float s1 = orc_uniform(prd->rs);
                prd->newdir = sample_hemisphere_cos(N, s0, s1);
            }
            break;
        } else if (m->type == ORX_MAT_TEXTURE) {
            /* Texture.cu:83-110: normal-mapped normal, no depth++ */
            v3 wsn = normalize(h.sn);
            prd->flags |= PRD_HIT_NON_SPECULAR;
            prd->normal = tex_normal(r, m, &h, wsn);
            prd->position = hitPoint;
            if (prd->flags & PRD_PATH_TRACING) {
                float s0 = orc_uniform(prd->rs);
                float s1 = orc_uniform(prd->rs);
                prd->newdir = sample_hemisphere_cos(wsn, s0, s1);
            }
            prd->attenuation = mul(prd->attenuation, tex_color(r, m, &h));
            break;
        } else if (m->type == ORX_MAT_DIFFUSE_EMITTER) {
            /* DiffuseEmitter.cu:40-51 */
            v3 N = normalize(h.sn);
            prd->flags |= PRD_HIT_EMITTER;
            if (dot(N, neg(d)) < 0.f) break;
            v3 Le = divs(m->powerPerArea, ORX_PI_F);
            prd->radiance = add(prd->radiance, mul(prd->attenuation, Le));
            break;
        } else if (m->type == ORX_MAT_MIRROR) {
            /* Mirror.cu:50-63 */
            v3 N = normalize(h.sn);
            prd->depth++;
            if (prd->depth <= maxd) {
                prd->attenuation = mul(prd->attenuation, m->Kr);
                d = reflect(d, N);
                o = hitPoint;
                tmin = 0.0001f;
                inmed = 0;
                continue;
            }
            break;
        } else { /* ORX_MAT_GLASS, Glass.cu:90-143 */
            v3 wsn = normalize(h.sn);
            int outside = dot(wsn, d) < 0;
            v3 N = outside ? wsn : neg(wsn);
            float n1 = outside ? 1.0f : m->ior, n2 = outside ? m->ior : 1.0f;
            v3 refr;
            int valid = refract(&refr, d, N, n2 / n1);
            float cosI = -dot(d, N);
            float cosT = -dot(refr, N);
            float refl = 1.f;
            if (valid) {
                float rp = (n2 * cosI - n1 * cosT) / (n2 * cosI + n1 * cosT);
                float rsv = (n1 * cosI - n2 * cosT) / (n1 * cosI + n2 * cosT);
                refl = (rp * rp + rsv * rsv) / 2.f;
            }
            float sample = orc_uniform(prd->rs);
            int isReflected = sample <= refl;
            v3 nd;
            if (isReflected) nd = reflect(d, N);
            else {
                nd = refr;
                prd->attenuation = scl(prd->attenuation, (n2 * n2) / (n1 * n1));
            }
            prd->flags |= PRD_HIT_SPECULAR;
            prd->flags &= ~PRD_HIT_NON_SPECULAR;
            prd->depth++;
            if (prd->depth <= maxd) {
                o = hitPoint; d = nd; tmin = 0.0001f;
                inmed = (outside && !isReflected) || (!outside && isReflected);
                continue;
            }
            prd->attenuation = scl(prd->attenuation, 0.f);
            break;
        }
    }
    if (med) prd->attenuation = scl(prd->attenuation, P);
}

/* ------------------------------------------------------------------ */
/* frame buffers                                                       */
/* ------------------------------------------------------------------ */
static uint32_t orc_pow2roundup(uint32_t x);
static orx_status resize(orc_renderer* r, uint32_t W, uint32_t H) {
    free_frame(r);
    const uint32_t PW = r->cfg.photon_launch_width, PH = r->cfg.photon_launch_height;
    r->W = W; r->H = H;
    r->RW = PW > W ? PW : W;
    r->RH = PH > H ? PH : H;
    r->rows = H > r->rank ? (H - r->rank + r->world - 1) / r->world : 0;
    r->max_rows = (H + r->world - 1) / r->world;
    r->prows = PH > r->rank ? (PH - r->rank + r->world - 1) / r->world : 0;
    size_t npx = (size_t)r->max_rows * W;
    const int hash = r->cfg.photon_map == 1;
    /* stochastic hash: store_photon.h never counts deposits, so a path deposits at every
     * non-specular hit at depth 1..max depth - 1 */
    r->dslot = hash ? (r->cfg.max_photon_trace_depth < 8 ? r->cfg.max_photon_trace_depth : 8) : r->cfg.max_photon_deposits;
    size_t S = (size_t)PW * r->prows * r->dslot;
    if (hash) {
        r->hnum = (size_t)PW * PH * r->cfg.max_photon_deposits; /* NUM_PHOTONS (OptixRenderer.cpp:50) */
        r->ndep = (uint8_t*)calloc((size_t)PW * r->prows + 1, 1);
        r->hcount = (uint32_t*)calloc(r->hnum, 4);
        r->hwin = (uint32_t*)calloc(r->hnum, 4);
        if (!r->ndep || !r->hcount || !r->hwin) return fail(r, ORX_ERR_OUT_OF_MEMORY, "oracle: out of memory");
    }
    if (r->cfg.photon_map == 2) {
        /* m_photonKdTreeSize = pow2roundup(NUM_PHOTONS + 1) - 1 (OptixRenderer.cpp:65-74, :207) */
        r->kdsize = (size_t)orc_pow2roundup((uint32_t)S + 1u) - 1u;
        r->kdwork = (kdphoton_t*)calloc(S + 1, sizeof(kdphoton_t));
        r->kdtree = (kdphoton_t*)calloc(r->kdsize + 1, sizeof(kdphoton_t));
        if (!r->kdwork || !r->kdtree) return fail(r, ORX_ERR_OUT_OF_MEMORY, "oracle: out of memory");
    }
    size_t G = r->cfg.photon_grid_max_size;
    r->rng = (uint32_t*)malloc((size_t)r->RW * r->RH * 6 * 4);
    r->hp = (hitpoint_t*)calloc(npx, sizeof(hitpoint_t));
    r->photons = (photon_t*)calloc(S, sizeof(photon_t));
    r->sort_tmp = (photon_t*)calloc(S, sizeof(photon_t));
    r->keys = (uint32_t*)calloc(S, 4);
    r->offsets = (uint32_t*)calloc(G + 2, 4);
    r->hist = (uint32_t*)calloc(G + 3, 4);
    r->indirect = (v3*)calloc(npx, sizeof(v3));
    r->direct = (v3*)calloc(npx, sizeof(v3));
    r->output = (v3*)calloc(npx, sizeof(v3));
    r->dbg = (uint32_t*)calloc(npx * 2, 4);
    if (r->med_on) {
        const size_t np = (size_t)PW * r->prows + 1;
        r->ev_n = (uint32_t*)calloc(np, 4);
        r->ev_pos = (v3*)calloc(np, sizeof(v3));
        r->ev_pow = (v3*)calloc(np, sizeof(v3));
        r->volR = (v3*)calloc(npx + 1, sizeof(v3));
        if (!r->ev_n || !r->ev_pos || !r->ev_pow || !r->volR) return fail(r, ORX_ERR_OUT_OF_MEMORY, "oracle: out of memory");
    }
    if (!r->rng || !r->hp || !r->photons || !r->sort_tmp || !r->keys || !r->offsets || !r->hist ||
        !r->indirect || !r->direct || !r->output || !r->dbg)
        return fail(r, ORX_ERR_OUT_OF_MEMORY, "oracle: out of memory");
    /* initializeRandomStates (OptixRenderer_SpatialHash.cu:310-347) */
    uint32_t seed = r->cfg.seed;
    if (seed == 0) seed = 574133u * (uint32_t)clock() + (uint32_t)(47844152748ull * (uint32_t)time(NULL));
    size_t n = (size_t)r->RW * r->RH;
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)n; i++) orc_xorwow_init((uint64_t)(uint32_t)(seed + (uint32_t)i), r->rng + 6 * i);
    r->rng_ready = 1;
    return ORX_OK;
}

/* ------------------------------------------------------------------ */
/* PPM passes                                                          */
/* ------------------------------------------------------------------ */
/* RayGeneratorPPM.cu:31-66 */
static void ppm_eye_pass(orc_renderer* r, const cam_t* cam) {
    const uint32_t W = r->W, H = r->H;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long j = 0; j < (long long)r->rows; j++) {
        const uint32_t y = r->rank + r->world * (uint32_t)j;
        for (uint32_t x = 0; x < W; x++) {
            uint32_t rs[6];
            uint32_t* g = r->rng + 6 * ((size_t)y * r->RW + x);
            memcpy(rs, g, 24);
            rprd_t prd;
            memset(&prd, 0, sizeof prd);
            prd.attenuation = mk1(1.0f);
            prd.rs = rs;
            v3 o, d;
            primary_ray(cam, x, y, W, H, rs, &o, &d);
            v3 vr = mk1(0.f); /* RayGeneratorPPM.cu:39-41 */
            trace_radiance(r, o, d, 0.001f, &prd, r->med_on ? &vr : NULL);
            if (r->med_on) r->volR[(size_t)j * W + x] = vr;
            hitpoint_t* h = &r->hp[(size_t)j * W + x];
            h->position = prd.position;
            h->normal = prd.normal;
            h->attenuation = prd.attenuation;
            h->radiance = prd.radiance;
            h->flags = prd.flags;
            memcpy(g, rs, 24);
        }
    }
}

/* Photon closest-hit chain (Diffuse.cu:92-135, Mirror.cu:65-77, Glass.cu:164-205,
 * DiffuseEmitter.cu:56-59) in iterative form.
 *
 * With a medium (ev != NULL): ParticipatingMedium.cu:110-201.  Every medium hit counts a depth.
 * An IN_PARTICIPATING_MEDIUM ray leaving the box continues as PHOTON from hit + 0.0001 d (tmin
 * 0.001); any other medium hit samples scatterT = -log(1 - u)/sigma_t and probes [0.001, scatterT]
 * with an IN_PARTICIPATING_MEDIUM ray.  The probe's frame scatters when the photon depth came
 * back unchanged: the probe met nothing (miss), an emitter (no program for that ray type), or a
 * diffuse/texture surface whose Russian roulette ended the path after its deposit (the scatter
 * position then lies beyond that surface, as in the reference).  A scatter survives with
 * probability sigma_s/sigma_t, is recorded as this photon's latest volumetric event and, below
 * the depth limit, continues as PHOTON in a uniform direction from the scatter position (tmin
 * 0.001).  Glass rays travelling inside the glass are IN_PARTICIPATING_MEDIUM rays. */
typedef struct { uint32_t n; v3 pos, pow; } vev_t;
static void trace_photon(const orc_renderer* r, v3 o, v3 d, v3 power, uint32_t pm_index, uint32_t* rs,
                         uint8_t* ndep, vev_t* ev) {
    /* uniform grid: at most maxDeposits, then the path ends (Diffuse.cu:97, :128-131); stochastic
     * hash: STORE_PHOTON never counts (store_photon.h:19-25), every hit at depth >= 1 deposits */
    const int hash = r->cfg.photon_map == 1;
    const uint32_t maxDeposits = hash ? r->dslot : r->cfg.max_photon_deposits;
    const uint32_t depositLimit = hash ? 0xffffffffu : maxDeposits;
    const uint32_t maxDepth = r->cfg.max_photon_trace_depth;
    const int med = r->med_on && ev;
    const float sig_t = r->sig_a + r->sig_s;
    uint32_t numStored = 0, depth = 0;
    float weight = 1.0f;
    float tmin = 0.0001f, tmax = ORC_RT_DEFAULT_MAX;
    int inmed = 0, probe = 0;
    uint32_t pdepth = 0;
    v3 spos = mk1(0.f);
    for (;;) {
        hit_t h;
        const int had_probe = probe;
        probe = 0;
        int end = 0;
        const int hit = med ? trace_closest_m(r, o, d, tmin, tmax, inmed, &h)
                            : trace_closest(r, o, d, tmin, ORC_RT_DEFAULT_MAX, &h);
        if (!hit) {
            end = 1; /* PhotonGenerator.cu:132-135 */
        } else if (h.prim == MED_PRIM) {
            depth++;
            const v3 N = normalize(h.sn);
            const v3 hitPoint = add(o, scl(d, h.t));
            if (dot(N, d) > 0 && inmed) { /* leaving the box */
                o = add(hitPoint, scl(d, 0.0001f));
                tmin = 0.001f;
                tmax = ORC_RT_DEFAULT_MAX;
                inmed = 0;
            } else {
                const float sample = orc_uniform(rs);
                const float st = -orx_logf(1 - sample) / sig_t;
                spos = add(hitPoint, scl(d, st));
                probe = 1;
                pdepth = depth;
                o = hitPoint;
                tmin = 0.001f;
                tmax = st;
                inmed = 1;
            }
        } else {
            const mat_t* m = &r->mats[prim_material(r, h.prim)];
            v3 hitPoint = add(o, scl(d, h.t));
            tmax = ORC_RT_DEFAULT_MAX;
            if (m->type == ORX_MAT_DIFFUSE || m->type == ORX_MAT_GLOSSY || m->type == ORX_MAT_TEXTURE) {
                /* Texture.cu:116-175 differs only in Kd = texel colour, the weight cutoff (0.01)
                 * and the new ray's tmin (0.01) */
                const int tex = m->type == ORX_MAT_TEXTURE;
                v3 N = normalize(h.sn);
                if (depth >= 1 && numStored < maxDeposits) {
                    photon_t* p = &r->photons[pm_index + numStored];
                    p->power = power;
                    p->position = hitPoint;
                    p->direction = d;
                    numStored++;
                    if (ndep) *ndep = (uint8_t)numStored;
                }
                const v3 kd = tex ? tex_color(r, m, &h) : m->Kd;
                power = mul(power, kd);
                weight *= fmax3(kd);
                if (depth >= 3) { /* PHOTON_TRACING_RR_START_DEPTH */
                    float probContinue = favgf(kd);
                    float probSample = orc_uniform(rs);
                    if (probSample >= probContinue) end = 1;
                    else power = divs(power, probContinue);
                }
                if (!end) {
                    depth++;
                    if (depth >= maxDepth || (double)weight < (tex ? 0.01 : 0.001)) end = 1;
                    else if (numStored >= depositLimit) end = 1;
                    else {
                        float s0 = orc_uniform(rs);
                        float s1 = orc_uniform(rs);
                        d = sample_hemisphere_cos(N, s0, s1);
                        o = hitPoint;
                        tmin = tex ? 0.01f : 0.0001f;
                        inmed = 0;
                    }
                }
            } else if (m->type == ORX_MAT_DIFFUSE_EMITTER) {
                if (!inmed) depth++; /* closestHitPhoton is the PHOTON program only */
                end = 1;
            } else if (m->type == ORX_MAT_MIRROR) {
                v3 N = normalize(h.sn);
                depth++;
                if (depth <= maxDepth) {
                    power = mul(power, m->Kr);
                    d = reflect(d, N);
                    o = hitPoint;
                    tmin = 0.0001f;
                    inmed = 0;
                } else {
                    end = 1;
                }
            } else { /* glass */
                v3 wsn = normalize(h.sn);
                int outside = dot(wsn, d) < 0;
                v3 N = outside ? wsn : neg(wsn);
                float n1 = outside ? 1.0f : m->ior, n2 = outside ? m->ior : 1.0f;
                v3 refr;
                int valid = refract(&refr, d, N, n2 / n1);
                float cosI = -dot(d, N);
                float cosT = -dot(refr, N);
                float refl = 1.f;
                if (valid) {
                    float rp = (n2 * cosI - n1 * cosT) / (n2 * cosI + n1 * cosT);
                    float rsv = (n1 * cosI - n2 * cosT) / (n1 * cosI + n2 * cosT);
                    refl = (rp * rp + rsv * rsv) / 2.f;
                }
                float sample = orc_uniform(rs);
                const int isReflected = sample <= refl;
                v3 nd = isReflected ? reflect(d, N) : refr;
                depth++;
                if (depth <= maxDepth) {
                    o = hitPoint; d = nd; tmin = 0.0001f;
                    inmed = (outside && !isReflected) || (!outside && isReflected);
                } else {
                    end = 1;
                }
            }
        }
        if (had_probe && depth == pdepth) { /* scatter at the probe's end */
            if (orc_uniform(rs) >= r->sig_s / sig_t) return;
            ev->n++;
            ev->pos = spos;
            ev->pow = power;
            if (depth >= maxDepth) return;
            const float s0 = orc_uniform(rs), s1 = orc_uniform(rs);
            d = sample_unit_sphere(s0, s1);
            o = spos;
            tmin = 0.001f;
            tmax = ORC_RT_DEFAULT_MAX;
            inmed = 0;
            continue;
        }
        if (end) return;
    }
}

/* PhotonGenerator.cu:40-79 + :81-128 */
static void ppm_photon_pass(orc_renderer* r) {
    const uint32_t PW = r->cfg.photon_launch_width, PH = r->cfg.photon_launch_height;
    const uint32_t maxDeposits = r->dslot;
    const uint32_t nl = r->nl;
    (void)PH;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long j = 0; j < (long long)r->prows; j++) {
        const uint32_t y = r->rank + r->world * (uint32_t)j;
        for (uint32_t x = 0; x < PW; x++) {
            uint32_t pm_index = ((uint32_t)j * PW + x) * maxDeposits;
            uint32_t* g = r->rng + 6 * ((size_t)y * r->RW + x);
            uint32_t rs[6];
            memcpy(rs, g, 24);
            int lightIndex = 0;
            if (nl > 1) {
                float sample = orc_uniform(rs);
                int li = (int)(sample * nl);
                lightIndex = li < (int)(nl - 1) ? li : (int)(nl - 1);
            }
            const light_t* L = &r->lights[lightIndex];
            float powerScale = (float)nl;
            v3 power = scl(L->power, powerScale);
            v3 origin = L->position, dir = mk1(0);
            float photonPowerFactor = 1.f;
            float s1x = orc_uniform(rs), s1y = orc_uniform(rs);
            if (L->type == ORX_LIGHT_AREA) {
                float s2x = orc_uniform(rs), s2y = orc_uniform(rs);
                origin = add(origin, add(scl(L->v1, s1x), scl(L->v2, s1y)));
                dir = sample_hemisphere(L->normal, s2x, s2y);
            } else if (L->type == ORX_LIGHT_POINT) {
                v3 sceneCenterToLight = sub(L->position, r->bs_center);
                float lightDistance = length(sceneCenterToLight);
                sceneCenterToLight = divs(sceneCenterToLight, lightDistance);
                int wellOutside = (double)lightDistance > 1.5 * (double)r->bs_radius;
                if (wellOutside) {
                    v3 pointOnDisc = sample_disc(s1x, s1y, r->bs_center, r->bs_radius, sceneCenterToLight);
                    dir = normalize(sub(pointOnDisc, origin));
                    float rr = r->bs_radius * r->bs_radius + lightDistance * lightDistance;
                    photonPowerFactor = (1 - lightDistance * (1.0f / sqrtf(rr))) / 2.f;
                } else {
                    dir = sample_unit_sphere(s1x, s1y);
                }
            } else { /* SPOT */
                v3 pointOnDisc = sample_disc(s1x, s1y, add(origin, L->direction), orx_sinf(L->angle / 2), L->direction);
                dir = normalize(sub(pointOnDisc, origin));
            }
            power = scl(power, photonPowerFactor);
            for (uint32_t i = 0; i < maxDeposits; i++) {
                r->photons[pm_index + i].position = mk1(0.0f);
                r->photons[pm_index + i].power = mk1(0.0f);
            }
            uint8_t* nd = r->ndep ? &r->ndep[(size_t)j * PW + x] : NULL;
            if (nd) *nd = 0;
            vev_t ev = {0, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
            trace_photon(r, origin, dir, power, pm_index, rs, nd, r->med_on ? &ev : NULL);
            if (r->med_on) {
                const size_t pi = (size_t)j * PW + x;
                r->ev_n[pi] = ev.n;
                r->ev_pos[pi] = ev.pos;
                r->ev_pow[pi] = ev.pow;
            }
            memcpy(g, rs, 24);
        }
    }
}

/* The volumetric photon table of this photon pass (VolumetricPhotonInitialize.cu:19-24 clears it,
 * ParticipatingMedium.cu:170-177 stores): photon p's scatter events all land in slot
 * pm_index % NUM_VOLUMETRIC_PHOTONS (pm_index = p * maxPhotonDepositsPerEmitted) and bump its
 * numDeposits; the reference's racing stores leave an arbitrary event's power and position in
 * the slot, here the last event of the highest photon index (the device's atomicMax).  The
 * table and this iteration's radius (volumetricRadius = PPMRadius, OptixRenderer.cpp:592-593)
 * serve the next eye pass. */
static void vol_resolve(orc_renderer* r, float ppmRadius) {
    memset(r->vcnt, 0, (size_t)r->nvol * 4);
    memset(r->vpow, 0, (size_t)r->nvol * sizeof(v3));
    memset(r->vpos, 0, (size_t)r->nvol * sizeof(v3));
    const size_t np = (size_t)r->cfg.photon_launch_width * r->prows;
    for (size_t p = 0; p < np; p++) {
        if (!r->ev_n[p]) continue;
        const uint32_t slot = (uint32_t)((uint32_t)p * r->dslot) % r->nvol;
        r->vcnt[slot] += r->ev_n[p];
        r->vpow[slot] = r->ev_pow[p];
        r->vpos[slot] = r->ev_pos[p];
    }
    r->vol_R = ppmRadius;
    r->vol_ready = 1;
}

/* OptixRenderer_SpatialHash.cu:62-71 (host code: glibc-free detmath pow) */
static float smallest_possible_cell_size(v3 ext, uint32_t maxGridSize) {
    float sceneVolume = ext.x * ext.y * ext.z;
    float minVolumePerCell = sceneVolume / (float)maxGridSize;
    float radiusC = orx_powf(minVolumePerCell, 1.0f / 3.0f);
    v3 numCellsF = divs(ext, radiusC);
    uint32_t nx = orx_f2u_sat(orx_floorf(numCellsF.x));
    uint32_t ny = orx_f2u_sat(orx_floorf(numCellsF.y));
    uint32_t nz = orx_f2u_sat(orx_floorf(numCellsF.z));
    v3 each = mk(ext.x / (float)nx, ext.y / (float)ny, ext.z / (float)nz);
    return fmax3(each);
}

/* createUniformGridPhotonMap (OptixRenderer_SpatialHash.cu:209-282) */
static orx_status ppm_build_grid_n(orc_renderer* r, size_t S, const uint32_t* box);
static orx_status ppm_build_grid(orc_renderer* r) {
    return ppm_build_grid_n(r, (size_t)r->cfg.photon_launch_width * r->prows * r->cfg.max_photon_deposits, NULL);
}
/* order-preserving float <-> uint32 (the slab mode's AABB words, include/orx.h) */
static inline uint32_t f2ord(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
static inline float ord2f(uint32_t u) {
    uint32_t v = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    float f;
    memcpy(&f, &v, 4);
    return f;
}
/* AABB of the valid photons among the first S entries, as ordered words (empty: ~0, 0) */
static void photon_box_words(const photon_t* ph, size_t S, uint32_t w[6]) {
    w[0] = w[1] = w[2] = 0xffffffffu;
    w[3] = w[4] = w[5] = 0u;
    for (size_t i = 0; i < S; i++) {
        if (!(fmax3(ph[i].power) > 0)) continue;
        const float c[3] = {ph[i].position.x, ph[i].position.y, ph[i].position.z};
        for (int k = 0; k < 3; k++) {
            const uint32_t o = f2ord(c[k]);
            if (o < w[k]) w[k] = o;
            if (o > w[k + 3]) w[k + 3] = o;
        }
    }
}
/* over the first S entries of r->photons; box: the grid bounds as ordered words (slab mode: all
 * ranks' photons), NULL: the AABB of these photons */
static orx_status ppm_build_grid_n(orc_renderer* r, size_t S, const uint32_t* box) {
    photon_t* ph = r->photons;
    /* getPhotonsBoundingBox: transform_reduce over valid photons (:123-128) */
    uint32_t w[6];
    if (box) memcpy(w, box, sizeof w);
    else photon_box_words(ph, S, w);
    const int any = w[0] != 0xffffffffu;
    v3 lo = any ? mk(ord2f(w[0]), ord2f(w[1]), ord2f(w[2])) : mk1(0);
    v3 hi = any ? mk(ord2f(w[3]), ord2f(w[4]), ord2f(w[5])) : mk1(0);
    /* padAABB (:135-141) */
    lo = sub_s(lo, 0.0000001f);
    hi = mk(hi.x + 0.0000001f, hi.y + 0.0000001f, hi.z + 0.0000001f);
    v3 ext = sub(hi, lo);
    float smallest = smallest_possible_cell_size(ext, r->cfg.photon_grid_max_size);
    float cellSize = (float)((double)smallest + 0.001);
    /* calculateGridSize (:42-50) */
    v3 f = divs(ext, cellSize);
    uint32_t g[3] = {orx_f2u_sat(orx_ceilf(f.x)), orx_f2u_sat(orx_ceilf(f.y)), orx_f2u_sat(orx_ceilf(f.z))};
    for (int k = 0; k < 3; k++) if (g[k] < 1) g[k] = 1;
    uint64_t G64 = (uint64_t)g[0] * g[1] * g[2];
    if (G64 > r->cfg.photon_grid_max_size)
        return fail(r, ORX_ERR_GRID_TOO_LARGE, "Too many cells in SpatialHash.cu, over defined PHOTON_GRID_MAX_SIZE.");
    uint32_t G = (uint32_t)G64;
    r->gsize[0] = g[0]; r->gsize[1] = g[1]; r->gsize[2] = g[2];
    r->cell = cellSize; r->origo = lo; r->ncells = G;
    const uint32_t invalid = G + 1;
    memset(r->hist, 0, (size_t)(G + 2) * 4);
    const float inv = 1.f / cellSize;
    /* calculateHashCellsKernel (:152-173) */
    for (size_t i = 0; i < S; i++) {
        uint32_t key;
        if (fmax3(ph[i].power) > 0) {
            v3 pp = scl(sub(ph[i].position, lo), inv);
            uint32_t gx = orx_f2u_sat(orx_floorf(pp.x));
            uint32_t gy = orx_f2u_sat(orx_floorf(pp.y));
            uint32_t gz = orx_f2u_sat(orx_floorf(pp.z));
            key = gx + gy * g[0] + gz * g[0] * g[1];
            if (key > G) key = G; /* out-of-grid edge: parked past the last cell, never gathered */
            r->hist[key]++;
        } else {
            key = invalid;
        }
        r->keys[i] = key;
    }
    /* exclusive_scan of G+1 entries (:202-207) */
    uint32_t run = 0;
    for (uint32_t c = 0; c <= G; c++) { r->offsets[c] = run; run += r->hist[c]; }
    r->valid = r->offsets[G];
    /* sort_by_key, stable (:193-196): counting sort over keys 0..G+1 */
    uint32_t* pos = (uint32_t*)malloc((size_t)(G + 2) * 4);
    uint32_t acc = 0;
    for (uint32_t c = 0; c <= G; c++) { pos[c] = acc; acc += r->hist[c]; }
    pos[G + 1] = acc;
    for (size_t i = 0; i < S; i++) r->sort_tmp[pos[r->keys[i]]++] = ph[i];
    free(pos);
    photon_t* t = r->photons; r->photons = r->sort_tmp; r->sort_tmp = t;
    return ORX_OK;
}

/* Stochastic hash (ACCELERATION_STRUCTURE_STOCHASTIC_HASH).
 * initializeStochasticHashPhotonMap (OptixRenderer_SpatialHash.cu:286-302): scene AABB padded
 * by r + 0.0001 (the sum in double, as written), cell = r, grid = calculateGridSize (:42-50);
 * the table counts are cleared (UniformGridPhotonInitialize.cu:20-23).  STORE_PHOTON
 * (store_photon.h:19-25) puts every deposit at getHashValue(getPhotonGridIndex(pos))
 * (PhotonGrid.h:19-33) and bumps the count; the reference's racing stores leave an arbitrary
 * deposit in the entry, here the one with the highest slot index (the device's atomicMax). */
static void ppm_build_hash(orc_renderer* r, float ppmRadius) {
    const float a = (float)((double)ppmRadius + 0.0001);
    const v3 lo = sub_s(r->aabb_min, a), hi = mk(r->aabb_max.x + a, r->aabb_max.y + a, r->aabb_max.z + a);
    const v3 f = divs(sub(hi, lo), ppmRadius);
    uint32_t g[3] = {orx_f2u_sat(orx_ceilf(f.x)), orx_f2u_sat(orx_ceilf(f.y)), orx_f2u_sat(orx_ceilf(f.z))};
    for (int k = 0; k < 3; k++) if (g[k] < 1) g[k] = 1;
    r->gsize[0] = g[0]; r->gsize[1] = g[1]; r->gsize[2] = g[2];
    r->cell = ppmRadius;
    r->origo = lo;
    r->ncells = (uint32_t)r->hnum;
    const uint32_t mask = (uint32_t)r->hnum - 1u;
    memset(r->hcount, 0, r->hnum * 4);
    memset(r->hwin, 0, r->hnum * 4);
    const size_t np = (size_t)r->cfg.photon_launch_width * r->prows;
    const float inv = 1.f / ppmRadius;
    uint32_t total = 0;
    for (size_t p = 0; p < np; p++) {
        for (uint32_t k = 0; k < r->ndep[p]; k++) {
            const uint32_t slot = (uint32_t)(p * r->dslot + k);
            const v3 pp = scl(sub(r->photons[slot].position, lo), inv);
            const uint32_t cx = orx_f2u_sat(orx_floorf(pp.x)), cy = orx_f2u_sat(orx_floorf(pp.y)),
                           cz = orx_f2u_sat(orx_floorf(pp.z));
            const uint32_t h = (cx + cy * g[0] + cz * g[0] * g[1]) & mask;
            r->hcount[h]++;
            if (slot + 1u > r->hwin[h]) r->hwin[h] = slot + 1u;
            total++;
        }
    }
    r->valid = total;
}

/* IndirectRadianceEstimation.cu:131-162: the 27 cells around the hit point's cell, one photon
 * per cell weighted by the cell's count; 27 cells and 27 photons counted as visited. */
static void ppm_gather_hash(orc_renderer* r, float ppmRadiusSquared, float emittedF) {
    const uint32_t W = r->W, H = r->rows;
    const uint32_t gx = r->gsize[0], gy = r->gsize[1];
    const uint32_t mask = (uint32_t)r->hnum - 1u;
    const v3 origo = r->origo;
    const float inv = 1.f / r->cell;
    uint64_t sumP = 0, sumC = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : sumP, sumC)
    for (long long y = 0; y < (long long)H; y++) {
        for (uint32_t x = 0; x < W; x++) {
            const size_t px = (size_t)y * W + x;
            const hitpoint_t rec = r->hp[px];
            v3 acc = mk1(0.0f);
            uint32_t dP = 0, dC = 0;
            if (rec.flags & PRD_HIT_NON_SPECULAR) {
                const float radius2 = ppmRadiusSquared;
                const v3 pp = scl(sub(rec.position, origo), inv);
                const uint32_t hx = orx_f2u_sat(orx_floorf(pp.x)), hy = orx_f2u_sat(orx_floorf(pp.y)),
                               hz = orx_f2u_sat(orx_floorf(pp.z));
                const float alpha = 1.818f, beta = 1.953f, expNegativeBeta = 0.141847f;
                const float inv2r2 = 1.0f / (2 * radius2);
                const float invDen = 1.0f / (1 - expNegativeBeta);
                for (int dz = -1; dz <= 1; dz++)
                    for (int dy = -1; dy <= 1; dy++)
                        for (int dx = -1; dx <= 1; dx++) {
                            const uint32_t cx = hx + (uint32_t)dx, cy = hy + (uint32_t)dy, cz = hz + (uint32_t)dz;
                            dC++;
                            dP++;
                            const uint32_t h = (cx + cy * gx + cz * gx * gy) & mask;
                            const uint32_t n = r->hcount[h];
                            if (!n) continue; /* an empty entry contributes power * 0 */
                            const photon_t* p = &r->photons[r->hwin[h] - 1u];
                            const v3 diff = sub(rec.position, p->position);
                            const float distance2 = dot(diff, diff);
                            if (distance2 <= radius2 && dot(neg(p->direction), rec.normal) >= 0) {
                                const float e = orx_expf_unit((-beta * distance2) * inv2r2);
                                const float wgt = alpha * (1 - (1 - e) * invDen);
                                acc = add(acc, scl(scl(p->power, wgt), (float)n));
                            }
                        }
            }
            const float s1 = 1.0f / (ORX_PI_F * ppmRadiusSquared);
            const float s2 = 1.0f / emittedF;
            r->indirect[px] = scl(scl(mul(acc, rec.attenuation), s1), s2);
            if (r->dbg) {
                r->dbg[2 * px] = dC;
                r->dbg[2 * px + 1] = dP;
            }
            sumP += dP;
            sumC += dC;
        }
    }
    r->sum_photons_visited = sumP;
    r->sum_cells_visited = sumC;
}

/* hitpoint source for the gather: the own rows, or `segments` export buffers of the sharded
 * gather (include/orx.h orx_export_hitpoints: plane A pos + flags float4, plane N the normal
 * float3; seg_rows*W pixels per plane padded to a multiple of 4, 28 B per pixel).  The export carries no attenuation: the
 * sharded gather returns the unattenuated estimate and the owner applies its hit point's
 * attenuation in orc_ppm_finish. */
typedef struct {
    const hitpoint_t* own;
    const float* ext;
    uint32_t seg_rows;
} hp_src;
static hitpoint_t hp_fetch(const orc_renderer* r, const hp_src* src, size_t px) {
    if (src->own) return src->own[px];
    const size_t plane = (size_t)src->seg_rows * r->W, p4 = (plane + 3) & ~(size_t)3;
    size_t seg = px / plane, li = px - seg * plane;
    const float* b = src->ext + seg * p4 * 7;
    const float* A = b + 4 * li;
    const float* N = b + 4 * p4 + 3 * li;
    hitpoint_t h;
    memset(&h, 0, sizeof h);
    h.position = mk(A[0], A[1], A[2]);
    memcpy(&h.flags, &A[3], 4);
    if (h.flags & PRD_HIT_NON_SPECULAR) h.normal = mk(N[0], N[1], N[2]);
    else h.radiance = mk(N[0], N[1], N[2]);
    h.attenuation = mk1(1.0f);
    return h;
}

/* IndirectRadianceEstimation.cu:54-67, :69-129, :211-221 */
static inline uint32_t slab_bin(const orc_renderer* r, v3 p, uint32_t a, uint32_t nb);
/* slab mode: a hit point outside this rank's bins is gathered by its owner */
static inline int hit_owned(const orc_renderer* r, v3 p) {
    if (!r->own_on) return 1;
    const uint32_t b = slab_bin(r, p, r->own_axis, r->own_nb);
    return b >= r->own_lo && b <= r->own_hi;
}
static void ppm_gather_src(orc_renderer* r, const hp_src* src, uint32_t rows_total, v3* out, uint32_t* dbg,
                           float ppmRadius, float ppmRadiusSquared, float emittedF) {
    const uint32_t W = r->W, H = rows_total;
    const uint32_t gx = r->gsize[0], gy = r->gsize[1], gz = r->gsize[2];
    const v3 origo = r->origo;
    const float cell = r->cell;
    uint64_t sumP = 0, sumC = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : sumP, sumC)
    for (long long y = 0; y < (long long)H; y++) {
        for (uint32_t x = 0; x < W; x++) {
            size_t px = (size_t)y * W + x;
            const hitpoint_t rec = hp_fetch(r, src, px);
            v3 acc = mk1(0.0f);
            uint32_t dP = 0, dC = 0;
            if ((rec.flags & PRD_HIT_NON_SPECULAR) && hit_owned(r, rec.position)) {
                float radius2 = ppmRadiusSquared;
                float radius = ppmRadius;
                float invCellSize = 1.f / cell;
                v3 np = sub(rec.position, origo);
                int32_t ixl = orx_f2i_sat((np.x - radius) * invCellSize);
                int32_t iyl = orx_f2i_sat((np.y - radius) * invCellSize);
                int32_t izl = orx_f2i_sat((np.z - radius) * invCellSize);
                uint32_t x_lo = (uint32_t)(ixl > 0 ? ixl : 0);
                uint32_t y_lo = (uint32_t)(iyl > 0 ? iyl : 0);
                uint32_t z_lo = (uint32_t)(izl > 0 ? izl : 0);
                uint32_t ux = orx_f2u_sat((np.x + radius) * invCellSize);
                uint32_t uy = orx_f2u_sat((np.y + radius) * invCellSize);
                uint32_t uz = orx_f2u_sat((np.z + radius) * invCellSize);
                uint32_t x_hi = (gx - 1) < ux ? (gx - 1) : ux;
                uint32_t y_hi = (gy - 1) < uy ? (gy - 1) : uy;
                uint32_t z_hi = (gz - 1) < uz ? (gz - 1) : uz;
                const float alpha = 1.818f, beta = 1.953f, expNegativeBeta = 0.141847f;
                const float inv2r2 = 1.0f / (2 * radius2);
                const float invDen = 1.0f / (1 - expNegativeBeta);
                if (x_lo <= x_hi) {
                    for (uint32_t z = z_lo; z <= z_hi; z++) {
                        for (uint32_t yy = y_lo; yy <= y_hi; yy++) {
                            uint32_t from = x_lo + yy * gx + z * gx * gy;
                            uint32_t to = from + (x_hi - x_lo);
                            uint32_t offset = r->offsets[from];
                            uint32_t offsetTo = r->offsets[to + 1];
                            uint32_t numPhotons = offsetTo - offset;
                            dC++;
                            for (uint32_t i = offset; i < offset + numPhotons; i++) {
                                const photon_t* p = &r->photons[i];
                                v3 diff = sub(rec.position, p->position);
                                float distance2 = dot(diff, diff);
                                if (distance2 <= radius2 && dot(neg(p->direction), rec.normal) >= 0) {
                                    /* photonPower (:59-67); its two divisions compile to div.approx
                                     * under -use_fast_math and are restated as multiplications by
                                     * the IEEE reciprocal of the (loop-invariant) divisor */
                                    float e = orx_expf_unit((-beta * distance2) * inv2r2);
                                    float wgt = alpha * (1 - (1 - e) * invDen);
                                    acc = add(acc, scl(p->power, wgt));
                                }
                                dP++;
                            }
                        }
                    }
                }
            }
            float s1 = 1.0f / (ORX_PI_F * ppmRadiusSquared);
            float s2 = 1.0f / emittedF;
            out[px] = scl(scl(mul(acc, rec.attenuation), s1), s2);
            if (dbg) {
                dbg[2 * px] = dC;
                dbg[2 * px + 1] = dP;
            }
            sumP += dP;
            sumC += dC;
        }
    }
    r->sum_photons_visited = sumP;
    r->sum_cells_visited = sumC;
}
static void ppm_gather(orc_renderer* r, float ppmRadius, float ppmRadiusSquared, float emittedF) {
    hp_src src = {r->hp, NULL, 0};
    ppm_gather_src(r, &src, r->rows, r->indirect, r->dbg, ppmRadius, ppmRadiusSquared, emittedF);
}

/* ------------------------------------------------------------------ */
/* kd-tree photon map (ACCELERATION_STRUCTURE_KD_TREE_CPU)             */
/* ------------------------------------------------------------------ */
/* pow2roundup (OptixRenderer.cpp:65-74) */
static uint32_t orc_pow2roundup(uint32_t x) {
    --x;
    x |= x >> 1;
    x |= x >> 2;
    x |= x >> 4;
    x |= x >> 8;
    x |= x >> 16;
    return x + 1;
}
#define PPM_X (1u << 0) /* config.h:12-16 */
#define PPM_Y (1u << 1)
#define PPM_Z (1u << 2)
#define PPM_LEAF (1u << 3)
#define PPM_NULL (1u << 4)

static inline float kd_coord(const kdphoton_t* e, int axis) {
    return axis == 0 ? e->p.position.x : axis == 1 ? e->p.position.y : e->p.position.z;
}
static inline void kd_swap(kdphoton_t* list, int a, int b) {
    kdphoton_t t = list[a];
    list[a] = list[b];
    list[b] = t;
}
/* select.h `partition` (the variant that puts the pivot at its sorted position) */
static int kd_partition(kdphoton_t* list, int left, int right, int pivotIndex, int axis) {
    const kdphoton_t pivotValue = list[pivotIndex];
    const float pv = kd_coord(&pivotValue, axis);
    kd_swap(list, right, pivotIndex);
    pivotIndex = right;
    left--;
    for (;;) {
        do {
            left++;
        } while (left < right && kd_coord(&list[left], axis) < pv);
        do {
            right--;
        } while (left < right && kd_coord(&list[right], axis) > pv);
        if (left < right) {
            kd_swap(list, left, right);
        } else {
            kd_swap(list, left, pivotIndex);
            return left;
        }
    }
}
/* select.h `select`: pivot at the middle, loop until the k-th lands */
static void kd_select(kdphoton_t* list, int left, int right, int k, int axis) {
    for (;;) {
        const int pivotIndex = (left + right) / 2;
        const int pivotNewIndex = kd_partition(list, left, right, pivotIndex, axis);
        if (k == pivotNewIndex) return;
        if (k < pivotNewIndex) right = pivotNewIndex - 1;
        else left = pivotNewIndex + 1;
    }
}
/* max_component (OptixRenderer_CPUKdTree.cpp:14-25) */
static int kd_max_component(v3 a) {
    if (a.x > a.y && a.x > a.z) return 0;
    if (a.y > a.z) return 1;
    return 2;
}
/* buildKDTree (OptixRenderer_CPUKdTree.cpp:27-88) */
static void kd_build(kdphoton_t* photons, int start, int end, uint32_t depth, kdphoton_t* kd_tree, size_t current_root,
                     v3 bbmin, v3 bbmax, uint32_t* maxdepth) {
    if (depth > *maxdepth) *maxdepth = depth;
    if (end - start == 0) { /* NULL node: only axis and power are written */
        kd_tree[current_root].axis = PPM_NULL;
        kd_tree[current_root].p.power = mk1(0.0f);
        return;
    }
    if (end - start == 1) {
        photons[start].axis = PPM_LEAF;
        kd_tree[current_root] = photons[start];
        return;
    }
    const int axis = kd_max_component(sub(bbmax, bbmin));
    const int median = (start + end) / 2;
    kd_select(photons + start, 0, end - start - 1, median - start, axis);
    photons[median].axis = axis == 0 ? PPM_X : axis == 1 ? PPM_Y : PPM_Z;
    v3 rightMin = bbmin, leftMax = bbmax;
    const v3 midPoint = photons[median].p.position;
    if (axis == 0) { rightMin.x = midPoint.x; leftMax.x = midPoint.x; }
    else if (axis == 1) { rightMin.y = midPoint.y; leftMax.y = midPoint.y; }
    else { rightMin.z = midPoint.z; leftMax.z = midPoint.z; }
    kd_tree[current_root] = photons[median];
    kd_build(photons, start, median, depth + 1, kd_tree, 2 * current_root + 1, bbmin, leftMax, maxdepth);
    kd_build(photons, median + 1, end, depth + 1, kd_tree, 2 * current_root + 2, rightMin, bbmax, maxdepth);
}
/* createPhotonKdTreeOnCPU (OptixRenderer_CPUKdTree.cpp:90-127): drop invalid photons by moving
 * the last one into their place, bound the rest, build.  Nodes the build does not reach keep
 * what earlier iterations left there (the reference never clears m_photonKdTree). */
static void ppm_build_kdtree(orc_renderer* r) {
    const size_t S = (size_t)r->cfg.photon_launch_width * r->prows * r->cfg.max_photon_deposits;
    kdphoton_t* ph = r->kdwork;
    for (size_t i = 0; i < S; i++) {
        ph[i].p = r->photons[i];
        ph[i].axis = 0;
    }
    uint32_t numValidPhotons = (uint32_t)(S >= r->kdsize ? r->kdsize : S);
    for (uint32_t i = 0; i < numValidPhotons; ++i) {
        if (!(fmax3(ph[i].p.power) > 0.0f)) {
            ph[i] = ph[numValidPhotons - 1];
            numValidPhotons--;
            i--;
        }
    }
    v3 bbmin = mk1(FLT_MAX), bbmax = mk1(-FLT_MAX);
    for (uint32_t i = 0; i < numValidPhotons; ++i) {
        bbmin = vmin(bbmin, ph[i].p.position);
        bbmax = vmax(bbmax, ph[i].p.position);
    }
    uint32_t maxdepth = 0;
    kd_build(ph, 0, (int)numValidPhotons, 0, r->kdtree, 0, bbmin, bbmax, &maxdepth);
    r->kddepth = maxdepth;
    r->valid = numValidPhotons;
    r->ncells = (uint32_t)r->kdsize;
}
/* IndirectRadianceEstimation.cu:164-209 (the OptiX SDK PPM sample's traversal): visit a node,
 * add its photon if valid, push the far child when the split plane is within the radius, go
 * near.  The reference's stack of MAX_DEPTH = 21 entries overflows on trees deeper than 20
 * levels (undefined behaviour there); the stack here holds a full 32-bit tree. */
#define KD_STACK 40
static void ppm_gather_kd_src(orc_renderer* r, const hp_src* src, uint32_t rows_total, v3* out, uint32_t* dbg,
                              float ppmRadiusSquared, float emittedF) {
    const uint32_t W = r->W, H = rows_total;
    const kdphoton_t* tree = r->kdtree;
    uint64_t sumP = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : sumP)
    for (long long y = 0; y < (long long)H; y++) {
        for (uint32_t x = 0; x < W; x++) {
            const size_t px = (size_t)y * W + x;
            const hitpoint_t rec = hp_fetch(r, src, px);
            v3 acc = mk1(0.0f);
            uint32_t dP = 0;
            if (rec.flags & PRD_HIT_NON_SPECULAR) {
                const float radius2 = ppmRadiusSquared;
                const float alpha = 1.818f, beta = 1.953f, expNegativeBeta = 0.141847f;
                const float inv2r2 = 1.0f / (2 * radius2);
                const float invDen = 1.0f / (1 - expNegativeBeta);
                size_t stack[KD_STACK];
                uint32_t sc = 0;
                size_t node = 0;
                stack[sc++] = 0;
                do {
                    const kdphoton_t* photon = &tree[node];
                    dP++;
                    const uint32_t axis = photon->axis;
                    if (!(axis & PPM_NULL)) {
                        const v3 diff = sub(rec.position, photon->p.position);
                        const float distance2 = dot(diff, diff);
                        if (distance2 <= radius2 && dot(neg(photon->p.direction), rec.normal) >= 0) {
                            const float e = orx_expf_unit((-beta * distance2) * inv2r2);
                            const float wgt = alpha * (1 - (1 - e) * invDen);
                            acc = add(acc, scl(photon->p.power, wgt));
                        }
                        if (!(axis & PPM_LEAF)) {
                            const float d = (axis & PPM_X) ? diff.x : (axis & PPM_Y) ? diff.y : diff.z;
                            const size_t selector = d < 0.0f ? 0 : 1;
                            if (d * d < radius2) stack[sc++] = (node << 1) + 2 - selector;
                            node = (node << 1) + 1 + selector;
                        } else {
                            node = stack[--sc];
                        }
                    } else {
                        node = stack[--sc];
                    }
                } while (node);
            }
            const float s1 = 1.0f / (ORX_PI_F * ppmRadiusSquared);
            const float s2 = 1.0f / emittedF;
            out[px] = scl(scl(mul(acc, rec.attenuation), s1), s2);
            if (dbg) {
                dbg[2 * px] = 0;
                dbg[2 * px + 1] = dP;
            }
            sumP += dP;
        }
    }
    r->sum_photons_visited = sumP;
    r->sum_cells_visited = 0;
}

/* helpers/light.h:29-87 */
static v3 light_contribution(const orc_renderer* r, const light_t* light, v3 pos, v3 normal, uint32_t* rs) {
    float lightFactor = 1;
    v3 pointOnLight = mk1(0);
    if (light->type == ORX_LIGHT_AREA) {
        float sx = orc_uniform(rs), sy = orc_uniform(rs);
        pointOnLight = add(add(light->position, scl(light->v1, sx)), scl(light->v2, sy));
    } else if (light->type == ORX_LIGHT_POINT) {
        pointOnLight = light->position;
        lightFactor *= 1.f / 4.f;
    } else {
        return mk1(0); /* SPOT: lightFactor = 0 */
    }
    v3 towardsLight = sub(pointOnLight, pos);
    float lightDistance = length(towardsLight);
    towardsLight = divs(towardsLight, lightDistance);
    float n_dot_l = maxf(0, dot(normal, towardsLight));
    lightFactor *= n_dot_l / (ORX_PI_F * lightDistance * lightDistance);
    if (light->type == ORX_LIGHT_AREA) lightFactor *= maxf(0, dot(neg(towardsLight), light->normal));
    if (lightFactor > 0.0f) {
        float tmax = (float)((double)lightDistance - 0.0001);
        float att = trace_any(r, pos, towardsLight, 0.0001f, tmax) ? 0.0f : 1.0f;
        lightFactor *= att;
        return scl(light->power, lightFactor);
    }
    return mk1(0);
}

/* DirectRadianceEstimation.cu:29-77 */
static void ppm_direct(orc_renderer* r) {
    const uint32_t W = r->W;
    const int numLights = (int)r->nl;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long j = 0; j < (long long)r->rows; j++) {
        const uint32_t y = r->rank + r->world * (uint32_t)j;
        for (uint32_t x = 0; x < W; x++) {
            size_t px = (size_t)j * W + x;
            const hitpoint_t rec = r->hp[px];
            if (!(rec.flags & PRD_HIT_NON_SPECULAR)) {
                if ((rec.flags & PRD_HIT_EMITTER) && !(rec.flags & PRD_HIT_SPECULAR))
                    r->direct[px] = mk(fminf(rec.radiance.x, 1), fminf(rec.radiance.y, 1), fminf(rec.radiance.z, 1));
                else
                    r->direct[px] = rec.radiance;
                continue;
            }
            if (r->med_on) { /* numShadowSamples = ENABLE_PARTICIPATING_MEDIA ? 0 : 4 (:54) */
                r->direct[px] = mk1(0.f);
                continue;
            }
            uint32_t* rs = r->rng + 6 * ((size_t)y * r->RW + x);
            v3 avg = mk1(0.f);
            for (int s = 0; s < 4; s++) {
                float sample = orc_uniform(rs);
                int li = (int)(sample * numLights);
                int randomLightIndex = li < numLights - 1 ? li : numLights - 1;
                float scale = (float)numLights;
                v3 c = light_contribution(r, &r->lights[randomLightIndex], rec.position, rec.normal, rs);
                avg = add(avg, scl(c, scale));
            }
            r->direct[px] = divs(mul(rec.attenuation, avg), (float)4);
        }
    }
}

/* Output.cu:32-37 */
static void ppm_output(orc_renderer* r, uint64_t local) {
    size_t n = (size_t)r->W * r->rows;
    for (size_t i = 0; i < n; i++) {
        v3 f = add(r->direct[i], r->indirect[i]);
        r->output[i] = local == 0 ? f : add(r->output[i], f);
    }
}

/* RayGeneratorPT.cu:46-131 */
static void pt_pass(orc_renderer* r, const cam_t* cam, uint64_t local) {
    const uint32_t W = r->W, H = r->H;
    const int numLights = (int)r->nl;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long j = 0; j < (long long)r->rows; j++) {
        const uint32_t y = r->rank + r->world * (uint32_t)j;
        for (uint32_t x = 0; x < W; x++) {
            size_t px = (size_t)j * W + x;
            uint32_t* G = r->rng + 6 * ((size_t)y * r->RW + x);
            uint32_t rs[6];
            memcpy(rs, G, 24);
            rprd_t prd;
            memset(&prd, 0, sizeof prd);
            prd.attenuation = mk1(1.0f);
            prd.rs = rs;
            v3 o, d;
            primary_ray(cam, x, y, W, H, rs, &o, &d);
            v3 fin = mk1(0);
            for (int i = 0; i < 5; i++) {
                prd.flags = PRD_PATH_TRACING;
                trace_radiance(r, o, d, 0.001f, &prd, NULL);
                if (prd.flags & PRD_HIT_EMITTER) {
                    if ((prd.flags & PRD_HIT_SPECULAR) || i == 0) fin = prd.radiance;
                    break;
                } else if (prd.flags & PRD_HIT_NON_SPECULAR) {
                    v3 accum = mk1(0);
                    int li = (int)(orc_uniform(G) * numLights);
                    float scale = (float)numLights;
                    v3 c = scl(light_contribution(r, &r->lights[li], prd.position, prd.normal, rs), scale);
                    accum = add(accum, c);
                    v3 direct = divs(mul(prd.attenuation, accum), (float)1);
                    fin = add(fin, direct);
                    o = prd.position;
                    d = prd.newdir;
                } else {
                    break;
                }
                if (i >= 3) { /* PATH_TRACING_RR_START_DEPTH */
                    float sample = orc_uniform(G);
                    float p = fmax3(prd.attenuation);
                    if (sample > p) break;
                    prd.attenuation = divs(prd.attenuation, p);
                }
            }
            if (!isnan3(fin)) r->output[px] = local == 0 ? fin : add(r->output[px], fin);
            memcpy(G, rs, 24);
        }
    }
}

static orx_status begin_iteration(orc_renderer* r, uint64_t local, const orx_request* det);
#include "orx_oracle_vcm.c.inc"

/* ------------------------------------------------------------------ */
/* OptixRenderer::renderNextIteration (OptixRenderer.cpp:507-821)     */
/* ------------------------------------------------------------------ */
static orx_status begin_iteration(orc_renderer* r, uint64_t local, const orx_request* det) {
    if (!r->scene_ready) return fail(r, ORX_ERR_STATE, "Traced before OptixRenderer was initialized.");
    if (det->width == 0 || det->height == 0) return fail(r, ORX_ERR_INVALID_ARGUMENT, "zero-sized request");
    if (det->width != r->W || det->height != r->H) { /* resizeBuffers (OptixRenderer.cpp:826-848) */
        r->psf_x = 1.0f / (float)det->width;
        r->psf_y = 1.0f / (float)det->height;
        r->vcm_estimated = 0;
    }
    if (det->width != r->W || det->height != r->H || !r->rng_ready) {
        orx_status s = resize(r, det->width, det->height);
        if (s != ORX_OK) return s;
    }
    if (local == 0) memset(r->output, 0, (size_t)r->W * r->max_rows * sizeof(v3));
    return ORX_OK;
}

orx_status orc_render_next_iteration(orc_renderer* r, uint64_t iter, uint64_t local, float ppmRadius,
                                     int create_output, const orx_request* det) {
    (void)create_output;
    (void)iter;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    if (det->method == ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING && r->world > 1)
        return fail(r, ORX_ERR_STATE, "sharded PPM runs through the phase API");
    if (det->method == ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING && r->world > 1)
        return fail(r, ORX_ERR_STATE, "sharded VCM runs through the phase API");
    if (det->method != ORX_METHOD_PATH_TRACING && det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING &&
        det->method != ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING)
        return fail(r, ORX_ERR_UNSUPPORTED, "oracle: method not implemented");
    if (r->med_on && det->method != ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING)
        return fail(r, ORX_ERR_UNSUPPORTED, "participating media: progressive photon mapping only");
    if (r->med_on && r->cfg.photon_map == 1)
        return fail(r, ORX_ERR_UNSUPPORTED, "participating media: uniform grid or kd-tree photon map");
    orx_status s0 = begin_iteration(r, local, det);
    if (s0 != ORX_OK) return s0;
    cam_t cam = camera_setup(&det->camera);
    if (det->method == ORX_METHOD_PATH_TRACING) {
        pt_pass(r, &cam, local);
    } else if (det->method == ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING) {
        return vcm_iteration(r, det, ppmRadius);
    } else {
        ppm_eye_pass(r, &cam);
        const float ppmRadiusSquared = ppmRadius * ppmRadius;
        ppm_photon_pass(r);
        if (r->med_on) vol_resolve(r, ppmRadius);
        float emittedF = (float)(r->cfg.photon_launch_width * r->cfg.photon_launch_height);
        if (r->cfg.photon_map == 1) {
            ppm_build_hash(r, ppmRadius);
            ppm_gather_hash(r, ppmRadiusSquared, emittedF);
        } else if (r->cfg.photon_map == 2) {
            ppm_build_kdtree(r);
            hp_src src = {r->hp, NULL, 0};
            ppm_gather_kd_src(r, &src, r->rows, r->indirect, r->dbg, ppmRadiusSquared, emittedF);
        } else {
            orx_status s = ppm_build_grid(r);
            if (s != ORX_OK) return s;
            ppm_gather(r, ppmRadius, ppmRadiusSquared, emittedF);
        }
        if (r->med_on) /* IndirectRadianceEstimation.cu:215-218 */
            for (size_t i = 0; i < (size_t)r->W * r->rows; i++) r->indirect[i] = add(r->indirect[i], divs(r->volR[i], emittedF));
        ppm_direct(r);
        ppm_output(r, local);
    }
    return ORX_OK;
}

/* ---- sharded phase API (mirrors orx_ppm_* in include/orx.h) ---- */
orx_status orc_set_shard(orc_renderer* r, uint32_t rank, uint32_t world) {
    if (!r || world == 0 || rank >= world) return ORX_ERR_INVALID_ARGUMENT;
    if (world > 1 && r->cfg.enable_media)
        return fail(r, ORX_ERR_UNSUPPORTED, "participating media are single-device");
    if (world > 1 && r->cfg.photon_map == 1)
        return fail(r, ORX_ERR_UNSUPPORTED, "the stochastic hash photon map is single-device");
    r->rank = rank;
    r->world = world;
    r->rng_ready = 0;
    return ORX_OK;
}
uint32_t orc_max_local_rows(const orc_renderer* r) { return (r->H + r->world - 1) / r->world; }
uint32_t orc_local_rows(const orc_renderer* r) { return r->rows; }
size_t orc_hitpoint_export_bytes(const orc_renderer* r) {
    return (((size_t)orc_max_local_rows(r) * r->W + 3) & ~(size_t)3) * 28;
}

orx_status orc_ppm_local_passes(orc_renderer* r, uint64_t iter, uint64_t local, float ppmRadius, const orx_request* det) {
    (void)iter;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    orx_status s0 = begin_iteration(r, local, det);
    if (s0 != ORX_OK) return s0;
    cam_t cam = camera_setup(&det->camera);
    ppm_eye_pass(r, &cam);
    ppm_photon_pass(r);
    if (r->cfg.photon_map == 2) {
        ppm_build_kdtree(r);
    } else {
        orx_status s = ppm_build_grid(r);
        if (s != ORX_OK) return s;
    }
    r->last_radius = ppmRadius;
    r->last_radius2 = ppmRadius * ppmRadius;
    r->last_local = local;
    return ORX_OK;
}
/* Slab mode of the sharded gather (include/orx.h orx_set_slab_partition): the same phases on the
 * oracle's photon array.  A photon is valid if fmaxf(power) > 0 (the grid's own test). */
orx_status orc_ppm_local_trace(orc_renderer* r, uint64_t iter, uint64_t local, float ppmRadius, const orx_request* det) {
    (void)iter;
    if (!r || !det) return ORX_ERR_INVALID_ARGUMENT;
    orx_status s0 = begin_iteration(r, local, det);
    if (s0 != ORX_OK) return s0;
    cam_t cam = camera_setup(&det->camera);
    ppm_eye_pass(r, &cam);
    ppm_photon_pass(r);
    r->last_radius = ppmRadius;
    r->last_radius2 = ppmRadius * ppmRadius;
    r->last_local = local;
    return ORX_OK;
}
static inline uint32_t slab_bin(const orc_renderer* r, v3 p, uint32_t a, uint32_t nb) {
    const float lo = a == 0 ? r->aabb_min.x : a == 1 ? r->aabb_min.y : r->aabb_min.z;
    const float hi = a == 0 ? r->aabb_max.x : a == 1 ? r->aabb_max.y : r->aabb_max.z;
    const float ext = hi - lo, inv = ext > 0.f ? (float)nb / ext : 0.f;
    const float v = a == 0 ? p.x : a == 1 ? p.y : p.z;
    const int32_t b = orx_f2i_sat(orx_floorf((v - lo) * inv));
    return b < 0 ? 0u : (b >= (int32_t)nb ? nb - 1u : (uint32_t)b);
}
uint32_t orc_ppm_slab_halo(const orc_renderer* r, uint32_t nb, uint32_t axis, float radius) {
    if (!r || axis > 2 || nb == 0) return 2u;
    const float lo = axis == 0 ? r->aabb_min.x : axis == 1 ? r->aabb_min.y : r->aabb_min.z;
    const float hi = axis == 0 ? r->aabb_max.x : axis == 1 ? r->aabb_max.y : r->aabb_max.z;
    const float ext = hi - lo, inv = ext > 0.f ? (float)nb / ext : 0.f;
    const float h = orx_floorf(radius * inv);
    return (h >= 0.f && h < 1e6f ? (uint32_t)h : 0u) + 2u;
}
static size_t local_slots(const orc_renderer* r) {
    return (size_t)r->cfg.photon_launch_width * r->prows * r->cfg.max_photon_deposits;
}
static inline uint32_t slab_voxel(const orc_renderer* r, v3 p) {
    const uint32_t V = ORX_SLAB_VOXELS;
    return slab_bin(r, p, 0, V) + V * (slab_bin(r, p, 1, V) + V * slab_bin(r, p, 2, V));
}
orx_status orc_ppm_slab_histogram(orc_renderer* r, uint32_t* hist, uint32_t nb) {
    if (!r || !hist || nb < ORX_SLAB_VOXELS || nb > 1024 || nb % ORX_SLAB_VOXELS) return ORX_ERR_INVALID_ARGUMENT;
    memset(hist, 0, ((size_t)6 * nb + 6 + 2 * (size_t)ORX_SLAB_VOXELS * ORX_SLAB_VOXELS * ORX_SLAB_VOXELS) * 4);
    const size_t S = local_slots(r);
    const size_t NV = (size_t)ORX_SLAB_VOXELS * ORX_SLAB_VOXELS * ORX_SLAB_VOXELS;
    uint32_t* hv = hist + 6 * (size_t)nb + 6;
    photon_box_words(r->photons, S, hist + 6 * (size_t)nb);
    for (size_t i = 0; i < S; i++) {
        if (!(fmax3(r->photons[i].power) > 0)) continue;
        for (uint32_t a = 0; a < 3; a++) hist[a * nb + slab_bin(r, r->photons[i].position, a, nb)]++;
        hv[slab_voxel(r, r->photons[i].position)]++;
    }
    for (size_t i = 0; i < (size_t)r->rows * r->W; i++) {
        if (!(r->hp[i].flags & PRD_HIT_NON_SPECULAR)) continue;
        for (uint32_t a = 0; a < 3; a++) hist[(3 + a) * nb + slab_bin(r, r->hp[i].position, a, nb)]++;
        hv[NV + slab_voxel(r, r->hp[i].position)]++;
    }
    return ORX_OK;
}
orx_status orc_ppm_slab_pack(orc_renderer* r, const uint8_t* bin_dest, uint32_t nb, uint32_t axis, uint32_t halo,
                             const uint32_t* dest_base, uint64_t send_records, float* send) {
    if (!r || !bin_dest || !dest_base || !send || nb == 0 || axis > 2) return ORX_ERR_INVALID_ARGUMENT;
    uint32_t cur[256];
    if (r->world > 256) return ORX_ERR_UNSUPPORTED;
    memcpy(cur, dest_base, (size_t)r->world * 4);
    const size_t S = local_slots(r);
    for (size_t i = 0; i < S; i++) {
        const photon_t* p = &r->photons[i];
        if (!(fmax3(p->power) > 0)) continue;
        const uint32_t b = slab_bin(r, p->position, axis, nb);
        const uint32_t d0 = bin_dest[b > halo ? b - halo : 0u], d1 = bin_dest[b + halo < nb ? b + halo : nb - 1u];
        for (uint32_t d = d0; d <= d1; d++) { /* the owner and the ranks within the halo */
            if (d >= r->world || cur[d] >= send_records)
                return fail(r, ORX_ERR_INVALID_ARGUMENT, "slab plan overflows the send buffer");
            float* w = send + 9 * (size_t)cur[d]++;
            w[0] = p->position.x; w[1] = p->position.y; w[2] = p->position.z;
            w[3] = p->direction.x; w[4] = p->direction.y; w[5] = p->direction.z;
            w[6] = p->power.x; w[7] = p->power.y; w[8] = p->power.z;
        }
    }
    return ORX_OK;
}
orx_status orc_ppm_slab_import(orc_renderer* r, const float* recv, uint64_t n, const uint32_t* box, uint32_t axis,
                               uint32_t nb, uint32_t own_lo, uint32_t own_hi) {
    if (!r || (!recv && n) || axis > 2 || nb == 0) return ORX_ERR_INVALID_ARGUMENT;
    r->own_on = 1;
    r->own_axis = axis;
    r->own_nb = nb;
    r->own_lo = own_lo;
    r->own_hi = own_hi;
    const size_t S = local_slots(r);
    const size_t need = n > S ? n : S;
    if (need > S) { /* realloc keeps the contents; the own photon pass uses the first S entries */
        photon_t* a = (photon_t*)realloc(r->photons, need * sizeof(photon_t));
        if (a) r->photons = a;
        photon_t* b = (photon_t*)realloc(r->sort_tmp, need * sizeof(photon_t));
        if (b) r->sort_tmp = b;
        uint32_t* k = (uint32_t*)realloc(r->keys, need * 4);
        if (k) r->keys = k;
        if (!a || !b || !k) return fail(r, ORX_ERR_OUT_OF_MEMORY, "oracle: out of memory");
    }
    for (size_t i = 0; i < n; i++) {
        const float* w = recv + 9 * i;
        photon_t* p = &r->photons[i];
        p->position = mk(w[0], w[1], w[2]);
        p->direction = mk(w[3], w[4], w[5]);
        p->power = mk(w[6], w[7], w[8]);
    }
    return ppm_build_grid_n(r, (size_t)n, box);
}

orx_status orc_export_hitpoints(orc_renderer* r, void* dst, size_t bytes) {
    const size_t plane = (((size_t)r->max_rows * r->W) + 3) & ~(size_t)3; /* padded: 16-B aligned planes */
    if (!dst || bytes < plane * 28) return ORX_ERR_INVALID_ARGUMENT;
    float* b = (float*)dst;
    memset(b, 0, plane * 28);
    for (size_t i = 0; i < (size_t)r->rows * r->W; i++) {
        const hitpoint_t* h = &r->hp[i];
        float* A = b + 4 * i;
        float* N = b + 4 * plane + 3 * i;
        A[0] = h->position.x; A[1] = h->position.y; A[2] = h->position.z;
        memcpy(&A[3], &h->flags, 4);
        v3 nr = (h->flags & PRD_HIT_NON_SPECULAR) ? h->normal : h->radiance;
        N[0] = nr.x; N[1] = nr.y; N[2] = nr.z;
    }
    return ORX_OK;
}
orx_status orc_ppm_gather_external(orc_renderer* r, const void* hp, uint32_t segments, void* indirect, size_t bytes) {
    if (!hp || !indirect || bytes < (size_t)segments * r->max_rows * r->W * 12) return ORX_ERR_INVALID_ARGUMENT;
    hp_src src = {NULL, (const float*)hp, r->max_rows};
    float emittedF = (float)(r->cfg.photon_launch_width * r->cfg.photon_launch_height);
    if (r->cfg.photon_map == 2)
        ppm_gather_kd_src(r, &src, segments * r->max_rows, (v3*)indirect, NULL, r->last_radius2, emittedF);
    else
        ppm_gather_src(r, &src, segments * r->max_rows, (v3*)indirect, NULL, r->last_radius, r->last_radius2, emittedF);
    return ORX_OK;
}
orx_status orc_ppm_finish(orc_renderer* r, const void* indirect, size_t bytes) {
    if (!indirect || bytes < (size_t)r->max_rows * r->W * 12) return ORX_ERR_INVALID_ARGUMENT;
    /* the summed unattenuated estimates of the own rows times each hit point's attenuation
     * (the single-device gather multiplies inside, IndirectRadianceEstimation.cu:220: the same
     * value up to fp32 order) */
    const v3* in = (const v3*)indirect;
    for (size_t i = 0; i < (size_t)r->rows * r->W; i++) r->indirect[i] = mul(in[i], r->hp[i].attenuation);
    ppm_direct(r);
    ppm_output(r, r->last_local);
    return ORX_OK;
}

orx_status orc_get_output(orc_renderer* r, float* dst, size_t bytes) {
    size_t need = (size_t)r->W * r->rows * 12;
    if (!dst || bytes < need) return ORX_ERR_INVALID_ARGUMENT;
    memcpy(dst, r->output, need);
    return ORX_OK;
}

orx_status orc_read_buffer(orc_renderer* r, int32_t id, void* dst, size_t bytes, size_t* out_bytes) {
    size_t npx = (size_t)r->W * r->rows;
    size_t need = 0;
    switch (id) {
    case ORX_BUF_RNG: need = (size_t)r->RW * r->RH * 24; break;
    case ORX_BUF_HITPOINTS: need = npx * 13 * 4; break;
    case ORX_BUF_PHOTONS: need = (r->hcount ? r->hnum : (size_t)r->valid) * 36; break;
    case ORX_BUF_GRID_OFFSETS: need = (r->hcount ? r->hnum : (size_t)r->ncells + 1) * 4; break;
    case ORX_BUF_INDIRECT: case ORX_BUF_DIRECT: case ORX_BUF_OUTPUT: need = npx * 12; break;
    case ORX_BUF_DEBUG_VISITED: need = npx * 8; break;
    case ORX_BUF_VCM_VERTEX_COUNT: need = r->vcm_npx * 4; break;
    case ORX_BUF_VCM_VERTICES: need = r->vcm_npx * VCM_MAX_VERTS * 64; break;
    case ORX_BUF_VCM_SPLAT: case ORX_BUF_VCM_CAMERA: need = r->vcm_npx * 12; break; /* own rows */
    case ORX_BUF_KD_TREE: need = r->kdsize * 40; break;
    case ORX_BUF_PHOTON_SLOTS: need = (size_t)r->cfg.photon_launch_width * r->prows * r->dslot * 36; break;
    case ORX_BUF_VOLUMETRIC: need = r->med_on ? npx * 12 : 0; break;
    case ORX_BUF_VOLUMETRIC_PHOTONS: need = r->med_on ? (size_t)r->nvol * 28 : 0; break;
    default: return fail(r, ORX_ERR_INVALID_ARGUMENT, "unknown buffer id");
    }
    if (out_bytes) *out_bytes = need;
    if (!dst) return ORX_OK;
    if (bytes < need) return fail(r, ORX_ERR_INVALID_ARGUMENT, "destination too small");
    switch (id) {
    case ORX_BUF_RNG: memcpy(dst, r->rng, need); break;
    case ORX_BUF_HITPOINTS: {
        float* f = (float*)dst;
        for (size_t i = 0; i < npx; i++) {
            const hitpoint_t* h = &r->hp[i];
            float v[13] = {h->position.x, h->position.y, h->position.z, h->normal.x, h->normal.y, h->normal.z,
                           h->attenuation.x, h->attenuation.y, h->attenuation.z, h->radiance.x, h->radiance.y,
                           h->radiance.z, orx_as_float(h->flags)};
            memcpy(f + 13 * i, v, sizeof v);
        }
        break;
    }
    case ORX_BUF_PHOTONS:
        if (r->hcount) { /* the table: each entry's photon, zeros when empty */
            float* f = (float*)dst;
            for (size_t h = 0; h < r->hnum; h++) {
                float v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                if (r->hcount[h]) memcpy(v, &r->photons[r->hwin[h] - 1u], sizeof v);
                memcpy(f + 9 * h, v, sizeof v);
            }
        } else {
            memcpy(dst, r->photons, need);
        }
        break;
    case ORX_BUF_GRID_OFFSETS: memcpy(dst, r->hcount ? r->hcount : r->offsets, need); break;
    case ORX_BUF_INDIRECT: memcpy(dst, r->indirect, need); break;
    case ORX_BUF_DIRECT: memcpy(dst, r->direct, need); break;
    case ORX_BUF_OUTPUT: memcpy(dst, r->output, need); break;
    case ORX_BUF_DEBUG_VISITED: memcpy(dst, r->dbg, need); break;
    case ORX_BUF_VCM_VERTEX_COUNT: memcpy(dst, r->vcount, need); break;
    case ORX_BUF_VCM_VERTICES: memcpy(dst, r->vverts, need); break;
    case ORX_BUF_VCM_SPLAT: memcpy(dst, r->vsplat + (size_t)r->rank * r->max_rows * r->W, need); break;
    case ORX_BUF_VCM_CAMERA: memcpy(dst, r->vcam, need); break;
    case ORX_BUF_PHOTON_SLOTS: /* slot order: the grid build swapped the unsorted slots into sort_tmp */
        memcpy(dst, (r->cfg.photon_map == 0 && r->ncells) ? r->sort_tmp : r->photons, need);
        break;
    case ORX_BUF_VOLUMETRIC: if (need) memcpy(dst, r->volR, need); break;
    case ORX_BUF_VOLUMETRIC_PHOTONS: {
        float* f = (float*)dst;
        for (size_t i = 0; need && i < r->nvol; i++) {
            const int on = r->vol_ready && r->vcnt[i];
            float v[7] = {on ? r->vpow[i].x : 0.f, on ? r->vpow[i].y : 0.f, on ? r->vpow[i].z : 0.f,
                          on ? r->vpos[i].x : 0.f, on ? r->vpos[i].y : 0.f, on ? r->vpos[i].z : 0.f, 0.f};
            const uint32_t c = on ? r->vcnt[i] : 0u;
            memcpy(&v[6], &c, 4);
            memcpy(f + 7 * i, v, sizeof v);
        }
        break;
    }
    case ORX_BUF_KD_TREE: {
        float* f = (float*)dst;
        for (size_t i = 0; i < r->kdsize; i++) {
            memcpy(f + 10 * i, &r->kdtree[i].p, 36);
            memcpy(f + 10 * i + 9, &r->kdtree[i].axis, 4);
        }
        break;
    }
    }
    return ORX_OK;
}

orx_status orc_get_stats(orc_renderer* r, orx_stats* out) {
    memset(out, 0, sizeof *out);
    out->grid_size[0] = r->gsize[0]; out->grid_size[1] = r->gsize[1]; out->grid_size[2] = r->gsize[2];
    out->cell_size = r->cell;
    out->world_origin[0] = r->origo.x; out->world_origin[1] = r->origo.y; out->world_origin[2] = r->origo.z;
    out->valid_photons = r->valid;
    out->num_cells = r->ncells;
    out->photons_visited = r->sum_photons_visited;
    out->cells_visited = r->sum_cells_visited;
    return ORX_OK;
}

void orc_default_config(orx_config* c) {
    memset(c, 0, sizeof *c);
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
