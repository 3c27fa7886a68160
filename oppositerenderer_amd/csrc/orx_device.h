/*
 * orx_device.h — gfx950 device-side building blocks of the render core.
 *
 * Replaces the OptiX device runtime + helper headers of the reference:
 *   helpers/random.h (cuRAND XORWOW), helpers/samplers.h, helpers/helpers.h,
 *   helpers/camera.h, helpers/light.h (getLightContribution),
 *   geometry_instance/{parallelogram,Sphere,TriangleMesh}.cu (intersection),
 *   OptiX closest-hit / any-hit dispatch (flattened into switch-on-material).
 * Float expressions keep the reference's operand order; the library is built
 * with -ffp-contract=off and correctly rounded div/sqrt so the kernels agree
 * bit for bit with the CPU oracle on every control-flow decision.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orx_detmath.h"

namespace orx {

/* ------------------------------------------------------------------ */
/* float3 with OptiX semantics                                          */
/* ------------------------------------------------------------------ */
struct f3 {
    float x, y, z;
};
__host__ __device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__host__ __device__ __forceinline__ f3 mk1(float a) { return f3{a, a, a}; }
__host__ __device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__host__ __device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__host__ __device__ __forceinline__ f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__host__ __device__ __forceinline__ f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
__host__ __device__ __forceinline__ f3 operator*(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
__host__ __device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
/* optix float3 / float = a * (1.0f / s) */
__host__ __device__ __forceinline__ f3 operator/(f3 a, float s) {
    float inv = 1.0f / s;
    return a * inv;
}
__host__ __device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__host__ __device__ __forceinline__ float length(f3 a) { return sqrtf(dot(a, a)); }
__host__ __device__ __forceinline__ f3 normalize(f3 a) {
    float inv = 1.0f / sqrtf(dot(a, a));
    return a * inv;
}
__host__ __device__ __forceinline__ float maxf(float a, float b) { return a > b ? a : b; }
__host__ __device__ __forceinline__ float fmax3(f3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
__host__ __device__ __forceinline__ float favgf(f3 v) { return (v.x + v.y + v.z) * 0.3333333333f; }
__host__ __device__ __forceinline__ f3 reflect(f3 i, f3 n) { return i - (n * 2.0f) * dot(n, i); }
__host__ __device__ __forceinline__ bool isnan3(f3 v) { return v.x != v.x || v.y != v.y || v.z != v.z; }

__host__ __device__ inline bool refract(f3& r, f3 i, f3 n, float ior) {
    f3 nn = n;
    float negNdotV = dot(i, nn);
    float eta;
    if (negNdotV > 0.0f) {
        eta = ior;
        nn = -n;
        negNdotV = -negNdotV;
    } else {
        eta = 1.f / ior;
    }
    const float k = 1.f - eta * eta * (1.f - negNdotV * negNdotV);
    if (k < 0.0f) {
        r = mk1(0.f);
        return false;
    }
    r = normalize(i * eta - nn * (eta * negNdotV + sqrtf(k)));
    return true;
}

/* ------------------------------------------------------------------ */
/* RadiancePRD flags (renderer/RadiancePRD.h:30-35)                    */
/* ------------------------------------------------------------------ */
constexpr uint32_t PRD_HIT_EMITTER = 1u << 31;
constexpr uint32_t PRD_ERROR = 1u << 30;
constexpr uint32_t PRD_MISS = 1u << 29;
constexpr uint32_t PRD_HIT_SPECULAR = 1u << 28;
constexpr uint32_t PRD_HIT_NON_SPECULAR = 1u << 27;
constexpr uint32_t PRD_PATH_TRACING = 1u << 26;
constexpr float RT_DEFAULT_MAX = 1.e27f;

/* ------------------------------------------------------------------ */
/* cuRAND XORWOW state, kept in registers; SoA planes in HBM           */
/* ------------------------------------------------------------------ */
struct Rng {
    uint32_t v0, v1, v2, v3, v4, d;
};
struct RngPlanes {
    uint32_t* p[6]; /* v0..v4, d : [slots] each, coalesced dword access */
};
__device__ __forceinline__ Rng rng_load(const RngPlanes& P, size_t s) {
    return Rng{P.p[0][s], P.p[1][s], P.p[2][s], P.p[3][s], P.p[4][s], P.p[5][s]};
}
__device__ __forceinline__ void rng_store(const RngPlanes& P, size_t s, const Rng& r) {
    P.p[0][s] = r.v0; P.p[1][s] = r.v1; P.p[2][s] = r.v2;
    P.p[3][s] = r.v3; P.p[4][s] = r.v4; P.p[5][s] = r.d;
}
/* curand_init(seed, 0, 0) — subsequence and offset 0: no skip-ahead */
__host__ __device__ __forceinline__ Rng rng_init(uint64_t seed) {
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    Rng r;
    r.d = 6615241u + t1 + t0;
    r.v0 = 123456789u + t0;
    r.v1 = 362436069u ^ t0;
    r.v2 = 521288629u + t1;
    r.v3 = 88675123u ^ t1;
    r.v4 = 5783321u + t0;
    return r;
}
__host__ __device__ __forceinline__ uint32_t rng_next(Rng& s) {
    uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}
/* getRandomUniformFloat (helpers/random.h:65-69): curand_uniform is
 * x*2^-32 + 2^-33 which nvcc contracts into one FMA. */
__device__ __forceinline__ float rnd(Rng& s) {
    uint32_t x = rng_next(s);
    float u = __builtin_fmaf((float)x, 2.3283064e-10f, 2.3283064e-10f / 2.0f);
    return maxf(u - ORX_FLT_EPSILON, 0.0f);
}

/* ------------------------------------------------------------------ */
/* samplers (helpers/samplers.h, helpers.h:119-134)                    */
/* ------------------------------------------------------------------ */
__device__ __forceinline__ void create_coordinate_system(f3 N, f3& U, f3& V) {
    if (fabsf(N.x) > fabsf(N.y)) {
        float invLength = 1.f / sqrtf(N.x * N.x + N.z * N.z);
        U = mk(-N.z * invLength, 0.f, N.x * invLength);
    } else {
        float invLength = 1.f / sqrtf(N.y * N.y + N.z * N.z);
        U = mk(0.f, N.z * invLength, -N.y * invLength);
    }
    V = cross(N, U);
}
/* sampleUnitHemisphereCos (samplers.h:24-43) */
__device__ __forceinline__ f3 sample_hemisphere_cos(f3 normal, float sx, float sy) {
    float theta = orx_acosf(sqrtf(sx));
    float phi = 2.0f * ORX_PI_F * sy;
    float st = orx_sinf(theta);
    float xs = st * orx_cosf(phi);
    float ys = orx_cosf(theta);
    float zs = st * orx_sinf(phi);
    f3 U, V;
    create_coordinate_system(normal, U, V);
    return normalize(U * xs + normal * ys + V * zs);
}
/* sampleUnitHemisphere (samplers.h:46-57) */
__device__ __forceinline__ f3 sample_hemisphere(f3 normal, float sx, float sy) {
    f3 U, V;
    create_coordinate_system(normal, U, V);
    float phi = 2.0f * ORX_PI_F * sx;
    float r = sqrtf(sy);
    float x = r * orx_cosf(phi);
    float y = r * orx_sinf(phi);
    float z = 1.0f - x * x - y * y;
    z = z > 0.0f ? sqrtf(z) : 0.0f;
    return normalize(U * x + V * y + normal * z);
}
/* sampleUnitSphere (samplers.h:59-72) */
__device__ __forceinline__ f3 sample_unit_sphere(float sx, float sy) {
    f3 v;
    v.z = 1.f - 2.f * sx;
    float phi = 2 * ORX_PI_F * sy;
    float r = sqrtf(1.f - v.z * v.z);
    v.x = r * orx_cosf(phi);
    v.y = r * orx_sinf(phi);
    return v;
}
/* sampleDisc (samplers.h:74-93) */
__device__ __forceinline__ f3 sample_disc(float sx, float sy, f3 center, float radius, f3 normal) {
    f3 U, V;
    create_coordinate_system(normal, U, V);
    float r = sqrtf(sx);
    float theta = 2.f * ORX_PI_F * sy;
    float x = r * orx_cosf(theta);
    float y = r * orx_sinf(theta);
    return center + (U * x + V * y) * radius;
}

/* ------------------------------------------------------------------ */
/* scene                                                               */
/* ------------------------------------------------------------------ */
enum : int32_t { MAT_DIFFUSE = 0, MAT_EMITTER = 1, MAT_MIRROR = 2, MAT_GLASS = 3, MAT_GLOSSY = 4, MAT_TEXTURE = 5 };
enum : int32_t { LIGHT_AREA = 0, LIGHT_POINT = 1, LIGHT_SPOT = 2 };

struct DevMaterial {
    int32_t type;
    f3 Kd, Ks, Kr, Kt;
    float ior, exponent;
    f3 powerPerArea, Lemit;
    float inverseArea;
    int32_t tex; /* Texture: index into DevScene::tex */
};
/* Texture images (material/Texture.cpp:83-107): RGBA8 texels in HBM */
struct DevTexture {
    const uint8_t* rgba;
    const uint8_t* nrgba; /* normal map or NULL */
    uint32_t w, h, nw, nh;
};
struct DevLight {
    int32_t type;
    f3 power, position, v1, v2, normal, Lemit; /* Lemit doubles as intensity */
    f3 direction;
    float area, inverseArea, angle;
};
/* parallelogram: plane (n,d), anchor, v1/|v1|^2, v2/|v2|^2 (Cornell.cpp:45-56) */
struct DevQuad {
    float nx, ny, nz, d;
    float ax, ay, az, v1x;
    float v1y, v1z, v2x, v2y;
    float v2z, pad0, pad1, pad2;
};
struct DevSphere {
    float cx, cy, cz, r;
};
/* Binary BVH node (host-side build only): 32 B, leaves hold a primitive range */
struct DevBvhNode {
    float lo[3];
    uint32_t left_or_first; /* inner: left child index; leaf: first prim in prim_index */
    float hi[3];
    uint32_t count_or_right; /* leaf: 0x80000000 | count; inner: right child */
};

/* Four-wide BVH node, 64 B (one 64-B segment, four dwordx4 loads), collapsed
 * from the binary SAH tree.  Child boxes are quantised to 8 bits per bound
 * against the node's origin with a power-of-two scale per axis, rounded
 * outward (so every decoded box contains the child's conservative box):
 *   lo_k(child i) = origin_k + qlo_k[i] * s_k,   s_k = 2^e_k
 * The scales are stored as floats (the x scale in the first 16 B, y and z in
 * the last), so the node test reads them instead of decoding exponent bytes.
 * Child reference: inner node index, or ORX_LEAF | first << 3 | (count - 1)
 * for a triangle range in leaf order, or ORX_EMPTY. */
struct DevBvh4 {
    float ox, oy, oz;
    float sx;          /* 2^e_x */
    uint32_t qlo[3];   /* per axis: byte i = child i */
    uint32_t qhi[3];
    uint32_t child[4];
    float sy, sz;      /* 2^e_y, 2^e_z */
};
/* fp32 variant (ORX_BVH_FP32): 128 B, child bounds unquantised, SoA by
 * axis so the near/far bound quadruples are picked by address */
struct DevBvh4F {
    float b[6][4];     /* lo_x, hi_x, lo_y, hi_y, lo_z, hi_z; [child] */
    uint32_t child[4];
    uint32_t pad[4];
};
#ifdef ORX_BVH_FP32
typedef DevBvh4F DevNode4;
#else
typedef DevBvh4 DevNode4;
#endif
constexpr uint32_t ORX_LEAF = 0x80000000u;
constexpr uint32_t ORX_EMPTY = 0xffffffffu;
constexpr uint32_t ORX_DONE = 0x7fffffffu; /* traversal sentinel: no node */

struct DevScene {
    uint32_t nq, ns, nt;
    const DevQuad* quads;
    const uint32_t* qmat;
    const DevSphere* spheres;
    const uint32_t* smat;
    /* triangles in BVH leaf order: tri_v[3k] = {p0.xyz, original triangle id bits},
     * tri_v[3k+1] = p1, tri_v[3k+2] = p2 (48 B per triangle, no index indirection) */
    const float4* tri_v;
    const float4* tri_n;       /* [nt][3] vertex normals in leaf order, or NULL */
    const float2* tri_uv;      /* [nt][3] texcoords in leaf order, or NULL (TriangleMesh.cu:74-84) */
    const float4* tri_t;       /* [nt][3] tangents, [nt][3] bitangents in leaf order, or NULL */
    const float4* tri_bt;
    const DevTexture* tex;
    uint32_t ntex;
    const uint32_t* tmat;      /* leaf order */
    const DevMaterial* mats;
    const DevLight* lights;
    uint32_t nl;
    /* bounding sphere (AAB::getBoundingSphere with Vector3::length bug) */
    float bs_cx, bs_cy, bs_cz, bs_r;
    /* triangle BVH4 (nt > 0); a traversal pushes at most stack_entries refs */
    const DevNode4* bvh4;
    uint32_t bvh_nodes;
    uint32_t stack_entries;
    unsigned long long* trav_stats; /* [16] in ORX_TRAV_STATS builds, else unused */
};

/* Traversal stack: per-lane column of a dynamic LDS array [stack_entries][64]
 * owned by a 64-thread (one-wave) block; entry k of a lane at s[k * 64].  The
 * depth bound is computed from the tree at orx_init_scene and the launch
 * passes ORX_STACK_BYTES(S) of dynamic LDS. */
#define ORX_BVH_STACK 32 /* depth cap of the binary build */
#define ORX_STACK_DECL extern __shared__ uint32_t orx_stack_lds[]
#define ORX_STACK_PTR (&orx_stack_lds[threadIdx.x & 63])
#define ORX_STACK_BYTES(S) ((size_t)((S).stack_entries + 2) * 64 * 4) /* + 2: StackL::put past the bound */

struct Hit {
    float t;
    int32_t prim;  /* global id: quads, spheres, triangles (original triangle order) */
    uint32_t slot; /* triangles: index in leaf order */
    float b, g;    /* triangle barycentrics */
    f3 sn;         /* sphere normal attribute */
};

/* parallelogram.cu:49-76 */
__device__ __forceinline__ bool isect_quad(const DevQuad& q, f3 o, f3 d, float tmin, float tmax, float& tout) {
    f3 n = mk(q.nx, q.ny, q.nz);
    float dt = dot(d, n);
    float t = (q.d - dot(n, o)) / dt;
    if (t > tmin && t < tmax) {
        f3 p = o + d * t;
        f3 vi = p - mk(q.ax, q.ay, q.az);
        float a1 = dot(mk(q.v1x, q.v1y, q.v1z), vi);
        if (a1 >= 0 && a1 <= 1) {
            float a2 = dot(mk(q.v2x, q.v2y, q.v2z), vi);
            if (a2 >= 0 && a2 <= 1) {
                tout = t;
                return true;
            }
        }
    }
    return false;
}
/* Sphere.cu:32-56 */
__device__ __forceinline__ bool isect_sphere(const DevSphere& s, f3 o, f3 d, float tmin, float tmax, float& tout,
                                             f3& nout) {
    f3 O = o - mk(s.cx, s.cy, s.cz);
    float b = dot(O, d);
    float c = dot(O, O) - s.r * s.r;
    float disc = b * b - c;
    if (disc > 0.0f) {
        float sdisc = sqrtf(disc);
        float root1 = (-b - sdisc);
        if (root1 > tmin && root1 < tmax) {
            tout = root1;
            nout = (O + d * root1) / s.r;
            return true;
        }
        float root2 = (-b + sdisc);
        if (root2 > tmin && root2 < tmax) {
            tout = root2;
            nout = (O + d * root2) / s.r;
            return true;
        }
    }
    return false;
}
/* OptiX intersect_triangle_branchless (TriangleMesh.cu:46) */
__device__ __forceinline__ bool isect_tri(f3 p0, f3 p1, f3 p2, f3 o, f3 d, float tmin, float tmax, float& tout,
                                          float& bout, float& gout) {
    f3 e0 = p1 - p0;
    f3 e1 = p0 - p2;
    f3 n = cross(e1, e0);
    f3 e2 = (p0 - o) * (1.0f / dot(n, d));
    f3 i = cross(d, e2);
    float beta = dot(i, e1);
    float gamma = dot(i, e0);
    float t = dot(n, e2);
    if ((t < tmax) & (t > tmin) & (beta >= 0.0f) & (gamma >= 0.0f) & (beta + gamma <= 1)) {
        tout = t;
        bout = beta;
        gout = gamma;
        return true;
    }
    return false;
}
__device__ __forceinline__ f3 ld_f3(const float4& v) { return mk(v.x, v.y, v.z); }

/* Per-ray slab-test constants.  A zero direction component is replaced by
 * +-1e-30 for the box tests only: the tilted ray leaves a conservative box
 * (>= 1e-20 margin, see the builder) only beyond t = 1e10, so no box the exact
 * ray reaches is culled; the triangle tests use the exact direction. */
struct RayBox {
    f3 o, inv;
    bool nx, ny, nz; /* negative direction: the near slab of that axis is the box's hi bound */
    f3 oinv;         /* -o * inv (fp32 boxes: t = fma(bound, inv, oinv)) */
};
__device__ __forceinline__ RayBox ray_box(f3 o, f3 d) {
    auto safe = [](float v) { return fabsf(v) > 1e-30f ? v : copysignf(1e-30f, v); };
    RayBox rb;
    rb.o = o;
    /* v_rcp_f32 (1 ulp): the builder's 1e-6 relative box expansion covers it */
    rb.inv = mk(__builtin_amdgcn_rcpf(safe(d.x)), __builtin_amdgcn_rcpf(safe(d.y)), __builtin_amdgcn_rcpf(safe(d.z)));
    rb.nx = rb.inv.x < 0.f;
    rb.ny = rb.inv.y < 0.f;
    rb.nz = rb.inv.z < 0.f;
    rb.oinv = mk(-o.x * rb.inv.x, -o.y * rb.inv.y, -o.z * rb.inv.z);
    return rb;
}
/* Test the four quantised child boxes of a node against (tmin, tmax):
 * t = (origin + q*s - o) * inv evaluated as fma(q, s*inv, (origin - o)*inv);
 * the rounding of that form is far below the builder's 1e-6 relative box
 * expansion, so the test stays conservative.  The near/far bound of each
 * axis is picked once per node from the ray's direction signs, so a child
 * costs 6 fma + 4 min/max (identical values to the min/max slab form).
 * Returns entry distances (+inf for misses) and child refs. */
__device__ __forceinline__ void node_test_q(const float4 A, const float4 B, const float4 C, const float4 D,
                                            const RayBox& rb, float tmin, float tmax, float t[4], uint32_t c[4]) {
    const float sx = A.w, sy = D.z, sz = D.w;
    const float ax = (A.x - rb.o.x) * rb.inv.x, bx = sx * rb.inv.x;
    const float ay = (A.y - rb.o.y) * rb.inv.y, by = sy * rb.inv.y;
    const float az = (A.z - rb.o.z) * rb.inv.z, bz = sz * rb.inv.z;
    const uint32_t lx = __float_as_uint(B.x), ly = __float_as_uint(B.y), lz = __float_as_uint(B.z);
    const uint32_t hx = __float_as_uint(B.w), hy = __float_as_uint(C.x), hz = __float_as_uint(C.y);
    const uint32_t nxq = rb.nx ? hx : lx, fxq = rb.nx ? lx : hx;
    const uint32_t nyq = rb.ny ? hy : ly, fyq = rb.ny ? ly : hy;
    const uint32_t nzq = rb.nz ? hz : lz, fzq = rb.nz ? lz : hz;
    c[0] = __float_as_uint(C.z);
    c[1] = __float_as_uint(C.w);
    c[2] = __float_as_uint(D.x);
    c[3] = __float_as_uint(D.y);
    /* two children per v_pk_fma_f32 */
    typedef float v2q __attribute__((ext_vector_type(2)));
    auto q2 = [](uint32_t w, int i) {
        return v2q{(float)((w >> (8 * i)) & 0xffu), (float)((w >> (8 * i + 8)) & 0xffu)};
    };
    const v2q ax2 = v2q{ax, ax}, bx2 = v2q{bx, bx}, ay2 = v2q{ay, ay}, by2 = v2q{by, by};
    const v2q az2 = v2q{az, az}, bz2 = v2q{bz, bz};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const v2q tnx = __builtin_elementwise_fma(q2(nxq, 2 * h), bx2, ax2);
        const v2q tfx = __builtin_elementwise_fma(q2(fxq, 2 * h), bx2, ax2);
        const v2q tny = __builtin_elementwise_fma(q2(nyq, 2 * h), by2, ay2);
        const v2q tfy = __builtin_elementwise_fma(q2(fyq, 2 * h), by2, ay2);
        const v2q tnz = __builtin_elementwise_fma(q2(nzq, 2 * h), bz2, az2);
        const v2q tfz = __builtin_elementwise_fma(q2(fzq, 2 * h), bz2, az2);
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const int i = 2 * h + e;
            const float t0 = fmaxf(fmaxf(fmaxf(tnx[e], tny[e]), tnz[e]), tmin);
            const float t1 = fminf(fminf(fminf(tfx[e], tfy[e]), tfz[e]), tmax);
            t[i] = t0 <= t1 ? t0 : INFINITY; /* an empty slot holds an empty box (lo 255 > hi 0) */
        }
    }
}
/* Node and triangle loads are buffer loads: one 32-bit byte offset per lane (a shift, where a
 * 64-bit address costs two 64-bit VALU operations), the resource in SGPRs.  orx_init_scene keeps
 * the node and triangle arrays below 4 GiB. */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t orx_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0xffffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t bo) {
    typedef uint32_t u4b __attribute__((ext_vector_type(4)));
    const u4b v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)bo, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ void node_test(const DevBvh4* nodes, uint32_t idx, const RayBox& rb, float tmin, float tmax,
                                          float t[4], uint32_t c[4]) {
    const __amdgpu_buffer_rsrc_t r = orx_rsrc(nodes);
    const uint32_t bo = idx << 6;
    node_test_q(ld16(r, bo), ld16(r, bo + 16), ld16(r, bo + 32), ld16(r, bo + 48), rb, tmin, tmax, t, c);
}
typedef float v2t __attribute__((ext_vector_type(2)));
/* fp32-box node test: t = fma(bound, inv, -o*inv), two children per
 * v_pk_fma_f32; same conservativeness argument as the quantised form */
__device__ __forceinline__ void node_test(const DevBvh4F* nodes, uint32_t idx, const RayBox& rb, float tmin, float tmax,
                                          float t[4], uint32_t c[4]) {
    const float* base = reinterpret_cast<const float*>(nodes + idx);
    const float4 NX = *(const float4*)(base + (rb.nx ? 4 : 0)), FX = *(const float4*)(base + (rb.nx ? 0 : 4));
    const float4 NY = *(const float4*)(base + (rb.ny ? 12 : 8)), FY = *(const float4*)(base + (rb.ny ? 8 : 12));
    const float4 NZ = *(const float4*)(base + (rb.nz ? 20 : 16)), FZ = *(const float4*)(base + (rb.nz ? 16 : 20));
    const uint4 CC = *(const uint4*)(base + 24);
    c[0] = CC.x;
    c[1] = CC.y;
    c[2] = CC.z;
    c[3] = CC.w;
    const v2t ix = v2t{rb.inv.x, rb.inv.x}, iy = v2t{rb.inv.y, rb.inv.y}, iz = v2t{rb.inv.z, rb.inv.z};
    const v2t ox = v2t{rb.oinv.x, rb.oinv.x}, oy = v2t{rb.oinv.y, rb.oinv.y}, oz = v2t{rb.oinv.z, rb.oinv.z};
    const v2t tnx0 = __builtin_elementwise_fma(v2t{NX.x, NX.y}, ix, ox), tnx1 = __builtin_elementwise_fma(v2t{NX.z, NX.w}, ix, ox);
    const v2t tfx0 = __builtin_elementwise_fma(v2t{FX.x, FX.y}, ix, ox), tfx1 = __builtin_elementwise_fma(v2t{FX.z, FX.w}, ix, ox);
    const v2t tny0 = __builtin_elementwise_fma(v2t{NY.x, NY.y}, iy, oy), tny1 = __builtin_elementwise_fma(v2t{NY.z, NY.w}, iy, oy);
    const v2t tfy0 = __builtin_elementwise_fma(v2t{FY.x, FY.y}, iy, oy), tfy1 = __builtin_elementwise_fma(v2t{FY.z, FY.w}, iy, oy);
    const v2t tnz0 = __builtin_elementwise_fma(v2t{NZ.x, NZ.y}, iz, oz), tnz1 = __builtin_elementwise_fma(v2t{NZ.z, NZ.w}, iz, oz);
    const v2t tfz0 = __builtin_elementwise_fma(v2t{FZ.x, FZ.y}, iz, oz), tfz1 = __builtin_elementwise_fma(v2t{FZ.z, FZ.w}, iz, oz);
    const float tn[4][3] = {{tnx0.x, tny0.x, tnz0.x}, {tnx0.y, tny0.y, tnz0.y}, {tnx1.x, tny1.x, tnz1.x}, {tnx1.y, tny1.y, tnz1.y}};
    const float tf[4][3] = {{tfx0.x, tfy0.x, tfz0.x}, {tfx0.y, tfy0.y, tfz0.y}, {tfx1.x, tfy1.x, tfz1.x}, {tfx1.y, tfy1.y, tfz1.y}};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float t0 = fmaxf(fmaxf(fmaxf(tn[i][0], tn[i][1]), tn[i][2]), tmin);
        const float t1 = fminf(fminf(fminf(tf[i][0], tf[i][1]), tf[i][2]), tmax);
        t[i] = (t0 <= t1 && c[i] != 0xffffffffu) ? t0 : INFINITY;
    }
}
/* compare-exchange by entry distance; the distances by min/max (never NaN here: +inf or a
 * max with tmin), which leaves the compare's mask to the two reference selects */
__device__ __forceinline__ void cswap(float& ta, uint32_t& ca, float& tb, uint32_t& cb) {
    /* the distances are >= tmin >= 0 or +inf, so their bit patterns order like the values: unsigned
     * compare and min/max (fminf/fmaxf had cost two NaN-quieting v_max_f32 per exchange) */
    const uint32_t ua = __float_as_uint(ta), ub = __float_as_uint(tb);
    const bool sw = ub < ua;
    const uint32_t c = sw ? cb : ca;
    cb = sw ? ca : cb;
    ca = c;
    ta = __uint_as_float(ua < ub ? ua : ub);
    tb = __uint_as_float(ua < ub ? ub : ua);
}

/* Traversal policies (trace_closest_t / trace_any_t): the stack (StackL: the
 * lane's column of the dynamic-LDS array [stack_entries][64]; StackH below) and the
 * node source (NodesG: S.bvh4).  Measured and dropped: the top 85 / 341 nodes in LDS
 * (DESIGN.md §4). */
struct StackL {
    uint32_t* s;
    __device__ __forceinline__ void push(int& sp, uint32_t v) const { s[(sp++) * 64] = v; }
    __device__ __forceinline__ uint32_t pop(int& sp) const { return s[(--sp) * 64]; }
    /* write entry k without moving the stack pointer (k may run two past the bound) */
    __device__ __forceinline__ void put(int k, uint32_t v) const { s[k * 64] = v; }
    /* the whole stack is in LDS: every wave is shallow */
    __device__ __forceinline__ bool shallow(int, int) const { return true; }
    __device__ __forceinline__ void put_l(int k, uint32_t v) const { put(k, v); }
    __device__ __forceinline__ uint32_t pop_l(int& sp) const { return pop(sp); }
};
/* A short LDS stack continued in global memory: entries k < NL in the lane's LDS column, deeper
 * ones in the block's own global array [depth][64] at column `lane` (g_ = the block's base, so the
 * 32-bit buffer offsets stay below depth * 256 B whatever the launch size), through buffer
 * loads/stores (kept apart from the LDS accesses, which the compiler would otherwise merge with
 * them into flat loads).  The LDS column holds NL + 1 entries: a push always writes LDS, at min(k, NL) (entry
 * NL is a dump slot), and only a push or pop past NL takes the branch to global memory.  The traversal
 * loops test once per node step whether any lane of the wave could pass NL (shallow(): one ballot) and
 * otherwise push and pop through put_l / pop_l, LDS only, without the clamp and the per-entry branch
 * (hall photon pass 3.555 -> 3.494 ms serial, frame +1.1 %, profiles/r06za_stack_fast_path_ab.txt).  For kernels whose occupancy
 * the full-depth LDS stack limits (k_vcm_shadow: 61 VGPRs, 4 waves per SIMD with 35 LDS entries,
 * 8 with 16; k_ppm_photon). */
template <int NL>
struct StackH {
    uint32_t* s;
    __amdgpu_buffer_rsrc_t g;
    uint32_t lane;
    static constexpr uint32_t gstride = 64;
    static constexpr size_t lds_bytes() { return (size_t)(NL + 1) * 64 * 4; }
    /* global entries per lane for a tree whose stack bound is `entries` (the pushes run two past it) */
    __host__ __device__ static constexpr uint32_t deep(uint32_t entries) { return entries + 2 > NL ? entries + 2 - NL : 1u; }
    /* g_: the buffer of every block's [deep][64] entries, block `blk`'s part is used */
    __device__ __forceinline__ StackH(uint32_t* s_, uint32_t* g_, uint32_t blk, uint32_t ndeep, uint32_t lane_)
        : s(s_), g(__builtin_amdgcn_make_buffer_rsrc(g_ + (size_t)blk * ndeep * 64u, 0, ndeep * 256u, 0x00020000)),
          lane(lane_) {}
    __device__ __forceinline__ void push(int& sp, uint32_t v) const { put(sp++, v); }
    __device__ __forceinline__ uint32_t pop(int& sp) const {
        --sp;
        uint32_t v = s[(sp < NL ? sp : NL) * 64];
        if (sp >= NL) v = __builtin_amdgcn_raw_buffer_load_b32(g, (int)(((uint32_t)(sp - NL) * gstride + lane) * 4u), 0, 0);
        return v;
    }
    __device__ __forceinline__ void put(int k, uint32_t v) const {
        s[(k < NL ? k : NL) * 64] = v;
        if (k >= NL) __builtin_amdgcn_raw_buffer_store_b32(v, g, (int)(((uint32_t)(k - NL) * gstride + lane) * 4u), 0, 0);
    }
    /* wave-uniform: no lane's next `n` entries (from sp) reach past the LDS column, so put_l / pop_l
     * (LDS only, no clamp and no per-entry branch to global memory) serve this step */
    __device__ __forceinline__ bool shallow(int sp, int n) const { return !__ballot(sp + n > NL); }
    __device__ __forceinline__ void put_l(int k, uint32_t v) const { s[k * 64] = v; }
    __device__ __forceinline__ uint32_t pop_l(int& sp) const { return s[(--sp) * 64]; }
};
struct NodesG {
    __device__ __forceinline__ void test(const DevScene& S, uint32_t idx, const RayBox& rb, float tmin, float tmax,
                                         float t[4], uint32_t c[4]) const {
        node_test(S.bvh4, idx, rb, tmin, tmax, t, c);
    }
};

/* Optional traversal statistics (build with -DORX_TRAV_STATS): rays, inner
 * nodes visited, leaves visited, triangle tests — per ray type (closest/any). */
#ifdef ORX_TRAV_STATS
#define ORX_TS_DECL uint32_t ts_nodes = 0, ts_leaves = 0, ts_tris = 0, ts_wn = 0, ts_wl = 0
#define ORX_TS_INC(v, n) (v) += (n)
/* wave-level loop iterations: counted by the wave's first active lane */
#define ORX_TS_WAVE(v) (v) += ((uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1) == (threadIdx.x & 63u))
#define ORX_TS_DECL_TOP uint32_t ts_top[4] = {0, 0, 0, 0}
#define ORX_TS_TOP(idx)                                                     \
    do {                                                                    \
        ts_top[0] += (idx) < 21u;                                           \
        ts_top[1] += (idx) < 85u;                                           \
        ts_top[2] += (idx) < 341u;                                          \
        ts_top[3] += (idx) < 1365u;                                         \
    } while (0)
#define ORX_TS_FLUSH_TOP()                                                  \
    do {                                                                    \
        for (int q_ = 0; q_ < 4; q_++) atomicAdd(&S.trav_stats[16 + q_], (unsigned long long)ts_top[q_]); \
    } while (0)
#define ORX_TS_FLUSH(base)                                                  \
    do {                                                                    \
        atomicAdd(&S.trav_stats[(base) + 0], 1ull);                       \
        atomicAdd(&S.trav_stats[(base) + 1], (unsigned long long)ts_nodes);  \
        atomicAdd(&S.trav_stats[(base) + 2], (unsigned long long)ts_leaves); \
        atomicAdd(&S.trav_stats[(base) + 3], (unsigned long long)ts_tris);   \
        atomicAdd(&S.trav_stats[8 + (base) / 2], (unsigned long long)ts_wn);  \
        atomicAdd(&S.trav_stats[9 + (base) / 2], (unsigned long long)ts_wl);  \
    } while (0)
#else
#define ORX_TS_DECL
#define ORX_TS_DECL_TOP
#define ORX_TS_TOP(idx)
#define ORX_TS_FLUSH_TOP()
#define ORX_TS_INC(v, n)
#define ORX_TS_WAVE(v)
#define ORX_TS_FLUSH(base)
#endif

/* Closest hit over all primitives; equal t resolves to the lowest global
 * primitive id, which is OptiX NoAccel's child order (Cornell.cpp:183-189)
 * and is independent of traversal order, so BVH and brute force agree.
 * Triangles: near-first BVH4 traversal; the hit children of a node are
 * sorted by entry distance, the nearest is taken and the others are pushed
 * far-to-near on the lane's LDS stack. */
template <class STK, class NODES>
__device__ inline bool trace_closest_t(const DevScene& S, f3 o, f3 d, float tmin, float tmax, Hit& h, const STK& stk,
                                       const NODES& nodes) {
    float best = tmax;
    int32_t bp = -1;
    uint32_t bslot = 0;
    float t;
    for (uint32_t i = 0; i < S.nq; i++) {
        if (isect_quad(S.quads[i], o, d, tmin, best, t)) {
            best = t;
            bp = (int32_t)i;
        }
    }
    f3 sn = mk1(0);
    for (uint32_t i = 0; i < S.ns; i++) {
        f3 n;
        if (isect_sphere(S.spheres[i], o, d, tmin, best, t, n)) {
            best = t;
            bp = (int32_t)(S.nq + i);
            sn = n;
        }
    }
    float bb = 0, bg = 0;
    if (S.nt) {
        const uint32_t base = S.nq + S.ns;
        const RayBox rb = ray_box(o, d);
        int sp = 0;
        uint32_t ref = 0; /* root */
        ORX_TS_DECL;
        ORX_TS_DECL_TOP;
        /* speculative while-while (Aila & Laine 2009): a lane that reaches a
         * leaf postpones it and keeps descending until every lane of the wave
         * holds a leaf, then all process theirs together */
        uint32_t lf = 0; /* postponed leaf, or a non-leaf value for none */
        while (ref != ORX_DONE) {
            while (!(ref & ORX_LEAF) && ref != ORX_DONE) {
                float ct[4];
                uint32_t cc[4];
                nodes.test(S, ref, rb, tmin, best, ct, cc);
                ORX_TS_INC(ts_nodes, 1);
                ORX_TS_TOP(ref);
                ORX_TS_WAVE(ts_wn);
                cswap(ct[0], cc[0], ct[1], cc[1]);
                cswap(ct[2], cc[2], ct[3], cc[3]);
                cswap(ct[0], cc[0], ct[2], cc[2]);
                cswap(ct[1], cc[1], ct[3], cc[3]);
                cswap(ct[1], cc[1], ct[2], cc[2]);
                /* (dropping the last two exchanges, a near-first order only for the first
                 * child, measured 4.03 -> 4.29 ms on the hall photon pass: order matters) */
                {
                    /* branch-free pushes: the three entries are written unconditionally at
                     * their final positions (misses sort last), then the pointer moves by the
                     * hits (photon pass 4.03 -> 3.98 ms against one branch per push) */
                    const int n3 = ct[3] != INFINITY, n2 = ct[2] != INFINITY, n1 = ct[1] != INFINITY;
                    if (stk.shallow(sp, 3)) { /* the common case: the three entries in LDS */
                        stk.put_l(sp, cc[3]);
                        stk.put_l(sp + n3, cc[2]);
                        stk.put_l(sp + n3 + n2, cc[1]);
                        sp += n3 + n2 + n1;
                        ref = ct[0] != INFINITY ? cc[0] : (sp ? stk.pop_l(sp) : ORX_DONE);
                    } else {
                        stk.put(sp, cc[3]);
                        stk.put(sp + n3, cc[2]);
                        stk.put(sp + n3 + n2, cc[1]);
                        sp += n3 + n2 + n1;
                        ref = ct[0] != INFINITY ? cc[0] : (sp ? stk.pop(sp) : ORX_DONE);
                    }
                }
                if ((ref & ORX_LEAF) && !(lf & ORX_LEAF)) {
                    lf = ref;
                    ref = sp ? stk.pop(sp) : ORX_DONE;
                }
                if (!__ballot(!(lf & ORX_LEAF))) break;
            }
            while (lf & ORX_LEAF) {
                const uint32_t first = (lf & 0x7fffffffu) >> 3, cnt = (lf & 7u) + 1u;
                ORX_TS_INC(ts_leaves, 1);
                ORX_TS_INC(ts_tris, cnt);
                ORX_TS_WAVE(ts_wl);
                const __amdgpu_buffer_rsrc_t tr = orx_rsrc(S.tri_v);
                for (uint32_t k = first; k < first + cnt; k++) {
                    const uint32_t tb = k * 48u;
                    const float4 v0 = ld16(tr, tb), v1 = ld16(tr, tb + 16), v2 = ld16(tr, tb + 32);
                    const int32_t gid = (int32_t)(base + __float_as_uint(v0.w));
                    float b, g;
                    /* accept t < best, or t == best from a lower primitive id */
                    float lim = bp >= 0 ? orx_as_float(orx_as_uint(best) + 1u) : best;
                    if (isect_tri(ld_f3(v0), ld_f3(v1), ld_f3(v2), o, d, tmin, lim, t, b, g) &&
                        (t < best || gid < bp)) {
                        best = t;
                        bp = gid;
                        bslot = k;
                        bb = b;
                        bg = g;
                    }
                }
                lf = ref; /* another leaf postponed behind it: process it too */
                if (ref & ORX_LEAF) ref = sp ? stk.pop(sp) : ORX_DONE;
            }
        }
        ORX_TS_FLUSH(0);
        ORX_TS_FLUSH_TOP();
    }
    if (bp < 0) return false;
    h.t = best;
    h.prim = bp;
    h.slot = bslot;
    h.b = bb;
    h.g = bg;
    h.sn = sn;
    return true;
}
__device__ __forceinline__ bool trace_closest(const DevScene& S, f3 o, f3 d, float tmin, float tmax, Hit& h,
                                              uint32_t* stk) {
    return trace_closest_t(S, o, d, tmin, tmax, h, StackL{stk}, NodesG{});
}

/* any hit in (tmin,tmax): every material's RayType::SHADOW any-hit is
 * gatherAnyHitOnNonEmitter (Material.cpp:18-26, DirectRadianceEstimation.cu:79-83) */
template <class STK, class NODES>
__device__ inline bool trace_any_t(const DevScene& S, f3 o, f3 d, float tmin, float tmax, const STK& stk,
                                   const NODES& nodes) {
    float t;
    for (uint32_t i = 0; i < S.nq; i++)
        if (isect_quad(S.quads[i], o, d, tmin, tmax, t)) return true;
    for (uint32_t i = 0; i < S.ns; i++) {
        f3 n;
        if (isect_sphere(S.spheres[i], o, d, tmin, tmax, t, n)) return true;
    }
    if (S.nt) {
        const RayBox rb = ray_box(o, d);
        int sp = 0;
        uint32_t ref = 0;
        ORX_TS_DECL;
        uint32_t lf = 0; /* speculative while-while, as trace_closest */
        while (ref != ORX_DONE) {
            while (!(ref & ORX_LEAF) && ref != ORX_DONE) {
                float ct[4];
                uint32_t cc[4];
                nodes.test(S, ref, rb, tmin, tmax, ct, cc);
                ORX_TS_INC(ts_nodes, 1);
                ORX_TS_WAVE(ts_wn);
                /* branch-free: every hit child is written to the stack (the order does not
                 * matter for any hit), the last one is taken back from registers */
                const int h0 = ct[0] != INFINITY, h1 = ct[1] != INFINITY, h2 = ct[2] != INFINITY,
                          h3 = ct[3] != INFINITY;
                const uint32_t next = h3 ? cc[3] : h2 ? cc[2] : h1 ? cc[1] : h0 ? cc[0] : ORX_DONE;
                if (stk.shallow(sp, 4)) { /* the common case: the four entries in LDS */
                    stk.put_l(sp, cc[0]);
                    sp += h0;
                    stk.put_l(sp, cc[1]);
                    sp += h1;
                    stk.put_l(sp, cc[2]);
                    sp += h2;
                    stk.put_l(sp, cc[3]);
                    sp += h3;
                    sp -= next != ORX_DONE;
                    ref = next != ORX_DONE ? next : (sp ? stk.pop_l(sp) : ORX_DONE);
                } else {
                    stk.put(sp, cc[0]);
                    sp += h0;
                    stk.put(sp, cc[1]);
                    sp += h1;
                    stk.put(sp, cc[2]);
                    sp += h2;
                    stk.put(sp, cc[3]);
                    sp += h3;
                    sp -= next != ORX_DONE;
                    ref = next != ORX_DONE ? next : (sp ? stk.pop(sp) : ORX_DONE);
                }
                if ((ref & ORX_LEAF) && !(lf & ORX_LEAF)) {
                    lf = ref;
                    ref = sp ? stk.pop(sp) : ORX_DONE;
                }
                if (!__ballot(!(lf & ORX_LEAF))) break;
            }
            while (lf & ORX_LEAF) {
                const uint32_t first = (lf & 0x7fffffffu) >> 3, cnt = (lf & 7u) + 1u;
                ORX_TS_INC(ts_leaves, 1);
                ORX_TS_WAVE(ts_wl);
                const __amdgpu_buffer_rsrc_t tr = orx_rsrc(S.tri_v);
                for (uint32_t k = first; k < first + cnt; k++) {
                    float b, g;
                    ORX_TS_INC(ts_tris, 1);
                    const uint32_t tb = k * 48u;
                    if (isect_tri(ld_f3(ld16(tr, tb)), ld_f3(ld16(tr, tb + 16)), ld_f3(ld16(tr, tb + 32)), o, d,
                                  tmin, tmax, t, b, g)) {
                        ORX_TS_FLUSH(4);
                        return true;
                    }
                }
                lf = ref;
                if (ref & ORX_LEAF) ref = sp ? stk.pop(sp) : ORX_DONE;
            }
        }
        ORX_TS_FLUSH(4);
    }
    return false;
}

__device__ __forceinline__ bool trace_any(const DevScene& S, f3 o, f3 d, float tmin, float tmax, uint32_t* stk) {
    return trace_any_t(S, o, d, tmin, tmax, StackL{stk}, NodesG{});
}

/* Several shadow rays per lane in one traversal loop: a lane whose ray has ended (occluder found,
 * or stack empty) starts its next ray at once instead of waiting for the slowest lane of the wave
 * to finish the current one, so a wave runs for the maximum over its lanes of their summed walks,
 * not for the sum over the rays of the slowest walk.  Each ray's own test sequence is trace_any's
 * (the same result, occluded or not).  RAYS supplies the lane's rays in order:
 *   bool next(f3& o, f3& d, float& tmin, float& tmax)  — false when the lane has no more;
 *   void result(bool occluded)                          — the outcome of the ray `next` gave last. */
template <class RAYS, class STK>
__device__ __forceinline__ void trace_any_chain_t(const DevScene& S, RAYS& R, const STK& stk) {
    f3 o = mk1(0.f), d = mk1(0.f);
    float tmin = 0.f, tmax = 0.f;
    RayBox rb = ray_box(o, mk1(1.f));
    int sp = 0;
    uint32_t ref = ORX_DONE, lf = 0;
    /* the lane's next ray that needs a BVH walk (quad and sphere hits, and scenes without
     * triangles, are decided here) */
    auto fetch = [&]() -> bool {
        while (R.next(o, d, tmin, tmax)) {
            float t;
            bool hit = false;
            for (uint32_t i = 0; i < S.nq && !hit; i++) hit = isect_quad(S.quads[i], o, d, tmin, tmax, t);
            for (uint32_t i = 0; i < S.ns && !hit; i++) {
                f3 n;
                hit = isect_sphere(S.spheres[i], o, d, tmin, tmax, t, n);
            }
            if (hit || !S.nt) {
                R.result(hit);
                continue;
            }
            rb = ray_box(o, d);
            sp = 0;
            ref = 0;
            lf = 0;
            return true;
        }
        return false;
    };
    bool have = fetch();
    const __amdgpu_buffer_rsrc_t tr = orx_rsrc(S.tri_v);
    while (__ballot(have)) {
        if (!have) continue;
        /* one round of trace_any_t's speculative while-while */
        while (!(ref & ORX_LEAF) && ref != ORX_DONE) {
            float ct[4];
            uint32_t cc[4];
            node_test(S.bvh4, ref, rb, tmin, tmax, ct, cc);
            const int h0 = ct[0] != INFINITY, h1 = ct[1] != INFINITY, h2 = ct[2] != INFINITY, h3 = ct[3] != INFINITY;
            const uint32_t next = h3 ? cc[3] : h2 ? cc[2] : h1 ? cc[1] : h0 ? cc[0] : ORX_DONE;
            if (stk.shallow(sp, 4)) { /* the common case: the four entries in LDS */
                stk.put_l(sp, cc[0]);
                sp += h0;
                stk.put_l(sp, cc[1]);
                sp += h1;
                stk.put_l(sp, cc[2]);
                sp += h2;
                stk.put_l(sp, cc[3]);
                sp += h3;
                sp -= next != ORX_DONE;
                ref = next != ORX_DONE ? next : (sp ? stk.pop_l(sp) : ORX_DONE);
            } else {
                stk.put(sp, cc[0]);
                sp += h0;
                stk.put(sp, cc[1]);
                sp += h1;
                stk.put(sp, cc[2]);
                sp += h2;
                stk.put(sp, cc[3]);
                sp += h3;
                sp -= next != ORX_DONE;
                ref = next != ORX_DONE ? next : (sp ? stk.pop(sp) : ORX_DONE);
            }
            if ((ref & ORX_LEAF) && !(lf & ORX_LEAF)) {
                lf = ref;
                ref = sp ? stk.pop(sp) : ORX_DONE;
            }
            if (!__ballot(!(lf & ORX_LEAF))) break;
        }
        bool occl = false;
        while ((lf & ORX_LEAF) && !occl) {
            const uint32_t first = (lf & 0x7fffffffu) >> 3, cnt = (lf & 7u) + 1u;
            for (uint32_t k = first; k < first + cnt && !occl; k++) {
                float t, b, g;
                const uint32_t tb = k * 48u;
                occl = isect_tri(ld_f3(ld16(tr, tb)), ld_f3(ld16(tr, tb + 16)), ld_f3(ld16(tr, tb + 32)), o, d, tmin,
                                 tmax, t, b, g);
            }
            if (!occl) {
                lf = ref;
                if (ref & ORX_LEAF) ref = sp ? stk.pop(sp) : ORX_DONE;
            }
        }
        if (occl || ref == ORX_DONE) {
            R.result(occl);
            have = fetch();
        }
    }
}
template <class RAYS>
__device__ __forceinline__ void trace_any_chain(const DevScene& S, RAYS& R, uint32_t* stkp) {
    trace_any_chain_t(S, R, StackL{stkp});
}

__device__ __forceinline__ uint32_t prim_material(const DevScene& S, const Hit& h) {
    if ((uint32_t)h.prim < S.nq) return S.qmat[h.prim];
    if ((uint32_t)h.prim < S.nq + S.ns) return S.smat[h.prim - S.nq];
    return S.tmat[h.slot];
}
/* world shading normal as the closest-hit programs see it:
 * normalize(rtTransformNormal(shadingNormal)) with identity transforms. */
__device__ __forceinline__ f3 shading_normal(const DevScene& S, const Hit& h) {
    if ((uint32_t)h.prim < S.nq) {
        const DevQuad& q = S.quads[h.prim];
        return normalize(mk(q.nx, q.ny, q.nz));
    }
    if ((uint32_t)h.prim < S.nq + S.ns) return normalize(h.sn);
    const uint32_t ti = h.slot;
    if (S.tri_n) {
        f3 n0 = ld_f3(S.tri_n[3 * ti]), n1 = ld_f3(S.tri_n[3 * ti + 1]), n2 = ld_f3(S.tri_n[3 * ti + 2]);
        return normalize(normalize(n1 * h.b + n2 * h.g + n0 * (1.0f - h.b - h.g)));
    }
    f3 p0 = ld_f3(S.tri_v[3 * ti]), p1 = ld_f3(S.tri_v[3 * ti + 1]), p2 = ld_f3(S.tri_v[3 * ti + 2]);
    return normalize(normalize(cross(p0 - p2, p1 - p0)));
}
/* geometric normal as the VCM closest-hit programs see it */
__device__ __forceinline__ f3 geometric_normal(const DevScene& S, const Hit& h) {
    if ((uint32_t)h.prim < S.nq) {
        const DevQuad& q = S.quads[h.prim];
        return normalize(mk(q.nx, q.ny, q.nz));
    }
    if ((uint32_t)h.prim < S.nq + S.ns) return normalize(h.sn);
    const uint32_t ti = h.slot;
    f3 p0 = ld_f3(S.tri_v[3 * ti]), p1 = ld_f3(S.tri_v[3 * ti + 1]), p2 = ld_f3(S.tri_v[3 * ti + 2]);
    return normalize(normalize(cross(p0 - p2, p1 - p0)));
}

/* Texture attributes (TriangleMesh.cu:61-84); parallelograms and spheres
 * write no textureCoordinate / tangent attributes: (0,0), no normal map. */
__device__ __forceinline__ void hit_texcoord(const DevScene& S, const Hit& h, float& u, float& v) {
    u = 0.f;
    v = 0.f;
    if ((uint32_t)h.prim < S.nq + S.ns || !S.tri_uv) return;
    const float2 t0 = S.tri_uv[3 * h.slot], t1 = S.tri_uv[3 * h.slot + 1], t2 = S.tri_uv[3 * h.slot + 2];
    const float w0 = 1.0f - h.b - h.g;
    u = (t1.x * h.b + t2.x * h.g) + t0.x * w0;
    v = (t1.y * h.b + t2.y * h.g) + t0.y * w0;
}
/* tex2D(diffuseSampler, textureCoordinate).xyz (Texture.cu:107-109) */
__device__ inline f3 tex_color(const DevScene& S, const DevMaterial& m, const Hit& h) {
    const DevTexture& t = S.tex[m.tex];
    float u, v, c[4];
    hit_texcoord(S, h, u, v);
    orx_tex2d_linear(t.rgba, t.w, t.h, u, v, c);
    return mk(c[0], c[1], c[2]);
}
/* getNormalMappedNormal when hasNormals (Texture.cu:69-77, :88-95) */
__device__ inline f3 tex_normal(const DevScene& S, const DevMaterial& m, const Hit& h, f3 wsn) {
    const DevTexture& t = S.tex[m.tex];
    if (!t.nrgba || !S.tri_n || !S.tri_t || (uint32_t)h.prim < S.nq + S.ns) return wsn;
    const uint32_t k = 3 * h.slot;
    const float w0 = 1.0f - h.b - h.g;
    f3 T = normalize(ld_f3(S.tri_t[k + 1]) * h.b + ld_f3(S.tri_t[k + 2]) * h.g + ld_f3(S.tri_t[k]) * w0);
    f3 B = normalize(ld_f3(S.tri_bt[k + 1]) * h.b + ld_f3(S.tri_bt[k + 2]) * h.g + ld_f3(S.tri_bt[k]) * w0);
    T = normalize(T);
    B = normalize(B);
    float u, v, c[4];
    hit_texcoord(S, h, u, v);
    orx_tex2d_linear(t.nrgba, t.nw, t.nh, u, v, c);
    const float nx = 2.f * c[0] - 1.f, ny = 2.f * c[1] - 1.f, nz = 2.f * c[2] - 1.f;
    return normalize(mk(nx * T.x + ny * B.x + nz * wsn.x, nx * T.y + ny * B.y + nz * wsn.y,
                        nx * T.z + ny * B.z + nz * wsn.z));
}

/* ------------------------------------------------------------------ */
/* camera (Camera.cpp:333-345 derived on the host; helpers/camera.h)   */
/* ------------------------------------------------------------------ */
struct DevCamera {
    f3 eye, lookdir, u, v;
    float aperture;
};
/* RayGeneratorPPM.cu:40-48 / RayGeneratorPT.cu:53-61 + modifyRayForDepthOfField */
__device__ __forceinline__ void primary_ray(const DevCamera& cam, uint32_t x, uint32_t y, uint32_t W, uint32_t H,
                                            Rng& rs, f3& o, f3& d) {
    float sx = rnd(rs);
    float sy = rnd(rs);
    float dx = ((float)x + sx) / (float)W * 2.0f - 1.0f;
    float dy = ((float)y + sy) / (float)H * 2.0f - 1.0f;
    f3 origin = cam.eye;
    f3 dir = normalize(cam.u * dx + cam.v * dy + cam.lookdir);
    if (cam.aperture > 0) {
        f3 focal = cam.eye + cam.lookdir;
        f3 camLookDir = normalize(cam.lookdir);
        float focalPlaneT = (dot(camLookDir, focal) - dot(camLookDir, cam.eye)) / dot(camLookDir, dir);
        f3 lookAt = origin + dir * focalPlaneT;
        float ux = rnd(rs);
        float uy = rnd(rs);
        float rr = sqrtf(ux);
        float th = 2.f * ORX_PI_F * uy;
        float discx = rr * orx_cosf(th);
        float discy = rr * orx_sinf(th);
        origin = origin + ((cam.u * discx) * cam.aperture + (cam.v * discy) * cam.aperture);
        dir = normalize(lookAt - origin);
    }
    o = origin;
    d = dir;
}

/* ------------------------------------------------------------------ */
/* radiance ray: RadiancePRD through the closest-hit programs          */
/* ------------------------------------------------------------------ */
struct RadiancePRD {
    f3 attenuation, radiance;
    uint32_t depth;
    f3 position, normal;
    uint32_t flags;
    f3 newdir;
};

__device__ __forceinline__ float glass_reflect_factor(f3 d, f3 N, float n1, float n2, f3& refr, bool& valid) {
    valid = refract(refr, d, N, n2 / n1);
    float cosI = -dot(d, N);
    float cosT = -dot(refr, N);
    float refl = 1.f;
    if (valid) {
        float rp = (n2 * cosI - n1 * cosT) / (n2 * cosI + n1 * cosT);
        float rs = (n1 * cosI - n2 * cosT) / (n1 * cosI + n2 * cosT);
        refl = (rp * rp + rs * rs) / 2.f;
    }
    return refl;
}

/* Iterative form of the rtTrace(RADIANCE) recursion: Diffuse.cu:71-87,
 * Glossy.cu:74-90, DiffuseEmitter.cu:40-51, Mirror.cu:50-63, Glass.cu:90-143,
 * miss RayGeneratorPPM.cu:72-77. */
__device__ inline void trace_radiance(const DevScene& S, uint32_t maxd, f3 o, f3 d, float tmin, RadiancePRD& prd,
                                      Rng& rs, uint32_t* stk) {
    for (;;) {
        Hit h;
        if (!trace_closest(S, o, d, tmin, RT_DEFAULT_MAX, h, stk)) {
            prd.flags = PRD_MISS;
            prd.attenuation = mk1(0.f);
            prd.radiance = mk1(0.f);
            return;
        }
        const DevMaterial& m = S.mats[prim_material(S, h)];
        f3 hitPoint = o + d * h.t;
        f3 N = shading_normal(S, h);
        if (m.type == MAT_DIFFUSE || m.type == MAT_GLOSSY) {
            prd.flags |= PRD_HIT_NON_SPECULAR;
            prd.attenuation = prd.attenuation * m.Kd;
            prd.normal = N;
            prd.position = hitPoint;
            prd.depth++;
            if (prd.flags & PRD_PATH_TRACING) {
                float s0 = rnd(rs);
                float s1 = rnd(rs);
                prd.newdir = sample_hemisphere_cos(N, s0, s1);
            }
            return;
        } else if (m.type == MAT_TEXTURE) { /* Texture.cu:83-110: mapped normal, no depth++ */
            prd.flags |= PRD_HIT_NON_SPECULAR;
            prd.normal = tex_normal(S, m, h, N);
            prd.position = hitPoint;
            if (prd.flags & PRD_PATH_TRACING) {
                float s0 = rnd(rs);
                float s1 = rnd(rs);
                prd.newdir = sample_hemisphere_cos(N, s0, s1);
            }
            prd.attenuation = prd.attenuation * tex_color(S, m, h);
            return;
        } else if (m.type == MAT_EMITTER) {
            prd.flags |= PRD_HIT_EMITTER;
            if (dot(N, -d) < 0.f) return;
            f3 Le = m.powerPerArea / ORX_PI_F;
            prd.radiance = prd.radiance + prd.attenuation * Le;
            return;
        } else if (m.type == MAT_MIRROR) {
            prd.depth++;
            if (prd.depth <= maxd) {
                prd.attenuation = prd.attenuation * m.Kr;
                d = reflect(d, N);
                o = hitPoint;
                tmin = 0.0001f;
                continue;
            }
            return;
        } else { /* glass */
            bool outside = dot(N, d) < 0;
            f3 Nn = outside ? N : -N;
            float n1 = outside ? 1.0f : m.ior, n2 = outside ? m.ior : 1.0f;
            f3 refr;
            bool valid;
            float refl = glass_reflect_factor(d, Nn, n1, n2, refr, valid);
            float sample = rnd(rs);
            f3 nd;
            if (sample <= refl) {
                nd = reflect(d, Nn);
            } else {
                nd = refr;
                prd.attenuation = prd.attenuation * ((n2 * n2) / (n1 * n1));
            }
            prd.flags |= PRD_HIT_SPECULAR;
            prd.flags &= ~PRD_HIT_NON_SPECULAR;
            prd.depth++;
            if (prd.depth <= maxd) {
                o = hitPoint;
                d = nd;
                tmin = 0.0001f;
                continue;
            }
            prd.attenuation = prd.attenuation * 0.f;
            return;
        }
    }
}

/* ------------------------------------------------------------------ */
/* participating medium (cfg.enable_media, ENABLE_PARTICIPATING_MEDIA) */
/* ------------------------------------------------------------------ */
constexpr int32_t MED_PRIM = 0x7ffffff0; /* Hit::prim of the medium box (after every surface) */
/* The medium box and the volumetric photon table of the last photon pass: a uniform grid of
 * cells >= 1.01 R over the box padded by 2R (records of the cells in cell order, slot order
 * inside a cell, then the photons outside that box), read by the next eye pass. */
struct VolMap {
    uint32_t on;              /* media enabled */
    f3 lo, hi;                /* the box */
    float sig_s, sig_a;
    uint32_t valid;           /* a photon pass has filled the table (else it gathers nothing) */
    float R;                  /* volumetricRadius of the table */
    f3 glo;                   /* grid origin (box - 2R) */
    float cell;
    uint32_t n[3], G;         /* cells per axis, G = n0 n1 n2; bucket G: outside the grid */
    f3 ilo, ihi;              /* box +- R: a segment with both ends inside uses the grid */
    const uint32_t* start;    /* [G + 2]: start[c] first record of cell c, start[G + 1] = total */
    const float4* rec;        /* [total][2]: pos.xyz, pw.x | pw.y, pw.z (pw = power * numDeposits) */
};

/* geometry_instance/AAB.cu:24-157: slab test with the near/far axes; inside the box (tNear < 0.01,
 * tFar > 0) RADIANCE/PHOTON rays report t = 0.000115 with the far axis' normal against the ray,
 * the IN_PARTICIPATING_MEDIUM types report tFar with the normal along it */
__device__ __forceinline__ bool isect_medium(const VolMap& vm, f3 o, f3 d, float tmin, float tmax, bool in_medium,
                                             float& tout, f3& nout) {
    int axn = 0, axf = 0;
    float tn, tf;
    const float divx = 1 / d.x;
    if (divx >= 0) { tn = (vm.lo.x - o.x) * divx; tf = (vm.hi.x - o.x) * divx; }
    else { tn = (vm.hi.x - o.x) * divx; tf = (vm.lo.x - o.x) * divx; }
    if (tf < tn) return false;
    const float divy = 1 / d.y;
    float tyn, tyf;
    if (divy >= 0) { tyn = (vm.lo.y - o.y) * divy; tyf = (vm.hi.y - o.y) * divy; }
    else { tyn = (vm.hi.y - o.y) * divy; tyf = (vm.lo.y - o.y) * divy; }
    if (tyn > tn) { tn = tyn; axn = 1; }
    if (tyf < tf) { tf = tyf; axf = 1; }
    if (tf < tn) return false;
    const float divz = 1 / d.z;
    float tzn, tzf;
    if (divz >= 0) { tzn = (vm.lo.z - o.z) * divz; tzf = (vm.hi.z - o.z) * divz; }
    else { tzn = (vm.hi.z - o.z) * divz; tzf = (vm.lo.z - o.z) * divz; }
    if (tzn > tn) { tn = tzn; axn = 2; }
    if (tzf < tf) { tf = tzf; axf = 2; }
    if (tf < tn) return false;
    float t = tn, nvr = -1;
    int ax = axn;
    if (tn < 0.01f && tf > 0.0f) {
        ax = axf;
        if (!in_medium) t = (float)0.000115;
        else { t = tf; nvr = 1; }
    }
    if (!(t > tmin && t < tmax)) return false;
    const float dc = ax == 0 ? d.x : ax == 1 ? d.y : d.z;
    const float nc = dc >= 0 ? nvr : -nvr;
    nout = mk(ax == 0 ? nc : 0.f, ax == 1 ? nc : 0.f, ax == 2 ? nc : 0.f);
    tout = t;
    return true;
}
/* closest hit with the medium box as the last primitive (a surface at the same t wins) */
template <class STK, class NODES>
__device__ __forceinline__ bool trace_closest_m(const DevScene& S, const VolMap& vm, f3 o, f3 d, float tmin, float tmax,
                                                bool in_medium, Hit& h, const STK& stk, const NODES& nodes) {
    const bool hit = trace_closest_t(S, o, d, tmin, tmax, h, stk, nodes);
    float t;
    f3 n;
    if (isect_medium(vm, o, d, tmin, hit ? h.t : tmax, in_medium, t, n)) {
        h.t = t;
        h.prim = MED_PRIM;
        h.sn = n;
        h.b = h.g = 0.f;
        return true;
    }
    return hit;
}

/* The volumetric gather of one segment (VolumetricPhotonSphere.cu:24-59 +
 * VolumetricPhotonSphereRadiance.cu:24-34): every root of a photon's sphere inside (tmin, tmax)
 * adds the photon when its projection on the ray lies inside (tmin, tmax) (a photon with both
 * roots inside counts twice).  The photons are found by walking the grid cells of the segment
 * (3D DDA) and testing the 3x3x3 neighbourhood of each: cells are >= 1.01 R, so a photon within
 * R of a segment point lies in the neighbourhood of that point's cell, and the neighbourhoods
 * of consecutive cells differ by one 3x3 face, which is all a step visits (the walk is monotone
 * per axis, so no cell is visited twice).  A segment not inside box +- R (it can leave the box
 * only through a grazing corner) tests every record. */
__device__ __forceinline__ void vol_test(const VolMap& vm, uint32_t i, f3 o, f3 d, float tmin, float tmax, float R2,
                                         float coef, float sig_t, f3& acc) {
    const float4 A = vm.rec[2 * i], B = vm.rec[2 * i + 1];
    const f3 pos = mk(A.x, A.y, A.z);
    const f3 O = o - pos;
    const float b = dot(O, d), c = dot(O, O) - R2, disc = b * b - c;
    if (!(disc > 0.0f)) return;
    const float sd = sqrtf(disc), r1 = -b - sd, r2 = -b + sd;
    const float t = dot(pos - o, d);
    if (!(t < tmax && t > tmin)) return;
    const f3 pw = mk(A.w, B.x, B.y);
    const f3 add1 = ((pw * coef) * orx_expf(-sig_t * t)) * (1.f / (4.f * ORX_PI_F));
    if (r1 > tmin && r1 < tmax) acc = acc + add1;
    if (r2 > tmin && r2 < tmax) acc = acc + add1;
}
__device__ __forceinline__ void vol_cell(const VolMap& vm, int x, int y, int z, f3 o, f3 d, float tmin, float tmax,
                                         float R2, float coef, float sig_t, f3& acc) {
    if (x < 0 || y < 0 || z < 0 || x >= (int)vm.n[0] || y >= (int)vm.n[1] || z >= (int)vm.n[2]) return;
    const uint32_t c = (uint32_t)x + vm.n[0] * ((uint32_t)y + vm.n[1] * (uint32_t)z);
    const uint32_t e = vm.start[c + 1];
    for (uint32_t i = vm.start[c]; i < e; i++) vol_test(vm, i, o, d, tmin, tmax, R2, coef, sig_t, acc);
}
__device__ inline f3 vol_gather(const VolMap& vm, f3 o, f3 d, float tmin, float tmax, float sig_t) {
    f3 acc = mk1(0.f);
    if (!vm.valid || !(tmax > tmin)) return acc;
    const float R = vm.R, R2 = R * R, coef = 1 / (ORX_PI_F * R * R);
    const f3 p0 = o + d * tmin, p1 = o + d * tmax;
    const bool in0 = p0.x >= vm.ilo.x && p0.y >= vm.ilo.y && p0.z >= vm.ilo.z && p0.x <= vm.ihi.x &&
                     p0.y <= vm.ihi.y && p0.z <= vm.ihi.z;
    const bool in1 = p1.x >= vm.ilo.x && p1.y >= vm.ilo.y && p1.z >= vm.ilo.z && p1.x <= vm.ihi.x &&
                     p1.y <= vm.ihi.y && p1.z <= vm.ihi.z;
    if (!(in0 && in1)) {
        const uint32_t total = vm.start[vm.G + 1];
        for (uint32_t i = 0; i < total; i++) vol_test(vm, i, o, d, tmin, tmax, R2, coef, sig_t, acc);
        return acc;
    }
    const float inv = 1.f / vm.cell;
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z}, pp[3] = {p0.x, p0.y, p0.z};
    const float gl[3] = {vm.glo.x, vm.glo.y, vm.glo.z};
    int c[3], st[3];
    float tn[3];
    for (int k = 0; k < 3; k++) {
        int ck = (int)orx_floorf((pp[k] - gl[k]) * inv);
        ck = ck < 0 ? 0 : (ck >= (int)vm.n[k] ? (int)vm.n[k] - 1 : ck);
        c[k] = ck;
        st[k] = dd[k] > 0.f ? 1 : (dd[k] < 0.f ? -1 : 0);
        tn[k] = st[k] ? (gl[k] + (float)(ck + (st[k] > 0)) * vm.cell - oo[k]) / dd[k] : INFINITY;
    }
    for (int dz = -1; dz <= 1; dz++)
        for (int dy = -1; dy <= 1; dy++)
            for (int dx = -1; dx <= 1; dx++)
                vol_cell(vm, c[0] + dx, c[1] + dy, c[2] + dz, o, d, tmin, tmax, R2, coef, sig_t, acc);
    const int maxsteps = (int)(vm.n[0] + vm.n[1] + vm.n[2]) + 3;
    for (int s = 0; s < maxsteps; s++) {
        const int k = tn[0] <= tn[1] ? (tn[0] <= tn[2] ? 0 : 2) : (tn[1] <= tn[2] ? 1 : 2);
        if (!(tn[k] <= tmax)) break;
        c[k] += st[k];
        if (c[k] < 0 || c[k] >= (int)vm.n[k]) break;
        tn[k] = (gl[k] + (float)(c[k] + (st[k] > 0)) * vm.cell - oo[k]) / dd[k];
        const int f = c[k] + st[k]; /* the neighbourhood's new face */
        const int u = (k + 1) % 3, v = (k + 2) % 3;
        for (int a = -1; a <= 1; a++)
            for (int b2 = -1; b2 <= 1; b2++) {
                int q[3];
                q[k] = f;
                q[u] = c[u] + a;
                q[v] = c[v] + b2;
                vol_cell(vm, q[0], q[1], q[2], o, d, tmin, tmax, R2, coef, sig_t, acc);
            }
    }
    return acc;
}

/* trace_radiance with the medium (ParticipatingMedium.cu:53-104; the frames and their unrolled
 * accumulation are described at the oracle's trace_radiance): volR = the path's
 * Hitpoint::volumetricRadiance, the attenuation leaves multiplied by every frame's T. */
__device__ inline void trace_radiance_vol(const DevScene& S, const VolMap& vm, uint32_t maxd, f3 o, f3 d, float tmin,
                                          RadiancePRD& prd, Rng& rs, uint32_t* stk, f3& volR) {
    const float sig_t = vm.sig_a + vm.sig_s;
    bool inmed = false, frame = false;
    f3 fa = mk1(0.f), fh = mk1(0.f), fd = mk1(0.f);
    float P = 1.f;
    volR = mk1(0.f);
    for (;;) {
        Hit h;
        const bool hit = trace_closest_m(S, vm, o, d, tmin, RT_DEFAULT_MAX, inmed, h, StackL{stk}, NodesG{});
        if (frame) {
            frame = false;
            float dist = 0.f;
            if (hit) {
                if (h.prim == MED_PRIM) {
                    dist = (float)(((double)h.t + 0.1) - 0.1);
                } else {
                    const DevMaterial& fm = S.mats[prim_material(S, h)];
                    if (fm.type != MAT_EMITTER || !(dot(shading_normal(S, h), -d) < 0.f)) dist = h.t;
                }
            }
            const float T = orx_expf(-dist * sig_t);
            const f3 V = vol_gather(vm, fh, fd, (float)0.0000001, dist, sig_t);
            volR = volR + (fa * V) * P;
            P = P * T;
        }
        if (!hit) {
            prd.flags = PRD_MISS;
            prd.attenuation = mk1(0.f);
            prd.radiance = mk1(0.f);
            break;
        }
        const f3 hitPoint = o + d * h.t;
        if (h.prim == MED_PRIM) {
            const f3 N = normalize(h.sn);
            if (dot(N, d) < 0) {
                frame = true;
                fa = (prd.attenuation + mk1(0.1f)) - mk1(0.1f);
                fh = hitPoint;
                fd = d;
                inmed = true;
            } else {
                inmed = false;
            }
            o = hitPoint;
            tmin = 0.01f;
            continue;
        }
        const DevMaterial& m = S.mats[prim_material(S, h)];
        const f3 N = shading_normal(S, h);
        if (m.type == MAT_DIFFUSE || m.type == MAT_GLOSSY) {
            prd.flags |= PRD_HIT_NON_SPECULAR;
            prd.attenuation = prd.attenuation * m.Kd;
            prd.normal = N;
            prd.position = hitPoint;
            prd.depth++;
            break;
        } else if (m.type == MAT_TEXTURE) {
            prd.flags |= PRD_HIT_NON_SPECULAR;
            prd.normal = tex_normal(S, m, h, N);
            prd.position = hitPoint;
            prd.attenuation = prd.attenuation * tex_color(S, m, h);
            break;
        } else if (m.type == MAT_EMITTER) {
            prd.flags |= PRD_HIT_EMITTER;
            if (dot(N, -d) < 0.f) break;
            const f3 Le = m.powerPerArea / ORX_PI_F;
            prd.radiance = prd.radiance + prd.attenuation * Le;
            break;
        } else if (m.type == MAT_MIRROR) {
            prd.depth++;
            if (prd.depth <= maxd) {
                prd.attenuation = prd.attenuation * m.Kr;
                d = reflect(d, N);
                o = hitPoint;
                tmin = 0.0001f;
                inmed = false;
                continue;
            }
            break;
        } else { /* glass */
            const bool outside = dot(N, d) < 0;
            const f3 Nn = outside ? N : -N;
            const float n1 = outside ? 1.0f : m.ior, n2 = outside ? m.ior : 1.0f;
            f3 refr;
            bool valid;
            const float refl = glass_reflect_factor(d, Nn, n1, n2, refr, valid);
            const float sample = rnd(rs);
            const bool reflected = sample <= refl;
            f3 nd;
            if (reflected) {
                nd = reflect(d, Nn);
            } else {
                nd = refr;
                prd.attenuation = prd.attenuation * ((n2 * n2) / (n1 * n1));
            }
            prd.flags |= PRD_HIT_SPECULAR;
            prd.flags &= ~PRD_HIT_NON_SPECULAR;
            prd.depth++;
            if (prd.depth <= maxd) {
                o = hitPoint;
                d = nd;
                tmin = 0.0001f;
                inmed = (outside && !reflected) || (!outside && reflected);
                continue;
            }
            prd.attenuation = prd.attenuation * 0.f;
            break;
        }
    }
    prd.attenuation = prd.attenuation * P;
}

/* getLightContribution (helpers/light.h:29-87) */
/* The sample half of light_contribution: the point on the light, the unshadowed contribution
 * power * lightFactor and the shadow ray; false (contribution 0, no ray) when lightFactor <= 0 */
__device__ inline bool light_sample(const DevLight& light, f3 pos, f3 normal, Rng& rs, f3& lc, f3& dir, float& tmax) {
    float lightFactor = 1;
    f3 pointOnLight;
    if (light.type == LIGHT_AREA) {
        float sx = rnd(rs);
        float sy = rnd(rs);
        pointOnLight = light.position + light.v1 * sx + light.v2 * sy;
    } else if (light.type == LIGHT_POINT) {
        pointOnLight = light.position;
        lightFactor *= 1.f / 4.f;
    } else {
        return false;
    }
    f3 towardsLight = pointOnLight - pos;
    float lightDistance = length(towardsLight);
    towardsLight = towardsLight / lightDistance;
    float n_dot_l = maxf(0, dot(normal, towardsLight));
    lightFactor *= n_dot_l / (ORX_PI_F * lightDistance * lightDistance);
    if (light.type == LIGHT_AREA) lightFactor *= maxf(0, dot(-towardsLight, light.normal));
    if (!(lightFactor > 0.0f)) return false;
    tmax = (float)((double)lightDistance - 0.0001);
    dir = towardsLight;
    lc = light.power * lightFactor; /* = power * (lightFactor * att) for att = 1; occluded: 0 */
    return true;
}
/* helpers/light.h:29-87 (shadow ray from pos + 0.0001 towards the light sample) */
__device__ inline f3 light_contribution(const DevScene& S, const DevLight& light, f3 pos, f3 normal, Rng& rs,
                                        uint32_t* stk) {
    f3 lc, dir;
    float tmax;
    if (!light_sample(light, pos, normal, rs, lc, dir, tmax)) return mk1(0);
    return trace_any(S, pos, dir, 0.0001f, tmax, stk) ? mk1(0.f) : lc;
}

}  // namespace orx
