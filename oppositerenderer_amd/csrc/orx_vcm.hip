/*
 * orx_vcm.hip — VCM (bidirectional path tracing with vertex connection) for
 * gfx950: the reference's VCM_LIGHT_PASS and VCM_CAMERA_PASS launches
 * (OptixRenderer.cpp:675-795) as two megakernels, one lane per subpath.
 *
 * Reference programs restated (RenderEngine/):
 *   renderer/vcm/VCMLightPass.cu, VCMCameraPass.cu, vcm.h, mis.h,
 *   renderer/BSDF.h (VcmBSDF), BxDF.h, reflection.h, math/DifferentialGeometry.h,
 *   helpers/light.h (lightEmit / lightIlluminate), helpers/samplers.h,
 *   material/{Diffuse,Glossy,Mirror,Glass,DiffuseEmitter}.cu vcmClosestHit*.
 * Shipped configuration: VCM_UNIFORM_VERTEX_SAMPLING 0, vcmUseVC 1, vcmUseVM 0.
 *
 * Data layout (HBM):
 *   light vertex cache: slot k of subpath p (p = x + y*W) in four float4
 *   planes [9][W*H] — A: pos.xyz|material, B: throughput.xyz|dVCM,
 *   C: normal.xyz|dVC, D: localDirFix.xyz|dVM.  The reference appends
 *   vertices to one atomically-bumped LightVertex array and keeps a
 *   [W*H][9] index table; camera subpath p only ever reads light subpath p,
 *   so the direct [k][p] layout needs neither the atomic nor the table and
 *   every per-k access of a wave is one contiguous 1 KiB run.
 *   light-tracing splats (connectCameraT1) go to a per-iteration float
 *   buffer with hardware fp32 atomics; the camera pass folds it into the
 *   running-sum output together with the camera subpath colour.
 * The same quirks as the CPU restatement (oracle/orx_oracle_vcm.c.inc) are
 * reproduced; everything but the splat sums is bit-identical to it.
 */
#include <algorithm>

#include "orx_kernels.h"

namespace orx {

constexpr float VCM_EPS_COSINE = 1e-6f;  /* config.h:42 */
constexpr float VCM_EPS_RAY = 1e-3f;     /* config.h:43 */
constexpr float VCM_RAY_LEN_MIN = 0.0001f;
constexpr float VCM_EPS_PHONG = 1e-3f;   /* BxDF.h:253 */

/* BxDF::Type (BxDF.h:47-67) */
enum : uint32_t {
    BX_REFLECTION = 1, BX_TRANSMISSION = 2, BX_DIFFUSE = 4, BX_GLOSSY = 8, BX_SPECULAR = 16, BX_ALL = 31,
    BX_LAMBERTIAN = 32, BX_SPEC_REFLECTION = 64, BX_SPEC_TRANSMISSION = 128, BX_PHONG = 256
};

__device__ __forceinline__ bool iszero(f3 v) { return v.x == 0.f && v.y == 0.f && v.z == 0.f; }
__device__ __forceinline__ float luminance_cie(f3 c) { return c.x * 0.2126f + c.y * 0.7152f + c.z * 0.0722f; }
__device__ __forceinline__ f3 local_reflect(f3 w) { return mk(-w.x, -w.y, w.z); }

/* DifferentialGeometry (math/DifferentialGeometry.h) */
struct Frame {
    f3 b, t, n;
    __device__ __forceinline__ f3 to_world(f3 a) const { return b * a.x + t * a.y + n * a.z; }
    __device__ __forceinline__ f3 to_local(f3 a) const { return mk(dot(b, a), dot(t, a), dot(n, a)); }
};
__device__ __forceinline__ Frame frame_from_normal(f3 nrm) {
    Frame f;
    f.n = normalize(nrm);
    f3 tmp = fabsf(f.n.x) > 0.99f ? mk(0.f, 1.f, 0.f) : mk(1.f, 0.f, 0.f);
    f.t = normalize(cross(f.n, tmp));
    f.b = cross(f.t, f.n);
    return f;
}

/* FresnelDielectric::evaluate (reflection.h:106-133) */
__device__ inline float fresnel_dielectric(float cosi, float eta_i, float eta_t) {
    cosi = fmaxf(-1.0f, fminf(cosi, 1.0f));
    const bool entering = cosi > 0.0f;
    float ei = entering ? eta_i : eta_t, et = entering ? eta_t : eta_i;
    float sint = ei / et * sqrtf(fmaxf(0.0f, 1.0f - cosi * cosi));
    if (sint >= 1.0f) return 1.0f;
    cosi = fabsf(cosi);
    float cost = sqrtf(fmaxf(0.0f, 1.0f - sint * sint));
    float Rparl = ((et * cosi) - (ei * cost)) / ((et * cosi) + (ei * cost));
    float Rperp = ((ei * cosi) - (et * cost)) / ((ei * cosi) + (et * cost));
    return (Rparl * Rparl + Rperp * Rperp) * 0.5f;
}

struct Bxdf {
    uint32_t type;
    f3 R;
    float exponent;
    float ei, et;
    bool dielectric;
};
__device__ __forceinline__ bool bx_match(uint32_t type, uint32_t mask) {
    return (type & BX_ALL & mask) == (type & BX_ALL);
}
__device__ __forceinline__ float bx_fresnel(const Bxdf& b, float c) {
    return b.dielectric ? fresnel_dielectric(c, b.ei, b.et) : 1.0f;
}
__device__ __forceinline__ float bx_cont(const Bxdf& b, f3 wo) {
    const uint32_t k = b.type & ~BX_ALL;
    if (k == BX_LAMBERTIAN || k == BX_PHONG) return fmaxf(b.R.x, maxf(b.R.y, b.R.z));
    if (k == BX_SPEC_REFLECTION) return bx_fresnel(b, wo.z) * fmaxf(b.R.x, maxf(b.R.y, b.R.z));
    return 1.f - bx_fresnel(b, wo.z);
}
__device__ __forceinline__ float bx_albedo(const Bxdf& b, f3 wo) {
    const uint32_t k = b.type & ~BX_ALL;
    if (k == BX_LAMBERTIAN || k == BX_PHONG) return luminance_cie(b.R);
    if (k == BX_SPEC_REFLECTION) return bx_fresnel(b, wo.z) * luminance_cie(b.R);
    return (1.f - bx_fresnel(b, wo.z)) * luminance_cie(b.R);
}
__device__ __forceinline__ Bxdf mk_bx(uint32_t type, f3 R, float e = 0.f, float ei = 1.f, float et = 1.f,
                                      bool diel = false) {
    Bxdf b;
    b.type = type; b.R = R; b.exponent = e; b.ei = ei; b.et = et; b.dielectric = diel;
    return b;
}
constexpr uint32_t T_LAMBERT = BX_LAMBERTIAN | BX_REFLECTION | BX_DIFFUSE;
constexpr uint32_t T_PHONG = BX_PHONG | BX_REFLECTION | BX_GLOSSY;
constexpr uint32_t T_SREFL = BX_SPEC_REFLECTION | BX_REFLECTION | BX_SPECULAR;
constexpr uint32_t T_STRANS = BX_SPEC_TRANSMISSION | BX_TRANSMISSION | BX_SPECULAR;

__device__ __forceinline__ float pow_cos_pdf(f3 n, f3 d, float power) {
    const float cosTheta = fmaxf(0.f, dot(n, d));
    return (power + 1.f) * orx_powf(cosTheta, power) * (ORX_1_PI_F * 0.5f);
}
__device__ inline float bx_pdf(const Bxdf& b, f3 wo, f3 wi, bool rev) {
    const uint32_t k = b.type & ~BX_ALL;
    if (k == BX_LAMBERTIAN) {
        if (wo.z * wi.z > 0.0f) return rev ? fabsf(wo.z) * ORX_1_PI_F : fabsf(wi.z) * ORX_1_PI_F;
        return 0.f;
    }
    if (k == BX_PHONG) {
        f3 r = local_reflect(wo);
        if (dot(r, wi) <= VCM_EPS_PHONG) return 0.f;
        return pow_cos_pdf(r, wi, b.exponent);
    }
    return 0.f;
}
__device__ inline f3 phong_f(const Bxdf& b, f3 wo, f3 wi, float* pdf) {
    if (wo.z < VCM_EPS_COSINE || wi.z < VCM_EPS_COSINE) {
        if (pdf) *pdf = 0.f;
        return mk1(0.f);
    }
    f3 r = local_reflect(wo);
    float d = dot(r, wi);
    if (d <= VCM_EPS_PHONG) {
        if (pdf) *pdf = 0.f;
        return mk1(0.f);
    }
    if (pdf) *pdf = pow_cos_pdf(r, wi, b.exponent);
    f3 rho = ((b.R * (b.exponent + 2.f)) * 0.5f) * ORX_1_PI_F;
    return rho * orx_powf(d, b.exponent);
}
__device__ inline f3 bx_f(const Bxdf& b, f3 wo, f3 wi) {
    const uint32_t k = b.type & ~BX_ALL;
    if (k == BX_LAMBERTIAN) return b.R * ORX_1_PI_F;
    if (k == BX_PHONG) return phong_f(b, wo, wi, nullptr);
    return mk1(0.f);
}
__device__ inline f3 bx_vcm_f(const Bxdf& b, f3 wo, f3 wi, float& dpdf, float& rpdf) {
    const uint32_t k = b.type & ~BX_ALL;
    if (k == BX_LAMBERTIAN) {
        if (wo.z < VCM_EPS_COSINE || wi.z < VCM_EPS_COSINE) return mk1(0.f);
        dpdf = fmaxf(0.f, wi.z * ORX_1_PI_F);
        rpdf = fmaxf(0.f, wo.z * ORX_1_PI_F);
        return b.R * ORX_1_PI_F;
    }
    if (k == BX_PHONG) {
        float pdf = 0.f;
        f3 f = phong_f(b, wo, wi, &pdf);
        dpdf = pdf;
        rpdf = pdf;
        return f;
    }
    dpdf = 0.f;
    rpdf = 0.f;
    return mk1(0.f);
}
__device__ inline f3 bx_sample_f(const Bxdf& b, f3 wo, f3& wi, float s0, float s1, float& pdf, bool adjoint) {
    const uint32_t k = b.type & ~BX_ALL;
    if (k == BX_LAMBERTIAN) {
        if (wo.z < VCM_EPS_COSINE) { pdf = 0.f; return mk1(0.f); }
        /* optixu cosine_sample_hemisphere */
        const float r = sqrtf(s0);
        const float phi = 2.0f * ORX_PI_F * s1;
        wi.x = r * orx_cosf(phi);
        wi.y = r * orx_sinf(phi);
        wi.z = sqrtf(fmaxf(0.0f, 1.0f - wi.x * wi.x - wi.y * wi.y));
        pdf = bx_pdf(b, wo, wi, false);
        return b.R * ORX_1_PI_F;
    }
    if (k == BX_PHONG) {
        const float phi = 2.f * ORX_PI_F * s0;
        const float z = orx_powf(s1, 1.f / (b.exponent + 1.f));
        const float r = sqrtf(1.f - z * z);
        wi = mk(orx_cosf(phi) * r, orx_sinf(phi) * r, z);
        if (wo.z < VCM_EPS_COSINE || wi.z < VCM_EPS_COSINE) { pdf = 0.f; return mk1(0.f); }
        const f3 refl = local_reflect(wo);
        const Frame dg = frame_from_normal(refl);
        wi = dg.to_world(wi);
        const float d = dot(refl, wi);
        if (d <= VCM_EPS_PHONG) { pdf = 0.f; return mk1(0.f); }
        pdf = bx_pdf(b, wo, wi, false);
        f3 rho = ((b.R * (b.exponent + 2.f)) * 0.5f) * ORX_1_PI_F;
        return rho * orx_powf(d, b.exponent);
    }
    if (k == BX_SPEC_REFLECTION) {
        wi = mk(-wo.x, -wo.y, wo.z);
        pdf = 1.0f;
        const float R = bx_fresnel(b, wo.z);
        return (b.R * R) / fabsf(wi.z);
    }
    const bool entering = wo.z > 0.0f;
    const float ei = entering ? b.ei : b.et, et = entering ? b.et : b.ei;
    const float sini2 = 1.0f - wo.z * wo.z;
    const float eta = ei / et;
    const float sint2 = eta * eta * sini2;
    if (sint2 >= 1.f) return mk1(0.f); /* pdf left untouched (BxDF.h:496) */
    float cost = sqrtf(fmaxf(0.f, 1.f - sint2));
    if (entering) cost = -cost;
    wi = mk(eta * -wo.x, eta * -wo.y, cost);
    pdf = 1.f;
    const float T = 1.f - bx_fresnel(b, wo.z);
    if (adjoint) return (b.R * T) / fabsf(wi.z);
    return ((b.R * T) * (eta * eta)) / fabsf(wi.z);
}

struct VBsdf {
    Frame dg;
    f3 gn;
    f3 fix;
    Bxdf bx[2];
    float pick[2];
    float cont;
    int n;
    bool fix_is_light;

    __device__ __forceinline__ void init(f3 world_normal, f3 incident, bool is_light) {
        dg = frame_from_normal(world_normal);
        gn = world_normal;
        fix_is_light = is_light;
        fix = dg.to_local(incident);
        n = 0;
        cont = 0.f;
        pick[0] = pick[1] = 0.f;
    }
    /* (all BxDF slots are addressed with compile-time indices so the BSDF
     * stays in registers: no scratch) */
    __device__ __forceinline__ void add(const Bxdf& b) {
        float rr = 0.f;
        rr += bx_cont(b, fix);
        cont = fminf(1.f, cont + rr);
        float albedo = 0.f;
        albedo += bx_albedo(b, fix);
        if (n == 0) {
            bx[0] = b;
            pick[0] = albedo;
        } else {
            bx[1] = b;
            pick[1] = albedo;
        }
        n++;
    }
    __device__ __forceinline__ int count(uint32_t mask) const {
        int c = 0;
#pragma unroll
        for (int i = 0; i < 2; i++) c += (i < n && bx_match(bx[i].type, mask)) ? 1 : 0;
        return c;
    }
    __device__ __forceinline__ bool is_specular() const { return count(BX_ALL & ~BX_SPECULAR) == 0; }
    __device__ __forceinline__ float sum_pick(uint32_t mask) const {
        float c = 0.f;
#pragma unroll
        for (int i = 0; i < 2; i++)
            if (i < n && bx_match(bx[i].type, mask)) c += pick[i];
        return c;
    }
    /* VcmBSDF::sampleF via vcmSampleF (BSDF.h:411-485) */
    __device__ f3 sample_f(float sx, float sy, float sz, f3& world_wi, float& pdf, float& cos_out,
                           uint32_t& sampled) const {
        int index = 0;
        float sum = 0.f;
        const int nMatched = count(BX_ALL);
        if (nMatched) {
            sum = sum_pick(BX_ALL);
            float prev = 0.f;
            bool found = false;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                if (!found && i < n && bx_match(bx[i].type, BX_ALL)) {
                    const float cp = pick[i] / sum;
                    if (sx < prev + cp) { index = i; found = true; }
                    else prev += cp;
                }
            }
        }
        if (sum == 0.f) { pdf = 0.0f; return mk1(0.f); }
        const Bxdf b = index ? bx[1] : bx[0];
        const float pick_index = index ? pick[1] : pick[0];
        const f3 world_wo = dg.to_world(fix);
        const f3 wo = dg.to_local(world_wo);
        f3 wi = mk1(0.f);
        f3 f = bx_sample_f(b, wo, wi, sy, sz, pdf, fix_is_light);
        const float q = pick_index / sum;
        pdf *= q;
        if (pdf == 0.0f) { sampled = 0; return mk1(0.f); }
        sampled = b.type;
        world_wi = dg.to_world(wi);
        cos_out = fabsf(wi.z);
        if (!(b.type & BX_SPECULAR)) {
            if (nMatched > 1) {
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    if (i >= n || i == index || !bx_match(bx[i].type, BX_ALL)) continue;
                    float comp = 0.f;
                    comp += bx_pdf(bx[i], wo, wi, false);
                    pdf += comp * q;
                }
            }
            uint32_t m2 = BX_ALL;
            if (dot(gn, world_wi) * dot(gn, world_wo) >= 0.0f) m2 &= ~BX_TRANSMISSION;
            else m2 &= ~BX_REFLECTION;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                if (i >= n || i == index || !bx_match(bx[i].type, m2)) continue;
                f = f + bx_f(bx[i], wo, wi);
            }
        }
        return f;
    }
    /* VcmBSDF::pdf(dir, All & ~Specular, aEvalRevPdf = true) (BSDF.h:391-407) */
    __device__ float pdf_rev(f3 world_gen) const {
        const uint32_t mask = BX_ALL & ~BX_SPECULAR;
        const f3 wi = dg.to_local(world_gen);
        const float sum = sum_pick(mask);
        if (sum == 0.f) return 0.f;
        float pdf = 0.f;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            if (i < n && bx_match(bx[i].type, mask)) {
                float comp = 0.f;
                comp += bx_pdf(bx[i], fix, wi, true);
                pdf += comp * pick[i] / sum;
            }
        }
        return pdf;
    }
    /* VcmBSDF::vcmF (BSDF.h:488-541) */
    __device__ f3 vcm_f(f3 world_gen, float& cos_gen, float& dpdf, float& rpdf) const {
        const f3 gen = dg.to_local(world_gen);
        const f3 world_fix = dg.to_world(fix);
        dpdf = 0.f;
        rpdf = 0.f;
        if (fix.z < VCM_EPS_COSINE || gen.z < VCM_EPS_COSINE) return mk1(0.f);
        cos_gen = gen.z;
        uint32_t mask = BX_ALL;
        if (dot(gn, world_gen) * dot(gn, world_fix) >= 0.0f) mask &= ~BX_TRANSMISSION;
        else mask &= ~BX_REFLECTION;
        const float sum = sum_pick(mask);
        if (sum == 0.f) return mk1(0.f);
        f3 f = mk1(0.f);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            if (i < n && bx_match(bx[i].type, mask)) {
                float dp = 0.f, rp = 0.f;
                f = f + bx_vcm_f(bx[i], fix, gen, dp, rp);
                const float q = pick[i] / sum;
                dp *= q;
                rp *= q;
                dpdf += dp;
                rpdf += rp;
            }
        }
        return f;
    }
};

/* material vcmClosestHit{Light,Camera}: false = program ends the subpath */
/* kd: m.Kd, or the texel colour for Texture (Texture.cu:215-286) */
__device__ inline bool material_bsdf(const DevMaterial& m, f3 kd, f3 gn, f3 dir, bool is_light, VBsdf& s, f3& N) {
    switch (m.type) {
    case MAT_DIFFUSE:
    case MAT_TEXTURE:
        N = gn;
        s.init(gn, -dir, is_light);
        s.add(mk_bx(T_LAMBERT, kd));
        return true;
    case MAT_GLOSSY:
        N = gn;
        s.init(gn, -dir, is_light);
        s.add(mk_bx(T_LAMBERT, kd));
        s.add(mk_bx(T_PHONG, m.Ks, m.exponent));
        return true;
    case MAT_MIRROR:
        if (iszero(m.Kr)) return false;
        N = gn;
        s.init(gn, -dir, is_light);
        s.add(mk_bx(T_SREFL, m.Kr));
        return true;
    case MAT_GLASS: {
        const bool outside = dot(gn, dir) < 0;
        const f3 nn = outside ? gn : -gn;
        const float n1 = outside ? 1.f : m.ior, n2 = outside ? m.ior : 1.f;
        const bool krBlack = iszero(m.Kr), ktBlack = iszero(m.Kt);
        if (krBlack && ktBlack) return false;
        N = nn;
        s.init(nn, -dir, is_light);
        if (!ktBlack) s.add(mk_bx(T_STRANS, m.Kt, 0.f, n1, n2, true));
        if (!krBlack) s.add(mk_bx(T_SREFL, m.Kr, 0.f, n1, n2, true));
        return true;
    }
    default:
        return false;
    }
}

struct Subpath {
    f3 origin, direction, throughput, color;
    uint32_t depth;
    float dVCM, dVC, dVM;
    bool done;
};

__device__ __forceinline__ bool occluded(const DevScene& S, f3 p, f3 d, float tmax, uint32_t* stk) {
    if (tmax < 3.f * VCM_EPS_RAY) return false;
    return trace_any(S, p, d, VCM_EPS_RAY, tmax - 2.f * VCM_EPS_RAY, stk);
}
__device__ __forceinline__ void mis_on_hit(Subpath& p, float cosIn, float t) {
    p.dVCM *= t * t;
    p.dVCM /= cosIn;
    p.dVC /= cosIn;
    p.dVM /= cosIn;
}
/* sampleScattering (vcm.h:153-202) + updateMisTermsOnScatter (mis.h:110-160) */
__device__ inline void sample_scattering(Subpath& p, f3 hit, const VBsdf& bs, const VcmConsts& c, Rng& rs) {
    const float contProb = bs.cont;
    const float rrSample = rnd(rs);
    if (contProb < rrSample) { p.done = true; return; }
    float pdf = 0.f, cosOut = 0.f;
    const float s0 = rnd(rs);
    const float s1 = rnd(rs);
    const float s2 = rnd(rs);
    uint32_t ev = 0;
    const f3 f = bs.sample_f(s0, s1, s2, p.direction, pdf, cosOut, ev);
    if (iszero(f)) return;
    float rev = pdf;
    if (!bx_match(ev, BX_SPECULAR)) rev = bs.pdf_rev(p.direction);
    pdf *= contProb;
    rev *= contProb;
    if (ev & BX_SPECULAR) {
        p.dVCM = 0.f;
        p.dVC *= cosOut;
        p.dVM *= cosOut;
    } else {
        const float g = cosOut / pdf;
        p.dVC = g * (p.dVC * rev + p.dVCM + c.misVm);
        p.dVM = g * (p.dVM * rev + p.dVCM * c.misVc * 1.f + 1.f);
        p.dVCM = 1.f / pdf;
    }
    p.throughput = p.throughput * (f * (cosOut / pdf));
    p.origin = hit;
}

/* connectCameraT1 (vcm.h:52-150) without its shadow ray: true when the connection contributes,
 * with the ray (hit, dirToCamera, distance) and the splat (float offset in the owner-block
 * splat buffer, contribution) in the queue entry qa/qb/qc (LightShadowRays traces it) */
__device__ inline bool connect_camera_prep(const Subpath& L, const VBsdf& bs, f3 hit, const VcmConsts& c, float4& qa,
                                           float4& qb, float4& qc) {
    f3 dirToCamera = c.eye - hit;
    if (dot(c.lookdir, -dirToCamera) <= 0.f) return false;
    const float distance = length(dirToCamera);
    dirToCamera = dirToCamera / distance;
    const float cosAtCamera = dot(c.lookdirN, -dirToCamera);
    const float ipd = c.lookdirLen / cosAtCamera;
    const f3 ippw = c.eye + (-dirToCamera) * ipd;
    const f3 ipc = c.eye + c.lookdir;
    const f3 c2p = ippw - ipc;
    const float pu = dot(c2p, c.unitU);
    const float pv = dot(c2p, c.unitV);
    if (!(2.f * fabsf(pu) < c.ipsx && 2.f * fabsf(pv) < c.ipsy)) return false;
    const float pcx = (pu + 0.5f * c.ipsx) / c.ipsx;
    const float pcy = (pv + 0.5f * c.ipsy) / c.ipsy;
    uint32_t ix = orx_f2u_sat(pcx * (float)c.W), iy = orx_f2u_sat(pcy * (float)c.H);
    ix = ix > c.W - 1 ? c.W - 1 : ix;
    iy = iy > c.H - 1 ? c.H - 1 : iy;
    float cosToCamera = 0.f, dpdf, rpdf;
    const f3 f = bs.vcm_f(dirToCamera, cosToCamera, dpdf, rpdf);
    if (iszero(f)) return false;
    rpdf *= bs.cont;
    const float i2s = (ipd * ipd) / cosAtCamera;
    const float pixelArea = c.psfx * c.ipsx * c.psfx * c.ipsy;
    const float imageSamplePdfA = 1.f / pixelArea;
    const float cameraPdfW = imageSamplePdfA * i2s;
    const float cameraPdfA = cameraPdfW * fabsf(cosToCamera) / (distance * distance);
    const float wLight = (cameraPdfA / (float)c.count) * (c.misVm + L.dVCM + L.dVC * rpdf);
    const float misWeight = 1.f / (wLight + 1.f);
    const float conv = 1.f / cameraPdfA;
    const f3 contrib = ((L.throughput * misWeight) * f) / ((float)c.count * conv);
    /* owner-block layout [world][max_rows][W]: row iy belongs to rank iy % world */
    const uint32_t o = 3u * (uint32_t)(((size_t)(iy % c.world) * c.max_rows + iy / c.world) * c.W + ix);
    qa = make_float4(hit.x, hit.y, hit.z, distance);
    qb = make_float4(dirToCamera.x, dirToCamera.y, dirToCamera.z, __uint_as_float(o));
    qc = make_float4(contrib.x, contrib.y, contrib.z, 0.f);
    return true;
}
/* The light pass's queued camera connections for trace_any_chain (entries e = lane, lane + 64,
 * ... of q[3e .. 3e + 2]): occluded()'s test, and the unoccluded ones splat (atomic adds, as the
 * inline form: their order was never fixed) */
struct LightShadowRays {
    const float4* q;
    float* splat;
    uint32_t e, total, cur;
    uint32_t stride = 64;
    uint32_t splat_n = 0xffffffffu; /* floats in splat: a pixel offset past it is dropped (a list entry the
                                     * light pass did not write this iteration, k_vcm_light_shadow) */
    __device__ __forceinline__ void add(uint32_t k) const {
        const float4 b = q[3 * k + 1], cc = q[3 * k + 2];
        const uint32_t at = __float_as_uint(b.w);
        if (at >= splat_n || splat_n - at < 3u) return;
        float* o = splat + at;
        unsafeAtomicAdd(o + 0, cc.x);
        unsafeAtomicAdd(o + 1, cc.y);
        unsafeAtomicAdd(o + 2, cc.z);
    }
    __device__ __forceinline__ bool next(f3& o, f3& d, float& tmin, float& tmax) {
        while (e < total) {
            cur = e;
            e += stride;
            const float4 a = q[3 * cur], b = q[3 * cur + 1];
            if (a.w < 3.f * VCM_EPS_RAY) { /* occluded() without a walk: not occluded */
                add(cur);
                continue;
            }
            o = mk(a.x, a.y, a.z);
            d = mk(b.x, b.y, b.z);
            tmin = VCM_EPS_RAY;
            tmax = a.w - 2.f * VCM_EPS_RAY;
            return true;
        }
        return false;
    }
    __device__ __forceinline__ void result(bool occluded) {
        if (!occluded) add(cur);
    }
};

/* A wave's queue of camera connections (lq, n entries): appended to the deferred list vb.lcq when
 * there is one and it has room, else traced here and splatted at once */
__device__ __forceinline__ void light_queue_flush(const DevScene& S, const VcmBufs& vb, const float4* lq, uint32_t n,
                                                  uint32_t lane, uint32_t* stk) {
    __threadfence_block();
    if (vb.lcq) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&vb.lctl[0], n);
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)base, 0, 64));
        if (base <= vb.lcap && n <= vb.lcap - base) {
            for (uint32_t k = lane; k < 3 * n; k += 64) vb.lcq[3 * (size_t)base + k] = lq[k];
            return;
        }
        /* no room: the part of the reserved range below lcap gets inert entries (distance 0: no walk;
         * contribution 0 added to splat[0..2], which leaves every value as it is) */
        for (uint32_t k = lane; k < 3 * n; k += 64)
            if ((size_t)base * 3 + k < (size_t)vb.lcap * 3) vb.lcq[3 * (size_t)base + k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (lane == 0) atomicAdd(&vb.lctl[1], n);
    }
    LightShadowRays R{lq, vb.splat, lane, n, 0u};
    trace_any_chain(S, R, stk);
}

/* lightPass (VCMLightPass.cu:52-93), initLightPayload (:120-176), lightHit (vcm.h:210-309)
 *
 * Persistent waves with per-lane refill, as the camera pass below: a lane whose light
 * subpath has ended starts the next subpath of its wave's 64-subpath work item, one
 * bounce per round.  Each subpath's arithmetic and RNG stream are unchanged. */
/* TEX: the scene has Texture materials (vb.vE != NULL); the texel fetch is
 * compiled out otherwise, it costs the camera kernel ~10% through spills */
struct LightSub {
    uint32_t p;
    size_t slot;
    uint32_t nverts;
};
__device__ __forceinline__ void light_start(const DevScene& S, const VcmBufs& vb, const VcmConsts& c, uint32_t p,
                                            LightSub& ls, Rng& rs, Subpath& L) {
    const uint32_t x = p % c.W, j = p / c.W;
    ls.p = p;
    ls.slot = (size_t)j * vb.RW + x; /* RNG planes hold the own rows */
    ls.nverts = 0;
    rs = rng_load(vb.rng, ls.slot);
    L.throughput = mk1(1.f);
    L.color = mk1(0.f);
    L.depth = 0;
    L.done = false;
    int li = 0;
    if (1 < S.nl) {
        const float s = rnd(rs);
        li = (int)(s * (float)S.nl);
        li = li > (int)S.nl - 1 ? (int)S.nl - 1 : li;
    }
    const DevLight& light = S.lights[li];
    const float lightPickPdf = 1.f / (float)S.nl;
    float emissionPdfW, directPdfW, cosAtLight;
    f3 radiance;
    {   /* lightEmit (helpers/light.h:84-138) */
        const float dx = rnd(rs), dy = rnd(rs);
        if (light.type == LIGHT_AREA) {
            const float px = rnd(rs), py = rnd(rs);
            L.origin = light.position + light.v1 * px + light.v2 * py;
            const float theta = orx_acosf(sqrtf(dx));
            const float phi = 2.0f * ORX_PI_F * dy;
            const float st = orx_sinf(theta);
            const float xs = st * orx_cosf(phi);
            float ys = orx_cosf(theta);
            const float zs = st * orx_sinf(phi);
            f3 U, V;
            create_coordinate_system(light.normal, U, V);
            if (ys < VCM_EPS_COSINE) ys = VCM_EPS_COSINE;
            emissionPdfW = ys * ORX_1_PI_F;
            cosAtLight = ys;
            L.direction = normalize(U * xs + light.normal * ys + V * zs);
            emissionPdfW *= light.inverseArea;
            directPdfW = light.inverseArea;
            radiance = light.Lemit * cosAtLight;
        } else {
            L.origin = light.position;
            f3 toC = mk(S.bs_cx, S.bs_cy, S.bs_cz) - light.position;
            const float dist = length(toC);
            toC = toC / dist;
            if (S.bs_r < dist) {
                const float theta = orx_asinf(S.bs_r / dist);
                f3 U, V;
                create_coordinate_system(toC, U, V);
                const float cosTheta = orx_cosf(theta);
                const float z = cosTheta + (1.f - cosTheta) * dx;
                const float phi = 2 * ORX_PI_F * dy;
                const float rr = sqrtf(1.f - z * z);
                const float xx = rr * orx_cosf(phi);
                const float yy = rr * orx_sinf(phi);
                emissionPdfW = 1.f / (2.f * ORX_PI_F * (1.f - cosTheta));
                L.direction = normalize(U * xx + toC * z + V * yy);
            } else {
                L.direction = sample_unit_sphere(dx, dy);
                emissionPdfW = 0.25f * ORX_1_PI_F;
            }
            directPdfW = 1.f;
            cosAtLight = 1.f;
            radiance = light.Lemit;
        }
    }
    emissionPdfW *= lightPickPdf;
    directPdfW *= lightPickPdf;
    L.throughput = radiance / emissionPdfW;
    L.dVCM = directPdfW / emissionPdfW;
    L.dVC = light.type == LIGHT_AREA ? cosAtLight / emissionPdfW : 0.f;
    L.dVM = L.dVC * c.misVc;
}

#ifndef ORX_VCM_LIGHT_WAVES
#define ORX_VCM_LIGHT_WAVES 3 /* waves per SIMD the light kernel is register-capped for (4: 3.63 ms, 3: 3.33) */
#endif
template <bool ESTIMATE, bool TEX>
__global__ __launch_bounds__(64, ORX_VCM_LIGHT_WAVES) void k_vcm_light(DevScene S, VcmBufs vb, const VcmConsts* __restrict__ cp) {
    const VcmConsts& c = *cp;
    ORX_STACK_DECL;
    uint32_t* stk = ORX_STACK_PTR;
    const uint32_t lane = threadIdx.x & 63;
    LightSub ls;
    ls.p = 0;
    ls.slot = 0;
    ls.nverts = 0;
    Rng rs = {};
    Subpath L = {};
    bool alive = false;
    uint32_t next = 0, end = 0; /* the wave's current work item range (uniform) */
    bool exhausted = false;
    float4* lq = vb.shq + (size_t)blockIdx.x * VCM_SHQ_PER_WAVE; /* [128][3] queued camera connections */
    uint32_t lqn = 0;                                            /* queued (uniform) */
    for (;;) {
        for (;;) { /* refill: lanes without a subpath start the next ones of the wave's item */
            const uint64_t need = __ballot(!alive);
            if (!need) break;
            if (next >= end) {
                if (exhausted) break;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(vb.work + 1, 64u);
                base = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)base, 0, 64));
                if (base >= c.lcount) {
                    exhausted = true;
                    break;
                }
                next = base;
                end = base + 64u < c.lcount ? base + 64u : c.lcount;
            }
            const uint32_t avail = end - next;
            const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
            if (!alive && rank < avail) {
                light_start(S, vb, c, next + rank, ls, rs, L);
                alive = true;
            }
            const uint32_t n = (uint32_t)__popcll(need);
            next += n < avail ? n : avail;
        }
        if (!__ballot(alive)) break; /* only once the work is exhausted */
        /* one bounce */
        bool conn = false; /* this bounce's camera connection (connectCameraT1) is queued */
        float4 qa, qb, qc;
        if (alive) {
            bool end_path = false;
            Hit h;
            if (!trace_closest(S, L.origin, L.direction, VCM_RAY_LEN_MIN, RT_DEFAULT_MAX, h, stk)) {
                end_path = true;
            } else {
                const uint32_t mi = prim_material(S, h);
                const DevMaterial& m = S.mats[mi];
                const f3 hit = L.origin + L.direction * h.t;
                VBsdf bs;
                f3 N;
                const f3 kd = TEX && m.type == MAT_TEXTURE ? tex_color(S, m, h) : m.Kd;
                if (m.type == MAT_EMITTER || !material_bsdf(m, kd, geometric_normal(S, h), L.direction, true, bs, N)) {
                    end_path = true;
                } else {
                    L.depth++;
                    const float cosIn = dot(N, -L.direction);
                    if (cosIn < VCM_EPS_COSINE) {
                        end_path = true;
                    } else {
                        mis_on_hit(L, cosIn, h.t);
                        const bool spec = bs.is_specular();
                        if (!spec) {
                            const uint32_t k = ls.nverts++;
                            if (!ESTIMATE && k < VCM_MAX_VERTS) {
                                const size_t o = (size_t)k * c.lcount + ls.p;
                                vb.vA[o] = make_float4(hit.x, hit.y, hit.z, __uint_as_float(mi));
                                vb.vB[o] = make_float4(L.throughput.x, L.throughput.y, L.throughput.z, L.dVCM);
                                vb.vC[o] = make_float4(N.x, N.y, N.z, L.dVC);
                                vb.vD[o] = make_float4(bs.fix.x, bs.fix.y, bs.fix.z, L.dVM);
                                if (TEX && m.type == MAT_TEXTURE) vb.vE[o] = make_float4(kd.x, kd.y, kd.z, 0.f);
                            }
                            if (!ESTIMATE) conn = connect_camera_prep(L, bs, hit, c, qa, qb, qc);
                        }
                        if (c.maxPathLen < L.depth + 2) {
                            end_path = true;
                        } else {
                            sample_scattering(L, hit, bs, c, rs);
                            if (L.done) end_path = true;
                        }
                    }
                }
            }
            if (end_path) {
                vb.vcount[ls.p] = ls.nverts;
                rng_store(vb.rng, ls.slot, rs);
                alive = false;
            }
        }
        /* the connections' shadow rays wait in the wave's queue until 64 are pending, then all
         * lanes trace them, chained (traced in place, inside the divergent bounce, a wave ran
         * them at the lanes that happened to connect) */
        if (!ESTIMATE) {
            const uint64_t m = __ballot(conn);
            if (conn) {
                const uint32_t k = lqn + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                lq[3 * k] = qa;
                lq[3 * k + 1] = qb;
                lq[3 * k + 2] = qc;
            }
            lqn += (uint32_t)__popcll(m);
            if (lqn >= 64) {
                light_queue_flush(S, vb, lq, lqn, lane, stk);
                lqn = 0;
            }
        }
    }
    if (!ESTIMATE && lqn) light_queue_flush(S, vb, lq, lqn, lane, stk);
}


/* connectVertices (vcm.h:315-400) against light vertex k of this subpath */
template <bool TEX>
__device__ inline bool connect_vertex(const DevScene& S, const Subpath& C, const VBsdf& cb, f3 hit, const VcmBufs& vb,
                                      size_t o, const VcmConsts& c, f3& sdir, float& sdist, f3& add) {
    /* the vertex's planes and its material in flight together: loaded where first used, each
     * waited for a full memory latency after the BSDF work of the previous step (the empty asm
     * keeps the compiler from sinking them below the early return) */
    const float4 A = vb.vA[o], Cn = vb.vC[o], D = vb.vD[o];
    f3 direction = mk(A.x, A.y, A.z) - hit;
    const DevMaterial& m = S.mats[__float_as_uint(A.w)];
    const uint32_t mtype = m.type;
    const f3 mKd = m.Kd, mKs = m.Ks;
    const float mexp = m.exponent;
    const float dist2 = dot(direction, direction);
    const float distance = sqrtf(dist2);
    direction = direction / distance;
    float camCos = 0.f, cDir, cRev;
    const f3 camF = cb.vcm_f(direction, camCos, cDir, cRev);
    asm volatile("" ::"v"(Cn.x), "v"(Cn.y), "v"(Cn.z), "v"(Cn.w), "v"(D.x), "v"(D.y), "v"(D.z), "v"(mtype),
                 "v"(mKd.x), "v"(mKd.y), "v"(mKd.z));
    if (iszero(camF)) return false;
    cDir *= cb.cont;
    cRev *= cb.cont;
    VBsdf lb;
    const f3 N = mk(Cn.x, Cn.y, Cn.z);
    lb.dg = frame_from_normal(N);
    lb.gn = N;
    lb.fix_is_light = true;
    lb.fix = mk(D.x, D.y, D.z);
    lb.n = 0;
    lb.cont = 0.f;
    f3 kd = mKd;
    if (TEX && mtype == MAT_TEXTURE) { /* texel colour kept beside the 64-B record */
        const float4 E = vb.vE[o];
        kd = mk(E.x, E.y, E.z);
    }
    lb.add(mk_bx(T_LAMBERT, kd));
    if (mtype == MAT_GLOSSY) lb.add(mk_bx(T_PHONG, mKs, mexp));
    float lightCos = 0.f, lDir, lRev;
    const f3 lightF = lb.vcm_f(-direction, lightCos, lDir, lRev);
    if (iszero(lightF)) return false;
    lDir *= lb.cont;
    lRev *= lb.cont;
    const float geometryTerm = lightCos * camCos / dist2;
    if (geometryTerm < 0.f) return false;
    const float camDirPdfA = cDir * fabsf(camCos) / (distance * distance);
    const float lightDirPdfA = lDir * fabsf(lightCos) / (distance * distance);
    const float4 B = vb.vB[o];
    const float wLight = camDirPdfA * (c.misVm * 1.f + B.w + Cn.w * lRev);
    const float wCamera = lightDirPdfA * (c.misVm * 1.f + C.dVCM + C.dVC * cRev);
    const float misWeight = 1.f / (wLight + 1.f + wCamera);
    f3 contrib = ((camF * geometryTerm) * lightF) * 1.f;
    contrib = contrib * ((C.throughput * misWeight) * mk(B.x, B.y, B.z));
    sdir = direction; /* the caller traces occluded(hit, sdir, sdist) and adds `add` if clear */
    sdist = distance;
    add = contrib;
    return true;
}

/* connectLightSourceS1 (vcm.h:406-488) + lightIlluminate (helpers/light.h:141-203) */
__device__ inline bool connect_light(const DevScene& S, const Subpath& C, const VBsdf& cb, f3 hit, const VcmConsts& c,
                                     Rng& rs, f3& sdir, float& sdist, f3& add) {
    int li = 0;
    if (1 < S.nl) {
        const float s = rnd(rs);
        li = (int)(s * (float)S.nl);
        li = li > (int)S.nl - 1 ? (int)S.nl - 1 : li;
    }
    const DevLight& light = S.lights[li];
    const float lightPickProb = 1.f / (float)S.nl;
    float emissionPdfW, directPdfW, cosAtLight, distance;
    f3 dirToLight;
    if (light.type == LIGHT_AREA) {
        const float px = rnd(rs), py = rnd(rs);
        const f3 pl = light.position + light.v1 * px + light.v2 * py;
        dirToLight = pl - hit;
        distance = length(dirToLight);
        dirToLight = dirToLight / distance;
        const float cosThetaLight = dot(light.normal, -dirToLight);
        if (cosThetaLight < VCM_EPS_COSINE) return false;
        directPdfW = light.inverseArea * (distance * distance) / cosThetaLight;
        cosAtLight = cosThetaLight;
        emissionPdfW = light.inverseArea * cosThetaLight * ORX_1_PI_F;
    } else {
        dirToLight = light.position - hit;
        distance = length(dirToLight);
        dirToLight = dirToLight / distance;
        const f3 toC = mk(S.bs_cx, S.bs_cy, S.bs_cz) - light.position;
        const float d = length(toC);
        if (S.bs_r < d) {
            const float theta = orx_asinf(S.bs_r / d);
            emissionPdfW = 1.f / (2.f * ORX_PI_F * (1.f - orx_cosf(theta)));
        } else {
            emissionPdfW = 0.25f * ORX_1_PI_F;
        }
        directPdfW = distance * distance;
        cosAtLight = 1.f;
    }
    const f3 radiance = light.Lemit;
    if (iszero(radiance)) return false;
    float cosToLight = 0.f, bDir, bRev;
    const f3 f = cb.vcm_f(dirToLight, cosToLight, bDir, bRev);
    if (iszero(f)) return false;
    bDir *= light.type != LIGHT_AREA ? 0.f : cb.cont;
    bRev *= cb.cont;
    const float wLight = bDir / (lightPickProb * directPdfW);
    const float wCamera = (emissionPdfW * cosToLight / (directPdfW * cosAtLight)) * (c.misVm + C.dVCM + C.dVC * bRev);
    const float misWeight = 1.f / (wLight + 1.f + wCamera);
    const f3 contrib = (radiance * f) * (misWeight * cosToLight / (lightPickProb * directPdfW));
    if (iszero(contrib)) return false;
    sdir = dirToLight;
    sdist = distance;
    add = contrib * C.throughput;
    return true;
}

/* The camera pass's deferred shadow rays for trace_any_chain: entry e of the wave's compacted
 * list is row qqb[L] + e - qpb[L] of the lane L with qpb[L] <= e < qpb[L + 1] (binary search
 * over the lanes' pending-count prefix); a lane takes entries lane, lane + 64, ...  The test is
 * occluded()'s (segments shorter than 3 eps are unoccluded without a walk). */
struct CamShadowRays {
    float4* q;
    const float4* qhit;
    const uint32_t* pb;
    const uint32_t* qb;
    uint32_t e, total, row;
    __device__ __forceinline__ bool next(f3& o, f3& d, float& tmin, float& tmax) {
        while (e < total) {
            uint32_t L = 0;
#pragma unroll
            for (uint32_t st = 32; st; st >>= 1)
                if (pb[L + st] <= e) L += st;
            row = qb[L] + e - pb[L];
            e += 64;
            const float4 r0 = q[2 * row];
            if (r0.w < 3.f * VCM_EPS_RAY) {
                reinterpret_cast<float*>(q + 2 * row)[3] = -3.f;
                continue;
            }
            const float4 hp = qhit[__float_as_uint(q[2 * row + 1].w)];
            o = mk(hp.x, hp.y, hp.z);
            d = mk(r0.x, r0.y, r0.z);
            tmin = VCM_EPS_RAY;
            tmax = r0.w - 2.f * VCM_EPS_RAY;
            return true;
        }
        return false;
    }
    __device__ __forceinline__ void result(bool occluded) {
        reinterpret_cast<float*>(q + 2 * row)[3] = occluded ? -2.f : -3.f;
    }
};

/* cameraPass (VCMCameraPass.cu:48-80), initCameraPayload (:100-135), cameraHit (vcm.h:527-628)
 *
 * Persistent waves with per-lane refill: a wave takes 64-pixel work items (one 8x8 tile
 * each) from a device counter and a lane whose camera subpath has ended starts the next
 * pixel of the wave's item at the top of the following round, so the rounds stay full
 * instead of running, per wave, as long as its longest subpath (the one-pixel-per-lane
 * form measured a node-loop SIMT efficiency of 0.21).  Each subpath's arithmetic is
 * unchanged; only which lane runs it, and when, differs. */
#ifndef ORX_VCM_CAMERA_WAVES
#define ORX_VCM_CAMERA_WAVES 3 /* waves per SIMD the camera kernel is register-capped for: at 4 (128 VGPRs) it
                                 * spilled ~120 VGPRs to scratch, 7.00 ms against 6.37 at 3 (A/B: make vcm4) */
#endif
struct CamPixel {
    uint32_t p;
    size_t slot;
    uint32_t nverts;
};
template <int MODE>
__device__ __forceinline__ void camera_start(const VcmBufs& vb, const VcmConsts& c, uint32_t x, uint32_t j,
                                             CamPixel& px, Rng& rs, Subpath& C) {
    const uint32_t y = c.rank + j * c.world; /* own row j = image row rank + j*world */
    px.p = x + j * c.W;
    px.slot = (size_t)j * vb.RW + x;
    rs = rng_load(vb.rng, px.slot); /* MODE 2: vb.rng are the walk's rsave planes */
    if (MODE == 1) rng_store(vb.rsave, px.slot, rs); /* where an in-place rerun would start */
    C.throughput = mk1(1.0f);
    C.color = mk1(0.f);
    C.depth = 0;
    C.done = false;
    C.dVC = 0.f;
    C.dVM = 0.f;
    const float sx = rnd(rs), sy = rnd(rs);
    const float dx = ((float)x + sx) / (float)c.W * 2.0f - 1.0f;
    const float dy = ((float)y + sy) / (float)c.H * 2.0f - 1.0f;
    C.origin = c.eye;
    C.direction = normalize(c.u * dx + c.v * dy + c.lookdir);
    const float cosAtCamera = dot(c.lookdirN, C.direction);
    const float ipd = c.lookdirLen / cosAtCamera;
    const float i2s = (ipd * ipd) / cosAtCamera;
    const float pixelArea = c.psfx * c.ipsx * c.psfx * c.ipsy;
    const float areaSamplePdf = 1.f / pixelArea;
    const float cameraPdfW = areaSamplePdf * i2s;
    C.dVCM = (float)c.count / cameraPdfW;
    px.nverts = vb.vcount[px.p];
}
/* STORE_RNG false: the rerun, whose walk already left the RNG where the next light pass continues */
template <bool STORE_RNG>
__device__ __forceinline__ void camera_finish(const VcmBufs& vb, const CamPixel& px, const Rng& rs, const Subpath& C) {
    const size_t o3 = 3 * (size_t)px.p;
    vb.cam[o3 + 0] = C.color.x;
    vb.cam[o3 + 1] = C.color.y;
    vb.cam[o3 + 2] = C.color.z;
    const float ox = vb.output[o3 + 0] + vb.splat_in[o3 + 0];
    const float oy = vb.output[o3 + 1] + vb.splat_in[o3 + 1];
    const float oz = vb.output[o3 + 2] + vb.splat_in[o3 + 2];
    vb.output[o3 + 0] = ox + C.color.x;
    vb.output[o3 + 1] = oy + C.color.y;
    vb.output[o3 + 2] = oz + C.color.z;
    if (STORE_RNG) rng_store(vb.rng, px.slot, rs);
}

/* MODE 0: connection shadow rays traced in place (below); 1: the walk, connections deferred to
 * k_vcm_shadow and the colour summed by k_vcm_accum; 2: in place, only if the walk ran out of entries
 * (vb.dctl[1]), from the RNG words the walk started from (vb.rng = its rsave planes), without storing
 * the RNG.  A walk that runs out of entries finishes its subpaths without writing entries: its RNG use
 * does not depend on the shadow tests or the colour, so the RNG planes it leaves are right either way,
 * and only the colours need the rerun, which therefore runs in the resolve, off the RNG chain. */
#ifndef ORX_VCM_CAMERA_DEFER_WAVES
#define ORX_VCM_CAMERA_DEFER_WAVES 3 /* the deferred form (no traversal of the shadow rays inside) */
#endif
template <bool TEX, int MODE>
__global__ __launch_bounds__(64, MODE == 1 ? ORX_VCM_CAMERA_DEFER_WAVES : ORX_VCM_CAMERA_WAVES) void k_vcm_camera(DevScene S, VcmBufs vb, const VcmConsts* __restrict__ cp) {
    constexpr bool DEFER = MODE == 1;
    if (MODE == 2 && !vb.dctl[1]) return;
    const VcmConsts& c = *cp; /* read by scalar loads where used: as a by-value argument it kept ~40 more
                               * SGPRs live and the kernel spilled VGPRs */
    ORX_STACK_DECL;
    uint32_t* stk = ORX_STACK_PTR;
    const uint32_t tilesX = (c.W + 7) / 8;
    const uint32_t total = tilesX * ((c.rows + 7) / 8) * 64u; /* work item = tile * 64 + lane of the tile */
    const uint32_t lane = threadIdx.x & 63;
    /* The connections' shadow rays are deferred to a per-wave queue and traced
     * by all 64 lanes together (lanes whose subpath has ended help too): traced
     * in place, inside the divergent per-vertex loop, they ran at ~8 % lane
     * utilisation.  Every subpath still adds its unoccluded contributions in
     * the reference order (light sample, then light vertices 0..n-1), so the
     * colour is unchanged bit for bit. */
    __shared__ uint32_t qpb[64], qqb[64]; /* the lanes' pending-ray prefix and queue bases */
    float4* q = vb.shq + (size_t)blockIdx.x * VCM_SHQ_PER_WAVE;   /* [64 * 10][2] entries */
    float4* qhit = q + 2 * 64 * (VCM_MAX_VERTS + 1);              /* [64] connection points */
    CamPixel px;
    px.p = 0;
    px.slot = 0;
    px.nverts = 0;
    Rng rs = {};
    Subpath C = {};
    bool alive = false;
    uint32_t tail = VCM_END;  /* DEFER: the pixel's last entry so far */
    bool emis = false;        /* DEFER: the subpath ended on an emitter (its contribution is in C.color) */
    bool ovf = false;         /* DEFER: the entry list is full (wave-uniform); no more entries */
    uint32_t next = 0, end = 0; /* the wave's current work item range (uniform) */
    bool exhausted = false;
    for (;;) {
        /* refill: lanes without a subpath start the next pixels of the wave's item */
        for (;;) {
            const uint64_t need = __ballot(!alive);
            if (!need) break;
            if (next >= end) {
                if (exhausted) break;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(vb.work, 64u);
                base = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)base, 0, 64));
                if (base >= total) {
                    exhausted = true;
                    break;
                }
                next = base;
                end = base + 64u;
            }
            const uint32_t avail = end - next;
            const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
            if (!alive && rank < avail) {
                const uint32_t item = next + rank, tile = item >> 6;
                const uint32_t x = (tile % tilesX) * 8 + (item & 7), j = (tile / tilesX) * 8 + ((item >> 3) & 7);
                if (x < c.W && j < c.rows) {
                    camera_start<MODE>(vb, c, x, j, px, rs, C);
                    alive = true;
                    tail = VCM_END;
                    emis = false;
                }
            }
            const uint32_t n = (uint32_t)__popcll(need);
            next += n < avail ? n : avail;
        }
        const bool was_alive = alive;
        if (!__ballot(was_alive)) break; /* only once the work is exhausted */
        uint32_t npend = 0;
        bool spec = true, last = false;
        VBsdf bs;
        f3 hit = mk1(0.f);
        if (alive) {
            Hit h;
            if (!trace_closest(S, C.origin, C.direction, VCM_RAY_LEN_MIN, RT_DEFAULT_MAX, h, stk)) {
                alive = false;
            } else {
                const DevMaterial& m = S.mats[prim_material(S, h)];
                hit = C.origin + C.direction * h.t;
                if (m.type == MAT_EMITTER) { /* DiffuseEmitter.cu:95-120 + connectLightSourceS0 (vcm.h:493-522) */
                    alive = false;
                    C.depth++;
                    const f3 N = geometric_normal(S, h);
                    if (!iszero(m.Lemit) && !(dot(N, -C.direction) < 0.f)) {
                        const float lightPickProb = 1.f / (float)S.nl;
                        float directPdfA = m.inverseArea;
                        float emissionPdfW = maxf(0.f, dot(N, -C.direction)) * ORX_1_PI_F * m.inverseArea;
                        emis = true;
                        if (C.depth == 1) {
                            C.color = C.color + C.throughput * m.Lemit;
                        } else {
                            directPdfA *= lightPickProb;
                            emissionPdfW *= lightPickProb;
                            const float wCamera = directPdfA * C.dVCM + emissionPdfW * C.dVC;
                            const float misWeight = 1.f / (1.f + wCamera);
                            C.color = C.color + (C.throughput * misWeight) * m.Lemit;
                        }
                    }
                } else {
                    f3 N;
                    const f3 kd = TEX && m.type == MAT_TEXTURE ? tex_color(S, m, h) : m.Kd;
                    if (!material_bsdf(m, kd, geometric_normal(S, h), C.direction, false, bs, N)) {
                        alive = false;
                    } else {
                        C.depth++;
                        const float cosIn = dot(N, -C.direction);
                        if (cosIn < VCM_EPS_COSINE) {
                            alive = false;
                        } else {
                            mis_on_hit(C, cosIn, h.t);
                            spec = bs.is_specular();
                            last = c.maxPathLen <= C.depth;
                        }
                    }
                }
            }
        }
        /* connections of this vertex: pending shadow tests in the lane's rows */
        const bool conn = alive && !spec;
        uint32_t qbase = 0;
        {
            /* upper bound first (1 + n vertices), real count after building */
            const uint32_t nv = px.nverts < VCM_MAX_VERTS ? px.nverts : VCM_MAX_VERTS;
            const uint32_t want = conn ? 1u + nv : 0u;
            uint32_t incl = want;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= (uint32_t)o) incl += y;
            }
            qbase = incl - want;
            if (conn) {
                qhit[lane] = make_float4(hit.x, hit.y, hit.z, 0.f);
                f3 sd, ad;
                float sl;
                if (connect_light(S, C, bs, hit, c, rs, sd, sl, ad)) {
                    q[2 * (qbase + npend)] = make_float4(sd.x, sd.y, sd.z, sl);
                    q[2 * (qbase + npend) + 1] = make_float4(ad.x, ad.y, ad.z, __uint_as_float(lane));
                    npend++;
                }
                for (uint32_t k = 0; k < nv; ++k) {
                    if (connect_vertex<TEX>(S, C, bs, hit, vb, (size_t)k * c.lcount + px.p, c, sd, sl, ad)) {
                        q[2 * (qbase + npend)] = make_float4(sd.x, sd.y, sd.z, sl);
                        q[2 * (qbase + npend) + 1] = make_float4(ad.x, ad.y, ad.z, __uint_as_float(lane));
                        npend++;
                    }
                }
            }
            /* the next vertex's direction before the shadow tests: it consumes the RNG after
             * the connections (the reference order) and needs neither their outcome nor the
             * colour, and the BSDF is then dead during the traversals (fewer live registers) */
            if (alive) {
                if (last) {
                    alive = false;
                } else {
                    sample_scattering(C, hit, bs, c, rs);
                    if (C.done) alive = false;
                }
            }
            /* the wave's pending rays, compacted: entry e (of npend summed over the lanes) is row
             * qbase[L] + e - pbase[L] of the lane L with pbase[L] <= e < pbase[L] + npend[L] (the
             * largest lane with pbase[L] <= e), so every lane traces a ray in every round of the
             * loop below (the reserved rows of failed connections are skipped) */
            uint32_t pincl = npend;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(pincl, o, 64);
                if (lane >= (uint32_t)o) pincl += y;
            }
            const uint32_t pbase = pincl - npend;
            const uint32_t total_p = __shfl(pincl, 63, 64);
            if (DEFER) {
                /* the wave's connections go to the global entry list, each lane's in its reference order
                 * (light sample, then light vertices 0..n-1), linked behind the pixel's earlier ones */
                if (!ovf && total_p) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&vb.dctl[0], total_p);
                    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)base, 0, 64));
                    if (base > vb.dcap || total_p > vb.dcap - base) {
                        /* out of entries: the resolve reruns the pass in place (MODE 2); the wave walks on
                         * without entries, for the RNG the next light pass continues */
                        if (lane == 0) atomicOr(&vb.dctl[1], 1u);
                        ovf = true;
                    } else {
                        const uint32_t first = base + pbase;
                        const float4 hp4 = qhit[lane];
                        for (uint32_t k = 0; k < npend; ++k) {
                            const float4 r0 = q[2 * (qbase + k)];
                            const float4 r1 = q[2 * (qbase + k) + 1];
                            const uint32_t e = first + k;
                            vb.dq0[e] = make_float4(hp4.x, hp4.y, hp4.z, r0.w);
                            vb.dq1[e] = make_float4(r0.x, r0.y, r0.z, __uint_as_float(k + 1 < npend ? e + 1 : VCM_END));
                            vb.dq2[e] = make_float4(r1.x, r1.y, r1.z, 0.f);
                        }
                        if (npend) {
                            if (tail == VCM_END) vb.dhead[px.p] = first;
                            else reinterpret_cast<uint32_t*>(vb.dq1 + tail)[3] = first;
                            tail = first + npend - 1;
                        }
                    }
                }
                if (was_alive && !alive) {
                    /* camera_finish without the colour: RNG, the emitter term, the list end */
                    rng_store(vb.rng, px.slot, rs);
                    vb.demis[px.p] = make_float4(C.color.x, C.color.y, C.color.z, emis ? 1.f : 0.f);
                    if (tail == VCM_END) vb.dhead[px.p] = VCM_END;
                }
                continue;
            }
            qpb[lane] = pbase;
            qqb[lane] = qbase;
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            /* all lanes trace the wave's shadow rays (lane l: entries l, l + 64, ..., chained in
             * one traversal loop); the result goes into .w of the contribution row */
            {
                CamShadowRays R{q, qhit, qpb, qqb, lane, total_p, 0u};
#ifndef ORX_VCM_NO_SHADOW
                trace_any_chain(S, R, stk);
#else /* timing A/B only (make variant NAME=noshadow DEFS=-DORX_VCM_NO_SHADOW): every connection unoccluded */
                f3 o_, d_;
                float a_, b_;
                while (R.next(o_, d_, a_, b_)) R.result(false);
#endif
            }
            __threadfence_block();
            for (uint32_t k = 0; k < npend; ++k) {
                const float4 r0 = q[2 * (qbase + k)];
                const float4 r1 = q[2 * (qbase + k) + 1];
                if (r0.w == -3.f) C.color = C.color + mk(r1.x, r1.y, r1.z);
            }
        }
        if (was_alive && !alive) camera_finish<MODE != 2>(vb, px, rs, C);
    }
}

/* The camera pass's deferred connection shadow rays (k_vcm_camera<TEX, 1>), traced by a lean
 * any-hit kernel at the occupancy its registers allow: in the camera kernel they ran at its 3 waves
 * per SIMD and took 2.96 of its 6.21 ms on the hall (timing A/B against a build that skips them).
 * Entry e of the list goes to lane e mod (grid lanes); a lane chains its entries in one traversal
 * loop (trace_any_chain).  The test is occluded()'s (vcm.h:43-58): a segment shorter than 3 eps is
 * unoccluded without a walk. */
struct DeferredShadowRays {
    const float4* dq0;
    const float4* dq1;
    uint8_t* occ;
    uint32_t e, n, stride, cur;
    __device__ __forceinline__ bool next(f3& o, f3& d, float& tmin, float& tmax) {
        while (e < n) {
            cur = e;
            e += stride;
            const float4 a = dq0[cur];
            if (a.w < 3.f * VCM_EPS_RAY) {
                occ[cur] = 0;
                continue;
            }
            const float4 b = dq1[cur];
            o = mk(a.x, a.y, a.z);
            d = mk(b.x, b.y, b.z);
            tmin = VCM_EPS_RAY;
            tmax = a.w - 2.f * VCM_EPS_RAY;
            return true;
        }
        return false;
    }
    __device__ __forceinline__ void result(bool occluded) { occ[cur] = occluded ? 1 : 0; }
};
#ifndef ORX_VCM_SHADOW_WAVES
#define ORX_VCM_SHADOW_WAVES 8
#endif
constexpr int VCM_SHADOW_LDS_STACK = 16; /* LDS entries per lane; deeper ones in vb.shstk */
uint32_t vcm_shadow_stack_deep(uint32_t entries) { return StackH<VCM_SHADOW_LDS_STACK>::deep(entries); }
/* the light pass's deferred camera connections (vb.lcq), traced and splatted before the camera
 * pass's colours read the light image (launch_vcm_camera_resolve) */
__global__ __launch_bounds__(64, ORX_VCM_SHADOW_WAVES) void k_vcm_light_shadow(DevScene S, VcmBufs vb) {
    ORX_STACK_DECL;
    const uint32_t n = min(vb.lctl[0], vb.lcap);
    LightShadowRays R{vb.lcq, vb.splat, blockIdx.x * 64u + threadIdx.x, n, 0u, gridDim.x * 64u, vb.splat_n};
    const StackH<VCM_SHADOW_LDS_STACK> stk{ORX_STACK_PTR, vb.shstk, blockIdx.x, vb.shdeep, threadIdx.x};
    trace_any_chain_t(S, R, stk);
}
__global__ __launch_bounds__(64, ORX_VCM_SHADOW_WAVES) void k_vcm_shadow(DevScene S, VcmBufs vb) {
    if (blockIdx.x == 0 && threadIdx.x == 0) vb.work[2] = 0; /* the rerun's work counter (it follows on this stream) */
    if (vb.dctl[1]) return; /* out of entries: the camera pass reruns in place */
    ORX_STACK_DECL;
    const uint32_t n = min(vb.dctl[0], vb.dcap);
    const uint32_t gid = blockIdx.x * 64u + threadIdx.x;
    DeferredShadowRays R{vb.dq0, vb.dq1, vb.docc, gid, n, gridDim.x * 64u, 0u};
    const StackH<VCM_SHADOW_LDS_STACK> stk{ORX_STACK_PTR, vb.shstk, blockIdx.x, vb.shdeep, threadIdx.x};
    trace_any_chain_t(S, R, stk);
}
/* the colour of every own pixel's camera subpath from its deferred entries, in the order the
 * in-place pass adds them (C.color = C.color + contribution for each unoccluded connection, then the
 * emitter term), then camera_finish's writes */
__global__ __launch_bounds__(256) void k_vcm_accum(VcmBufs vb, uint32_t lcount, uint32_t max_per_px) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= lcount || vb.dctl[1]) return;
    /* the walk writes every own pixel's head and links only to entries below the count it reserved, so
     * these bounds hold by construction; they keep a list the walk did not write this pass (stale heads,
     * a stale count) from leading the loop outside the entries or round a cycle */
    const uint32_t n = min(vb.dctl[0], vb.dcap);
    f3 color = mk1(0.f);
    uint32_t steps = 0;
    for (uint32_t e = vb.dhead[p]; e < n && steps < max_per_px; e = __float_as_uint(vb.dq1[e].w), ++steps)
        if (!vb.docc[e]) {
            const float4 a = vb.dq2[e];
            color = color + mk(a.x, a.y, a.z);
        }
    const float4 em = vb.demis[p];
    if (em.w != 0.f) color = color + mk(em.x, em.y, em.z);
    const size_t o3 = 3 * (size_t)p;
    vb.cam[o3 + 0] = color.x;
    vb.cam[o3 + 1] = color.y;
    vb.cam[o3 + 2] = color.z;
    const float ox = vb.output[o3 + 0] + vb.splat_in[o3 + 0];
    const float oy = vb.output[o3 + 1] + vb.splat_in[o3 + 1];
    const float oz = vb.output[o3 + 2] + vb.splat_in[o3 + 2];
    vb.output[o3 + 0] = ox + color.x;
    vb.output[o3 + 1] = oy + color.y;
    vb.output[o3 + 2] = oz + color.z;
}
/* persistent light-pass waves: as many as can be resident at once (4 per SIMD) */
uint32_t vcm_light_waves(uint32_t items) {
    static uint32_t resident = 0;
    if (!resident) {
        int dev = 0, cus = 256;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        resident = (uint32_t)cus * 4u * ORX_VCM_LIGHT_WAVES;
    }
    return items < resident ? items : resident;
}
/* persistent camera-pass waves: as many as can be resident at once */
uint32_t vcm_camera_waves(uint32_t tiles) {
    static uint32_t resident = 0;
    if (!resident) {
        int dev = 0, cus = 256;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        resident = (uint32_t)cus * 4u * ORX_VCM_CAMERA_WAVES;
    }
    return tiles < resident ? tiles : resident;
}

/* a pass's prologue, one thread: the constants' device copies and the small control words the pass
 * counts in (work-item counters, entry-list control words), zeroed here instead of by separate
 * fill dispatches on the iteration's critical chain */
struct VcmZero {
    uint32_t* p[2] = {nullptr, nullptr};
    uint32_t n[2] = {0, 0};
};
__global__ void k_vcm_consts(VcmConsts c, VcmConsts* dst, VcmConsts* keep, VcmZero z) {
    *dst = c;
    if (keep) *keep = c;
    for (int i = 0; i < 2; i++)
        for (uint32_t k = 0; k < z.n[i]; k++) z.p[i][k] = 0;
}

void launch_vcm_light(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c, bool estimate) {
    VcmZero z;
    z.p[0] = vb.work + 1; /* the light pass's work counter */
    z.n[0] = 1;
    if (!estimate && vb.lcq) { /* the deferred camera connections: entries reserved, entries traced in place */
        z.p[1] = vb.lctl;
        z.n[1] = 2;
    }
    hipLaunchKernelGGL(k_vcm_consts, dim3(1), dim3(1), 0, s, c, vb.consts, (VcmConsts*)nullptr, z);
    const uint32_t blocks = vcm_light_waves((c.lcount + 63) / 64);
    if (blocks == 0) return;
    const size_t lds = ORX_STACK_BYTES(S);
    if (vb.vE) {
        if (estimate) hipLaunchKernelGGL((k_vcm_light<true, true>), dim3(blocks), dim3(64), lds, s, S, vb, vb.consts);
        else hipLaunchKernelGGL((k_vcm_light<false, true>), dim3(blocks), dim3(64), lds, s, S, vb, vb.consts);
    } else {
        if (estimate) hipLaunchKernelGGL((k_vcm_light<true, false>), dim3(blocks), dim3(64), lds, s, S, vb, vb.consts);
        else hipLaunchKernelGGL((k_vcm_light<false, false>), dim3(blocks), dim3(64), lds, s, S, vb, vb.consts);
    }
}
template <int MODE>
static void launch_camera_kernel(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts* cp,
                                 uint32_t blocks) {
    if (vb.vE) hipLaunchKernelGGL((k_vcm_camera<true, MODE>), dim3(blocks), dim3(64), ORX_STACK_BYTES(S), s, S, vb, cp);
    else hipLaunchKernelGGL((k_vcm_camera<false, MODE>), dim3(blocks), dim3(64), ORX_STACK_BYTES(S), s, S, vb, cp);
}
/* The camera pass in two parts.  The walk (k_vcm_camera<., 1>): everything that reads or advances the RNG
 * planes, reads the light vertices or the pass constants -- the subpaths, their connections written to the
 * entry list, and the RNG words each subpath starts from (vb.rsave).  The resolve: the light pass's
 * deferred camera connections (k_vcm_light_shadow, splats into the light image), the entries' shadow rays
 * (k_vcm_shadow), the colours (k_vcm_accum), and -- only if the walk ran out of entries (more than vb.dcap
 * connections in all, ORX_VCM_DEFER per own pixel) -- the in-place rerun k_vcm_camera<., 2>, which starts
 * from vb.rsave, reads this iteration's light vertices and constants (vb.consts_keep) and the finished light
 * image, and accumulates into the output; k_vcm_shadow and k_vcm_accum exit at once after an overflow, the
 * rerun otherwise.  The resolve reads nothing the next iteration's light pass and walk write (their light
 * vertices, light image, entry list, rsave and constants copy are the other set, orx_capi.hip
 * vcm_iteration), so it runs beside them (orx_capi.hip vcm_camera).  vb.dq0 == NULL: in place only. */
void launch_vcm_camera_walk(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c) {
    VcmZero z;
    z.p[0] = vb.work; /* the camera pass's work counter */
    z.n[0] = 1;
    if (vb.dq0) { /* entries reserved, overflow flag */
        z.p[1] = vb.dctl;
        z.n[1] = 4;
    }
    hipLaunchKernelGGL(k_vcm_consts, dim3(1), dim3(1), 0, s, c, vb.consts, vb.dq0 ? vb.consts_keep : nullptr, z);
    const uint32_t blocks = vcm_camera_waves(((c.W + 7) / 8) * ((c.rows + 7) / 8));
    if (blocks == 0) return;
    if (!vb.dq0) launch_camera_kernel<0>(s, S, vb, vb.consts, blocks);
    else launch_camera_kernel<1>(s, S, vb, vb.consts, blocks);
}
void launch_vcm_camera_resolve(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c) {
    if (!vb.dq0 || c.W == 0 || c.rows == 0) return;
    static const uint32_t cus = [] {
        int dev = 0, n = 256;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return (uint32_t)n;
    }();
    /* persistent one-wave blocks: half as many as can be resident at once (the register cap, or the short
     * LDS stacks, 160 KB per CU), so the next iteration's light pass and camera walk beside them keep room:
     * the stand-alone resolve is as fast, the overlapped frame +0.3 % (hall 581.5 -> 583.3 Mpaths/s over four
     * alternating runs; a quarter is 9 % slower; profiles/r06zm_vcm_shadow_frac_ab.txt, ORX_VCM_SHADOW_FRAC);
     * vb.shstk holds the deeper entries of that many lanes */
    const size_t lds = (size_t)(VCM_SHADOW_LDS_STACK + 2) * 64 * 4;
    const uint32_t per_cu = std::min<uint32_t>(4u * ORX_VCM_SHADOW_WAVES, (uint32_t)((160u << 10) / lds));
    static const float frac = [] { /* the fraction of the resident capacity */
        const char* e = getenv("ORX_VCM_SHADOW_FRAC");
        const float f = e ? (float)atof(e) : 0.5f;
        return f > 0.f && f <= 1.f ? f : 1.f;
    }();
    const uint32_t sblocks = std::max(1u, (uint32_t)((float)std::min(cus * std::max(1u, per_cu), vb.shstk_lanes / 64u) * frac));
    if (vb.lcq) hipLaunchKernelGGL(k_vcm_light_shadow, dim3(sblocks), dim3(64), lds, s, S, vb);
    hipLaunchKernelGGL(k_vcm_shadow, dim3(sblocks), dim3(64), lds, s, S, vb); /* also zeroes work[2] */
    /* a pixel's list holds at most (1 + VCM_MAX_VERTS) connections per camera vertex */
    const uint32_t max_per_px = (c.maxPathLen + 1) * (1 + VCM_MAX_VERTS);
    hipLaunchKernelGGL(k_vcm_accum, dim3((c.lcount + 255) / 256), dim3(256), 0, s, vb, c.lcount, max_per_px);
    const uint32_t blocks = vcm_camera_waves(((c.W + 7) / 8) * ((c.rows + 7) / 8));
    if (blocks == 0) return;
    VcmBufs rv = vb; /* the rerun: RNG from the walk's start words, its own queues and work counter */
    rv.rng = vb.rsave;
    rv.shq = vb.shq_rerun;
    rv.work = vb.work + 2;
    launch_camera_kernel<2>(s, S, rv, vb.consts_keep, blocks);
}
void launch_vcm_camera(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c) {
    launch_vcm_camera_walk(s, S, vb, c);
    launch_vcm_camera_resolve(s, S, vb, c);
}

}  // namespace orx
