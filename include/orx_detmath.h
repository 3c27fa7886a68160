/*
 * orx_detmath.h — deterministic single-precision math for the orx render core.
 *
 * The reference compiles every OptiX program with nvcc -use_fast_math
 * (RenderEngine/RenderEngine.vcxproj:129), i.e. __sinf/__cosf/__expf/__powf
 * hardware approximations that neither an x86 host nor gfx950 can reproduce.
 * Progressive photon mapping and path tracing are chaotic in their control
 * flow (Russian roulette, Fresnel picks), so a 1-ulp difference between the
 * CPU oracle and the GPU kernels would fork whole paths and blow the 1e-4
 * rel-L2 parity bar.  This header therefore DEFINES the transcendental
 * functions the renderer uses, built only from IEEE-754 +,-,*,/,sqrt and
 * integer bit operations.  Both the HIP kernels and the C oracle are
 * compiled with -ffp-contract=off (no FMA contraction) and correctly rounded
 * fp32 division/sqrt (hipcc default, verified in the gfx950 ISA), so every
 * function below returns bit-identical results on host and device.
 *
 * Accuracy (checked against libm in tests/test_detmath.py): sin/cos/exp/acos
 * within a few ulp over the ranges the renderer feeds them; pow is evaluated
 * in double and rounded to float.
 *
 * Portable C99 / HIP C++.  Every function is `static inline` and tagged
 * ORX_HD so the same text compiles for the host and for gfx950.
 */
#ifndef ORX_DETMATH_H
#define ORX_DETMATH_H

#include <stddef.h>
#include <stdint.h>
#if !defined(__HIPCC__)
#include <math.h>
#endif

#if defined(__HIPCC__)
#define ORX_HD __host__ __device__
#else
#define ORX_HD
#endif

#ifdef __cplusplus
extern "C++" {
#endif

#define ORX_PI_F 3.14159265358979323846f   /* optix M_PIf */
#define ORX_1_PI_F 0.318309886183790671538f /* optix M_1_PIf */
#define ORX_FLT_EPSILON 1.19209290e-7f

static inline ORX_HD float orx_as_float(uint32_t u) {
    union { uint32_t u; float f; } c; c.u = u; return c.f;
}
static inline ORX_HD uint32_t orx_as_uint(float f) {
    union { uint32_t u; float f; } c; c.f = f; return c.u;
}
static inline ORX_HD double orx_as_double(uint64_t u) {
    union { uint64_t u; double d; } c; c.u = u; return c.d;
}
static inline ORX_HD uint64_t orx_as_u64(double d) {
    union { uint64_t u; double d; } c; c.d = d; return c.u;
}

/* floor without relying on libm: exact for every float (v_floor_f32 on gfx950
 * is exact too, so device code uses it). */
static inline ORX_HD float orx_floorf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_floorf(x);
#endif
    if (!(x < 8388608.0f && x > -8388608.0f)) return x; /* |x| >= 2^23 or NaN: integral */
    int32_t i = (int32_t)x;                               /* truncation toward zero */
    float t = (float)i;
    return (t > x) ? t - 1.0f : t;
}
static inline ORX_HD float orx_ceilf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_ceilf(x);
#endif
    if (!(x < 8388608.0f && x > -8388608.0f)) return x;
    int32_t i = (int32_t)x;
    float t = (float)i;
    return (t < x) ? t + 1.0f : t;
}

/* CUDA cvt.rzi.{s32,u32}.f32 semantics: truncate, saturate, NaN -> 0.
 * C leaves out-of-range float->int conversion undefined; the reference relies
 * on the CUDA behaviour (IndirectRadianceEstimation.cu:86-92). */
static inline ORX_HD int32_t orx_f2i_sat(float x) {
    if (!(x == x)) return 0;
    if (x >= 2147483648.0f) return 2147483647;
    if (x <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)x;
}
static inline ORX_HD uint32_t orx_f2u_sat(float x) {
    if (!(x > 0.0f)) return 0u; /* negatives, -0, NaN */
    if (x >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)x;
}

/* ---- sin / cos : Cody-Waite reduction by pi/2, minimax on [-pi/4, pi/4] ---- */
#define ORX_PIO2_1 1.5703125f
#define ORX_PIO2_2 4.837512969970703125e-4f
#define ORX_PIO2_3 7.54978995489188216e-8f
#define ORX_2_PI 0.636619772367581343076f

static inline ORX_HD float orx_sin_poly(float r) {
    float z = r * r;
    float p = -1.9515295891e-4f;
    p = p * z + 8.3321608736e-3f;
    p = p * z + -1.6666654611e-1f;
    return r + (r * z) * p;
}
static inline ORX_HD float orx_cos_poly(float r) {
    float z = r * r;
    float p = 2.443315711809948e-5f;
    p = p * z + -1.388731625493765e-3f;
    p = p * z + 4.166664568298827e-2f;
    return (1.0f - 0.5f * z) + (z * z) * p;
}
/* quadrant-reduced argument: returns r, writes quadrant k mod 4 */
static inline ORX_HD float orx_reduce_pio2(float x, int32_t* q) {
    float kf = orx_floorf(x * ORX_2_PI + 0.5f);
    float r = x - kf * ORX_PIO2_1;
    r = r - kf * ORX_PIO2_2;
    r = r - kf * ORX_PIO2_3;
    *q = ((int32_t)kf) & 3;
    return r;
}
static inline ORX_HD float orx_sinf(float x) {
    int32_t q;
    float r = orx_reduce_pio2(x, &q);
    float s;
    switch (q) {
    case 0: s = orx_sin_poly(r); break;
    case 1: s = orx_cos_poly(r); break;
    case 2: s = -orx_sin_poly(r); break;
    default: s = -orx_cos_poly(r); break;
    }
    return s;
}
static inline ORX_HD float orx_cosf(float x) {
    int32_t q;
    float r = orx_reduce_pio2(x, &q);
    float c;
    switch (q) {
    case 0: c = orx_cos_poly(r); break;
    case 1: c = -orx_sin_poly(r); break;
    case 2: c = -orx_cos_poly(r); break;
    default: c = orx_sin_poly(r); break;
    }
    return c;
}

/* ---- exp : Cody-Waite by ln2, degree-6 polynomial on [-ln2/2, ln2/2] ---- */
/* Branch-free core, exact same arithmetic as orx_expf for x in [-87, 88]
 * (normal results); the photon-gather weight only feeds it [-1, 0]. */
static inline ORX_HD float orx_expf_core(float x) {
    float kf = orx_floorf(x * 1.44269504088896341f + 0.5f);
    float r = x - kf * 0.693359375f;
    r = r - kf * -2.12194440e-4f;
    float p = 1.9875691500e-4f;
    p = p * r + 1.3981999507e-3f;
    p = p * r + 8.3334519073e-3f;
    p = p * r + 4.1665795894e-2f;
    p = p * r + 1.6666665459e-1f;
    p = p * r + 5.0000001201e-1f;
    float e = (r + (r * r) * p) + 1.0f;
    int32_t k = (int32_t)kf;
    return e * orx_as_float((uint32_t)(k + 127) << 23);
}
/* exp(x) for x in [-1, 0]: the photon-gather kernel weight's only input range
 * (IndirectRadianceEstimation.cu:59-67: x = -beta*d^2/(2r^2), d^2 <= r^2,
 * beta = 1.953).  One Horner chain of degree 6 (least-squares fit in relative
 * error, c0 = 1 so w(0) = alpha exactly): <= 3.5 ulp, mean 0.5 ulp against
 * exp — the reference's fast-math __expf is itself ~2 ulp — with no range
 * reduction, so the gather evaluates it with packed fp32 math.  Oracle and
 * kernels evaluate the same operation sequence (no FMA contraction). */
#define ORX_EXPU_C1 0.9999984502792358f
#define ORX_EXPU_C2 0.49997302889823914f
#define ORX_EXPU_C3 0.16650275886058807f
#define ORX_EXPU_C4 0.04119604453444481f
#define ORX_EXPU_C5 0.007628436665982008f
#define ORX_EXPU_C6 0.0008400468504987657f
static inline ORX_HD float orx_expf_unit(float x) {
    float p = ORX_EXPU_C6;
    p = p * x + ORX_EXPU_C5;
    p = p * x + ORX_EXPU_C4;
    p = p * x + ORX_EXPU_C3;
    p = p * x + ORX_EXPU_C2;
    p = p * x + ORX_EXPU_C1;
    return p * x + 1.0f;
}
static inline ORX_HD float orx_expf(float x) {
    if (!(x == x)) return x;
    if (x > 88.72283f) return orx_as_float(0x7f800000u);
    if (x < -103.0f) return 0.0f;
    float kf = orx_floorf(x * 1.44269504088896341f + 0.5f);
    float r = x - kf * 0.693359375f;
    r = r - kf * -2.12194440e-4f;
    float p = 1.9875691500e-4f;
    p = p * r + 1.3981999507e-3f;
    p = p * r + 8.3334519073e-3f;
    p = p * r + 4.1665795894e-2f;
    p = p * r + 1.6666665459e-1f;
    p = p * r + 5.0000001201e-1f;
    float e = (r + (r * r) * p) + 1.0f;
    int32_t k = (int32_t)kf;
    /* scale by 2^k in two steps so that subnormal results stay exact-ish */
    if (k < -125) {
        e = e * orx_as_float((uint32_t)(k + 127 + 64) << 23);
        return e * orx_as_float((uint32_t)(127 - 64) << 23);
    }
    if (k > 127) {
        e = e * 2.0f;
        k -= 1;
    }
    return e * orx_as_float((uint32_t)(k + 127) << 23);
}

/* ---- asin / acos (cephes-style) ---- */
static inline ORX_HD float orx_asin_core(float x) { /* |x| <= 0.5 */
    float z = x * x;
    float p = 4.2163199048e-2f;
    p = p * z + 2.4181311049e-2f;
    p = p * z + 4.5470025998e-2f;
    p = p * z + 7.4953002686e-2f;
    p = p * z + 1.6666752422e-1f;
    return x + (x * z) * p;
}
static inline ORX_HD float orx_asinf(float x) {
    float a = x < 0.0f ? -x : x;
    float r;
    if (a > 1.0f) return orx_as_float(0x7fc00000u);
    if (a > 0.5f) {
        float z = 0.5f * (1.0f - a);
        float s = sqrtf(z);
        r = 1.57079632679489661923f - 2.0f * orx_asin_core(s);
    } else {
        r = orx_asin_core(a);
    }
    return x < 0.0f ? -r : r;
}
static inline ORX_HD float orx_acosf(float x) {
    if (x < -1.0f || x > 1.0f) return orx_as_float(0x7fc00000u);
    if (x < -0.5f) {
        float s = sqrtf(0.5f * (1.0f + x));
        return ORX_PI_F - 2.0f * orx_asin_core(s);
    }
    if (x > 0.5f) {
        float s = sqrtf(0.5f * (1.0f - x));
        return 2.0f * orx_asin_core(s);
    }
    return 1.57079632679489661923f - orx_asin_core(x);
}

/* ---- pow : evaluated in double (log via atanh series, exp via Cody-Waite) ---- */
static inline ORX_HD double orx_log_d(double x) { /* x > 0, finite, normal */
    uint64_t b = orx_as_u64(x);
    int32_t e = (int32_t)((b >> 52) & 0x7ff) - 1023;
    double m = orx_as_double((b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL); /* [1,2) */
    if (m > 1.41421356237309504880) { m = m * 0.5; e += 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
    double t = 1.0 / 19.0;
    t = t * s2 + 1.0 / 17.0;
    t = t * s2 + 1.0 / 15.0;
    t = t * s2 + 1.0 / 13.0;
    t = t * s2 + 1.0 / 11.0;
    t = t * s2 + 1.0 / 9.0;
    t = t * s2 + 1.0 / 7.0;
    t = t * s2 + 1.0 / 5.0;
    t = t * s2 + 1.0 / 3.0;
    t = t * s2 + 1.0;
    double lm = 2.0 * s * t;
    return (double)e * 0.693147180559945309417 + lm;
}
static inline ORX_HD double orx_exp_d(double x) {
    if (x > 709.0) return orx_as_double(0x7ff0000000000000ULL);
    if (x < -745.0) return 0.0;
    double kd = x * 1.44269504088896340736 + 0.5;
    /* floor for doubles in range */
    int64_t ki = (int64_t)kd;
    if ((double)ki > kd) ki -= 1;
    double k = (double)ki;
    double r = x - k * 6.93147180369123816490e-01;
    r = r - k * 1.90821492927058770002e-10;
    double p = 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    int64_t kk = ki;
    double scale = 1.0;
    if (kk < -1000) { scale = orx_as_double(((uint64_t)(1023 - 1000)) << 52); kk += 1000; }
    return p * orx_as_double(((uint64_t)(kk + 1023)) << 52) * scale;
}
/* logf(x) through the double log (ParticipatingMedium.cu:138's scatter distance); log(0) = -inf */
static inline ORX_HD float orx_logf(float x) {
    if (x == 0.0f) return -orx_as_float(0x7f800000u);
    if (!(x > 0.0f)) return orx_as_float(0x7fc00000u);
    if (x == orx_as_float(0x7f800000u)) return x;
    return (float)orx_log_d((double)x);
}
static inline ORX_HD float orx_powf(float x, float y) {
    if (y == 0.0f) return 1.0f;
    if (x == 1.0f) return 1.0f;
    if (!(x == x) || !(y == y)) return orx_as_float(0x7fc00000u);
    if (x == 0.0f) return y > 0.0f ? 0.0f : orx_as_float(0x7f800000u);
    if (x < 0.0f) return orx_as_float(0x7fc00000u); /* renderer never raises negatives */
    double l = orx_log_d((double)x);
    return (float)orx_exp_d((double)y * l);
}

/* tex2D(sampler, u, v) for rtTextureSampler<uchar4, 2, cudaReadModeNormalizedFloat>
 * with RT_WRAP_REPEAT, RT_FILTER_LINEAR and normalised coordinates
 * (Texture.cpp:109-122), restating the CUDA programming guide's texture
 * fetching rules: wrap u -> u - floor(u), x_B = u*W - 0.5, i = floor(x_B),
 * alpha = frac(x_B) held in 9-bit fixed point with 8 fractional bits (rounded
 * here), texel indices wrapped, texels read as byte / 255, and
 *   (1-a)(1-b) T[i,j] + a(1-b) T[i+1,j] + (1-a)b T[i,j+1] + ab T[i+1,j+1].
 * `rgba` holds w*h RGBA8 texels, row j at rgba + 4*w*j, 4-byte aligned.  Non-finite
 * coordinates sample texel (0,0).  Parity unpinned (no CUDA here). */
static inline ORX_HD void orx_tex2d_linear(const uint8_t* rgba, uint32_t w, uint32_t h, float u, float v,
                                           float out[4]) {
    if (!(u - u == 0.0f)) u = 0.0f;
    if (!(v - v == 0.0f)) v = 0.0f;
    const float uw = u - orx_floorf(u), vw = v - orx_floorf(v);
    const float xb = uw * (float)w - 0.5f, yb = vw * (float)h - 0.5f;
    const float fx = orx_floorf(xb), fy = orx_floorf(yb);
    const float a = orx_floorf((xb - fx) * 256.0f + 0.5f) * (1.0f / 256.0f);
    const float b = orx_floorf((yb - fy) * 256.0f + 0.5f) * (1.0f / 256.0f);
    int32_t i0 = (int32_t)fx, j0 = (int32_t)fy;
    i0 = i0 < 0 ? i0 + (int32_t)w : (i0 >= (int32_t)w ? i0 - (int32_t)w : i0);
    j0 = j0 < 0 ? j0 + (int32_t)h : (j0 >= (int32_t)h ? j0 - (int32_t)h : j0);
    const uint32_t i1 = (uint32_t)i0 + 1u == w ? 0u : (uint32_t)i0 + 1u;
    const uint32_t j1 = (uint32_t)j0 + 1u == h ? 0u : (uint32_t)j0 + 1u;
    const uint32_t* tx = (const uint32_t*)(const void*)rgba; /* one RGBA8 texel per dword (little endian) */
    const uint32_t t00 = tx[(size_t)j0 * w + (uint32_t)i0], t10 = tx[(size_t)j0 * w + i1];
    const uint32_t t01 = tx[(size_t)j1 * w + (uint32_t)i0], t11 = tx[(size_t)j1 * w + i1];
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    for (int c = 0; c < 4; c++) {
        const uint32_t sh = 8u * (uint32_t)c;
        const float s = w00 * ((float)((t00 >> sh) & 255u) / 255.0f) + w10 * ((float)((t10 >> sh) & 255u) / 255.0f) +
                        w01 * ((float)((t01 >> sh) & 255u) / 255.0f) + w11 * ((float)((t11 >> sh) & 255u) / 255.0f);
        out[c] = s;
    }
}

#ifdef __cplusplus
}
#endif

#endif /* ORX_DETMATH_H */
