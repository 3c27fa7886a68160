/*
 * orx_kernels.hip — gfx950 kernels of the render core.
 *
 * One kernel per reference OptiX entry point / Thrust step:
 *   k_rng_init          initRandomStateBuffer  (OptixRenderer_SpatialHash.cu:310-334)
 *   k_ppm_eye           PPM_RAYTRACE_PASS      (ppm/RayGeneratorPPM.cu:31-66)
 *   k_ppm_photon        PPM_PHOTON_PASS        (ppm/PhotonGenerator.cu:81-128 + material
 *                       closest-hit photon programs) fused with the photon AABB
 *                       reduction of getPhotonsBoundingBox (SpatialHash.cu:123-128)
 *   k_grid_setup        cell size / grid dims  (SpatialHash.cu:229-249), on device
 *   k_bs_*              calculateHashCellsKernel + sort_by_key + exclusive_scan
 *                       (SpatialHash.cu:152-207) as an LDS bucket counting sort
 *   k_grid_permute      the sorted photon array, as SoA planes
 *   k_ppm_gather_union  PPM_INDIRECT_RADIANCE_ESTIMATION_PASS (ppm/IndirectRadianceEstimation.cu:69-227),
 *                       wave-union form; k_ppm_gather the per-lane form (sharded gathers at N >= 8)
 *   k_ppm_direct_output PPM_DIRECT + PPM_OUTPUT (ppm/DirectRadianceEstimation.cu:29-77, ppm/Output.cu:32-37)
 *   k_pt                PT_RAYTRACE_PASS       (pt/RayGeneratorPT.cu:46-131)
 * Wave size is 64 on CDNA4; block reductions below are written for it.
 */
#include <algorithm>
#include <cstdlib>

#include "orx_kernels.h"

namespace orx {

/* ------------------------------------------------------------------ */
/* helpers                                                             */
/* ------------------------------------------------------------------ */
__device__ __forceinline__ uint32_t f2ord(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ float wave_min(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ void store_hitpoint(const PixelBufs& px, size_t i, const RadiancePRD& prd) {
    /* Union: non-specular hits carry normal, others carry radiance (the
     * unused one is identically zero in RayGeneratorPPM's PRD). */
    bool ns = (prd.flags & PRD_HIT_NON_SPECULAR) != 0;
    f3 nr = ns ? prd.normal : prd.radiance;
    px.hpA[i] = make_float4(prd.position.x, prd.position.y, prd.position.z, __uint_as_float(prd.flags));
    px.hpB[i] = make_float4(nr.x, nr.y, nr.z, prd.attenuation.x);
    px.hpC[i] = make_float2(prd.attenuation.y, prd.attenuation.z);
}

/* ------------------------------------------------------------------ */
/* RNG init: curand_init(seed + slot, 0, 0)                            */
/* ------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_rng_init(RngPlanes rng, uint32_t RW, uint32_t rows, uint32_t rank,
                                                  uint32_t world, uint32_t seed) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t n = (size_t)rows * RW;
    if (i >= n) return;
    uint32_t j = (uint32_t)(i / RW), x = (uint32_t)(i % RW);
    uint32_t y = rank + world * j;
    uint32_t gslot = y * RW + x;
    rng_store(rng, i, rng_init((uint64_t)(uint32_t)(seed + gslot)));
}
void launch_rng_init(hipStream_t s, RngPlanes rng, uint32_t RW, uint32_t rows, uint32_t rank, uint32_t world,
                     uint32_t seed) {
    size_t n = (size_t)rows * RW;
    hipLaunchKernelGGL(k_rng_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rng, RW, rows, rank, world,
                       seed);
}

/* Pixel tile of a 64-lane wave for the per-pixel passes (eye, direct, PT): 8x8 local pixels
 * on one device; a shard owns image rows rank + world*j, so 8 local rows would span 8*world
 * image rows (incoherent primary and shadow rays): 16x4 local pixels for 2-4 ranks, 32x2 for 8+ */
__host__ __device__ __forceinline__ uint32_t pix_tile_shift(uint32_t world) { return world >= 8 ? 2u : world >= 2 ? 1u : 0u; }
__device__ __forceinline__ void pix_tile(const PixelBufs& px, uint32_t& x, uint32_t& j) {
    const uint32_t sh = pix_tile_shift(px.world), tw = 8u << sh;
    x = blockIdx.x * tw + (threadIdx.x & (tw - 1));
    j = blockIdx.y * (8u >> sh) + (threadIdx.x >> (3 + sh));
}
static dim3 pix_grid(const PixelBufs& px) {
    const uint32_t sh = pix_tile_shift(px.world), tw = 8u << sh, th = 8u >> sh;
    return dim3((px.W + tw - 1) / tw, (px.rows + th - 1) / th);
}

/* ------------------------------------------------------------------ */
/* PPM eye pass                                                        */
/* ------------------------------------------------------------------ */
template <bool MEDIA>
__global__ __launch_bounds__(64) void k_ppm_eye(DevScene S, DevCamera cam, PixelBufs px, Consts c, VolMap vm,
                                                float* volR) {
    ORX_STACK_DECL;
    uint32_t x, j;
    pix_tile(px, x, j);
    if (x >= px.W || j >= px.rows) return;
    uint32_t y = px.rank + px.world * j;
    size_t slot = (size_t)j * px.RW + x;
    Rng rs = rng_load(px.rng, slot);
    RadiancePRD prd;
    prd.attenuation = mk1(1.0f);
    prd.radiance = mk1(0.f);
    prd.depth = 0;
    prd.flags = 0;
    prd.position = mk1(0.f);
    prd.normal = mk1(0.f);
    prd.newdir = mk1(0.f);
    f3 o, d;
    primary_ray(cam, x, y, px.W, px.H, rs, o, d);
    if (MEDIA) {
        f3 vr;
        trace_radiance_vol(S, vm, c.max_radiance_depth, o, d, 0.001f, prd, rs, ORX_STACK_PTR, vr);
        const size_t i = (size_t)j * px.W + x;
        volR[3 * i + 0] = vr.x;
        volR[3 * i + 1] = vr.y;
        volR[3 * i + 2] = vr.z;
    } else {
        trace_radiance(S, c.max_radiance_depth, o, d, 0.001f, prd, rs, ORX_STACK_PTR);
    }
    store_hitpoint(px, (size_t)j * px.W + x, prd);
    rng_store(px.rng, slot, rs);
}
void launch_ppm_eye(hipStream_t s, const DevScene& S, const DevCamera& cam, const PixelBufs& px, const Consts& c,
                    const MediaBufs* mb) {
    const dim3 grid = pix_grid(px);
    if (mb) hipLaunchKernelGGL((k_ppm_eye<true>), grid, dim3(64), ORX_STACK_BYTES(S), s, S, cam, px, c, mb->vm, mb->volR);
    else hipLaunchKernelGGL((k_ppm_eye<false>), grid, dim3(64), ORX_STACK_BYTES(S), s, S, cam, px, c, VolMap{}, nullptr);
}

/* ------------------------------------------------------------------ */
/* PPM photon pass (+ AABB of the valid deposits)                      */
/* ------------------------------------------------------------------ */
/* Photon pass (PhotonGenerator.cu:83-128 + the photon closest-hit programs).  Each lane carries
 * one photon path.  Photon p = j*PW + x always uses RNG slot (j, x) and deposit slots
 * [p*D, p*D + D), so the result does not depend on which lane traced it. */
struct PhotonPath {
    f3 o, d, power;
    float weight, tmin;
    uint32_t p_local, depth, numStored, mask;
    size_t slot;
};
/* the medium's extra photon state (ParticipatingMedium.cu:110-201): ray type and tmax, the open
 * scatter probe (depth at its start, scatter position) and the volumetric events so far */
struct PhotonMedia {
    float tmax;
    bool inmed, probe;
    uint32_t pdepth, nev;
    f3 spos, ev_pos, ev_pow;
};
__device__ __forceinline__ void photon_emit(const DevScene& S, const PixelBufs& px, const PhotonBufs& pb, uint32_t p,
                                            PhotonPath& P, Rng& rs) {
    const uint32_t j = p / pb.PW, x = p - j * pb.PW;
    P.p_local = p;
    P.slot = (size_t)j * px.RW + x;
    rs = rng_load(px.rng, P.slot);
    /* PhotonGenerator.cu:91-107 */
    int lightIndex = 0;
    if (S.nl > 1) {
        float sample = rnd(rs);
        int li = (int)(sample * (float)S.nl);
        lightIndex = li < (int)(S.nl - 1) ? li : (int)(S.nl - 1);
    }
    const DevLight& L = S.lights[lightIndex];
    float powerScale = (float)S.nl;
    f3 power = L.power * powerScale;
    f3 origin = L.position, dir = mk1(0.f);
    float photonPowerFactor = 1.f;
    float s1x = rnd(rs), s1y = rnd(rs);
    /* generatePhotonOriginAndDirection (PhotonGenerator.cu:40-79) */
    if (L.type == LIGHT_AREA) {
        float s2x = rnd(rs), s2y = rnd(rs);
        origin = origin + (L.v1 * s1x + L.v2 * s1y);
        dir = sample_hemisphere(L.normal, s2x, s2y);
    } else if (L.type == LIGHT_POINT) {
        f3 bc = mk(S.bs_cx, S.bs_cy, S.bs_cz);
        f3 sceneCenterToLight = L.position - bc;
        float lightDistance = length(sceneCenterToLight);
        sceneCenterToLight = sceneCenterToLight / lightDistance;
        bool wellOutside = (double)lightDistance > 1.5 * (double)S.bs_r;
        if (wellOutside) {
            f3 pointOnDisc = sample_disc(s1x, s1y, bc, S.bs_r, sceneCenterToLight);
            dir = normalize(pointOnDisc - origin);
            float rr = S.bs_r * S.bs_r + lightDistance * lightDistance;
            photonPowerFactor = (1 - lightDistance * (1.0f / sqrtf(rr))) / 2.f;
        } else {
            dir = sample_unit_sphere(s1x, s1y);
        }
    } else {
        f3 pointOnDisc = sample_disc(s1x, s1y, origin + L.direction, orx_sinf(L.angle / 2), L.direction);
        dir = normalize(pointOnDisc - origin);
    }
    P.power = power * photonPowerFactor;
    P.o = origin;
    P.d = dir;
    P.weight = 1.0f;
    P.tmin = 0.0001f;
    P.depth = 0;
    P.numStored = 0;
    P.mask = 0;
}

/* What a photon does at the end of its ray (Diffuse.cu:92-135, Glossy.cu:94-137, Mirror.cu:65-77,
 * Glass.cu:164-205, DiffuseEmitter.cu:56-59, ParticipatingMedium.cu:110-201): deposit,
 * Russian roulette and the next ray in P; false once the path has ended (its deposit mask and
 * RNG state are then stored). */
template <bool MEDIA>
__device__ __forceinline__ bool photon_after_hit(const DevScene& S, const PixelBufs& px, const PhotonBufs& pb,
                                                 const Consts& c, PhotonPath& P, Rng& rs, bool hit, const Hit& h,
                                                 bool had_probe, float& lo_x, float& lo_y, float& lo_z, float& hi_x,
                                                 float& hi_y, float& hi_z, const VolMap& vm, PhotonMedia& M,
                                                 const MediaBufs& mb) {
    bool done = false;
    if (!hit) {
        done = true;
    } else if (MEDIA && h.prim == MED_PRIM) {
        P.depth++;
        const f3 N = normalize(h.sn);
        const f3 hitPoint = P.o + P.d * h.t;
        if (dot(N, P.d) > 0 && M.inmed) { /* leaving the box */
            P.o = hitPoint + P.d * 0.0001f;
            P.tmin = 0.001f;
            M.tmax = RT_DEFAULT_MAX;
            M.inmed = false;
        } else { /* sample the scatter distance, probe [0.001, scatterT] */
            const float sig_t = vm.sig_a + vm.sig_s;
            const float sample = rnd(rs);
            const float st = -orx_logf(1 - sample) / sig_t;
            M.spos = hitPoint + P.d * st;
            M.probe = true;
            M.pdepth = P.depth;
            P.o = hitPoint;
            P.tmin = 0.001f;
            M.tmax = st;
            M.inmed = true;
        }
    } else {
        if (MEDIA) M.tmax = RT_DEFAULT_MAX;
        const DevMaterial& m = S.mats[prim_material(S, h)];
        const f3 hitPoint = P.o + P.d * h.t;
        if (m.type == MAT_DIFFUSE || m.type == MAT_GLOSSY || m.type == MAT_TEXTURE) {
            /* Texture.cu:116-175 differs only in Kd = texel colour,
             * the weight cutoff (0.01) and the new ray's tmin (0.01) */
            const bool tex = m.type == MAT_TEXTURE;
            const f3 N = shading_normal(S, h);
            if (P.depth >= 1 && P.numStored < pb.D) {
                const uint32_t si = P.p_local * pb.D + P.numStored;
                float4* rec = pb.slots + 4 * (size_t)si;
                rec[0] = make_float4(hitPoint.x, hitPoint.y, hitPoint.z, P.power.x);
                pb.pos4[si] = make_float4(hitPoint.x, hitPoint.y, hitPoint.z, 0.f);
                rec[1] = make_float4(P.d.x, P.d.y, P.d.z, P.power.y);
                rec[2].x = P.power.z;
                /* the hash's STORE_PHOTON (store_photon.h:19-25) counts every deposit */
                if (fmax3(P.power) > 0 || pb.hash) {
                    P.mask |= 1u << P.numStored;
                    lo_x = fminf(lo_x, hitPoint.x); lo_y = fminf(lo_y, hitPoint.y); lo_z = fminf(lo_z, hitPoint.z);
                    hi_x = fmaxf(hi_x, hitPoint.x); hi_y = fmaxf(hi_y, hitPoint.y); hi_z = fmaxf(hi_z, hitPoint.z);
                }
                P.numStored++;
            }
            const f3 Kd = tex ? tex_color(S, m, h) : m.Kd;
            P.power = P.power * Kd;
            P.weight *= fmax3(Kd);
            if (P.depth >= 3) {
                float probContinue = favgf(Kd);
                float probSample = rnd(rs);
                if (probSample >= probContinue) done = true;
                else P.power = P.power / probContinue;
            }
            if (!done) {
                P.depth++;
                if (P.depth >= c.max_photon_depth || (double)P.weight < (tex ? 0.01 : 0.001) ||
                    P.numStored >= pb.Dlim) {
                    done = true;
                } else {
                    float s0 = rnd(rs);
                    float s1 = rnd(rs);
                    P.d = sample_hemisphere_cos(N, s0, s1);
                    P.o = hitPoint;
                    P.tmin = tex ? 0.01f : 0.0001f;
                    if (MEDIA) M.inmed = false;
                }
            }
        } else if (m.type == MAT_EMITTER) {
            if (MEDIA && !M.inmed) P.depth++; /* closestHitPhoton is the PHOTON program only */
            done = true;
        } else if (m.type == MAT_MIRROR) {
            const f3 N = shading_normal(S, h);
            P.depth++;
            if (P.depth <= c.max_photon_depth) {
                P.power = P.power * m.Kr;
                P.d = reflect(P.d, N);
                P.o = hitPoint;
                P.tmin = 0.0001f;
                if (MEDIA) M.inmed = false;
            } else {
                done = true;
            }
        } else {
            const f3 wsn = shading_normal(S, h);
            const bool outside = dot(wsn, P.d) < 0;
            const f3 N = outside ? wsn : -wsn;
            const float n1 = outside ? 1.0f : m.ior, n2 = outside ? m.ior : 1.0f;
            f3 refr;
            bool valid;
            const float refl = glass_reflect_factor(P.d, N, n1, n2, refr, valid);
            const float sample = rnd(rs);
            const bool reflected = sample <= refl;
            const f3 nd = reflected ? reflect(P.d, N) : refr;
            P.depth++;
            if (P.depth <= c.max_photon_depth) {
                P.o = hitPoint;
                P.d = nd;
                P.tmin = 0.0001f;
                if (MEDIA) M.inmed = (outside && !reflected) || (!outside && reflected);
            } else {
                done = true;
            }
        }
    }
    if (MEDIA && had_probe && P.depth == M.pdepth) { /* the probe met nothing that took the path over */
        done = true;
        if (rnd(rs) < vm.sig_s / (vm.sig_a + vm.sig_s)) {
            M.nev++;
            M.ev_pos = M.spos;
            M.ev_pow = P.power;
            if (P.depth < c.max_photon_depth) {
                const float s0 = rnd(rs), s1 = rnd(rs);
                P.d = sample_unit_sphere(s0, s1);
                P.o = M.spos;
                P.tmin = 0.001f;
                M.tmax = RT_DEFAULT_MAX;
                M.inmed = false;
                done = false;
            }
        }
    }
    if (done) {
        pb.vmask[P.p_local] = (uint8_t)P.mask;
        rng_store(px.rng, P.slot, rs);
        if (MEDIA) {
            mb.ev_a[P.p_local] = make_float4(M.ev_pos.x, M.ev_pos.y, M.ev_pos.z, __uint_as_float(M.nev));
            mb.ev_b[P.p_local] = make_float4(M.ev_pow.x, M.ev_pow.y, M.ev_pow.z, 0.f);
        }
        return false;
    }
    return true;
}

/* One bounce of a photon path: its ray, then photon_after_hit. */
template <bool MEDIA, class STK, class NODES>
__device__ __forceinline__ bool photon_bounce(const DevScene& S, const PixelBufs& px, const PhotonBufs& pb,
                                              const Consts& c, PhotonPath& P, Rng& rs, const STK& stk,
                                              const NODES& nodes, float& lo_x, float& lo_y, float& lo_z,
                                              float& hi_x, float& hi_y, float& hi_z, const VolMap& vm,
                                              PhotonMedia& M, const MediaBufs& mb) {
    Hit h;
    bool had_probe = false;
    bool hit;
    if (MEDIA) {
        had_probe = M.probe;
        M.probe = false;
        hit = trace_closest_m(S, vm, P.o, P.d, P.tmin, M.tmax, M.inmed, h, stk, nodes);
    } else {
        hit = trace_closest_t(S, P.o, P.d, P.tmin, RT_DEFAULT_MAX, h, stk, nodes);
    }
    return photon_after_hit<MEDIA>(S, px, pb, c, P, rs, hit, h, had_probe, lo_x, lo_y, lo_z, hi_x, hi_y, hi_z, vm, M, mb);
}

__device__ __forceinline__ void photon_bbox_flush(const PhotonBufs& pb, float lo_x, float lo_y, float lo_z, float hi_x,
                                                  float hi_y, float hi_z, uint32_t rep, uint32_t lane) {
    /* wave AABB -> device-wide ordered-int atomics (one lane per component) */
    lo_x = wave_min(lo_x); lo_y = wave_min(lo_y); lo_z = wave_min(lo_z);
    hi_x = wave_max(hi_x); hi_y = wave_max(hi_y); hi_z = wave_max(hi_z);
    /* 64 replicas per component keep same-address atomic contention low */
    if (lane < 6) {
        float v = lane == 0 ? lo_x : lane == 1 ? lo_y : lane == 2 ? lo_z : lane == 3 ? hi_x : lane == 4 ? hi_y : hi_z;
        if (lane < 3) {
            if (v != INFINITY) atomicMin(&pb.bbox[lane * BBOX_REPLICAS + rep], f2ord(v));
        } else {
            if (v != -INFINITY) atomicMax(&pb.bbox[lane * BBOX_REPLICAS + rep], f2ord(v));
        }
    }
}

/* One photon per lane: block b traces photons [64b, 64b + 64).  The kernel is register-capped at
 * ORX_PHOTON_WAVES waves per SIMD (6: 80 VGPRs and 13 spilled; uncapped it took 121 and ran at 4;
 * hall frame 6.43 ms at 4 waves, 6.33 at 5, 6.19 at 6, 7 no better) and its traversal stack is PHOTON_LDS_STACK entries per lane in LDS continued in global memory
 * (StackH, one column per photon): the whole stack in LDS (35 entries on the hall, 9.5 KB per wave)
 * would hold a CU to 16 waves.  (Persistent waves on a work counter spilled at 5 waves and ran
 * slower; per-lane refill from a device counter, a wavefront pass with
 * per-bounce queues and a direction-binned photon order were measured slower on the hall: DESIGN.md
 * section 4.) */
#ifndef ORX_PHOTON_WAVES
#define ORX_PHOTON_WAVES 6
#endif
constexpr int PHOTON_LDS_STACK = 16;
template <bool MEDIA>
__global__ __launch_bounds__(64, ORX_PHOTON_WAVES) void k_ppm_photon(DevScene S, PixelBufs px, PhotonBufs pb, Consts c,
                                                                     MediaBufs mb) {
    ORX_STACK_DECL;
    const uint32_t lane = threadIdx.x;
    const uint32_t total = pb.prows * pb.PW;
    const uint32_t p = blockIdx.x * 64u + lane;
    const StackH<PHOTON_LDS_STACK> stk{ORX_STACK_PTR, pb.tstk, blockIdx.x, pb.tdeep, lane};
    float lo_x = INFINITY, lo_y = INFINITY, lo_z = INFINITY;
    float hi_x = -INFINITY, hi_y = -INFINITY, hi_z = -INFINITY;
    PhotonPath P;
    PhotonMedia M;
    M.tmax = RT_DEFAULT_MAX;
    M.inmed = M.probe = false;
    M.pdepth = M.nev = 0;
    M.spos = M.ev_pos = M.ev_pow = mk1(0.f);
    Rng rs;
    bool alive = p < total;
    if (alive) photon_emit(S, px, pb, p, P, rs);
    while (__ballot(alive)) {
        if (alive)
            alive = photon_bounce<MEDIA>(S, px, pb, c, P, rs, stk, NodesG{}, lo_x, lo_y, lo_z, hi_x, hi_y, hi_z, mb.vm,
                                         M, mb);
    }
    photon_bbox_flush(pb, lo_x, lo_y, lo_z, hi_x, hi_y, hi_z, blockIdx.x & (BBOX_REPLICAS - 1), lane);
}

uint32_t photon_stack_deep(uint32_t entries) { return StackH<PHOTON_LDS_STACK>::deep(entries); }
/* false (nothing launched): the deep-stack buffer does not cover the launch (the caller reports
 * ORX_ERR_STATE; photon_stack_ensure sizes it at every scene and resize) */
bool launch_ppm_photon(hipStream_t s, const DevScene& S, const PixelBufs& px, const PhotonBufs& pb, const Consts& c,
                       const MediaBufs* mb) {
    const uint32_t total = pb.prows * pb.PW;
    if (total == 0) return true;
    const uint32_t blocks = (total + 63) / 64;
    if ((size_t)blocks * 64 > pb.tlanes || pb.tdeep < StackH<PHOTON_LDS_STACK>::deep(S.stack_entries)) return false;
    const size_t lds = StackH<PHOTON_LDS_STACK>::lds_bytes();
    if (mb)
        hipLaunchKernelGGL((k_ppm_photon<true>), dim3(blocks), dim3(64), lds, s, S, px, pb, c, *mb);
    else
        hipLaunchKernelGGL((k_ppm_photon<false>), dim3(blocks), dim3(64), lds, s, S, px, pb, c, MediaBufs{});
    return true;
}

/* ------------------------------------------------------------------ */
/* grid setup: createUniformGridPhotonMap host math, on one thread     */
/* ------------------------------------------------------------------ */
__global__ void k_grid_setup(PhotonBufs pb, GridBox gb) {
    /* lanes k*64..: fold the replicas, then reset them for the next photon pass */
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
    uint32_t b[6];
    GridParams* g = pb.grid;
    /* the photons' own AABB: the slab gather's cull box */
    const bool own = red[0] != 0xffffffffu;
    for (int k = 0; k < 3; k++) {
        g->clo[k] = own ? ord2f(red[k]) : INFINITY;
        g->chi[k] = own ? ord2f(red[k + 3]) : -INFINITY;
    }
    for (int k = 0; k < 6; k++) b[k] = gb.on ? gb.b[k] : red[k];
    bool any = b[0] != 0xffffffffu; /* min initialised to ord(+max) */
    f3 lo, hi;
    if (any) {
        lo = mk(ord2f(b[0]), ord2f(b[1]), ord2f(b[2]));
        hi = mk(ord2f(b[3]), ord2f(b[4]), ord2f(b[5]));
    } else {
        lo = mk1(0.f);
        hi = mk1(0.f);
    }
    /* padAABB (SpatialHash.cu:135-141) */
    lo = mk(lo.x - 0.0000001f, lo.y - 0.0000001f, lo.z - 0.0000001f);
    hi = mk(hi.x + 0.0000001f, hi.y + 0.0000001f, hi.z + 0.0000001f);
    f3 ext = hi - lo;
    /* getSmallestPossibleCellSize (SpatialHash.cu:62-71) */
    float sceneVolume = ext.x * ext.y * ext.z;
    float minVolumePerCell = sceneVolume / (float)pb.gcells;
    float radiusC = orx_powf(minVolumePerCell, 1.0f / 3.0f);
    f3 ncf = ext / radiusC;
    uint32_t nx = orx_f2u_sat(orx_floorf(ncf.x)), ny = orx_f2u_sat(orx_floorf(ncf.y)),
             nz = orx_f2u_sat(orx_floorf(ncf.z));
    f3 each = mk(ext.x / (float)nx, ext.y / (float)ny, ext.z / (float)nz);
    float smallest = fmax3(each);
    float cellSize = (float)((double)smallest + 0.001);
    /* calculateGridSize (SpatialHash.cu:42-50) */
    f3 f = ext / cellSize;
    uint32_t gx = orx_f2u_sat(orx_ceilf(f.x)), gy = orx_f2u_sat(orx_ceilf(f.y)), gz = orx_f2u_sat(orx_ceilf(f.z));
    gx = gx < 1 ? 1 : gx;
    gy = gy < 1 ? 1 : gy;
    gz = gz < 1 ? 1 : gz;
    uint64_t G = (uint64_t)gx * gy * gz;
    g->ox = lo.x; g->oy = lo.y; g->oz = lo.z;
    g->cell = cellSize;
    g->gx = gx; g->gy = gy; g->gz = gz;
    g->any_valid = any;
    g->photons_visited = 0;
    g->cells_visited = 0;
    if (G > pb.gmax) {
        g->error = 1;
        g->G = 0;
    } else {
        g->error = 0;
        g->G = (uint32_t)G;
    }
}
void launch_grid_setup(hipStream_t s, const PhotonBufs& pb, const GridBox& gb) {
    hipLaunchKernelGGL(k_grid_setup, dim3(1), dim3(64), 0, s, pb, gb);
}

/* ------------------------------------------------------------------ */
/* block-wide exclusive scan (the bucket sort's table scan)             */
/* ------------------------------------------------------------------ */
constexpr int SCAN_BLOCK = 1024; /* elements per block: 256 threads x 4 */

__device__ __forceinline__ uint32_t block_exclusive_scan_256(uint32_t v, uint32_t* total) {
    __shared__ uint32_t ws[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int q = 0; q < w; q++) pre += ws[q];
    *total = ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
    return pre + x - v;
}

/* Direction prefilter word of a grid photon (sorted plane SP_DIRQ): the
 * direction as three int8 snorm bytes q = rint(127 d).  The gather's facing
 * test dot(d, n) <= 0 is decided from v_dot4_i32_i8(q, qn) (qn the same
 * quantisation of the hit point's normal) whenever that integer dot lies
 * outside +-DIRQ_BAND; inside the band the exact fp32 direction planes decide.
 * Bound: |q/127 - d|_inf <= 0.5/127 + eps, so for |d|_1, |n|_1 <= 1.7325
 *   |qd.qn - 127^2 d.n| <= 127^2 (0.5/127 (|d|_1 + |n|_1) + 3 (0.5/127)^2) <= 221
 * and every decision taken from the integer dot equals the exact one.  A
 * direction (or normal) outside that 1-norm bound, with a component above 1 in
 * magnitude (which would wrap in the byte) or NaN quantises to 0, which always
 * lands in the band. */
constexpr int32_t DIRQ_BAND = 232;
__device__ __forceinline__ uint32_t dir_q8(float x, float y, float z) {
    /* the 1-norm bound of the error estimate, and |c| <= 1 so rint(127 c) fits an int8 */
    if (!(fabsf(x) + fabsf(y) + fabsf(z) <= 1.7325f) || !(fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z))) <= 1.0f))
        return 0u;
    const int32_t qx = (int32_t)rintf(x * 127.f), qy = (int32_t)rintf(y * 127.f), qz = (int32_t)rintf(z * 127.f);
    return ((uint32_t)qx & 0xffu) | (((uint32_t)qy & 0xffu) << 8) | (((uint32_t)qz & 0xffu) << 16);
}

/* one grid photon: a deposit record -> the SoA planes at grid
 * position dst (the reference's sorted photon array, SpatialHash.cu:193-196) */
__device__ __forceinline__ void grid_put(const PhotonBufs& pb, uint32_t dst, const float4 a, const float4 b, float cz) {
    const size_t P = pb.splane;
    float* o = pb.sorted + dst;
    o[SP_X * P] = a.x;
    o[SP_Y * P] = a.y;
    o[SP_Z * P] = a.z;
    o[SP_DIRQ * P] = __uint_as_float(dir_q8(b.x, b.y, b.z));
    o[SP_DX * P] = b.x;
    o[SP_DY * P] = b.y;
    o[SP_DZ * P] = b.z;
    o[SP_PX * P] = a.w;
    o[SP_PY * P] = b.w;
    o[SP_PZ * P] = cz;
}
/* grid order -> SoA planes: destination-major, so the ten plane writes are
 * coalesced and the source reads are whole float4s */
__global__ __launch_bounds__(256) void k_grid_permute(PhotonBufs pb) {
    const uint32_t valid = pb.grid->valid;
    const uint32_t T = gridDim.x * blockDim.x;
    for (uint32_t d0 = blockIdx.x * blockDim.x + threadIdx.x; d0 < valid; d0 += 4 * T) {
        uint32_t src[4];
        float4 a[4], b[4];
        float cz[4];
#pragma unroll
        for (int q = 0; q < 4; q++) src[q] = d0 + q * T < valid ? pb.perm[d0 + q * T] : 0xffffffffu;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (src[q] != 0xffffffffu) {
                const float4* rec = pb.slots + 4 * (size_t)src[q];
                a[q] = rec[0];
                b[q] = rec[1];
                cz[q] = rec[2].x;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (src[q] != 0xffffffffu) grid_put(pb, d0 + q * T, a[q], b[q], cz[q]);
    }
}
/* ------------------------------------------------------------------ */
/* photon grid without global atomics: two-level bucket counting sort  */
/* ------------------------------------------------------------------ */
/* The atomic-rank counting sort above issues one device-scope atomic per
 * photon into a 4 MB histogram; across 8 XCDs those resolve at the memory
 * side (~25 G/s measured), which makes the hash pass the slowest of the grid
 * build.  Here:
 *   A  k_bs_count    per chunk of BS_CHUNK slots: keys, LDS histogram of the
 *                    coarse bucket key >> bshift -> table[bucket][chunk]
 *   S  scan of the table (bucket-major) -> where each chunk's bucket run starts
 *   B  k_bs_place    per chunk: LDS cursors from the table, (key, slot) pairs
 *                    appended to their bucket run
 *   C  k_bs_cells    one block per bucket: LDS histogram of its cells, LDS
 *                    scan -> offsets of those cells, permutation by LDS cursors
 *   D  k_grid_coarse_offsets (nsub > 1) the reference's cell offsets
 * All counting is in LDS.  Offsets equal the reference's exclusive scan over
 * the cell histogram (keys >= G are the reference's overflow cell G and, as
 * there, fall beyond offsets[G] = valid: they are dropped).
 *
 * Sub-row layout (nsub = SUBR^2 = 4).  Photons are ordered by a virtual cell
 *   vc = ((y + z gy) nsub + s) gx + x,   s = 2 (z half) + (y half),
 * then by the x quarter: every cell row (y,z) is stored as four sub-rows, each
 * holding the photons of one (y,z) quarter of the row's cells in x order.  A
 * gather chord on a sub-row is one contiguous range of subofs, and the
 * quarter-height sub-rows hug the sphere (fewer photons tested per pixel);
 * the photons of a reference cell are the union of its four sub-row pieces,
 * so the reference offsets (the visit counters, the exported grid) come from
 * the sub-row offsets by k_grid_coarse_offsets. */
constexpr uint32_t BS_CHUNK = 16384;
constexpr uint32_t BS_THREADS = 512;
constexpr uint32_t BS_MAXB = 2048; /* buckets */

__global__ __launch_bounds__(BS_THREADS) void k_bs_count(PhotonBufs pb) {
    __shared__ uint32_t hist[BS_MAXB];
    const GridParams g = *pb.grid;
    const uint32_t nb = (g.G * pb.nsub + (1u << pb.bshift) - 1) >> pb.bshift;
    for (uint32_t i = threadIdx.x; i < BS_MAXB; i += BS_THREADS) hist[i] = 0;
    __syncthreads();
    const float inv = 1.f / g.cell;
    const uint32_t c0 = blockIdx.x * BS_CHUNK;
    for (uint32_t k = threadIdx.x; k < BS_CHUNK; k += BS_THREADS) {
        const uint32_t s = c0 + k;
        if (s >= pb.S) break;
        uint32_t key = 0xffffffffu;
        const uint32_t p = s / pb.D, d = s - p * pb.D;
        if (g.G && ((pb.vmask[p] >> d) & 1u)) {
            const float4 a = pb.pos4[s];
            const f3 pp = (mk(a.x, a.y, a.z) - mk(g.ox, g.oy, g.oz)) * inv;
            const uint32_t cx = orx_f2u_sat(orx_floorf(pp.x));
            const uint32_t cy = orx_f2u_sat(orx_floorf(pp.y));
            const uint32_t cz = orx_f2u_sat(orx_floorf(pp.z));
            const uint32_t kk = cx + cy * g.gx + cz * g.gx * g.gy;
            if (kk < g.G) { /* calculateHashCellsKernel clamps to G: the overflow cell, beyond valid */
                /* sub-cell key: the x quarter of the cell, so that the gather can
                 * trim a row to the chord at quarter-cell granularity */
                int32_t q = (int32_t)orx_floorf(pp.x * (float)SUBX) - (int32_t)SUBX * (int32_t)cx;
                q = q < 0 ? 0 : (q > (int32_t)SUBX - 1 ? (int32_t)SUBX - 1 : q);
                uint32_t vc = kk;
                if (pb.nsub > 1) { /* sub-row: y and z halves (x2 is exact, so the halves nest in the cells) */
                    int32_t hy = (int32_t)orx_floorf(pp.y * (float)SUBR) - (int32_t)SUBR * (int32_t)cy;
                    int32_t hz = (int32_t)orx_floorf(pp.z * (float)SUBR) - (int32_t)SUBR * (int32_t)cz;
                    hy = hy < 0 ? 0 : (hy > (int32_t)SUBR - 1 ? (int32_t)SUBR - 1 : hy);
                    hz = hz < 0 ? 0 : (hz > (int32_t)SUBR - 1 ? (int32_t)SUBR - 1 : hz);
                    const uint32_t row = cy + cz * g.gy;
                    vc = (row * pb.nsub + (uint32_t)hz * SUBR + (uint32_t)hy) * g.gx + cx;
                }
                key = vc * SUBX + (uint32_t)q;
                atomicAdd(&hist[vc >> pb.bshift], 1u);
            }
        }
        pb.keys[s] = key;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += BS_THREADS) pb.bs_table[(size_t)b * pb.bs_nchunk + blockIdx.x] = hist[b];
}

/* exclusive scan of n = nb * nchunk table entries in place (three kernels) */
__global__ __launch_bounds__(256) void k_bs_scan_reduce(PhotonBufs pb) {
    const uint32_t nb = (pb.grid->G * pb.nsub + (1u << pb.bshift) - 1) >> pb.bshift;
    const uint32_t n = nb * pb.bs_nchunk;
    const uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * 4;
    uint32_t sum = 0;
    for (int k = 0; k < 4; k++)
        if (base + k < n) sum += pb.bs_table[base + k];
    uint32_t total;
    (void)block_exclusive_scan_256(sum, &total);
    if (threadIdx.x == 0) pb.bs_partials[blockIdx.x] = total;
}
__global__ __launch_bounds__(256) void k_bs_scan_partials(PhotonBufs pb, uint32_t nblocks) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nblocks; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nblocks ? pb.bs_partials[i] : 0;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan_256(v, &total);
        if (i < nblocks) pb.bs_partials[i] = carry + ex;
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) pb.bs_partials[nblocks] = carry; /* grand total = valid photons */
}
__global__ __launch_bounds__(256) void k_bs_scan_apply(PhotonBufs pb) {
    const uint32_t nb = (pb.grid->G * pb.nsub + (1u << pb.bshift) - 1) >> pb.bshift;
    const uint32_t n = nb * pb.bs_nchunk;
    if (blockIdx.x * SCAN_BLOCK >= n) return;
    const uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * 4;
    uint32_t v[4], sum = 0;
    for (int k = 0; k < 4; k++) {
        v[k] = base + k < n ? pb.bs_table[base + k] : 0;
        sum += v[k];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan_256(sum, &total) + pb.bs_partials[blockIdx.x];
    for (int k = 0; k < 4; k++) {
        if (base + k < n) pb.bs_table[base + k] = ex;
        ex += v[k];
    }
}

__global__ __launch_bounds__(BS_THREADS) void k_bs_place(PhotonBufs pb) {
    __shared__ uint32_t cur[BS_MAXB];
    const uint32_t G = pb.grid->G * pb.nsub;
    const uint32_t nb = (G + (1u << pb.bshift) - 1) >> pb.bshift;
    for (uint32_t b = threadIdx.x; b < nb; b += BS_THREADS) cur[b] = pb.bs_table[(size_t)b * pb.bs_nchunk + blockIdx.x];
    __syncthreads();
    const uint32_t c0 = blockIdx.x * BS_CHUNK;
    constexpr uint32_t U = 4;
    for (uint32_t k0 = threadIdx.x; k0 < BS_CHUNK; k0 += U * BS_THREADS) {
        uint32_t kv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t s = c0 + k0 + u * BS_THREADS;
            kv[u] = s < pb.S ? pb.keys[s] : 0xffffffffu;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            if (kv[u] != 0xffffffffu) {
                const uint32_t pos = atomicAdd(&cur[(kv[u] / SUBX) >> pb.bshift], 1u);
                pb.bs_pairs[pos] = make_uint2(kv[u], c0 + k0 + u * BS_THREADS);
            }
        }
    }
}

/* one block per bucket: histogram of its sub-cells (virtual cell x quarter),
 * LDS scan -> sub-cell offsets (the gather's chord trimming) and, for nsub = 1,
 * the cell offsets (the reference's), permutation by LDS cursors */
__global__ __launch_bounds__(1024) void k_bs_cells(PhotonBufs pb, uint32_t cb, uint32_t nscan) {
    extern __shared__ uint32_t lds[]; /* [SUBX * cb] histogram / cursors */
    const uint32_t G = pb.grid->G * pb.nsub; /* virtual cells */
    const uint32_t nb = (G + cb - 1) / cb;
    const uint32_t b = blockIdx.x;
    const uint32_t total = pb.bs_partials[nscan]; /* grand total written by k_bs_scan_partials */
    if (b > nb) return;
    /* bucket nb (one past the last) only writes offsets[G] = valid when G is a multiple of cb */
    const uint32_t start = b < nb ? pb.bs_table[(size_t)b * pb.bs_nchunk] : total;
    const uint32_t end = b + 1 < nb ? pb.bs_table[(size_t)(b + 1) * pb.bs_nchunk] : total;
    const uint32_t nf = SUBX * cb, f0 = b * nf;
    for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) lds[i] = 0;
    __syncthreads();
    for (uint32_t i0 = start + threadIdx.x; i0 < end; i0 += 4 * blockDim.x) {
        uint32_t kv[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t i = i0 + u * blockDim.x;
            kv[u] = i < end ? pb.bs_pairs[i].x : 0xffffffffu;
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; u++)
            if (kv[u] != 0xffffffffu) atomicAdd(&lds[kv[u] - f0], 1u);
    }
    __syncthreads();
    /* exclusive scan of lds[0..nf) by 1024 threads, nf/1024 entries each */
    __shared__ uint32_t wsum[16];
    const uint32_t per = nf / blockDim.x;
    const uint32_t t0 = threadIdx.x * per;
    uint32_t run = 0;
    for (uint32_t k = 0; k < per; k++) run += lds[t0 + k];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = run;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t q = 0; q < w; q++) pre += wsum[q];
    uint32_t ex = start + pre + x - run;
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t f = f0 + t0 + k, c = f / SUBX;
        const uint32_t v = lds[t0 + k];
        if (c <= G) {
            if (f % SUBX == 0 && pb.nsub == 1) pb.offsets[c] = ex;
            if (c < G || f % SUBX == 0) pb.subofs[f] = ex;
        }
        lds[t0 + k] = ex; /* becomes the sub-cell's cursor */
        ex += v;
    }
    if (threadIdx.x == 0 && b == 0) {
        pb.grid->valid = total;
        pb.grid->valid_total += total;
    }
    __syncthreads();
    for (uint32_t i0 = start + threadIdx.x; i0 < end; i0 += 4 * blockDim.x) {
        uint2 kv[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t i = i0 + u * blockDim.x;
            kv[u] = i < end ? pb.bs_pairs[i] : make_uint2(0xffffffffu, 0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; u++)
            if (kv[u].x != 0xffffffffu) {
                const uint32_t pos = atomicAdd(&lds[kv[u].x - f0], 1u);
                pb.perm[pos] = kv[u].y;
            }
    }
}

/* the reference's cell offsets from the sub-row offsets: cell (x, row) starts
 * after all photons of the earlier rows and, in each of the row's nsub
 * sub-rows, after the photons of cells x' < x */
__global__ __launch_bounds__(256) void k_grid_coarse_offsets(PhotonBufs pb) {
    const GridParams g = *pb.grid;
    const uint32_t rowlen = g.gx * SUBX;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c <= g.G; c += gridDim.x * blockDim.x) {
        const uint32_t row = c / g.gx, x = c - row * g.gx;
        const size_t r0 = (size_t)row * pb.nsub * rowlen;
        uint32_t o = pb.subofs[r0];
        if (c < g.G)
            for (uint32_t s = 0; s < pb.nsub; s++) {
                const size_t b = r0 + (size_t)s * rowlen;
                o += pb.subofs[b + x * SUBX] - pb.subofs[b];
            }
        pb.offsets[c] = o;
    }
}

static uint32_t bs_nscan(const PhotonBufs& pb) {
    const uint32_t nbmax = (pb.gmax * pb.nsub + (1u << pb.bshift) - 1) >> pb.bshift;
    return (nbmax * pb.bs_nchunk + SCAN_BLOCK - 1) / SCAN_BLOCK;
}
void launch_grid_bucket_count(hipStream_t s, const PhotonBufs& pb) {
    hipLaunchKernelGGL(k_bs_count, dim3(pb.bs_nchunk), dim3(BS_THREADS), 0, s, pb);
}
void launch_grid_bucket_scan(hipStream_t s, const PhotonBufs& pb) {
    const uint32_t nscan = bs_nscan(pb);
    hipLaunchKernelGGL(k_bs_scan_reduce, dim3(nscan), dim3(256), 0, s, pb);
    hipLaunchKernelGGL(k_bs_scan_partials, dim3(1), dim3(256), 0, s, pb, nscan);
    hipLaunchKernelGGL(k_bs_scan_apply, dim3(nscan), dim3(256), 0, s, pb);
}
void launch_grid_bucket_place(hipStream_t s, const PhotonBufs& pb) {
    /* (staging a half chunk's pairs in LDS bucket by bucket, so that the writes of a wave go out in
     * runs, measured slower on the pipelined hall frame: 1034-1035 -> 1026-1028 Mpaths/s) */
    hipLaunchKernelGGL(k_bs_place, dim3(pb.bs_nchunk), dim3(BS_THREADS), 0, s, pb);
    const uint32_t cb = 1u << pb.bshift;
    const uint32_t nbmax = (pb.gmax * pb.nsub + cb - 1) / cb;
    static const uint32_t cells_threads = [] {
        const char* e = getenv("ORX_BS_CELLS_THREADS");
        const int v = e ? atoi(e) : 512; /* 512: co-schedules better beside the pipelined gather */
        return (uint32_t)(v == 256 || v == 1024 ? v : 512);
    }();
    hipLaunchKernelGGL(k_bs_cells, dim3(nbmax + 1), dim3(cells_threads), SUBX * cb * 4, s, pb, cb, bs_nscan(pb));
    if (pb.nsub > 1) {
        unsigned cblocks = (pb.gmax + 1 + 255) / 256;
        if (cblocks > 4096) cblocks = 4096;
        hipLaunchKernelGGL(k_grid_coarse_offsets, dim3(cblocks), dim3(256), 0, s, pb);
    }
    /* applying the permutation inside k_bs_cells (one block per bucket, scattered
     * record reads at its occupancy) measured 3.5 ms against 0.5 ms for this pass */
    /* (the record reads shared by a quad of lanes through LDS, 16 record lines per load instead
     * of 64, measured slower: hall grid build 1.20 -> 1.41 ms) */
    unsigned blocks = (pb.S + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_grid_permute, dim3(blocks), dim3(256), 0, s, pb);
}

/* ------------------------------------------------------------------ */
/* indirect radiance estimate: uniform-grid gather                     */
/* ------------------------------------------------------------------ */
/* XCD-aware tile order: block b runs on XCD b % 8; XCD k takes tiles [k per, (k+1) per) of the
 * image's tiles, or of the slab mode's list of tiles that gather here (a band of the image
 * would otherwise leave most XCDs idle when the rank's hit points cluster in the image).
 * gi.order = S > 0: the image's tiles taken in super-tiles of S x S tiles (super-tiles row-major,
 * tiles row-major inside), XCD k a contiguous run of that order, so the blocks an XCD runs at
 * once cover a patch S tiles tall instead of a strip one tile tall (fewer photon-plane lines
 * fetched into its L2 per tile).  false: no tile for this block. */
__host__ __device__ __forceinline__ uint32_t gather_order_count(uint32_t order, uint32_t ntx, uint32_t nty) {
    if (!order) return ntx * nty;
    return ((ntx + order - 1) / order) * ((nty + order - 1) / order) * order * order;
}
__device__ __forceinline__ bool gather_tile(const GatherIn& gi, uint32_t ntx, uint32_t ntiles, uint32_t& tile) {
    if (!gi.tile_list) {
        if (!gi.order) {
            const uint32_t per = (ntiles + 7) / 8;
            tile = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
            return true;
        }
        const uint32_t S = gi.order, nty = ntiles / ntx, nsx = (ntx + S - 1) / S;
        const uint32_t total = gather_order_count(S, ntx, nty), per = (total + 7) / 8;
        const uint32_t o = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
        if (o >= total) return false;
        const uint32_t st = o / (S * S), w = o - st * (S * S);
        const uint32_t tx = (st % nsx) * S + w % S, ty = (st / nsx) * S + w / S;
        if (tx >= ntx || ty >= nty) return false;
        tile = ty * ntx + tx;
        return true;
    }
    const uint32_t n = *gi.tile_count, per = (n + 7) / 8;
    const uint32_t i = blockIdx.x >> 3, k = (blockIdx.x & 7u) * per + i;
    if (i >= per || k >= n) return false;
    tile = gi.tile_list[k];
    return true;
}

/* Per-pixel gather, packed fp32: one lane per pixel, four 8x8 wave tiles per
 * 256-thread block (neighbouring lanes share photons in L1), tiles dealt to
 * the eight XCDs in contiguous bands (neighbouring tiles share one L2).
 *
 * The work of a lane is the list of sub-row chords of its window (see the
 * photon-grid layout above); the reference walks the (z,y) cell rows of the
 * window (IndirectRadianceEstimation.cu:95-129) and so would a nested loop
 * here, but then a wave runs, per row and sub-row, as long as its longest
 * lane: the sum of maxima.  Instead the chords are collected first (phase A:
 * up to GQ non-empty [first, end) photon ranges per lane, in LDS) and then
 * walked as one flat stream of batches (phase B), so the wave runs for the
 * maximum of the lanes' sums.  A batch is four consecutive photons, one
 * dwordx4 buffer load per SoA plane (one VGPR offset, plane offsets in
 * SGPRs), two photons per packed instruction:
 *   1. positions -> d^2 <= r^2 (the oracle's unfused operations);
 *   2. if any lane photon is within r: the int8 direction word -> facing
 *      test by v_dot4_i32_i8, exact fp32 directions only inside the band
 *      (DIRQ_BAND; same decisions as the exact test, by the bound at dir_q8);
 *   3. if any photon is accepted: powers, kernel weight, accumulation.
 * So the accepted photon set is bit-identical to the reference's; the kernel
 * weight (photonPower, :59-67) and the sums, which the device accumulates in
 * a different order anyway, use fused multiply-adds (within ~1e-7 per term).
 * The visit counters are the reference's whole-window counts (:113/:124). */
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4))); /* dword-aligned float4 */
__device__ __forceinline__ v2f lo2(float4 v) { return v2f{v.x, v.y}; }
__device__ __forceinline__ v2f hi2(float4 v) { return v2f{v.z, v.w}; }
__device__ __forceinline__ v2f lo2(f4u v) { return v2f{v.x, v.y}; }
__device__ __forceinline__ v2f hi2(f4u v) { return v2f{v.z, v.w}; }
/* sorted-photon plane load: one buffer resource over the planes, the plane's
 * byte offset in an SGPR (soffset) and the photon's byte offset in a VGPR, so
 * the loads of a batch share one address register */
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4u ldp(__amdgpu_buffer_rsrc_t rs, uint32_t so, uint32_t bo) {
    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)bo, (int)so, 0);
    return f4u{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0; }

/* The reference's visit counters of a window (IndirectRadianceEstimation.cu:113/:124): every
 * (z,y) row from x_lo to x_hi, whole rows, two offset reads per row.  Eight rows' reads are
 * issued before any is used (one memory round trip per eight rows instead of per row). */
__device__ __forceinline__ void window_visits(const uint32_t* __restrict__ offsets, uint32_t gx, uint32_t gy,
                                              uint32_t x_lo, uint32_t x_hi, uint32_t y_lo, uint32_t ny,
                                              uint32_t z_lo, uint32_t nrows, uint32_t& dC, uint32_t& dP) {
    uint32_t z = z_lo, yy = y_lo;
    for (uint32_t t0 = 0; t0 < nrows; t0 += 8) {
        uint32_t a[8], b[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            a[k] = b[k] = 0;
            if (t0 + k < nrows) {
                const uint32_t from = x_lo + yy * gx + z * gx * gy;
                a[k] = offsets[from];
                b[k] = offsets[from + (x_hi - x_lo) + 1];
                if (++yy == y_lo + ny) yy = y_lo, z++;
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) dP += b[k] - a[k];
    }
    dC += nrows;
}

/* photonPower (IndirectRadianceEstimation.cu:59-67), w = alpha*(1 - (1 - exp(-beta d^2 / 2r^2)) /
 * (1 - e^-beta)), evaluated as one degree-5 polynomial in u = d^2/r^2: the minimax fit of w(u) on
 * [0, 1] (relative error 7.7e-7; 1.2e-6 with fp32 coefficients and Horner rounding).  One v_pk_mul
 * and five v_pk_fma_f32 per pair of photons, the coefficients compile-time constants (SGPRs); the
 * accepted photons are decided by the exact distance test, so only the weights (and the sums,
 * summed in another order anyway) differ from the oracle's. */
constexpr float ORX_W5_C0 = 1.8179986476898193f, ORX_W5_C1 = -2.0686328411102295f;
constexpr float ORX_W5_C2 = 1.0091534852981567f, ORX_W5_C3 = -0.32518523931503296f;
constexpr float ORX_W5_C4 = 0.07352562248706818f, ORX_W5_C5 = -0.009477914310991764f;
__device__ __forceinline__ v2f weight2u(v2f u);
__device__ __forceinline__ v2f weight2(v2f ir2, v2f d2) { return weight2u(d2 * ir2); }
/* packed broadcasts through op_sel: `pair.lo - x`, `pair.hi - x`, `a * pair.lo`, `a * pair.hi`
 * on both halves of x / a.  The union kernel keeps its hit point, normal and 1/r^2 two to a
 * register pair (four pairs instead of seven broadcast pairs: the kernel's VGPR budget sets its
 * waves per SIMD); the arithmetic is the same IEEE operation as the broadcast form. */
__device__ __forceinline__ v2f pk_sub_blo(v2f pair, v2f x) {
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(pair), "v"(x));
    return r;
}
__device__ __forceinline__ v2f pk_sub_bhi(v2f pair, v2f x) {
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(pair), "v"(x));
    return r;
}
__device__ __forceinline__ v2f pk_mul_blo(v2f a, v2f pair) {
    v2f r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(pair));
    return r;
}
__device__ __forceinline__ v2f pk_mul_bhi(v2f a, v2f pair) {
    v2f r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(pair));
    return r;
}
__device__ __forceinline__ v2f weight2u(v2f u) {
    v2f p = __builtin_elementwise_fma(v2f{ORX_W5_C5, ORX_W5_C5}, u, v2f{ORX_W5_C4, ORX_W5_C4});
    p = __builtin_elementwise_fma(p, u, v2f{ORX_W5_C3, ORX_W5_C3});
    p = __builtin_elementwise_fma(p, u, v2f{ORX_W5_C2, ORX_W5_C2});
    p = __builtin_elementwise_fma(p, u, v2f{ORX_W5_C1, ORX_W5_C1});
    return __builtin_elementwise_fma(p, u, v2f{ORX_W5_C0, ORX_W5_C0});
}
/* The union gather's form: the same polynomial in d^2 with coefficients c_k / r^(2k) (one radius per
 * launch: uniform, in SGPRs), so the u = d^2 / r^2 multiply per pair leaves the batch, and divided
 * through by the d^8 coefficient c_4 / r^8 (`scale`), so the first Horner step adds the inline
 * constant 1 (a coefficient pair in the first step would need a VGPR copy per batch: the packed
 * FMA reads one SGPR operand); the lane's sums are multiplied by `scale` once at the end.  The host
 * takes it only where the coefficients and the scale keep the sums in range (launch_ppm_gather). */
struct WPoly {
    float k[6]; /* k[4] = 1 */
    float scale;
};
__device__ __forceinline__ v2f weight2d(v2f d2, const WPoly& w) {
    v2f p = __builtin_elementwise_fma(v2f{w.k[5], w.k[5]}, d2, v2f{1.f, 1.f});
    p = __builtin_elementwise_fma(p, d2, v2f{w.k[3], w.k[3]});
    p = __builtin_elementwise_fma(p, d2, v2f{w.k[2], w.k[2]});
    p = __builtin_elementwise_fma(p, d2, v2f{w.k[1], w.k[1]});
    return __builtin_elementwise_fma(p, d2, v2f{w.k[0], w.k[0]});
}
/* int8 facing prefilter dot products of four photons' direction words with the hit point's nq.
 * gfx950 runs v_dot* like its matrix-core instructions: another VALU instruction may read a dot's
 * result only three wait states after it.  The compiler pads the instructions it emits but not
 * those inside inline assembly, so the four dots and the wait states are one asm block (outputs
 * early-clobbered: no dot overwrites a word a later one reads), with the inline 0 accumulator (the
 * builtin selects v_dot4c_i32_i8, whose accumulator costs a v_mov per dot: hall 1026 -> 1020
 * Mpaths/s).  A single-dot asm statement was correct only while the scheduler happened to put
 * three instructions between each dot and its compare; the two-hit-point gather variant's schedule
 * read a result one instruction later and dropped photons (profiles/r05h_gather_two_hitpoints_ab.txt).
 * tests/test_asm_hazards.py checks every inline dot of the compiled kernels. */
__device__ __forceinline__ void sdot4x4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int32_t nq, int32_t& q0,
                                        int32_t& q1, int32_t& q2, int32_t& q3) {
    asm("v_dot4_i32_i8 %0, %4, %8, 0\n\t"
        "v_dot4_i32_i8 %1, %5, %8, 0\n\t"
        "v_dot4_i32_i8 %2, %6, %8, 0\n\t"
        "v_dot4_i32_i8 %3, %7, %8, 0\n\t"
        "s_nop 2"
        : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3)
        : "v"(w0), "v"(w1), "v"(w2), "v"(w3), "v"(nq));
}

constexpr uint32_t GQ = 8; /* chord ranges per lane per phase A (LDS: GQ * 8 B per lane) */

/* the hit point's sphere (grown by a margin far above the rounding of the distance test) misses
 * the AABB of this rank's photons */
__device__ __forceinline__ bool sphere_misses_grid(const GridParams& g, f3 pos, float r) {
    const float m = r * 1e-3f + g.cell * 1e-3f, rr = r + m;
    return pos.x + rr < g.clo[0] || pos.x - rr > g.chi[0] || pos.y + rr < g.clo[1] || pos.y - rr > g.chi[1] ||
           pos.z + rr < g.clo[2] || pos.z - rr > g.chi[2];
}
/* a hit point this rank does not gather: cull 1, its sphere misses the rank's photons; cull 2
 * (slab mode), its position's bin on the slab axis is another rank's (every photon within r of
 * an owned hit point was sent here with the halo, so owners gather complete windows) */
__device__ __forceinline__ bool gather_skips(const GatherIn& gi, const GridParams& g, f3 pos, float r) {
    if (gi.cull == 2) {
        const float v = gi.own_axis == 0 ? pos.x : gi.own_axis == 1 ? pos.y : pos.z;
        const uint32_t b = slab_bin(gi.own_sb, v, gi.own_axis);
        return b < gi.own_lo || b > gi.own_hi;
    }
    return gi.cull == 1 && sphere_misses_grid(g, pos, r);
}

/* NSUB: sub-rows per cell row (SUBR^2, or 1 for the cell-order layout) */
template <uint32_t NSUB>
#ifndef ORX_GATHER_LANE_WAVES
#define ORX_GATHER_LANE_WAVES 7 /* waves per SIMD the per-lane gather is register-capped for (72 VGPRs, no spills) */
#endif
__global__ __launch_bounds__(256, ORX_GATHER_LANE_WAVES) void k_ppm_gather(GatherIn gi, PhotonBufs pb, Consts c, uint32_t ntx,
                                                    uint32_t ntiles) {
    __shared__ uint2 rq[GQ][256];
    const uint32_t tid = threadIdx.x;
    uint32_t tile;
    if (!gather_tile(gi, ntx, ntiles, tile)) return; /* block-uniform */
    const uint32_t w = tid >> 6, l = tid & 63;
    const uint32_t x = (tile % ntx) * 16 + (w & 1) * 8 + (l & 7);
    const uint32_t y = (tile / ntx) * 16 + (w >> 1) * 8 + (l >> 3);
    const uint32_t j = gather_row(gi, y);
    const GridParams g = *pb.grid;
    uint32_t dC = 0, dP = 0;
    ORX_TS_DECL;
    const bool live = tile < ntiles && x < gi.W && y < gi.segments * gi.seg_rows;
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    float2 Cc = make_float2(0.f, 0.f);
    size_t i = 0;
    if (live) {
        i = (size_t)j * gi.W + x;
        hp_load(gi, j, x, A, B, Cc);
    }
    const uint32_t flags = __float_as_uint(A.w);
    const f3 pos = mk(A.x, A.y, A.z);
    const float radius2 = c.ppm_radius2;
    const float radius = c.ppm_radius;
    const float invCellSize = 1.f / g.cell;
    const f3 np = pos - mk(g.ox, g.oy, g.oz);
    uint32_t x_lo = 0, x_hi = 0, y_lo = 0, z_lo = 0, ny = 0, nrows = 0;
    if (live && (flags & PRD_HIT_NON_SPECULAR) && g.G && !gather_skips(gi, g, pos, radius)) {
        const int32_t ixl = orx_f2i_sat((np.x - radius) * invCellSize);
        const int32_t iyl = orx_f2i_sat((np.y - radius) * invCellSize);
        const int32_t izl = orx_f2i_sat((np.z - radius) * invCellSize);
        x_lo = (uint32_t)(ixl > 0 ? ixl : 0);
        y_lo = (uint32_t)(iyl > 0 ? iyl : 0);
        z_lo = (uint32_t)(izl > 0 ? izl : 0);
        const uint32_t ux = orx_f2u_sat((np.x + radius) * invCellSize);
        const uint32_t uy = orx_f2u_sat((np.y + radius) * invCellSize);
        const uint32_t uz = orx_f2u_sat((np.z + radius) * invCellSize);
        x_hi = (g.gx - 1) < ux ? (g.gx - 1) : ux;
        const uint32_t y_hi = (g.gy - 1) < uy ? (g.gy - 1) : uy;
        const uint32_t z_hi = (g.gz - 1) < uz ? (g.gz - 1) : uz;
        if (x_lo <= x_hi && y_lo <= y_hi && z_lo <= z_hi) {
            ny = y_hi - y_lo + 1;
            nrows = (z_hi - z_lo + 1) * ny;
            if (gi.visits) window_visits(pb.offsets, g.gx, g.gy, x_lo, x_hi, y_lo, ny, z_lo, nrows, dC, dP);
        }
    }
    const v2f irr = v2f{1.0f / radius2, 0.f}; /* pairs broadcast through op_sel (pk_sub_blo ...) */
    v2f accx = v2f{0.f, 0.f}, accy = accx, accz = accx;
    const v2f pxy = v2f{pos.x, pos.y}, pzn = v2f{pos.z, B.x}, nyz = v2f{B.y, B.z};
    const int32_t nq = (int32_t)dir_q8(B.x, B.y, B.z);
    /* SP_PLANES * splane * 4 < 4 GiB: checked on the host (resize) */
    const __amdgpu_buffer_rsrc_t SR = __builtin_amdgcn_make_buffer_rsrc((void*)pb.sorted, 0, 0xffffffff, 0x00020000);
    const uint32_t PB = pb.splane * 4u;
    /* a sub-row's box grown by m (covers the rounding of the cell / half-cell
     * assignment) that misses the sphere holds no photon within r; otherwise
     * only the x quarters the chord [p.x - rx, p.x + rx] (+m) touches are walked */
    const float m = g.cell * 1e-3f;
    constexpr uint32_t HS = NSUB > 1 ? SUBR : 1u;
    const float hc = g.cell / (float)HS; /* exact: HS is 1 or 2 */
    uint32_t t = 0;
    while (wave_any(t < nrows)) {
        /* phase A: the next up to GQ non-empty chords of this lane's window, in LDS */
        ORX_TS_WAVE(ts_wl); /* trav stats: wave-level phase-A rounds */
        uint32_t n = 0;
        while (t < nrows && n + NSUB <= GQ) {
            const uint32_t zq = t / ny;
            const uint32_t z = z_lo + zq, yy = y_lo + (t - zq * ny);
            t++;
            uint32_t offs[NSUB], ends[NSUB];
#pragma unroll
            for (uint32_t sr = 0; sr < NSUB; sr++) {
                offs[sr] = ends[sr] = 0;
                const uint32_t hz = z * HS + sr / HS, hy = yy * HS + sr % HS;
                const float zc0 = g.oz + (float)hz * hc - m, zc1 = g.oz + (float)(hz + 1) * hc + m;
                const float dz = fmaxf(0.f, fmaxf(zc0 - pos.z, pos.z - zc1));
                const float yc0 = g.oy + (float)hy * hc - m, yc1 = g.oy + (float)(hy + 1) * hc + m;
                const float dy = fmaxf(0.f, fmaxf(yc0 - pos.y, pos.y - yc1));
                const float rem = radius2 - dy * dy - dz * dz;
                if (rem < 0.f) continue;
                const float rx = sqrtf(rem) + m;
                const int32_t cxl = orx_f2i_sat(orx_floorf((np.x - rx) * invCellSize));
                const int32_t cxh = orx_f2i_sat(orx_floorf((np.x + rx) * invCellSize));
                const uint32_t xl = cxl > (int32_t)x_lo ? (uint32_t)cxl : x_lo;
                const uint32_t xh = cxh < (int32_t)x_hi ? (uint32_t)cxh : x_hi;
                if (cxh < 0 || xl > xh) continue;
                /* x-quarter trimming of the chord's end cells */
                const float sx = invCellSize * (float)SUBX;
                const int32_t q0 = orx_f2i_sat(orx_floorf((np.x - rx) * sx));
                const int32_t q1 = orx_f2i_sat(orx_floorf((np.x + rx) * sx));
                const uint32_t a0 = q0 > (int32_t)(SUBX * xl) ? (uint32_t)q0 : SUBX * xl;
                const uint32_t a1 = q1 < (int32_t)(SUBX * xh + SUBX - 1) ? (uint32_t)q1 : SUBX * xh + SUBX - 1;
                if (q1 < 0 || a0 > a1) continue;
                const uint32_t* so = pb.subofs + ((size_t)(yy + z * g.gy) * NSUB + sr) * g.gx * SUBX;
                offs[sr] = so[a0];
                ends[sr] = so[a1 + 1];
            }
#pragma unroll
            for (uint32_t sr = 0; sr < NSUB; sr++)
                if (ends[sr] > offs[sr]) rq[n++][tid] = make_uint2(offs[sr], ends[sr]);
        }
        /* phase B: one flat stream of batches over the collected chords */
        uint32_t k = 0, kb = 0, kend = 0;
        for (;;) {
            while (kb >= kend && k < n) {
                const uint2 r = rq[k++][tid];
                kb = r.x;
                kend = r.y;
                ORX_TS_INC(ts_leaves, 1);
            }
            const bool has = kb < kend;
            if (!wave_any(has)) break;
            if (!has) continue;
            ORX_TS_INC(ts_nodes, 1);
            ORX_TS_WAVE(ts_wn);
            const uint32_t bo = kb << 2;
            const f4u X = ldp(SR, SP_X * PB, bo), Y = ldp(SR, SP_Y * PB, bo), Z = ldp(SR, SP_Z * PB, bo);
            const v2f dx0 = pk_sub_blo(pxy, lo2(X)), dx1 = pk_sub_blo(pxy, hi2(X));
            const v2f dy0 = pk_sub_bhi(pxy, lo2(Y)), dy1 = pk_sub_bhi(pxy, hi2(Y));
            const v2f dz0 = pk_sub_blo(pzn, lo2(Z)), dz1 = pk_sub_blo(pzn, hi2(Z));
            const v2f d20 = (dx0 * dx0 + dy0 * dy0) + dz0 * dz0;
            const v2f d21 = (dx1 * dx1 + dy1 * dy1) + dz1 * dz1;
            bool in0 = d20.x <= radius2;
            bool in1 = kb + 1 < kend && d20.y <= radius2;
            bool in2 = kb + 2 < kend && d21.x <= radius2;
            bool in3 = kb + 3 < kend && d21.y <= radius2;
            kb += 4;
            if (!(in0 | in1 | in2 | in3)) continue;
            /* facing: dot(-dir, n) >= 0  <=>  dot(dir, n) <= 0 (negation is exact) */
            const u4v Q = __builtin_amdgcn_raw_buffer_load_b128(SR, (int)bo, (int)(SP_DIRQ * PB), 0);
            int32_t q0, q1, q2, q3;
            sdot4x4(Q.x, Q.y, Q.z, Q.w, nq, q0, q1, q2, q3);
            in0 = in0 && q0 <= DIRQ_BAND;
            in1 = in1 && q1 <= DIRQ_BAND;
            in2 = in2 && q2 <= DIRQ_BAND;
            in3 = in3 && q3 <= DIRQ_BAND;
            const bool u0 = in0 && q0 >= -DIRQ_BAND, u1 = in1 && q1 >= -DIRQ_BAND;
            const bool u2 = in2 && q2 >= -DIRQ_BAND, u3 = in3 && q3 >= -DIRQ_BAND;
            if (u0 | u1 | u2 | u3) { /* inside the band: the exact test */
                const f4u DX = ldp(SR, SP_DX * PB, bo), DY = ldp(SR, SP_DY * PB, bo), DZ = ldp(SR, SP_DZ * PB, bo);
                const v2f nd0 = (pk_mul_bhi(lo2(DX), pzn) + pk_mul_blo(lo2(DY), nyz)) + pk_mul_bhi(lo2(DZ), nyz);
                const v2f nd1 = (pk_mul_bhi(hi2(DX), pzn) + pk_mul_blo(hi2(DY), nyz)) + pk_mul_bhi(hi2(DZ), nyz);
                in0 = in0 && (!u0 || nd0.x <= 0.f);
                in1 = in1 && (!u1 || nd0.y <= 0.f);
                in2 = in2 && (!u2 || nd1.x <= 0.f);
                in3 = in3 && (!u3 || nd1.y <= 0.f);
            }
            if (!(in0 | in1 | in2 | in3)) continue;
            const f4u WX = ldp(SR, SP_PX * PB, bo), WY = ldp(SR, SP_PY * PB, bo), WZ = ldp(SR, SP_PZ * PB, bo);
            /* the weight of every photon of the batch (rejected ones get 0 by select) */
            v2f w0 = weight2u(pk_mul_blo(d20, irr)), w1 = weight2u(pk_mul_blo(d21, irr));
            ORX_TS_INC(ts_tris, (uint32_t)in0 + (uint32_t)in1 + (uint32_t)in2 + (uint32_t)in3);
            w0.x = in0 ? w0.x : 0.f;
            w0.y = in1 ? w0.y : 0.f;
            w1.x = in2 ? w1.x : 0.f;
            w1.y = in3 ? w1.y : 0.f;
            accx = __builtin_elementwise_fma(lo2(WX), w0, accx);
            accy = __builtin_elementwise_fma(lo2(WY), w0, accy);
            accz = __builtin_elementwise_fma(lo2(WZ), w0, accz);
            accx = __builtin_elementwise_fma(hi2(WX), w1, accx);
            accy = __builtin_elementwise_fma(hi2(WY), w1, accy);
            accz = __builtin_elementwise_fma(hi2(WZ), w1, accz);
        }
    }
    if (live) {
        const float ax = accx.x + accx.y, ay = accy.x + accy.y, az = accz.x + accz.y;
        const f3 att = mk(B.w, Cc.x, Cc.y);
        const float s1 = 1.0f / (ORX_PI_F * c.ppm_radius2);
        const float s2 = 1.0f / c.emitted_f;
        const f3 ind = ((mk(ax, ay, az) * att) * s1) * s2;
        gi.indirect[3 * i + 0] = ind.x;
        gi.indirect[3 * i + 1] = ind.y;
        gi.indirect[3 * i + 2] = ind.z;
        if (gi.dbg) {
            gi.dbg[2 * i] = dC;
            gi.dbg[2 * i + 1] = dP;
        }
    }
#ifdef ORX_TRAV_STATS
    atomicAdd((unsigned long long*)&pb.grid->st_lane_batches, (unsigned long long)ts_nodes);
    atomicAdd((unsigned long long*)&pb.grid->st_wave_batches, (unsigned long long)ts_wn);
    atomicAdd((unsigned long long*)&pb.grid->st_lane_rows, (unsigned long long)ts_leaves);
    atomicAdd((unsigned long long*)&pb.grid->st_wave_rows, (unsigned long long)ts_wl);
    atomicAdd((unsigned long long*)&pb.grid->st_accepted, (unsigned long long)ts_tris);
#endif
    const uint64_t sp = wave_sum_u64(dP), sc = wave_sum_u64(dC);
    if ((threadIdx.x & 63) == 0 && sp) {
        atomicAdd((unsigned long long*)&pb.grid->photons_visited, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->cells_visited, (unsigned long long)sc);
        atomicAdd((unsigned long long*)&pb.grid->photons_visited_total, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->cells_visited_total, (unsigned long long)sc);
    }
}

/* Wave-broadcast gather over the union of a wave's chords.
 *
 * The per-lane gather above is bound by the vector-memory address path: every
 * dwordx4 photon load costs the TA ~16-20 cycles whatever the lanes share, for
 * four photons of one lane.  Here a wave walks, sub-row by sub-row, the union
 * of its 64 lanes' chords and reads each photon ONCE: 64 photons per coalesced
 * load into the wave's LDS image, then every lane reads the same batch of four
 * (ds_read_b128 broadcast), so the cost per photon is the lanes' arithmetic
 * (union_chunk_lds; only the exact directions inside the facing band are
 * scalar loads).
 * Each lane accepts exactly the photons of its own chord range (the per-lane
 * kernel's candidate set, [subofs[a0], subofs[a1 + 1]) inside its reference
 * window) that pass its distance and facing tests, so the accepted set per
 * pixel is the per-lane kernel's (= the reference's); the union only adds
 * photons a lane rejects.  Lanes are 8x8 pixel tiles (hitpoints of neighbouring
 * pixels are near each other in the scene).
 * Per batch of four photons: positions -> d^2 test and the lane's range test;
 * a batch no lane accepts ends there (one ballot); then the int8 direction
 * words -> facing, exact directions only inside the band; then powers. */
/* Wave-uniform min / max over the 64 lanes (callers run with EXEC all ones): DPP moves inside
 * each row of 16 lanes (quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, row_ror 8: VALU operands, no
 * LDS round trip), then the four row results by v_readlane and scalar min/max.  A __shfl_xor
 * butterfly is six dependent ds_bpermute_b32 round trips; the union gather reduces twice per
 * sub-row. */
template <bool MIN>
__device__ __forceinline__ uint32_t wave_minmax_u32(uint32_t v) {
    auto op = [](uint32_t a, uint32_t b) { return MIN ? min(a, b) : max(a, b); };
    v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false));
    v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return wave_minmax_u32<true>(v); }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) { return wave_minmax_u32<false>(v); }
/* uniform 16-B read of a photon plane through the scalar unit */
__device__ __forceinline__ f4u sload4(const float* __restrict__ plane, uint32_t k) {
    return *reinterpret_cast<const f4u*>(plane + k);
}
__device__ __forceinline__ u4v sload4u(const float* __restrict__ plane, uint32_t k) {
    return *reinterpret_cast<const u4v*>(plane + k);
}
struct UChunk { /* lane k: photon c + k of the chunk */
    float X, Y, Z, WX, WY, WZ;
    uint32_t Q;
};
__device__ __forceinline__ UChunk uload_chunk(const float* __restrict__ SX, const float* __restrict__ SY,
                                              const float* __restrict__ SZ, const float* __restrict__ SQ,
                                              const float* __restrict__ SPX, const float* __restrict__ SPY,
                                              const float* __restrict__ SPZ, uint32_t k) {
    UChunk b;
    b.X = SX[k];
    b.Y = SY[k];
    b.Z = SZ[k];
    b.Q = __float_as_uint(SQ[k]);
    b.WX = SPX[k];
    b.WY = SPY[k];
    b.WZ = SPZ[k];
    return b;
}
/* The union kernel's per-batch constants and accumulators (LDS-broadcast form) */
struct UAcc {
    v2f accx, accy, accz;
};
struct UConst {
    v2f pxy, pzn, nyz, irr; /* (p.x, p.y), (p.z, n.x), (n.y, n.z), (1/r^2, -) */
    int32_t nq;
    const float* SDX;
    const float* SDY;
    const float* SDZ;
};
/* One 64-photon chunk of a sub-row's union, staged in the wave's LDS image L[7][64]
 * (x y z dirq px py pz; slots past the sub-row's end hold x = +inf, so no lane can
 * accept them).  Batches of four photons are read by every lane from the same LDS
 * address (ds_read_b128 broadcast: LDS-array cycles, no VALU), then:
 *   d^2 <= r2 (r2 = -1 for a lane without a chord on this sub-row), and with RANGE the
 *   lane's chord test [lo, lo + len); the facing prefilter; the weight and sums.
 * RANGE = false when every lane's chord is its whole margin-grown extent on the
 * sub-row (not cut by its reference window): then a union photon outside the chord
 * is farther than r from the lane's hit point (the margin argument of the chord
 * trimming), so the distance test alone decides, as the per-lane kernel's chord +
 * distance tests do. */
template <bool RANGE, bool DF>
__device__ __forceinline__ void union_chunk_lds(const float* __restrict__ L, uint32_t c, uint32_t ce, uint32_t lo,
                                                uint32_t len, float r2, const UConst& k, const WPoly& wp, UAcc& a) {
    const float4* L4 = reinterpret_cast<const float4*>(L);
    /* one batch of four; two per loop step, so the second batch's LDS reads take the first's address
     * plus an offset (one address increment per two batches) */
    auto batch = [&](const uint32_t e) {
        const uint32_t kb = c + e;
        const float4 X = L4[e >> 2], Y = L4[16 + (e >> 2)], Z = L4[32 + (e >> 2)];
        const v2f dx0 = pk_sub_blo(k.pxy, lo2(X)), dx1 = pk_sub_blo(k.pxy, hi2(X));
        const v2f dy0 = pk_sub_bhi(k.pxy, lo2(Y)), dy1 = pk_sub_bhi(k.pxy, hi2(Y));
        const v2f dz0 = pk_sub_blo(k.pzn, lo2(Z)), dz1 = pk_sub_blo(k.pzn, hi2(Z));
        const v2f d20 = (dx0 * dx0 + dy0 * dy0) + dz0 * dz0;
        const v2f d21 = (dx1 * dx1 + dy1 * dy1) + dz1 * dz1;
        bool in0 = d20.x <= r2, in1 = d20.y <= r2, in2 = d21.x <= r2, in3 = d21.y <= r2;
        if (RANGE) {
            const uint32_t t = kb - lo;
            in0 = in0 && t < len;
            in1 = in1 && t + 1 < len;
            in2 = in2 && t + 2 < len;
            in3 = in3 && t + 3 < len;
        }
        if (!wave_any(in0 | in1 | in2 | in3)) return;
        const uint4 Q = reinterpret_cast<const uint4*>(L4)[48 + (e >> 2)];
        int32_t q0, q1, q2, q3;
        sdot4x4(Q.x, Q.y, Q.z, Q.w, k.nq, q0, q1, q2, q3);
        in0 = in0 && q0 <= DIRQ_BAND;
        in1 = in1 && q1 <= DIRQ_BAND;
        in2 = in2 && q2 <= DIRQ_BAND;
        in3 = in3 && q3 <= DIRQ_BAND;
        const bool u0 = in0 && q0 >= -DIRQ_BAND, u1 = in1 && q1 >= -DIRQ_BAND;
        const bool u2 = in2 && q2 >= -DIRQ_BAND, u3 = in3 && q3 >= -DIRQ_BAND;
        /* The two tests below are lane-divergent ifs, not wave_any: the exec-mask save and skip is
         * scalar, where a ballot of these combined masks compiled to a select and a compare (two
         * VALU each, of ~56 per batch).  A lane that skips the sums adds fma(w, 0, acc) = acc. */
        if (u0 | u1 | u2 | u3) { /* inside the band: the exact test (rare) */
            const uint32_t ku = (uint32_t)__builtin_amdgcn_readfirstlane((int)kb);
            const f4u DX = sload4(k.SDX, ku), DY = sload4(k.SDY, ku), DZ = sload4(k.SDZ, ku);
            const v2f nd0 = (pk_mul_bhi(lo2(DX), k.pzn) + pk_mul_blo(lo2(DY), k.nyz)) + pk_mul_bhi(lo2(DZ), k.nyz);
            const v2f nd1 = (pk_mul_bhi(hi2(DX), k.pzn) + pk_mul_blo(hi2(DY), k.nyz)) + pk_mul_bhi(hi2(DZ), k.nyz);
            in0 = in0 && (!u0 || nd0.x <= 0.f);
            in1 = in1 && (!u1 || nd0.y <= 0.f);
            in2 = in2 && (!u2 || nd1.x <= 0.f);
            in3 = in3 && (!u3 || nd1.y <= 0.f);
        }
        if (in0 | in1 | in2 | in3) {
            const float4 WX = L4[64 + (e >> 2)], WY = L4[80 + (e >> 2)], WZ = L4[96 + (e >> 2)];
            v2f w0, w1;
            if (DF) {
                w0 = weight2d(d20, wp);
                w1 = weight2d(d21, wp);
            } else {
                w0 = weight2u(pk_mul_blo(d20, k.irr));
                w1 = weight2u(pk_mul_blo(d21, k.irr));
            }
            w0.x = in0 ? w0.x : 0.f;
            w0.y = in1 ? w0.y : 0.f;
            w1.x = in2 ? w1.x : 0.f;
            w1.y = in3 ? w1.y : 0.f;
            a.accx = __builtin_elementwise_fma(lo2(WX), w0, a.accx);
            a.accy = __builtin_elementwise_fma(lo2(WY), w0, a.accy);
            a.accz = __builtin_elementwise_fma(lo2(WZ), w0, a.accz);
            a.accx = __builtin_elementwise_fma(hi2(WX), w1, a.accx);
            a.accy = __builtin_elementwise_fma(hi2(WY), w1, a.accy);
            a.accz = __builtin_elementwise_fma(hi2(WZ), w1, a.accz);
        }
    };
    for (uint32_t e = 0; e < ce; e += 8) {
        batch(e);
        if (e + 4 < ce) batch(e + 4);
    }
}


/* Photons are broadcast through the wave's LDS image (union_chunk_lds), with the chord test
 * dropped on sub-rows where no lane's chord is cut by its window.  (A v_readlane broadcast from
 * the chunk registers measured 2.81 ms against 1.91 on the serial hall gather, 16x4 and 4x16
 * wave tiles slower than 8x8.)  Block = 16x16 pixels, four 8x8 wave tiles; blocks are dealt
 * XCD-major (block b runs on XCD b % 8 and takes the tiles [k per, (k+1) per) of XCD k). */
/* 7 waves per SIMD (at most 72 VGPRs): the next chunk's loads are not issued ahead of the
 * current chunk's batches (that prefetch held 7 VGPRs and kept the kernel at 5 waves), and the
 * hit point, normal and 1/r^2 sit two to a register pair, broadcast by op_sel (pk_sub_blo ...);
 * the extra waves hide more of the load latency than the prefetch did: 4K conference serial
 * gather 26.2 -> 24.7 ms at 6 waves, 24.2 at 7; configs[4] 8-rank gather 6.39 -> 6.01 ms; hall
 * unchanged.  The cell-order instance spills 8 VGPRs outside the batch loop. */
#ifndef ORX_UNION_WAVES
#define ORX_UNION_WAVES 7 /* waves per SIMD the union gather is register-capped for (at 8 it spills 37-49 VGPRs) */
#endif
template <uint32_t NSUB, bool DF>
__global__ __launch_bounds__(256, ORX_UNION_WAVES) void k_ppm_gather_union(GatherIn gi, PhotonBufs pb, Consts c, uint32_t ntx,
                                                          uint32_t ntiles, WPoly wp) {
    __shared__ float ulds[4][7 * 64];
    const uint32_t tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    uint32_t tile;
    if (!gather_tile(gi, ntx, ntiles, tile)) return; /* block-uniform */
    const uint32_t x = (tile % ntx) * 16 + (w & 1) * 8 + (l & 7);
    const uint32_t y = (tile / ntx) * 16 + (w >> 1) * 8 + (l >> 3);
    const uint32_t j = gather_row(gi, y);
    const bool live = tile < ntiles && x < gi.W && y < gi.segments * gi.seg_rows;
    const GridParams g = *pb.grid;
    uint32_t dC = 0, dP = 0;
    ORX_TS_DECL;
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    float2 Cc = make_float2(0.f, 0.f);
    size_t i = 0;
    if (live) {
        i = (size_t)j * gi.W + x;
        hp_load(gi, j, x, A, B, Cc);
    }
    const uint32_t flags = __float_as_uint(A.w);
    const f3 pos = mk(A.x, A.y, A.z);
    const float radius2 = c.ppm_radius2;
    const float radius = c.ppm_radius;
    const float invCellSize = 1.f / g.cell;
    const f3 np = pos - mk(g.ox, g.oy, g.oz);
    uint32_t x_lo = 1, x_hi = 0, y_lo = 1, y_hi = 0, z_lo = 1, z_hi = 0;
    bool act = false;
    if (live && (flags & PRD_HIT_NON_SPECULAR) && g.G && !gather_skips(gi, g, pos, radius)) {
        const int32_t ixl = orx_f2i_sat((np.x - radius) * invCellSize);
        const int32_t iyl = orx_f2i_sat((np.y - radius) * invCellSize);
        const int32_t izl = orx_f2i_sat((np.z - radius) * invCellSize);
        x_lo = (uint32_t)(ixl > 0 ? ixl : 0);
        y_lo = (uint32_t)(iyl > 0 ? iyl : 0);
        z_lo = (uint32_t)(izl > 0 ? izl : 0);
        const uint32_t ux = orx_f2u_sat((np.x + radius) * invCellSize);
        const uint32_t uy = orx_f2u_sat((np.y + radius) * invCellSize);
        const uint32_t uz = orx_f2u_sat((np.z + radius) * invCellSize);
        x_hi = (g.gx - 1) < ux ? (g.gx - 1) : ux;
        y_hi = (g.gy - 1) < uy ? (g.gy - 1) : uy;
        z_hi = (g.gz - 1) < uz ? (g.gz - 1) : uz;
        act = x_lo <= x_hi && y_lo <= y_hi && z_lo <= z_hi;
        if (act && gi.visits) /* the reference's visit counters: every (z,y) row of the window, whole rows */
            window_visits(pb.offsets, g.gx, g.gy, x_lo, x_hi, y_lo, y_hi - y_lo + 1, z_lo,
                          (z_hi - z_lo + 1) * (y_hi - y_lo + 1), dC, dP);
    }
    v2f accx = v2f{0.f, 0.f}, accy = accx, accz = accx;
    const int32_t nq = (int32_t)dir_q8(B.x, B.y, B.z);
    const float* __restrict__ SX = pb.sorted + (size_t)SP_X * pb.splane;
    const float* __restrict__ SY = pb.sorted + (size_t)SP_Y * pb.splane;
    const float* __restrict__ SZ = pb.sorted + (size_t)SP_Z * pb.splane;
    const float* __restrict__ SQ = pb.sorted + (size_t)SP_DIRQ * pb.splane;
    const float* __restrict__ SDX = pb.sorted + (size_t)SP_DX * pb.splane;
    const float* __restrict__ SDY = pb.sorted + (size_t)SP_DY * pb.splane;
    const float* __restrict__ SDZ = pb.sorted + (size_t)SP_DZ * pb.splane;
    const float* __restrict__ SPX = pb.sorted + (size_t)SP_PX * pb.splane;
    const float* __restrict__ SPY = pb.sorted + (size_t)SP_PY * pb.splane;
    const float* __restrict__ SPZ = pb.sorted + (size_t)SP_PZ * pb.splane;
    const float m = g.cell * 1e-3f;
    constexpr uint32_t HS = NSUB > 1 ? SUBR : 1u;
    const float hc = g.cell / (float)HS;
    const UConst UK{v2f{pos.x, pos.y}, v2f{pos.z, B.x}, v2f{B.y, B.z}, v2f{1.0f / radius2, 0.f}, nq, SDX, SDY, SDZ};
    UAcc UA{accx, accy, accz};
    /* the union of the lanes' windows (rows) */
    const uint32_t UZ0 = wave_min_u32(act ? z_lo : 0xffffffffu), UZ1 = wave_max_u32(act ? z_hi : 0u);
    const uint32_t UY0 = wave_min_u32(act ? y_lo : 0xffffffffu), UY1 = wave_max_u32(act ? y_hi : 0u);
    for (uint32_t z = UZ0; z <= UZ1 && UZ0 <= UZ1; z++) {
        for (uint32_t yy = UY0; yy <= UY1; yy++) {
            const bool inrow = act && z >= z_lo && z <= z_hi && yy >= y_lo && yy <= y_hi;
            const uint32_t rowc = yy + z * g.gy;
            for (uint32_t sr = 0; sr < NSUB; sr++) {
                /* this lane's chord on the sub-row (the per-lane kernel's), as quarter indices;
                 * cut: the chord is shorter than the margin-grown extent [q0, q1] inside the grid
                 * (its reference window ends inside it) */
                uint32_t a0 = 0xffffffffu, a1 = 0u;
                bool cut = false;
                if (inrow) {
                    const uint32_t hz = z * HS + sr / HS, hy = yy * HS + sr % HS;
                    const float zc0 = g.oz + (float)hz * hc - m, zc1 = g.oz + (float)(hz + 1) * hc + m;
                    const float dz = fmaxf(0.f, fmaxf(zc0 - pos.z, pos.z - zc1));
                    const float yc0 = g.oy + (float)hy * hc - m, yc1 = g.oy + (float)(hy + 1) * hc + m;
                    const float dy = fmaxf(0.f, fmaxf(yc0 - pos.y, pos.y - yc1));
                    const float rem = radius2 - dy * dy - dz * dz;
                    if (rem >= 0.f) {
                        const float rx = sqrtf(rem) + m;
                        const int32_t cxl = orx_f2i_sat(orx_floorf((np.x - rx) * invCellSize));
                        const int32_t cxh = orx_f2i_sat(orx_floorf((np.x + rx) * invCellSize));
                        const uint32_t xl = cxl > (int32_t)x_lo ? (uint32_t)cxl : x_lo;
                        const uint32_t xh = cxh < (int32_t)x_hi ? (uint32_t)cxh : x_hi;
                        if (cxh >= 0 && xl <= xh) {
                            const float sx = invCellSize * (float)SUBX;
                            const int32_t q0 = orx_f2i_sat(orx_floorf((np.x - rx) * sx));
                            const int32_t q1 = orx_f2i_sat(orx_floorf((np.x + rx) * sx));
                            const uint32_t b0 = q0 > (int32_t)(SUBX * xl) ? (uint32_t)q0 : SUBX * xl;
                            const uint32_t b1 =
                                q1 < (int32_t)(SUBX * xh + SUBX - 1) ? (uint32_t)q1 : SUBX * xh + SUBX - 1;
                            if (q1 >= 0 && b0 <= b1) {
                                a0 = b0;
                                a1 = b1;
                                const int32_t qmax = (int32_t)(SUBX * g.gx) - 1;
                                cut = (int32_t)b0 > (q0 > 0 ? q0 : 0) || (int32_t)b1 < (q1 < qmax ? q1 : qmax);
                            }
                        }
                    }
                }
                const uint32_t A0 = wave_min_u32(a0), A1 = wave_max_u32(a1);
                if (A0 > A1) continue;
                if (l == 0) ORX_TS_INC(ts_wl, 1); /* trav stats: sub-rows a wave walks */
                const uint32_t* so = pb.subofs + ((size_t)rowc * NSUB + sr) * g.gx * SUBX;
                const uint32_t U0 = so[A0], U1 = so[A1 + 1]; /* uniform: scalar loads */
                if (U0 >= U1) continue;
                if (l == 0) ORX_TS_INC(ts_tris, 1); /* trav stats (union kernel): sub-rows with photons */
                /* this lane's candidates [lo, lo + len): needed only on sub-rows where some lane's
                 * chord is cut (two scattered loads) */
#ifdef ORX_TRAV_STATS
                constexpr bool need_all = true;
#else
                constexpr bool need_all = false;
#endif
                const bool range = wave_any(cut);
                uint32_t lo = 0, len = 0;
                if ((need_all || range) && a0 <= a1) {
                    lo = so[a0];
                    len = so[a1 + 1] - lo;
                }
                ORX_TS_INC(ts_nodes, len);              /* trav stats: lane candidate photons */
                if (l == 0) ORX_TS_INC(ts_wn, U1 - U0); /* union photons of the wave */
                ORX_TS_INC(ts_leaves, 1);
                /* a lane without a chord here accepts nothing (its window excludes the
                 * sub-row, or its sphere misses it) */
                const float r2 = a0 <= a1 ? radius2 : -1.f;
                float* L = ulds[w];
                uint32_t cc = U0;
                while (cc < U1) {
                    const uint32_t cn = cc + 64;
                    const UChunk cur = uload_chunk(SX, SY, SZ, SQ, SPX, SPY, SPZ, cc + l);
                    const uint32_t ce = U1 - cc < 64 ? U1 - cc : 64;
                    L[l] = cc + l < U1 ? cur.X : INFINITY;
                    L[64 + l] = cur.Y;
                    L[128 + l] = cur.Z;
                    L[192 + l] = __uint_as_float(cur.Q);
                    L[256 + l] = cur.WX;
                    L[320 + l] = cur.WY;
                    L[384 + l] = cur.WZ;
                    __builtin_amdgcn_wave_barrier();
                    if (range) union_chunk_lds<true, DF>(L, cc, ce, lo, len, r2, UK, wp, UA);
                    else union_chunk_lds<false, DF>(L, cc, ce, lo, len, r2, UK, wp, UA);
                    __builtin_amdgcn_wave_barrier();
                    cc = cn;
                }
            }
        }
    }
    accx = UA.accx;
    accy = UA.accy;
    accz = UA.accz;
#ifdef ORX_TRAV_STATS
    atomicAdd((unsigned long long*)&pb.grid->st_lane_batches, (unsigned long long)ts_nodes);
    atomicAdd((unsigned long long*)&pb.grid->st_wave_batches, (unsigned long long)ts_wn);
    atomicAdd((unsigned long long*)&pb.grid->st_lane_rows, (unsigned long long)ts_leaves);
    atomicAdd((unsigned long long*)&pb.grid->st_wave_rows, (unsigned long long)ts_wl);
    atomicAdd((unsigned long long*)&pb.grid->st_accepted, (unsigned long long)ts_tris);
#endif
    if (live) {
        float ax = accx.x + accx.y, ay = accy.x + accy.y, az = accz.x + accz.y;
        if (DF) {
            ax *= wp.scale;
            ay *= wp.scale;
            az *= wp.scale;
        }
        const f3 att = mk(B.w, Cc.x, Cc.y);
        const float s1 = 1.0f / (ORX_PI_F * c.ppm_radius2);
        const float s2 = 1.0f / c.emitted_f;
        const f3 ind = ((mk(ax, ay, az) * att) * s1) * s2;
        gi.indirect[3 * i + 0] = ind.x;
        gi.indirect[3 * i + 1] = ind.y;
        gi.indirect[3 * i + 2] = ind.z;
        if (gi.dbg) {
            gi.dbg[2 * i] = dC;
            gi.dbg[2 * i + 1] = dP;
        }
    }
    const uint64_t sp = wave_sum_u64(dP), sc = wave_sum_u64(dC);
    if ((threadIdx.x & 63) == 0 && sp) {
        atomicAdd((unsigned long long*)&pb.grid->photons_visited, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->cells_visited, (unsigned long long)sc);
        atomicAdd((unsigned long long*)&pb.grid->photons_visited_total, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->cells_visited_total, (unsigned long long)sc);
    }
}

__global__ __launch_bounds__(256) void k_gather_tiles(GatherIn gi, PhotonBufs pb, Consts c, uint32_t ntx,
                                                      uint8_t* flags) {
    const uint32_t tile = blockIdx.x, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const uint32_t x = (tile % ntx) * 16 + (w & 1) * 8 + (l & 7);
    const uint32_t y = (tile / ntx) * 16 + (w >> 1) * 8 + (l >> 3);
    const uint32_t j = gather_row(gi, y);
    const bool live = x < gi.W && y < gi.segments * gi.seg_rows;
    const GridParams g = *pb.grid;
    bool act = false;
    if (live) {
        const float4 A = hp_load_a(gi, j, x);
        act = (__float_as_uint(A.w) & PRD_HIT_NON_SPECULAR) && g.G &&
              !gather_skips(gi, g, mk(A.x, A.y, A.z), c.ppm_radius);
    }
    const int any = __syncthreads_or(act);
    if (tid == 0) flags[tile] = (uint8_t)(any != 0);
    if (!any && live) {
        const size_t i = (size_t)j * gi.W + x;
        gi.indirect[3 * i + 0] = 0.f;
        gi.indirect[3 * i + 1] = 0.f;
        gi.indirect[3 * i + 2] = 0.f;
    }
}
/* one block: the flagged tiles in ascending order */
__global__ __launch_bounds__(1024) void k_tile_compact(const uint8_t* flags, uint32_t ntiles, uint32_t* list,
                                                       uint32_t* count) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t base;
    const uint32_t tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    if (tid == 0) base = 0;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < ntiles; t0 += 1024) {
        const uint32_t t = t0 + tid;
        const bool f = t < ntiles && flags[t];
        const uint64_t m = __ballot(f);
        const uint32_t pre = (uint32_t)__popcll(m & ((1ull << l) - 1ull));
        if (l == 0) wsum[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = base;
        for (uint32_t k = 0; k < w; k++) off += wsum[k];
        if (f) list[off + pre] = t;
        __syncthreads();
        if (tid == 0) {
            uint32_t tot = 0;
            for (uint32_t k = 0; k < 16; k++) tot += wsum[k];
            base += tot;
        }
        __syncthreads();
    }
    if (tid == 0) *count = base;
}
/* orx_export_hitpoints: the own rows' gather inputs in the 28-B exchange layout (plane A
 * pos|flags float4, plane N normal float3; GatherIn.raw) — the attenuation stays with the owner */
__global__ __launch_bounds__(256) void k_export_hp(PixelBufs px, uint32_t n, float* __restrict__ dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 B = px.hpB[i];
    reinterpret_cast<float4*>(dst)[i] = px.hpA[i];
    float* N = dst + 4 * hp_export_plane(n) + 3 * (size_t)i;
    N[0] = B.x;
    N[1] = B.y;
    N[2] = B.z;
}
/* orx_ppm_finish of a shard: own-row indirect = the summed unattenuated estimate times the hit
 * point's attenuation (IndirectRadianceEstimation.cu:220 multiplies before the normalisation;
 * the same value up to fp32 order) */
__global__ __launch_bounds__(256) void k_indirect_atten(PixelBufs px, uint32_t n, const float* __restrict__ in) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 B = px.hpB[i];
    const float2 Cc = px.hpC[i];
    px.indirect[3 * (size_t)i + 0] = in[3 * (size_t)i + 0] * B.w;
    px.indirect[3 * (size_t)i + 1] = in[3 * (size_t)i + 1] * Cc.x;
    px.indirect[3 * (size_t)i + 2] = in[3 * (size_t)i + 2] * Cc.y;
}
void launch_export_hp(hipStream_t s, const PixelBufs& px, uint32_t n, float* dst) {
    hipLaunchKernelGGL(k_export_hp, dim3((n + 255) / 256), dim3(256), 0, s, px, n, dst);
}
void launch_indirect_atten(hipStream_t s, const PixelBufs& px, uint32_t n, const float* in) {
    hipLaunchKernelGGL(k_indirect_atten, dim3((n + 255) / 256), dim3(256), 0, s, px, n, in);
}
void launch_gather_tiles(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const Consts& c, uint8_t* flags,
                         uint32_t* list, uint32_t* count) {
    const uint32_t rows = gi.segments * gi.seg_rows;
    const uint32_t ntx = (gi.W + 15) / 16, nty = (rows + 15) / 16, ntiles = ntx * nty;
    hipLaunchKernelGGL(k_gather_tiles, dim3(ntiles), dim3(256), 0, s, gi, pb, c, ntx, flags);
    hipLaunchKernelGGL(k_tile_compact, dim3(1), dim3(1024), 0, s, flags, ntiles, list, count);
}

void launch_ppm_gather(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const Consts& c) {
    const uint32_t rows = gi.segments * gi.seg_rows;
    const uint32_t ntx = (gi.W + 15) / 16, nty = (rows + 15) / 16, ntiles = ntx * nty;
    const uint32_t norder = gi.tile_list ? ntiles : gather_order_count(gi.order, ntx, nty);
    const dim3 grid(8 * ((norder + 7) / 8));
    /* The sharded gather (segments = ranks, cell-order layout, no visit counters) meets 1/N of
     * the photons.  Where a rank's photons are sparse in the grid the wave union's per-row work
     * outweighs the photons it shares and the per-lane kernel is faster: hall 1080p, 2048^2
     * launch (tools/shard_model.py, per-rank gather union / per-lane: N=2 1.29 / 1.56 ms, N=4
     * 0.73 / 0.80, N=8 0.47 / 0.43, i.e. 4.2 / 2.1 slots per grid cell at N=4 / 8); at the 4K
     * conference's 16M-photon launch the union is far ahead at N=8 too (8.4 slots per cell:
     * 6.41 / 9.34 ms).  So the per-lane kernel takes row shards of 8+ segments below 3 slots per
     * cell.  Measured on one device (serial hall gather / 4K conference frame): per-lane 2.5 ms /
     * 120 ms, union 1.91 / 53.3. */
    static const int kern = [] { /* ORX_GATHER_KERNEL: 0 auto, 1 union, 2 per-lane (A/B) */
        const char* e = getenv("ORX_GATHER_KERNEL");
        return e ? atoi(e) : 0;
    }();
    const bool lane = kern == 2 || (kern == 0 && gi.segments >= 8 && !gi.cull && pb.S < 3u * pb.gcells);
    if (lane) {
        if (pb.nsub == 1) hipLaunchKernelGGL((k_ppm_gather<1>), grid, dim3(256), 0, s, gi, pb, c, ntx, ntiles);
        else hipLaunchKernelGGL((k_ppm_gather<SUBR * SUBR>), grid, dim3(256), 0, s, gi, pb, c, ntx, ntiles);
        return;
    }
    /* the weight polynomial in d^2 divided through by c_4 / r^8 (weight2d) where that scale and the
     * coefficients are normal floats; else in u = d^2 / r^2 (weight2u) */
    static const int dform_env = [] {
        const char* e = getenv("ORX_GATHER_DFORM");
        return e ? atoi(e) : 1;
    }();
    WPoly wp{};
    bool df = dform_env != 0;
    {
        const double irr = (double)(1.0f / c.ppm_radius2);
        const double ck[6] = {ORX_W5_C0, ORX_W5_C1, ORX_W5_C2, ORX_W5_C3, ORX_W5_C4, ORX_W5_C5};
        const double c4 = ck[4] * irr * irr * irr * irr;
        /* a lane's sums carry a factor 1 / scale until the end: far inside fp32 for a scale in [1e-20, 1e20] */
        df = df && std::isfinite(c4) && std::fabs(c4) >= 1e-20 && std::fabs(c4) <= 1e20;
        double sc = 1.0;
        for (int k = 0; k < 6; k++, sc *= irr) {
            const double v = ck[k] * sc / c4;
            df = df && std::isfinite(v) && std::fabs(v) < 1e37 && std::fabs(v) > 1e-37;
            wp.k[k] = (float)v;
        }
        wp.k[4] = 1.f;
        wp.scale = (float)c4;
    }
    if (pb.nsub == 1) {
        if (df) hipLaunchKernelGGL((k_ppm_gather_union<1, true>), grid, dim3(256), 0, s, gi, pb, c, ntx, ntiles, wp);
        else hipLaunchKernelGGL((k_ppm_gather_union<1, false>), grid, dim3(256), 0, s, gi, pb, c, ntx, ntiles, wp);
    } else {
        if (df) hipLaunchKernelGGL((k_ppm_gather_union<SUBR * SUBR, true>), grid, dim3(256), 0, s, gi, pb, c, ntx, ntiles, wp);
        else hipLaunchKernelGGL((k_ppm_gather_union<SUBR * SUBR, false>), grid, dim3(256), 0, s, gi, pb, c, ntx, ntiles, wp);
    }
}

/* ------------------------------------------------------------------ */
/* spatial photon partition of the sharded gather (slab mode)          */
/* ------------------------------------------------------------------ */
/* Rank g of N receives every photon whose position falls in its slab of one axis of the scene
 * AABB, and gathers only the hit points whose sphere reaches its photons; the bins and the
 * bin -> rank table are the host's plan (multigpu.slab_plan) over the all-gathered histograms.
 * The bin of a position is computed by the one function below in the histogram and in the
 * pack, so the host's per-rank counts are exact. */
__device__ __forceinline__ bool slot_valid(const PhotonBufs& pb, uint32_t s) {
    const uint32_t p = s / pb.D, k = s - p * pb.D;
    return (pb.vmask[p] >> k) & 1u;
}
/* [2][3][nb] counts: the valid deposits of the own photon pass and the own rows' non-specular
 * hit points per bin of each axis; then [2][SLAB_VOX^3] counts of both over a coarse voxel grid
 * of the scene AABB (voxel x + V (y + V z)), which the plan uses to weigh each hit point by the
 * photon density around it.  LDS histograms, one global add per non-empty bin and block; the
 * voxel counters are 16-bit halves of one word (photons low, hit points high), so a block takes
 * a contiguous chunk of at most 65535 slots and 65535 pixels. */
constexpr uint32_t SLAB_MAX_BINS = 1024;
/* 24 KB of axis bins + 128 KB of voxel counts: one block per CU on gfx950's 160 KB LDS
 * (the Makefile's ARCH is gfx950 only; a smaller-LDS target fails here, not at launch) */
static_assert((6 * SLAB_MAX_BINS + SLAB_VOX * SLAB_VOX * SLAB_VOX) * 4 <= 160 * 1024,
              "k_slab_hist's LDS histograms exceed gfx950's 160 KB per workgroup");
__global__ __launch_bounds__(256) void k_slab_hist(PhotonBufs pb, PixelBufs px, SlabBins sb, SlabBins vb,
                                                   uint32_t cs, uint32_t cp, uint32_t* hist) {
    __shared__ uint32_t lh[6 * SLAB_MAX_BINS];
    __shared__ uint32_t lv[SLAB_VOX * SLAB_VOX * SLAB_VOX];
    const uint32_t n6 = 6 * sb.nb, NV = SLAB_VOX * SLAB_VOX * SLAB_VOX;
    for (uint32_t k = threadIdx.x; k < n6; k += blockDim.x) lh[k] = 0;
    for (uint32_t k = threadIdx.x; k < NV; k += blockDim.x) lv[k] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * cs, s1 = s0 + cs < pb.S ? s0 + cs : pb.S;
    for (uint32_t s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
        if (!slot_valid(pb, s)) continue;
        const float4 q = pb.pos4[s];
        atomicAdd(&lh[0 * sb.nb + slab_bin(sb, q.x, 0)], 1u);
        atomicAdd(&lh[1 * sb.nb + slab_bin(sb, q.y, 1)], 1u);
        atomicAdd(&lh[2 * sb.nb + slab_bin(sb, q.z, 2)], 1u);
        atomicAdd(&lv[slab_bin(vb, q.x, 0) + SLAB_VOX * (slab_bin(vb, q.y, 1) + SLAB_VOX * slab_bin(vb, q.z, 2))], 1u);
    }
    const uint32_t npx = px.rows * px.W;
    const uint32_t p0 = blockIdx.x * cp, p1 = p0 + cp < npx ? p0 + cp : npx;
    for (uint32_t i = p0 + threadIdx.x; i < p1; i += blockDim.x) {
        const float4 A = px.hpA[i];
        if (!(__float_as_uint(A.w) & PRD_HIT_NON_SPECULAR)) continue;
        atomicAdd(&lh[3 * sb.nb + slab_bin(sb, A.x, 0)], 1u);
        atomicAdd(&lh[4 * sb.nb + slab_bin(sb, A.y, 1)], 1u);
        atomicAdd(&lh[5 * sb.nb + slab_bin(sb, A.z, 2)], 1u);
        atomicAdd(&lv[slab_bin(vb, A.x, 0) + SLAB_VOX * (slab_bin(vb, A.y, 1) + SLAB_VOX * slab_bin(vb, A.z, 2))],
                  1u << 16);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < n6; k += blockDim.x)
        if (lh[k]) atomicAdd(&hist[k], lh[k]);
    uint32_t* hv = hist + n6 + 6; /* past the photon AABB words (k_slab_bbox) */
    for (uint32_t k = threadIdx.x; k < NV; k += blockDim.x) {
        const uint32_t v = lv[k];
        if (v & 0xffffu) atomicAdd(&hv[k], v & 0xffffu);
        if (v >> 16) atomicAdd(&hv[NV + k], v >> 16);
    }
}
void launch_slab_hist(hipStream_t s, const PhotonBufs& pb, const PixelBufs& px, const SlabBins& sb,
                      const SlabBins& vb, uint32_t* hist) {
    const uint32_t npx = px.rows * px.W;
    uint32_t blocks = std::max((pb.S + 65534) / 65535, (npx + 65534) / 65535);
    blocks = std::max(blocks, 64u);
    const uint32_t cs = (pb.S + blocks - 1) / blocks, cp = (npx + blocks - 1) / blocks;
    hipLaunchKernelGGL(k_slab_hist, dim3(blocks), dim3(256), 0, s, pb, px, sb, vb, cs, cp, hist);
}

/* valid deposits -> the send buffer, rank-major: photon record (9 floats: position, direction,
 * power) at cursor[rank]++.  A block takes SLAB_CHUNK slots: counts per destination in LDS,
 * one device atomic per destination reserves the block's run, then every photon takes its
 * place in it (the order inside a run is not the slot order: it only changes the gather's
 * fp32 summation order on the receiving rank) */
constexpr uint32_t SLAB_CHUNK = 4096;
constexpr uint32_t SLAB_MAX_RANKS = 64;
__global__ __launch_bounds__(256) void k_slab_pack(PhotonBufs pb, SlabBins sb, uint32_t axis, uint32_t halo,
                                                   const uint8_t* __restrict__ bin_dest, uint32_t world,
                                                   uint32_t* cursor, uint32_t cap, float* __restrict__ send) {
    __shared__ uint32_t cnt[SLAB_MAX_RANKS], base[SLAB_MAX_RANKS];
    for (uint32_t c0 = blockIdx.x * SLAB_CHUNK; c0 < pb.S; c0 += gridDim.x * SLAB_CHUNK) {
        const uint32_t c1 = c0 + SLAB_CHUNK < pb.S ? c0 + SLAB_CHUNK : pb.S;
        if (threadIdx.x < SLAB_MAX_RANKS) cnt[threadIdx.x] = 0;
        __syncthreads();
        for (uint32_t s = c0 + threadIdx.x; s < c1; s += blockDim.x) {
            if (!slot_valid(pb, s)) continue;
            const float4 q = pb.pos4[s];
            const float v = axis == 0 ? q.x : axis == 1 ? q.y : q.z;
            const uint32_t b = slab_bin(sb, v, axis);
            const uint32_t d0 = bin_dest[b > halo ? b - halo : 0u];
            const uint32_t d1 = bin_dest[b + halo < sb.nb ? b + halo : sb.nb - 1u];
            for (uint32_t d = d0; d <= d1; d++) atomicAdd(&cnt[d], 1u);
        }
        __syncthreads();
        if (threadIdx.x < world) {
            const uint32_t n = cnt[threadIdx.x];
            base[threadIdx.x] = n ? atomicAdd(&cursor[threadIdx.x], n) : 0u;
            cnt[threadIdx.x] = 0;
        }
        __syncthreads();
        for (uint32_t s = c0 + threadIdx.x; s < c1; s += blockDim.x) {
            if (!slot_valid(pb, s)) continue;
            const float4* rec = pb.slots + 4 * (size_t)s;
            const float4 a = rec[0], b = rec[1];
            const float pz = rec[2].x;
            const float v = axis == 0 ? a.x : axis == 1 ? a.y : a.z;
            const uint32_t bn = slab_bin(sb, v, axis);
            const uint32_t d0 = bin_dest[bn > halo ? bn - halo : 0u];
            const uint32_t d1 = bin_dest[bn + halo < sb.nb ? bn + halo : sb.nb - 1u];
            for (uint32_t d = d0; d <= d1; d++) { /* the owner and the ranks within the halo */
                const uint32_t o = base[d] + atomicAdd(&cnt[d], 1u);
                if (o >= cap) continue; /* a plan whose counts disagree with the photons: never write past */
                float* w = send + 9 * (size_t)o;
                w[0] = a.x; w[1] = a.y; w[2] = a.z;
                w[3] = b.x; w[4] = b.y; w[5] = b.z;
                w[6] = a.w; w[7] = b.w; w[8] = pz;
            }
        }
        __syncthreads();
    }
}
void launch_slab_pack(hipStream_t s, const PhotonBufs& pb, const SlabBins& sb, uint32_t axis, uint32_t halo,
                      const uint8_t* bin_dest, uint32_t world, uint32_t* cursor, uint32_t cap, float* send) {
    uint32_t blocks = (pb.S + SLAB_CHUNK - 1) / SLAB_CHUNK;
    blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
    hipLaunchKernelGGL(k_slab_pack, dim3(blocks), dim3(256), 0, s, pb, sb, axis, halo, bin_dest, world, cursor, cap,
                       send);
}

/* received photon records -> this rank's deposit records: record i is slot i of photon group
 * i / D (deposit mask bit i % D), with its compact position and the photon AABB of the grid
 * setup (the replicas k_grid_setup folds; reset beforehand) */
__global__ __launch_bounds__(256) void k_slab_import(PhotonBufs pb, const float* __restrict__ recv, uint32_t n) {
    float lo_x = INFINITY, lo_y = INFINITY, lo_z = INFINITY;
    float hi_x = -INFINITY, hi_y = -INFINITY, hi_z = -INFINITY;
    const uint32_t groups = (n + pb.D - 1) / pb.D;
    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t g_end = ((groups + T - 1) / T) * T; /* every lane runs the same trip count */
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < g_end; g += T) {
        if (g >= groups) continue;
        uint32_t mask = 0;
        for (uint32_t k = 0; k < pb.D; k++) {
            const uint32_t i = g * pb.D + k;
            if (i >= n) break;
            const float* w = recv + 9 * (size_t)i;
            const float x = w[0], y = w[1], z = w[2];
            float4* rec = pb.slots + 4 * (size_t)i;
            rec[0] = make_float4(x, y, z, w[6]);
            rec[1] = make_float4(w[3], w[4], w[5], w[7]);
            rec[2].x = w[8];
            pb.pos4[i] = make_float4(x, y, z, 0.f);
            mask |= 1u << k;
            lo_x = fminf(lo_x, x); lo_y = fminf(lo_y, y); lo_z = fminf(lo_z, z);
            hi_x = fmaxf(hi_x, x); hi_y = fmaxf(hi_y, y); hi_z = fmaxf(hi_z, z);
        }
        pb.vmask[g] = (uint8_t)mask;
    }
    photon_bbox_flush(pb, lo_x, lo_y, lo_z, hi_x, hi_y, hi_z, (blockIdx.x * 4 + (threadIdx.x >> 6)) & (BBOX_REPLICAS - 1),
                      threadIdx.x & 63);
}
__global__ void k_slab_bbox(PhotonBufs pb, uint32_t* out) {
    const uint32_t lane = threadIdx.x;
    for (int k = 0; k < 6; k++) {
        uint32_t v = pb.bbox[k * BBOX_REPLICAS + lane];
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
            v = k < 3 ? min(v, w) : max(v, w);
        }
        if (lane == 0) out[k] = v;
    }
}
void launch_slab_bbox(hipStream_t s, const PhotonBufs& pb, uint32_t* out) {
    hipLaunchKernelGGL(k_slab_bbox, dim3(1), dim3(64), 0, s, pb, out);
}
void launch_slab_import(hipStream_t s, const PhotonBufs& pb, const float* recv, uint32_t n) {
    const uint32_t groups = (n + pb.D - 1) / pb.D;
    uint32_t blocks = (groups + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
    hipLaunchKernelGGL(k_slab_import, dim3(blocks), dim3(256), 0, s, pb, recv, n);
}

/* ------------------------------------------------------------------ */
/* stochastic-hash photon map (ACCELERATION_STRUCTURE_STOCHASTIC_HASH)  */
/* ------------------------------------------------------------------ */
/* STORE_PHOTON of the hash configuration (helpers/store_photon.h:19-25):
 * every deposit lands in table entry getHashValue(cell) and bumps its
 * count.  The reference lets the racing stores pick the entry's photon; here
 * the entry keeps the deposit with the highest slot index (atomicMax), so the
 * table is reproducible and equals the oracle's.  Deposits come from the
 * slots the photon pass wrote (vmask), positions from the compact plane. */
__global__ __launch_bounds__(256) void k_hash_build(PhotonBufs pb, HashParams hp) {
    const uint32_t np = pb.prows * pb.PW;
    const float inv = 1.f / hp.cell;
    uint32_t deposits = 0;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < np; p += gridDim.x * blockDim.x) {
        uint32_t m = pb.vmask[p];
        deposits += (uint32_t)__builtin_popcount(m);
        while (m) {
            const uint32_t k = (uint32_t)__builtin_ctz(m);
            m &= m - 1;
            const uint32_t si = p * pb.D + k;
            const float4 a = pb.pos4[si];
            /* getPhotonGridIndex (PhotonGrid.h:19-23) */
            const f3 pp = (mk(a.x, a.y, a.z) - mk(hp.ox, hp.oy, hp.oz)) * inv;
            const uint32_t cx = orx_f2u_sat(orx_floorf(pp.x)), cy = orx_f2u_sat(orx_floorf(pp.y)),
                           cz = orx_f2u_sat(orx_floorf(pp.z));
            const uint32_t h = (cx + cy * hp.gx + cz * hp.gx * hp.gy) & hp.mask;
            atomicAdd(&pb.hcount[h], 1u);
            atomicMax(&pb.hwin[h], si + 1u);
        }
    }
    const uint64_t t = wave_sum_u64(deposits);
    if ((threadIdx.x & 63) == 0 && t) {
        atomicAdd(&pb.grid->valid, (uint32_t)t);
        atomicAdd((unsigned long long*)&pb.grid->valid_total, (unsigned long long)t);
    }
}
/* the grid record the stats and exports read: the hash grid, the table size as
 * the cell count, zeroed per-iteration counters (k_hash_build adds the deposits) */
__global__ void k_hash_setup(PhotonBufs pb, HashParams hp) {
    GridParams* g = pb.grid;
    g->ox = hp.ox;
    g->oy = hp.oy;
    g->oz = hp.oz;
    g->cell = hp.cell;
    g->gx = hp.gx;
    g->gy = hp.gy;
    g->gz = hp.gz;
    g->G = pb.hnum;
    g->valid = 0;
    g->error = 0;
    g->any_valid = 1;
    g->photons_visited = 0;
    g->cells_visited = 0;
}
void launch_hash_build(hipStream_t s, const PhotonBufs& pb, const HashParams& hp) {
    hipMemsetAsync(pb.hcount, 0, (size_t)pb.hnum * 4, s); /* UniformGridPhotonInitialize.cu:20-23 */
    hipMemsetAsync(pb.hwin, 0, (size_t)pb.hnum * 4, s);
    hipLaunchKernelGGL(k_hash_setup, dim3(1), dim3(1), 0, s, pb, hp);
    const uint32_t np = pb.prows * pb.PW;
    unsigned blocks = (np + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks) hipLaunchKernelGGL(k_hash_build, dim3(blocks), dim3(256), 0, s, pb, hp);
}

/* IndirectRadianceEstimation.cu:131-162: the 27 cells around the hit point's
 * cell, one photon per cell weighted by the cell's count; the visit counters
 * count 27 cells and 27 photons (:150-151).  Cells in a fixed order and
 * unfused arithmetic, so the sum is the oracle's bit for bit. */
__global__ __launch_bounds__(64) void k_ppm_gather_hash(GatherIn gi, PhotonBufs pb, HashParams hp, Consts c) {
    const uint32_t x = blockIdx.x * 8 + (threadIdx.x & 7);
    const uint32_t y = blockIdx.y * 8 + (threadIdx.x >> 3);
    const uint32_t j = gather_row(gi, y);
    const bool inimg = x < gi.W && y < gi.segments * gi.seg_rows;
    const size_t i = (size_t)j * gi.W + x;
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    float2 Cc = make_float2(0.f, 0.f);
    if (inimg) {
        hp_load(gi, j, x, A, B, Cc);
    }
    const uint32_t flags = __float_as_uint(A.w);
    f3 acc = mk1(0.0f);
    uint32_t dC = 0, dP = 0;
    if (inimg && (flags & PRD_HIT_NON_SPECULAR)) {
        const f3 pos = mk(A.x, A.y, A.z), nrm = mk(B.x, B.y, B.z);
        const float radius2 = c.ppm_radius2;
        const f3 pp = (pos - mk(hp.ox, hp.oy, hp.oz)) * (1.f / hp.cell);
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
                    const uint32_t h = (cx + cy * hp.gx + cz * hp.gx * hp.gy) & hp.mask;
                    const uint32_t n = pb.hcount[h];
                    if (!n) continue; /* an empty entry contributes power * 0 */
                    const float4* rec = pb.slots + 4 * (size_t)(pb.hwin[h] - 1u);
                    const float4 a = rec[0], b = rec[1];
                    const float pz = rec[2].x;
                    const f3 diff = pos - mk(a.x, a.y, a.z);
                    const float distance2 = dot(diff, diff);
                    if (distance2 <= radius2 && dot(-mk(b.x, b.y, b.z), nrm) >= 0) {
                        const float e = orx_expf_unit((-beta * distance2) * inv2r2);
                        const float wgt = alpha * (1 - (1 - e) * invDen);
                        acc = acc + (mk(a.w, b.w, pz) * wgt) * (float)n;
                    }
                }
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
            gi.dbg[2 * i] = dC;
            gi.dbg[2 * i + 1] = dP;
        }
    }
    const uint64_t sp = wave_sum_u64(dP), sc = wave_sum_u64(dC);
    if ((threadIdx.x & 63) == 0 && sp) {
        atomicAdd((unsigned long long*)&pb.grid->photons_visited, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->cells_visited, (unsigned long long)sc);
        atomicAdd((unsigned long long*)&pb.grid->photons_visited_total, (unsigned long long)sp);
        atomicAdd((unsigned long long*)&pb.grid->cells_visited_total, (unsigned long long)sc);
    }
}
void launch_ppm_gather_hash(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const HashParams& hp,
                            const Consts& c) {
    const uint32_t rows = gi.segments * gi.seg_rows;
    dim3 grid((gi.W + 7) / 8, (rows + 7) / 8);
    hipLaunchKernelGGL(k_ppm_gather_hash, grid, dim3(64), 0, s, gi, pb, hp, c);
}

/* ------------------------------------------------------------------ */
/* direct radiance (4 shadow samples) + output accumulation            */
/* ------------------------------------------------------------------ */
/* MODE 0: direct + output fused; 1: direct only (overlapping the grid build
 * and gather on a second stream); 2: output only (out = [out +] direct + indirect) */
template <int MODE>
__global__ __launch_bounds__(64) void k_ppm_direct_output(DevScene S, PixelBufs px, Consts c) {
    ORX_STACK_DECL;
    uint32_t x, j;
    pix_tile(px, x, j);
    if (x >= px.W || j >= px.rows) return;
    const size_t i = (size_t)j * px.W + x;
    if (MODE == 2) {
        const f3 d = mk(px.direct[3 * i], px.direct[3 * i + 1], px.direct[3 * i + 2]);
        const f3 ind = mk(px.indirect[3 * i], px.indirect[3 * i + 1], px.indirect[3 * i + 2]);
        const f3 fin = d + ind;
        f3 out = fin;
        if (c.local_iteration != 0) out = mk(px.output[3 * i], px.output[3 * i + 1], px.output[3 * i + 2]) + fin;
        px.output[3 * i + 0] = out.x;
        px.output[3 * i + 1] = out.y;
        px.output[3 * i + 2] = out.z;
        return;
    }
    const float4 A = px.hpA[i];
    const float4 B = px.hpB[i];
    const float2 Cc = px.hpC[i];
    const uint32_t flags = __float_as_uint(A.w);
    f3 direct;
    if (!(flags & PRD_HIT_NON_SPECULAR)) {
        f3 rad = mk(B.x, B.y, B.z);
        if ((flags & PRD_HIT_EMITTER) && !(flags & PRD_HIT_SPECULAR))
            direct = mk(fminf(rad.x, 1.f), fminf(rad.y, 1.f), fminf(rad.z, 1.f));
        else
            direct = rad;
    } else if (c.media) { /* numShadowSamples = ENABLE_PARTICIPATING_MEDIA ? 0 : 4 (DirectRadianceEstimation.cu:54) */
        direct = mk1(0.f);
    } else {
        const size_t slot = (size_t)j * px.RW + x;
        Rng rs = rng_load(px.rng, slot);
        const int numLights = (int)S.nl;
        const f3 pos = mk(A.x, A.y, A.z), nrm = mk(B.x, B.y, B.z);
        f3 avg = mk1(0.f);
        for (int s = 0; s < 4; s++) {
            float sample = rnd(rs);
            int li = (int)(sample * (float)numLights);
            int randomLightIndex = li < numLights - 1 ? li : numLights - 1;
            float scale = (float)numLights;
            f3 lc = light_contribution(S, S.lights[randomLightIndex], pos, nrm, rs, ORX_STACK_PTR);
            avg = avg + lc * scale;
        }
        direct = (mk(B.w, Cc.x, Cc.y) * avg) / (float)4;
        rng_store(px.rng, slot, rs);
    }
    px.direct[3 * i + 0] = direct.x;
    px.direct[3 * i + 1] = direct.y;
    px.direct[3 * i + 2] = direct.z;
    if (MODE == 1) return;
    f3 ind = mk(px.indirect[3 * i], px.indirect[3 * i + 1], px.indirect[3 * i + 2]);
    f3 fin = direct + ind;
    f3 out = fin;
    if (c.local_iteration != 0) out = mk(px.output[3 * i], px.output[3 * i + 1], px.output[3 * i + 2]) + fin;
    px.output[3 * i + 0] = out.x;
    px.output[3 * i + 1] = out.y;
    px.output[3 * i + 2] = out.z;
}
void launch_ppm_direct_output(hipStream_t s, const DevScene& S, const PixelBufs& px, const Consts& c, int mode) {
    const dim3 grid = pix_grid(px);
    if (mode == 1) hipLaunchKernelGGL(k_ppm_direct_output<1>, grid, dim3(64), ORX_STACK_BYTES(S), s, S, px, c);
    else if (mode == 2) hipLaunchKernelGGL(k_ppm_direct_output<2>, grid, dim3(64), 0, s, S, px, c);
    else hipLaunchKernelGGL(k_ppm_direct_output<0>, grid, dim3(64), ORX_STACK_BYTES(S), s, S, px, c);
}

/* ------------------------------------------------------------------ */
/* path tracing                                                        */
/* ------------------------------------------------------------------ */
__global__ __launch_bounds__(64) void k_pt(DevScene S, DevCamera cam, PixelBufs px, Consts c) {
    ORX_STACK_DECL;
    uint32_t x, j;
    pix_tile(px, x, j);
    if (x >= px.W || j >= px.rows) return;
    const uint32_t y = px.rank + px.world * j;
    const size_t i = (size_t)j * px.W + x;
    const size_t slot = (size_t)j * px.RW + x;
    /* the PRD copy and the global slot start from the same state and are
     * advanced independently (RayGeneratorPT.cu:52, :89, :111, :130) */
    Rng G = rng_load(px.rng, slot);
    Rng rs = G;
    const int numLights = (int)S.nl;
    RadiancePRD prd;
    prd.attenuation = mk1(1.0f);
    prd.radiance = mk1(0.f);
    prd.depth = 0;
    prd.flags = 0;
    prd.position = mk1(0.f);
    prd.normal = mk1(0.f);
    prd.newdir = mk1(0.f);
    f3 o, d;
    primary_ray(cam, x, y, px.W, px.H, rs, o, d);
    f3 fin = mk1(0);
    for (int it = 0; it < 5; it++) {
        prd.flags = PRD_PATH_TRACING;
        trace_radiance(S, c.max_radiance_depth, o, d, 0.001f, prd, rs, ORX_STACK_PTR);
        if (prd.flags & PRD_HIT_EMITTER) {
            if ((prd.flags & PRD_HIT_SPECULAR) || it == 0) fin = prd.radiance;
            break;
        } else if (prd.flags & PRD_HIT_NON_SPECULAR) {
            f3 accum = mk1(0);
            int li = (int)(rnd(G) * (float)numLights);
            float scale = (float)numLights;
            f3 lc = light_contribution(S, S.lights[li], prd.position, prd.normal, rs, ORX_STACK_PTR) * scale;
            accum = accum + lc;
            f3 direct = (prd.attenuation * accum) / (float)1;
            fin = fin + direct;
            o = prd.position;
            d = prd.newdir;
        } else {
            break;
        }
        if (it >= 3) {
            float sample = rnd(G);
            float p = fmax3(prd.attenuation);
            if (sample > p) break;
            prd.attenuation = prd.attenuation / p;
        }
    }
    if (!isnan3(fin)) {
        f3 out = fin;
        if (c.local_iteration != 0) out = mk(px.output[3 * i], px.output[3 * i + 1], px.output[3 * i + 2]) + fin;
        px.output[3 * i + 0] = out.x;
        px.output[3 * i + 1] = out.y;
        px.output[3 * i + 2] = out.z;
    }
    rng_store(px.rng, slot, rs);
}
void launch_pt(hipStream_t s, const DevScene& S, const DevCamera& cam, const PixelBufs& px, const Consts& c) {
    const dim3 grid = pix_grid(px);
    hipLaunchKernelGGL(k_pt, grid, dim3(64), ORX_STACK_BYTES(S), s, S, cam, px, c);
}

}  // namespace orx
