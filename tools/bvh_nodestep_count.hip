// Design tool (not product): the VALU cost of one 8-wide quantised node step (any-hit, all hits pushed) against
// the shipped 4-wide one, compiled for gfx950 and counted in the ISA (tools/bvh_nodestep_count.sh); with the
// per-ray node counts of tools/bvh_sim.cpp this prices a BVH8 before building one.
#include <hip/hip_runtime.h>
#include "orx_device.h"
using namespace orx;
struct DevBvh8 {
    float ox, oy, oz; uint32_t ebits;
    uint32_t qlo_x[2], qhi_x[2], qlo_y[2], qhi_y[2], qlo_z[2], qhi_z[2];
    uint32_t child[8];
};
__device__ __forceinline__ void node8(const DevBvh8* nodes, uint32_t idx, const RayBox& rb, float tmin, float tmax,
                                      uint32_t& hits, uint32_t c[8]) {
    const __amdgpu_buffer_rsrc_t r = orx_rsrc(nodes);
    const uint32_t bo = idx * 96u;
    const float4 A = ld16(r, bo), B = ld16(r, bo + 16), C = ld16(r, bo + 32), D = ld16(r, bo + 48);
    const float4 E = ld16(r, bo + 64), F = ld16(r, bo + 80);
    const uint32_t eb = __float_as_uint(A.w);
    const float sx = __uint_as_float((eb & 0xffu) << 23), sy = __uint_as_float(((eb >> 8) & 0xffu) << 23),
                sz = __uint_as_float(((eb >> 16) & 0xffu) << 23);
    const float ax = (A.x - rb.o.x) * rb.inv.x, bx = sx * rb.inv.x;
    const float ay = (A.y - rb.o.y) * rb.inv.y, by = sy * rb.inv.y;
    const float az = (A.z - rb.o.z) * rb.inv.z, bz = sz * rb.inv.z;
    uint32_t w[12] = {__float_as_uint(B.x), __float_as_uint(B.y), __float_as_uint(B.z), __float_as_uint(B.w),
                      __float_as_uint(C.x), __float_as_uint(C.y), __float_as_uint(C.z), __float_as_uint(C.w),
                      __float_as_uint(D.x), __float_as_uint(D.y), __float_as_uint(D.z), __float_as_uint(D.w)};
    const uint32_t nx0 = rb.nx ? w[2] : w[0], nx1 = rb.nx ? w[3] : w[1], fx0 = rb.nx ? w[0] : w[2], fx1 = rb.nx ? w[1] : w[3];
    const uint32_t ny0 = rb.ny ? w[6] : w[4], ny1 = rb.ny ? w[7] : w[5], fy0 = rb.ny ? w[4] : w[6], fy1 = rb.ny ? w[5] : w[7];
    const uint32_t nz0 = rb.nz ? w[10] : w[8], nz1 = rb.nz ? w[11] : w[9], fz0 = rb.nz ? w[8] : w[10], fz1 = rb.nz ? w[9] : w[11];
    c[0] = __float_as_uint(E.x); c[1] = __float_as_uint(E.y); c[2] = __float_as_uint(E.z); c[3] = __float_as_uint(E.w);
    c[4] = __float_as_uint(F.x); c[5] = __float_as_uint(F.y); c[6] = __float_as_uint(F.z); c[7] = __float_as_uint(F.w);
    typedef float v2q __attribute__((ext_vector_type(2)));
    auto q2 = [](uint32_t wd, int i) { return v2q{(float)((wd >> (8 * i)) & 0xffu), (float)((wd >> (8 * i + 8)) & 0xffu)}; };
    const v2q ax2 = v2q{ax, ax}, bx2 = v2q{bx, bx}, ay2 = v2q{ay, ay}, by2 = v2q{by, by}, az2 = v2q{az, az}, bz2 = v2q{bz, bz};
    uint32_t h = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const uint32_t NX = g < 2 ? nx0 : nx1, FX = g < 2 ? fx0 : fx1, NY = g < 2 ? ny0 : ny1, FY = g < 2 ? fy0 : fy1;
        const uint32_t NZ = g < 2 ? nz0 : nz1, FZ = g < 2 ? fz0 : fz1;
        const int sh = 2 * (g & 1);
        const v2q tnx = __builtin_elementwise_fma(q2(NX, sh), bx2, ax2), tfx = __builtin_elementwise_fma(q2(FX, sh), bx2, ax2);
        const v2q tny = __builtin_elementwise_fma(q2(NY, sh), by2, ay2), tfy = __builtin_elementwise_fma(q2(FY, sh), by2, ay2);
        const v2q tnz = __builtin_elementwise_fma(q2(NZ, sh), bz2, az2), tfz = __builtin_elementwise_fma(q2(FZ, sh), bz2, az2);
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const float t0 = fmaxf(fmaxf(fmaxf(tnx[e], tny[e]), tnz[e]), tmin);
            const float t1 = fminf(fminf(fminf(tfx[e], tfy[e]), tfz[e]), tmax);
            h |= (t0 <= t1 ? 1u : 0u) << (2 * g + e);
        }
    }
    hits = h;
}
__global__ void k8(const DevBvh8* nodes, const float* rays, uint32_t* out, uint32_t* stkbuf) {
    ORX_STACK_DECL;
    const StackL stk{ORX_STACK_PTR};
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const f3 o = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), d = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    const RayBox rb = ray_box(o, d);
    int sp = 0;
    uint32_t ref = 0, cnt = 0;
    while (ref != ORX_DONE && !(ref & ORX_LEAF)) {
        uint32_t h, c[8];
        node8(nodes, ref, rb, 0.f, 1e30f, h, c);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            stk.put(sp, c[k]);
            sp += (h >> k) & 1;
        }
        ref = sp ? stk.pop(sp) : ORX_DONE;
        cnt++;
    }
    out[i] = cnt + ref;
}
__global__ void k4(const DevBvh4* nodes, const float* rays, uint32_t* out, uint32_t* stkbuf) {
    ORX_STACK_DECL;
    const StackL stk{ORX_STACK_PTR};
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const f3 o = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), d = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    const RayBox rb = ray_box(o, d);
    int sp = 0;
    uint32_t ref = 0, cnt = 0;
    while (ref != ORX_DONE && !(ref & ORX_LEAF)) {
        float ct[4];
        uint32_t cc[4];
        node_test(nodes, ref, rb, 0.f, 1e30f, ct, cc);
        const int h0 = ct[0] != INFINITY, h1 = ct[1] != INFINITY, h2 = ct[2] != INFINITY, h3 = ct[3] != INFINITY;
        stk.put(sp, cc[0]); sp += h0;
        stk.put(sp, cc[1]); sp += h1;
        stk.put(sp, cc[2]); sp += h2;
        stk.put(sp, cc[3]); sp += h3;
        ref = sp ? stk.pop(sp) : ORX_DONE;
        cnt++;
    }
    out[i] = cnt + ref;
}
