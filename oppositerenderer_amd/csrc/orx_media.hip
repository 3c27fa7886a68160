/* Participating medium: the volumetric photon table of a photon pass and its grid.
 *
 * ParticipatingMedium.cu:170-177 stores each scatter event of photon p at slot
 * pm_index % NUM_VOLUMETRIC_PHOTONS (pm_index = p * maxPhotonDepositsPerEmitted, so every event of
 * a path lands in one slot) and bumps the slot's numDeposits; its racing stores leave an
 * arbitrary event's power and position in a slot.  Here the photon pass keeps each photon's
 * last event and its event count (k_ppm_photon<true>), and the table takes, per slot, the sum of
 * the counts and the last event of the highest photon index (the oracle's vol_resolve).  The
 * valid slots (numDeposits > 0, power > 0: VolumetricPhotonSphere.cu:61-85's non-empty boxes) are
 * then sorted by grid cell (hipcub radix sort of (cell, slot): cell order, slot order inside a
 * cell, deterministic) into records the eye pass's DDA walks (vol_gather, orx_device.h).
 */
#include <hipcub/hipcub.hpp>

#include "orx_kernels.h"

namespace orx {

__global__ __launch_bounds__(256) void k_vol_clear(VolBuild vb) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= vb.NV) return;
    vb.vcnt[s] = 0;
    vb.vwin[s] = 0;
}
__global__ __launch_bounds__(256) void k_vol_resolve(VolBuild vb) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= vb.nphot) return;
    const uint32_t n = __float_as_uint(vb.ev_a[p].w);
    if (!n) return;
    const uint32_t slot = (p * vb.D) % vb.NV;
    atomicAdd(&vb.vcnt[slot], n);
    atomicMax(&vb.vwin[slot], p + 1u);
}
__global__ __launch_bounds__(256) void k_vol_fill(VolBuild vb) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= vb.nphot) return;
    const float4 a = vb.ev_a[p];
    if (!__float_as_uint(a.w)) return;
    const uint32_t slot = (p * vb.D) % vb.NV;
    if (vb.vwin[slot] != p + 1u) return;
    vb.vA[slot] = make_float4(a.x, a.y, a.z, 0.f);
    vb.vB[slot] = vb.ev_b[p];
}
__global__ __launch_bounds__(256) void k_vol_keys(VolBuild vb, VolMap vm) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= vb.NV) return;
    uint32_t key = vm.G + 1u;
    if (vb.vcnt[s]) {
        const float4 b = vb.vB[s];
        if (fmax3(mk(b.x, b.y, b.z)) > 0) {
            const float4 a = vb.vA[s];
            const float inv = 1.f / vm.cell;
            const int cx = (int)orx_floorf((a.x - vm.glo.x) * inv), cy = (int)orx_floorf((a.y - vm.glo.y) * inv),
                      cz = (int)orx_floorf((a.z - vm.glo.z) * inv);
            const bool in = cx >= 0 && cy >= 0 && cz >= 0 && cx < (int)vm.n[0] && cy < (int)vm.n[1] &&
                            cz < (int)vm.n[2] && a.x == a.x && a.y == a.y && a.z == a.z;
            key = in ? (uint32_t)cx + vm.n[0] * ((uint32_t)cy + vm.n[1] * (uint32_t)cz) : vm.G;
        }
    }
    vb.keys[s] = key;
    vb.vals[s] = s;
}
/* start[c] = first sorted record of cell c (lower bound), c in [0, G + 1] */
__global__ __launch_bounds__(256) void k_vol_starts(VolBuild vb, uint32_t G) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c > G + 1u) return;
    uint32_t lo = 0, hi = vb.NV;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (vb.keys_sorted[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    vb.start[c] = lo;
}
__global__ __launch_bounds__(256) void k_vol_records(VolBuild vb, uint32_t G) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= vb.start[G + 1u]) return;
    const uint32_t s = vb.vals_sorted[i];
    const float4 a = vb.vA[s], b = vb.vB[s];
    const f3 pw = mk(b.x, b.y, b.z) * (float)vb.vcnt[s]; /* photon.power*photon.numDeposits */
    vb.rec[2 * i] = make_float4(a.x, a.y, a.z, pw.x);
    vb.rec[2 * i + 1] = make_float4(pw.y, pw.z, 0.f, 0.f);
}

size_t vol_sort_tmp_bytes(uint32_t NV) {
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)NV);
    return bytes;
}

void launch_vol_build(hipStream_t s, const VolBuild& vb, const VolMap& vm) {
    const uint32_t bNV = (vb.NV + 255) / 256, bP = (vb.nphot + 255) / 256;
    hipLaunchKernelGGL(k_vol_clear, dim3(bNV), dim3(256), 0, s, vb);
    if (bP) {
        hipLaunchKernelGGL(k_vol_resolve, dim3(bP), dim3(256), 0, s, vb);
        hipLaunchKernelGGL(k_vol_fill, dim3(bP), dim3(256), 0, s, vb);
    }
    hipLaunchKernelGGL(k_vol_keys, dim3(bNV), dim3(256), 0, s, vb, vm);
    int end_bit = 1;
    while (end_bit < 32 && ((uint64_t)vm.G + 1u) >> end_bit) end_bit++;
    size_t bytes = vb.sort_tmp_bytes;
    hipcub::DeviceRadixSort::SortPairs(vb.sort_tmp, bytes, (const uint32_t*)vb.keys, vb.keys_sorted,
                                       (const uint32_t*)vb.vals, vb.vals_sorted, (int)vb.NV, 0, end_bit, s);
    hipLaunchKernelGGL(k_vol_starts, dim3((vm.G + 2u + 255) / 256), dim3(256), 0, s, vb, vm.G);
    hipLaunchKernelGGL(k_vol_records, dim3(bNV), dim3(256), 0, s, vb, vm.G);
}

__global__ __launch_bounds__(256) void k_vol_indirect(PixelBufs px, const float* volR, float emitted_f) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)px.rows * px.W) return;
    const f3 v = mk(volR[3 * i], volR[3 * i + 1], volR[3 * i + 2]) / emitted_f;
    px.indirect[3 * i + 0] = px.indirect[3 * i + 0] + v.x;
    px.indirect[3 * i + 1] = px.indirect[3 * i + 1] + v.y;
    px.indirect[3 * i + 2] = px.indirect[3 * i + 2] + v.z;
}
void launch_vol_indirect(hipStream_t s, const PixelBufs& px, const float* volR, float emitted_f) {
    const size_t n = (size_t)px.rows * px.W;
    if (!n) return;
    hipLaunchKernelGGL(k_vol_indirect, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, px, volR, emitted_f);
}

}  // namespace orx
