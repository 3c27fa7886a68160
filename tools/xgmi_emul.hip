// Stand-in for an RCCL collective's local footprint on one GPU (tools/shard_model.py --interfere; design
// tool, not product).  A ring all-gather / reduce-scatter kernel of RCCL holds a few dozen workgroups for as
// long as the transfer takes over xGMI and moves the received bytes through HBM: the all-gather writes what
// it receives and reads what it forwards (a copy), the reduce-scatter reads the received chunk and the local
// one and writes the sum (an add).  This kernel does the same work with the same footprint: `blocks`
// workgroups copy (add = 0) or accumulate (add = 1) n float4s, paced by the wall clock so the whole transfer
// takes `ns` nanoseconds (the link time), i.e. the workgroups stay resident for the collective's duration.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_xgmi_emul(const float4* __restrict__ src, float4* __restrict__ dst, size_t n,
                                                   uint64_t ticks, int add) {
    const uint64_t t0 = wall_clock64();
    constexpr uint32_t CHUNKS = 64; /* pacing steps per block */
    const size_t per_block = (n + gridDim.x - 1) / gridDim.x;
    const size_t b0 = (size_t)blockIdx.x * per_block, b1 = b0 + per_block < n ? b0 + per_block : n;
    const size_t per_chunk = (per_block + CHUNKS - 1) / CHUNKS;
    for (uint32_t c = 0; c < CHUNKS; c++) {
        const size_t c0 = b0 + c * per_chunk, c1 = c0 + per_chunk < b1 ? c0 + per_chunk : b1;
        for (size_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            float4 v = src[i];
            if (add) {
                const float4 w = dst[i];
                v.x += w.x, v.y += w.y, v.z += w.z, v.w += w.w;
            }
            dst[i] = v;
        }
        /* the link delivers chunk c by t0 + (c + 1) * ticks / CHUNKS: wait for it (bounded by the clock) */
        const uint64_t due = t0 + (uint64_t)(c + 1) * ticks / CHUNKS;
        while (wall_clock64() < due) __builtin_amdgcn_s_sleep(8);
    }
}

extern "C" int xgmi_emul(const void* src, void* dst, size_t bytes, double ns, int add, int blocks, void* stream) {
    static uint64_t khz = 0;
    if (!khz) {
        int dev = 0, rate = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
            rate = 0;
        khz = rate > 0 ? (uint64_t)rate : 100000;
    }
    const uint64_t ticks = (uint64_t)(ns * 1e-6 * (double)khz);
    hipLaunchKernelGGL(k_xgmi_emul, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)src, (float4*)dst,
                       bytes / 16, ticks, add);
    return (int)hipGetLastError();
}
