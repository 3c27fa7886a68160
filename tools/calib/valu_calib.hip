// VALU issue-cost calibration for gfx950 (tools/calib): what one wave64 instruction of each
// kind occupies a SIMD-32 for, and how the SQ counters count it.  Four kernels, each a
// dependency-free stream of one instruction kind (8 independent chains per lane, 8 waves per
// SIMD so issue, not latency, bounds them):
//   fma    v_fma_f32          pk_fma  v_pk_fma_f32
//   mul    v_mul_f32          pk_mul  v_pk_mul_f32
// Each launch runs ITERS x 8 instructions per lane.  The host prints the wall time of each
// launch (hipEvents); under rocprofv3 --pmc the SQ counters give instructions, FLOPs and
// SQ_ACTIVE_INST_VALU per kernel, and GRBM_GUI_ACTIVE the cycles.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int ITERS = 2048;

__global__ __launch_bounds__(256) void k_cal_fma(float* out, float a, float b) {
    float x[8];
    for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 0.001f + k;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = __builtin_fmaf(x[k], a, b);
    float s = 0.f;
    for (int k = 0; k < 8; k++) s += x[k];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cal_pk_fma(float* out, float a, float b) {
    v2f x[8];
    for (int k = 0; k < 8; k++) x[k] = v2f{threadIdx.x * 0.001f + k, threadIdx.x * 0.002f - k};
    const v2f A = v2f{a, a}, B = v2f{b, b};
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = __builtin_elementwise_fma(x[k], A, B);
    float s = 0.f;
    for (int k = 0; k < 8; k++) s += x[k].x + x[k].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cal_mul(float* out, float a, float b) {
    float x[8];
    for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 0.001f + k;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = x[k] * a;
    float s = 0.f;
    for (int k = 0; k < 8; k++) s += x[k];
    if (s == 12345.f + b) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cal_pk_mul(float* out, float a, float b) {
    v2f x[8];
    for (int k = 0; k < 8; k++) x[k] = v2f{threadIdx.x * 0.001f + k, threadIdx.x * 0.002f - k};
    const v2f A = v2f{a, b};
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = x[k] * A;
    float s = 0.f;
    for (int k = 0; k < 8; k++) s += x[k].x + x[k].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    float* out;
    hipMalloc(&out, 4096);
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K { const char* name; void (*f)(float*, float, float); } ks[] = {
        {"k_cal_fma", k_cal_fma}, {"k_cal_pk_fma", k_cal_pk_fma}, {"k_cal_mul", k_cal_mul}, {"k_cal_pk_mul", k_cal_pk_mul}};
    for (int rep = 0; rep < 3; rep++)
        for (auto& k : ks) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double winst = (double)blocks * 4 * ITERS * 8; /* wave-instructions */
            if (rep == 2)
                printf("%-14s %.3f ms  %.3e wave-instructions  %.2f ns per wave-instruction per SIMD\n", k.name, ms,
                       winst, ms * 1e6 / (winst / 1024.0));
        }
    hipFree(out);
    return 0;
}
