// Microbenchmark: issue cost of v_fma_f32 vs v_pk_fma_f32 (and a few other
// VALU ops used by the march/traversal loops) at 8 waves/SIMD on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int N = 4096;

__global__ __launch_bounds__(256) void k_scalar(float *o, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x + i;
    for (int n = 0; n < N; n++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_fmaf(x[i], a, b);
    float s = 0; for (int i = 0; i < 8; i++) s += x[i];
    o[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_packed(float *o, float a, float b) {
    f2 x[4];
    const f2 av = {a, a}, bv = {b, b};
    for (int i = 0; i < 4; i++) x[i] = (f2){(float)threadIdx.x + i, (float)i};
    for (int n = 0; n < N; n++)
#pragma unroll
        for (int i = 0; i < 4; i++) x[i] = __builtin_elementwise_fma(x[i], av, bv);
    float s = 0; for (int i = 0; i < 4; i++) s += x[i].x + x[i].y;
    o[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_floor(float *o, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x + i;
    for (int n = 0; n < N; n++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = floorf(x[i]) + a;   // v_floor + v_add
    float s = 0; for (int i = 0; i < 8; i++) s += x[i];
    o[blockIdx.x * 256 + threadIdx.x] = s + b;
}
__global__ __launch_bounds__(256) void k_cvt(float *o, float a, float b) {
    int x[8];
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x + i;
    for (int n = 0; n < N; n++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = (int)((float)x[i] * a);   // v_cvt_f32_i32, v_mul, v_cvt_i32_f32
    float s = 0; for (int i = 0; i < 8; i++) s += x[i];
    o[blockIdx.x * 256 + threadIdx.x] = s + b;
}

int main() {
    float *o;
    hipMalloc(&o, 256 * 8192 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8 * 4;   // 8 blocks/CU x 256 CUs, x4 rounds
    auto run = [&](const char *name, void (*k)(float *, float, float), double ops_per_iter) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o, 1.0001f, 0.5f);
        hipEventRecord(e0);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o, 1.0001f, 0.5f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double waves = blocks * 4.0, instr = waves * N * ops_per_iter;
        // SIMD-cycles per wave-instruction at 2.4 GHz nominal
        const double cyc = ms * 1e-3 * 2.4e9 * 1024.0 / instr;
        printf("%-8s %.3f ms  %.2f SIMD-cycles per wave-instruction (@2.4GHz)\n", name, ms, cyc);
    };
    run("fma", k_scalar, 8);
    run("pk_fma", k_packed, 4);
    run("floor", k_floor, 16);
    run("cvt", k_cvt, 24);
    return 0;
}
