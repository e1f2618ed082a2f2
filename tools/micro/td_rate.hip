// Data-path (TA/TD) issue cost of the load forms the shading uses on gfx950:
// CU cycles per wave64 load instruction, loads independent of each other
// (throughput, not latency), every lane on its own 4-byte-aligned address in
// 64 contiguous dwords (one or four 128-B lines per wave load), L1-resident.
//   dword    buffer_load_dword                        (4 B per lane, raw)
//   dwordx4  buffer_load_dwordx4                      (16 B per lane, raw)
//   fmt_x    buffer_load_format_x, 8-bit UNORM        (1 texel -> 1 float)
//   fmt_xy   buffer_load_format_xy, 8_8 UNORM         (2 -> 2 floats)
//   fmt_xyzw buffer_load_format_xyzw, 8_8_8_8 UNORM   (4 -> 4 floats: AO pair, noise quad)
// 8 waves per SIMD, 8 loads in flight per wave.  The render kernel's TD busy
// (0.82 of its cycles at C3) is set against these per-form costs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITERS = 2048;
constexpr int BATCH = 8;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ float ld_f1(u32x4 r, unsigned v, int s, int a) __asm("llvm.amdgcn.raw.buffer.load.format.f32");
__device__ f32x2 ld_f2(u32x4 r, unsigned v, int s, int a) __asm("llvm.amdgcn.raw.buffer.load.format.v2f32");
__device__ f32x4 ld_f4(u32x4 r, unsigned v, int s, int a) __asm("llvm.amdgcn.raw.buffer.load.format.v4f32");
__device__ unsigned ld_u1(u32x4 r, unsigned v, int s, int a) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ u32x4 ld_u4(u32x4 r, unsigned v, int s, int a) __asm("llvm.amdgcn.raw.buffer.load.v4i32");

__device__ __forceinline__ u32x4 rsrc(const void *base, unsigned w3) {
    const unsigned long long p = (unsigned long long)base;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((unsigned)p);
    r.y = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32) & 0xffffu);
    r.z = 0xffffffffu;
    r.w = w3;
    return r;
}

template <int KIND>
__global__ __launch_bounds__(256) void k_td(const uint32_t *buf, float *out) {
    const unsigned lane = threadIdx.x & 63;
    const unsigned gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    // 4 KiB per wave slot, 32 slots: 128 KiB, L1/L2-resident
    const unsigned base = (gw & 31) * 4096u;
    // word 3: DST_SEL [0:11], NUM_FORMAT [12:14] (0 UNORM), DATA_FORMAT [15:18] (1: 8, 3: 8_8, 10: 8_8_8_8)
    const unsigned w3 = KIND == 2 ? 0x00008004u : KIND == 3 ? 0x0001802Cu : KIND == 4 ? 0x00050FACu : 0x00020000u;
    const u32x4 r = rsrc(buf, w3);
    float acc = 0.0f;
    unsigned uacc = 0;
    const unsigned step = KIND == 1 ? 16u : 4u;
    for (int it = 0; it < ITERS; it += BATCH) {
#pragma unroll
        for (int b = 0; b < BATCH; b++) {
            const unsigned off = base + ((lane * step + (unsigned)(b * 256 + it * 4)) & 4095u);
            if (KIND == 0) uacc += ld_u1(r, off, 0, 0);
            else if (KIND == 1) { const u32x4 v = ld_u4(r, off, 0, 0); uacc += v.x + v.y + v.z + v.w; }
            else if (KIND == 2) acc += ld_f1(r, off, 0, 0);
            else if (KIND == 3) { const f32x2 v = ld_f2(r, off, 0, 0); acc += v.x + v.y; }
            else { const f32x4 v = ld_f4(r, off, 0, 0); acc += (v.x + v.y) + (v.z + v.w); }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc + (float)uacc;
}

template <int KIND>
static double run(const uint32_t *buf, float *out, int cus) {
    const int blocks = cus * 8;                   // 8 blocks of 4 waves per CU = 8 waves per SIMD
    hipLaunchKernelGGL(k_td<KIND>, dim3(blocks), dim3(256), 0, 0, buf, out);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL(k_td<KIND>, dim3(blocks), dim3(256), 0, 0, buf, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    const double loads_per_cu = (double)8 * 4 * ITERS;    // waves per CU x loads per wave
    return (ms / reps) * 1e-3 * 2.4e9 / loads_per_cu;     // CU cycles per wave load at 2.4 GHz
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    uint32_t *buf;
    float *out;
    hipMalloc(&buf, 32 * 4096 + 4096);
    hipMemset(buf, 0x7f, 32 * 4096 + 4096);
    hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
    printf("CU cycles per wave64 load (2.4 GHz nominal), independent loads, 8 waves/SIMD, %d CUs\n", cus);
    printf("  dword    %.2f\n", run<0>(buf, out, cus));
    printf("  dwordx4  %.2f\n", run<1>(buf, out, cus));
    printf("  fmt_x    %.2f\n", run<2>(buf, out, cus));
    printf("  fmt_xy   %.2f\n", run<3>(buf, out, cus));
    printf("  fmt_xyzw %.2f\n", run<4>(buf, out, cus));
    hipFree(buf);
    hipFree(out);
    return 0;
}
