// Vector-memory address-path cost of the march's texel load on gfx950: CU
// cycles per wave64 load instruction as a function of how many distinct
// 128-B cache lines the 64 lanes touch (1..64), for the load forms the march
// can use.  Each lane runs a dependent chain (the next address adds the loaded
// value, which is 0), 8 waves/SIMD, L2-resident 4 MiB footprint: the shape of
// march_pad's step without its VALU.  A CU has one address (TA) / data (TD)
// path shared by its 4 SIMDs, so cycles per wave-load per CU bounds a loop
// whose every step issues one such load.
//   sbyte   global_load_sbyte (saddr + 32-bit voffset)
//   fmt     buffer_load_format_x, 8-bit SSCALED (march_pad's VX_FMT_LOAD)
//   ubyte   buffer_load_ubyte (untyped)
//   dword   global_load_dword
// Also: CHAINS independent chains per lane (2 = two loads in flight per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITERS = 1024;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 rsrc(const void *base, unsigned w3) {
    const unsigned long long p = (unsigned long long)base;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((unsigned)p);
    r.y = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32) & 0xffffu);
    r.z = 0xffffffffu;
    r.w = w3;
    return r;
}

template <int KIND, int CHAINS>
__global__ __launch_bounds__(256) void k_load(const int8_t *buf, int lines, int *out) {
    const unsigned lane = threadIdx.x & 63;
    const unsigned gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const unsigned region = (gw & 63) * 65536u;               // 64 regions of 64 KiB: 4 MiB footprint
    // line j of the wave at ((j * 193) mod 512) * 128 B: scattered over the 64 KiB region, so
    // the lines fall on different cache channels (a 256-B stride puts them all on one)
    const unsigned lanepart = (((lane % lines) * 193u) & 511u) * 128u + (lane / lines) * (KIND == 3 ? 4u : 1u);
    const u32x4 rf = rsrc(buf, 0x0000B004u), ru = rsrc(buf, 0x00020000u);
    unsigned acc[CHAINS];
    for (int c = 0; c < CHAINS; c++) acc[c] = 0;
    for (int i = 0; i < ITERS; i++) {
        unsigned v[CHAINS];
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            const unsigned off = region + ((((unsigned)(i * CHAINS + c) & 3u) * 37u) << 7) + lanepart + acc[c];
            if (KIND == 0) {
                int t;
                asm volatile("global_load_sbyte %0, %1, %2" : "=v"(t) : "v"(off), "s"(buf));
                v[c] = (unsigned)t;
            } else if (KIND == 1) {
                float t;
                asm volatile("buffer_load_format_x %0, %1, %2, 0 offen" : "=v"(t) : "v"(off), "s"(rf));
                v[c] = __float_as_uint(t);
            } else if (KIND == 2) {
                unsigned t;
                asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen" : "=v"(t) : "v"(off), "s"(ru));
                v[c] = t;
            } else {
                unsigned t;
                asm volatile("global_load_dword %0, %1, %2" : "=v"(t) : "v"(off), "s"(buf));
                v[c] = t;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int c = 0; c < CHAINS; c++) asm volatile("v_add_u32 %0, %1, %0" : "+v"(acc[c]) : "v"(v[c]));
    }
    unsigned s = 0;
    for (int c = 0; c < CHAINS; c++) s += acc[c];
    if (s == 12345u) out[0] = 1;
}

template <int KIND, int CHAINS>
static double run(const int8_t *buf, int lines, int *out, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_load<KIND, CHAINS>), dim3(blocks), dim3(256), 0, 0, buf, lines, out);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_load<KIND, CHAINS>), dim3(blocks), dim3(256), 0, 0, buf, lines, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    // CU cycles per wave-load at 2.4 GHz (nominal; the clock under load may be lower)
    const double loads_per_cu = (double)blocks * 4 * ITERS * CHAINS / 256.0;
    return best * 1e-3 * 2.4e9 / loads_per_cu;
}

int main() {
    int8_t *buf;
    int *out;
    (void)hipMalloc(&buf, 8u << 20);
    (void)hipMemset(buf, 0, 8u << 20);
    (void)hipMalloc(&out, 4);
    const int blocks = 256 * 8;        // 8 blocks of 4 waves per CU: 8 waves/SIMD
    const int L[] = {1, 2, 4, 8, 16, 32, 64};
    printf("CU cycles per wave64 load (2.4 GHz nominal), dependent chain per lane, 8 waves/SIMD, L2-resident\n");
    printf("%6s %9s %9s %9s %9s %11s %11s\n", "lines", "sbyte", "fmt", "ubyte", "dword", "sbyte x2ch", "fmt x2ch");
    for (int l : L) {
        printf("%6d %9.2f %9.2f %9.2f %9.2f %11.2f %11.2f\n", l, run<0, 1>(buf, l, out, blocks),
               run<1, 1>(buf, l, out, blocks), run<2, 1>(buf, l, out, blocks), run<3, 1>(buf, l, out, blocks),
               run<0, 2>(buf, l, out, blocks), run<1, 2>(buf, l, out, blocks));
    }
    return 0;
}
