// Exhaustive check on gfx950 of the one-correction Markstein division
//   y = 1.0f / b (IEEE), q0 = RN(a*y), q1 = RN(q0 + RN(a - q0*b)*y)
// against the IEEE quotient a / b for EVERY pair of significands
// a, b in [1, 2) (2^46 pairs).  Scaling a or b by a power of two scales every
// intermediate exactly while nothing under/overflows, and the sign is
// symmetric, so 0 mismatches here means div_const (vx_kernels.hip) is the
// IEEE quotient for all normal a, b whose quotient and residual stay normal —
// which licenses a per-pixel divisor (normalize3), not only per-frame ones.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_check(unsigned b_lo, unsigned b_count, unsigned long long *bad, unsigned *first) {
    const unsigned ma = blockIdx.x * blockDim.x + threadIdx.x;        // numerator significand, 2^23 threads
    const float a = __uint_as_float(0x3f800000u | ma);
    unsigned long long nb = 0;
    for (unsigned j = 0; j < b_count; j++) {
        const float b = __uint_as_float(0x3f800000u | (b_lo + j));
        const float y = 1.0f / b;
        const float q = a / b;
        const float q0 = a * y;
        const float r0 = __builtin_fmaf(-q0, b, a);
        const float q1 = __builtin_fmaf(r0, y, q0);
        if (__float_as_uint(q1) != __float_as_uint(q)) {
            nb++;
            atomicCAS(first, 0xffffffffu, ma);
            atomicCAS(first + 1, 0xffffffffu, b_lo + j);
        }
    }
    if (nb) atomicAdd(bad, nb);
}

int main(int argc, char **argv) {
    const unsigned per = 256;                                         // divisors per launch
    unsigned long long *d;
    unsigned *df;
    (void)hipMalloc(&d, 8);
    (void)hipMalloc(&df, 8);
    (void)hipMemset(d, 0, 8);
    (void)hipMemset(df, 0xff, 8);
    const unsigned nb_total = 1u << 23;
    for (unsigned b = 0; b < nb_total; b += per) {
        hipLaunchKernelGGL(k_check, dim3((1u << 23) / 256), dim3(256), 0, 0, b, per, d, df);
        if ((b / per) % 4096 == 4095) {
            (void)hipDeviceSynchronize();
            std::printf("divisor significands done: %u / %u\n", b + per, nb_total);
            std::fflush(stdout);
        }
    }
    unsigned long long h = 0;
    unsigned f[2];
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f, df, 8, hipMemcpyDeviceToHost);
    std::printf("significand pairs %llu: one-correction Markstein mismatches %llu", 1ull << 46, h);
    if (h) std::printf(" (first a=0x%06x b=0x%06x)", f[0], f[1]);
    std::printf("\n");
    return h != 0;
}
