// Exhaustive check on gfx950: is y1 = fma(fma(-d, r, 1), r, r) with
// r = v_rcp_f32(d) equal to the IEEE quotient 1.0f / d (hipcc's correctly
// rounded division) for every float d of the tested exponent range, both
// signs?  Prints the mismatch count per exponent.  (Decides whether the
// primary-ray slab setup may use it: DESIGN.md §5.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void k_check(int e, unsigned long long *bad, unsigned long long *bad0) {
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;   // mantissa
    if (m >= (1u << 23)) return;
    unsigned long long nb = 0, nb0 = 0;
    for (int sgn = 0; sgn < 2; sgn++) {
        const unsigned u = ((unsigned)sgn << 31) | ((unsigned)(e + 127) << 23) | m;
        const float d = __uint_as_float(u);
        const float q = 1.0f / d;                                  // IEEE (correctly rounded)
        const float r = __builtin_amdgcn_rcpf(d);
        const float y1 = __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
        nb += __float_as_uint(y1) != __float_as_uint(q);
        nb0 += __float_as_uint(r) != __float_as_uint(q);
    }
    if (nb) atomicAdd(bad, nb);
    if (nb0) atomicAdd(bad0, nb0);
}

int main() {
    unsigned long long *d_bad;
    (void)hipMalloc(&d_bad, 16);
    unsigned long long tot = 0, tot0 = 0, n = 0;
    for (int e = -40; e <= 40; e++) {
        (void)hipMemset(d_bad, 0, 16);
        hipLaunchKernelGGL(k_check, dim3((1u << 23) / 256), dim3(256), 0, 0, e, d_bad, d_bad + 1);
        unsigned long long h[2];
        (void)hipMemcpy(h, d_bad, 16, hipMemcpyDeviceToHost);
        tot += h[0]; tot0 += h[1]; n += 2ull << 23;
        if (h[0]) printf("exponent %d: %llu mismatches (rcp+newton)\n", e, h[0]);
    }
    printf("inputs %llu (exponents -40..40, both signs): rcp+newton mismatches %llu, bare v_rcp mismatches %llu\n", n,
           tot, tot0);
    return tot != 0;
}
