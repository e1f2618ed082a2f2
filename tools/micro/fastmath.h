// Correctly rounded fp32 sqrt and reciprocal: hipcc's core sequences without
// their special-input handling, plus a per-lane branch to the library form for
// the inputs that need it.  EQUAL to sqrtf / 1.0f / x on every input
// (fastmath_check.hip, all 2^32 bit patterns: profiles/r01_fastmath_check.txt)
// but slower inside the render kernel than the branch-free library sequences
// (+1.4..3.8 %, DESIGN.md "rejected"), so the kernel does not use it.
#pragma once

#include <hip/hip_runtime.h>

namespace vx {

// The residual-corrected core of hipcc's correctly rounded sqrtf on gfx950:
// s = v_sqrt(x), then the neighbours s -+ 1 ulp are taken when the exact
// residuals x - s'*s say so.  Valid as is for x = +0, +inf and every x >=
// 2^-96 (below that the residual loses bits: the library scales by 2^32).
__device__ __forceinline__ float sqrt_core(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __builtin_bit_cast(float, __builtin_bit_cast(int, s) - 1);
    const float up = __builtin_bit_cast(float, __builtin_bit_cast(int, s) + 1);
    float r = __builtin_fmaf(-dn, s, x) <= 0.0f ? dn : s;
    r = __builtin_fmaf(-up, s, x) > 0.0f ? up : r;
    return r;
}

// sqrtf(x) exactly: the core where it is valid, the library sequence for the
// rest (tiny, negative, NaN) -- a divergent branch that almost never runs.
__device__ __forceinline__ float fsqrt(float x) {
    float r = sqrt_core(x);
    if (!(x >= 0x1p-96f || x == 0.0f)) r = sqrtf(x);
    return r;
}

// 1.0f / x exactly: v_rcp + one Newton step equals the IEEE reciprocal for
// |x| in [2^-40, 2^41) (exhaustively, both signs); the library division for
// the rest (zero, huge, tiny, inf, NaN).
__device__ __forceinline__ float frcp(float x) {
    const float r0 = __builtin_amdgcn_rcpf(x);
    float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
    const float ax = __builtin_fabsf(x);
    if (!(ax >= 0x1p-40f && ax < 0x1p41f)) r = 1.0f / x;
    return r;
}

}  // namespace vx
