// vx_render.h — the fused render kernel of the Voxmap shading path (gfx950),
// shared by the translation units that instantiate it.
//
// One fused kernel per frame: primary visibility (the build's replacement for
// rasterising vertex.bin) -> render.frag main() shading with
// the sun march() (render.frag:75-142) -> glass blend -> framebuffer store.
// Lane = pixel; a wave64 covers an 8x8 pixel tile, a 256-thread workgroup a
// 32x8 block, so the rays of a wave march through neighbouring cells.
//
// Each EXT mode's instantiations are compiled in a translation unit of their
// own (vx_render_e*.hip): the same template text, so every mode's code is what
// it would be in one file, the units build in parallel, and the general shading
// modes (EXT 5/6) get a register budget of their own (VX_OCC_ATTR) without a
// shared body function for the others.
//
// Numerical contract: fp32, IEEE div/sqrt, no FMA contraction
// (built with -ffp-contract=off), GLSL built-ins spelled out, vexp2 below, so
// every pixel matches the scalar oracle (oracle/vxo_render.c) bit for bit.
// Exactness-preserving rewrites used here (each justified in DESIGN.md §5):
//   * a / b with b a per-frame constant -> one Markstein correction from
//     y = RN(1/b) computed on the host (exhaustively checked:
//     tools/micro/markstein_all.hip);
//   * length(m*t) with a single selected axis -> t (sqrt(RN(t*t)) == t);
//   * unorm8 decode b/255 -> typed UNORM buffer loads (the texture data unit
//     returns RN(b/255) for every byte, tools/micro/unorm_check.hip);
//   * per-frame uniform-only expressions -> host (vx_frame.cpp).
// Rejected experiments (bricked layouts, LDS r*k tables, hand-batched sky
// loads, typed primary loads, ...) are measured in profiles/ and kept in git
// history, not here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vx_internal.h"
#ifndef VX_QSPEC
#define VX_QSPEC 1
#endif

namespace vx {
namespace {

constexpr int kWG = 256;      // threads per render workgroup (4 waves)
constexpr int kGlass = 21;  // render.vert:21, sdf.cpp:337
constexpr float kInf = __builtin_inff();

// ---------------- GLSL built-ins (GLSL ES 3.00 §8) ----------------
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float gclamp(float x, float a, float b) { return gmin(gmax(x, a), b); }
__device__ __forceinline__ float gmix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
// ivec(float) of the contract: NaN -> 0, saturate at +-2^24 (branch-free)
__device__ __forceinline__ int f2i(float x) {
    const float c = __builtin_fminf(__builtin_fmaxf(x, -16777216.0f), 16777216.0f);
    const int r = (int)c;
    return x == x ? r : 0;
}

// a / b, b a per-frame constant with y = RN(1/b), a > 0 (no signed zero):
// exactly the IEEE quotient.  q0 = RN(a*y) is faithful and one Markstein
// correction q1 = RN(q0 + fma(-q0, b, a)*y) is already correctly rounded
// (Markstein's theorem for y = RN(1/b); tools/markstein_check.c: 0 mismatches
// over every numerator in [1e-4, 1.0002] for thousands of divisors, random
// and adversarial mantissas; tools/micro/markstein_all.hip: every pair of
// significands).
__device__ __forceinline__ float div_const(float a, float b, float y) {
    const float q0 = a * y;
    const float r0 = __builtin_fmaf(-q0, b, a);
    return __builtin_fmaf(r0, y, q0);
}

// a / b for any sign of a (b > 0, y = RN(1/b)): div_const with the sign of a
// copied onto the result, so a = -0 gives -0 as the IEEE quotient does.
// One correction is exact for every pair of significands
// (tools/micro/markstein_all.hip, profiles/r01_markstein_all.txt), so the
// divisor may vary per pixel.
__device__ __forceinline__ float div_shared(float a, float b, float y) {
    return __builtin_copysignf(div_const(a, b, y), a);
}

// RN(1/l) for l with |l| in [2^-40, 2^41): v_rcp + one Newton step equals the
// IEEE reciprocal on every such input (tools/micro/rcp_check.hip, exhaustive
// over exponents -40..40, both signs: profiles/r01_rcp_check.txt).  Callers
// guarantee the range.
__device__ __forceinline__ float rcp_ranged(float l) {
    const float r = __builtin_amdgcn_rcpf(l);
    return __builtin_fmaf(__builtin_fmaf(-l, r, 1.0f), r, r);
}


// Correctly rounded sqrt without the wrapper hipcc puts around it.  sqrtf
// (-fhip-fp32-correctly-rounded-divide-sqrt) is v_sqrt_f32 plus a one-ulp
// residual correction, wrapped in a 2^32 input scaling for x < 2^-96 and a
// class test for zero / inf; sqrt_ranged is the correction alone, bit-identical
// to sqrtf on +-0 and on [2^-96, FLT_MAX] (tools/micro/sqrt_ranged_check.hip,
// every float of that domain: profiles/r03_sqrt_ranged_check.txt).
__device__ __forceinline__ float sqrt_ranged(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u), up = __uint_as_float(__float_as_uint(s) + 1u);
    float r = __builtin_fmaf(-dn, s, x) <= 0.0f ? dn : s;
    r = __builtin_fmaf(-up, s, x) > 0.0f ? up : r;
    return r;
}

// exp2 by the fixed degree-9 polynomial of the numerical contract.
__device__ __forceinline__ float vexp2(float x) {
    if (x != x) return x;
    if (x >= 128.0f) return kInf;
    if (x < -126.0f) return 0.0f;
    const float n = floorf(x);
    const float f = x - n;
    float p = 1.0178086e-07f;
    p = p * f + 1.3215487e-06f;
    p = p * f + 1.5252734e-05f;
    p = p * f + 1.5403530e-04f;
    p = p * f + 1.3333558e-03f;
    p = p * f + 9.6181291e-03f;
    p = p * f + 5.5504109e-02f;
    p = p * f + 2.4022651e-01f;
    p = p * f + 6.9314718e-01f;
    p = p * f + 1.0f;
    return ldexpf(p, (int)n);
}
__device__ __forceinline__ float vexp(float x) { return vexp2(x * 1.44269504f); }

// The GL blend stage (oracle blend_canvas).  Every draw blends SRC_ALPHA /
// ONE_MINUS_SRC_ALPHA (render.js:84-86) into an RGBA8 canvas (map.js:7): for a
// fixed-point buffer GLES 3.0 §4.1.7 clamps source, destination and blend
// factors to [0, 1], and the destination is the byte the canvas holds for the
// colour written before (pack_rgba8's floor(clamp(v) * 255 + 0.5)), read back
// as RN(byte / 255).  A pane over dst: clamp(src) * a + canvas8(dst) * (1 - a)
// with a = clamp(src.a); the next pane reads that back through canvas8 again.
constexpr float kRcp255 = 1.0f / 255.0f;     // RN(1/255): div_const's reciprocal
__device__ __forceinline__ float canvas8(float v) {
    return div_const(floorf(gclamp(v, 0.0f, 1.0f) * 255.0f + 0.5f), 255.0f, kRcp255);   // exactly RN(q / 255)
}
__device__ __forceinline__ void blend_canvas(const float src[4], const float dst[3], float out[3]) {
    const float al = gclamp(src[3], 0.0f, 1.0f);
#pragma unroll
    for (int i = 0; i < 3; i++) out[i] = gclamp(src[i], 0.0f, 1.0f) * al + canvas8(dst[i]) * (1.0f - al);
}

__constant__ float kPalette[22][3] = {
    {0.0f, 0.0f, 0.0f},
    {0.0431373f, 0.0627451f, 0.0745098f},
    {0.133333f, 0.490196f, 0.317647f},
    {0.321569f, 0.262745f, 0.239216f},
    {0.337255f, 0.423529f, 0.45098f},
    {0.392157f, 0.211765f, 0.235294f},
    {0.396078f, 0.403922f, 0.396078f},
    {0.439216f, 0.486275f, 0.454902f},
    {0.454902f, 0.403922f, 0.243137f},
    {0.52549f, 0.65098f, 0.592157f},
    {0.52549f, 0.756863f, 0.4f},
    {0.568627f, 0.596078f, 0.623529f},
    {0.647059f, 0.870588f, 0.894118f},
    {0.666667f, 0.666667f, 0.666667f},
    {0.741176f, 0.752941f, 0.729412f},
    {0.768627f, 0.384314f, 0.262745f},
    {0.780392f, 0.243137f, 0.227451f},
    {0.854902f, 0.788235f, 0.65098f},
    {0.964706f, 0.772549f, 0.333333f},
    {0.984314f, 0.886275f, 0.317647f},
    {1.0f, 1.0f, 1.0f},
    {0.505882f, 0.780392f, 0.831373f},
};

struct Surf {            // one G-buffer record (what render.vert hands render.frag)
    int id;              // 0 block, 1 sky, 2 glass
    int color;           // palette index
    int nidx;            // normal index 0..5 (render.vert:14-17)
    float c0, c1, c2;    // v_cellPos (exact integers: fp32 keeps the consumers' arithmetic convert-free)
    float f0, f1, f2;    // v_fractPos
};

struct Counters {
    unsigned prim_fetch, shadow_rays, shadow_fetch, ao, noise_px, cap_hit;
    unsigned refl_rays, refl_fetch, rough;   // extensions
    unsigned prim_witers, march_witers;      // loop iterations per wave (diagnostic: lane utilisation)
    unsigned march_slots;                    // per march wave iteration: the lanes that began that march
    unsigned shadow_resolved;                // shadow rays resolved by the first-step table test (not marched)
};

// (float)((t >> 8k) & 0xff) as one v_cvt_f32_ubyteK (left to itself the
// compiler may fold the mask away and emit a shift + convert)
__device__ __forceinline__ float cvt_f32_ubyte0(uint32_t t) {
    float r;
    asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
__device__ __forceinline__ float cvt_f32_ubyte1(uint32_t t) {
    float r;
    asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
__device__ __forceinline__ float cvt_f32_ubyte2(uint32_t t) {
    float r;
    asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
__device__ __forceinline__ float cvt_f32_ubyte3(uint32_t t) {
    float r;
    asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

// v counted once per wave: by the first active lane (wave-uniform loop counts)
__device__ __forceinline__ unsigned once_per_wave(unsigned v) {
    const unsigned long long act = __ballot(1);
    return __lane_id() == (unsigned)(__ffsll((unsigned long long)act) - 1) ? v : 0u;
}
// the lanes of the wave that run this code (a march's marching lanes, taken at its start)
__device__ __forceinline__ unsigned active_lanes() { return (unsigned)__popcll(__ballot(1)); }

// Field data in HBM, each array shaped for the loop that
// reads it, so a cache line holds as many useful cells as possible:
//   prim  8 copies, one per ray octant, u32 per cell: vis colour | ex << 8 |
//         ey << 16 | ez << 24 (vis colour = map.bin B if it is a meshed palette
//         index 1..21, else 0 = never a surface; extents of the all-unmeshed box
//         ahead, vxo_field_box), inside a border of P = cap sentinel cells
//         (0xFFFFFFFF: colour 0xFF is no vis colour, extents are <= cap - 1 <=
//         254), so the primary traversal detects leaving the grid from the value
//         it loads;
//   sunp  map.bin's R ("up") and G ("down") channels, int8 each, inside a
//         border of -1 cells: the sun march reads one of them;
//   sun   the same channels u8, unpadded (the literal march);
//   rg    R | G << 8, u16, linear: the AO trilinear sample.
// Every read is in bounds: the traversal stays within P of the grid, march()
// returns before reading outside it, the AO sample clamps.
constexpr uint32_t kSentinel = 0xFFFFFFFFu;   // border cells: colour 0xFF, extents 255

// Loads at a 32-bit byte offset from a wave-uniform base: lets the compiler
// use the saddr form (SGPR base + VGPR offset) instead of 64-bit per-lane
// address arithmetic.  Offsets here are < 2^31 (vx_scene_create limits).
template <typename T>
__device__ __forceinline__ T ld_off(const T *base, unsigned byte_off) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + byte_off);
}

// Typed buffer loads: the texture data unit converts the texel.
//   * the march texel: descriptor "8-bit, SSCALED" (DATA_FORMAT 1, NUM_FORMAT
//     3, DST_SEL_X = X) returns (float)(int8)texel, so the loop has no
//     byte -> float convert; base = the channel moved down by the offset bias
//     (0x4B000000, march_pad), num_records = 2^32 - 1 (offsets are in bounds
//     by the -1 border);
//   * AO and noise texels: NUM_FORMAT UNORM returns RN(b / 255) for every
//     byte b, the exact render.frag:38 decode (tools/micro/unorm_check.hip: all
//     256 bytes, 8, 8_8 and 8_8_8_8 formats, profiles/r02_unorm_check.txt).
// All of them through the LLVM intrinsic: the compiler sees the loads, places
// the waits, schedules independent work under them and never copies or spills
// a register a load has not written yet.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 buf_rsrc(const void *base, unsigned w3) {
    const unsigned long long p = (unsigned long long)base;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((unsigned)p);
    r.y = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32) & 0xffffu);
    r.z = 0xffffffffu;
    r.w = w3;
    return r;
}
constexpr unsigned kRsrcS8 = 0x0000B004u;  // 8, SSCALED, dst X: the march texel
constexpr unsigned kRsrcRGBA = 0x50FACu;   // 8_8_8_8, UNORM, dst (X, Y, Z, W): AO pairs, noise quads
__device__ float vx_ld_format_f32(u32x4 rsrc, unsigned voff, int soff, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.format.f32");
__device__ f32x4 vx_ld_format_v4f32(u32x4 rsrc, unsigned voff, int soff, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.format.v4f32");
__device__ __forceinline__ float ld_fmt1(u32x4 rsrc, unsigned off) { return vx_ld_format_f32(rsrc, off, 0, 0); }
__device__ __forceinline__ f32x4 ld_fmt4(u32x4 rsrc, unsigned off) { return vx_ld_format_v4f32(rsrc, off, 0, 0); }

// x + X*y + XY*z; X*Y < 2^23 (vx_scene_create): full-rate 24-bit multiplies
__device__ __forceinline__ unsigned lin_index(const KernelArgs &a, int x, int y, int z) {
    return (unsigned)x + __umul24((unsigned)a.X, (unsigned)y) + __umul24(a.XY, (unsigned)z);
}

// ---------------- sun march: render.frag:75-142 ----------------
// Fast exact path for sun directions with every |r_i| >= 2^-10 (no zero
// component, so no 0*inf NaN; every t finite and < 1025).  `sun` is the
// channel sdf_dir reads (R "up" for r.z > 0, else G "down").  Returns "lit"
// (step == MAX_STEPS, render.frag:234).
//
// Loop shape: rotated so that the step length of the NEXT step (fract,
// three divisions, min3: it depends only on f) is computed while the texel
// load of this step is in flight; the dependent chain of a step is then just
// safe -> f -> floor -> cell -> address -> load.  One exit test per step
// (sky, safe == 0 or the step budget); cells kept as exact fp32 integers; the
// three-way min and its tie test as min3/med3 (two or more axes share the
// minimum iff med3 == min3, then the literal length of render.frag:105-116).
__device__ __forceinline__ float march_len(const SunRay &S, float f0, float f1, float f2) {
    const float x0 = -f0 * S.sign[0], x1 = -f1 * S.sign[1], x2 = -f2 * S.sign[2];     // :94
    const float d0 = (x0 - floorf(x0)) + 1e-4f;
    const float d1 = (x1 - floorf(x1)) + 1e-4f;
    const float d2 = (x2 - floorf(x2)) + 1e-4f;
    const float t0 = div_const(d0, S.abs[0], S.rcp[0]);                                // :97
    const float t1 = div_const(d1, S.abs[1], S.rcp[1]);
    const float t2 = div_const(d2, S.abs[2], S.rcp[2]);
    float len = __builtin_fminf(__builtin_fminf(t0, t1), t2);                         // :100-105, one axis
    if (__builtin_amdgcn_fmed3f(t0, t1, t2) == len) {                                  // ties: literal length
        const float v0 = t0 == len ? t0 : 0.0f, v1 = t1 == len ? t1 : 0.0f, v2 = t2 == len ? t2 : 0.0f;
        len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
    }
    return len;
}

// march_len with the sun's axis signs known at compile time (SG bit i: r_i > 0;
// the fast paths have no zero component): fract(-f*s) + 1e-4 without the
// multiply -- for s > 0 it is (-f) - floor(-f) = ceil(f) - f, the same single
// IEEE subtraction (floor(-f) = -ceil(f)); for s < 0, f - floor(f).
// the step length from the distance terms d_i = fract(-f_i*s_i) + 1e-4 (:94-105)
__device__ __forceinline__ float march_len_d(const SunRay &S, float d0, float d1, float d2) {
    const float t0 = div_const(d0, S.abs[0], S.rcp[0]);                                // :97
    const float t1 = div_const(d1, S.abs[1], S.rcp[1]);
    const float t2 = div_const(d2, S.abs[2], S.rcp[2]);
    float len = __builtin_fminf(__builtin_fminf(t0, t1), t2);                         // :100-105, one axis
    if (__builtin_amdgcn_fmed3f(t0, t1, t2) == len) {                                  // ties: literal length
        const float v0 = t0 == len ? t0 : 0.0f, v1 = t1 == len ? t1 : 0.0f, v2 = t2 == len ? t2 : 0.0f;
        len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
    }
    return len;
}

template <int SG>
__device__ __forceinline__ float march_len_sg(const SunRay &S, float f0, float f1, float f2) {
    const float d0 = ((SG & 1) ? ceilf(f0) - f0 : f0 - floorf(f0)) + 1e-4f;
    const float d1 = ((SG & 2) ? ceilf(f1) - f1 : f1 - floorf(f1)) + 1e-4f;
    const float d2 = ((SG & 4) ? ceilf(f2) - f2 : f2 - floorf(f2)) + 1e-4f;
    const float t0 = div_const(d0, S.abs[0], S.rcp[0]);                                // :97
    const float t1 = div_const(d1, S.abs[1], S.rcp[1]);
    const float t2 = div_const(d2, S.abs[2], S.rcp[2]);
    float len = __builtin_fminf(__builtin_fminf(t0, t1), t2);                         // :100-105, one axis
    if (__builtin_amdgcn_fmed3f(t0, t1, t2) == len) {                                  // ties: literal length
        const float v0 = t0 == len ? t0 : 0.0f, v1 = t1 == len ? t1 : 0.0f, v2 = t2 == len ? t2 : 0.0f;
        len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
    }
    return len;
}

// march_len_sg inside the march loop, where every f_i is a step's
// f - floor(f), so f_i in [0, 1]: each fract term is one v_fract_f32 (a
// 4-cycle op, against floor/ceil + subtract = 6).  v_fract(x) is x - floor(x)
// clamped below 1.0; the two uses never reach the clamp:
//   s < 0: v_fract(f) = f for f in [0, 1), 0 for f = 1 -- exactly f - floor(f);
//   s > 0: v_fract(-f) = RN(1 - f) for f in (0, 1], 0 for f = 0 -- exactly
//          ceil(f) - f, unless RN(1 - f) = 1.0, i.e. 0 < f <= 2^-25.  That f
//          never occurs after a step taken from an f >= 0 (every step after
//          the first): the axis moves by RN(RN(r*safe)*len) >= 2^-10 * 1e-4
//          (|r_i| >= 2^-10 on the fast path, safe >= 1, len >= 1e-4 since
//          every d >= 1e-4 and |r| <= 1), so f_u >= 9.7e-8 and its fraction
//          is f_u itself or a multiple of ulp(1) = 2^-23.
// The first step starts from the surface's fract, which can be slightly
// negative (the hit point's rounding), so march_pad keeps march_len_sg there.
template <int SG>
__device__ __forceinline__ float march_len_fract(const SunRay &S, float f0, float f1, float f2) {
    const float d0 = __builtin_amdgcn_fractf((SG & 1) ? -f0 : f0) + 1e-4f;
    const float d1 = __builtin_amdgcn_fractf((SG & 2) ? -f1 : f1) + 1e-4f;
    const float d2 = __builtin_amdgcn_fractf((SG & 4) ? -f2 : f2) + 1e-4f;
    const float t0 = div_const(d0, S.abs[0], S.rcp[0]);                                // :97
    const float t1 = div_const(d1, S.abs[1], S.rcp[1]);
    const float t2 = div_const(d2, S.abs[2], S.rcp[2]);
    float len = __builtin_fminf(__builtin_fminf(t0, t1), t2);                         // :100-105, one axis
    if (__builtin_amdgcn_fmed3f(t0, t1, t2) == len) {                                  // ties: literal length
        const float v0 = t0 == len ? t0 : 0.0f, v1 = t1 == len ? t1 : 0.0f, v2 = t2 == len ? t2 : 0.0f;
        len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
    }
    return len;
}

__device__ __forceinline__ bool march_fast(const KernelArgs &a, const SunRay &S, const uint8_t *sun, float c0, float c1, float c2, float f0,
                           float f1, float f2, Counters &cnt) {
    const FrameConsts &F = a.fc;
    const float r0 = S.r[0], r1 = S.r[1], r2 = S.r[2];
    const int maxs = F.max_steps;
    if (maxs <= 0) return maxs == 0;
    float safe = 1.0f;
    float e0 = c0, e1 = c1, e2 = c2;
    float len = march_len(S, f0, f1, f2);
    int step = 0;
    const unsigned nl = active_lanes();
    do {
        f0 = f0 + (r0 * safe) * len;                                             // :118
        f1 = f1 + (r1 * safe) * len;
        f2 = f2 + (r2 * safe) * len;
        const float fl0 = floorf(f0), fl1 = floorf(f1), fl2 = floorf(f2);
        e0 += fl0; e1 += fl1; e2 += fl2;                                         // :119 (exact)
        f0 = f0 - fl0; f1 = f1 - fl1; f2 = f2 - fl2;                             // :120
        const int i0 = (int)e0, i1 = (int)e1, i2 = (int)e2;
        const bool sky = (unsigned)i0 >= (unsigned)a.X || (unsigned)i1 >= (unsigned)a.Y || (unsigned)i2 >= (unsigned)a.Z;
        const uint32_t t = sun[sky ? 0u : lin_index(a, i0, i1, i2)];             // :123-128
        cnt.shadow_fetch += sky ? 0u : 1u;
        cnt.march_witers += once_per_wave(1u);
        cnt.march_slots += once_per_wave(nl);
        len = march_len(S, f0, f1, f2);                                          // next step, under the load
        // safe < 0 marks "lit": left the grid (:123-126), or the step that
        // reaches MAX_STEPS, whatever it read (:234 tests step, not safe)
        safe = sky ? -1.0f : (float)t;
        if (++step >= maxs) safe = -1.0f;
    } while (safe > 0.0f);
    return safe < 0.0f;
}

// The same march over the int8 sun channels inside a border of -1 cells
// (vx_scene_create, Z <= 126): a step moves at most safe + 1 <= Z + 1 cells
// per axis, so the texel a lane loads after leaving the grid is a border
// cell and its -1 is the exit ("lit", render.frag:123-126) -- no bounds test.
// The last step (step MAX_STEPS-1 -> MAX_STEPS) is lit whatever it reads
// (:234), so the loop runs MAX_STEPS-1 steps with the step test on the scalar
// unit, and a lane still marching afterwards is lit.
//
// Cells as fp32 integers, x and z biased by 2^23 (exact below 2^24): the bit
// pattern of 2^23 + n is 0x4B000000 + n, so the x + Xp*y part of the offset is
// the bit pattern of one exact fma and the low 24 bits of the z pattern are z
// itself -- no float -> int converts in the loop:
//   bits(fma(y, Xp, 2^23 + x)) + u24(bits(2^23 + z)) * XpYp
//     = 0x4B000000 + x + Xp*y + XpYp*z,
// read from the channel base moved down by 0x4B000000 (vx_scene_create checks
// Xp*Yp < 2^23 and the sum < 2^32).  The x + Xp*y part is carried as one
// biased fp32 integer exy (2^23 <= exy < 2^24) and moved by fma(fl1, Xp, fl0)
// per step.  The texel arrives as a float (kRsrcS8): safe directly, -1 = left
// the grid.
// march_pad's loop from a start state: exy, e2 = the start cell's biased
// offset terms, len = the first step's length (march_len_sg), rsrc = the
// channel's typed-load descriptor (march_pad; march_soft shares these across
// the samples of a fragment).
// A doom code (a frame's cone copy, launch_sun_doom: kDoomBase - C)
// read at landing j: the cell is one from which every ray of the frame's window
// meets a solid cell after at most C boundary crossings, so the march lands on
// a 0 texel within 2 C landings -- unlit (0) if that is before MAX_STEPS, else
// the march goes on from the cell's texel T, read from the plain channel
// (oracle march_ex).  Anything else is returned as read.
__device__ __forceinline__ float doom_resolve(const KernelArgs &a, float t, int j, int maxs, unsigned off) {
    if (t <= -8.5f) {
        const int c = (int)(-8.0f - t);                                           // C
        t = j + 2 * c < maxs ? 0.0f : ld_fmt1(buf_rsrc(a.sunp - 0x4B000000, kRsrcS8), off);
    }
    return t;
}

// DOOM (kDoomAfter): the copy may hold doom codes.  The peeled first landing
// resolves its own; a code read in the loop ends the loop like any negative
// value and is resolved after it (landing j), a late one marching on in a
// per-lane loop of its own, so the main loop keeps its scalar step count.
// (Resolving in the loop at the wave's landing instead measured slower on C5
// and C3, though it keeps the hard units' step loop free of spills:
// profiles/r06_ab_doom3_c5.txt, r06_ab_doom10_*.txt.)
constexpr int kDoomNone = 0, kDoomAfter = 1;
template <int SG, int DOOM = kDoomNone>
__device__ __forceinline__ bool march_pad_from(const KernelArgs &a, const SunRay &S, u32x4 rsrc, float exy, float e2,
                                               float len, float f0, float f1, float f2, Counters &cnt) {
    const float r0 = S.r[0], r1 = S.r[1], r2 = S.r[2];
    const int maxs = a.fc.max_steps;
    if (maxs <= 0) return maxs == 0;
    const float xpf = (float)a.SXp;
    const unsigned sxpyp = a.SXpYp;
    float tv = 1.0f;                            // texel of the current cell = safe (render.frag:86: 1)
    // one step of :94-128 -> the offset of the texel to load
    auto advance = [&]() -> unsigned {
        f0 = f0 + (r0 * tv) * len;                                                // :118
        f1 = f1 + (r1 * tv) * len;
        f2 = f2 + (r2 * tv) * len;
        const float fl0 = floorf(f0), fl1 = floorf(f1), fl2 = floorf(f2);
        f0 = f0 - fl0; f1 = f1 - fl1; f2 = f2 - fl2;                              // :120
        exy += __builtin_fmaf(fl1, xpf, fl0); e2 += fl2;                          // :119 (exact)
        return __umul24(__float_as_uint(e2), sxpyp) + __float_as_uint(exy);
    };
    // the offset of the cell the last step landed in
    auto cell_off = [&]() -> unsigned { return __umul24(__float_as_uint(e2), sxpyp) + __float_as_uint(exy); };
    int step = 0;                                                                // wave-uniform
    const unsigned nl = active_lanes();
    if (maxs > 1) {                            // the first step, peeled: its len from march_len_sg
        float t = ld_fmt1(rsrc, advance());                                        // :123-128
        len = march_len_sg<SG>(S, f0, f1, f2);  // next step, under the load
        cnt.shadow_fetch += t >= 0.0f ? 1u : 0u;
        if constexpr (DOOM != kDoomNone) t = doom_resolve(a, t, 1, maxs, cell_off());
        tv = t;
        cnt.march_witers += once_per_wave(1u);
        cnt.march_slots += once_per_wave(nl);
        ++step;
    }
    if (maxs > 1 && tv > 0.0f && step < maxs - 1) {
        int j = 1;                             // DOOM: the lane's landings (the loop's exit leaves step behind)
        do {
            float t = ld_fmt1(rsrc, advance());
            len = march_len_fract<SG>(S, f0, f1, f2);   // next step, under the load
            cnt.shadow_fetch += t >= 0.0f ? 1u : 0u;
            tv = t;
            if constexpr (DOOM == kDoomAfter) ++j;
            cnt.march_witers += once_per_wave(1u);   // counted in the loop: step stays a scalar
            cnt.march_slots += once_per_wave(nl);
        } while (tv > 0.0f && ++step < maxs - 1);
        if constexpr (DOOM == kDoomAfter) {
            if (tv <= -8.5f) {                 // a doom code at landing j
                tv = doom_resolve(a, tv, j, maxs, cell_off());
                while (tv > 0.0f && j < maxs - 1) {   // late: on from the cell's texel (rare)
                    const unsigned o = advance();
                    const float t2 = ld_fmt1(rsrc, o);
                    len = march_len_fract<SG>(S, f0, f1, f2);
                    cnt.shadow_fetch += t2 >= 0.0f ? 1u : 0u;
                    cnt.march_witers += once_per_wave(1u);
                    cnt.march_slots += once_per_wave(nl);
                    tv = doom_resolve(a, t2, ++j, maxs, o);
                }
            }
        }
    }
    if (tv > 0.0f) {                           // the MAX_STEPS-th step: only its fetch (stats) matters
        const float t = ld_fmt1(rsrc, advance());   // (dropped unless counted)
        cnt.shadow_fetch += t >= 0.0f ? 1u : 0u;
    }
    return tv != 0.0f;
}

template <int SG, int DOOM = kDoomNone>   // the sun's axis signs (bit i: r_i > 0); DOOM: see march_pad_from
__device__ __forceinline__ bool march_pad(const KernelArgs &a, const SunRay &S, const int8_t *sun, float c0, float c1,
                                          float c2, float f0, float f1, float f2, Counters &cnt) {
    const float xpf = (float)a.SXp;
    constexpr float kBias = 8388608.0f;
    const float exy = __builtin_fmaf(c1 + a.SBf, xpf, (c0 + a.SBf) + kBias);   // exact integers
    const float e2 = (c2 + a.SBf) + kBias;
    const u32x4 rsrc = buf_rsrc(sun - 0x4B000000, kRsrcS8);   // (pointer arithmetic: keeps the global address space)
    return march_pad_from<SG, DOOM>(a, S, rsrc, exy, e2, march_len_sg<SG>(S, f0, f1, f2), f0, f1, f2, cnt);
}

// The soft-shadow samples of one fragment (every sample on the padded path with
// sign pattern SG, all reading `sun`): the start cell's offset terms, the
// descriptor and the first step's fract terms d_i are the same for every
// sample, so they are formed once; only the three quotients by |r_k| differ.
template <int SG>
__device__ __forceinline__ int march_soft(const KernelArgs &a, const int8_t *sun, float c0, float c1, float c2, float f0,
                                          float f1, float f2, Counters &cnt) {
    const FrameConsts &F = a.fc;
    const float xpf = (float)a.SXp;
    constexpr float kBias = 8388608.0f;
    const float exy = __builtin_fmaf(c1 + a.SBf, xpf, (c0 + a.SBf) + kBias);
    const float e2 = (c2 + a.SBf) + kBias;
    const u32x4 rsrc = buf_rsrc(sun - 0x4B000000, kRsrcS8);
    const float d0 = ((SG & 1) ? ceilf(f0) - f0 : f0 - floorf(f0)) + 1e-4f;     // march_len_sg's terms
    const float d1 = ((SG & 2) ? ceilf(f1) - f1 : f1 - floorf(f1)) + 1e-4f;
    const float d2 = ((SG & 4) ? ceilf(f2) - f2 : f2 - floorf(f2)) + 1e-4f;
    int lit = 0;
    for (int k = 0; k < F.n_sun; k++) {
        cnt.shadow_rays++;
        const SunRay S = F.sun_k[k];
        lit += march_pad_from<SG, kDoomAfter>(a, S, rsrc, exy, e2, march_len_d(S, d0, d1, d2), f0, f1, f2, cnt) ? 1 : 0;
    }
    return lit;
}

// march_pad with an LDS brick (VX_FLAG_SOFT_BRICK, the EXT 4 instantiation:
// north_star's "8^3 brick staging"): the pooled pass stages, per fragment, the
// 8x8x8 block of the march channel around its start cell in LDS (origin at or
// one cell behind the start on a positive axis, four to seven cells behind on a
// negative one, x aligned to 4 bytes, so the first steps toward the sun stay
// inside), and a step reads LDS when its cell lies in that brick, the global
// channel otherwise.  Same step arithmetic as
// march_pad (fract peel, exact cells), cells kept per axis for the brick test:
// local = cell - origin as exact fp32 integers, inside iff the largest of the
// three bit patterns is below bits(8.0f) (a negative local has its sign bit set).
template <int SG>
__device__ __forceinline__ bool march_brick(const KernelArgs &a, const SunRay &S, const int8_t *sun,
                                            const int8_t *brick, int ox, int oy, int oz, float c0, float c1, float c2,
                                            float f0, float f1, float f2, Counters &cnt) {
    const float r0 = S.r[0], r1 = S.r[1], r2 = S.r[2];
    const int maxs = a.fc.max_steps;
    if (maxs <= 0) return maxs == 0;
    constexpr float kBias = 8388608.0f;
    const float xpf = (float)a.SXp;
    const int8_t *sunb = sun - 0x4B000000;
    float e0 = (c0 + a.SBf) + kBias, e1 = c1 + a.SBf, e2 = (c2 + a.SBf) + kBias;
    // brick origin (padded cells, same biases as the cells)
    const float b0 = (float)ox + kBias, b1 = (float)oy, b2 = (float)oz + kBias;
    const unsigned sxpyp = a.SXpYp;
    float len = march_len_sg<SG>(S, f0, f1, f2);
    int tv = 1;
    int step = 0;
    const unsigned nl = active_lanes();
    bool first = true;
    do {
        const float safe = cvt_f32_ubyte0((uint32_t)tv);
        f0 = f0 + (r0 * safe) * len;                                              // :118
        f1 = f1 + (r1 * safe) * len;
        f2 = f2 + (r2 * safe) * len;
        const float fl0 = floorf(f0), fl1 = floorf(f1), fl2 = floorf(f2);
        f0 = f0 - fl0; f1 = f1 - fl1; f2 = f2 - fl2;                              // :120
        e0 += fl0; e1 += fl1; e2 += fl2;                                          // :119
        const float l0 = e0 - b0, l1 = e1 - b1, l2 = e2 - b2;                     // exact small integers
        const unsigned m = max(max(__float_as_uint(l0), __float_as_uint(l1)), __float_as_uint(l2));
        int t;
        if (m < 0x41000000u) {                                                    // inside the brick
            t = brick[(int)__builtin_fmaf(l2, 64.0f, __builtin_fmaf(l1, 8.0f, l0))];
        } else {
            const unsigned off = __umul24(__float_as_uint(e2), sxpyp) + __float_as_uint(__builtin_fmaf(e1, xpf, e0));
            t = (int)ld_off(sunb, off);
        }
        len = first ? march_len_sg<SG>(S, f0, f1, f2) : march_len_fract<SG>(S, f0, f1, f2);
        first = false;
        cnt.shadow_fetch += t >= 0 ? 1u : 0u;
        tv = t;
        cnt.march_witers += once_per_wave(1u);
        cnt.march_slots += once_per_wave(nl);
    } while (tv > 0 && ++step < maxs);
    // lit: left the grid (-1), or the MAX_STEPS-th step taken whatever it read
    // (render.frag:234: a block on the last step still ends with step == MAX_STEPS);
    // a block found earlier ends the loop with step + 1 < maxs
    return tv != 0 || step + 1 >= maxs;
}

// Literal path for any other sun direction (zero or tiny components: the
// 0*inf = NaN and ivec3(floor(NaN)) := 0 rules of the contract apply).
__device__ __forceinline__ bool march_literal(const KernelArgs &a, const SunRay &S, const uint8_t *sun, float cf0, float cf1,
                                              float cf2, float f0, float f1, float f2, Counters &cnt) {
    int c0 = (int)cf0, c1 = (int)cf1, c2 = (int)cf2;      // exact integers
    const FrameConsts &F = a.fc;
    const float s0 = S.sign[0], s1 = S.sign[1], s2 = S.sign[2];
    const float a0 = S.abs[0], a1 = S.abs[1], a2 = S.abs[2];
    const float r0 = S.r[0], r1 = S.r[1], r2 = S.r[2];
    const int maxs = F.max_steps;
    float safe = 1.0f;
    int step = 0;
    const unsigned nl = active_lanes();
    while (step < maxs && safe != 0.0f) {
        const float x0 = -f0 * s0, x1 = -f1 * s1, x2 = -f2 * s2;
        const float d0 = (x0 - floorf(x0)) + 1e-4f;
        const float d1 = (x1 - floorf(x1)) + 1e-4f;
        const float d2 = (x2 - floorf(x2)) + 1e-4f;
        const float t0 = d0 / a0, t1 = d1 / a1, t2 = d2 / a2;
        const float m0 = t0 <= gmin(t1, t2) ? 1.0f : 0.0f;
        const float m1 = t1 <= gmin(t2, t0) ? 1.0f : 0.0f;
        const float m2 = t2 <= gmin(t0, t1) ? 1.0f : 0.0f;
        const float v0 = m0 * t0, v1 = m1 * t1, v2 = m2 * t2;
        const float len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
        f0 = f0 + (r0 * safe) * len;
        f1 = f1 + (r1 * safe) * len;
        f2 = f2 + (r2 * safe) * len;
        const float fl0 = floorf(f0), fl1 = floorf(f1), fl2 = floorf(f2);
        c0 += f2i(fl0); c1 += f2i(fl1); c2 += f2i(fl2);
        f0 = f0 - fl0; f1 = f1 - fl1; f2 = f2 - fl2;
        cnt.march_witers += once_per_wave(1u);
        cnt.march_slots += once_per_wave(nl);
        if (c0 >= a.X || c1 >= a.Y || c2 >= a.Z || c0 < 0 || c1 < 0 || c2 < 0) return true;
        const uint32_t t = sun[lin_index(a, c0, c1, c2)];
        cnt.shadow_fetch++;
        safe = (float)t;
        step++;
    }
    return step == maxs;
}

// The first step of a march from a face (DESIGN.md §3 "Sun exit tables", the
// first step).  A fragment starts on its face plane (f = 0 on the face axis a)
// at in-face cells c_j + floor(f_j), c_k + floor(f_k) with fractions in
// [0, 1) (RN(f + d) is monotone in d, so the step's cell moves by floor(f) +
// 0 or 1 toward the sun on each in-face axis); when the sun lies on the face's normal
// side, the first step -- len <= sqrt(3) * 1e-4/|r_a| (a tie takes the literal
// length), so it moves under 0.2 cell on the other axes -- lands in the air
// cell on the normal side or a neighbour of it toward the sun on the in-face
// axes (f_j, f_k in [0, 1)): the 2 x 2 block of bit a.  If the air cell's value
// in the exit copy carries bit a, every cell the step can land in is marked,
// so the march ends there, lit, with no fetch counted: the same lit flag and
// counters without its setup, first step and load.  Used for the soft-shadow
// samples of a fragment (one test for all of them); for the single hard
// shadow it measured +-0 on C3.  ch = the exit copy every sample reads (sg =
// their sign pattern, fast path); true = lit.
__device__ __forceinline__ bool first_step_exit(const KernelArgs &a, const int8_t *ch, int sg, const Surf &g) {
    if (a.fc.max_steps < 1) return false;
    const int ax = g.nidx >> 1;
    const bool nneg = (g.nidx & 1) != 0;                   // face normal -e_a (render.vert:14-17)
    const bool spos = (sg >> ax) & 1;                      // sun toward +e_a
    // the in-face start: cell c + floor(f), fraction f - floor(f) (a quad-relative
    // v_fractPos spans the quad: f up to CHUNK); a fraction that rounds to 1
    // (f just below 0) fails the test and the samples march
    const float fl0 = floorf(g.f0), fl1 = floorf(g.f1), fl2 = floorf(g.f2);
    const float fj = ax == 0 ? g.f1 - fl1 : g.f0 - fl0, fk = ax == 2 ? g.f1 - fl1 : g.f2 - fl2;
    const bool ok = spos != nneg && fj >= 0.0f && fj < 1.0f && fk >= 0.0f && fk < 1.0f;
    const float nb = nneg ? -1.0f : 0.0f;
    const int x = (int)(g.c0 + (ax == 0 ? nb : fl0)), y = (int)(g.c1 + (ax == 1 ? nb : fl1)),
              z = (int)(g.c2 + (ax == 2 ? nb : fl2));                 // exact integers
    // the air cell is inside the padded copy (a face lies inside the grid or on its edge)
    const unsigned off = (unsigned)(x + a.SB) + (unsigned)a.SXp * (unsigned)(y + a.SB) + a.SXpYp * (unsigned)(z + a.SB);
    const float v = ok ? ld_fmt1(buf_rsrc(ch, kRsrcS8), off) : 0.0f;
    return v <= -2.0f && v >= -8.5f && (((int)(-1.0f - v) >> ax) & 1);   // face bits, not a doom code
}

// march(cell, fract, S.r) of render.frag:233 -> "lit" (step == MAX_STEPS, :234).
// S by value: the soft-shadow loop indexes sun_k[k] dynamically, and a
// reference into the kernel argument there made the compiler copy the whole
// KernelArgs (1.5 KB) to scratch.
// (the per-sample soft loop runs only where no cone copy serves every sample,
// so it never reads a doom code; it keeps the same form, which measured faster)
template <int DOOM = kDoomAfter>
__device__ __forceinline__ bool march_sun(const KernelArgs &a, const SunRay S, float c0, float c1, float c2, float f0,
                                          float f1, float f2, Counters &cnt) {
    if (S.fast && a.sunp) {
        // wave-uniform switch on the frame's sun signs: one specialised loop each
        const int sg = (S.sign[0] > 0.0f ? 1 : 0) | (S.sign[1] > 0.0f ? 2 : 0) | (S.sign[2] > 0.0f ? 4 : 0);
        // the frame's cone copy, else the octant's orthant copy, else the plain channel
        const int8_t *ch = a.sunc ? a.sunc
                         : a.sunx ? a.sunx + (size_t)sg * a.sunp_texels : S.up ? a.sunp : a.sunp + a.sunp_texels;
        switch (sg) {
        // (DOOM: the frame's cone copy may hold doom codes, launch_sun_doom)
#define VX_SG(K) case K: return march_pad<K, DOOM>(a, S, ch, c0, c1, c2, f0, f1, f2, cnt);
            VX_SG(0) VX_SG(1) VX_SG(2) VX_SG(3) VX_SG(4) VX_SG(5) VX_SG(6)
            default: return march_pad<7, DOOM>(a, S, ch, c0, c1, c2, f0, f1, f2, cnt);
#undef VX_SG
        }
    }
    const uint8_t *ch = S.up ? a.sun : a.sun + a.XYZ;
    return S.fast ? march_fast(a, S, ch, c0, c1, c2, f0, f1, f2, cnt)
                  : march_literal(a, S, ch, c0, c1, c2, f0, f1, f2, cnt);
}

// The offset (per axis, as exact fp32 integers) of the face with normal index
// nidx of cell (x, y, z) from the origin of the greedy quad covering it
// (a.qface: du along u = (ax+1)%3, dv along v = (ax+2)%3, 0 on the face axis);
// a cell without that face (never a primary hit) counts as its own origin,
// as in the oracle.
__device__ __forceinline__ void quad_offsets(const KernelArgs &a, int ax, int nidx, int x, int y, int z, float &o0,
                                             float &o1, float &o2) {
    unsigned q = a.qface[(size_t)nidx * a.XYZ + lin_index(a, x, y, z)];
    q = q == 0xFFFFu ? 0u : q;
    const float lo = (float)(q & 0xffu), hi = (float)(q >> 8);
    o0 = ax == 2 ? lo : (ax == 1 ? hi : 0.0f);
    o1 = ax == 0 ? lo : (ax == 2 ? hi : 0.0f);
    o2 = ax == 1 ? lo : (ax == 0 ? hi : 0.0f);
}

// The same offsets from a qcopy word (the octant's entry faces, 10 bits per
// face axis ax: du | dv << 5, launch_qcopy) -- chunks of at most 32 cells.
__device__ __forceinline__ void qcopy_offsets(uint32_t w, int ax, float &o0, float &o1, float &o2) {
    const unsigned q = (w >> (10 * ax)) & 0x3ffu;
    const float lo = (float)(q & 31u), hi = (float)(q >> 5);
    o0 = ax == 2 ? lo : (ax == 1 ? hi : 0.0f);
    o1 = ax == 0 ? lo : (ax == 2 ? hi : 0.0f);
    o2 = ax == 1 ? lo : (ax == 0 ? hi : 0.0f);
}

// ---------------- primary visibility ----------------
// The nearest front face of the greedy mesh of sdf.cpp:281-356 after back-face
// culling = the first step along the view ray that ENTERS a meshed cell (vis
// colour 1..21, vx_scene_create) from a cell of another colour.  Air (map.bin
// B = pal_size = 22, sdf.cpp:229-233) is never meshed (sdf.cpp:284), so a
// glass -> air step is no surface: glass blends over the next entry behind
// it.  The walk records the nearest glass entry and the surface behind it;
// a second glass entry before that surface sets `multi` (the panes' draw
// order then decides the pixel: k_render's stacked pass, glass_scan).  Box-exit
// stepping (oracle/vxo_render.c vxo_primary): in the ray octant's field copy
// the extents E of a cell say the box [c, c + E*s] ahead of it is air, so one
// step goes to the face where the ray leaves that box (E = 0: an exact DDA
// step).  Returns 0 sky, 1 surface, 2 glass + what is behind.
//
// The loop runs on camera-relative cells held as fp32 integers (exact: the
// host keeps |cam_cell| < 2^22), with x and y in packed-fp32 pairs:
//   h = c + hp (hp = 1 on a positive axis, 0 on a negative one), s = +-1;
//   far face    A  = c + (s > 0 ? E + 1 : -E) = fma(s, E, h)       (exact, per axis)
//   crossing    tb = (A - o) * iv                                   (= oracle)
//   exit axis   next h = A + s; others med3(floor(o + te*d) + hp, h, A)
// d == 0 is a positive axis with iv = +inf: A - o >= 1 - o > 0 (0 <= o < 1 is
// checked by vx_render), so tb = +inf exactly as the oracle's.  The box
// [c, c + E*s] lies ahead of the ray: h and A bracket it on every axis.
template <bool F32IDX>
__device__ __forceinline__ int primary(const KernelArgs &a, int oct, float d0, float d1, float d2, Surf &g0, Surf &g1,
                       Counters &cnt, float &t_hit, int &multi) {
    const FrameConsts &F = a.fc;
    const float o0 = F.cam_fract[0], o1 = F.cam_fract[1], o2 = F.cam_fract[2];
    const int cc0 = F.cam_cell[0], cc1 = F.cam_cell[1], cc2 = F.cam_cell[2];
    // iv = RN(1/d) (kInf for d = 0): rcp_ranged is exact for |d| in [2^-40,
    // 2^41) -- every lane of nearly every wave (|d| = O(1)); a wave with a lane
    // outside it (a zero or tiny component) takes the IEEE division
    // grid slabs (bounds per frame: FrameConsts::slab_lo/hi); a zero component
    // misses unless the camera lies inside that slab
    float iv0, iv1, iv2;
    float tlo = 0.0f, thi = kInf;
    bool miss = false;
    {
        const unsigned lo_b = 0x2B800000u, span = 0x54000000u - 0x2B800000u;   // 2^-40, 2^41
        const bool ok = (__float_as_uint(fabsf(d0)) - lo_b) < span && (__float_as_uint(fabsf(d1)) - lo_b) < span &&
                        (__float_as_uint(fabsf(d2)) - lo_b) < span;
        if (__builtin_expect(__ballot(!ok) == 0, 1)) {
            iv0 = rcp_ranged(d0); iv1 = rcp_ranged(d1); iv2 = rcp_ranged(d2);
            // no zero component: every slab crossing lo*iv, hi*iv is finite, and
            // the running max / min below is the general form's (a select of one
            // of its finite inputs; the sign of a zero t changes neither the
            // entry point o + t*d nor tlo < thi)
            const float a0 = F.slab_lo[0] * iv0, b0 = F.slab_hi[0] * iv0;
            const float a1 = F.slab_lo[1] * iv1, b1 = F.slab_hi[1] * iv1;
            const float a2 = F.slab_lo[2] * iv2, b2 = F.slab_hi[2] * iv2;
            tlo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(a0, b0), __builtin_fminf(a1, b1)),
                                  __builtin_fmaxf(__builtin_fminf(a2, b2), 0.0f));
            thi = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(a0, b0), __builtin_fmaxf(a1, b1)),
                                  __builtin_fmaxf(a2, b2));
        } else {
            iv0 = d0 != 0.0f ? 1.0f / d0 : kInf;
            iv1 = d1 != 0.0f ? 1.0f / d1 : kInf;
            iv2 = d2 != 0.0f ? 1.0f / d2 : kInf;
#define VX_SLAB(D, IV, I)                                                     \
            {                                                                 \
                const float lo = F.slab_lo[I], hi = F.slab_hi[I];             \
                const float t0 = lo * IV, t1 = hi * IV;                       \
                const bool sw = t0 > t1, nz = D != 0.0f;                      \
                tlo = nz ? gmax(tlo, sw ? t1 : t0) : tlo;                     \
                thi = nz ? gmin(thi, sw ? t0 : t1) : thi;                     \
                miss |= !nz && !(lo <= 0.0f && 0.0f < hi);                    \
            }
            VX_SLAB(d0, iv0, 0)
            VX_SLAB(d1, iv1, 1)
            VX_SLAB(d2, iv2, 2)
#undef VX_SLAB
        }
    }
    if (miss || !(tlo < thi)) return 0;
    // entry cell, camera-relative, as exact fp32 integers: floor, then clamped
    // into the grid (the former int convert + clamp; o + tlo*d is finite)
    const float cf0 = __builtin_amdgcn_fmed3f(floorf(o0 + tlo * d0), F.cell_lo[0], F.cell_hi[0]);
    const float cf1 = __builtin_amdgcn_fmed3f(floorf(o1 + tlo * d1), F.cell_lo[1], F.cell_hi[1]);
    const float cf2 = __builtin_amdgcn_fmed3f(floorf(o2 + tlo * d2), F.cell_lo[2], F.cell_hi[2]);
    const bool p0 = !(d0 < 0.0f), p1 = !(d1 < 0.0f), p2 = !(d2 < 0.0f);
    const int ip0 = p0, ip1 = p1, ip2 = p2;
    const float s0 = p0 ? 1.0f : -1.0f, s1 = p1 ? 1.0f : -1.0f, s2 = p2 ? 1.0f : -1.0f;
    const float hp0 = p0 ? 1.0f : 0.0f, hp1 = p1 ? 1.0f : 0.0f, hp2 = p2 ? 1.0f : 0.0f;
    float h0 = cf0 + hp0, h1 = cf1 + hp1, h2 = cf2 + hp2;
    // padded index of h: kray + hx + Xp*hy + XpYp*hz, mod 2^32 with 24-bit
    // signed products (|h| < 2^23)
    const uint32_t *ppad = a.prim + (size_t)oct * a.copy_texels;
    const int kray = (int)a.kcam - ip0 - a.Xp * ip1 - (int)a.XpYp * ip2;
    // F32IDX (a.prim_f32): the byte offset 4*(x + Xp*y) in fp32 (exact, <
    // 2^23), z by a 24-bit multiply-add, 32 bits from a.prim, all without
    // float -> int converts: the x/y sum is biased by 2^23 (its bit pattern is
    // 0x4B000000 + the sum) and z by 2^23 + 2^22 (|z| < 2^21: the low 24 bits
    // of the pattern are 2^22 + z); kz takes both constants back, mod 2^32
    const float kx4 = a.kx4 - (float)(4 * ip0) + 8388608.0f, ky = a.ky - (float)ip1;
    const float fXp4 = (float)(4 * a.Xp);
    const unsigned XpYp4 = 4u * a.XpYp;
    const unsigned kz = a.kz - XpYp4 * (unsigned)ip2 + (((unsigned)oct * a.copy_texels) << 2) - 0x4B000000u -
                        (XpYp4 << 22);
    // QSPEC (the fp32-index path, a.qcopy): every step also loads the cell's
    // entry-face quad offsets from a.qcopy at the same byte offset (the copy has
    // the prim layout), so the hit's offsets arrive with its colour instead of
    // by one more dependent load after the walk (quad_offsets)
    constexpr bool QSPEC = F32IDX && VX_QSPEC;
    uint32_t qw = 0, gqw = 0;
    auto fetch = [&](float x, float y, float z) -> uint32_t {
        if (F32IDX) {
            const float xy = __builtin_fmaf(fXp4, y + ky, __builtin_fmaf(4.0f, x, kx4));
            const unsigned off = __umul24(__float_as_uint(z + 12582912.0f), XpYp4) + __float_as_uint(xy) + kz;
            if (QSPEC) qw = ld_off(a.qcopy, off);
            return ld_off(a.prim, off);
        }
        const int idx = kray + (int)x + __mul24(a.Xp, (int)y) + __mul24((int)a.XpYp, (int)z);
        return ppad[(unsigned)idx];
    };
    uint32_t t = fetch(h0, h1, h2);
    cnt.prim_fetch++;
    cnt.prim_witers += once_per_wave(1u);          // the entry fetch is a wave iteration too
    int prev = t & 0xff;
    float E0 = cvt_f32_ubyte1(t), E1 = cvt_f32_ubyte2(t), E2 = cvt_f32_ubyte3(t);
    // gmark: the colour whose entry is "the first glass" -- glass until a glass
    // entry is recorded, then 256 (matches nothing).  The sentinel's colour
    // byte 0xFF is no vis colour (those are 0..21), so leaving the grid is an
    // entry that stops the walk.
    int gmark = kGlass, stop, col, mul = 0;
    float g0h = 0.0f, g1h = 0.0f, g2h = 0.0f, gt = 0.0f, te;
    float tb0, tb1, tb2;
    int gax = 0;
    const int cap = 4 * (a.X + a.Y + a.Z);
    int it = 0;
    do {
        // far face of the air box [c, c + E*s] ahead: A = h + s*E (exact)
        const float A0 = __builtin_fmaf(s0, E0, h0), A1 = __builtin_fmaf(s1, E1, h1), A2 = __builtin_fmaf(s2, E2, h2);
        tb0 = (A0 - o0) * iv0;
        tb1 = (A1 - o1) * iv1;
        tb2 = (A2 - o2) * iv2;
        te = __builtin_fminf(__builtin_fminf(tb0, tb1), tb2);
        const bool e0 = tb0 == te;
        const bool e1 = !e0 && tb1 == te;
        // other axes: floor(o + te*d) as h, clamped into the box, whose h
        // range is [h, A] (positive axis) or [A, h] (negative): med3(q, h, A)
        const float q0 = floorf(o0 + te * d0) + hp0;
        const float q1 = floorf(o1 + te * d1) + hp1;
        const float q2 = floorf(o2 + te * d2) + hp2;
        h0 = e0 ? A0 + s0 : __builtin_amdgcn_fmed3f(q0, h0, A0);
        h1 = e1 ? A1 + s1 : __builtin_amdgcn_fmed3f(q1, h1, A1);
        h2 = (!e0 && !e1) ? A2 + s2 : __builtin_amdgcn_fmed3f(q2, h2, A2);
        t = fetch(h0, h1, h2);
        cnt.prim_fetch += t >= kSentinel ? 0u : 1u;
        col = t & 0xff;
        // a face of the mesh: entering a meshed cell (vis colour != 0) from a
        // cell of another colour; air is never meshed (sdf.cpp:229-233,284)
        const bool enter = col != prev && col != 0;
        if (enter && col == kGlass) {                  // a glass entry (rare, divergent)
            if (gmark == kGlass) {                     // the first: blend over the next surface
                gmark = 256;
                g0h = h0; g1h = h1; g2h = h2; gt = te;
                gax = e0 ? 0 : (e1 ? 1 : 2);
                if (QSPEC) gqw = qw;
            } else {
                mul = 1;                               // a second pane in front of the surface
            }
        }
        stop = (enter && col != kGlass) ? 1 : 0;       // later glass entries are passed (the stacked pass blends them)
        asm volatile("" : "+v"(stop));                 // keep the lane flag in a VGPR
        prev = col;
        E0 = cvt_f32_ubyte1(t); E1 = cvt_f32_ubyte2(t); E2 = cvt_f32_ubyte3(t);
        cnt.prim_witers += once_per_wave(1u);      // counted in the loop: it stays a scalar
    } while (stop == 0 && ++it < cap);
    // opaque after the loop: otherwise the compiler keeps the loop's compare
    // masks (stop, tb == te) alive past it, at 3 SALU merges per mask per step
    asm volatile("" : "+v"(col), "+v"(stop), "+v"(tb0), "+v"(tb1), "+v"(te), "+v"(mul));
    multi = mul;
    if (stop == 0) cnt.cap_hit++;
    const bool hit = stop != 0 && t < kSentinel;
    const int hax = tb0 == te ? 0 : (tb1 == te ? 1 : 2);    // exit axis of the last step (ties x < y < z)
    // G-buffer records as the raster hands them over (render.vert:25-28):
    // v_cellPos = the origin of the greedy quad covering the face (the face
    // axis: its plane), v_fractPos = the hit point minus it, rounded once --
    // p - (c - off) with c the entered cell and off its offset in the quad
    // (a.qface; 0 with VX_FLAG_UNIT_GBUF: the unit cell's split p - c).  Both
    // tables are read before either record is formed.
    int nrec = 0;
    const bool gl = gmark != kGlass;
    const bool gpos = gax == 0 ? p0 : (gax == 1 ? p1 : p2);
    const bool hpos = hax == 0 ? p0 : (hax == 1 ? p1 : p2);
    const float gr0 = g0h - hp0, gr1 = g1h - hp1, gr2 = g2h - hp2;   // relative cells
    const float hr0 = h0 - hp0, hr1 = h1 - hp1, hr2 = h2 - hp2;
    float gq0 = 0.0f, gq1 = 0.0f, gq2 = 0.0f, hq0 = 0.0f, hq1 = 0.0f, hq2 = 0.0f;
    if (a.quad_gbuf) {
        if (QSPEC) {
            // the loaded entry-face word of the recorded step: 10 bits per face
            // axis (the glass record's only in a wave that has one: most have none)
            if (__ballot(gl) != 0) qcopy_offsets(gqw, gax, gq0, gq1, gq2);
            qcopy_offsets(qw, hax, hq0, hq1, hq2);
        } else {
            if (gl) quad_offsets(a, gax, 2 * gax + (gpos ? 1 : 0), (int)gr0 + cc0, (int)gr1 + cc1, (int)gr2 + cc2, gq0, gq1, gq2);
            if (hit) quad_offsets(a, hax, 2 * hax + (hpos ? 1 : 0), (int)hr0 + cc0, (int)hr1 + cc1, (int)hr2 + cc2, hq0, hq1, hq2);
        }
    }
    if (gl) {
        const float upf = gpos ? 0.0f : 1.0f;
        const float r0 = gr0 - gq0, r1 = gr1 - gq1, r2 = gr2 - gq2;   // quad origin (exact small integers)
        g0.id = 2;
        g0.color = kGlass;
        g0.nidx = 2 * gax + (gpos ? 1 : 0);
        g0.c0 = (r0 + F.cam_cell_f[0]) + (gax == 0 ? upf : 0.0f);      // exact integers
        g0.c1 = (r1 + F.cam_cell_f[1]) + (gax == 1 ? upf : 0.0f);
        g0.c2 = (r2 + F.cam_cell_f[2]) + (gax == 2 ? upf : 0.0f);
        g0.f0 = gax == 0 ? 0.0f : (o0 + gt * d0) - r0;
        g0.f1 = gax == 1 ? 0.0f : (o1 + gt * d1) - r1;
        g0.f2 = gax == 2 ? 0.0f : (o2 + gt * d2) - r2;
        nrec = 1;
    }
    if (hit) {
        Surf &h = gl ? g1 : g0;
        const float upf = hpos ? 0.0f : 1.0f;
        const float r0 = hr0 - hq0, r1 = hr1 - hq1, r2 = hr2 - hq2;
        h.id = col == kGlass ? 2 : 0;
        h.color = (int)col;
        h.nidx = 2 * hax + (hpos ? 1 : 0);
        h.c0 = (r0 + F.cam_cell_f[0]) + (hax == 0 ? upf : 0.0f);
        h.c1 = (r1 + F.cam_cell_f[1]) + (hax == 1 ? upf : 0.0f);
        h.c2 = (r2 + F.cam_cell_f[2]) + (hax == 2 ? upf : 0.0f);
        h.f0 = hax == 0 ? 0.0f : (o0 + te * d0) - r0;
        h.f1 = hax == 1 ? 0.0f : (o1 + te * d1) - r1;
        h.f2 = hax == 2 ? 0.0f : (o2 + te * d2) - r2;
        nrec++;
    }
    t_hit = te;
    return nrec;
}

// ---------------- glass in draw order (VX_FLAG_GLASS_ORDER) ----------------
// The reference draws the glass quads after every opaque one, in vertex.bin
// order, with depth test LESS and depth writes on, blending SRC_ALPHA
// (render.js:82-91, sdf.cpp:284,337).  face_key is that order for a glass
// face (oracle vxo_face_order): forChunkXYZ chunk, axis d, normal, slice, quad
// origin row j, column i; a face on an interior chunk plane is emitted first
// by the lower chunk (its slice CH-1).
__device__ __forceinline__ unsigned long long face_key(const KernelArgs &a, int x, int y, int z, int nidx,
                                                       unsigned q) {
    const int CH = a.chunk;
    const int d = nidx >> 1, normal = nidx & 1;
    const int cd_ = d == 0 ? x : (d == 1 ? y : z);                  // cell along d, u, v
    const int cu = d == 0 ? y : (d == 1 ? z : x);
    const int cv = d == 0 ? z : (d == 1 ? x : y);
    const int plane = cd_ + (normal ? 0 : 1);
    int kd = plane / CH, pd = plane % CH - 1;
    if (pd < 0) { kd -= 1; pd = CH - 1; }
    const int ou = cu - (int)(q & 0xffu), ov = cv - (int)(q >> 8);
    const int ku = ou / CH, kv = ov / CH;
    const int kx = d == 0 ? kd : (d == 1 ? kv : ku);
    const int ky = d == 1 ? kd : (d == 2 ? kv : ku);
    const int kz = d == 2 ? kd : (d == 0 ? kv : ku);
    const unsigned long long ny = (unsigned long long)((a.Y + CH - 1) / CH), nz = (unsigned long long)((a.Z + CH - 1) / CH);
    const unsigned long long S = (unsigned long long)CH + 1;
    const unsigned long long chunk = ((unsigned long long)kx * ny + (unsigned long long)ky) * nz + (unsigned long long)kz;
    return ((((chunk * 3 + (unsigned long long)d) * 2 + (unsigned long long)normal) * S + (unsigned long long)(pd + 1)) * S +
            (unsigned long long)(ov - kv * CH)) * S + (unsigned long long)(ou - ku * CH);
}

// One pass over the view ray's glass faces (the walk of primary visibility,
// scalar form like walk_reflect; oracle walk() with glass_layer 3): of the
// front-facing glass entries before the first opaque entry, the one drawn
// first after key `klast` (none: have_last false) among those nearer than
// tmax.  Returns false if there is none; else its G-buffer record
// (quad-relative unless a.quad_gbuf is 0), depth and key, and whether it is
// the ray's nearest pane.  No storage per pane, so a pixel blends every pane
// its ray crosses, as the raster does.  Its fetches repeat the primary walk's
// and are not counted again.
__device__ __forceinline__ bool glass_scan(const KernelArgs &a, float d0, float d1, float d2, bool have_last,
                                           unsigned long long klast, float tmax, Surf &h, float &t_out,
                                           unsigned long long &k_out, bool &nearest) {
    const FrameConsts &F = a.fc;
    const float o0 = F.cam_fract[0], o1 = F.cam_fract[1], o2 = F.cam_fract[2];
    const int cc0 = F.cam_cell[0], cc1 = F.cam_cell[1], cc2 = F.cam_cell[2];
    const float iv0 = d0 != 0.0f ? 1.0f / d0 : 0.0f, iv1 = d1 != 0.0f ? 1.0f / d1 : 0.0f,
                iv2 = d2 != 0.0f ? 1.0f / d2 : 0.0f;
    float tlo = 0.0f, thi = kInf;
    bool miss = false;
    auto slab = [&](float d, float iv, int i) {
        const float lo = F.slab_lo[i], hi = F.slab_hi[i];
        if (d != 0.0f) {
            float t0 = lo * iv, t1 = hi * iv;
            if (t0 > t1) { const float tt = t0; t0 = t1; t1 = tt; }
            tlo = gmax(tlo, t0);
            thi = gmin(thi, t1);
        } else if (!(lo <= 0.0f && 0.0f < hi)) {
            miss = true;
        }
    };
    slab(d0, iv0, 0); slab(d1, iv1, 1); slab(d2, iv2, 2);
    if (miss || !(tlo < thi)) return false;
    auto entry = [&](float o, float d, int cc, int dim) {
        const int c = f2i(floorf(o + tlo * d));
        return min(max(c, -cc), dim - cc - 1);
    };
    int c0 = entry(o0, d0, cc0, a.X), c1 = entry(o1, d1, cc1, a.Y), c2 = entry(o2, d2, cc2, a.Z);
    const int oct = (d0 < 0.0f ? 1 : 0) | (d1 < 0.0f ? 2 : 0) | (d2 < 0.0f ? 4 : 0);
    const uint32_t *pp = a.prim + (size_t)oct * a.copy_texels;
    auto fetch = [&](int x, int y, int z) -> uint32_t {
        return pp[(unsigned)(x + a.pad) + (unsigned)a.Xp * (unsigned)(y + a.pad) + a.XpYp * (unsigned)(z + a.pad)];
    };
    const int st0 = d0 > 0.0f ? 1 : -1, st1 = d1 > 0.0f ? 1 : -1, st2 = d2 > 0.0f ? 1 : -1;
    uint32_t t = fetch(c0 + cc0, c1 + cc1, c2 + cc2);
    int prev = t & 0xff, e0 = (int)((t >> 8) & 0xff), e1 = (int)((t >> 16) & 0xff), e2 = (int)(t >> 24);
    bool found = false, bfirst = false, first = true;
    int bx = 0, by = 0, bz = 0, bax = 0, bst = 0;
    unsigned bq = 0;
    float bt = 0.0f;
    unsigned long long bk = 0;
    const int cap = 4 * (a.X + a.Y + a.Z);
    for (int it = 0; it < cap; it++) {
        const float tb0 = d0 != 0.0f ? ((float)(c0 + (st0 > 0 ? e0 + 1 : -e0)) - o0) * iv0 : kInf;
        const float tb1 = d1 != 0.0f ? ((float)(c1 + (st1 > 0 ? e1 + 1 : -e1)) - o1) * iv1 : kInf;
        const float tb2 = d2 != 0.0f ? ((float)(c2 + (st2 > 0 ? e2 + 1 : -e2)) - o2) * iv2 : kInf;
        const int ax = (tb0 <= tb1 && tb0 <= tb2) ? 0 : (tb1 <= tb2 ? 1 : 2);
        const float te = ax == 0 ? tb0 : (ax == 1 ? tb1 : tb2);
        // the walk's crossings never decrease, and a pane qualifies only nearer
        // than tmax: past it no later entry can, so the scan ends there (each
        // scan of the chain walks only up to the last surface written)
        if (!(te < tmax)) break;
        auto side = [&](int c, float o, float d, int e) {
            const int v = f2i(floorf(o + te * d));
            const int lo = d < 0.0f ? c - e : c, hi = d < 0.0f ? c : c + e;
            return v < lo ? lo : (v > hi ? hi : v);
        };
        const int n0 = ax == 0 ? c0 + st0 * (e0 + 1) : side(c0, o0, d0, e0);
        const int n1 = ax == 1 ? c1 + st1 * (e1 + 1) : side(c1, o1, d1, e1);
        const int n2 = ax == 2 ? c2 + st2 * (e2 + 1) : side(c2, o2, d2, e2);
        c0 = n0; c1 = n1; c2 = n2;
        const int x = c0 + cc0, y = c1 + cc1, z = c2 + cc2;
        if ((unsigned)x >= (unsigned)a.X || (unsigned)y >= (unsigned)a.Y || (unsigned)z >= (unsigned)a.Z) break;
        t = fetch(x, y, z);
        const int col = t & 0xff;
        e0 = (int)((t >> 8) & 0xff); e1 = (int)((t >> 16) & 0xff); e2 = (int)(t >> 24);
        if (col != prev && col != 0) {             // a front face
            if (col != kGlass) break;              // the opaque surface: no glass behind it is drawn
            const int stp = ax == 0 ? st0 : (ax == 1 ? st1 : st2);
            const int nidx = 2 * ax + (stp > 0 ? 1 : 0);
            unsigned q = a.qface[(size_t)nidx * a.XYZ + lin_index(a, x, y, z)];
            q = q == 0xFFFFu ? 0u : q;
            const unsigned long long k = face_key(a, x, y, z, nidx, q);
            if ((!have_last || k > klast) && te < tmax && (!found || k < bk)) {
                found = true;
                bfirst = first;
                bk = k; bt = te; bq = q; bax = ax; bst = stp;
                bx = c0; by = c1; bz = c2;
            }
            first = false;
        }
        prev = col;
    }
    if (!found) return false;
    // the record (primary()'s rule): face axis on its plane, the others quad-relative
    unsigned q = a.quad_gbuf ? bq : 0u;
    const int lo = (int)(q & 0xffu), hi = (int)(q >> 8);
    const int of0 = bax == 2 ? lo : (bax == 1 ? hi : 0);
    const int of1 = bax == 0 ? lo : (bax == 2 ? hi : 0);
    const int of2 = bax == 1 ? lo : (bax == 0 ? hi : 0);
    const int up = bst > 0 ? 0 : 1;
    h.id = 2;
    h.color = kGlass;
    h.nidx = 2 * bax + (bst > 0 ? 1 : 0);
    h.c0 = (float)(bx - of0 + cc0 + (bax == 0 ? up : 0));
    h.c1 = (float)(by - of1 + cc1 + (bax == 1 ? up : 0));
    h.c2 = (float)(bz - of2 + cc2 + (bax == 2 ? up : 0));
    h.f0 = bax == 0 ? 0.0f : (o0 + bt * d0) - (float)(bx - of0);
    h.f1 = bax == 1 ? 0.0f : (o1 + bt * d1) - (float)(by - of1);
    h.f2 = bax == 2 ? 0.0f : (o2 + bt * d2) - (float)(bz - of2);
    t_out = bt;
    k_out = bk;
    nearest = bfirst;
    return true;
}

// ---------------- sampling ----------------
__device__ __forceinline__ void lin_axis(float coord, int size, int &i0, int &i1, float &w) {
    const float u = coord * (float)size - 0.5f;
    const float fl = floorf(u);
    w = u - fl;
    // AO coordinates are finite and far inside +-2^24 ((cell + fract) of a
    // fragment next to the grid): ivec3()'s NaN / saturation rules never
    // apply, so a plain convert is f2i here
    const int i = (int)fl;
    const int j = i + 1;
    i0 = min(max(i, 0), size - 1);
    i1 = min(max(j, 0), size - 1);
}

// sdf(ivec3, vec3) (render.frag:55-58) = min of trilinear R, G at LOD 0.
// The x-neighbours come in pairs (a.rg2): entry p of a row holds (R, G) of
// cells clamp(p - 1) and clamp(p), so the lerp's two x corners i0 =
// clamp(i), i1 = clamp(i + 1) are ONE typed load at p = clamp(i, -1, X - 1) + 1
// (i <= -1: (0, 0); i >= X - 1: (X - 1, X - 1); else (i, i + 1) -- exactly
// lin_axis's CLAMP_TO_EDGE pair).  Four 8_8_8_8 UNORM loads per sample
// instead of eight 8_8 ones, the same RN(b / 255) values, the same lerps.
__device__ __forceinline__ float sdf_lin(const KernelArgs &a, float c0, float c1, float c2, float f0, float f1, float f2) {
    const FrameConsts &F = a.fc;
    int y0, y1, z0, z1;
    float wx, wy, wz;
    const float ux = (c0 + f0) * F.sf[0] * (float)a.X - 0.5f;
    const float flx = floorf(ux);
    wx = ux - flx;
    const int px = min(max((int)flx, -1), a.X - 1) + 1;     // pair index (AO coordinates are far inside +-2^24)
    lin_axis((c1 + f1) * F.sf[1], a.Y, y0, y1, wy);
    lin_axis((c2 + f2) * F.sf[2], a.Z, z0, z1, wz);
    // one byte offset and two deltas (0 or one row / plane: the clamped corners
    // differ by at most one cell per axis)
    const unsigned row = (unsigned)a.X + 1u;
    const unsigned b00 = ((unsigned)px + __umul24(row, (unsigned)y0) + __umul24(__umul24(row, (unsigned)a.Y), (unsigned)z0)) << 2;
    const unsigned dy = __umul24((unsigned)(y1 - y0), 4u * row), dz = __umul24((unsigned)(z1 - z0), 4u * row * (unsigned)a.Y);
    const u32x4 rs = buf_rsrc(a.rg2, kRsrcRGBA);
    const f32x4 u00 = ld_fmt4(rs, b00), u10 = ld_fmt4(rs, b00 + dy);
    const f32x4 u01 = ld_fmt4(rs, b00 + dz), u11 = ld_fmt4(rs, b00 + dy + dz);
    float res[2];
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
        const float v00 = gmix(u00[ch], u00[2 + ch], wx);
        const float v01 = gmix(u10[ch], u10[2 + ch], wx);
        const float v10 = gmix(u01[ch], u01[2 + ch], wx);
        const float v11 = gmix(u11[ch], u11[2 + ch], wx);
        const float w0 = gmix(v00, v01, wy);
        const float w1 = gmix(v10, v11, wy);
        res[ch] = gmix(w0, w1, wz) * 255.0f;
    }
    return gmin(res[0], res[1]);
}

// REPEAT wrap of an integer-valued float onto [0, n), n a power of two:
// |fl| < 2^24 (every cloud lookup; a mountain lookup unless r1 ~ 0): fl - q*n
// is exact and in [0, n), i.e. (int)fl mod n = (int)fl & (n - 1).  The literal
// form only for the lanes outside that range (NaN included): floor(fl / n)
// with the IEEE quotient by n = 2^k, which is exactly fl * 2^-k (fl is 0 or
// |fl| >= 1: no underflow).
__device__ __forceinline__ int wrap_idx(float fl, int n) {
    int r = (int)fl & (n - 1);
    if (!(fabsf(fl) < 16777216.0f)) {
        // 1/n from n (exact: a power of two), not from a kernel argument: a
        // load sunk into this rare block would be tail-merged across the u/v
        // calls into a pointer phi -- a KernelArgs copy to scratch
        const float q = floorf(fl * (1.0f / (float)n));
        r = f2i(fl - q * (float)n) & (n - 1);
    }
    return r;
}

// fbm(p) = 1 - 2*texture(u_noise, p).a (render.frag:16-24), bilinear, REPEAT, LOD 0.
// The four A texels of the bilinear footprint are one typed load from the quad
// texture a.noise4 (entry (x, y) = A of (x, y), (x+1, y), (x, y+1), (x+1, y+1),
// REPEAT-wrapped when it was built): the same RN(b / 255) values.
__device__ __forceinline__ float fbm(const KernelArgs &a, float px, float py) {
    const int W = a.noise_w, H = a.noise_h;
    const float u = px * (float)W - 0.5f, v = py * (float)H - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const float wa = u - fu, wb = v - fv;
    const int x0 = wrap_idx(fu, W), y0 = wrap_idx(fv, H);
    const u32x4 rs = buf_rsrc(a.noise4, kRsrcRGBA);
    const f32x4 t = ld_fmt4(rs, (((unsigned)y0 << a.noise_lw) | (unsigned)x0) << 2);
    const float r0 = gmix(t.x, t.y, wa), r1 = gmix(t.z, t.w, wa);
    return 1.0f - 2.0f * gmix(r0, r1, wb);
}

// normalize3 of a vector whose length lies in [2^-40, 2^41) (exactly the IEEE result)
__device__ __forceinline__ void normalize3_ranged(float v0, float v1, float v2, float &o0, float &o1, float &o2) {
    const float l = sqrt_ranged(v0 * v0 + v1 * v1 + v2 * v2);   // callers: |v|^2 in [2^-80, 2^82)
    const float y = rcp_ranged(l);
    o0 = div_shared(v0, l, y); o1 = div_shared(v1, l, y); o2 = div_shared(v2, l, y);
}
__device__ __forceinline__ void normalize3(float v0, float v1, float v2, float &o0, float &o1, float &o2) {
    const float l = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
    const float y = 1.0f / l;       // one IEEE reciprocal, three exact corrections
    o0 = div_shared(v0, l, y); o1 = div_shared(v1, l, y); o2 = div_shared(v2, l, y);
}

// ---------------- render.frag main(), sky branch (render.frag:148-205) ----------------
__device__ __forceinline__ void shade_sky(const KernelArgs &a, float d0, float d1, float d2, float o[4],
                          Counters &cnt) {
    const FrameConsts &F = a.fc;
    float r0, r1, r2;
    normalize3(d0, d1, d2, r0, r1, r2);          // skybox modelled at infinity
    // reflect(rayDir, (-1,0,0)) (render.frag:155); only .z is read
    const float k = 2.0f * ((-1.0f * r0 + 0.0f * r1) + 0.0f * r2);
    const float refl_z = r2 - k * 0.0f;
    const float sunCol[3] = {1.4f, 1.0f, 0.5f};
    float sunFactor = gmax(0.0f, F.sun[0] * r0 + F.sun[1] * r1 + F.sun[2] * r2) - 1.0f;
    const float glow = vexp2(8.0f * sunFactor);
    sunFactor = vexp2(4000.0f * sunFactor) + 0.3f * glow;
    const float rz = sqrtf(gmax(0.0f, refl_z));
    float sky[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float atm = gmix(F.scatterCol[i], F.spaceCol[i], rz);
        sky[i] = gclamp(sunCol[i] * sunFactor + atm, 0.0f, 1.0f);
    }
    r2 = fabsf(r2);                                                               // :179
    if (F.flags & VX_FLAG_NO_CLOUDS) {
        o[0] = sky[0]; o[1] = sky[1]; o[2] = sky[2]; o[3] = 1.0f;
        return;
    }
    cnt.noise_px++;
    const float ct = F.cloudTime;
    const float den = sqrt_ranged(fabsf(r2) + 0.03f);   // in [0.03, 1.03]
    float sx, sy;                                                                 // :184
    {
        const float y = rcp_ranged(den);    // den = sqrt(|r2| + 0.03) in [0.17, 1.02]
        sx = div_shared(r0, den, y); sy = div_shared(r1, den, y);
    }
    sx = sx * 0.1f; sy = sy * 0.1f;
    const float sl = sqrtf(sqrtf(sx * sx + sy * sy));
    sx = sx * sl; sy = sy * sl;
    // render.frag:184-203 computes both the clouds and the mountains and keeps
    // one (:199-203).  The three samples that decide or feed the first step of
    // either (the mountain height, the two cloud warps) load together; then only
    // the kept branch's last sample is taken (the mountain factor or the cloud
    // factor): the same values, one noise sample less per sky pixel.
    const float n0 = fbm(a, 2.0f * sx + ct, 2.0f * sy + ct);
    const float n1 = fbm(a, 2.0f * sx - ct, 2.0f * sy - ct);
    const float mountainPos = r0 / r1;                                            // :195
    float mountainHeight = 1.0f - fbm(a, 0.3f * mountainPos, 0.3f * mountainPos);
    mountainHeight = mountainHeight / (vexp(0.3f * mountainPos * mountainPos) * 6.0f);
    if (mountainHeight > r2 && r1 > 0.0f && r2 > 0.0f) {
        const float mountainFactor = 2.0f - fbm(a, 2.0f * (mountainPos + r1), 2.0f * (mountainPos + r2));
        const float mt[3] = {0.7f, 0.8f, 0.7f};
        const float w = mountainFactor * r2;
#pragma unroll
        for (int i = 0; i < 3; i++) sky[i] = gmix(sky[i], sky[i] * mt[i], w);
    } else {
        sx = sx * (3.0f + n0); sy = sy * (3.0f + n1);
        sx = sx + F.skyOff[0];
        sy = sy + F.skyOff[1];
        const float cloudFactor = vexp2(6.0f * (fbm(a, sx + 2.0f * ct, sy + -9.0f * ct) - 1.0f));
        const float scf = sqrtf(cloudFactor);
#pragma unroll
        for (int i = 0; i < 3; i++) sky[i] = gmix(sky[i], gmix(sunCol[i], 0.8f, scf), cloudFactor);
    }
    o[0] = sky[0]; o[1] = sky[1]; o[2] = sky[2]; o[3] = 1.0f;
}

// ---------------- extensions (DESIGN.md §3 "Extensions") ----------------
// white(p) = 1 - 2*texture(u_noise, p).rgb (render.frag:16-21), bilinear REPEAT LOD 0.
// The bilinear footprint's four texels of each channel are one typed load
// from that channel's plane of the quad texture (a.noise4 planes 1..3).
__device__ __forceinline__ void white(const KernelArgs &a, float px, float py, float &w0, float &w1, float &w2) {
    const int W = a.noise_w, H = a.noise_h;
    const float u = px * (float)W - 0.5f, v = py * (float)H - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const float wa = u - fu, wb = v - fv;
    const int x0 = wrap_idx(fu, W), y0 = wrap_idx(fv, H);
    const unsigned off = (((unsigned)y0 << a.noise_lw) | (unsigned)x0) << 2, plane = ((unsigned)W * (unsigned)H) << 2;
    const u32x4 rs = buf_rsrc(a.noise4, kRsrcRGBA);
    const f32x4 tr = ld_fmt4(rs, off + plane), tg = ld_fmt4(rs, off + 2u * plane), tb = ld_fmt4(rs, off + 3u * plane);
    auto bil = [&](const f32x4 &t) { return 1.0f - 2.0f * gmix(gmix(t.x, t.y, wa), gmix(t.z, t.w, wa), wb); };
    w0 = bil(tr); w1 = bil(tg); w2 = bil(tb);
}

constexpr float kRoughScale = 0.00390625f;   // 1/256: 4 noise texels per voxel
constexpr float kRoughAmp = 0.1f;

// ---------------- render.frag main(), block branch (render.frag:148-176, 207-251) ----------------
// EXT: the extension instantiation (rough normals, soft shadows); has_ray:
// rayDir is given (a surface seen in a reflection) instead of the camera ray
// to the fragment (:154).  ray_out receives the rayDir used.
// The sun-facing factor of render.frag:228-229 with the (ext ROUGH) shading
// normal, exactly as shade_block computes it: the soft-shadow pass of k_render
// asks it first, to know which fragments march.
template <int EXT>
__device__ __forceinline__ float block_shade_factor(const KernelArgs &a, const Surf &g) {
    const FrameConsts &F = a.fc;
    const int ni = g.nidx;
    if (!(EXT && (F.flags & VX_FLAG_ROUGH))) return F.shadeFactor[ni];
    const float n0 = ni == 0 ? 1.0f : (ni == 1 ? -1.0f : 0.0f);
    const float n1 = ni == 2 ? 1.0f : (ni == 3 ? -1.0f : 0.0f);
    const float n2 = ni == 4 ? 1.0f : (ni == 5 ? -1.0f : 0.0f);
    const int ax = ni >> 1;
    const float u = ax == 0 ? g.c1 + g.f1 : g.c0 + g.f0;
    const float v = ax == 2 ? g.c1 + g.f1 : g.c2 + g.f2;
    float w0, w1, w2, m0, m1, m2;
    white(a, u * kRoughScale, v * kRoughScale, w0, w1, w2);
    normalize3_ranged(n0 + kRoughAmp * w0, n1 + kRoughAmp * w1, n2 + kRoughAmp * w2, m0, m1, m2);
    return F.sun[2] < 0.0f ? 0.0f : sqrtf(gmax(0.0f, (m0 * F.sun[0] + m1 * F.sun[1]) + m2 * F.sun[2]));
}

// lit_given >= 0 (EXT 2): the soft-shadow samples of this fragment were
// marched by k_render's wave pass, lit_given of them lit.
template <int EXT>
__device__ __forceinline__ void shade_block(const KernelArgs &a, const Surf &g, float o[4], Counters &cnt,
                            bool has_ray = false, float q0 = 0.0f, float q1 = 0.0f, float q2 = 0.0f,
                            float *ray_out = nullptr, int lit_given = -1) {
    const FrameConsts &F = a.fc;
    const int ni = g.nidx;
    const float n0 = ni == 0 ? 1.0f : (ni == 1 ? -1.0f : 0.0f);
    const float n1 = ni == 2 ? 1.0f : (ni == 3 ? -1.0f : 0.0f);
    const float n2 = ni == 4 ? 1.0f : (ni == 5 ? -1.0f : 0.0f);
    float r0, r1, r2;
    if (EXT && has_ray) {
        r0 = q0; r1 = q1; r2 = q2;
    } else {
        normalize3((g.c0 - F.cam_cell_f[0]) + (g.f0 - F.cam_fract[0]),        // exact cell differences
                   (g.c1 - F.cam_cell_f[1]) + (g.f1 - F.cam_fract[1]),
                   (g.c2 - F.cam_cell_f[2]) + (g.f2 - F.cam_fract[2]), r0, r1, r2);   // :154
    }
    if (EXT && ray_out) { ray_out[0] = r0; ray_out[1] = r1; ray_out[2] = r2; }
    // shading normal: geometric, or (ext ROUGH) jittered by white() noise
    float m0 = n0, m1 = n1, m2 = n2;
    const bool rough = EXT && (F.flags & VX_FLAG_ROUGH);
    if (rough) {
        cnt.rough++;
        const int ax = ni >> 1;
        const float u = ax == 0 ? g.c1 + g.f1 : g.c0 + g.f0;   // first in-face axis
        const float v = ax == 2 ? g.c1 + g.f1 : g.c2 + g.f2;   // second
        float w0, w1, w2;
        white(a, u * kRoughScale, v * kRoughScale, w0, w1, w2);
        // |n + 0.1 w| lies in [0.89, 1.11] (unit axis n, |w_i| <= 1): rcp_ranged is exact
        normalize3_ranged(n0 + kRoughAmp * w0, n1 + kRoughAmp * w1, n2 + kRoughAmp * w2, m0, m1, m2);
    }
    float base0 = 1.0f, base1 = 1.0f, base2 = 1.0f;
    if (g.color < 22) { base0 = kPalette[g.color][0]; base1 = kPalette[g.color][1]; base2 = kPalette[g.color][2]; }
    float amb0 = 1.0f, amb1 = 1.0f, amb2 = 1.0f;
    if (!(F.flags & VX_FLAG_NO_AO)) {                                                  // :223-225
        cnt.ao++;
        const float ambDist = sdf_lin(a, g.c0 + n0, g.c1 + n1, g.c2 + n2, g.f0, g.f1, g.f2);
        const float ambFactor = gmin(1.0f - sqrtf(ambDist), 0.8f);
        amb0 = gmix(1.0f, F.shadeCol[0], ambFactor);
        amb1 = gmix(1.0f, F.shadeCol[1], ambFactor);
        amb2 = gmix(1.0f, F.shadeCol[2], ambFactor);
    }
    float shadeFactor = F.shadeFactor[ni];                                             // :228-229
    if (rough)
        shadeFactor = F.sun[2] < 0.0f ? 0.0f : sqrtf(gmax(0.0f, (m0 * F.sun[0] + m1 * F.sun[1]) + m2 * F.sun[2]));
    if (shadeFactor > 0.0f && !(F.flags & VX_FLAG_NO_SHADOW)) {                        // :232-235
        // the exit copy every sample reads (sunc, or the octant's orthant copy
        // when they share one sign pattern): a first step into a marked block is lit
        const int sg0 = (F.sun_k[0].sign[0] > 0.0f ? 1 : 0) | (F.sun_k[0].sign[1] > 0.0f ? 2 : 0) |
                        (F.sun_k[0].sign[2] > 0.0f ? 4 : 0);
        const int8_t *xch = EXT != 2 || !a.sunp || !F.sun_k[0].fast ? nullptr
                          : a.sunc ? a.sunc
                          : a.sunx && F.soft_sg >= 0 ? a.sunx + (size_t)sg0 * a.sunp_texels : nullptr;
        const bool first_exit = xch && lit_given < 0 && first_step_exit(a, xch, sg0, g);
        if (EXT != 2) {                // the reference's hard shadow: one sun ray
            cnt.shadow_rays++;
            const bool lit = march_sun(a, F.sun_k[0], g.c0, g.c1, g.c2, g.f0, g.f1, g.f2, cnt);
            shadeFactor = shadeFactor * (lit ? 1.0f : 0.0f);
        } else if (lit_given >= 0) {   // marched by the wave pass (k_render)
            shadeFactor = shadeFactor * ((float)lit_given / (float)F.n_sun);
        } else if (first_exit) {       // every sample's first step lands in the marked block
            cnt.shadow_rays += (unsigned)F.n_sun;
            cnt.shadow_resolved += (unsigned)F.n_sun;
        } else {                       // ext soft shadows (EXT == 2): lit fraction of the sun samples
            int lit = 0;
            if (xch) {                 // one sign pattern, one copy: the shared-start loop
                switch (sg0) {
#define VX_SGS(K) case K: lit = march_soft<K>(a, xch, g.c0, g.c1, g.c2, g.f0, g.f1, g.f2, cnt); break;
                    VX_SGS(0) VX_SGS(1) VX_SGS(2) VX_SGS(3) VX_SGS(4) VX_SGS(5) VX_SGS(6)
                    default: lit = march_soft<7>(a, xch, g.c0, g.c1, g.c2, g.f0, g.f1, g.f2, cnt);
#undef VX_SGS
                }
            } else {
                for (int k = 0; k < F.n_sun; k++) {
                    cnt.shadow_rays++;
                    lit += march_sun(a, F.sun_k[k], g.c0, g.c1, g.c2, g.f0, g.f1, g.f2, cnt) ? 1 : 0;
                }
            }
            shadeFactor = shadeFactor * ((float)lit / (float)F.n_sun);
        }
    }
    const float l0 = F.shadeCol[0] + 0.4f * shadeFactor;                               // :238
    const float l1 = F.shadeCol[1] + 0.35f * shadeFactor;
    const float l2 = F.shadeCol[2] + 0.3f * shadeFactor;
    o[0] = base0; o[1] = base1; o[2] = base2; o[3] = 1.0f;
    if (F.quality > 0) {                                                               // :242-244
        float nc0 = F.normalCol[ni][0], nc1 = F.normalCol[ni][1], nc2 = F.normalCol[ni][2];
        if (rough) {                                                                   // :211-217 per fragment
            const float an0 = fabsf(m0), an1 = fabsf(m1), an2 = fabsf(m2);
            nc0 = (0.90f * an0 + 0.95f * an1) + 1.0f * an2;
            nc1 = (0.90f * an0 + 0.95f * an1) + 1.0f * an2;
            nc2 = (0.95f * an0 + 1.00f * an1) + 1.0f * an2;
            if (m2 < 0.0f) { nc0 = nc0 * 0.8f; nc1 = nc1 * 0.8f; nc2 = nc2 * 0.8f; }
        }
        o[0] = o[0] * ((nc0 * l0) * amb0);
        o[1] = o[1] * ((nc1 * l1) * amb1);
        o[2] = o[2] * ((nc2 * l2) * amb2);
    }
    if (g.id == 2) {                                                                   // :246-249
        const float k = 2.0f * ((m0 * r0 + m1 * r1) + m2 * r2);
        const float rz = sqrtf(gmax(0.0f, r2 - k * m2));
        o[3] = 0.8f * vexp2((r0 * m0 + r1 * m1) + r2 * m2);
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const float atm = gmix(F.scatterCol[i], F.spaceCol[i], rz);
            o[i] = o[i] * (0.2f * atm);
        }
    }
}

// ext REFLECT: octant-cube walk of a reflection ray B + o + t*d (B integer,
// 0 <= o < 1, start cell B + c) to the first colour change (oracle walk()
// with glass_layer = 0).  Scalar form of primary(): reflection rays are few.
// Returns 1 and the surface record, or 0 (sky: left the grid, or the start
// cell is outside it).
__device__ __forceinline__ int walk_reflect(const KernelArgs &a, int B0, int B1, int B2, float o0, float o1, float o2, float d0,
                            float d1, float d2, int c0, int c1, int c2, Surf &h, Counters &cnt) {
    // primary()'s stepping on exact fp32 cells relative to B, h = c + hp (hp = 1
    // on a positive axis, d = 0 counting positive), far face A = fma(s, E, h),
    // crossing (A - o) * iv (iv = +inf for d = 0: A - o > 0, so +inf, as the
    // integer form's explicit infinity), exit axis ties x < y < z, next h = A + s
    // on it and med3(floor(o + te*d) + hp, h, A) on the others (= the integer
    // form's clamp of floor(o + te*d) into [c, c+e] or [c-e, c]).  The octant
    // copy's sentinel border (colour 0xFF) marks leaving the grid: no fetch
    // counted, no hit, as the integer form's bounds test.
    const int oct = (d0 < 0.0f ? 1 : 0) | (d1 < 0.0f ? 2 : 0) | (d2 < 0.0f ? 4 : 0);
    const uint32_t *pp = a.prim + (size_t)oct * a.copy_texels;
    float iv0, iv1, iv2;
    {
        const unsigned lo_b = 0x2B800000u, span = 0x54000000u - 0x2B800000u;   // 2^-40, 2^41
        const bool ok = (__float_as_uint(fabsf(d0)) - lo_b) < span && (__float_as_uint(fabsf(d1)) - lo_b) < span &&
                        (__float_as_uint(fabsf(d2)) - lo_b) < span;
        if (__builtin_expect(__ballot(!ok) == 0, 1)) {
            iv0 = rcp_ranged(d0); iv1 = rcp_ranged(d1); iv2 = rcp_ranged(d2);
        } else {
            iv0 = d0 != 0.0f ? 1.0f / d0 : kInf;
            iv1 = d1 != 0.0f ? 1.0f / d1 : kInf;
            iv2 = d2 != 0.0f ? 1.0f / d2 : kInf;
        }
    }
    const bool p0 = !(d0 < 0.0f), p1 = !(d1 < 0.0f), p2 = !(d2 < 0.0f);
    const float s0 = p0 ? 1.0f : -1.0f, s1 = p1 ? 1.0f : -1.0f, s2 = p2 ? 1.0f : -1.0f;
    const float hp0 = p0 ? 1.0f : 0.0f, hp1 = p1 ? 1.0f : 0.0f, hp2 = p2 ? 1.0f : 0.0f;
    float h0 = (float)c0 + hp0, h1 = (float)c1 + hp1, h2 = (float)c2 + hp2;
    // element index of the padded cell B + pad + h - hp: the x + Xp*y part as the
    // bits of one exact fp32 fma biased by 2^23 (Xp*Yp < 2^23), z by a 24-bit
    // multiply of the biased bits (their low 24 bits are z)
    const float bx = (float)(B0 + a.pad) - hp0 + 8388608.0f, by = (float)(B1 + a.pad) - hp1,
                bz = (float)(B2 + a.pad) - hp2 + 8388608.0f;
    const float fXp = (float)a.Xp;
    auto fetch = [&]() -> uint32_t {
        const unsigned xy = __float_as_uint(__builtin_fmaf(h1 + by, fXp, h0 + bx)) - 0x4B000000u;
        return pp[xy + __umul24(__float_as_uint(h2 + bz), a.XpYp)];
    };
    uint32_t t = fetch();
    if (t >= kSentinel) return 0;
    cnt.refl_fetch++;
    int prev = t & 0xff;
    float E0 = cvt_f32_ubyte1(t), E1 = cvt_f32_ubyte2(t), E2 = cvt_f32_ubyte3(t);
    const int cap = 4 * (a.X + a.Y + a.Z);
    for (int it = 0; it < cap; it++) {
        const float A0 = __builtin_fmaf(s0, E0, h0), A1 = __builtin_fmaf(s1, E1, h1), A2 = __builtin_fmaf(s2, E2, h2);
        const float tb0 = (A0 - o0) * iv0, tb1 = (A1 - o1) * iv1, tb2 = (A2 - o2) * iv2;
        const float te = __builtin_fminf(__builtin_fminf(tb0, tb1), tb2);
        const bool e0 = tb0 == te;
        const bool e1 = !e0 && tb1 == te;
        const int ax = e0 ? 0 : (e1 ? 1 : 2);
        h0 = e0 ? A0 + s0 : __builtin_amdgcn_fmed3f(floorf(o0 + te * d0) + hp0, h0, A0);
        h1 = e1 ? A1 + s1 : __builtin_amdgcn_fmed3f(floorf(o1 + te * d1) + hp1, h1, A1);
        h2 = (!e0 && !e1) ? A2 + s2 : __builtin_amdgcn_fmed3f(floorf(o2 + te * d2) + hp2, h2, A2);
        t = fetch();
        if (t >= kSentinel) return 0;
        cnt.refl_fetch++;
        const int col = t & 0xff;
        E0 = cvt_f32_ubyte1(t); E1 = cvt_f32_ubyte2(t); E2 = cvt_f32_ubyte3(t);
        if (col != prev && col != 0) {                 // entering a meshed cell (air never is)
            const bool pos = ax == 0 ? p0 : (ax == 1 ? p1 : p2);
            const float r0 = h0 - hp0, r1 = h1 - hp1, r2 = h2 - hp2;   // relative cells (exact)
            h.color = col;
            h.id = col == kGlass ? 2 : 0;
            h.nidx = 2 * ax + (pos ? 1 : 0);
            h.c0 = ((float)B0 + r0) + (ax == 0 && !pos ? 1.0f : 0.0f);
            h.c1 = ((float)B1 + r1) + (ax == 1 && !pos ? 1.0f : 0.0f);
            h.c2 = ((float)B2 + r2) + (ax == 2 && !pos ? 1.0f : 0.0f);
            h.f0 = ax == 0 ? 0.0f : (o0 + te * d0) - r0;
            h.f1 = ax == 1 ? 0.0f : (o1 + te * d1) - r1;
            h.f2 = ax == 2 ? 0.0f : (o2 + te * d2) - r2;
            return 1;
        }
        prev = col;
    }
    cnt.cap_hit++;
    return 0;
}

// ext REFLECT: colour seen along the mirror reflection at glass record gl
// (rd = the camera rayDir at the fragment; R = rd with the face-axis
// component negated = reflect(rd, n) exactly), oracle reflect_color().
template <int EXT>
__device__ __forceinline__ void reflect_color(const KernelArgs &a, const Surf &gl, const float rd[3], float out[3],
                              Counters &cnt) {
    const int ax = gl.nidx >> 1;
    const float R0 = ax == 0 ? -rd[0] : rd[0], R1 = ax == 1 ? -rd[1] : rd[1], R2 = ax == 2 ? -rd[2] : rd[2];
    const float fl0 = floorf(gl.f0), fl1 = floorf(gl.f1), fl2 = floorf(gl.f2);
    const int B0 = (int)(ax == 0 ? gl.c0 : gl.c0 + fl0);                // exact integers
    const int B1 = (int)(ax == 1 ? gl.c1 : gl.c1 + fl1);
    const int B2 = (int)(ax == 2 ? gl.c2 : gl.c2 + fl2);
    const float o0 = ax == 0 ? 0.0f : gl.f0 - fl0;
    const float o1 = ax == 1 ? 0.0f : gl.f1 - fl1;
    const float o2 = ax == 2 ? 0.0f : gl.f2 - fl2;
    const int s0 = ax == 0 ? (R0 > 0.0f ? 0 : -1) : 0;
    const int s1 = ax == 1 ? (R1 > 0.0f ? 0 : -1) : 0;
    const int s2 = ax == 2 ? (R2 > 0.0f ? 0 : -1) : 0;
    cnt.refl_rays++;
    Surf h;
    float rgba[4];
    if (walk_reflect(a, B0, B1, B2, o0, o1, o2, R0, R1, R2, s0, s1, s2, h, cnt))
        shade_block<EXT>(a, h, rgba, cnt, true, R0, R1, R2);
    else
        shade_sky(a, R0, R1, R2, rgba, cnt);
    out[0] = rgba[0]; out[1] = rgba[1]; out[2] = rgba[2];
}

// Glass in draw order (render.js:82-91; DESIGN.md §5 "Glass"): the reference
// draws the glass quads after every opaque one, in vertex.bin order, depth test
// LESS with writes on, SRC_ALPHA blending -- a pane is blended iff it is
// nearer than the last surface written when its quad is drawn.  The nearest
// pane P1 of a ray is nearer than every other surface, so it always passes and
// is always the last pane blended: the pixel is P1 over dst', where dst' is the
// surface behind the panes with the panes drawn before P1 (key order, each
// nearer than the last one written) blended over it.  glass_chain turns dst
// (the surface behind, depth its depth) into dst'; k_render's one-blend path
// then blends P1 (g[0]) over it.  It runs for pixels whose ray crosses two or
// more panes in front of its surface (primary()'s multi): with one pane dst' =
// dst.
template <int XE>
__device__ __forceinline__ void glass_chain(const KernelArgs &a, float d0, float d1, float d2, float dst[4], float depth,
                                            Counters &cnt) {
    const FrameConsts &F = a.fc;
    unsigned long long klast = 0;
    bool have_last = false, nearest = false;
    Surf cur;
    float tc;
    unsigned long long kc;
    while (glass_scan(a, d0, d1, d2, have_last, klast, depth, cur, tc, kc, nearest) && !nearest) {
        depth = tc; klast = kc; have_last = true;
        float src[4], rd[3];
        shade_block<XE>(a, cur, src, cnt, false, 0.0f, 0.0f, 0.0f, rd);
        if (XE && (F.flags & (VX_FLAG_REFLECT | VX_FLAG_REFLECT_ALL))) {   // ext REFLECT: panes mirror
            float refl[3];
            reflect_color<XE>(a, cur, rd, refl, cnt);
            const int ax = cur.nidx >> 1;
            const float cs = gmin(fabsf(ax == 0 ? rd[0] : (ax == 1 ? rd[1] : rd[2])), 1.0f);
            const float x = 1.0f - cs, x2 = x * x;
            const float fr = 0.04f + 0.96f * ((x2 * x2) * x);
#pragma unroll
            for (int i = 0; i < 3; i++) src[i] = src[i] + fr * refl[i];
        }
        blend_canvas(src, dst, dst);        // the pane over the canvas (render.js:84-86)
    }
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned v) {
    unsigned long long s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

__device__ __forceinline__ uint32_t pack_rgba8(const float rgba[4]) {
    uint32_t pk = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) pk |= (uint32_t)(gclamp(rgba[i], 0.0f, 1.0f) * 255.0f + 0.5f) << (8 * i);
    return pk;
}

template <int FMT>
__device__ __forceinline__ void store_pixel(const KernelArgs &a, size_t idx, const float rgba[4]) {
    if (FMT == VX_PIXEL_RGBA32F)
        reinterpret_cast<float4 *>(a.out)[idx] = make_float4(rgba[0], rgba[1], rgba[2], rgba[3]);
    else
        reinterpret_cast<uint32_t *>(a.out)[idx] = pack_rgba8(rgba);
}

// output index of pixel (px, py), at (x, y) inside tile k of a tiled launch:
// compact tile-major (tile k at k * tile_h * pitch, rows pitch apart) or,
// tile_inplace, the pixel's own place in the w-wide frame
template <bool TILED>
__device__ __forceinline__ size_t out_index(const KernelArgs &a, int k, int x, int y, int px, int py) {
    if (TILED && !a.tile_inplace) return (size_t)k * a.tile_h * a.tile_pitch + (size_t)y * a.tile_pitch + x;
    return (size_t)py * a.w + px;
}

// view ray of pixel (px, py): nx = (2px+1)/w - 1, ny = 1 - (2py+1)/h with exact quotients
__device__ __forceinline__ void view_ray(const FrameConsts &F, int px, int py, float &d0, float &d1, float &d2) {
    const float nx = div_const((float)(2 * px + 1), F.fw, F.rcp_w) - 1.0f;
    const float ny = 1.0f - div_const((float)(2 * py + 1), F.fh, F.rcp_h);
    d0 = (F.fwd[0] + nx * F.right[0]) + ny * F.up[0];
    d1 = (F.fwd[1] + nx * F.right[1]) + ny * F.up[1];
    d2 = (F.fwd[2] + nx * F.right[2]) + ny * F.up[2];
}

__device__ __forceinline__ void primary_only_colour(int n, const Surf &g0, float rgba[4]) {
    const int pc = n == 0 ? 0 : g0.color;
    rgba[0] = pc < 22 ? kPalette[pc][0] : 1.0f;
    rgba[1] = pc < 22 ? kPalette[pc][1] : 1.0f;
    rgba[2] = pc < 22 ? kPalette[pc][2] : 1.0f;
    rgba[3] = 1.0f;
}

// ---------------- 2D mode (u_quality = 0) ----------------
// drawScene binds the vertex2d mesh when mode == MODE_2D and sets u_quality = 0
// (render.js:278, 287): the footprint quads of sdf.cpp:362-401 on the z = 0
// plane (vert2d: normal byte 0 -> v_normal = (1, 0, 0), render.vert:16; id 2
// for glass), front-facing from above (tri2d winding, culled from below,
// render.js:88-91), over the clear colour (0.9, 0.9, 0.9) (render.js:274-275:
// from the second frame on).  render.frag with u_quality = 0 outputs the
// palette colour (:241-244); glass: alpha 0.8 exp2(dot(rayDir, n)), rgb *=
// 0.2 atmCol (:246-249), blended over the clear colour.  The march and the
// AO sample the reference also runs there do not reach the output (:244): not
// run.  Oracle: vxo_render.c shade_2d.
constexpr float kClear2d = 0.9f;
__device__ __forceinline__ void shade_2d(const KernelArgs &a, float d0, float d1, float d2, float rgba[4], Counters &cnt,
                         unsigned &n_sky, unsigned &n_block, unsigned &n_glass) {
    const FrameConsts &F = a.fc;
    rgba[0] = rgba[1] = rgba[2] = kClear2d;
    rgba[3] = 1.0f;
    const float zr = (float)(0 - F.cam_cell[2]) - F.cam_fract[2];      // the plane, camera-relative
    int c = 0, x = 0, y = 0;
    float hx = 0.0f, hy = 0.0f;
    if (zr < 0.0f && d2 < 0.0f) {                                       // camera above, ray going down
        const float t = zr / d2;
        hx = F.cam_fract[0] + t * d0;
        hy = F.cam_fract[1] + t * d1;
        x = F.cam_cell[0] + f2i(floorf(hx));
        y = F.cam_cell[1] + f2i(floorf(hy));
        if ((unsigned)x < (unsigned)a.X && (unsigned)y < (unsigned)a.Y) {
            c = (int)a.fp2d[2 * ((size_t)y * a.X + x)];
            cnt.prim_fetch++;
        }
    }
    if (c == 0) {
        n_sky = 1;
        return;
    }
    const uint32_t org = a.fp2d[2 * ((size_t)y * a.X + x) + 1];
    const int x0 = (int)(org & 0xffffu), y0 = (int)(org >> 16);
    const float pc0 = kPalette[c][0], pc1 = kPalette[c][1], pc2 = kPalette[c][2];
    if (c != kGlass) {
        n_block = 1;
        rgba[0] = pc0; rgba[1] = pc1; rgba[2] = pc2;
        return;
    }
    n_glass = 1;
    // v_cellPos = the quad corner (x0, y0, 0), v_fractPos = hit - corner (render.vert:27-28)
    const float f0 = (float)(F.cam_cell[0] - x0) + hx, f1 = (float)(F.cam_cell[1] - y0) + hy;
    float r0, r1, r2;
    normalize3((float)(x0 - F.cam_cell[0]) + (f0 - F.cam_fract[0]), (float)(y0 - F.cam_cell[1]) + (f1 - F.cam_fract[1]),
               (float)(0 - F.cam_cell[2]) + (0.0f - F.cam_fract[2]), r0, r1, r2);     // render.frag:154
    const float k = 2.0f * ((1.0f * r0 + 0.0f * r1) + 0.0f * r2);                  // reflect(rayDir, n)
    const float rz = sqrtf(gmax(0.0f, r2 - k * 0.0f));
    float src[4];
    src[3] = 0.8f * vexp2((r0 * 1.0f + r1 * 0.0f) + r2 * 0.0f);
    const float pc[3] = {pc0, pc1, pc2};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float atm = gmix(F.scatterCol[i], F.spaceCol[i], rz);
        src[i] = pc[i] * (0.2f * atm);
    }
    blend_canvas(src, rgba, rgba);          // over the clear colour in the canvas
}

// Lane = pixel, wave = 8x8 tile, workgroup = 32x8 pixels.
// EXT: 0 = v1 (the reference's shader), 1 = extensions (REFLECT, ROUGH,
// REFLECT_ALL) with the hard shadow, 2 = extensions with soft shadows (n sun
// samples), 3 = 2 with the first surface's samples marched by the pooled wave
// pass (VX_FLAG_SOFT_POOL), 4 = 3 with LDS brick staging (VX_FLAG_SOFT_BRICK),
// 5 / 6 = 1 / 2 with glass in draw order (VX_FLAG_GLASS_ORDER).  Each
// instantiation carries only its own code and registers; soft shadows in a
// kernel of their own also keep the sun_k[0] / sun_k[k] addresses apart (a
// pointer phi between them makes the compiler copy KernelArgs to scratch).
// Occupancy: 8 waves/SIMD needs <= 64 VGPRs and <= 80 SGPRs (8 256-thread
// blocks per CU, MI355X_MICROARCH.md "Residency"); every instantiation is held
// to that budget explicitly (left alone the EXT ones take 66 VGPRs + 100 SGPRs
// and run at 6 waves/SIMD).
#ifndef VX_OCC_ATTR
#define VX_OCC_ATTR __attribute__((amdgpu_waves_per_eu(8, 8), amdgpu_num_sgpr(80)))
#endif
// Workgroup = 256 threads = four 8x8-pixel waves side by side: a 32x8 pixel
// block.  Each wave stores its own 8x8 tile (32-B row pieces): staging the
// block in LDS for whole 128-B rows needs a block barrier, and the waves of a
// block finish at very different times (round 5: per-wave stores C3 full
// quality -1.7 %, v1 -1.1 %, C5 -0.5..-1.2 %, profiles/r05_ab_wave_store_*.txt).
constexpr int kBX = 32;                    // block width in pixels
constexpr int kBY = kWG / kBX;             // block height
constexpr int kBXS = 5;                    // log2(kBX)
constexpr int kBYS = 3;                    // log2(kBY)
constexpr int kWX = kBX / 8;               // waves per block row
static_assert(kBX == 1 << kBXS && kBY == 1 << kBYS, "block shape");

// F32IDX: the fp32 primary index (a.prim_f32) -- a kernel of its own: two
// inlined primary() copies in one kernel make the compiler copy KernelArgs
// to scratch.
template <int FMT, bool STATS, bool TILED, int EXT, bool F32IDX>
__global__ __launch_bounds__(kWG) VX_OCC_ATTR
void k_render(KernelArgs a) {
    // the shading instantiation: EXT 3/4 shade as 2; 5/6 are 1/2 with the general
    // shading block (glass in draw order, REFLECT_ALL)
    constexpr int XE = EXT == 5 ? 1 : (EXT >= 2 ? 2 : EXT);
    constexpr bool kPool = EXT == 3 || EXT == 4;   // VX_FLAG_SOFT_POOL: the pooled wave pass
    constexpr bool kBrick = EXT == 4;              // VX_FLAG_SOFT_BRICK: + LDS brick staging
    constexpr bool kGeneral = EXT >= 5;            // VX_FLAG_GLASS_ORDER / VX_FLAG_REFLECT_ALL
    // pooled pass: the frame's sun samples (r, |r|, RN(1/|r|)) and per wave
    // the compacted marching fragments' start (fract, cell) and lit counts
    __shared__ float4 s_sunk[kPool ? 3 * VX_MAX_SHADOW_SAMPLES : 1];
    __shared__ float4 s_pf[kPool ? kWG : 1];
    __shared__ float4 s_pc[kPool ? kWG : 1];
    __shared__ int s_plit[kPool ? kWG : 1];
    __shared__ int s_brick[kBrick ? 4 * 4 * 128 : 1];      // per wave: 4 bricks of 8x8x8 int8 (dwords)
    if (kPool) {
        for (int k = 0; k < a.fc.n_sun; k++) {          // uniform k: scalar loads of the kernel argument
            if (threadIdx.x == k) {
                const SunRay &Sk = a.fc.sun_k[k];
                s_sunk[3 * k] = make_float4(Sk.r[0], Sk.r[1], Sk.r[2], 0.0f);
                s_sunk[3 * k + 1] = make_float4(Sk.abs[0], Sk.abs[1], Sk.abs[2], 0.0f);
                s_sunk[3 * k + 2] = make_float4(Sk.rcp[0], Sk.rcp[1], Sk.rcp[2], 0.0f);
            }
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lx = ((wave % kWX) << 3) | (lane & 7);
    const int ly = ((wave / kWX) << 3) | (lane >> 3);
    int ox, oy, tx0 = 0, ty0 = 0, tile_k = 0;
    if (TILED) {
        // tiles of tile_w x tile_h pixels (multiples of the block), tile k of the
        // list at k * tile_w * tile_h in the compact output (or at its own
        // place in a w-wide frame: tile_inplace)
        // (launch_render_ext: a grid of (block columns, block rows, tiles), so no
        // integer division; a list of more than 65535 tiles takes a 1-D grid)
        const int perx = a.tile_w >> kBXS;
        int sx, sy;
        if (gridDim.y > 1 || gridDim.z > 1) {
            tile_k = blockIdx.z;
            sx = blockIdx.x;
            sy = blockIdx.y;
        } else {
            const int bpt = perx * (a.tile_h >> kBYS);
            tile_k = blockIdx.x / bpt;
            const int sub = blockIdx.x % bpt;
            sx = sub % perx;
            sy = sub / perx;
        }
        const int tid = a.tile_ids[tile_k];
        tx0 = sx << kBXS;
        ty0 = sy << kBYS;
        if (a.tiles_x == 1) {               // bands (vx_render_bands): one tile spans the row
            ox = tx0;
            oy = tid * a.tile_h + ty0;
        } else {
            ox = (tid % a.tiles_x) * a.tile_w + tx0;
            oy = (tid / a.tiles_x) * a.tile_h + ty0;
        }
    } else {
        ox = blockIdx.x << kBXS;
        // diagnostics (VX_FLAG_ROWS_BOTTOM_UP): block rows dispatched bottom row first
        oy = ((a.fc.flags & VX_FLAG_ROWS_BOTTOM_UP) ? gridDim.y - 1 - blockIdx.y : blockIdx.y) << kBYS;
    }
    const int px = ox + lx, py = oy + ly;
    const bool inframe = px < a.w && py < a.h;
    // the tiled launch's output index, formed once: only it stays live across the
    // shading instead of the tile's coordinates (the host keeps it below 2^32)
    const unsigned toidx = TILED ? (unsigned)out_index<TILED>(a, tile_k, tx0 + lx, ty0 + ly, px, py) : 0u;
    const FrameConsts &F = a.fc;
    Counters cnt = {};
#ifdef VX_BLOCK_TIMING
    // diagnostics build only (tools/block_times.py): the block's start and end
    // on the 100 MHz constant clock
    const unsigned long long t_blk0 = __builtin_amdgcn_s_memrealtime();
#endif
    unsigned n_sky = 0, n_block = 0, n_glass = 0, n_px = 0;
    // The pooled pass deals work over all 64 lanes of a wave, so there every
    // lane runs: a lane off the frame (a partial edge wave) takes the nearest
    // in-frame pixel's ray, marches for the others, and neither counts its own
    // primary work nor shades nor stores.
    if (kPool || inframe) {
        float d0, d1, d2;
        view_ray(F, kPool ? min(px, a.w - 1) : px, kPool ? min(py, a.h - 1) : py, d0, d1, d2);
        // the field copy of this ray's octant (zero components count positive)
        const int oct = (d0 < 0.0f ? 1 : 0) | (d1 < 0.0f ? 2 : 0) | (d2 < 0.0f ? 4 : 0);
        Surf g[2];
        float t_hit;
        int multi;
        const int n = primary<F32IDX>(a, oct, d0, d1, d2, g[0], g[1], cnt, t_hit, multi);
        // glass in draw order (render.js:82-91): the nearest pane is blended last,
        // over what is behind it; a ray that crosses two or more panes in front
        // of its surface first blends the panes drawn before the nearest one over
        // that (glass_chain), with one pane there are none.  VX_FLAG_GLASS_SINGLE:
        // the nearest pane only (diagnostic).  The general modes (VX_FLAG_GLASS_ORDER,
        // REFLECT_ALL) are instantiations of their own (EXT 5, 6), so their mirror
        // walk per surface adds no code or registers here.
        const bool order = !(F.flags & VX_FLAG_GLASS_SINGLE);
        const bool stacked = multi != 0 && order && !(F.flags & VX_FLAG_PRIMARY_ONLY) && inframe;
        int lit0 = -1;
        if (kPool && !inframe) cnt = Counters{};
        if (kPool && F.soft_sg >= 0 && a.sunp) {
            // Pooled soft shadows: the fragments of the wave that march are
            // compacted by a ballot, and each pass deals 64 / G of them with
            // G = 2^soft_lg lanes per fragment, lane k of a group marching sample
            // k.  A wave load then touches the few cache lines around 64 / G
            // surface points instead of one line per pixel, and lanes whose own
            // pixel does not march (sky, faces turned from the sun) march for
            // the others.  Same exact march_pad, lit counted per fragment in LDS.
            // (a glass pixel in draw order may shade other panes first: it marches in shade_block)
            const bool need = inframe && n != 0 && !(F.flags & (VX_FLAG_PRIMARY_ONLY | VX_FLAG_NO_SHADOW)) &&
                              block_shade_factor<XE>(a, g[0]) > 0.0f;
            const unsigned long long mask = __ballot(need);
            if (mask) {
                const int wb = threadIdx.x & ~63;                // this wave's 64 slots
                const int nf = __popcll(mask);
                const int slot = __popcll(mask & ((1ull << lane) - 1ull));
                if (need) {
                    s_pf[wb + slot] = make_float4(g[0].f0, g[0].f1, g[0].f2, 0.0f);
                    s_pc[wb + slot] = make_float4(g[0].c0, g[0].c1, g[0].c2, 0.0f);
                    s_plit[wb + slot] = 0;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const int lg = F.soft_lg;
                const int k = lane & ((1 << lg) - 1);
                const bool klane = k < F.n_sun;
                SunRay S;                                         // this lane's sample (per-lane values)
                const float4 q0 = s_sunk[3 * k], q1 = s_sunk[3 * k + 1], q2 = s_sunk[3 * k + 2];
                S.r[0] = q0.x; S.r[1] = q0.y; S.r[2] = q0.z;
                S.abs[0] = q1.x; S.abs[1] = q1.y; S.abs[2] = q1.z;
                S.rcp[0] = q2.x; S.rcp[1] = q2.y; S.rcp[2] = q2.z;
                const int8_t *ch = a.sunc ? a.sunc
                                         : a.sunx ? a.sunx + (size_t)F.soft_sg * a.sunp_texels
                                         : F.sun_k[0].up ? a.sunp : a.sunp + a.sunp_texels;
                // EXT 4 is launched only when the bricks fit (launch_render): <= 4 fragments per
                // pass, 4-byte aligned rows, a border of >= 9 cells around the grid
                const int sgv = F.soft_sg;
                const int bx = (sgv & 1) ? 0 : 4, by = (sgv & 2) ? 1 : 6, bz = (sgv & 4) ? 1 : 6;
                const int fpp = 64 >> lg;
                for (int base = 0; base < nf; base += fpp) {          // wave-uniform passes
                    const int fs = base + (lane >> lg);
                    if (kBrick) {
                        // stage the pass's bricks: 4 x 64 rows x 2 dwords, 8 dword loads per lane
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        int *wbrick = s_brick + (wb >> 6) * 512;
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const int d = lane + 64 * j, bi = d >> 7, row = (d & 127) >> 1, half = d & 1;
                            const int fb = min(base + bi, nf - 1);
                            const float4 pc = s_pc[wb + fb];
                            const float4 pf = s_pf[wb + fb];     // anchor: the start's unit cell c + floor(f)
                            const int ox = ((int)(pc.x + floorf(pf.x)) + a.SB - bx) & ~3,
                                      oy = (int)(pc.y + floorf(pf.y)) + a.SB - by, oz = (int)(pc.z + floorf(pf.z)) + a.SB - bz;
                            const size_t off = (size_t)(unsigned)ox + 4u * half +
                                               (size_t)(unsigned)a.SXp * (unsigned)(oy + (row & 7)) +
                                               (size_t)a.SXpYp * (unsigned)(oz + (row >> 3));
                            wbrick[d] = *reinterpret_cast<const int *>(ch + off);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                    }
                    if (klane && fs < nf) {
                        const float4 pf = s_pf[wb + fs];
                        const float4 pc = s_pc[wb + fs];
                        cnt.shadow_rays++;
                        bool lit;
                        if constexpr (kBrick) {
                            const int8_t *br = reinterpret_cast<const int8_t *>(s_brick + (wb >> 6) * 512) +
                                               512 * (lane >> lg);
                            const int ox = ((int)(pc.x + floorf(pf.x)) + a.SB - bx) & ~3,
                                      oy = (int)(pc.y + floorf(pf.y)) + a.SB - by, oz = (int)(pc.z + floorf(pf.z)) + a.SB - bz;
                            switch (sgv) {
#define VX_SGB(K) case K: lit = march_brick<K>(a, S, ch, br, ox, oy, oz, pc.x, pc.y, pc.z, pf.x, pf.y, pf.z, \
                                               cnt); break;
                                VX_SGB(0) VX_SGB(1) VX_SGB(2) VX_SGB(3) VX_SGB(4) VX_SGB(5) VX_SGB(6)
                                default: lit = march_brick<7>(a, S, ch, br, ox, oy, oz, pc.x, pc.y, pc.z, pf.x, pf.y,
                                                              pf.z, cnt);
#undef VX_SGB
                            }
                        } else {
                            switch (sgv) {
#define VX_SGP(K) case K: lit = march_pad<K, kDoomAfter>(a, S, ch, pc.x, pc.y, pc.z, pf.x, pf.y, pf.z, \
                                                   cnt); break;
                                VX_SGP(0) VX_SGP(1) VX_SGP(2) VX_SGP(3) VX_SGP(4) VX_SGP(5) VX_SGP(6)
                                default: lit = march_pad<7, kDoomAfter>(a, S, ch, pc.x, pc.y, pc.z, pf.x, pf.y, pf.z,
                                                                  cnt);
#undef VX_SGP
                            }
                        }
                        if (lit) atomicAdd(&s_plit[wb + fs], 1);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (need) lit0 = s_plit[wb + slot];
            }
        }
        if (!kPool || inframe) {
            float rgba[4];
            if (F.flags & VX_FLAG_PRIMARY_ONLY) {
                primary_only_colour(n, g[0], rgba);
                n_sky = n == 0;
                n_glass = n != 0 && g[0].id == 2;
                n_block = n != 0 && g[0].id != 2;
            } else if (n == 0) {
                n_sky = 1;
                shade_sky(a, d0, d1, d2, rgba, cnt);
            } else {
                // what a glass pane blends over is shaded FIRST: only its colour
                // then stays live across the pane's shading (the record g[1]
                // itself would be: 9 registers, spilled to scratch at the
                // 64-VGPR budget).  Shading has no side effects besides the
                // counters (sums), so the order changes no result.
if constexpr (!kGeneral) {
                float dst[4];
                if (g[0].id == 2) {
                    if (n == 2) shade_block<XE>(a, g[1], dst, cnt);
                    else shade_sky(a, d0, d1, d2, dst, cnt);
                    // two or more panes (rare: a wave-uniform branch): the panes drawn
                    // before the nearest one, in draw order, over what is behind
                    if (__builtin_expect(__ballot(stacked) != 0, 0) && stacked)
                        glass_chain<XE>(a, d0, d1, d2, dst, n == 2 ? t_hit : kInf, cnt);
                }
                float rd[3];
                shade_block<XE>(a, g[0], rgba, cnt, false, 0.0f, 0.0f, 0.0f, rd, lit0);
                if (g[0].id == 2) {
                    n_glass = 1;
                    if (XE && (F.flags & VX_FLAG_REFLECT)) {
                        float refl[3];
                        reflect_color<XE>(a, g[0], rd, refl, cnt);
                        const int ax = g[0].nidx >> 1;
                        const float cs = gmin(fabsf(ax == 0 ? rd[0] : (ax == 1 ? rd[1] : rd[2])), 1.0f);
                        const float x = 1.0f - cs, x2 = x * x;
                        const float fr = 0.04f + 0.96f * ((x2 * x2) * x);
#pragma unroll
                        for (int i = 0; i < 3; i++) rgba[i] = rgba[i] + fr * refl[i];
                    }
                    blend_canvas(rgba, dst, rgba);      // the nearest pane over the canvas
                } else {
                    n_block = 1;
                }
                (void)t_hit;
} else {
                // the general modes (REFLECT_ALL, VX_FLAG_GLASS_ORDER): every first
                // surface may mirror the scene; glass as in the one-blend path
                float dst[4];
                const bool glass = g[0].id == 2;
                if (glass) {
                    if (n == 2) shade_block<XE>(a, g[1], dst, cnt);
                    else shade_sky(a, d0, d1, d2, dst, cnt);
                    if (__builtin_expect(__ballot(stacked) != 0, 0) && stacked)
                        glass_chain<XE>(a, d0, d1, d2, dst, n == 2 ? t_hit : kInf, cnt);
                }
                float rd[3];
                shade_block<XE>(a, g[0], rgba, cnt, false, 0.0f, 0.0f, 0.0f, rd, lit0);
                // ext REFLECT (glass panes) / REFLECT_ALL (every first surface and pane)
                if (XE && (F.flags & (glass ? (VX_FLAG_REFLECT | VX_FLAG_REFLECT_ALL) : VX_FLAG_REFLECT_ALL))) {
                    // Schlick Fresnel, F0 = 0.04, on the geometric normal (cos = |rayDir| on the face axis)
                    float refl[3];
                    reflect_color<XE>(a, g[0], rd, refl, cnt);
                    const int ax = g[0].nidx >> 1;
                    const float cs = gmin(fabsf(ax == 0 ? rd[0] : (ax == 1 ? rd[1] : rd[2])), 1.0f);
                    const float x = 1.0f - cs, x2 = x * x;
                    const float fr = 0.04f + 0.96f * ((x2 * x2) * x);
#pragma unroll
                    for (int i = 0; i < 3; i++) rgba[i] = rgba[i] + fr * refl[i];
                }
                if (glass) {
                    n_glass = 1;
                    blend_canvas(rgba, dst, rgba);
                } else {
                    n_block = 1;
                }
}
            }
            rgba[3] = 1.0f;
            // each wave stores its own 8x8 tile (eight 32-B row pieces per RGBA8 wave
            // store): no block barrier, so a wave that finishes early frees its slot
            store_pixel<FMT>(a, TILED ? (size_t)toidx : out_index<TILED>(a, tile_k, tx0 + lx, ty0 + ly, px, py), rgba);
            n_px = 1;
        }
    }
#ifdef VX_BLOCK_TIMING
    __syncthreads();
    if (threadIdx.x == 0 && a.blk_time) {
        const size_t b = (size_t)blockIdx.x + (size_t)blockIdx.y * gridDim.x;
        a.blk_time[2 * b] = t_blk0;
        a.blk_time[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (STATS) {
        unsigned long long v[ST_COUNT];
        v[ST_PIXELS] = wave_sum(n_px);
        v[ST_SKY] = wave_sum(n_sky);
        v[ST_BLOCK] = wave_sum(n_block);
        v[ST_GLASS] = wave_sum(n_glass);
        v[ST_PRIM_FETCH] = wave_sum(cnt.prim_fetch);
        v[ST_SHADOW_RAYS] = wave_sum(cnt.shadow_rays);
        v[ST_SHADOW_FETCH] = wave_sum(cnt.shadow_fetch);
        v[ST_AO] = wave_sum(cnt.ao);
        v[ST_NOISE_PX] = wave_sum(cnt.noise_px);
        v[ST_CAP_HITS] = wave_sum(cnt.cap_hit);
        v[ST_REFL_RAYS] = wave_sum(cnt.refl_rays);
        v[ST_REFL_FETCH] = wave_sum(cnt.refl_fetch);
        v[ST_ROUGH] = wave_sum(cnt.rough);
        v[ST_PRIM_WITERS] = wave_sum(cnt.prim_witers);
        v[ST_MARCH_WITERS] = wave_sum(cnt.march_witers);
        v[ST_MARCH_SLOTS] = wave_sum(cnt.march_slots);
        v[ST_SHADOW_RESOLVED] = wave_sum(cnt.shadow_resolved);
        if (lane == 0) {
            // spread the adds over 64 slot rows to avoid one hot line per counter
            unsigned long long *row = a.stats + (size_t)((blockIdx.x + blockIdx.y * 7) & 63) * ST_COUNT;
#pragma unroll
            for (int i = 0; i < ST_COUNT; i++) atomicAdd(row + i, v[i]);
        }
    }
}

// One EXT mode's render launches: every (format, stats, tiled, primary index)
// instantiation of that mode, compiled in the unit that calls it.
template <int F, bool S, bool T, int E>
void launch_k(const KernelArgs &a, dim3 grid, hipStream_t s) {
    if constexpr (E >= 5) {           // the general shading modes: the integer primary index only
        hipLaunchKernelGGL((k_render<F, S, T, E, false>), grid, dim3(kWG), 0, s, a);
    } else {
        if (a.prim_f32)
            hipLaunchKernelGGL((k_render<F, S, T, E, true>), grid, dim3(kWG), 0, s, a);
        else
            hipLaunchKernelGGL((k_render<F, S, T, E, false>), grid, dim3(kWG), 0, s, a);
    }
}

template <int E>
int launch_render_ext(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    const hipStream_t s = (hipStream_t)stream;
    // a tiled launch as (block columns, block rows, tiles) while the list fits the z dimension
    const bool t3 = a.tile_ids != nullptr && a.n_tiles <= 65535;
    const dim3 grid = t3 ? dim3((unsigned)(a.tile_w >> kBXS), (unsigned)(a.tile_h >> kBYS), (unsigned)a.n_tiles)
                         : dim3(gx, gy);
    const bool st = a.stats != nullptr, tiled = a.tile_ids != nullptr;
    if (fmt == VX_PIXEL_RGBA32F) {
        if (st) { if (tiled) launch_k<0, true, true, E>(a, grid, s); else launch_k<0, true, false, E>(a, grid, s); }
        else { if (tiled) launch_k<0, false, true, E>(a, grid, s); else launch_k<0, false, false, E>(a, grid, s); }
    } else {
        if (st) { if (tiled) launch_k<1, true, true, E>(a, grid, s); else launch_k<1, true, false, E>(a, grid, s); }
        else { if (tiled) launch_k<1, false, true, E>(a, grid, s); else launch_k<1, false, false, E>(a, grid, s); }
    }
    return (int)hipGetLastError();
}

}  // namespace

// the per-mode launchers (vx_render_e*.hip), called by launch_render (vx_kernels.hip)
int launch_render_e0(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream);
int launch_render_e1(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream);
int launch_render_e2(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream);
int launch_render_e3(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream);
int launch_render_e4(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream);
int launch_render_e56(int ext, const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream);

}  // namespace vx
