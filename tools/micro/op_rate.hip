// Per-instruction issue cost at 8 waves/SIMD on gfx950 (SIMD-cycles per
// wave64 instruction, nominal 2.4 GHz): 8 independent register chains per
// lane, one instruction per chain per iteration, inline asm so the compiler
// cannot substitute.  Used to price the traversal / march loop rewrites.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int N = 2048;

#define CHAIN8(INS)                                                                                     \
    asm volatile(INS : "+v"(x0)); asm volatile(INS : "+v"(x1)); asm volatile(INS : "+v"(x2));             \
    asm volatile(INS : "+v"(x3)); asm volatile(INS : "+v"(x4)); asm volatile(INS : "+v"(x5));             \
    asm volatile(INS : "+v"(x6)); asm volatile(INS : "+v"(x7));

#define KERNEL(NAME, INS)                                                                               \
    __global__ __launch_bounds__(256) void NAME(float *o) {                                             \
        float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,          \
              x6 = x0 + 6, x7 = x0 + 7;                                                                 \
        for (int n = 0; n < N; n++) { CHAIN8(INS) }                                                    \
        o[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                     \
    }
// 64-bit register pairs for packed ops
#define KERNEL2(NAME, INS)                                                                              \
    __global__ __launch_bounds__(256) void NAME(float *o) {                                             \
        typedef float f2 __attribute__((ext_vector_type(2)));                                         \
        f2 x0 = {1, 2}, x1 = {3, 4}, x2 = {5, 6}, x3 = {7, 8}, x4 = {1, 3}, x5 = {2, 5}, x6 = {4, 7},     \
           x7 = {6, 9};                                                                                 \
        for (int n = 0; n < N; n++) { CHAIN8(INS) }                                                    \
        f2 s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                                  \
        o[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;                                                 \
    }

KERNEL(k_add, "v_add_f32 %0, 1.0, %0")
KERNEL(k_mul, "v_mul_f32 %0, 0.5, %0")
KERNEL(k_fma, "v_fma_f32 %0, %0, 0.5, 1.0")
KERNEL(k_floor, "v_floor_f32 %0, %0")
KERNEL(k_min3, "v_min3_f32 %0, %0, 1.0, 2.0")
KERNEL(k_med3, "v_med3_f32 %0, %0, 1.0, 2.0")
KERNEL(k_cvt_i, "v_cvt_i32_f32 %0, %0")
KERNEL(k_cvt_f, "v_cvt_f32_i32 %0, %0")
KERNEL(k_cvt_ub, "v_cvt_f32_ubyte0 %0, %0")
KERNEL(k_addu, "v_add_u32 %0, 1, %0")
KERNEL(k_mul24, "v_mul_u32_u24 %0, 3, %0")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, 3, 1")
KERNEL(k_add3, "v_add3_u32 %0, %0, 1, 2")
KERNEL(k_and, "v_and_b32 %0, 0xff, %0")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 8, %0")
KERNEL(k_cnd, "v_cndmask_b32 %0, %0, 1.0, vcc")
KERNEL(k_cmp, "v_cmp_gt_f32 vcc, %0, 1.0")
KERNEL(k_sqrt, "v_sqrt_f32 %0, %0")
KERNEL(k_rcp, "v_rcp_f32 %0, %0")
KERNEL(k_mov, "v_mov_b32 %0, 1.0")
KERNEL2(k_pkfma, "v_pk_fma_f32 %0, %0, 0.5, 1.0 op_sel_hi:[1,0,0]")
KERNEL2(k_pkadd, "v_pk_add_f32 %0, %0, 1.0 op_sel_hi:[1,0]")
KERNEL2(k_pkmul, "v_pk_mul_f32 %0, %0, 0.5 op_sel_hi:[1,0]")

int main() {
    float *o;
    (void)hipMalloc(&o, 256 * 8192 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int blocks = 256 * 8 * 4;
    auto run = [&](const char *name, void (*k)(float *)) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double instr = blocks * 4.0 * N * 8;
        printf("%-8s %.3f ms  %.2f SIMD-cycles/wave-instr\n", name, ms, ms * 1e-3 * 2.4e9 * 1024.0 / instr);
    };
    run("add", k_add); run("mul", k_mul); run("fma", k_fma); run("floor", k_floor); run("min3", k_min3);
    run("med3", k_med3); run("cvt_i", k_cvt_i); run("cvt_f", k_cvt_f); run("cvt_ub", k_cvt_ub);
    run("add_u32", k_addu); run("mul24", k_mul24); run("mad24", k_mad24); run("add3", k_add3);
    run("and", k_and); run("lshr", k_lshr); run("cndmask", k_cnd); run("cmp", k_cmp); run("sqrt", k_sqrt);
    run("rcp", k_rcp); run("mov", k_mov); run("pk_fma", k_pkfma); run("pk_add", k_pkadd); run("pk_mul", k_pkmul);
    return 0;
}
