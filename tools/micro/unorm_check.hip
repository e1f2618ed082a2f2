// Exhaustive check of the typed buffer loads' UNORM8 conversion on gfx950:
// buffer_load_format_{x,xy,xyzw} with NUM_FORMAT UNORM over 8 / 8_8 / 8_8_8_8
// data must return the IEEE quotient RN(b / 255.0f) for every byte b -- the
// render.frag:38 decode the kernel takes from an LDS table today.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ u32x4 rsrc(const void *p, unsigned w3) {
    const unsigned long long a = (unsigned long long)p;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((unsigned)a);
    r.y = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32) & 0xffffu);
    r.z = 0xffffffffu;
    r.w = w3;
    return r;
}

__global__ void k(const uint8_t *b8, const uint32_t *b32, float *out) {
    const unsigned i = threadIdx.x;       // 256 threads
    float x, y0, y1, z0, z1, z2, z3;
    const u32x4 r8 = rsrc(b8, 0x8004u);              // 8, UNORM, dst X
    const u32x4 r88 = rsrc(b32, 0x1802Cu);           // 8_8, UNORM, dst XY (from a 4-B texel's low half)
    const u32x4 r8888 = rsrc(b32, 0x50FACu);         // 8_8_8_8, UNORM, dst XYZW
    asm volatile("buffer_load_format_x %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(i), "s"(r8));
    float2 v2;
    asm volatile("buffer_load_format_xy %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)" : "=v"(v2) : "v"(4 * i), "s"(r88));
    float4 v4;
    asm volatile("buffer_load_format_xyzw %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)" : "=v"(v4) : "v"(4 * i), "s"(r8888));
    y0 = v2.x; y1 = v2.y; z0 = v4.x; z1 = v4.y; z2 = v4.z; z3 = v4.w;
    float *o = out + 8 * i;
    o[0] = x; o[1] = y0; o[2] = y1; o[3] = z0; o[4] = z1; o[5] = z2; o[6] = z3;
}

int main() {
    uint8_t h8[256];
    uint32_t h32[256];
    for (int i = 0; i < 256; i++) {
        h8[i] = (uint8_t)i;
        h32[i] = (uint32_t)i | (uint32_t)(255 - i) << 8 | (uint32_t)((i * 7) & 255) << 16 | (uint32_t)((i * 13) & 255) << 24;
    }
    uint8_t *d8; uint32_t *d32; float *dout;
    hipMalloc(&d8, 256); hipMalloc(&d32, 1024); hipMalloc(&dout, 256 * 8 * 4);
    hipMemcpy(d8, h8, 256, hipMemcpyHostToDevice);
    hipMemcpy(d32, h32, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d8, d32, dout);
    static float out[256 * 8];
    if (hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 2; }
    int bad = 0;
    auto q = [](unsigned b) { return (float)b / 255.0f; };
    for (int i = 0; i < 256; i++) {
        const uint32_t t = h32[i];
        const float want[7] = {q(i), q(t & 255), q((t >> 8) & 255), q(t & 255), q((t >> 8) & 255), q((t >> 16) & 255),
                               q(t >> 24)};
        for (int c = 0; c < 7; c++)
            if (out[8 * i + c] != want[c]) {
                if (bad < 10) printf("mismatch byte lane %d comp %d: got %a want %a\n", i, c, out[8 * i + c], want[c]);
                bad++;
            }
    }
    printf("unorm8 typed-load check: %d mismatches over 256 x 7 conversions (8, 8_8 xy, 8_8_8_8 xyzw)\n", bad);
    return bad ? 1 : 0;
}
