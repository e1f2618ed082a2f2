// vx_kernels.hip — CDNA4 (gfx950) kernels of the Voxmap shading path.
//
// One fused kernel per frame: primary visibility (the build's replacement for
// rasterising vertex.bin) -> render.frag main() shading with
// the sun march() (render.frag:75-142) -> glass blend -> framebuffer store.
// Lane = pixel; a wave64 covers an 8x8 pixel tile, a 256-thread workgroup a
// 16x16 tile, so the rays of a wave march through neighbouring cells.
//
// Numerical contract: fp32, IEEE div/sqrt, no FMA contraction
// (built with -ffp-contract=off), GLSL built-ins spelled out, vx_exp2 below,
// so every pixel matches the scalar oracle (oracle/vxo_render.c) bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "vx_internal.h"

namespace vx {
namespace {

constexpr int kGlass = 21;  // render.vert:21, sdf.cpp:337

// ---------------- GLSL built-ins (GLSL ES 3.00 §8) ----------------
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float gclamp(float x, float a, float b) { return gmin(gmax(x, a), b); }
__device__ __forceinline__ float gmix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
__device__ __forceinline__ float gsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
__device__ __forceinline__ int f2i(float x) {
    if (x != x) return 0;
    if (x > 16777216.0f) return 16777216;
    if (x < -16777216.0f) return -16777216;
    return (int)x;
}

// exp2 by the fixed degree-9 polynomial of the numerical contract.
__device__ __forceinline__ float vexp2(float x) {
    if (x != x) return x;
    if (x >= 128.0f) return __builtin_inff();
    if (x < -126.0f) return 0.0f;
    float n = floorf(x);
    float f = x - n;
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

struct Surf {            // one G-buffer record (render.vert outputs)
    int id;              // 0 block, 1 sky, 2 glass
    int color;
    int nidx;            // normal index 0..5
    int cell[3];
    float fr[3];
};

struct Counters {
    unsigned prim_fetch, shadow_rays, shadow_fetch, ao, noise_px, cap_hit;
};

__device__ __forceinline__ uint32_t texel(const KernelArgs &a, int x, int y, int z) {
    return a.field[(size_t)x + (size_t)a.X * ((size_t)y + (size_t)a.Y * (size_t)z)];
}
__device__ __forceinline__ float unorm(uint32_t b) { return (float)b / 255.0f; }

// ---------------- sun march: render.frag:75-142 ----------------
// Returns true when the ray reaches MAX_STEPS (lit, render.frag:234).
__device__ bool march_lit(const KernelArgs &a, const int cell[3], const float fr[3], const float r[3],
                          int max_steps, unsigned &fetches) {
    int c0 = cell[0], c1 = cell[1], c2 = cell[2];
    float f0 = fr[0], f1 = fr[1], f2 = fr[2];
    const float s0 = gsign(r[0]), s1 = gsign(r[1]), s2 = gsign(r[2]);
    const float a0 = fabsf(r[0]), a1 = fabsf(r[1]), a2 = fabsf(r[2]);
    const int ch = r[2] > 0.0f ? 0 : 8;   // sdf_dir: R (up) for up-going rays, else G
    float safe = 1.0f;
    int step = 0;
    while (step < max_steps && safe != 0.0f) {
        float x0 = -f0 * s0, x1 = -f1 * s1, x2 = -f2 * s2;
        float d0 = (x0 - floorf(x0)) + 1e-4f;
        float d1 = (x1 - floorf(x1)) + 1e-4f;
        float d2 = (x2 - floorf(x2)) + 1e-4f;
        float t0 = d0 / a0, t1 = d1 / a1, t2 = d2 / a2;
        float m0 = t0 <= gmin(t1, t2) ? 1.0f : 0.0f;
        float m1 = t1 <= gmin(t2, t0) ? 1.0f : 0.0f;
        float m2 = t2 <= gmin(t0, t1) ? 1.0f : 0.0f;
        float v0 = m0 * t0, v1 = m1 * t1, v2 = m2 * t2;
        float len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
        f0 += r[0] * safe * len;
        f1 += r[1] * safe * len;
        f2 += r[2] * safe * len;
        float fl0 = floorf(f0), fl1 = floorf(f1), fl2 = floorf(f2);
        c0 += f2i(fl0); c1 += f2i(fl1); c2 += f2i(fl2);
        f0 = f0 - fl0; f1 = f1 - fl1; f2 = f2 - fl2;
        if (c0 >= a.X || c1 >= a.Y || c2 >= a.Z || c0 < 0 || c1 < 0 || c2 < 0) return true;
        uint32_t t = texel(a, c0, c1, c2);
        fetches++;
        safe = (float)((t >> ch) & 0xffu);   // unorm8 * 255 == b exactly; mix() selects a channel
        step++;
    }
    return step == max_steps;
}

// ---------------- primary visibility ----------------
// First in-grid colour change along the view ray (faces of the greedy mesh of
// sdf.cpp:281-356 after back-face culling); Chebyshev skips in air cells.
// Returns number of records (0 sky, 1 surface, 2 glass + what is behind).
__device__ int primary(const KernelArgs &a, const float d[3], Surf g[2], Counters &cnt) {
    const int dims[3] = {a.X, a.Y, a.Z};
    const float *o = a.p.cam_fract;
    const int *cc = a.p.cam_cell;
    float inv[3];
    int stp[3];
    float tlo = 0.0f, thi = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 3; i++) {
        stp[i] = d[i] > 0.0f ? 1 : -1;
        float lo = (float)(0 - cc[i]) - o[i];
        float hi = (float)(dims[i] - cc[i]) - o[i];
        if (d[i] != 0.0f) {
            inv[i] = 1.0f / d[i];
            float t0 = lo * inv[i], t1 = hi * inv[i];
            if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
            tlo = gmax(tlo, t0);
            thi = gmin(thi, t1);
        } else {
            inv[i] = 0.0f;
            if (!(lo <= 0.0f && 0.0f < hi)) return 0;
        }
    }
    if (!(tlo < thi)) return 0;
    const float amax = gmax(gmax(fabsf(d[0]), fabsf(d[1])), fabsf(d[2]));
    const float inv_inf = 1.0f / amax;
    int c[3];
    float tmax[3];
    float tcur = tlo;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float p = o[i] + tcur * d[i];
        int ci = f2i(floorf(p));
        int lo = -cc[i], hi = dims[i] - cc[i] - 1;
        c[i] = ci < lo ? lo : (ci > hi ? hi : ci);
    }
#pragma unroll
    for (int i = 0; i < 3; i++)
        tmax[i] = d[i] != 0.0f ? ((float)(c[i] + (stp[i] > 0 ? 1 : 0)) - o[i]) * inv[i] : __builtin_inff();
    int nrec = 0;
    uint32_t t = texel(a, c[0] + cc[0], c[1] + cc[1], c[2] + cc[2]);
    cnt.prim_fetch++;
    int prev = (t >> 16) & 0xff;
    int dist = t >> 24;
    const int cap = 4 * (dims[0] + dims[1] + dims[2]);
    for (int iter = 0; iter < cap; iter++) {
        if (prev == 0 && dist >= 3) {
            tcur = tcur + ((float)dist - 1.5f) * inv_inf;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                float p = o[i] + tcur * d[i];
                c[i] = f2i(floorf(p));
                tmax[i] = d[i] != 0.0f ? ((float)(c[i] + (stp[i] > 0 ? 1 : 0)) - o[i]) * inv[i] : __builtin_inff();
            }
            int x = c[0] + cc[0], y = c[1] + cc[1], z = c[2] + cc[2];
            if (x < 0 || y < 0 || z < 0 || x >= a.X || y >= a.Y || z >= a.Z) return nrec;
            t = texel(a, x, y, z);
            cnt.prim_fetch++;
            dist = t >> 24;
            continue;
        }
        int ax = (tmax[0] <= tmax[1] && tmax[0] <= tmax[2]) ? 0 : (tmax[1] <= tmax[2] ? 1 : 2);
        float tcross = tmax[ax];
        c[ax] += stp[ax];
        tmax[ax] = ((float)(c[ax] + (stp[ax] > 0 ? 1 : 0)) - o[ax]) * inv[ax];
        tcur = tcross;
        int ac[3] = {c[0] + cc[0], c[1] + cc[1], c[2] + cc[2]};
        if (ac[0] < 0 || ac[1] < 0 || ac[2] < 0 || ac[0] >= a.X || ac[1] >= a.Y || ac[2] >= a.Z) return nrec;
        t = texel(a, ac[0], ac[1], ac[2]);
        cnt.prim_fetch++;
        int col = (t >> 16) & 0xff;
        dist = t >> 24;
        if (col != prev) {
            Surf &h = g[nrec];
            h.color = col;
            h.id = col == kGlass ? 2 : 0;
            h.nidx = 2 * ax + (stp[ax] > 0 ? 1 : 0);
#pragma unroll
            for (int i = 0; i < 3; i++) {
                if (i == ax) {
                    h.cell[i] = ac[i] + (stp[ax] > 0 ? 0 : 1);
                    h.fr[i] = 0.0f;
                } else {
                    float p = o[i] + tcross * d[i];
                    h.cell[i] = ac[i];
                    h.fr[i] = p - (float)c[i];
                }
            }
            nrec++;
            if (h.id != 2 || nrec == 2) return nrec;
        }
        prev = col;
    }
    cnt.cap_hit++;
    return nrec;
}

// ---------------- sampling ----------------
__device__ __forceinline__ void lin_axis(float coord, int size, int &i0, int &i1, float &w) {
    float u = coord * (float)size - 0.5f;
    float fl = floorf(u);
    w = u - fl;
    int i = f2i(fl);
    int j = i + 1;
    i0 = i < 0 ? 0 : (i > size - 1 ? size - 1 : i);
    i1 = j < 0 ? 0 : (j > size - 1 ? size - 1 : j);
}

// sdf(ivec3, vec3) (render.frag:55-58) = min of trilinear R, G (LOD 0).
__device__ float sdf_lin(const KernelArgs &a, const int c[3], const float f[3]) {
    const int dims[3] = {a.X, a.Y, a.Z};
    int i0[3], i1[3];
    float w[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float sf = 1.0f / (float)dims[k];
        float coord = ((float)c[k] + f[k]) * sf;
        lin_axis(coord, dims[k], i0[k], i1[k], w[k]);
    }
    uint32_t t[2][2][2];
#pragma unroll
    for (int kz = 0; kz < 2; kz++)
#pragma unroll
        for (int ky = 0; ky < 2; ky++)
#pragma unroll
            for (int kx = 0; kx < 2; kx++)
                t[kz][ky][kx] = texel(a, kx ? i1[0] : i0[0], ky ? i1[1] : i0[1], kz ? i1[2] : i0[2]);
    float res[2];
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
        float v[2][2];
#pragma unroll
        for (int kz = 0; kz < 2; kz++)
#pragma unroll
            for (int ky = 0; ky < 2; ky++)
                v[kz][ky] = gmix(unorm((t[kz][ky][0] >> (8 * ch)) & 0xffu),
                                 unorm((t[kz][ky][1] >> (8 * ch)) & 0xffu), w[0]);
        float w0 = gmix(v[0][0], v[0][1], w[1]);
        float w1 = gmix(v[1][0], v[1][1], w[1]);
        res[ch] = gmix(w0, w1, w[2]) * 255.0f;
    }
    return gmin(res[0], res[1]);
}

__device__ __forceinline__ int wrap_idx(float fl, int n) {
    float q = floorf(fl / (float)n);
    return f2i(fl - q * (float)n) & (n - 1);
}

// fbm(p) = 1 - 2*texture(u_noise, p).a (render.frag:16-24), bilinear, REPEAT.
__device__ float fbm(const KernelArgs &a, float px, float py) {
    const int W = a.noise_w, H = a.noise_h;
    float u = px * (float)W - 0.5f, v = py * (float)H - 0.5f;
    float fu = floorf(u), fv = floorf(v);
    float wa = u - fu, wb = v - fv;
    int x0 = wrap_idx(fu, W), y0 = wrap_idx(fv, H);
    int x1 = (x0 + 1) & (W - 1), y1 = (y0 + 1) & (H - 1);
    float t00 = unorm(a.noise[(size_t)y0 * W + x0] >> 24);
    float t10 = unorm(a.noise[(size_t)y0 * W + x1] >> 24);
    float t01 = unorm(a.noise[(size_t)y1 * W + x0] >> 24);
    float t11 = unorm(a.noise[(size_t)y1 * W + x1] >> 24);
    float r0 = gmix(t00, t10, wa), r1 = gmix(t01, t11, wa);
    float t = gmix(r0, r1, wb);
    return 1.0f - 2.0f * t;
}

__device__ __forceinline__ float dot3(const float x[3], const float y[3]) {
    return x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
}
__device__ __forceinline__ void normalize3(const float v[3], float out[3]) {
    float l = sqrtf(dot3(v, v));
    out[0] = v[0] / l; out[1] = v[1] / l; out[2] = v[2] / l;
}

// ---------------- render.frag main() (render.frag:147-252) ----------------
__device__ void shade(const KernelArgs &a, const Surf &g, const float prim_dir[3], float o[4],
                      Counters &cnt) {
    const vx_frame_params &P = a.p;
    o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f; o[3] = 1.0f;
    const bool isSky = g.id == 1, isGlass = g.id == 2;
    const float litCol[3] = {0.4f, 0.35f, 0.3f};
    float nrm[3] = {0.0f, 0.0f, 0.0f};
    const int ni = isSky ? 1 : g.nidx;
    nrm[ni >> 1] = (ni & 1) ? -1.0f : 1.0f;
    float rayDir[3];
    if (isSky) {
        normalize3(prim_dir, rayDir);
    } else {
        float v[3];
#pragma unroll
        for (int i = 0; i < 3; i++) v[i] = (float)(g.cell[i] - P.cam_cell[i]) + (g.fr[i] - P.cam_fract[i]);
        normalize3(v, rayDir);
    }
    float refl[3];
    {
        float k = 2.0f * dot3(nrm, rayDir);
#pragma unroll
        for (int i = 0; i < 3; i++) refl[i] = rayDir[i] - k * nrm[i];
    }
    const float sunCol[3] = {1.4f, 1.0f, 0.5f};
    float sunFactor = gmax(0.0f, dot3(P.sun_dir, rayDir)) - 1.0f;
    float glow = vexp2(8.0f * sunFactor);
    sunFactor = vexp2(4000.0f * sunFactor) + 0.3f * glow;
    float scatter = 1.0f - sqrtf(gmax(0.0f, P.sun_dir[2]));
    const float sp0[3] = {0.2f, 0.4f, 0.7f}, sp1[3] = {0.2f, 0.3f, 0.5f};
    const float sc0[3] = {0.7f, 0.9f, 1.0f}, sc1[3] = {1.0f, 0.3f, 0.2f};
    float scatterCol[3], atmCol[3], skyCol[3];
    float rz = sqrtf(gmax(0.0f, refl[2]));
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float spaceCol = gmix(sp0[i], sp1[i], scatter);
        scatterCol[i] = gmix(sc0[i], sc1[i], scatter);
        atmCol[i] = gmix(scatterCol[i], spaceCol, rz);
        skyCol[i] = gclamp(sunCol[i] * sunFactor + atmCol[i], 0.0f, 1.0f);
    }
    if (isSky) {
        rayDir[2] = fabsf(rayDir[2]);
        if (P.flags & VX_FLAG_NO_CLOUDS) {
            o[0] = skyCol[0]; o[1] = skyCol[1]; o[2] = skyCol[2];
            return;
        }
        cnt.noise_px++;
        float cloudTime = P.time * 4e-3f;
        float den = sqrtf(fabsf(rayDir[2]) + 0.03f);
        float sx = rayDir[0] / den, sy = rayDir[1] / den;
        sx = sx * 0.1f; sy = sy * 0.1f;
        float sl = sqrtf(sqrtf(sx * sx + sy * sy));
        sx = sx * sl; sy = sy * sl;
        float n0 = fbm(a, 2.0f * sx + cloudTime, 2.0f * sy + cloudTime);
        float n1 = fbm(a, 2.0f * sx - cloudTime, 2.0f * sy - cloudTime);
        sx = sx * (3.0f + n0); sy = sy * (3.0f + n1);
        sx = sx + 1e-4f * ((float)P.cam_cell[0] + P.cam_fract[0]);
        sy = sy + 1e-4f * ((float)P.cam_cell[1] + P.cam_fract[1]);
        float cloudFactor = vexp2(6.0f * (fbm(a, sx + 2.0f * cloudTime, sy + -9.0f * cloudTime) - 1.0f));
        float scf = sqrtf(cloudFactor);
        float mountainPos = rayDir[0] / rayDir[1];
        float mountainHeight = 1.0f - fbm(a, 0.3f * mountainPos, 0.3f * mountainPos);
        float mountainFactor = 2.0f - fbm(a, 2.0f * (mountainPos + rayDir[1]), 2.0f * (mountainPos + rayDir[2]));
        mountainHeight = mountainHeight / (vexp(0.3f * mountainPos * mountainPos) * 6.0f);
        if (mountainHeight > rayDir[2] && rayDir[1] > 0.0f && rayDir[2] > 0.0f) {
            const float mt[3] = {0.7f, 0.8f, 0.7f};
            float w = mountainFactor * rayDir[2];
#pragma unroll
            for (int i = 0; i < 3; i++) skyCol[i] = gmix(skyCol[i], skyCol[i] * mt[i], w);
        } else {
#pragma unroll
            for (int i = 0; i < 3; i++) skyCol[i] = gmix(skyCol[i], gmix(sunCol[i], 0.8f, scf), cloudFactor);
        }
        o[0] = skyCol[0]; o[1] = skyCol[1]; o[2] = skyCol[2];
        return;
    }
    // block branch (render.frag:207-251)
    const int pidx = g.color;
    float base[3];
    if (pidx < 22) { base[0] = kPalette[pidx][0]; base[1] = kPalette[pidx][1]; base[2] = kPalette[pidx][2]; }
    else { base[0] = base[1] = base[2] = 1.0f; }
    const float an0 = fabsf(nrm[0]), an1 = fabsf(nrm[1]), an2 = fabsf(nrm[2]);
    const float M0[3] = {0.90f, 0.90f, 0.95f}, M1[3] = {0.95f, 0.95f, 1.00f};
    float normalCol[3];
#pragma unroll
    for (int i = 0; i < 3; i++) normalCol[i] = (M0[i] * an0 + M1[i] * an1) + 1.0f * an2;
    if (nrm[2] < 0.0f) {
#pragma unroll
        for (int i = 0; i < 3; i++) normalCol[i] = normalCol[i] * 0.8f;
    }
    float shadeCol[3];
#pragma unroll
    for (int i = 0; i < 3; i++) shadeCol[i] = 0.7f * scatterCol[i];
    float ambCol[3] = {1.0f, 1.0f, 1.0f};
    if (!(P.flags & VX_FLAG_NO_AO)) {
        cnt.ao++;
        int ac[3];
#pragma unroll
        for (int i = 0; i < 3; i++) ac[i] = g.cell[i] + f2i(nrm[i]);
        float ambDist = sdf_lin(a, ac, g.fr);
        float ambFactor = gmin(1.0f - sqrtf(ambDist), 0.8f);
#pragma unroll
        for (int i = 0; i < 3; i++) ambCol[i] = gmix(1.0f, shadeCol[i], ambFactor);
    }
    float shadeFactor = P.sun_dir[2] < 0.0f ? 0.0f : sqrtf(gmax(0.0f, dot3(nrm, P.sun_dir)));
    if (shadeFactor > 0.0f && !(P.flags & VX_FLAG_NO_SHADOW)) {
        cnt.shadow_rays++;
        bool lit = march_lit(a, g.cell, g.fr, P.sun_dir, a.max_shadow_steps, cnt.shadow_fetch);
        shadeFactor = shadeFactor * (lit ? 1.0f : 0.0f);
    }
    float lightCol[3];
#pragma unroll
    for (int i = 0; i < 3; i++) lightCol[i] = shadeCol[i] + litCol[i] * shadeFactor;
#pragma unroll
    for (int i = 0; i < 3; i++) o[i] = base[i];
    if (P.quality > 0) {
#pragma unroll
        for (int i = 0; i < 3; i++) o[i] = o[i] * ((normalCol[i] * lightCol[i]) * ambCol[i]);
    }
    if (isGlass) {
        o[3] = 0.8f * vexp2(dot3(rayDir, nrm));
#pragma unroll
        for (int i = 0; i < 3; i++) o[i] = o[i] * (0.2f * atmCol[i]);
    }
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned v) {
    unsigned long long s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

template <int FMT, bool STATS, bool TILED>
__global__ __launch_bounds__(256) void k_render(KernelArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lx = ((wave & 1) << 3) | (lane & 7);
    const int ly = ((wave >> 1) << 3) | (lane >> 3);
    int px, py;
    size_t out_idx;
    if (TILED) {
        const int bpt = (a.tile_size >> 4) * (a.tile_size >> 4);  // 16x16 blocks per tile
        const int k = blockIdx.x / bpt, sub = blockIdx.x % bpt;
        const int tid = a.tile_ids[k];
        const int sbx = sub % (a.tile_size >> 4), sby = sub / (a.tile_size >> 4);
        const int tx = (sbx << 4) + lx, ty = (sby << 4) + ly;
        px = (tid % a.tiles_x) * a.tile_size + tx;
        py = (tid / a.tiles_x) * a.tile_size + ty;
        out_idx = (size_t)k * a.tile_size * a.tile_size + (size_t)ty * a.tile_size + tx;
    } else {
        px = (blockIdx.x << 4) + lx;
        py = (blockIdx.y << 4) + ly;
        out_idx = (size_t)py * a.w + px;
    }
    const bool active = px < a.w && py < a.h;
    Counters cnt = {0, 0, 0, 0, 0, 0};
    unsigned n_sky = 0, n_block = 0, n_glass = 0;
    float rgba[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    if (active) {
        const float nx = (float)(2 * px + 1) / (float)a.w - 1.0f;
        const float ny = 1.0f - (float)(2 * py + 1) / (float)a.h;
        float d[3];
#pragma unroll
        for (int i = 0; i < 3; i++) d[i] = (a.p.ray_fwd[i] + nx * a.p.ray_right[i]) + ny * a.p.ray_up[i];
        Surf g[2];
        const int n = primary(a, d, g, cnt);
        Surf sky;
        sky.id = 1; sky.color = 0; sky.nidx = 1;
        sky.cell[0] = sky.cell[1] = sky.cell[2] = 0;
        sky.fr[0] = sky.fr[1] = sky.fr[2] = 0.0f;
        if (n == 0) {
            n_sky = 1;
            shade(a, sky, d, rgba, cnt);
        } else if (g[0].id != 2) {
            n_block = 1;
            shade(a, g[0], d, rgba, cnt);
        } else {
            n_glass = 1;
            float src[4], dst[4];
            shade(a, g[0], d, src, cnt);
            shade(a, n == 2 ? g[1] : sky, d, dst, cnt);
            const float al = src[3];
#pragma unroll
            for (int i = 0; i < 3; i++) rgba[i] = src[i] * al + dst[i] * (1.0f - al);
        }
        rgba[3] = 1.0f;
        if (FMT == VX_PIXEL_RGBA32F) {
            reinterpret_cast<float4 *>(a.out)[out_idx] = make_float4(rgba[0], rgba[1], rgba[2], rgba[3]);
        } else {
            uint32_t pk = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                float v = gclamp(rgba[i], 0.0f, 1.0f) * 255.0f + 0.5f;
                pk |= (uint32_t)v << (8 * i);
            }
            reinterpret_cast<uint32_t *>(a.out)[out_idx] = pk;
        }
    }
    if (STATS) {
        unsigned long long v[ST_COUNT];
        v[ST_PIXELS] = wave_sum(active ? 1u : 0u);
        v[ST_SKY] = wave_sum(n_sky);
        v[ST_BLOCK] = wave_sum(n_block);
        v[ST_GLASS] = wave_sum(n_glass);
        v[ST_PRIM_FETCH] = wave_sum(cnt.prim_fetch);
        v[ST_SHADOW_RAYS] = wave_sum(cnt.shadow_rays);
        v[ST_SHADOW_FETCH] = wave_sum(cnt.shadow_fetch);
        v[ST_AO] = wave_sum(cnt.ao);
        v[ST_NOISE_PX] = wave_sum(cnt.noise_px);
        v[ST_CAP_HITS] = wave_sum(cnt.cap_hit);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < ST_COUNT; i++) atomicAdd(a.stats + i, v[i]);
        }
    }
}

// Scatter compact tile-major pixels into a frame.
template <typename T>
__global__ void k_detile(const T *tiles, T *frame, int w, int h, int ts, int tiles_x, const int *ids, int n_tiles) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per = (size_t)ts * ts;
    if (i >= per * n_tiles) return;
    const int k = (int)(i / per), r = (int)(i % per);
    const int tid = ids[k];
    const int x = (tid % tiles_x) * ts + r % ts, y = (tid / tiles_x) * ts + r / ts;
    if (x < w && y < h) frame[(size_t)y * w + x] = tiles[i];
}

// ---- A channel: capped Chebyshev distance to the nearest non-air cell ----
__global__ void k_dist_x(const uint32_t *field, uint8_t *g1, int X, int Y, int Z, int cap) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t N = (size_t)X * Y * Z;
    if (i >= N) return;
    const int x = (int)(i % X);
    const size_t row = i - x;
    int best = cap;
    for (int k = 0; k < cap; k++) {
        const int xa = x - k, xb = x + k;
        if ((xa >= 0 && (field[row + xa] & 0x00ff0000u)) || (xb < X && (field[row + xb] & 0x00ff0000u))) {
            best = k;
            break;
        }
    }
    g1[i] = (uint8_t)best;
}
__global__ void k_dist_yz(const uint8_t *gin, uint8_t *gout, uint32_t *field, int X, int Y, int Z, int cap, int axis) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t N = (size_t)X * Y * Z;
    if (i >= N) return;
    const int x = (int)(i % X);
    const int y = (int)((i / X) % Y);
    const int z = (int)(i / ((size_t)X * Y));
    const int pos = axis == 1 ? y : z, n = axis == 1 ? Y : Z;
    const size_t stride = axis == 1 ? (size_t)X : (size_t)X * Y;
    const size_t base = i - (size_t)pos * stride;
    int best = cap;
    const int lo = pos - (cap - 1) < 0 ? 0 : pos - (cap - 1);
    const int hi = pos + (cap - 1) > n - 1 ? n - 1 : pos + (cap - 1);
    for (int q = lo; q <= hi; q++) {
        const int v = gin[base + (size_t)q * stride];
        const int ak = q > pos ? q - pos : pos - q;
        const int m = v > ak ? v : ak;
        best = m < best ? m : best;
    }
    if (axis == 1) {
        gout[i] = (uint8_t)best;
    } else {
        field[i] = (field[i] & 0x00ffffffu) | ((uint32_t)best << 24);
    }
    (void)x;
}

}  // namespace

int launch_render(const KernelArgs &a, int fmt, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    dim3 block(256);
    dim3 grid;
    const bool tiled = a.tile_ids != nullptr;
    if (tiled) {
        grid = dim3(a.n_tiles * (a.tile_size >> 4) * (a.tile_size >> 4));
    } else {
        grid = dim3((a.w + 15) / 16, (a.h + 15) / 16);
    }
    const bool st = a.stats != nullptr;
#define VX_LAUNCH(F, S, T) hipLaunchKernelGGL((k_render<F, S, T>), grid, block, 0, s, a)
    if (fmt == VX_PIXEL_RGBA32F) {
        if (tiled) { if (st) VX_LAUNCH(0, true, true); else VX_LAUNCH(0, false, true); }
        else { if (st) VX_LAUNCH(0, true, false); else VX_LAUNCH(0, false, false); }
    } else {
        if (tiled) { if (st) VX_LAUNCH(1, true, true); else VX_LAUNCH(1, false, true); }
        else { if (st) VX_LAUNCH(1, true, false); else VX_LAUNCH(1, false, false); }
    }
#undef VX_LAUNCH
    return (int)hipGetLastError();
}

int launch_detile(const void *tiles, void *frame, int w, int h, int ts, int tiles_x, const int *ids,
                  int n_tiles, int fmt, void *stream) {
    const size_t n = (size_t)ts * ts * n_tiles;
    dim3 grid((unsigned)((n + 255) / 256));
    hipStream_t s = (hipStream_t)stream;
    if (fmt == VX_PIXEL_RGBA32F)
        hipLaunchKernelGGL(k_detile<float4>, grid, dim3(256), 0, s, (const float4 *)tiles, (float4 *)frame, w, h, ts,
                           tiles_x, ids, n_tiles);
    else
        hipLaunchKernelGGL(k_detile<uint32_t>, grid, dim3(256), 0, s, (const uint32_t *)tiles, (uint32_t *)frame, w,
                           h, ts, tiles_x, ids, n_tiles);
    return (int)hipGetLastError();
}

int launch_field_dist(uint32_t *field, int X, int Y, int Z, int cap, uint8_t *ga, uint8_t *gb, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    dim3 grid((unsigned)((N + 255) / 256)), block(256);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_dist_x, grid, block, 0, s, field, ga, X, Y, Z, cap);
    hipLaunchKernelGGL(k_dist_yz, grid, block, 0, s, ga, gb, field, X, Y, Z, cap, 1);
    hipLaunchKernelGGL(k_dist_yz, grid, block, 0, s, gb, ga, field, X, Y, Z, cap, 2);
    return (int)hipGetLastError();
}

}  // namespace vx
