// vx_frame.cpp — per-frame constants of the render kernel.
//
// render.frag recomputes several per-frame quantities in every fragment
// (scatterCol, shade factors of the six axis normals, ...).  They depend only
// on uniforms, so the host derives them once here with exactly the fp32
// operations, operation order and IEEE rounding the oracle uses per pixel
// (x86-64 SSE, -ffp-contract=off): the kernel then reads bit-identical values.
#include <cmath>
#include <cstring>

#include "vx_internal.h"

namespace vx {

static inline float gmax(float x, float y) { return x < y ? y : x; }
static inline float gmix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
static inline float gsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

void frame_consts(const vx_frame_params &p, int w, int h, int X, int Y, int Z, int max_steps, FrameConsts &fc) {
    std::memset(&fc, 0, sizeof fc);
    for (int i = 0; i < 3; i++) {
        fc.cam_cell[i] = p.cam_cell[i];
        fc.cam_fract[i] = p.cam_fract[i];
        fc.fwd[i] = p.ray_fwd[i];
        fc.right[i] = p.ray_right[i];
        fc.up[i] = p.ray_up[i];
        fc.sun[i] = p.sun_dir[i];
        fc.sun_sign[i] = gsign(p.sun_dir[i]);
        fc.sun_abs[i] = std::fabs(p.sun_dir[i]);
        fc.sun_rcp[i] = fc.sun_abs[i] != 0.0f ? 1.0f / fc.sun_abs[i] : 0.0f;
    }
    fc.fw = (float)w;
    fc.fh = (float)h;
    fc.rcp_w = 1.0f / fc.fw;
    fc.rcp_h = 1.0f / fc.fh;
    fc.sun_up = p.sun_dir[2] > 0.0f ? 1 : 0;
    const float lim = 0.0009765625f;   // 2^-10: keeps every t = d/|r| < 1025, every cell index in int range
    fc.march_fast = fc.sun_abs[0] >= lim && fc.sun_abs[1] >= lim && fc.sun_abs[2] >= lim;
    fc.max_steps = max_steps;
    // render.frag:168-170, 220
    const float scatter = 1.0f - std::sqrt(gmax(0.0f, p.sun_dir[2]));
    const float sp0[3] = {0.2f, 0.4f, 0.7f}, sp1[3] = {0.2f, 0.3f, 0.5f};
    const float sc0[3] = {0.7f, 0.9f, 1.0f}, sc1[3] = {1.0f, 0.3f, 0.2f};
    for (int i = 0; i < 3; i++) {
        fc.spaceCol[i] = gmix(sp0[i], sp1[i], scatter);
        fc.scatterCol[i] = gmix(sc0[i], sc1[i], scatter);
        fc.shadeCol[i] = 0.7f * fc.scatterCol[i];
    }
    // per axis normal n (render.vert:14-17): normalCol (render.frag:211-217), shadeFactor (:228-229)
    const float M0[3] = {0.90f, 0.90f, 0.95f}, M1[3] = {0.95f, 0.95f, 1.00f}, M2[3] = {1.0f, 1.0f, 1.0f};
    for (int n = 0; n < 6; n++) {
        float nv[3] = {0.0f, 0.0f, 0.0f};
        nv[n >> 1] = (n & 1) ? -1.0f : 1.0f;
        const float an[3] = {std::fabs(nv[0]), std::fabs(nv[1]), std::fabs(nv[2])};
        for (int i = 0; i < 3; i++) {
            float c = (M0[i] * an[0] + M1[i] * an[1]) + M2[i] * an[2];
            if (nv[2] < 0.0f) c = c * 0.8f;
            fc.normalCol[n][i] = c;
        }
        const float dot = nv[0] * p.sun_dir[0] + nv[1] * p.sun_dir[1] + nv[2] * p.sun_dir[2];
        fc.shadeFactor[n] = p.sun_dir[2] < 0.0f ? 0.0f : std::sqrt(gmax(0.0f, dot));
    }
    const int dims[3] = {X, Y, Z};
    for (int k = 0; k < 3; k++) fc.sf[k] = 1.0f / (float)dims[k];
    fc.cloudTime = p.time * 4e-3f;
    fc.skyOff[0] = 1e-4f * ((float)p.cam_cell[0] + p.cam_fract[0]);
    fc.skyOff[1] = 1e-4f * ((float)p.cam_cell[1] + p.cam_fract[1]);
    fc.quality = p.quality;
    fc.flags = p.flags;
}

}  // namespace vx
