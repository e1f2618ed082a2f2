// vx_frame.cpp — per-frame constants of the render kernel.
//
// render.frag recomputes several per-frame quantities in every fragment
// (scatterCol, shade factors of the six axis normals, ...).  They depend only
// on uniforms, so the host derives them once here with exactly the fp32
// operations, operation order and IEEE rounding the oracle uses per pixel
// (x86-64 SSE, -ffp-contract=off): the kernel then reads bit-identical values.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "vx_internal.h"

namespace vx {

static inline float gmax(float x, float y) { return x < y ? y : x; }
static inline float gmix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
static inline float gsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

void sun_ray(const float r[3], SunRay &s) {
    for (int i = 0; i < 3; i++) {
        s.r[i] = r[i];
        s.sign[i] = gsign(r[i]);
        s.abs[i] = std::fabs(r[i]);
        s.rcp[i] = s.abs[i] != 0.0f ? 1.0f / s.abs[i] : 0.0f;
    }
    s.up = r[2] > 0.0f ? 1 : 0;
    const float lim = 0.0009765625f;   // 2^-10: keeps every t = d/|r| < 1025, every cell index in int range
    s.fast = s.abs[0] >= lim && s.abs[1] >= lim && s.abs[2] >= lim;
}

// cos/sin of k * golden angle (Vogel spiral), k = 0..15, as literals: no libm
// trigonometry enters the directions, so host and oracle agree bit for bit.
static const double kVogel[VX_MAX_SHADOW_SAMPLES][2] = {
    {1.0, 0.0},
    {-0.7373688780783197, 0.6754902942615238},
    {0.08742572471695988, -0.9961710408648278},
    {0.6084388609788626, 0.7936007512916959},
    {-0.9847134853154287, -0.17418195037931164},
    {0.8437552948123972, -0.5367280526263227},
    {-0.25960430490148856, 0.9657150743757783},
    {-0.4609070247133692, -0.8874484292452546},
    {0.9393212963241181, 0.343038630874102},
    {-0.9243455561378048, 0.38155640847493627},
    {0.4238459950479107, -0.9057342725556136},
    {0.2992838644448729, 0.954164120307897},
    {-0.86521120975323, -0.5014075812324265},
    {0.976675773628176, -0.21471942904125782},
    {-0.5751294291397393, 0.8180624302199665},
    {-0.12851068979899324, -0.9917081236973845},
};

// Soft-shadow sample k of n: the sun pushed by radius*sqrt((k+0.5)/n) along
// spiral angle k in the plane normal to it (u = normalize(a x sun), v = sun x u,
// a = z, or x when |sun.z| >= 0.9), normalised; double, then rounded to float.
void sun_samples(const float sun[3], float radius, int n, float out[][3]) {
    if (n <= 1) {
        for (int i = 0; i < 3; i++) out[0][i] = sun[i];
        return;
    }
    n = n > VX_MAX_SHADOW_SAMPLES ? VX_MAX_SHADOW_SAMPLES : n;
    const double sd[3] = {sun[0], sun[1], sun[2]};
    const bool zax = std::fabs(sd[2]) < 0.9;
    const double ax[3] = {zax ? 0.0 : 1.0, 0.0, zax ? 1.0 : 0.0};
    double u[3] = {ax[1] * sd[2] - ax[2] * sd[1], ax[2] * sd[0] - ax[0] * sd[2], ax[0] * sd[1] - ax[1] * sd[0]};
    const double ul = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    for (double &c : u) c /= ul;
    const double v[3] = {sd[1] * u[2] - sd[2] * u[1], sd[2] * u[0] - sd[0] * u[2], sd[0] * u[1] - sd[1] * u[0]};
    for (int k = 0; k < n; k++) {
        const double r = (double)radius * std::sqrt(((double)k + 0.5) / (double)n);
        const double cu = r * kVogel[k][0], cv = r * kVogel[k][1];
        double x[3];
        for (int i = 0; i < 3; i++) x[i] = sd[i] + cu * u[i] + cv * v[i];
        const double l = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
        for (int i = 0; i < 3; i++) out[k][i] = (float)(x[i] / l);
    }
}

void frame_consts(const vx_frame_params &p, int w, int h, int X, int Y, int Z, int max_steps, FrameConsts &fc) {
    std::memset(&fc, 0, sizeof fc);
    for (int i = 0; i < 3; i++) {
        fc.cam_cell[i] = p.cam_cell[i];
        fc.cam_fract[i] = p.cam_fract[i];
        fc.cam_cell_f[i] = (float)p.cam_cell[i];
        fc.fwd[i] = p.ray_fwd[i];
        fc.right[i] = p.ray_right[i];
        fc.up[i] = p.ray_up[i];
        fc.sun[i] = p.sun_dir[i];
        fc.sun_sign[i] = gsign(p.sun_dir[i]);
        fc.sun_abs[i] = std::fabs(p.sun_dir[i]);
        fc.sun_rcp[i] = fc.sun_abs[i] != 0.0f ? 1.0f / fc.sun_abs[i] : 0.0f;
        const int dim = i == 0 ? X : (i == 1 ? Y : Z);
        fc.slab_lo[i] = (float)(0 - p.cam_cell[i]) - p.cam_fract[i];
        fc.slab_hi[i] = (float)(dim - p.cam_cell[i]) - p.cam_fract[i];
        fc.cell_lo[i] = (float)(-p.cam_cell[i]);
        fc.cell_hi[i] = (float)(dim - p.cam_cell[i] - 1);
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
    fc.n_sun = p.shadow_samples > 1 ? std::min(p.shadow_samples, VX_MAX_SHADOW_SAMPLES) : 1;
    float dirs[VX_MAX_SHADOW_SAMPLES][3];
    sun_samples(p.sun_dir, p.sun_radius, fc.n_sun, dirs);
    for (int k = 0; k < fc.n_sun; k++) sun_ray(dirs[k], fc.sun_k[k]);
    // the pooled soft-shadow march (vx_kernels.hip) runs one loop specialised on
    // the axis signs for every sample: only when they all agree
    fc.soft_sg = -1;
    fc.soft_lg = 0;
    while ((1 << fc.soft_lg) < fc.n_sun) fc.soft_lg++;
    if (fc.n_sun > 1) {
        auto sg = [](const SunRay &r) {
            return (r.sign[0] > 0.0f ? 1 : 0) | (r.sign[1] > 0.0f ? 2 : 0) | (r.sign[2] > 0.0f ? 4 : 0);
        };
        bool same = true;
        for (int k = 0; k < fc.n_sun; k++)
            same = same && fc.sun_k[k].fast && sg(fc.sun_k[k]) == sg(fc.sun_k[0]) && fc.sun_k[k].up == fc.sun_k[0].up;
        if (same) fc.soft_sg = sg(fc.sun_k[0]);
    }
}

}  // namespace vx

namespace vx {
// vx_internal.h exit_plan; the oracle's vxo_exit_plan restated (same double
// arithmetic on the same fp32 directions, so both pick the same table)
int exit_plan(const FrameConsts &fc, int SB, int *oct, int *kx, int *ky) {
    *oct = *kx = *ky = -1;
    if (fc.n_sun < 1) return 0;
    const float lim = 0.0009765625f;
    double ax = 0.0, ay = 0.0;
    int sg0 = -1;
    for (int k = 0; k < fc.n_sun; k++) {
        const float *r = fc.sun_k[k].r;
        if (!(std::fabs(r[0]) >= lim && std::fabs(r[1]) >= lim && std::fabs(r[2]) >= lim)) return 0;
        const int sg = (r[0] > 0.0f ? 1 : 0) | (r[1] > 0.0f ? 2 : 0) | (r[2] > 0.0f ? 4 : 0);
        if (k && sg != sg0) return 0;
        sg0 = sg;
        const double sx = std::fabs((double)r[0] / (double)r[2]), sy = std::fabs((double)r[1] / (double)r[2]);
        ax = sx > ax ? sx : ax;
        ay = sy > ay ? sy : ay;
    }
    // SB = Z + 2 >= 5 >= kx, ky (the window stays inside the -1 border) unless Z < 3
    if (!(sg0 & 4) || ax > 4.0 || ay > 4.0 || SB < 5) return 0;
    const int cx = (int)std::ceil(ax + 1.0 / 64.0), cy = (int)std::ceil(ay + 1.0 / 64.0);
    *oct = sg0; *kx = cx; *ky = cy;
    return 1;
}

// vx_internal.h doom_plan; the oracle's vxo_doom_plan restated (same double
// arithmetic on the same fp32 directions)
void doom_plan(const FrameConsts &fc, int plan[7]) {
    double axmin = 1e300, axmax = -1e300, aymin = 1e300, aymax = -1e300;
    for (int k = 0; k < fc.n_sun; k++) {
        const float *r = fc.sun_k[k].r;
        const double ax = std::fabs((double)r[0] / (double)r[2]), ay = std::fabs((double)r[1] / (double)r[2]);
        axmin = ax < axmin ? ax : axmin; axmax = ax > axmax ? ax : axmax;
        aymin = ay < aymin ? ay : aymin; aymax = ay > aymax ? ay : aymax;
    }
    const double eps = 1.0 / 64.0, Q = (double)kDoomQ;
    plan[0] = fc.sun_k[0].r[0] > 0.0f ? 1 : -1;
    plan[1] = fc.sun_k[0].r[1] > 0.0f ? 1 : -1;
    plan[2] = (int)std::floor(Q * (axmin - eps)); plan[3] = (int)std::ceil(Q * (axmax + eps));
    plan[4] = (int)std::floor(Q * (aymin - eps)); plan[5] = (int)std::ceil(Q * (aymax + eps));
    int hm = 0;
    while (hm < kDoomHCap && doom_cross(hm + 1, plan[3], plan[5]) <= kDoomHCap &&
           1 + 2 * doom_cross(hm + 1, plan[3], plan[5]) < fc.max_steps)
        hm++;
    plan[6] = hm;
}
}  // namespace vx
