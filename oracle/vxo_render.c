/*
 * vxo_render.c — CPU ORACLE (test infrastructure only; see vxo.h header).
 * "parity unpinned" against reference outputs (none exist); pinned by the
 * hand-derived KATs in tests/test_oracle_kat.py.
 *
 * Scalar restatement of /root/reference/src/shaders/render.frag (+ render.h,
 * render.vert) and of the primary-visibility rule the raster of vertex.bin
 * implements (sdf.cpp:281-356 mesh + render.js:82-91 GL state).
 *
 * Numerical contract (shared with the HIP kernel):
 *   - fp32 everywhere, IEEE +,-,*,/ and sqrt, no FMA contraction
 *     (build with -O2 -fno-fast-math -ffp-contract=off);
 *   - GLSL built-ins restated from the GLSL ES 3.00 definitions
 *     (mix(x,y,a)=x*(1-a)+y*a, fract(x)=x-floor(x), min(x,y)=y<x?y:x, ...);
 *   - exp2/exp use vxo_exp2 (one fixed polynomial, both sides);
 *   - unorm8 texels decode to b/255 (then *255 == b exactly, checked);
 *   - textures sampled at LOD 0 with fp32 weights, nested lerp x->y->z.
 */
#include "vxo.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GLASS_INDEX 21 /* palette slot of glass: render.vert:21, sdf.cpp:195,337 */

/* ---------------- GLSL built-ins (GLSL ES 3.00 §8) ---------------- */
static inline float g_min(float x, float y) { return y < x ? y : x; }
static inline float g_max(float x, float y) { return x < y ? y : x; }
static inline float g_clamp(float x, float a, float b) { return g_min(g_max(x, a), b); }
static inline float g_fract(float x) { return x - floorf(x); }
static inline float g_sign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
static inline float g_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
/* ivec(float): NaN -> 0 (gfx v_cvt_i32_f32 behaviour), saturate far outside
 * any grid (such cells are out of bounds either way). */
static inline int g_f2i(float x) {
    if (x != x) return 0;
    if (x > 16777216.0f) return 16777216;
    if (x < -16777216.0f) return -16777216;
    return (int)x;
}

/* exp2 on [0,1) by a fixed degree-9 Taylor polynomial in f, scaled by 2^n.
 * GLSL leaves exp2's precision to the implementation (3+2|x| ulp); both the
 * oracle and the kernel use this one definition so they agree bit for bit. */
float vxo_exp2(float x) {
    if (x != x) return x;
    if (x >= 128.0f) return INFINITY;
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
static inline float g_exp(float x) { return vxo_exp2(x * 1.44269504f); }

/* ---------------- palette / normals (render.vert:14-22) ---------------- */
static const float PALETTE[22][3] = {
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
static void palette(int p, float out[3]) {
    if (p >= 0 && p < 22) { out[0] = PALETTE[p][0]; out[1] = PALETTE[p][1]; out[2] = PALETTE[p][2]; }
    else { out[0] = out[1] = out[2] = 1.0f; } /* render.vert:21 trailing vec3(1) */
}
void vxo_palette(float out[22][3]) {
    for (int p = 0; p < 22; p++) palette(p, out[p]);
}
static void normal_vec(int n, float out[3]) {
    out[0] = out[1] = out[2] = 0.0f;
    if (n >= 0 && n < 6) out[n >> 1] = (n & 1) ? -1.0f : 1.0f;
}

/* ---------------- texture access ---------------- */
static inline const uint8_t *texel(const vxo_scene *s, int x, int y, int z) {
    /* render.js:62 project_xyzc: C*(X*(Y*z + y) + x) */
    return s->field + 4 * ((size_t)x + (size_t)s->X * ((size_t)y + (size_t)s->Y * (size_t)z));
}
static inline float unorm(uint8_t b) { return (float)b / 255.0f; }

/* tex(ivec3) (render.frag:37-39): texelFetch(...).rgb * 255. */
static void tex_fetch(const vxo_scene *s, const int c[3], float rgb[3]) {
    const uint8_t *t = texel(s, c[0], c[1], c[2]);
    rgb[0] = unorm(t[0]) * 255.0f;
    rgb[1] = unorm(t[1]) * 255.0f;
    rgb[2] = unorm(t[2]) * 255.0f;
}

/* Linear sampling along one axis with CLAMP_TO_EDGE (render.js:200-203). */
static inline void lin_axis(float coord, int size, int *i0, int *i1, float *a) {
    float u = coord * (float)size - 0.5f;
    float fl = floorf(u);
    *a = u - fl;
    int i = g_f2i(fl);
    int j = i + 1;
    *i0 = i < 0 ? 0 : (i > size - 1 ? size - 1 : i);
    *i1 = j < 0 ? 0 : (j > size - 1 ? size - 1 : j);
}

/* tex(ivec3, vec3) (render.frag:40-42): texture(u_map, (vec3(c)+f)*Sf).rgb*255
 * at LOD 0, channels R and G (the only ones sdf() uses). */
static void tex_linear_rg(const vxo_scene *s, const int c[3], const float f[3], float rg[2]) {
    const float Sf[3] = {1.0f / (float)s->X, 1.0f / (float)s->Y, 1.0f / (float)s->Z};
    int i0[3], i1[3];
    float a[3];
    const int dims[3] = {s->X, s->Y, s->Z};
    for (int k = 0; k < 3; k++) {
        float coord = ((float)c[k] + f[k]) * Sf[k];
        lin_axis(coord, dims[k], &i0[k], &i1[k], &a[k]);
    }
    for (int ch = 0; ch < 2; ch++) {
        float v[2][2];
        for (int kz = 0; kz < 2; kz++)
            for (int ky = 0; ky < 2; ky++) {
                int yy = ky ? i1[1] : i0[1], zz = kz ? i1[2] : i0[2];
                float t0 = unorm(texel(s, i0[0], yy, zz)[ch]);
                float t1 = unorm(texel(s, i1[0], yy, zz)[ch]);
                v[kz][ky] = g_mix(t0, t1, a[0]);
            }
        float w0 = g_mix(v[0][0], v[0][1], a[1]);
        float w1 = g_mix(v[1][0], v[1][1], a[1]);
        rg[ch] = g_mix(w0, w1, a[2]) * 255.0f;
    }
}

/* sdf(ivec3, vec3) (render.frag:55-58): min(r, g) of the filtered field. */
static float sdf_lin(const vxo_scene *s, const int c[3], const float f[3]) {
    float rg[2];
    tex_linear_rg(s, c, f, rg);
    return g_min(rg[0], rg[1]);
}

/* REPEAT wrap of an integer-valued float onto [0,n) (n a power of two). */
static inline int wrap_idx(float fl, int n) {
    float q = floorf(fl / (float)n);
    return g_f2i(fl - q * (float)n) & (n - 1);
}

/* fbm(p) = noise(p).a = 1 - 2*texture(u_noise, p).a (render.frag:16-24),
 * bilinear, REPEAT (render.js:141-146), LOD 0. */
static float fbm(const vxo_scene *s, float px, float py) {
    const int W = s->noise_w, H = s->noise_h;
    float u = px * (float)W - 0.5f, v = py * (float)H - 0.5f;
    float fu = floorf(u), fv = floorf(v);
    float a = u - fu, b = v - fv;
    int x0 = wrap_idx(fu, W), y0 = wrap_idx(fv, H);
    int x1 = (x0 + 1) & (W - 1), y1 = (y0 + 1) & (H - 1);
    float t00 = unorm(s->noise[4 * ((size_t)y0 * W + x0) + 3]);
    float t10 = unorm(s->noise[4 * ((size_t)y0 * W + x1) + 3]);
    float t01 = unorm(s->noise[4 * ((size_t)y1 * W + x0) + 3]);
    float t11 = unorm(s->noise[4 * ((size_t)y1 * W + x1) + 3]);
    float r0 = g_mix(t00, t10, a), r1 = g_mix(t01, t11, a);
    float t = g_mix(r0, r1, b);
    return 1.0f - 2.0f * t;
}

/* white(p) = noise(p).rgb = 1 - 2*texture(u_noise, p).rgb (render.frag:16-21),
 * same bilinear REPEAT LOD-0 filter as fbm().  Used by the ROUGH extension. */
static void white(const vxo_scene *s, float px, float py, float out[3]) {
    const int W = s->noise_w, H = s->noise_h;
    float u = px * (float)W - 0.5f, v = py * (float)H - 0.5f;
    float fu = floorf(u), fv = floorf(v);
    float a = u - fu, b = v - fv;
    int x0 = wrap_idx(fu, W), y0 = wrap_idx(fv, H);
    int x1 = (x0 + 1) & (W - 1), y1 = (y0 + 1) & (H - 1);
    for (int ch = 0; ch < 3; ch++) {
        float t00 = unorm(s->noise[4 * ((size_t)y0 * W + x0) + ch]);
        float t10 = unorm(s->noise[4 * ((size_t)y0 * W + x1) + ch]);
        float t01 = unorm(s->noise[4 * ((size_t)y1 * W + x0) + ch]);
        float t11 = unorm(s->noise[4 * ((size_t)y1 * W + x1) + ch]);
        float r0 = g_mix(t00, t10, a), r1 = g_mix(t01, t11, a);
        out[ch] = 1.0f - 2.0f * g_mix(r0, r1, b);
    }
}

/* ---------------- march() (render.frag:75-142), literally ---------------- */
/* ex: the build's exit table for this direction (vxo_exit_plan), or NULL for
 * the reference's literal march.  A march entering a flagged cell ends "lit"
 * without fetching it, as the kernel's march does on the -1 its table holds. */
/* dm: the frame's doom table (vxo_field_doom: C, the crossings to the block,
 * per doomed cell) or NULL.  A march landing (index j) in a doomed cell whose
 * march texel T is >= 1 ends unlit there, without a fetch, if j + 2 C < MAX:
 * every ray of the window enters a solid cell h layers up after at most C
 * boundary crossings, and the march crosses one at least every two landings
 * (DESIGN.md §3 "Doom table"); otherwise it goes on with safe = T, no fetch
 * counted. */
static void march_ex(const vxo_scene *s, const int cell[3], const float fract[3],
                     const float r[3], int max_steps, vxo_march_t *res, const uint8_t *ex,
                     const uint8_t *dm) {
    res->step = 0;
    res->fetches = 0;
    res->cell[0] = cell[0]; res->cell[1] = cell[1]; res->cell[2] = cell[2];
    res->fract[0] = fract[0]; res->fract[1] = fract[1]; res->fract[2] = fract[2];
    res->min_dist = (float)s->Z;                     /* :82 */
    float m[3] = {0.0f, 0.0f, 0.0f};                 /* minAxisDir */
    float safe = 1.0f;                               /* :86 */
    const float dir = r[2] > 0.0f ? 1.0f : 0.0f;     /* :89 */
    const float sg[3] = {g_sign(r[0]), g_sign(r[1]), g_sign(r[2])};
    const float ar[3] = {fabsf(r[0]), fabsf(r[1]), fabsf(r[2])};
    while (res->step < max_steps && safe != 0.0f) {  /* :92 */
        float d[3], t[3];
        for (int i = 0; i < 3; i++) d[i] = g_fract(-res->fract[i] * sg[i]) + 1e-4f;   /* :94 */
        for (int i = 0; i < 3; i++) t[i] = d[i] / ar[i];                                /* :97 */
        m[0] = t[0] <= g_min(t[1], t[2]) ? 1.0f : 0.0f;                                 /* :100-104 */
        m[1] = t[1] <= g_min(t[2], t[0]) ? 1.0f : 0.0f;
        m[2] = t[2] <= g_min(t[0], t[1]) ? 1.0f : 0.0f;
        float v0 = m[0] * t[0], v1 = m[1] * t[1], v2 = m[2] * t[2];
        float len = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);                                 /* :105 */
        for (int i = 0; i < 3; i++) res->fract[i] += r[i] * safe * len;                /* :118 */
        for (int i = 0; i < 3; i++) {
            float fl = floorf(res->fract[i]);
            res->cell[i] += g_f2i(fl);                                                  /* :119 */
            res->fract[i] = res->fract[i] - fl;                                         /* :120 */
        }
        if (res->cell[0] >= s->X || res->cell[1] >= s->Y || res->cell[2] >= s->Z ||
            res->cell[0] < 0 || res->cell[1] < 0 || res->cell[2] < 0) {                 /* :123-126 */
            res->step = max_steps;
            break;
        }
        if (ex && ex[(size_t)res->cell[0] + (size_t)s->X * ((size_t)res->cell[1] + (size_t)s->Y * res->cell[2])]) {
            res->step = max_steps;                       /* exit table: lit, no fetch */
            break;
        }
        if (dm) {                                        /* doom table: unlit, no fetch (see above) */
            const size_t ci = (size_t)res->cell[0] + (size_t)s->X * ((size_t)res->cell[1] + (size_t)s->Y * res->cell[2]);
            const int T = s->field[4 * ci];              /* the march channel R (doom: r_z > 0) */
            if (dm[ci] && T >= 1) {
                if (res->step + 1 + 2 * (int)dm[ci] < max_steps) break;
                safe = (float)T;
                res->step++;
                continue;
            }
        }
        float rgb[3];
        tex_fetch(s, res->cell, rgb);                                                   /* :128 */
        res->fetches++;
        safe = g_mix(rgb[0], rgb[1], 1.0f - dir);                                       /* :47-50 */
        res->step++;                                                                    /* :135 */
    }
    for (int i = 0; i < 3; i++) res->normal[i] = -g_sign(r[i] * m[i]);                /* :139 */
}

void vxo_march(const vxo_scene *s, const int cell[3], const float fract[3],
               const float r[3], int max_steps, vxo_march_t *res) {
    march_ex(s, cell, fract, r, max_steps, res, NULL, NULL);
}

/* The build's choice of exit table per sample (DESIGN.md §3 "Sun exit
 * tables"), restated: a sample with some |r_i| < 2^-10 takes the literal path
 * (no table).  If every sample is on the fast path with one sign pattern,
 * r_z > 0 and slopes |r_x / r_z|, |r_y / r_z| <= 4 (double), all share the cone
 * table kx = ceil(max |r_x / r_z| + 1/64), ky likewise; otherwise each fast
 * sample reads the orthant table of its own octant. */
int vxo_exit_plan(const float dirs[][3], int n, int allow_cone, int oct[], int *kx, int *ky) {
    const float lim = 0.0009765625f;
    int all_fast = 1, same = 1;
    double ax = 0.0, ay = 0.0;
    for (int k = 0; k < n; k++) {
        const float *r = dirs[k];
        const int fast = fabsf(r[0]) >= lim && fabsf(r[1]) >= lim && fabsf(r[2]) >= lim;
        oct[k] = fast ? ((r[0] > 0.0f ? 1 : 0) | (r[1] > 0.0f ? 2 : 0) | (r[2] > 0.0f ? 4 : 0)) : -1;
        all_fast &= fast;
        if (k && oct[k] != oct[0]) same = 0;
        if (fast) {
            const double sx = fabs((double)r[0] / (double)r[2]), sy = fabs((double)r[1] / (double)r[2]);
            ax = sx > ax ? sx : ax;
            ay = sy > ay ? sy : ay;
        }
    }
    *kx = *ky = -1;
    if (!allow_cone || !all_fast || !same || !(oct[0] & 4) || ax > 4.0 || ay > 4.0) return 0;
    *kx = (int)ceil(ax + 1.0 / 64.0);
    *ky = (int)ceil(ay + 1.0 / 64.0);
    return 1;
}

/* ---------------- primary visibility ----------------
 * The reference rasterises the greedy mesh of sdf.cpp:281-356.  For each
 * colour c < pal_size (sdf.cpp:284) it has a face wherever a cell of colour c
 * borders a cell of another colour, oriented out of the c cell (ccol() clamps
 * at the grid edge, so the grid boundary has no faces), and GL culls back
 * faces (render.js:88-91).  Air is remapped to B = pal_size (sdf.cpp:19,188,
 * 229-233) and so is never meshed.  The visible surface at a pixel is
 * therefore the first step along the view ray that ENTERS a meshed cell
 * (vxo_vis(B) != 0) from a cell of another colour; the entered cell gives
 * colour and id.  Glass (index 21) is drawn last and blended
 * (render.js:84-86): leaving glass into air is no face, so glass blends over
 * the next entry behind it.  Several glass layers blend in mesh order in the
 * reference (order-dependent); the build defines one layer: later glass
 * entries are skipped (the reference's result when the nearer pane is drawn
 * first and its depth write hides the farther one).
 *
 * Traversal ("box-exit" stepping): from the current cell c, the ray's octant
 * (direction signs s, zero counted positive) has the all-air cube
 * B = [c, c + R*s] ahead of c (R = vxo_field_octant), so the ray jumps straight
 * to the face where it leaves B: per axis the crossing time of the far face
 * (c + R + 1 for s > 0, c - R for s < 0), the earliest one (ties x, then y,
 * then z) is the exit axis; the next cell is one past B on that axis and
 * floor() of the exit point, clamped into B, on the others.  With R = 0 (next
 * to or inside a non-air cell) B is the cell itself: an exact DDA step.
 * Camera-relative cells keep the fp32 coordinates small.
 */
static inline int in_grid(const vxo_scene *s, const int a[3]) {
    return a[0] >= 0 && a[1] >= 0 && a[2] >= 0 && a[0] < s->X && a[1] < s->Y && a[2] < s->Z;
}

/* The pane a draw-order scan looks for (glass_layer 3): the front-facing glass
 * face with the smallest draw key above klast (any key if !have_last) among
 * those nearer than tmax. */
typedef struct {
    int have_last;
    uint64_t klast;
    float tmax;
} glass_sel;

/* Octant-box walk of the ray B + o + t*d (B an integer cell, camera- or
 * origin-relative cells c) from the start cell B + c to the first colour
 * change: from cell c the box [c, c + e*s] (vxo_field_box extents of the ray
 * octant) is all air, so the ray jumps to where it leaves the box.
 * glass_layer 1: the first glass entry is recorded and the walk goes on to
 * the next change behind it (primary visibility); 0: the first change ends the
 * walk (reflection rays); 3: a draw-order scan (sel): every glass entry before
 * the first opaque one is a candidate, the one sel picks is g[0], and the
 * return is 1 if there is one.  A start cell outside the grid is sky. */
static int walk(const vxo_scene *s, const int cc[3], const float o[3], const float d[3], int c[3],
                int glass_layer, vxo_gbuf g[2], int *fetches, int *cap_hit, int *glass_entries, int quad,
                const glass_sel *sel) {
    const int dims[3] = {s->X, s->Y, s->Z};
    float inv[3];
    int stp[3];
    for (int i = 0; i < 3; i++) {
        stp[i] = d[i] > 0.0f ? 1 : -1;
        inv[i] = d[i] != 0.0f ? 1.0f / d[i] : 0.0f;
    }
    int abs_c[3] = {c[0] + cc[0], c[1] + cc[1], c[2] + cc[2]};
    if (!in_grid(s, abs_c)) return 0;
    const uint8_t *tx = texel(s, abs_c[0], abs_c[1], abs_c[2]);
    (*fetches)++;
    const int oct = (d[0] < 0.0f ? 1 : 0) | (d[1] < 0.0f ? 2 : 0) | (d[2] < 0.0f ? 4 : 0);
    const uint8_t *octe = s->oct_e[oct];
#define OCT_E(a, e)                                                                                  \
    do {                                                                                             \
        const uint8_t *p_ = octe + 3 * ((size_t)(a)[0] + (size_t)s->X * ((size_t)(a)[1] + (size_t)s->Y * (size_t)(a)[2])); \
        (e)[0] = p_[0]; (e)[1] = p_[1]; (e)[2] = p_[2];                                              \
    } while (0)
    int prev = vxo_vis(tx[2]);
    int E[3];
    OCT_E(abs_c, E);
    int nrec = 0;
    const int cap = 4 * (dims[0] + dims[1] + dims[2]);
    for (int iter = 0; iter < cap; iter++) {
        float tb[3];
        for (int i = 0; i < 3; i++)
            tb[i] = d[i] != 0.0f ? ((float)(c[i] + (stp[i] > 0 ? E[i] + 1 : -E[i])) - o[i]) * inv[i] : INFINITY;
        const int a = (tb[0] <= tb[1] && tb[0] <= tb[2]) ? 0 : (tb[1] <= tb[2] ? 1 : 2);
        const float te = tb[a];
        for (int i = 0; i < 3; i++) {
            if (i == a) {
                c[i] = c[i] + stp[i] * (E[i] + 1);
            } else {
                const int v = g_f2i(floorf(o[i] + te * d[i]));
                const int lo = d[i] < 0.0f ? c[i] - E[i] : c[i], hi = d[i] < 0.0f ? c[i] : c[i] + E[i];
                c[i] = v < lo ? lo : (v > hi ? hi : v);
            }
        }
        abs_c[0] = c[0] + cc[0]; abs_c[1] = c[1] + cc[1]; abs_c[2] = c[2] + cc[2];
        if (!in_grid(s, abs_c)) return nrec;   /* left the grid: sky behind (scan: the pane found, if any) */
        tx = texel(s, abs_c[0], abs_c[1], abs_c[2]);
        (*fetches)++;
        const int col = vxo_vis(tx[2]);
        OCT_E(abs_c, E);                           /* air box ahead */
        if (glass_entries && col == GLASS_INDEX && prev != GLASS_INDEX) (*glass_entries)++;
        /* a front face: entering a meshed cell from a cell of another colour
         * (air is never meshed, sdf.cpp:229-233,284); glass_layer 1: the
         * first glass entry is recorded and the walk goes on, later glass
         * entries are passed (render_pixel blends them in draw order) */
        if (glass_layer == 3 && col != prev && col != 0 && col != GLASS_INDEX) return nrec;
        if (col != prev && col != 0 && !(glass_layer == 1 && col == GLASS_INDEX && nrec == 1)) {
            vxo_gbuf cand;
            vxo_gbuf *h = glass_layer == 3 ? &cand : &g[nrec];
            h->color = col;
            h->id = col == GLASS_INDEX ? 2 : 0;
            h->normal_idx = 2 * a + (stp[a] > 0 ? 1 : 0);
            /* quad-relative G-buffer (render.vert:25-28): v_cellPos = the origin of
             * the greedy quad covering the face, v_fractPos = the hit point minus
             * it, rounded once (the unit cell's split rounds p - c the same way) */
            int off[3] = {0, 0, 0};
            uint16_t q = VXO_NO_FACE;
            if (s->qoff)
                q = s->qoff[6 * ((size_t)abs_c[0] + (size_t)s->X * ((size_t)abs_c[1] + (size_t)s->Y * (size_t)abs_c[2])) +
                            (size_t)h->normal_idx];
            if (quad && q != VXO_NO_FACE) {
                off[(a + 1) % 3] = q & 0xff;
                off[(a + 2) % 3] = q >> 8;
            }
            h->t = te;
            h->key = q != VXO_NO_FACE ? vxo_face_order(abs_c, h->normal_idx, q, s->X, s->Y, s->Z, s->chunk) : 0;
            for (int i = 0; i < 3; i++) {
                if (i == a) {
                    h->cell[i] = abs_c[i] + (stp[a] > 0 ? 0 : 1);
                    h->fract[i] = 0.0f;
                } else {
                    float p = o[i] + te * d[i];
                    h->cell[i] = abs_c[i] - off[i];
                    h->fract[i] = p - (float)(c[i] - off[i]);
                }
            }
            if (glass_layer == 3) {
                if ((!sel->have_last || h->key > sel->klast) && h->t < sel->tmax && (!nrec || h->key < g[0].key)) {
                    g[0] = cand;
                    nrec = 1;
                }
            } else {
                nrec++;
                if (!glass_layer || h->id != 2) return nrec;
            }
        }
        prev = col;
    }
    *cap_hit = 1;
    return nrec;
#undef OCT_E
}

static int primary_walk(const vxo_scene *s, const vxo_frame *f, const float d[3], int glass_layer, vxo_gbuf *g,
                        int *fetches, int *cap_hit, int *glass_entries, const glass_sel *sel) {
    const int dims[3] = {s->X, s->Y, s->Z};
    const float *o = f->cam_fract;
    const int *cc = f->cam_cell;
    float tlo = 0.0f, thi = INFINITY;
    *fetches = 0;
    *cap_hit = 0;
    for (int i = 0; i < 3; i++) {        /* ray / grid AABB */
        float lo = (float)(0 - cc[i]) - o[i];
        float hi = (float)(dims[i] - cc[i]) - o[i];
        if (d[i] != 0.0f) {
            float inv = 1.0f / d[i];
            float t0 = lo * inv, t1 = hi * inv;
            if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
            tlo = g_max(tlo, t0);
            thi = g_min(thi, t1);
        } else {
            if (!(lo <= 0.0f && 0.0f < hi)) return 0;
        }
    }
    if (!(tlo < thi)) return 0;

    int c[3];                            /* camera-relative cell */
    for (int i = 0; i < 3; i++) {
        float p = o[i] + tlo * d[i];
        int ci = g_f2i(floorf(p));
        int lo = -cc[i], hi = dims[i] - cc[i] - 1;
        c[i] = ci < lo ? lo : (ci > hi ? hi : ci);
    }
    const int quad = !s->unit_split && !(f->flags & VXO_FLAG_UNIT_GBUF);
    return walk(s, cc, o, d, c, glass_layer, g, fetches, cap_hit, glass_entries, quad, sel);
}

int vxo_primary(const vxo_scene *s, const vxo_frame *f, const float d[3],
                vxo_gbuf g[2], int *fetches, int *cap_hit) {
    return primary_walk(s, f, d, 1, g, fetches, cap_hit, NULL, NULL);
}

/* Diagnostic (the single-layer glass deviation): per pixel, the
 * number of front-facing glass faces the view ray crosses before its opaque
 * surface or the grid exit -- the glass entries of vxo_primary's walk.  The
 * reference blends each of them in draw order (render.js:82-86, glass drawn
 * last, sdf.cpp:284,337); the build blends the first one only, so pixels with
 * 2 or more are where the two can differ. */
void vxo_glass_layers(const vxo_scene *s, const vxo_frame *f, int w, int h, uint8_t *out, int n_threads) {
    (void)n_threads;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int py = 0; py < h; py++)
        for (int px = 0; px < w; px++) {
            float d[3];
            vxo_pixel_dir(f, w, h, px, py, d);
            const int dims[3] = {s->X, s->Y, s->Z};
            const float *o = f->cam_fract;
            const int *cc = f->cam_cell;
            float tlo = 0.0f, thi = INFINITY;
            int miss = 0, n = 0;
            for (int i = 0; i < 3; i++) {
                float lo = (float)(0 - cc[i]) - o[i], hi = (float)(dims[i] - cc[i]) - o[i];
                if (d[i] != 0.0f) {
                    float inv = 1.0f / d[i], t0 = lo * inv, t1 = hi * inv;
                    if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
                    tlo = g_max(tlo, t0);
                    thi = g_min(thi, t1);
                } else if (!(lo <= 0.0f && 0.0f < hi)) miss = 1;
            }
            if (!miss && tlo < thi) {
                int c[3], fetches = 0, cap = 0;
                for (int i = 0; i < 3; i++) {
                    int ci = g_f2i(floorf(o[i] + tlo * d[i]));
                    int lo = -cc[i], hi = dims[i] - cc[i] - 1;
                    c[i] = ci < lo ? lo : (ci > hi ? hi : ci);
                }
                vxo_gbuf g[2];       /* (the grid boundary has no faces: a glass start cell is no entry) */
                walk(s, cc, o, d, c, 1, g, &fetches, &cap, &n, 0, NULL);
            }
            out[(size_t)py * w + px] = (uint8_t)(n > 255 ? 255 : n);
        }
}

void vxo_pixel_dir(const vxo_frame *f, int w, int h, int px, int py, float d[3]) {
    float nx = (float)(2 * px + 1) / (float)w - 1.0f;
    float ny = 1.0f - (float)(2 * py + 1) / (float)h;
    for (int i = 0; i < 3; i++) d[i] = (f->ray_fwd[i] + nx * f->ray_right[i]) + ny * f->ray_up[i];
}

/* ---------------- extensions (DESIGN.md §3 "Extensions") -------
 * The reference has no code for these (README.md:15-22 describes reflections
 * and rough normals of an earlier renderer, :56-57 lists soft shadows as to-do);
 * the definitions below are this build's, shared with the kernel. */

/* cos/sin of k * golden angle, k = 0..15 (Vogel spiral) as double literals,
 * so no libm trigonometry enters the sample directions. */
static const double VOGEL_CS[VXO_MAX_SAMPLES][2] = {
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

/* Soft-shadow directions: sample k of n is the sun direction pushed by
 * radius * sqrt((k + 0.5) / n) along the spiral angle of k in the plane
 * normal to the sun (basis u = normalize(a x sun), v = sun x u with
 * a = z unless the sun is within ~25 degrees of it, then x), normalised;
 * double precision (+ - * / sqrt only), rounded to float. */
void vxo_sun_samples(const float sun[3], float radius, int n, float out[][3]) {
    if (n <= 1) {
        out[0][0] = sun[0]; out[0][1] = sun[1]; out[0][2] = sun[2];
        return;
    }
    if (n > VXO_MAX_SAMPLES) n = VXO_MAX_SAMPLES;
    const double sd[3] = {sun[0], sun[1], sun[2]};
    const double ax[3] = {fabs(sd[2]) < 0.9 ? 0.0 : 1.0, 0.0, fabs(sd[2]) < 0.9 ? 1.0 : 0.0};
    double u[3] = {ax[1] * sd[2] - ax[2] * sd[1], ax[2] * sd[0] - ax[0] * sd[2], ax[0] * sd[1] - ax[1] * sd[0]};
    const double ul = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    u[0] /= ul; u[1] /= ul; u[2] /= ul;
    const double v[3] = {sd[1] * u[2] - sd[2] * u[1], sd[2] * u[0] - sd[0] * u[2], sd[0] * u[1] - sd[1] * u[0]};
    for (int k = 0; k < n; k++) {
        const double r = (double)radius * sqrt(((double)k + 0.5) / (double)n);
        const double cu = r * VOGEL_CS[k][0], cv = r * VOGEL_CS[k][1];
        double x[3];
        for (int i = 0; i < 3; i++) x[i] = sd[i] + cu * u[i] + cv * v[i];
        const double l = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
        for (int i = 0; i < 3; i++) out[k][i] = (float)(x[i] / l);
    }
}

#define ROUGH_SCALE 0.00390625f   /* 1/256: 4 noise texels per voxel on a 1024 texture */
#define ROUGH_AMP 0.1f

/* ROUGH: the shading normal of a face fragment is normalize(n + 0.1 * white(p))
 * with p the fragment's two in-face coordinates (axes other than the face
 * axis, in increasing order) times 1/256. */
static void rough_normal(const vxo_scene *s, const vxo_gbuf *g, const float n[3], float out[3]) {
    const int a = g->normal_idx >> 1;
    const int t1 = a == 0 ? 1 : 0, t2 = a == 2 ? 1 : 2;
    const float u = (float)g->cell[t1] + g->fract[t1], v = (float)g->cell[t2] + g->fract[t2];
    float w[3], m[3];
    white(s, u * ROUGH_SCALE, v * ROUGH_SCALE, w);
    for (int i = 0; i < 3; i++) m[i] = n[i] + ROUGH_AMP * w[i];
    float l = sqrtf(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
    out[0] = m[0] / l; out[1] = m[1] / l; out[2] = m[2] / l;
}

/* Diagnostic recorder (vxo_march_lengths): the fetch count of every sun march
 * of the pixel being rendered, in order.  Thread-local; NULL = off. */
static _Thread_local int *g_rec;
static _Thread_local int g_rec_n, g_rec_cap;
static inline void rec_march(int fetches) {
    if (g_rec && g_rec_n < g_rec_cap) g_rec[g_rec_n++] = fetches;
}

/* Diagnostic recorder (vxo_render_terms): the sun-march result and AO distance
 * of the fragment being shaded into slot g_term_slot (-1 = none).  Thread-local. */
static _Thread_local uint8_t *g_term_lit;
static _Thread_local float *g_term_amb;
static _Thread_local int g_term_slot = -1;

/* Per-frame state derived once (the kernel's FrameConsts play this role). */
typedef struct {
    const vxo_scene *s;
    const vxo_frame *f;
    int max_steps;
    int n_sun;                               /* >= 2: soft shadows */
    float sun_dirs[VXO_MAX_SAMPLES][3];
    const uint8_t *ex[VXO_MAX_SAMPLES];      /* exit table per sample (exit_mode), else NULL */
    uint8_t *owned[VXO_MAX_SAMPLES];
    int n_owned;
    const uint8_t *doom;                     /* the cone plan's doom table (vxo_field_doom), else NULL */
    uint8_t *doom_owned;
} shade_ctx;

static void ctx_init(shade_ctx *c, const vxo_scene *s, const vxo_frame *f) {
    c->s = s;
    c->f = f;
    c->max_steps = f->max_shadow_steps > 0 ? f->max_shadow_steps : 2 * s->Z;
    c->n_sun = f->shadow_samples > 1 ? (f->shadow_samples > VXO_MAX_SAMPLES ? VXO_MAX_SAMPLES : f->shadow_samples) : 1;
    vxo_sun_samples(f->sun_dir, f->sun_radius, c->n_sun, c->sun_dirs);
    c->n_owned = 0;
    for (int k = 0; k < VXO_MAX_SAMPLES; k++) c->ex[k] = NULL;
    c->doom = NULL;
    c->doom_owned = NULL;
}

/* the frame's exit tables (vxo_render only: a table is a pass over the field) */
static void ctx_tables(shade_ctx *c) {
    const vxo_scene *s = c->s;
    if (!s->exit_mode) return;
    int oct[VXO_MAX_SAMPLES], kx, ky, key[VXO_MAX_SAMPLES];
    /* the kernel's cone copies need Z >= 3 (their window inside its -1 border) */
    const int cone = vxo_exit_plan((const float(*)[3])c->sun_dirs, c->n_sun, s->exit_mode == 1 && s->Z >= 3, oct,
                                   &kx, &ky);
    if (cone && !(c->f->flags & (VXO_FLAG_NO_DOOM | VXO_FLAG_SOFT_BRICK))) {
        int p[7];
        vxo_doom_plan((const float(*)[3])c->sun_dirs, c->n_sun, c->max_steps, p);
        if (p[6] < 1) {
            /* no h can meet the stop rule at this MAX: no table */
        } else if (s->held_doom && !memcmp(p, s->held_dplan, sizeof p)) {
            c->doom = s->held_doom;
        } else {
            c->doom_owned = (uint8_t *)malloc((size_t)s->X * s->Y * s->Z);
            vxo_field_doom(s->field, s->X, s->Y, s->Z, p, c->doom_owned);
            c->doom = c->doom_owned;
        }
    }
    for (int k = 0; k < c->n_sun; k++) {
        if (oct[k] < 0) continue;
        int found = -1;
        for (int j = 0; j < c->n_owned; j++)
            if (key[j] == oct[k]) found = j;
        if (found < 0 && s->held && s->held_oct == oct[k] && s->held_kx == kx && s->held_ky == ky) {
            c->ex[k] = s->held;
            continue;
        }
        if (found < 0) {
            uint8_t *t = (uint8_t *)malloc((size_t)s->X * s->Y * s->Z);
            vxo_field_exit(s->field, s->X, s->Y, s->Z, oct[k], kx, ky, t);
            key[c->n_owned] = oct[k];
            c->owned[c->n_owned] = t;
            found = c->n_owned++;
        }
        c->ex[k] = c->owned[found];
    }
}

static void ctx_free(shade_ctx *c) {
    for (int j = 0; j < c->n_owned; j++) free(c->owned[j]);
    c->n_owned = 0;
    free(c->doom_owned);
    c->doom_owned = NULL;
}

/* ---------------- main() (render.frag:147-252) ----------------
 * ray: NULL = the camera ray to the fragment (:154); for sky records the
 * direction to normalise (the skybox is at infinity); for surfaces seen in a
 * reflection the (unit) reflected ray.  ray_used receives rayDir. */
static inline float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void normalize3(const float v[3], float out[3]) {
    float l = sqrtf(dot3(v, v));
    out[0] = v[0] / l; out[1] = v[1] / l; out[2] = v[2] / l;
}

static void shade_frag(const shade_ctx *c, const vxo_gbuf *g, const float ray[3], float o_color[4],
                       float ray_used[3], vxo_stats *st) {
    const vxo_scene *s = c->s;
    const vxo_frame *f = c->f;
    o_color[0] = 0.0f; o_color[1] = 0.0f; o_color[2] = 0.0f; o_color[3] = 1.0f;    /* :148 */
    const int isSky = g->id == 1, isGlass = g->id == 2;                            /* :150-151 */
    const float litCol[3] = {0.4f, 0.35f, 0.3f};                                   /* :153 */
    float v_normal[3], v_color[3];
    normal_vec(isSky ? 1 : g->normal_idx, v_normal);   /* sky quads carry normal 1 (sdf.cpp:249-278) */
    palette(isSky ? 0 : g->color, v_color);
    float rayDir[3];
    if (isSky) {
        normalize3(ray, rayDir);        /* skybox modelled at infinity */
    } else if (ray) {
        rayDir[0] = ray[0]; rayDir[1] = ray[1]; rayDir[2] = ray[2];   /* ext REFLECT: reflected ray */
    } else {
        float v[3];
        for (int i = 0; i < 3; i++)
            v[i] = (float)(g->cell[i] - f->cam_cell[i]) + (g->fract[i] - f->cam_fract[i]);   /* :154 */
        normalize3(v, rayDir);
    }
    if (ray_used) { ray_used[0] = rayDir[0]; ray_used[1] = rayDir[1]; ray_used[2] = rayDir[2]; }
    /* ext ROUGH: shading normal; geometry (AO offset, march start) keeps v_normal */
    float nrm[3] = {v_normal[0], v_normal[1], v_normal[2]};
    if (!isSky && (f->flags & VXO_FLAG_ROUGH)) {
        rough_normal(s, g, v_normal, nrm);
        if (st) st->rough_px++;
    }
    float reflectDir[3];                                                           /* :155 reflect() */
    {
        float k = 2.0f * dot3(nrm, rayDir);
        for (int i = 0; i < 3; i++) reflectDir[i] = rayDir[i] - k * nrm[i];
    }
    const float *sunDir = f->sun_dir;                                              /* :157 */
    const float sunCol[3] = {1.4f, 1.0f, 0.5f};                                    /* :162 */
    float sunFactor = g_max(0.0f, dot3(f->sun_dir, rayDir)) - 1.0f;                /* :163 */
    float glow = vxo_exp2(8.0f * sunFactor);                                       /* :164 */
    sunFactor = vxo_exp2(4000.0f * sunFactor) + 0.3f * glow;                       /* :165 */
    float scatter = 1.0f - sqrtf(g_max(0.0f, sunDir[2]));                          /* :168 */
    const float sp0[3] = {0.2f, 0.4f, 0.7f}, sp1[3] = {0.2f, 0.3f, 0.5f};
    const float sc0[3] = {0.7f, 0.9f, 1.0f}, sc1[3] = {1.0f, 0.3f, 0.2f};
    float spaceCol[3], scatterCol[3], atmCol[3], skyCol[3];
    float rz = sqrtf(g_max(0.0f, reflectDir[2]));
    for (int i = 0; i < 3; i++) {
        spaceCol[i] = g_mix(sp0[i], sp1[i], scatter);                               /* :169 */
        scatterCol[i] = g_mix(sc0[i], sc1[i], scatter);                             /* :170 */
        atmCol[i] = g_mix(scatterCol[i], spaceCol[i], rz);                          /* :171 */
        skyCol[i] = sunCol[i] * sunFactor + atmCol[i];                              /* :173 */
        skyCol[i] = g_clamp(skyCol[i], 0.0f, 1.0f);                                 /* :176 */
    }
    if (isSky) {                                                                   /* :178 */
        rayDir[2] = fabsf(rayDir[2]);                                               /* :179 */
        if (f->flags & 0x4u) {   /* VX_FLAG_NO_CLOUDS: plain sky colour */
            o_color[0] = skyCol[0]; o_color[1] = skyCol[1]; o_color[2] = skyCol[2];
            return;
        }
        if (st) st->noise_px++;
        float cloudCol[3];
        float cloudTime = f->time * 4e-3f;                                          /* :183 */
        float den = sqrtf(fabsf(rayDir[2]) + 0.03f);
        float sx = rayDir[0] / den, sy = rayDir[1] / den;                           /* :184 */
        sx = sx * 0.1f; sy = sy * 0.1f;                                             /* :185 */
        float sl = sqrtf(sqrtf(sx * sx + sy * sy));
        sx = sx * sl; sy = sy * sl;                                                 /* :186 */
        float n0 = fbm(s, 2.0f * sx + cloudTime, 2.0f * sy + cloudTime);            /* :188 */
        float n1 = fbm(s, 2.0f * sx - cloudTime, 2.0f * sy - cloudTime);            /* :189 */
        sx = sx * (3.0f + n0); sy = sy * (3.0f + n1);                               /* :187-190 */
        sx = sx + 1e-4f * ((float)f->cam_cell[0] + f->cam_fract[0]);                /* :191 */
        sy = sy + 1e-4f * ((float)f->cam_cell[1] + f->cam_fract[1]);
        float cloudFactor = vxo_exp2(6.0f * (fbm(s, sx + 2.0f * cloudTime, sy + -9.0f * cloudTime) - 1.0f)); /* :192 */
        float scf = sqrtf(cloudFactor);
        for (int i = 0; i < 3; i++) cloudCol[i] = g_mix(sunCol[i], 0.8f, scf);     /* :193 */
        float mountainPos = rayDir[0] / rayDir[1];                                  /* :195 */
        float mountainHeight = 1.0f - fbm(s, 0.3f * mountainPos, 0.3f * mountainPos); /* :196 */
        float mountainFactor = 2.0f - fbm(s, 2.0f * (mountainPos + rayDir[1]),
                                          2.0f * (mountainPos + rayDir[2]));         /* :197 */
        mountainHeight = mountainHeight / (g_exp(0.3f * mountainPos * mountainPos) * 6.0f); /* :198 */
        if (mountainHeight > rayDir[2] && rayDir[1] > 0.0f && rayDir[2] > 0.0f) {   /* :199 */
            const float mt[3] = {0.7f, 0.8f, 0.7f};
            float a = mountainFactor * rayDir[2];
            for (int i = 0; i < 3; i++) skyCol[i] = g_mix(skyCol[i], skyCol[i] * mt[i], a); /* :200 */
        } else {
            for (int i = 0; i < 3; i++) skyCol[i] = g_mix(skyCol[i], cloudCol[i], cloudFactor); /* :202 */
        }
        o_color[0] = skyCol[0]; o_color[1] = skyCol[1]; o_color[2] = skyCol[2];    /* :205 */
        return;
    }
    /* block branch :207-251 */
    const float *baseCol = v_color;                                                 /* :209 */
    float an[3] = {fabsf(nrm[0]), fabsf(nrm[1]), fabsf(nrm[2])};
    const float M0[3] = {0.90f, 0.90f, 0.95f}, M1[3] = {0.95f, 0.95f, 1.00f}, M2[3] = {1.0f, 1.0f, 1.0f};
    float normalCol[3];
    for (int i = 0; i < 3; i++) normalCol[i] = (M0[i] * an[0] + M1[i] * an[1]) + M2[i] * an[2]; /* :211-215 */
    if (nrm[2] < 0.0f)                                                              /* :217 */
        for (int i = 0; i < 3; i++) normalCol[i] = normalCol[i] * 0.8f;
    float shadeCol[3];
    for (int i = 0; i < 3; i++) shadeCol[i] = 0.7f * scatterCol[i];                 /* :220 */
    float ambCol[3] = {1.0f, 1.0f, 1.0f};
    if (!(f->flags & 0x2u)) {   /* VX_FLAG_NO_AO skips the sample */
        if (st) st->ao_samples++;
        int ac[3];
        for (int i = 0; i < 3; i++) ac[i] = g->cell[i] + g_f2i(v_normal[i]);
        float ambDist = sdf_lin(s, ac, g->fract);                                   /* :223 */
        if (g_term_amb && g_term_slot >= 0) g_term_amb[g_term_slot] = ambDist;
        float ambFactor = g_min(1.0f - sqrtf(ambDist), 0.8f);                       /* :224 */
        for (int i = 0; i < 3; i++) ambCol[i] = g_mix(1.0f, shadeCol[i], ambFactor); /* :225 */
    }
    float shadeFactor = f->sun_dir[2] < 0.0f ? 0.0f
                        : sqrtf(g_max(0.0f, dot3(nrm, f->sun_dir)));                /* :228-229 */
    if (shadeFactor > 0.0f && !(f->flags & 0x1u)) {  /* :232; VX_FLAG_NO_SHADOW skips */
        vxo_march_t sun;
        if (c->n_sun <= 1) {
            march_ex(s, g->cell, g->fract, sunDir, c->max_steps, &sun, c->ex[0], c->doom);   /* :233 */
            shadeFactor = shadeFactor * (sun.step == c->max_steps ? 1.0f : 0.0f);   /* :234 */
            if (st) { st->shadow_rays++; st->shadow_fetches += (uint64_t)sun.fetches; }
            rec_march(sun.fetches | (sun.step == c->max_steps ? 1 << 16 : 0));
        } else {                 /* ext soft shadows: lit fraction of the sun samples */
            int lit = 0;
            for (int k = 0; k < c->n_sun; k++) {
                march_ex(s, g->cell, g->fract, c->sun_dirs[k], c->max_steps, &sun, c->ex[k], c->doom);
                lit += sun.step == c->max_steps ? 1 : 0;
                if (st) { st->shadow_rays++; st->shadow_fetches += (uint64_t)sun.fetches; }
                rec_march(sun.fetches | (sun.step == c->max_steps ? 1 << 16 : 0));
            }
            shadeFactor = shadeFactor * ((float)lit / (float)c->n_sun);
            if (g_term_lit && g_term_slot >= 0) g_term_lit[g_term_slot] = (uint8_t)lit;
        }
        if (g_term_lit && g_term_slot >= 0 && c->n_sun <= 1) g_term_lit[g_term_slot] = sun.step == c->max_steps;
    }
    float lightCol[3];
    for (int i = 0; i < 3; i++) lightCol[i] = shadeCol[i] + litCol[i] * shadeFactor; /* :238 */
    for (int i = 0; i < 3; i++) o_color[i] = baseCol[i];                            /* :241 */
    if (f->quality > 0)                                                             /* :242-244 */
        for (int i = 0; i < 3; i++) o_color[i] = o_color[i] * ((normalCol[i] * lightCol[i]) * ambCol[i]);
    if (isGlass) {                                                                  /* :246-249 */
        o_color[3] = 0.8f * vxo_exp2(dot3(rayDir, nrm));
        for (int i = 0; i < 3; i++) o_color[i] = o_color[i] * (0.2f * atmCol[i]);
    }
}

void vxo_shade(const vxo_scene *s, const vxo_frame *f, const vxo_gbuf *g,
               const float prim_dir[3], float o_color[4], vxo_stats *st) {
    shade_ctx c;
    ctx_init(&c, s, f);
    shade_frag(&c, g, g->id == 1 ? prim_dir : NULL, o_color, NULL, st);
}

static void sky_record(vxo_gbuf *sky) {
    memset(sky, 0, sizeof *sky);
    sky->id = 1;
    sky->normal_idx = 1;
}

/* ext REFLECT: colour seen along the mirror reflection of the camera ray at a
 * glass fragment (geometric normal: R = rayDir with the face-axis component
 * negated, exactly reflect(rayDir, n)).  The ray starts on the face, in the
 * cell on the camera's side, and walks the octant cubes to the first colour
 * change; the surface found is shaded as a fragment seen along R (its own AO,
 * sun march, rough normal; no further reflection), a miss is the sky along R. */
static void reflect_color(const shade_ctx *c, const vxo_gbuf *gl, const float rd[3], float out[3],
                          vxo_stats *st) {
    const int a = gl->normal_idx >> 1;
    float R[3] = {rd[0], rd[1], rd[2]};
    R[a] = -R[a];
    int B[3], c0[3];
    float o[3];
    for (int i = 0; i < 3; i++) {
        if (i == a) {
            B[i] = gl->cell[i];
            o[i] = 0.0f;
            c0[i] = R[i] > 0.0f ? 0 : -1;
        } else {
            const float fl = floorf(gl->fract[i]);
            B[i] = gl->cell[i] + g_f2i(fl);
            o[i] = gl->fract[i] - fl;
            c0[i] = 0;
        }
    }
    vxo_gbuf h[2];
    int fetches = 0, cap_hit = 0;
    const int n = walk(c->s, B, o, R, c0, 0, h, &fetches, &cap_hit, NULL, 0, NULL);
    if (st) { st->reflect_rays++; st->reflect_fetches += (uint64_t)fetches; st->primary_cap_hits += (uint64_t)cap_hit; }
    float rgba[4];
    if (n == 0) {
        vxo_gbuf sky;
        sky_record(&sky);
        shade_frag(c, &sky, R, rgba, NULL, st);
    } else {
        shade_frag(c, &h[0], R, rgba, NULL, st);
    }
    out[0] = rgba[0]; out[1] = rgba[1]; out[2] = rgba[2];
}

/* ext REFLECT / REFLECT_ALL: rgb += F * the colour along the mirror ray, Schlick's
 * Fresnel with F0 = 0.04 on the geometric normal (cos = |rayDir| along the face axis) */
static void add_reflection(const shade_ctx *c, const vxo_gbuf *g, const float rd[3], float rgb[3], vxo_stats *st) {
    float refl[3];
    reflect_color(c, g, rd, refl, st);
    const float cs = g_min(fabsf(rd[g->normal_idx >> 1]), 1.0f);
    const float x = 1.0f - cs, x2 = x * x;
    const float F = 0.04f + 0.96f * ((x2 * x2) * x);
    for (int i = 0; i < 3; i++) rgb[i] = rgb[i] + F * refl[i];
}

/* The GL blend stage.  Every draw blends SRC_ALPHA / ONE_MINUS_SRC_ALPHA
 * (render.js:84-86) into the default framebuffer, an RGBA8 canvas (map.js:7,
 * {alpha: false}).  For a fixed-point colour buffer GLES 3.0 §4.1.7 clamps the
 * source, the destination and the blend factors to [0, 1] before the blend
 * equation, and the destination is what the 8-bit buffer holds: the colour
 * written before, stored as round(clamp(v) * 255) (the build's RGBA8 store,
 * pack_rgba8: floor(clamp(v) * 255 + 0.5) in fp32).  An opaque fragment has
 * alpha 1 and simply replaces the pixel.  So a pane turns the colour dst
 * written before it into clamp(src) * a + canvas8(dst) * (1 - a), a =
 * clamp(src.a); the next pane reads that back through canvas8 again, and the
 * RGBA8 frame stores the last one (the fp32 frame keeps it unquantised).
 * VXO_FLAG_BLEND_FLOAT: the round-5 fp32 blend (diagnostic). */
static inline float canvas8(float v) { return floorf(g_clamp(v, 0.0f, 1.0f) * 255.0f + 0.5f) / 255.0f; }
static void blend_canvas(const float src[4], float dst[3], unsigned flags) {
    if (flags & VXO_FLAG_BLEND_FLOAT) {
        const float a = src[3];
        for (int i = 0; i < 3; i++) dst[i] = src[i] * a + dst[i] * (1.0f - a);
        return;
    }
    const float a = g_clamp(src[3], 0.0f, 1.0f);
    for (int i = 0; i < 3; i++) dst[i] = g_clamp(src[i], 0.0f, 1.0f) * a + canvas8(dst[i]) * (1.0f - a);
}

/* 2D mode (u_quality = 0): drawScene binds the vertex2d mesh (render.js:278,
 * 287): the footprint quads of sdf.cpp:362-401 on the plane z = 0, vert2d
 * normal byte 0 -> v_normal = (1,0,0) (render.vert:16), culled from below
 * (render.js:88-91; tri2d winds counter-clockwise seen from +z), drawn over
 * the clear colour 0.9 (render.js:274-275, from the second frame on).
 * render.frag with u_quality = 0 outputs baseCol (:241-244); glass (id 2):
 * alpha = 0.8 exp2(dot(rayDir, n)), rgb *= 0.2 atmCol (:246-249).  The march
 * and AO it also runs never reach the output there (:244). */
#define CLEAR_2D 0.9f
static void shade_2d(const shade_ctx *c, const float d[3], float out[4], vxo_stats *st) {
    const vxo_scene *s = c->s;
    const vxo_frame *f = c->f;
    out[0] = out[1] = out[2] = CLEAR_2D;
    out[3] = 1.0f;
    const float zr = (float)(0 - f->cam_cell[2]) - f->cam_fract[2];
    int col = 0, x = 0, y = 0;
    float hx = 0.0f, hy = 0.0f;
    if (zr < 0.0f && d[2] < 0.0f && s->fp2d) {
        const float t = zr / d[2];
        hx = f->cam_fract[0] + t * d[0];
        hy = f->cam_fract[1] + t * d[1];
        x = f->cam_cell[0] + g_f2i(floorf(hx));
        y = f->cam_cell[1] + g_f2i(floorf(hy));
        if (x >= 0 && y >= 0 && x < s->X && y < s->Y) {
            col = (int)s->fp2d[2 * ((size_t)y * s->X + x)];
            if (st) st->primary_fetches++;
        }
    }
    if (col == 0) {
        if (st) st->sky_px++;
        return;
    }
    const uint32_t org = s->fp2d[2 * ((size_t)y * s->X + x) + 1];
    const int x0 = (int)(org & 0xffffu), y0 = (int)(org >> 16);
    float base[3];
    palette(col, base);
    if (col != GLASS_INDEX) {
        if (st) st->block_px++;
        out[0] = base[0]; out[1] = base[1]; out[2] = base[2];
        return;
    }
    if (st) st->glass_px++;
    /* v_cellPos = the quad corner (x0, y0, 0), v_fractPos = hit - corner */
    const float fx = (float)(f->cam_cell[0] - x0) + hx, fy = (float)(f->cam_cell[1] - y0) + hy;
    const float v[3] = {(float)(x0 - f->cam_cell[0]) + (fx - f->cam_fract[0]),
                        (float)(y0 - f->cam_cell[1]) + (fy - f->cam_fract[1]),
                        (float)(0 - f->cam_cell[2]) + (0.0f - f->cam_fract[2])};   /* :154 */
    float r[3];
    normalize3(v, r);
    const float n[3] = {1.0f, 0.0f, 0.0f};
    const float k = 2.0f * dot3(n, r);                                              /* :155 reflect() */
    const float rz = sqrtf(g_max(0.0f, r[2] - k * n[2]));
    const float scatter = 1.0f - sqrtf(g_max(0.0f, f->sun_dir[2]));                 /* :168 */
    const float sp0[3] = {0.2f, 0.4f, 0.7f}, sp1[3] = {0.2f, 0.3f, 0.5f};
    const float sc0[3] = {0.7f, 0.9f, 1.0f}, sc1[3] = {1.0f, 0.3f, 0.2f};
    float src[4];
    src[3] = 0.8f * vxo_exp2(dot3(r, n));                                           /* :247 */
    for (int i = 0; i < 3; i++) {
        const float atm = g_mix(g_mix(sc0[i], sc1[i], scatter), g_mix(sp0[i], sp1[i], scatter), rz);   /* :169-171 */
        src[i] = base[i] * (0.2f * atm);                                            /* :248 */
    }
    blend_canvas(src, out, f->flags);                                               /* over the clear colour */
}

/* One pixel: primary visibility, shading, glass blend (render.js:84-86
 * SRC_ALPHA / ONE_MINUS_SRC_ALPHA over the surface behind). */
static void render_pixel(const shade_ctx *c, int w, int h, int px, int py, float out[4], vxo_stats *st) {
    const vxo_scene *s = c->s;
    const vxo_frame *f = c->f;
    float d[3];
    vxo_pixel_dir(f, w, h, px, py, d);
    if (f->quality == 0) {           /* MODE_2D: the vertex2d mesh (render.js:278, 287) */
        if (st) st->pixels++;
        shade_2d(c, d, out, st);
        return;
    }
    vxo_gbuf g[2];
    int fetches = 0, cap_hit = 0, panes = 0;
    int n = primary_walk(s, f, d, 1, g, &fetches, &cap_hit, &panes, NULL);
    if (st) { st->pixels++; st->primary_fetches += (uint64_t)fetches; st->primary_cap_hits += (uint64_t)cap_hit; }
    vxo_gbuf sky;
    sky_record(&sky);
    if (f->flags & 0x8u) {   /* VX_FLAG_PRIMARY_ONLY: v_color of the first surface, sky = palette(0) */
        if (st) { if (n == 0) st->sky_px++; else if (g[0].id == 2) st->glass_px++; else st->block_px++; }
        palette(n == 0 ? 0 : g[0].color, out);
        out[3] = 1.0f;
        return;
    }
    if (n == 0) {
        if (st) st->sky_px++;
        shade_frag(c, &sky, d, out, NULL, st);
    } else if (panes >= 2 && !(f->flags & VXO_FLAG_GLASS_SINGLE)) {
        /* two or more panes in front of the surface: the reference's raster --
         * glass quads after every opaque one, in vertex.bin order; each passes
         * the depth test (LESS, depth writes on) iff it is nearer than the last
         * surface written, and blends over the colour there (render.js:82-91).
         * The next pane drawn is found by a scan of the ray's panes (walk mode 3,
         * no fetches counted: they repeat the primary walk's).  With one pane
         * this is the single blend below. */
        if (st) st->glass_px++;
        float dst[4], depth = INFINITY;
        g_term_slot = 1;
        if (n == 2) {
            shade_frag(c, &g[1], NULL, dst, NULL, st);
            depth = g[1].t;
        } else {
            shade_frag(c, &sky, d, dst, NULL, st);
        }
        g_term_slot = -1;
        glass_sel sel = {0, 0, depth};
        for (;;) {
            vxo_gbuf gl;
            int fx = 0, cx = 0;
            sel.tmax = depth;
            if (!primary_walk(s, f, d, 3, &gl, &fx, &cx, NULL, &sel)) break;
            float src[4], rd[3];
            g_term_slot = gl.key == g[0].key ? 0 : -1;
            shade_frag(c, &gl, NULL, src, rd, st);
            g_term_slot = -1;
            if (f->flags & (VXO_FLAG_REFLECT | VXO_FLAG_REFLECT_ALL)) add_reflection(c, &gl, rd, src, st);
            blend_canvas(src, dst, f->flags);
            depth = gl.t;
            sel.have_last = 1;
            sel.klast = gl.key;
        }
        out[0] = dst[0]; out[1] = dst[1]; out[2] = dst[2];
    } else if (g[0].id != 2) {
        if (st) st->block_px++;
        g_term_slot = 0;
        float rd[3];
        shade_frag(c, &g[0], NULL, out, rd, st);
        g_term_slot = -1;
        if (f->flags & VXO_FLAG_REFLECT_ALL) add_reflection(c, &g[0], rd, out, st);
    } else {
        if (st) st->glass_px++;
        float src[4], dst[4], rd[3];
        g_term_slot = 0;
        shade_frag(c, &g[0], NULL, src, rd, st);
        g_term_slot = -1;
        if (f->flags & (VXO_FLAG_REFLECT | VXO_FLAG_REFLECT_ALL)) add_reflection(c, &g[0], rd, src, st);
        g_term_slot = 1;
        if (n == 2) shade_frag(c, &g[1], NULL, dst, NULL, st);
        else shade_frag(c, &sky, d, dst, NULL, st);
        g_term_slot = -1;
        blend_canvas(src, dst, f->flags);
        out[0] = dst[0]; out[1] = dst[1]; out[2] = dst[2];
    }
    out[3] = 1.0f;
}

void vxo_render(const vxo_scene *s, const vxo_frame *f, int w, int h,
                int row0, int row_step, float *out, vxo_stats *st, int n_threads) {
    if (row_step <= 0) row_step = 1;
    int nrows = row0 < h ? (h - 1 - row0) / row_step + 1 : 0;
    shade_ctx ctx;
    ctx_init(&ctx, s, f);
    ctx_tables(&ctx);
    vxo_stats acc;
    memset(&acc, 0, sizeof acc);
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel num_threads(n_threads)
#endif
    {
        vxo_stats loc;
        memset(&loc, 0, sizeof loc);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int k = 0; k < nrows; k++) {
            int py = row0 + k * row_step;
            for (int px = 0; px < w; px++)
                render_pixel(&ctx, w, h, px, py, out + 4 * ((size_t)py * w + px), &loc);
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            uint64_t *a = (uint64_t *)&acc, *b = (uint64_t *)&loc;
            for (size_t i = 0; i < sizeof acc / sizeof(uint64_t); i++) a[i] += b[i];
        }
    }
    if (st) *st = acc;
    ctx_free(&ctx);
    (void)n_threads;
}

/* Diagnostic (tools/march_sched.py): per pixel of the tw x th block at (px0,
 * py0) of a w x h frame, the fetch counts of its sun marches in the order the
 * shading runs them, bit 16 set when the march ended lit (-1 = none beyond),
 * up to maxrec each, with the scene's exit mode.  Serial. */
void vxo_march_lengths(const vxo_scene *s, const vxo_frame *f, int w, int h, int px0, int py0, int tw, int th,
                       int *out, int maxrec) {
    shade_ctx ctx;
    ctx_init(&ctx, s, f);
    ctx_tables(&ctx);
    float rgba[4];
    for (int j = 0; j < th; j++)
        for (int i = 0; i < tw; i++) {
            int *o = out + ((size_t)j * tw + i) * maxrec;
            for (int k = 0; k < maxrec; k++) o[k] = -1;
            g_rec = o; g_rec_n = 0; g_rec_cap = maxrec;
            if (px0 + i < w && py0 + j < h) render_pixel(&ctx, w, h, px0 + i, py0 + j, rgba, NULL);
            g_rec = NULL;
        }
    ctx_free(&ctx);
}

void vxo_render_terms(const vxo_scene *s, const vxo_frame *f, int w, int h, int row0, int row_step,
                      uint8_t *lit, float *amb, int n_threads) {
    if (row_step <= 0) row_step = 1;
    const int nrows = row0 < h ? (h - 1 - row0) / row_step + 1 : 0;
    shade_ctx ctx;
    ctx_init(&ctx, s, f);
    ctx_tables(&ctx);
    (void)n_threads;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads)
#endif
    for (int k = 0; k < nrows; k++) {
        const int py = row0 + k * row_step;
        for (int px = 0; px < w; px++) {
            const size_t i = (size_t)py * w + px;
            float rgba[4];
            lit[2 * i] = lit[2 * i + 1] = 255;
            amb[2 * i] = amb[2 * i + 1] = NAN;
            g_term_lit = lit + 2 * i;
            g_term_amb = amb + 2 * i;
            render_pixel(&ctx, w, h, px, py, rgba, NULL);
            g_term_lit = NULL;
            g_term_amb = NULL;
        }
    }
    ctx_free(&ctx);
}
