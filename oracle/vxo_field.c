/*
 * vxo_field.c — CPU ORACLE (test infrastructure only; see vxo.h header).
 *
 * vxo_field_build: literal restatement of the distance-field part of
 * /root/reference/src/gen/sdf.cpp (lines 405-470), quirks included:
 *   - csum() clamps every index into the grid (sdf.cpp:36-42), so vol()'s
 *     "x0-1" term reads sum[0] instead of 0 when the box reaches index 0
 *     (sdf.cpp:63-83): blocks in the 0-slices are not counted for such boxes;
 *   - octant o=0 is the box [z, z+r] capped at r<Z, o=1 the box [z-r, z]
 *     capped at r<z (sdf.cpp:436-453) — R="up", G="down" (sdf.cpp:15's
 *     comment is inverted relative to the code);
 *   - the diagonal-neighbour shortcut mid = csdf(x-1,y-1,z-1,o) bounds r to
 *     [mid-1, mid+1] (sdf.cpp:439-444), which makes the serial x->y->z order
 *     (voxmap.h:50-55) part of the definition;
 *   - blocks keep sdf = 0; map.bin is written z->y->x as R,G,B=col,A=0
 *     (sdf.cpp:462-470), with air remapped to B = pal_size = 22
 *     (sdf.cpp:19,188,229-233).
 * The reference C++ itself is NOT compiled (SURVEY.md §8c permission denial);
 * this is a from-text restatement.
 *
 * vxo_field_octant: the build's own primary-traversal data:
 * per octant of ray directions, the size r of the all-air cube ahead of each
 * cell (r <= cap - 1 <= 254; the kernels keep 255 for their out-of-grid
 * sentinel).  vxo_field_box grows that cube into the box the traversal uses.
 */
#include "vxo.h"
#include <stdlib.h>
#include <string.h>
#include <math.h>

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

typedef struct { int X, Y, Z; int *sum; unsigned char *sdf; } fctx;

static inline size_t IDX(const fctx *c, int x, int y, int z) {
    return (size_t)x + (size_t)c->X * ((size_t)y + (size_t)c->Y * (size_t)z);
}
static inline int csum(const fctx *c, int x, int y, int z) {          /* sdf.cpp:36-42 */
    return c->sum[IDX(c, clampi(x, 0, c->X - 1), clampi(y, 0, c->Y - 1), clampi(z, 0, c->Z - 1))];
}
static inline int csdf(const fctx *c, int x, int y, int z, int o) {   /* sdf.cpp:54-61 */
    return c->sdf[2 * IDX(c, clampi(x, 0, c->X - 1), clampi(y, 0, c->Y - 1), clampi(z, 0, c->Z - 1)) + o];
}
static inline int vol(const fctx *c, int x0, int y0, int z0, int x1, int y1, int z1) { /* sdf.cpp:63-83 */
    x0--; y0--; z0--;
    return 0
        - csum(c, x1, y1, z0)
        - csum(c, x1, y0, z1)
        - csum(c, x0, y1, z1)
        + csum(c, x1, y1, z1)
        + csum(c, x0, y0, z1)
        + csum(c, x0, y1, z0)
        + csum(c, x1, y0, z0)
        - csum(c, x0, y0, z0);
}

void vxo_field_build(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba) {
    fctx c = {X, Y, Z, NULL, NULL};
    size_t N = (size_t)X * Y * Z;
    /* zero-initialised like the reference's global array: csum() of a clamped
     * index that lands on the cell being computed reads 0 (sdf.cpp:24, 36-42) */
    c.sum = (int *)calloc(N, sizeof(int));
    c.sdf = (unsigned char *)calloc(2 * N, 1);
    /* summed volume table, forXYZ order (sdf.cpp:407-422) */
    for (int x = 0; x < X; x++)
        for (int y = 0; y < Y; y++)
            for (int z = 0; z < Z; z++) {
                int bin = color[IDX(&c, x, y, z)] != 0;
                c.sum[IDX(&c, x, y, z)] = bin
                    + csum(&c, x, y, z - 1)
                    + csum(&c, x, y - 1, z)
                    + csum(&c, x - 1, y, z)
                    - csum(&c, x - 1, y - 1, z)
                    - csum(&c, x - 1, y, z - 1)
                    - csum(&c, x, y - 1, z - 1)
                    + csum(&c, x - 1, y - 1, z - 1);
            }
    /* half-cube radii, forXYZ order (sdf.cpp:429-457) */
    for (int x = 0; x < X; x++)
        for (int y = 0; y < Y; y++)
            for (int z = 0; z < Z; z++) {
                if (color[IDX(&c, x, y, z)] != 0) continue;
                for (int o = 0; o < 2; o++) {
                    int mn = 1;
                    int mx = (o == 0) ? Z : z;
                    if (x + y + z > 0) {
                        int mid = csdf(&c, x - 1, y - 1, z - 1, o);
                        mn = mn > mid - 1 ? mn : mid - 1;
                        mx = mx < mid + 1 ? mx : mid + 1;
                    }
                    int r = mn;
                    while (r < mx && 0 == vol(&c, x - r, y - r, z - o * r, x + r, y + r, z + (1 - o) * r)) r++;
                    c.sdf[2 * IDX(&c, x, y, z) + o] = (unsigned char)r;
                }
            }
    /* map.bin texels (sdf.cpp:462-470).  B is the remapped palette index:
     * sdf.cpp:229-233 scans pal[i] from i = 1 for the cell's colour; pal[]
     * is zero-initialised (sdf.cpp:19) and pal[0] = 0 is air (sdf.cpp:188),
     * so air finds the first zero entry past the palette, pal[pal_size]:
     * air is written as B = pal_size = VXO_PAL_SIZE. */
    for (size_t i = 0; i < N; i++) {
        rgba[4 * i + 0] = c.sdf[2 * i + 0];
        rgba[4 * i + 1] = c.sdf[2 * i + 1];
        rgba[4 * i + 2] = color[i] ? color[i] : (uint8_t)VXO_PAL_SIZE;
        rgba[4 * i + 3] = 0;
    }
    free(c.sum);
    free(c.sdf);
}

/* Octant box half-size: for octant o (bit 0: x negative,
 * bit 1: y, bit 2: z; a zero direction component counts as positive) the
 * largest L <= cap such that the cube of side L with corner c extending toward
 * the octant holds no meshed cell (vxo_vis(B) != 0: no face can be entered
 * there) of the grid; r = L - 1 (0 for meshed cells).  L = min over forward non-air q of max_i (q_i - c_i) s_i,
 * separable: L = min_dz max(dz, min_dy max(dy, min_dx dx)) over dx, dy, dz in
 * [0, cap).  Cells outside the grid count as air. */
void vxo_field_octant(const uint8_t *rgba, int X, int Y, int Z, int cap, int oct, uint8_t *r_out) {
    const size_t N = (size_t)X * Y * Z;
    const int sx = oct & 1 ? -1 : 1, sy = oct & 2 ? -1 : 1, sz = oct & 4 ? -1 : 1;
    unsigned char *g1 = (unsigned char *)malloc(N), *g2 = (unsigned char *)malloc(N);
#define I3(x, y, z) ((size_t)(x) + (size_t)X * ((size_t)(y) + (size_t)Y * (size_t)(z)))
#pragma omp parallel for schedule(static)
    for (int z = 0; z < Z; z++)          /* pass x: forward run to the first non-air cell */
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                int best = cap;
                for (int k = 0; k < cap; k++) {
                    const int xx = x + k * sx;
                    if (xx < 0 || xx >= X) break;
                    if (vxo_vis(rgba[4 * I3(xx, y, z) + 2])) { best = k; break; }
                }
                g1[I3(x, y, z)] = (unsigned char)best;
            }
#pragma omp parallel for schedule(static)
    for (int z = 0; z < Z; z++)          /* pass y */
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                int best = cap;
                for (int k = 0; k < cap; k++) {
                    const int yy = y + k * sy;
                    if (yy < 0 || yy >= Y) break;
                    const int v = g1[I3(x, yy, z)], m = v > k ? v : k;
                    if (m < best) best = m;
                }
                g2[I3(x, y, z)] = (unsigned char)best;
            }
#pragma omp parallel for schedule(static)
    for (int z = 0; z < Z; z++)          /* pass z -> r */
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                int best = cap;
                for (int k = 0; k < cap; k++) {
                    const int zz = z + k * sz;
                    if (zz < 0 || zz >= Z) break;
                    const int v = g2[I3(x, y, zz)], m = v > k ? v : k;
                    if (m < best) best = m;
                }
                r_out[I3(x, y, z)] = (unsigned char)(best > 0 ? best - 1 : 0);
            }
#undef I3
    free(g1);
    free(g2);
}

/* ---- vxo_field_box: the cube r grown to per-axis extents ----
 * Solid = meshed (vxo_vis(B) != 0); cells outside the grid count as air.
 * ex = max e in [r, cap-1] with box (e, r, r) empty, then ey with (ex, e, r),
 * then ez with (ex, ey, e).  Emptiness is monotone in each extent, so the
 * maximum is found by bisection (the kernel's k_oct_box does the same). */
typedef struct { int X, Y, Z; const int *S; } bctx;

static inline size_t PS(const bctx *b, int x, int y, int z) {
    return (size_t)x + (size_t)(b->X + 1) * ((size_t)y + (size_t)(b->Y + 1) * (size_t)z);
}
/* solid cells in the inclusive box between corners a and a + e*s */
static int box_solid(const bctx *b, int x, int y, int z, const int s[3], const int e[3]) {
    int lo[3] = {x, y, z}, hi[3] = {x + s[0] * e[0], y + s[1] * e[1], z + s[2] * e[2]};
    const int dim[3] = {b->X, b->Y, b->Z};
    for (int i = 0; i < 3; i++) {
        if (lo[i] > hi[i]) { const int t = lo[i]; lo[i] = hi[i]; hi[i] = t; }
        if (lo[i] < 0) lo[i] = 0;
        if (hi[i] > dim[i] - 1) hi[i] = dim[i] - 1;
        if (lo[i] > hi[i]) return 0;
        hi[i]++;
    }
    return b->S[PS(b, hi[0], hi[1], hi[2])] - b->S[PS(b, lo[0], hi[1], hi[2])] - b->S[PS(b, hi[0], lo[1], hi[2])] -
           b->S[PS(b, hi[0], hi[1], lo[2])] + b->S[PS(b, lo[0], lo[1], hi[2])] + b->S[PS(b, lo[0], hi[1], lo[2])] +
           b->S[PS(b, hi[0], lo[1], lo[2])] - b->S[PS(b, lo[0], lo[1], lo[2])];
}

void vxo_field_box(const uint8_t *rgba, int X, int Y, int Z, int cap, int oct, const uint8_t *r_cube,
                   uint8_t *e_out) {
    int *S = (int *)calloc((size_t)(X + 1) * (Y + 1) * (Z + 1), sizeof(int));
    bctx b = {X, Y, Z, S};
    for (int z = 1; z <= Z; z++)
        for (int y = 1; y <= Y; y++)
            for (int x = 1; x <= X; x++) {
                const size_t c = (size_t)(x - 1) + (size_t)X * ((size_t)(y - 1) + (size_t)Y * (size_t)(z - 1));
                S[PS(&b, x, y, z)] = (vxo_vis(rgba[4 * c + 2]) != 0) + S[PS(&b, x - 1, y, z)] + S[PS(&b, x, y - 1, z)] +
                                     S[PS(&b, x, y, z - 1)] - S[PS(&b, x - 1, y - 1, z)] - S[PS(&b, x - 1, y, z - 1)] -
                                     S[PS(&b, x, y - 1, z - 1)] + S[PS(&b, x - 1, y - 1, z - 1)];
            }
    const int s[3] = {oct & 1 ? -1 : 1, oct & 2 ? -1 : 1, oct & 4 ? -1 : 1};
#pragma omp parallel for schedule(static)
    for (int z = 0; z < Z; z++)
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                const size_t c = (size_t)x + (size_t)X * ((size_t)y + (size_t)Y * (size_t)z);
                int e[3] = {0, 0, 0};
                if (vxo_vis(rgba[4 * c + 2]) == 0) {
                    const int r = r_cube[c];
                    e[0] = e[1] = e[2] = r;
                    for (int a = 0; a < 3; a++) {
                        int lo = r, hi = cap - 1;          /* lo: known empty */
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) / 2;
                            e[a] = mid;
                            if (box_solid(&b, x, y, z, s, e) == 0) lo = mid; else hi = mid - 1;
                        }
                        e[a] = lo;
                    }
                }
                e_out[3 * c] = (uint8_t)e[0];
                e_out[3 * c + 1] = (uint8_t)e[1];
                e_out[3 * c + 2] = (uint8_t)e[2];
            }
    free(S);
}

/* Exit table of the build's sun march (DESIGN.md §3 "Sun exit tables") for
 * sun octant oct (bit i: r_i > 0) and the channel the march reads for it (R
 * if r_z > 0, else G: render.frag:47-50, 89).  out[c] = 1 marks a cell from
 * which the march cannot end unlit: it can only leave the grid or run out of
 * steps, "lit" either way (render.frag:123-126, 234).  Layer recursion along
 * z, from the far end in the ray's z direction:
 *   D(x, y, z) = AND over i = 0..kx, j = 0..ky of
 *                [T(x', y', z) != 0 and D(x', y', z + sz)],  x' = x + i*sx, y' = y + j*sy,
 * cells outside the grid counting as true (D beyond the last layer = true).
 * kx, ky < 0 mean unbounded (every x' from x to the grid edge): D(c) = "no 0
 * texel in the orthant ahead of c" -- valid for every direction of the
 * octant.  kx = ceil(max |r_x / r_z| + 1/64) (ky likewise) bounds the cells a
 * ray crossing one z layer can touch from any point of c: valid for every
 * direction of the octant with those slopes (the cone tables).  Why this is
 * exact is DESIGN.md §3; this is the definition the kernel's tables must equal.
 * Each layer: B = [T != 0] and D(next layer); R = the window AND of B along
 * x, D = the window AND of R along y, both from run lengths of trues counted
 * from the far end of the ray's side. */
void vxo_field_exit(const uint8_t *rgba, int X, int Y, int Z, int oct, int kx, int ky, uint8_t *out) {
    const int sx = (oct & 1) ? 1 : -1, sy = (oct & 2) ? 1 : -1, sz = (oct & 4) ? 1 : -1;
    const int ch = sz > 0 ? 0 : 1;
    const size_t XY = (size_t)X * Y;
    uint8_t *B = (uint8_t *)malloc(XY), *R = (uint8_t *)malloc(XY);
    int *run = (int *)malloc(sizeof(int) * (size_t)(X > Y ? X : Y));
    const int INF = 1 << 30;
    for (int k = 0; k < Z; k++) {
        const int z = sz > 0 ? Z - 1 - k : k;
        const uint8_t *prev = k ? out + (size_t)(z + sz) * XY : NULL;
        for (size_t j = 0; j < XY; j++)
            B[j] = rgba[4 * ((size_t)z * XY + j) + ch] != 0 && (!prev || prev[j]);
        /* R(x, y) = B true on x' = x, x + sx, ..., x + kx*sx (inside the grid) */
        for (int y = 0; y < Y; y++) {
            const uint8_t *b = B + (size_t)y * X;
            for (int t = 0; t < X; t++) {
                const int x = sx > 0 ? X - 1 - t : t;   /* from the far end */
                run[x] = !b[x] ? 0 : (t == 0 ? INF : (run[x + sx] >= INF ? INF : run[x + sx] + 1));
            }
            for (int x = 0; x < X; x++) R[(size_t)y * X + x] = run[x] >= INF || (kx >= 0 && run[x] > kx);
        }
        /* D(x, y) = R true on y' = y, ..., y + ky*sy */
        uint8_t *d = out + (size_t)z * XY;
        for (int x = 0; x < X; x++) {
            for (int t = 0; t < Y; t++) {
                const int y = sy > 0 ? Y - 1 - t : t;
                run[y] = !R[(size_t)y * X + x] ? 0 : (t == 0 ? INF : (run[y + sy] >= INF ? INF : run[y + sy] + 1));
            }
            for (int y = 0; y < Y; y++) d[(size_t)y * X + x] = run[y] >= INF || (ky >= 0 && run[y] > ky);
        }
    }
    free(B); free(R); free(run);
}

/* ---------------- the sun doom table (DESIGN.md §3 "Doom table") ----------------
 * In sun-aligned coordinates (x', y' grow toward the sun: x' = x if sx > 0,
 * else X - 1 - x), a ray of the frame's samples rises one layer while x' grows
 * by a slope in [ax_min, ax_max] (y' likewise).  Q = VXO_DOOM_Q sub-cells per cell and
 * axis.  State S_z(g) (g a sub-cell (gx, gy) at height z, the bottom of layer
 * z): every ray crossing height z inside g (within 1/64 cell) enters a solid
 * cell (R = G = 0, sdf.cpp:430) before leaving the grid; depth(g) = layers to
 * that entry.  Top-down:
 *   depth_Z = inf (leaving the grid);
 *   depth_z(g) = 0 if every cell covering g widened by 1/64 is solid,
 *                else 1 + max over g' in g + [xlo, xhi] x [ylo, yhi] of depth_{z+1}(g')
 * (sub-cells outside the grid: inf).  A cell (x', y', z) not solid is doomed
 * with h = 1 + max over g' in [Q x' - 1, Q x' + Q + xhi] x [Q y' - 1, Q y' + Q
 * + yhi] of depth_{z+1}(g'): from anywhere in the cell a ray meets height z + 1
 * inside that window.  Depths saturate at 254 (inf = 255); h <= the plan's hmax. */
int vxo_doom_cross(int h, int xhi, int yhi) {
    return h + (h * xhi) / VXO_DOOM_Q + 1 + (h * yhi) / VXO_DOOM_Q + 1;
}

void vxo_doom_plan(const float dirs[][3], int n, int max_steps, int plan[7]) {
    double axmin = 1e300, axmax = -1e300, aymin = 1e300, aymax = -1e300;
    for (int k = 0; k < n; k++) {
        const double ax = fabs((double)dirs[k][0] / (double)dirs[k][2]), ay = fabs((double)dirs[k][1] / (double)dirs[k][2]);
        if (ax < axmin) axmin = ax;
        if (ax > axmax) axmax = ax;
        if (ay < aymin) aymin = ay;
        if (ay > aymax) aymax = ay;
    }
    const double eps = 1.0 / 64.0, Q = (double)VXO_DOOM_Q;
    plan[0] = dirs[0][0] > 0.0f ? 1 : -1;
    plan[1] = dirs[0][1] > 0.0f ? 1 : -1;
    plan[2] = (int)floor(Q * (axmin - eps)); plan[3] = (int)ceil(Q * (axmax + eps));
    plan[4] = (int)floor(Q * (aymin - eps)); plan[5] = (int)ceil(Q * (aymax + eps));
    /* the stop rule j + 2 C(h) < MAX can hold (at j = 1) only for 1 + 2 C(h) < MAX; C grows with h */
    int hm = 0;
    while (hm < VXO_DOOM_HCAP && vxo_doom_cross(hm + 1, plan[3], plan[5]) <= VXO_DOOM_HCAP &&
           1 + 2 * vxo_doom_cross(hm + 1, plan[3], plan[5]) < max_steps)
        hm++;
    plan[6] = hm;
}

void vxo_field_doom(const uint8_t *rgba, int X, int Y, int Z, const int plan[7], uint8_t *code) {
    const int sx = plan[0], sy = plan[1], xlo = plan[2], xhi = plan[3], ylo = plan[4], yhi = plan[5], hmax = plan[6];
    const int Q = VXO_DOOM_Q, GX = X * Q, GY = Y * Q;
    const size_t XY = (size_t)X * Y, G = (size_t)GX * GY;
    uint8_t *d1 = (uint8_t *)malloc(G), *d0 = (uint8_t *)malloc(G), *rx = (uint8_t *)malloc(G);
    uint8_t *rc = (uint8_t *)malloc((size_t)GY * X);
    memset(d1, 255, G);
#define VXO_SOLID(z, xa, ya) ((xa) >= 0 && (xa) < X && (ya) >= 0 && (ya) < Y && \
    rgba[4 * ((size_t)(z) * XY + (size_t)((sy > 0 ? (ya) : Y - 1 - (ya))) * X + (size_t)(sx > 0 ? (xa) : X - 1 - (xa)))] == 0 && \
    rgba[4 * ((size_t)(z) * XY + (size_t)((sy > 0 ? (ya) : Y - 1 - (ya))) * X + (size_t)(sx > 0 ? (xa) : X - 1 - (xa))) + 1] == 0)
    for (int z = Z - 1; z >= 0; z--) {
        /* rows: rx(gy, gx) = max over [gx + xlo, gx + xhi], rc(gy, x') = max over [Q x' - 1, Q x' + Q + xhi] */
#pragma omp parallel for schedule(static)
        for (int gy = 0; gy < GY; gy++) {
            const uint8_t *row = d1 + (size_t)gy * GX;
            for (int gx = 0; gx < GX; gx++) {
                int m = 0;
                for (int k = gx + xlo; k <= gx + xhi; k++) {
                    const int v = (k < 0 || k >= GX) ? 255 : row[k];
                    if (v > m) m = v;
                }
                rx[(size_t)gy * GX + gx] = (uint8_t)m;
            }
            for (int x = 0; x < X; x++) {
                int m = 0;
                for (int k = Q * x - 1; k <= Q * x + Q + xhi; k++) {
                    const int v = (k < 0 || k >= GX) ? 255 : row[k];
                    if (v > m) m = v;
                }
                rc[(size_t)gy * X + x] = (uint8_t)m;
            }
        }
        /* cells of layer z (from the states at z + 1) */
#pragma omp parallel for schedule(static)
        for (int y = 0; y < Y; y++) {
            for (int x = 0; x < X; x++) {
                int m = 0;
                for (int k = Q * y - 1; k <= Q * y + Q + yhi; k++) {
                    const int v = (k < 0 || k >= GY) ? 255 : rc[(size_t)k * X + x];
                    if (v > m) m = v;
                }
                const int h = m + 1;
                const int xr = sx > 0 ? x : X - 1 - x, yr = sy > 0 ? y : Y - 1 - y;
                code[(size_t)z * XY + (size_t)yr * X + xr] =
                    (uint8_t)((m < 255 && h <= hmax && !VXO_SOLID(z, x, y)) ? vxo_doom_cross(h, xhi, yhi) : 0);
            }
        }
        /* states at height z */
#pragma omp parallel for schedule(static)
        for (int gy = 0; gy < GY; gy++) {
            const int y = gy / Q, b = gy % Q;
            const int y0 = b == 0 ? y - 1 : y, y1 = b == Q - 1 ? y + 1 : y;    /* cells covering the sub-cell +- 1/64 */
            for (int gx = 0; gx < GX; gx++) {
                const int x = gx / Q, a = gx % Q;
                const int x0 = a == 0 ? x - 1 : x, x1 = a == Q - 1 ? x + 1 : x;
                const int es = VXO_SOLID(z, x0, y0) && VXO_SOLID(z, x1, y0) && VXO_SOLID(z, x0, y1) && VXO_SOLID(z, x1, y1);
                int m = 0;
                for (int l = gy + ylo; l <= gy + yhi; l++) {
                    const int v = (l < 0 || l >= GY) ? 255 : rx[(size_t)l * GX + gx];
                    if (v > m) m = v;
                }
                d0[(size_t)gy * GX + gx] = (uint8_t)(es ? 0 : (m < 255 ? (m + 1 < 254 ? m + 1 : 254) : 255));
            }
        }
        uint8_t *t = d1; d1 = d0; d0 = t;
    }
#undef VXO_SOLID
    free(d1); free(d0); free(rx); free(rc);
}
