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
 *     (sdf.cpp:462-470).
 * The reference C++ itself is NOT compiled (SURVEY.md §8c permission denial);
 * this is a from-text restatement.
 *
 * vxo_field_dist: the build's own A-channel contents: the
 * half-size R of the all-air box around each cell, R = D - 1 for the capped
 * Chebyshev distance D >= 1 to the nearest non-air cell, 0 for non-air cells
 * (so A <= cap - 1 <= 254; 255 is free for the kernels' out-of-grid sentinel).
 */
#include "vxo.h"
#include <stdlib.h>
#include <string.h>

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
    /* map.bin texels (sdf.cpp:462-470) */
    for (size_t i = 0; i < N; i++) {
        rgba[4 * i + 0] = c.sdf[2 * i + 0];
        rgba[4 * i + 1] = c.sdf[2 * i + 1];
        rgba[4 * i + 2] = color[i];
        rgba[4 * i + 3] = 0;
    }
    free(c.sum);
    free(c.sdf);
}

/* Capped Chebyshev distance to the nearest non-air cell (B != 0), separable:
 * D = min_z' max(|dz|, min_y' max(|dy|, min_x' |dx|)). */
void vxo_field_dist(uint8_t *rgba, int X, int Y, int Z, int cap) {
    size_t N = (size_t)X * Y * Z;
    unsigned char *g1 = (unsigned char *)malloc(N), *g2 = (unsigned char *)malloc(N);
    const int dims[3] = {X, Y, Z};
    (void)dims;
    /* pass x: 1-D distance along x */
    for (int z = 0; z < Z; z++)
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                int best = cap;
                for (int k = 0; k < cap && best > k; k++) {
                    int xa = x - k, xb = x + k;
                    if ((xa >= 0 && rgba[4 * ((size_t)xa + (size_t)X * ((size_t)y + (size_t)Y * z)) + 2]) ||
                        (xb < X && rgba[4 * ((size_t)xb + (size_t)X * ((size_t)y + (size_t)Y * z)) + 2]))
                        best = k;
                }
                g1[(size_t)x + (size_t)X * ((size_t)y + (size_t)Y * z)] = (unsigned char)best;
            }
    /* pass y */
    for (int z = 0; z < Z; z++)
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                int best = cap;
                for (int k = -(cap - 1); k <= cap - 1; k++) {
                    int yy = y + k;
                    if (yy < 0 || yy >= Y) continue;
                    int v = g1[(size_t)x + (size_t)X * ((size_t)yy + (size_t)Y * z)];
                    int ak = k < 0 ? -k : k;
                    int m = v > ak ? v : ak;
                    if (m < best) best = m;
                }
                g2[(size_t)x + (size_t)X * ((size_t)y + (size_t)Y * z)] = (unsigned char)best;
            }
    /* pass z -> A channel */
    for (int z = 0; z < Z; z++)
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) {
                int best = cap;
                for (int k = -(cap - 1); k <= cap - 1; k++) {
                    int zz = z + k;
                    if (zz < 0 || zz >= Z) continue;
                    int v = g2[(size_t)x + (size_t)X * ((size_t)y + (size_t)Y * zz)];
                    int ak = k < 0 ? -k : k;
                    int m = v > ak ? v : ak;
                    if (m < best) best = m;
                }
                rgba[4 * ((size_t)x + (size_t)X * ((size_t)y + (size_t)Y * z)) + 3] =
                    (unsigned char)(best > 0 ? best - 1 : 0);
            }
    free(g1);
    free(g2);
}
