/* Primary-traversal step counts: octant cubes vs per-axis empty boxes.
 *
 * The walk (oracle/vxo_render.c walk()) may jump across any
 * all-air region anchored at the current cell in the ray's octant; the cube
 * [c, c + r*s] is one choice, a box [c, c + e*s] with per-axis extents another.
 * This replays the walk for every camera ray with each strategy, counts the
 * steps, and checks that the hit (cell, face, fp32 te) is the cube walk's.
 *
 * usage: box_sim GRID X Y Z RAYS   (GRID: u8 palette, x fastest; RAYS: binary
 *        header int cc[3], float o[3], int n, then n float d[3])
 * build: gcc -O2 -fopenmp -ffp-contract=off -o box_sim box_sim.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CAP 32          /* extents <= CAP - 1: the next cell stays inside the pad = CAP border */
#define NSTRAT 5
static const char *kName[NSTRAT] = {"cube", "cube+x,y,z", "cube+z,x,y", "round-robin", "cube+xy-rr,z"};

static int X, Y, Z;
static uint8_t *grid;
static int *S;          /* prefix sums of solid cells, (X+1)(Y+1)(Z+1) */

static inline size_t P(int x, int y, int z) { return (size_t)x + (size_t)(X + 1) * ((size_t)y + (size_t)(Y + 1) * (size_t)z); }

/* solid cells in [x0,x1]x[y0,y1]x[z0,z1] (inclusive, any order), outside = air */
static int solid(int x0, int x1, int y0, int y1, int z0, int z1) {
    if (x0 > x1) { int t = x0; x0 = x1; x1 = t; }
    if (y0 > y1) { int t = y0; y0 = y1; y1 = t; }
    if (z0 > z1) { int t = z0; z0 = z1; z1 = t; }
    if (x0 < 0) x0 = 0; if (y0 < 0) y0 = 0; if (z0 < 0) z0 = 0;
    if (x1 > X - 1) x1 = X - 1; if (y1 > Y - 1) y1 = Y - 1; if (z1 > Z - 1) z1 = Z - 1;
    if (x0 > x1 || y0 > y1 || z0 > z1) return 0;
    x1++; y1++; z1++;
    return S[P(x1, y1, z1)] - S[P(x0, y1, z1)] - S[P(x1, y0, z1)] - S[P(x1, y1, z0)] + S[P(x0, y0, z1)] +
           S[P(x0, y1, z0)] + S[P(x1, y0, z0)] - S[P(x0, y0, z0)];
}

static inline int empty(int x, int y, int z, const int s[3], const int e[3]) {
    return solid(x, x + s[0] * e[0], y, y + s[1] * e[1], z, z + s[2] * e[2]) == 0;
}

static void extents(int strat, int x, int y, int z, const int s[3], int e[3]) {
    e[0] = e[1] = e[2] = 0;
    if (grid[(size_t)x + (size_t)X * ((size_t)y + (size_t)Y * z)]) return;   /* non-air: DDA step */
    /* the cube */
    int r = 0;
    while (r + 1 < CAP) {
        int t[3] = {r + 1, r + 1, r + 1};
        if (!empty(x, y, z, s, t)) break;
        r++;
    }
    e[0] = e[1] = e[2] = r;
    if (strat == 0) return;
    static const int ord1[3] = {0, 1, 2}, ord2[3] = {2, 0, 1};
    if (strat == 1 || strat == 2) {
        const int *ord = strat == 1 ? ord1 : ord2;
        for (int k = 0; k < 3; k++) {
            const int a = ord[k];
            while (e[a] + 1 < CAP) {
                e[a]++;
                if (!empty(x, y, z, s, e)) { e[a]--; break; }
            }
        }
        return;
    }
    /* round-robin growth: all three axes (3) or x, y first then z (4) */
    const int naxes = strat == 3 ? 3 : 2;
    for (int pass = 0; pass < 2; pass++) {
        int grew = 1;
        while (grew) {
            grew = 0;
            for (int a = 0; a < naxes; a++) {
                if (e[a] + 1 >= CAP) continue;
                e[a]++;
                if (empty(x, y, z, s, e)) grew = 1; else e[a]--;
            }
        }
        if (strat == 3) break;
        while (e[2] + 1 < CAP) {
            e[2]++;
            if (!empty(x, y, z, s, e)) { e[2]--; break; }
        }
        break;
    }
}

typedef struct { int cell[3], axis, nrec; float te; int steps; } Hit;

static Hit walk(const int cc[3], const float o[3], const float d[3], const uint8_t *ext /* 3 B per cell */) {
    Hit h = {{0, 0, 0}, -1, 0, 0.0f, 0};
    const int dims[3] = {X, Y, Z};
    float inv[3], tlo = 0.0f, thi = INFINITY;
    int stp[3], c[3];
    for (int i = 0; i < 3; i++) {
        stp[i] = d[i] > 0.0f ? 1 : -1;
        inv[i] = d[i] != 0.0f ? 1.0f / d[i] : 0.0f;
        const float lo = (float)(0 - cc[i]) - o[i], hi = (float)(dims[i] - cc[i]) - o[i];
        if (d[i] != 0.0f) {
            float t0 = lo * inv[i], t1 = hi * inv[i];
            if (t0 > t1) { float t = t0; t0 = t1; t1 = t; }
            tlo = tlo < t0 ? t0 : tlo;
            thi = t1 < thi ? t1 : thi;
        } else if (!(lo <= 0.0f && 0.0f < hi)) return h;
    }
    if (!(tlo < thi)) return h;
    for (int i = 0; i < 3; i++) {
        int ci = (int)floorf(o[i] + tlo * d[i]);
        const int lo = -cc[i], hi = dims[i] - cc[i] - 1;
        c[i] = ci < lo ? lo : (ci > hi ? hi : ci);
    }
#define AT(a) ((size_t)(a)[0] + (size_t)X * ((size_t)(a)[1] + (size_t)Y * (size_t)(a)[2]))
    int ab[3] = {c[0] + cc[0], c[1] + cc[1], c[2] + cc[2]};
    int prev = grid[AT(ab)], nrec = 0;
    const uint8_t *E = ext + 3 * AT(ab);
    int e[3] = {E[0], E[1], E[2]};
    h.steps = 1;
    for (int it = 0; it < 4 * (X + Y + Z); it++) {
        float tb[3];
        for (int i = 0; i < 3; i++)
            tb[i] = d[i] != 0.0f ? ((float)(c[i] + (stp[i] > 0 ? e[i] + 1 : -e[i])) - o[i]) * inv[i] : INFINITY;
        const int a = (tb[0] <= tb[1] && tb[0] <= tb[2]) ? 0 : (tb[1] <= tb[2] ? 1 : 2);
        const float te = tb[a];
        for (int i = 0; i < 3; i++) {
            if (i == a) c[i] += stp[i] * (e[i] + 1);
            else {
                const int v = (int)floorf(o[i] + te * d[i]);
                const int lo = d[i] < 0.0f ? c[i] - e[i] : c[i], hi = d[i] < 0.0f ? c[i] : c[i] + e[i];
                c[i] = v < lo ? lo : (v > hi ? hi : v);
            }
        }
        for (int i = 0; i < 3; i++) ab[i] = c[i] + cc[i];
        if (ab[0] < 0 || ab[1] < 0 || ab[2] < 0 || ab[0] >= X || ab[1] >= Y || ab[2] >= Z) break;
        h.steps++;
        const int col = grid[AT(ab)];
        E = ext + 3 * AT(ab);
        e[0] = E[0]; e[1] = E[1]; e[2] = E[2];
        if (col != prev) {
            nrec++;
            if (col != 21 || nrec == 2) {
                memcpy(h.cell, ab, sizeof ab);
                h.axis = a;
                h.te = te;
                break;
            }
        }
        prev = col;
    }
    h.nrec = nrec;
    return h;
}

int main(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "usage: box_sim GRID X Y Z RAYS\n"); return 2; }
    X = atoi(argv[2]); Y = atoi(argv[3]); Z = atoi(argv[4]);
    const size_t N = (size_t)X * Y * Z;
    grid = malloc(N);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(grid, 1, N, f) != N) { fprintf(stderr, "grid read failed\n"); return 1; }
    fclose(f);
    int cc[3], n;
    float o[3];
    f = fopen(argv[5], "rb");
    if (!f || fread(cc, 4, 3, f) != 3 || fread(o, 4, 3, f) != 3 || fread(&n, 4, 1, f) != 1) return 1;
    float *dirs = malloc((size_t)n * 12);
    if (fread(dirs, 12, n, f) != (size_t)n) return 1;
    fclose(f);

    S = calloc((size_t)(X + 1) * (Y + 1) * (Z + 1), sizeof(int));
    for (int z = 1; z <= Z; z++)
        for (int y = 1; y <= Y; y++)
            for (int x = 1; x <= X; x++)
                S[P(x, y, z)] = (grid[(size_t)(x - 1) + (size_t)X * ((size_t)(y - 1) + (size_t)Y * (z - 1))] != 0) +
                                S[P(x - 1, y, z)] + S[P(x, y - 1, z)] + S[P(x, y, z - 1)] - S[P(x - 1, y - 1, z)] -
                                S[P(x - 1, y, z - 1)] - S[P(x, y - 1, z - 1)] + S[P(x - 1, y - 1, z - 1)];

    int used[8] = {0};
    for (int i = 0; i < n; i++) {
        const float *d = dirs + 3 * i;
        used[(d[0] < 0) | ((d[1] < 0) << 1) | ((d[2] < 0) << 2)] = 1;
    }
    uint8_t *ext[NSTRAT][8] = {{0}};
    for (int st = 0; st < NSTRAT; st++)
        for (int oc = 0; oc < 8; oc++) {
            if (!used[oc]) continue;
            const int s[3] = {oc & 1 ? -1 : 1, oc & 2 ? -1 : 1, oc & 4 ? -1 : 1};
            uint8_t *E = malloc(3 * N);
#pragma omp parallel for schedule(dynamic, 1)
            for (int z = 0; z < Z; z++)
                for (int y = 0; y < Y; y++)
                    for (int x = 0; x < X; x++) {
                        int e[3];
                        extents(st, x, y, z, s, e);
                        uint8_t *p = E + 3 * ((size_t)x + (size_t)X * ((size_t)y + (size_t)Y * z));
                        p[0] = (uint8_t)e[0]; p[1] = (uint8_t)e[1]; p[2] = (uint8_t)e[2];
                    }
            ext[st][oc] = E;
        }
    long long steps[NSTRAT] = {0}, mism[NSTRAT] = {0};
    for (int st = 0; st < NSTRAT; st++) {
        long long tot = 0, bad = 0;
#pragma omp parallel for reduction(+ : tot, bad) schedule(dynamic, 256)
        for (int i = 0; i < n; i++) {
            const float *d = dirs + 3 * i;
            const int oc = (d[0] < 0) | ((d[1] < 0) << 1) | ((d[2] < 0) << 2);
            const Hit h = walk(cc, o, d, ext[st][oc]);
            tot += h.steps;
            const Hit r = walk(cc, o, d, ext[0][oc]);
            if (h.axis != r.axis || h.nrec != r.nrec || memcmp(h.cell, r.cell, sizeof h.cell) ||
                memcmp(&h.te, &r.te, 4))
                bad++;
        }
        steps[st] = tot;
        mism[st] = bad;
        printf("%-14s steps/ray %.3f  (%.1f%% of cube)  hit mismatches vs cube %lld\n", kName[st],
               (double)tot / n, 100.0 * (double)tot / (double)steps[0], bad);
    }
    return 0;
}
