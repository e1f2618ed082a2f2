/*
 * vxo_mesh.c — CPU ORACLE (test infrastructure only; see vxo.h header).
 *
 * The greedy quad mesh of /root/reference/src/gen/sdf.cpp:281-356, restated
 * from the text per FACE instead of per quad: for every face the mesh has, the
 * offset of its cell from the origin of the quad that covers it.  That origin
 * is what the raster hands render.frag as the flat v_cellPos (render.vert:25,
 * the vert() records of sdf.cpp:94-102 carry the quad origin x, y, z and the
 * corner offset dx, dy, dz, which render.vert interpolates into v_fractPos,
 * :26-28), so the quad-relative G-buffer needs it per face.
 *
 * Restated rules (read as text, not copied; oracle/mesh_ref.py is the
 * quad-list restatement this is checked against in tests/test_quad_gbuf.py):
 *   - per colour c < pal_size (sdf.cpp:284), per chunk of CHUNK cells per axis
 *     in forChunkXYZ order (voxmap.h:62-67), per axis d and normal 0/1, slices
 *     p[d] = -1 .. CHUNK-1 (sdf.cpp:299-311): the mask of (u, v) =
 *     ((d+1)%3, (d+2)%3) cells is (normal 0) "cell is c, the cell ahead along
 *     +d is not" or (normal 1) "cell is not c, the cell ahead is"; ccol()
 *     clamps coordinates into the grid (sdf.cpp:44-51);
 *   - greedy merge, rows j (v) outer and i (u) inner: width along u while the
 *     mask holds, then height along v while the whole row of w holds; the
 *     quad's cells are cleared and the scan goes on at i + w (sdf.cpp:313-351);
 *   - the face's cell: the c cell, i.e. p for normal 0 and p + e_d for normal 1;
 *     its normal index 2d + normal (sdf.cpp:342, render.vert:14-17).
 * Colours are disjoint, so one pass over labelled slices (label = the face's
 * colour) emits exactly the quads of the per-colour passes: a colour's quads
 * depend only on its own mask cells, and the scan skips only cells of the
 * quad just emitted.  Faces on an interior chunk plane are emitted by both
 * chunks (slice CHUNK-1 of the lower one and slice -1 of the upper one) from
 * the same slice, so both give the same offset (slice -1 is skipped here).  For dims that are not
 * multiples of CHUNK the clamped cells past the grid repeat the edge cell;
 * those positions are not written (they belong to no cell of the grid).
 *
 * Colours are the vis colours of vxo.h (1..21 meshed, anything else air),
 * which compare exactly as sdf.cpp's remapped indices do for c < pal_size.
 */
#include "vxo.h"
#include <stdlib.h>
#include <string.h>

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

void vxo_face_quads(const uint8_t *rgba, int X, int Y, int Z, int chunk, uint16_t *out) {
    const int dims[3] = {X, Y, Z};
    const size_t N = (size_t)X * Y * Z;
    for (size_t i = 0; i < 6 * N; i++) out[i] = VXO_NO_FACE;
    if (chunk <= 0) chunk = Z;
    uint8_t *vis = (uint8_t *)malloc(N);
    for (size_t i = 0; i < N; i++) vis[i] = (uint8_t)vxo_vis(rgba[4 * i + 2]);
    const int CH = chunk;
    const int ncx = (X + CH - 1) / CH, ncy = (Y + CH - 1) / CH, ncz = (Z + CH - 1) / CH;
#define VIS(x, y, z) vis[(size_t)clampi(x, 0, X - 1) + (size_t)X * ((size_t)clampi(y, 0, Y - 1) + (size_t)Y * (size_t)clampi(z, 0, Z - 1))]
    /* slice p[d] = -1 repeats slice CHUNK-1 of the chunk below (the same cells,
     * mask and quads; at the grid's low edge it has no faces), so it is skipped:
     * every face is then written by exactly one chunk */
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int ci = 0; ci < ncx * ncy * ncz; ci++) {
        uint8_t *lab = (uint8_t *)malloc((size_t)CH * CH);
        uint8_t *done = (uint8_t *)malloc((size_t)CH * CH);
        {
                const int base[3] = {ci / (ncy * ncz) * CH, ci / ncz % ncy * CH, ci % ncz * CH};
                for (int d = 0; d < 3; d++) {
                    const int u = (d + 1) % 3, v = (d + 2) % 3;
                    for (int normal = 0; normal < 2; normal++)
                        for (int pd = 0; pd < CH; pd++) {
                            int any = 0;
                            for (int j = 0; j < CH; j++)
                                for (int i = 0; i < CH; i++) {
                                    int p[3], q[3];
                                    p[d] = base[d] + pd; p[u] = base[u] + i; p[v] = base[v] + j;
                                    q[0] = p[0]; q[1] = p[1]; q[2] = p[2];
                                    q[d] += 1;
                                    const int b = VIS(p[0], p[1], p[2]), a = VIS(q[0], q[1], q[2]);
                                    int l = 0;
                                    if (normal == 0 && b != 0 && a != b) l = b;      /* block c, ahead not c */
                                    if (normal == 1 && a != 0 && b != a) l = a;      /* block not c, ahead c */
                                    lab[j * CH + i] = (uint8_t)l;
                                    any |= l;
                                }
                            if (!any) continue;
                            memset(done, 0, (size_t)CH * CH);
                            for (int j = 0; j < CH; j++)
                                for (int i = 0; i < CH; i++) {
                                    const int c = lab[j * CH + i];
                                    if (!c || done[j * CH + i]) continue;
                                    int w = 1, h = 1;
                                    while (i + w < CH && lab[j * CH + i + w] == c && !done[j * CH + i + w]) w++;
                                    for (; j + h < CH; h++) {
                                        int ok = 1;
                                        for (int k = 0; k < w; k++)
                                            if (lab[(j + h) * CH + i + k] != c || done[(j + h) * CH + i + k]) { ok = 0; break; }
                                        if (!ok) break;
                                    }
                                    for (int l = 0; l < h; l++)
                                        for (int k = 0; k < w; k++) {
                                            done[(j + l) * CH + i + k] = 1;
                                            int cell[3];
                                            cell[d] = base[d] + pd + (normal ? 1 : 0);
                                            cell[u] = base[u] + i + k;
                                            cell[v] = base[v] + j + l;
                                            if (cell[0] < 0 || cell[1] < 0 || cell[2] < 0 || cell[0] >= dims[0] ||
                                                cell[1] >= dims[1] || cell[2] >= dims[2])
                                                continue;      /* a clamped position past the grid */
                                            const size_t cc = (size_t)cell[0] + (size_t)X * ((size_t)cell[1] + (size_t)Y * (size_t)cell[2]);
                                            out[6 * cc + 2 * d + normal] = (uint16_t)(k | (l << 8));
                                        }
                                    i += w - 1;
                                }
                        }
                }
        }
        free(done);
        free(lab);
    }
#undef VIS
    free(vis);
}

/* Emission order of the quad that covers a face (the order vertex.bin draws
 * it in, render.js:297): colour-major (sdf.cpp:284), then forChunkXYZ chunk
 * order, axis d, normal, slice p[d], quad origin row j, column i.  A face on an
 * interior chunk plane is emitted first by the lower chunk (its slice
 * CHUNK-1).  Only compared between faces of one colour (glass). */
uint64_t vxo_face_order(const int cell[3], int nidx, uint16_t off, int X, int Y, int Z, int chunk) {
    (void)X;
    const int CH = chunk > 0 ? chunk : Z;
    const int d = nidx >> 1, normal = nidx & 1;
    const int u = (d + 1) % 3, v = (d + 2) % 3;
    const int plane = cell[d] + (normal ? 0 : 1);        /* the quad's plane p[d] + 1 */
    int cd = plane / CH, pd = plane % CH - 1;
    if (pd < 0) { cd -= 1; pd = CH - 1; }                /* plane on a chunk boundary: the lower chunk */
    const int ou = cell[u] - (off & 0xff), ov = cell[v] - (off >> 8);
    int ch[3];
    ch[d] = cd;
    ch[u] = ou / CH;
    ch[v] = ov / CH;
    const int ny = (Y + CH - 1) / CH, nz = (Z + CH - 1) / CH;
    const uint64_t chunk_id = ((uint64_t)ch[0] * ny + (uint64_t)ch[1]) * nz + (uint64_t)ch[2];
    const uint64_t i0 = (uint64_t)(ou - ch[u] * CH), j0 = (uint64_t)(ov - ch[v] * CH);
    const uint64_t S = (uint64_t)CH + 1;                 /* slice (pd + 1 in 0..CH), rows and columns < CH + 1 */
    return ((((chunk_id * 3 + (uint64_t)d) * 2 + (uint64_t)normal) * S + (uint64_t)(pd + 1)) * S + j0) * S + i0;
}
