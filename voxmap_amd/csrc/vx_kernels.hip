// vx_kernels.hip — CDNA4 (gfx950) kernels of the Voxmap shading path besides
// the 3D render kernel: the render dispatch (each EXT mode's launches live in
// their own unit, vx_render_e*.hip), the 2D mode, the de-tile and stats
// passes, and the per-scene field preparation (octant boxes, sun exit tables,
// the greedy mesh per face, AO pairs, noise quads).
#include "vx_render.h"

namespace vx {
namespace {

// 2D mode frames (quality 0) in a kernel of their own: the 3D kernel keeps its
// code and registers (a third user of the frame constants in k_render made
// the compiler copy KernelArgs to scratch).  Same pixel mapping and stores.
template <int FMT, bool STATS, bool TILED>
__global__ __launch_bounds__(kWG) void k_render_2d(KernelArgs a) {
    __shared__ uint32_t s_px[kBY][kBX];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lx = ((wave % kWX) << 3) | (lane & 7);
    const int ly = ((wave / kWX) << 3) | (lane >> 3);
    int ox, oy, tx0 = 0, ty0 = 0, tile_k = 0;
    if (TILED) {
        const int perx = a.tile_w >> kBXS, pery = a.tile_h >> kBYS;
        const int bpt = perx * pery;
        tile_k = blockIdx.x / bpt;
        const int sub = blockIdx.x % bpt;
        const int tid = a.tile_ids[tile_k];
        tx0 = (sub % perx) << kBXS;
        ty0 = (sub / perx) << kBYS;
        ox = (tid % a.tiles_x) * a.tile_w + tx0;
        oy = (tid / a.tiles_x) * a.tile_h + ty0;
    } else {
        ox = blockIdx.x << kBXS;
        oy = blockIdx.y << kBYS;
    }
    const int px = ox + lx, py = oy + ly;
    Counters cnt = {};
    unsigned n_sky = 0, n_block = 0, n_glass = 0, n_px = 0;
    if (px < a.w && py < a.h) {
        float d0, d1, d2, rgba[4];
        view_ray(a.fc, px, py, d0, d1, d2);
        shade_2d(a, d0, d1, d2, rgba, cnt, n_sky, n_block, n_glass);
        if (FMT == VX_PIXEL_RGBA8)
            s_px[ly][lx] = pack_rgba8(rgba);
        else
            store_pixel<FMT>(a, out_index<TILED>(a, tile_k, tx0 + lx, ty0 + ly, px, py), rgba);
        n_px = 1;
    }
    if (FMT == VX_PIXEL_RGBA8) {
        __syncthreads();
        const int sx = threadIdx.x & (kBX - 1), sy = threadIdx.x >> kBXS;
        if (ox + sx < a.w && oy + sy < a.h)
            reinterpret_cast<uint32_t *>(a.out)[out_index<TILED>(a, tile_k, tx0 + sx, ty0 + sy, ox + sx, oy + sy)] =
                s_px[sy][sx];
    }
    if (STATS) {
        unsigned long long v[ST_COUNT] = {};
        v[ST_PIXELS] = wave_sum(n_px);
        v[ST_SKY] = wave_sum(n_sky);
        v[ST_BLOCK] = wave_sum(n_block);
        v[ST_GLASS] = wave_sum(n_glass);
        v[ST_PRIM_FETCH] = wave_sum(cnt.prim_fetch);
        if (lane == 0) {
            unsigned long long *row = a.stats + (size_t)((blockIdx.x + blockIdx.y * 7) & 63) * ST_COUNT;
#pragma unroll
            for (int i = 0; i < ST_COUNT; i++)
                if (v[i]) atomicAdd(row + i, v[i]);
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
    if (x >= 0 && y >= 0 && x < w && y < h) frame[(size_t)y * w + x] = tiles[i];
}

// ---- A channel of octant copy `oct`: size r of the air cube ahead of a cell
// (oracle vxo_field_octant), separable one-sided passes:
// L = min_dz max(dz, min_dy max(dy, min_dx dx)), dx, dy, dz in [0, cap) toward
// the octant, cells outside the grid air; r = L - 1 (0 for non-air) ----
__global__ void k_oct_x(const uint32_t *field, uint8_t *g1, int X, int Y, int Z, int cap, int sx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y * Z) return;
    const int x = (int)(i % X);
    int best = cap;
    for (int k = 0; k < cap; k++) {
        const int xx = x + k * sx;
        if (xx < 0 || xx >= X) break;
        if ((field[i + (ptrdiff_t)(k * sx)] >> 16) & 0xff) { best = k; break; }
    }
    g1[i] = (uint8_t)best;
}

__global__ void k_oct_yz(const uint8_t *gin, uint8_t *gout, uint32_t *field, int X, int Y, int Z, int cap, int axis,
                         int sgn) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y * Z) return;
    const int pos = axis == 1 ? (int)((i / X) % Y) : (int)(i / ((size_t)X * Y));
    const int n = axis == 1 ? Y : Z;
    const ptrdiff_t stride = axis == 1 ? (ptrdiff_t)X : (ptrdiff_t)X * Y;
    int best = cap;
    for (int k = 0; k < cap; k++) {
        const int q = pos + k * sgn;
        if (q < 0 || q >= n) break;
        const int v = gin[(ptrdiff_t)i + (ptrdiff_t)(k * sgn) * stride];
        const int m = v > k ? v : k;
        best = m < best ? m : best;
    }
    if (axis == 1) gout[i] = (uint8_t)best;
    else field[i] = (field[i] & 0x00ffffffu) | ((uint32_t)(best > 0 ? best - 1 : 0) << 24);
}

__global__ void k_reduce_stats(unsigned long long *stats) {
    const int i = threadIdx.x;
    if (i < ST_COUNT) {
        unsigned long long s = 0;
        for (int r = 0; r < 64; r++) s += stats[r * ST_COUNT + i];
        stats[i] = s;
    }
}

}  // namespace

int launch_render(const KernelArgs &a, int fmt, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const bool tiled = a.tile_ids != nullptr;
    const bool st = a.stats != nullptr;
    dim3 block(kWG);
    dim3 grid = tiled ? dim3(a.n_tiles * (a.tile_w >> kBXS) * (a.tile_h >> kBYS))
                      : dim3((a.w + kBX - 1) / kBX, (a.h + kBY - 1) / kBY);
    if (a.fc.quality == 0) {          // MODE_2D: the vertex2d mesh (render.js:278, 287)
#define VX_L2(F, S, T) hipLaunchKernelGGL((k_render_2d<F, S, T>), grid, block, 0, s, a)
#define VX_L2T(F, S) do { if (tiled) VX_L2(F, S, true); else VX_L2(F, S, false); } while (0)
        if (fmt == VX_PIXEL_RGBA32F) { if (st) VX_L2T(0, true); else VX_L2T(0, false); }
        else { if (st) VX_L2T(1, true); else VX_L2T(1, false); }
#undef VX_L2T
#undef VX_L2
        if (st) hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(64), 0, s, a.stats);
        return (int)hipGetLastError();
    }
    const bool brick_ok = a.fc.soft_sg >= 0 && a.sunp && a.fc.soft_lg >= 4 && (a.SXp & 3) == 0 && a.SB >= 9;
    // the general shading block (glass in draw order, REFLECT_ALL): EXT 5 / 6 (not with the pooled pass)
    const bool general = (a.fc.flags & (VX_FLAG_GLASS_ORDER | VX_FLAG_REFLECT_ALL)) != 0;
    const int ext = a.fc.n_sun > 1 ? (general ? 6 : (a.fc.flags & VX_FLAG_SOFT_BRICK) && brick_ok ? 4
                                      : (a.fc.flags & (VX_FLAG_SOFT_POOL | VX_FLAG_SOFT_BRICK)) ? 3 : 2)
                                   : (general ? 5 : (a.fc.flags & (VX_FLAG_REFLECT | VX_FLAG_ROUGH)) ? 1 : 0);
    int rc;
    switch (ext) {
        case 0: rc = launch_render_e0(a, fmt, grid.x, grid.y, stream); break;
        case 1: rc = launch_render_e1(a, fmt, grid.x, grid.y, stream); break;
        case 2: rc = launch_render_e2(a, fmt, grid.x, grid.y, stream); break;
        case 3: rc = launch_render_e3(a, fmt, grid.x, grid.y, stream); break;
        case 4: rc = launch_render_e4(a, fmt, grid.x, grid.y, stream); break;
        default: rc = launch_render_e56(ext, a, fmt, grid.x, grid.y, stream); break;
    }
    if (rc) return rc;
    if (st) hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(64), 0, s, a.stats);
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

namespace {
// ---- prefix sums of solid (non-air) cells, S[(X+1)(Y+1)(Z+1)], S(0, ., .) =
// S(., 0, .) = S(., ., 0) = 0: any box's solid count in 8 loads (k_oct_box)
__device__ __forceinline__ size_t ps_index(int x, int y, int z, int X, int Y) {
    return (size_t)x + (size_t)(X + 1) * ((size_t)y + (size_t)(Y + 1) * (size_t)z);
}
__global__ void k_psum_x(const uint32_t *lin, int *S, int X, int Y, int Z) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;     // (y, z) row of S
    if (i >= (size_t)(Y + 1) * (Z + 1)) return;
    const int y = (int)(i % (Y + 1)), z = (int)(i / (Y + 1));
    int acc = 0;
    S[ps_index(0, y, z, X, Y)] = 0;
    for (int x = 1; x <= X; x++) {
        if (y > 0 && z > 0)
            acc += ((lin[(size_t)(x - 1) + (size_t)X * ((size_t)(y - 1) + (size_t)Y * (size_t)(z - 1))] >> 16) & 0xffu) != 0;
        S[ps_index(x, y, z, X, Y)] = acc;
    }
}
__global__ void k_psum_yz(int *S, int X, int Y, int Z, int axis) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;     // x fastest: coalesced
    const int n = axis == 1 ? Y : Z, m = axis == 1 ? Z : Y;
    if (i >= (size_t)(X + 1) * (m + 1)) return;
    const int x = (int)(i % (X + 1)), j = (int)(i / (X + 1));
    int acc = 0;
    for (int k = 1; k <= n; k++) {
        const size_t q = axis == 1 ? ps_index(x, k, j, X, Y) : ps_index(x, j, k, X, Y);
        acc += S[q];
        S[q] = acc;
    }
}

// ---- one octant's prim copy: colour | ex << 8 | ey << 16 | ez << 24, the
// cube r (A byte of the upload, k_oct_*) grown to the largest x extent, then
// y, then z, each <= cap - 1, by bisection on box emptiness (oracle
// vxo_field_box: the same definition, the same maxima)
__global__ void k_oct_box(const uint32_t *lin, const int *S, uint32_t *dst, int X, int Y, int Z, int P, int cap,
                          int sx, int sy, int sz) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y * Z) return;
    const int x = (int)(i % X), y = (int)((i / X) % Y), z = (int)(i / ((size_t)X * Y));
    const uint32_t t = lin[i];
    const uint32_t col = (t >> 16) & 0xffu;
    int e[3] = {0, 0, 0};
    if (col == 0) {
        const int r = (int)(t >> 24);
        e[0] = e[1] = e[2] = r;
        const int s[3] = {sx, sy, sz}, c[3] = {x, y, z}, dim[3] = {X, Y, Z};
        auto solid = [&]() {
            int lo[3], hi[3];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                int a0 = c[k], a1 = c[k] + s[k] * e[k];
                if (a0 > a1) { const int tt = a0; a0 = a1; a1 = tt; }
                a0 = a0 < 0 ? 0 : a0;
                a1 = a1 > dim[k] - 1 ? dim[k] - 1 : a1;
                if (a0 > a1) return 0;
                lo[k] = a0;
                hi[k] = a1 + 1;
            }
            return S[ps_index(hi[0], hi[1], hi[2], X, Y)] - S[ps_index(lo[0], hi[1], hi[2], X, Y)] -
                   S[ps_index(hi[0], lo[1], hi[2], X, Y)] - S[ps_index(hi[0], hi[1], lo[2], X, Y)] +
                   S[ps_index(lo[0], lo[1], hi[2], X, Y)] + S[ps_index(lo[0], hi[1], lo[2], X, Y)] +
                   S[ps_index(hi[0], lo[1], lo[2], X, Y)] - S[ps_index(lo[0], lo[1], lo[2], X, Y)];
        };
        for (int k = 0; k < 3; k++) {
            int lo = r, hi = cap - 1;                 // lo: known empty
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                e[k] = mid;
                if (solid() == 0) lo = mid; else hi = mid - 1;
            }
            e[k] = lo;
        }
    }
    const size_t Xp = (size_t)X + 2 * P, Yp = (size_t)Y + 2 * P;
    dst[(size_t)(x + P) + Xp * ((size_t)(y + P) + Yp * (size_t)(z + P))] =
        col | ((uint32_t)e[0] << 8) | ((uint32_t)e[1] << 16) | ((uint32_t)e[2] << 24);
}
// ---- the greedy mesh per face (sdf.cpp:281-356; oracle vxo_face_quads): for
// every face the mesh has, its offset du | dv << 8 from the origin of the quad
// covering it, along u = (d+1)%3, v = (d+2)%3 -- the v_cellPos / v_fractPos
// split the raster hands render.frag (render.vert:25-28).  One workgroup per
// slice (chunk, d, normal, p[d] = 0 .. CH-1; the reference's slice -1 repeats
// slice CH-1 of the chunk below, same cells, same quads): the lanes label the slice's
// CH x CH mask in LDS (the face's colour, 0 = no face: normal 0 "cell is c, the
// cell ahead along +d is not", normal 1 the reverse, ccol() clamping the
// coordinates), then one lane runs the merge -- rows j outer, columns i inner,
// width along u while the label holds, height along v while the whole row of w
// holds, the quad's labels cleared (the reference clears its mask), the scan
// going on at i + w.  Colours are disjoint, so the labelled slice yields
// exactly the quads of the per-colour passes.  Positions past the grid (dims
// not multiples of CH repeat the clamped edge cell) are not written.
__global__ __launch_bounds__(64) void k_face_quads(const uint32_t *lin, uint16_t *qf, int X, int Y, int Z, int CH,
                                                   int ncy, int ncz, size_t N) {
    extern __shared__ uint8_t lab[];                       // CH * CH labels
    __shared__ int any;
    const int S = CH;                                      // slices p[d] = 0 .. CH-1 (-1 repeats the chunk below's CH-1)
    const int pd = (int)(blockIdx.x % (unsigned)S);
    const int normal = (int)((blockIdx.x / (unsigned)S) & 1u);
    const int d = (int)((blockIdx.x / (unsigned)(2 * S)) % 3u);
    const unsigned chunk = blockIdx.x / (unsigned)(6 * S);
    const int base[3] = {(int)(chunk / (unsigned)(ncy * ncz)) * CH, (int)((chunk / (unsigned)ncz) % (unsigned)ncy) * CH,
                         (int)(chunk % (unsigned)ncz) * CH};
    const int u = d == 2 ? 0 : d + 1, v = d == 0 ? 2 : d - 1;
    const int dims[3] = {X, Y, Z};
    auto vis = [&](int p0, int p1, int p2) -> int {
        p0 = min(max(p0, 0), X - 1); p1 = min(max(p1, 0), Y - 1); p2 = min(max(p2, 0), Z - 1);
        return (int)((lin[(size_t)p0 + (size_t)X * ((size_t)p1 + (size_t)Y * (size_t)p2)] >> 16) & 0xffu);
    };
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    int mine = 0;
    for (int k = threadIdx.x; k < CH * CH; k += 64) {
        const int j = k / CH, i = k % CH;
        int p[3];
        p[d] = base[d] + pd; p[u] = base[u] + i; p[v] = base[v] + j;
        const int b = vis(p[0], p[1], p[2]);
        p[d] += 1;
        const int a = vis(p[0], p[1], p[2]);
        int l = 0;
        if (normal == 0 && b != 0 && a != b) l = b;
        if (normal == 1 && a != 0 && b != a) l = a;
        lab[k] = (uint8_t)l;
        mine |= l;
    }
    if (mine) any = 1;
    __syncthreads();
    if (!any || threadIdx.x != 0) return;
    for (int j = 0; j < CH; j++)
        for (int i = 0; i < CH; i++) {
            const int c = lab[j * CH + i];
            if (!c) continue;
            int w = 1, h = 1;
            while (i + w < CH && lab[j * CH + i + w] == c) w++;
            for (; j + h < CH; h++) {
                bool ok = true;
                for (int k = 0; k < w && ok; k++) ok = lab[(j + h) * CH + i + k] == c;
                if (!ok) break;
            }
            for (int l = 0; l < h; l++)
                for (int k = 0; k < w; k++) {
                    lab[(j + l) * CH + i + k] = 0;
                    int cell[3];
                    cell[d] = base[d] + pd + normal;
                    cell[u] = base[u] + i + k;
                    cell[v] = base[v] + j + l;
                    if (cell[0] < 0 || cell[1] < 0 || cell[2] < 0 || cell[0] >= dims[0] || cell[1] >= dims[1] ||
                        cell[2] >= dims[2])
                        continue;
                    const size_t ci = (size_t)cell[0] + (size_t)X * ((size_t)cell[1] + (size_t)Y * (size_t)cell[2]);
                    qf[(size_t)(2 * d + normal) * N + ci] = (uint16_t)(k | (l << 8));
                }
            i += w - 1;
        }
}
// Per ray octant, a copy in the prim layout (padded, pad = P) of each cell's
// entry faces' quad offsets: a ray of octant oct (bit i: negative along i)
// enters a cell through the face with normal index 2a + (positive ? 1 : 0) on
// axis a; word = sum over a of (du | dv << 5) << 10a (CHUNK <= 32), 0 where the
// face does not exist (as quad_offsets) and on the border.  The fp32-index
// primary walk loads it beside every prim word (QSPEC).
__global__ void k_qcopy(const uint16_t *qf, uint32_t *dst, int X, int Y, int Z, int P, int oct, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int x = (int)(i % X), y = (int)((i / X) % Y), z = (int)(i / ((size_t)X * Y));
    uint32_t w = 0;
#pragma unroll
    for (int ax = 0; ax < 3; ax++) {
        const int nidx = 2 * ax + (((oct >> ax) & 1) ? 0 : 1);
        unsigned q = qf[(size_t)nidx * N + i];
        q = q == 0xFFFFu ? 0u : q;
        w |= ((q & 31u) | (((q >> 8) & 31u) << 5)) << (10 * ax);
    }
    const size_t Xp = (size_t)X + 2 * P, Yp = (size_t)Y + 2 * P;
    dst[(size_t)(x + P) + Xp * ((size_t)(y + P) + Yp * (size_t)(z + P))] = w;
}
// the table in the oracle's layout (6 per cell) for vx_scene_read_face_quads
__global__ void k_face_quads_interleave(const uint16_t *qf, uint16_t *out, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 6 * N) return;
    out[i] = qf[(i % 6) * N + i / 6];
}
// AO x-pairs (sdf_lin): entry (p, y, z), p = 0..X, = rg of cells clamp(p - 1) and clamp(p)
__global__ void k_ao_pairs(const uint16_t *rg, uint32_t *rg2, int X, int Y, int Z) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t row = (size_t)X + 1;
    if (i >= row * Y * Z) return;
    const int p = (int)(i % row);
    const size_t yz = i / row;
    const int x0 = max(p - 1, 0), x1 = min(p, X - 1);
    rg2[i] = (uint32_t)rg[yz * X + x0] | ((uint32_t)rg[yz * X + x1] << 16);
}
// noise quads: per texel (x, y), one u32 per channel plane holding that channel
// of texels (x, y), (x+1, y), (x, y+1), (x+1, y+1) (W, H powers of two, REPEAT):
// plane 0 = A (fbm), planes 1..3 = R, G, B (white)
__global__ void k_noise_quads(const uint32_t *noise, uint32_t *q, int W, int H) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t n = (size_t)W * H;
    if (i >= n) return;
    const int x = (int)(i % W), y = (int)(i / W);
    const int x1 = (x + 1) & (W - 1), y1 = (y + 1) & (H - 1);
    const uint32_t t00 = noise[(size_t)y * W + x], t10 = noise[(size_t)y * W + x1];
    const uint32_t t01 = noise[(size_t)y1 * W + x], t11 = noise[(size_t)y1 * W + x1];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int sh = p == 0 ? 24 : 8 * (p - 1);
        q[p * n + i] = ((t00 >> sh) & 0xffu) | (((t10 >> sh) & 0xffu) << 8) | (((t01 >> sh) & 0xffu) << 16) |
                       (((t11 >> sh) & 0xffu) << 24);
    }
}
// linear RGBA upload -> sun channel arrays and the AO array
__global__ void k_pack_sun(const uint32_t *src, uint8_t *sun, uint16_t *rg, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint32_t t = src[i];
    sun[i] = (uint8_t)(t & 0xffu);
    sun[N + i] = (uint8_t)((t >> 8) & 0xffu);
    rg[i] = (uint16_t)(t & 0xffffu);
}
// linear RGBA upload -> the padded int8 sun channels (border pre-filled with -1)
__global__ void k_sun_pad(const uint32_t *src, int8_t *sunp, int X, int Y, int Z, int SB) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y * Z) return;
    const int x = (int)(i % X), y = (int)((i / X) % Y), z = (int)(i / ((size_t)X * Y));
    const size_t Xp = (size_t)X + 2 * SB, Yp = (size_t)Y + 2 * SB, Zp = (size_t)Z + 2 * SB;
    const size_t j = (size_t)(x + SB) + Xp * ((size_t)(y + SB) + Yp * (size_t)(z + SB));
    const uint32_t t = src[i];
    sunp[j] = (int8_t)(t & 0xffu);
    sunp[Xp * Yp * Zp + j] = (int8_t)((t >> 8) & 0xffu);
}
// ---- first-step bits of an exit copy (DESIGN.md §3 "Sun exit tables", the
// first step).  A marked cell c (value < 0) gets bit a (a = face axis) when
// the 2 x 2 block c + {0, s_j} x {0, s_k} of the two other axes is marked
// too: the value becomes -1 - bits (-1 .. -8; every negative value is the
// march's exit).  k_render reads the bits at a fragment's air cell: a first
// step from the face lands in that block, so the march can end before it.
__global__ void k_exit_face_bits(int8_t *cp, int X, int Y, int Z, int SB, int SXp, size_t SXpYp, int sx, int sy,
                                 int sz) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y * Z) return;
    const int x = (int)(i % X), y = (int)((i / X) % Y), z = (int)(i / ((size_t)X * Y));
    const size_t p = (size_t)(x + SB) + (size_t)SXp * (size_t)(y + SB) + SXpYp * (size_t)(z + SB);
    if (cp[p] >= 0) return;
    const ptrdiff_t dx = sx, dy = (ptrdiff_t)sy * SXp, dz = (ptrdiff_t)sz * (ptrdiff_t)SXpYp;
    auto m = [&](ptrdiff_t o) { return cp[p + o] < 0; };      // marked (any negative value, border included)
    const int bx = m(dy) && m(dz) && m(dy + dz);
    const int by = m(dx) && m(dz) && m(dx + dz);
    const int bz = m(dx) && m(dy) && m(dx + dy);
    cp[p] = (int8_t)(-1 - (bx | (by << 1) | (bz << 2)));
}
// ---- orthant-exit march copies (DESIGN.md §3 "Orthant exit").  For ray
// octant o (bit i: r_i > 0) and its channel (R if r_z > 0, else G), a cell
// whose orthant ahead -- every cell c' with c'_i >= c_i on a positive axis,
// <= on a negative one, inside the grid -- holds no 0 texel becomes -1 (the
// "left the grid" mark).  Three one-sided OR scans of "texel == 0": along x
// (one lane per row), y, then z, the last one writing the copy.
__global__ void k_ox_x(const int8_t *ch, uint8_t *fl, int X, int Y, int Z, int SB, int SXp, size_t SXpYp, int sx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;     // (y, z) row
    if (i >= (size_t)Y * Z) return;
    const int y = (int)(i % Y), z = (int)(i / Y);
    const int8_t *src = ch + (size_t)SB + (size_t)SXp * (size_t)(y + SB) + SXpYp * (size_t)(z + SB);
    uint8_t *dst = fl + (size_t)X * i;
    uint8_t acc = 0;
    for (int k = 0; k < X; k++) {
        const int x = sx > 0 ? X - 1 - k : k;                          // from the far end of the ray's side
        acc |= src[x] == 0 ? 1 : 0;
        dst[x] = acc;
    }
}
__global__ void k_ox_y(uint8_t *fl, int X, int Y, int Z, int sy) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;     // (x, z), x fastest: coalesced
    if (i >= (size_t)X * Z) return;
    const int x = (int)(i % X), z = (int)(i / X);
    uint8_t *col = fl + (size_t)x + (size_t)X * Y * z;
    uint8_t acc = 0;
    for (int k = 0; k < Y; k++) {
        const int y = sy > 0 ? Y - 1 - k : k;
        acc |= col[(size_t)X * y];
        col[(size_t)X * y] = acc;
    }
}
__global__ void k_ox_z(const int8_t *ch, const uint8_t *fl, int8_t *out, int X, int Y, int Z, int SB, int SXp,
                       size_t SXpYp, int sz) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;     // (x, y), x fastest
    if (i >= (size_t)X * Y) return;
    const int x = (int)(i % X), y = (int)(i / X);
    const size_t p0 = (size_t)(x + SB) + (size_t)SXp * (size_t)(y + SB) + SXpYp * (size_t)SB;
    uint8_t acc = 0;
    for (int k = 0; k < Z; k++) {
        const int z = sz > 0 ? Z - 1 - k : k;
        acc |= fl[i + (size_t)X * Y * z];
        const size_t p = p0 + SXpYp * (size_t)z;
        out[p] = acc ? ch[p] : (int8_t)-1;
    }
}
// One layer z of a cone copy (oracle vxo_field_exit with a finite window):
// D(x, y, z) = AND over i <= kx, j <= ky of [T(x', y', z) != 0 and
// D(x', y', z + 1)], x' = x + i*sx, y' = y + j*sy; the channel's and the
// copy's -1 border make cells outside the grid true (kx, ky <= SB), and layer
// Z of the copy is border.  Layers are launched from the top down.
__global__ void k_sun_cone_layer(const int8_t *ch, int8_t *out, int X, int Y, int z, int SB, int SXp, size_t SXpYp,
                                 int sx, int sy, int kx, int ky) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;     // (x, y), x fastest
    if (i >= (size_t)X * Y) return;
    const int x = (int)(i % X), y = (int)(i / X);
    const size_t p = (size_t)(x + SB) + (size_t)SXp * (size_t)(y + SB) + SXpYp * (size_t)(z + SB);
    bool d = true;
    for (int j = 0; j <= ky; j++)
        for (int k = 0; k <= kx; k++) {
            const size_t q = p + (ptrdiff_t)(k * sx) + (ptrdiff_t)(j * sy) * SXp;
            d = d && ch[q] != 0 && out[q + SXpYp] == (int8_t)-1;
        }
    out[p] = d ? (int8_t)-1 : ch[p];
}
// ---- one layer z of the sun doom table (oracle vxo_field_doom; DESIGN.md §3
// "Doom table"), sun-aligned coordinates (x' = x if sx > 0, else X - 1 - x).
// d1 = the sub-cell states at height z + 1 (GX x GY, 255 = leaves the grid),
// d0 = those at height z.  A block (4 waves) takes 8 x 8 cells = 64 x 64
// sub-cells, one sub-cell column per lane: it stages d1 over the sub-cells its
// windows reach (the cells' [Q x' - 1, Q x' + Q + xhi] and the states' [gx +
// xlo, gx + xhi], xlo >= -1) in LDS, takes the window maxima separably (rows
// per wave; a cell's wide row window split over 8 lanes and joined by lane
// shuffles), writes d0 and turns each doomed cell (h <= hmax) of the cone copy
// whose march texel is >= 1 into kDoomBase - doom_cross(h).  Solid = R = G = 0
// (sdf.cpp:430) inside the grid.  No integer division: every loop walks rows
// by wave and columns by lane.
// xhi <= ceil(Q (4 + 1/64)) = 4 Q + 1 (cone plans: |r_x / r_z| <= 4)
constexpr int kDoomT = 8, kDoomS = kDoomT * kDoomQ, kDoomXhi = 4 * kDoomQ + 1, kDoomW = kDoomS + 2 + kDoomXhi + 1;
static_assert(kDoomS == 64 && kDoomQ == 8, "k_doom_layer maps one sub-cell column to each lane of a wave");
__global__ void __launch_bounds__(256) k_doom_layer(const int8_t *sunp, size_t np, int8_t *sunc, const uint8_t *d1,
                                                    uint8_t *d0, int X, int Y, int z, int SB, int SXp, size_t SXpYp,
                                                    int sx, int sy, int xlo, int xhi, int ylo, int yhi,
                                                    int hmax) {
    __shared__ uint8_t s_d[kDoomW][kDoomW];       // d1 rows H0 - 1 .., columns G0 - 1 ..
    __shared__ uint8_t s_rx[kDoomW][kDoomS];      // row maxima over the states' x windows
    __shared__ uint8_t s_rc[kDoomW][kDoomT];      // row maxima over the cells' x windows
    __shared__ uint8_t s_solid[kDoomT + 2][kDoomT + 2];
    const int GX = X * kDoomQ, GY = Y * kDoomQ;
    const int x0 = blockIdx.x * kDoomT, y0 = blockIdx.y * kDoomT;          // aligned cells
    const int G0 = x0 * kDoomQ, H0 = y0 * kDoomQ;
    const int W = kDoomS + 2 + xhi, H = kDoomS + 2 + yhi;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    {
        // every load of the wave's rows issued before the first LDS write (a
        // load-store pair per row kept one load in flight: 735 us a layer at C5)
        constexpr int kRows = (kDoomW + 3) / 4;
        uint32_t v[kRows];
#pragma unroll
        for (int k = 0; k < kRows; k++) {
            const int r = wv + 4 * k, gy = H0 - 1 + r;
            const bool rowin = r < H && gy >= 0 && gy < GY;
            const uint8_t *row = d1 + (size_t)(rowin ? gy : 0) * GX;
            const int g0 = G0 - 1 + lane, g1 = g0 + 64;
            const uint32_t a0 = (rowin && g0 >= 0 && g0 < GX) ? row[g0] : 255u;
            const uint32_t a1 = (rowin && lane + 64 < W && g1 < GX) ? row[g1] : 255u;
            v[k] = a0 | (a1 << 8);
        }
#pragma unroll
        for (int k = 0; k < kRows; k++) {
            const int r = wv + 4 * k;
            if (r < H) {
                s_d[r][lane] = (uint8_t)(v[k] & 0xffu);
                if (lane + 64 < W) s_d[r][lane + 64] = (uint8_t)(v[k] >> 8);
            }
        }
    }
    auto real = [&](int xa, int ya) {            // padded offset of aligned cell (xa, ya, z)
        const int xr = sx > 0 ? xa : X - 1 - xa, yr = sy > 0 ? ya : Y - 1 - ya;
        return (size_t)(xr + SB) + (size_t)SXp * (size_t)(yr + SB) + SXpYp * (size_t)(z + SB);
    };
    if (threadIdx.x < (kDoomT + 2) * (kDoomT + 2)) {
        const int j = threadIdx.x / (kDoomT + 2), i = threadIdx.x - j * (kDoomT + 2);   // constant divisor
        const int xa = x0 - 1 + i, ya = y0 - 1 + j;
        bool solid = false;
        if (xa >= 0 && xa < X && ya >= 0 && ya < Y) {
            const size_t p = real(xa, ya);
            solid = sunp[p] == 0 && sunp[np + p] == 0;
        }
        s_solid[j][i] = solid ? 1 : 0;
    }
    __syncthreads();
    // rows: lane c the state window [c + 1 + xlo, c + 1 + xhi]; the cells' windows
    // [Q i, Q i + Q + 1 + xhi] as 8 lanes per cell (lane = 8 i + p reads Q i + p + 8 k)
    // (windows of up to 4 taps, and the cells' strided reads, as fixed unrolled
    // loops with a wave-uniform bound: no per-tap loop control)
    const int ci = lane >> 3, cp = lane & 7, chi = kDoomQ * ci + kDoomQ + 1 + xhi;
    const int wx = xhi - xlo + 1, wy = yhi - ylo + 1;
    constexpr int kCellTaps = (kDoomQ + 2 + kDoomXhi + 7) / 8;
    for (int r = wv; r < H; r += 4) {
        int m = 0;
        if (wx <= 4) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (k < wx) m = max(m, (int)s_d[r][lane + 1 + xlo + k]);
        } else {
            for (int q = lane + 1 + xlo; q <= lane + 1 + xhi; q++) m = max(m, (int)s_d[r][q]);
        }
        s_rx[r][lane] = (uint8_t)m;
        int mc = 0;
#pragma unroll
        for (int k = 0; k < kCellTaps; k++) {
            const int q = kDoomQ * ci + cp + 8 * k;
            if (q <= chi) mc = max(mc, (int)s_d[r][q]);
        }
        mc = max(mc, __shfl_xor(mc, 1));
        mc = max(mc, __shfl_xor(mc, 2));
        mc = max(mc, __shfl_xor(mc, 4));
        if (cp == 0) s_rc[r][ci] = (uint8_t)mc;
    }
    __syncthreads();
    {                                                                        // states at height z
        const int i = lane, gx = G0 + i;
        const int cx = i >> 3, a = i & 7;
        const int xa0 = cx + 1 - (a == 0 ? 1 : 0), xa1 = cx + 1 + (a == kDoomQ - 1 ? 1 : 0);   // in s_solid
        for (int j = wv; j < kDoomS; j += 4) {
            const int gy = H0 + j;
            if (gx >= GX || gy >= GY) continue;
            int m = 0;
            if (wy <= 4) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (k < wy) m = max(m, (int)s_rx[j + 1 + ylo + k][i]);
            } else {
                for (int r = j + 1 + ylo; r <= j + 1 + yhi; r++) m = max(m, (int)s_rx[r][i]);
            }
            const int cj = j >> 3, b = j & 7;
            const int ya0 = cj + 1 - (b == 0 ? 1 : 0), ya1 = cj + 1 + (b == kDoomQ - 1 ? 1 : 0);
            const bool es = s_solid[ya0][xa0] && s_solid[ya0][xa1] && s_solid[ya1][xa0] && s_solid[ya1][xa1];
            d0[(size_t)gy * GX + gx] = (uint8_t)(es ? 0 : (m < 255 ? min(m + 1, 254) : 255));
        }
    }
    if (threadIdx.x < kDoomT * kDoomT) {                                    // cells of layer z (wave 0)
        const int j = threadIdx.x >> 3, i = threadIdx.x & 7;
        const int xa = x0 + i, ya = y0 + j;
        if (xa < X && ya < Y && !s_solid[j + 1][i + 1]) {
            int m = 0;
            for (int r = kDoomQ * j; r <= kDoomQ * j + kDoomQ + 1 + yhi; r++) m = max(m, (int)s_rc[r][i]);
            if (m < 255 && m + 1 <= hmax) {
                const size_t p = real(xa, ya);
                if (sunc[p] >= 1) sunc[p] = (int8_t)(kDoomBase - doom_cross(m + 1, xhi, yhi));
            }
        }
    }
}
// map.bin B -> the traversal's vis colour, in place in the linear upload (B
// kept in bcol for vx_scene_read_field): the meshed palette indices 1..21
// (sdf.cpp:284 meshes colours < pal_size = 22; render.vert:21) stay, anything
// else -- air = pal_size (sdf.cpp:229-233, 466-468), 0, >= 22 -- is 0: never a surface
__global__ void k_vis(uint32_t *lin, uint8_t *bcol, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint32_t t = lin[i];
    const uint32_t b = (t >> 16) & 0xffu;
    bcol[i] = (uint8_t)b;
    const uint32_t v = b - 1u < (uint32_t)(VX_PAL_SIZE - 1) ? b : 0u;
    lin[i] = (t & 0xff00ffffu) | (v << 16);
}
// 2D mode footprint (sdf.cpp:201-204, 235-239): per column the vis colour of
// the top block with z >= 1 (a block is R == 0, sdf.cpp:430), else 0
__global__ void k_footprint(const uint32_t *lin, uint8_t *c2d, int X, int Y, int Z) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y) return;
    uint8_t c = 0;
    for (int z = Z - 1; z >= 1; z--) {
        const uint32_t t = lin[i + (size_t)X * Y * z];
        if ((t & 0xffu) == 0) {
            c = (uint8_t)((t >> 16) & 0xffu);
            break;
        }
    }
    c2d[i] = c;
}
// One octant copy, linear: RGBA (R, G from rg; B = map.bin's B from bcol; A =
// the cube size = min(ex, ey, ez), since the box grows from the largest cube)
// for vx_scene_read_field_copy, or the raw texels (rg == nullptr: vis colour,
// ex, ey, ez) for vx_scene_read_boxes
__global__ void k_unpack(const uint16_t *rg, const uint8_t *bcol, const uint32_t *prim, uint32_t *dst, int X, int Y,
                         int Z, int P) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)X * Y * Z) return;
    const int x = (int)(i % X), y = (int)((i / X) % Y), z = (int)(i / ((size_t)X * Y));
    const size_t Xp = (size_t)X + 2 * P, Yp = (size_t)Y + 2 * P;
    const uint32_t p = prim[(size_t)(x + P) + Xp * ((size_t)(y + P) + Yp * (size_t)(z + P))];
    if (!rg) {
        dst[i] = p;
        return;
    }
    const uint32_t e0 = (p >> 8) & 0xffu, e1 = (p >> 16) & 0xffu, e2 = p >> 24;
    const uint32_t r = min(e0, min(e1, e2));
    dst[i] = (uint32_t)rg[i] | ((uint32_t)bcol[i] << 16) | (r << 24);
}
}  // namespace

int launch_ao_pairs(const uint16_t *rg, uint32_t *rg2, int X, int Y, int Z, void *stream) {
    const size_t N = ((size_t)X + 1) * Y * Z;
    hipLaunchKernelGGL(k_ao_pairs, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rg, rg2, X, Y,
                       Z);
    return (int)hipGetLastError();
}

int launch_face_quads(const uint32_t *lin, uint16_t *qface, int X, int Y, int Z, int chunk, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(qface, 0xFF, 12 * N, s);
    if (e != hipSuccess) return (int)e;
    const int ncx = (X + chunk - 1) / chunk, ncy = (Y + chunk - 1) / chunk, ncz = (Z + chunk - 1) / chunk;
    const size_t blocks = (size_t)ncx * ncy * ncz * 6 * chunk;
    if (blocks >= (1ull << 31)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_face_quads, dim3((unsigned)blocks), dim3(64), (size_t)chunk * chunk, s, lin, qface, X, Y, Z,
                       chunk, ncy, ncz, N);
    return (int)hipGetLastError();
}

int launch_qcopy(const uint16_t *qface, uint32_t *qcopy, int X, int Y, int Z, int pad, size_t texels, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(qcopy, 0, 8 * texels * 4, s);
    if (e != hipSuccess) return (int)e;
    for (int o = 0; o < 8; o++)
        hipLaunchKernelGGL(k_qcopy, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, qface, qcopy + o * texels, X,
                           Y, Z, pad, o, N);
    return (int)hipGetLastError();
}

int launch_face_quads_interleave(const uint16_t *qface, uint16_t *out, size_t N, void *stream) {
    hipLaunchKernelGGL(k_face_quads_interleave, dim3((unsigned)((6 * N + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, qface, out, N);
    return (int)hipGetLastError();
}

int launch_noise_quads(const uint32_t *noise, uint32_t *noise4, int W, int H, void *stream) {
    const size_t N = (size_t)W * H;
    hipLaunchKernelGGL(k_noise_quads, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, noise,
                       noise4, W, H);
    return (int)hipGetLastError();
}

int launch_field_pack(const uint32_t *lin, uint8_t *sun, uint16_t *rg, int X, int Y, int Z, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    const dim3 grid((unsigned)((N + 255) / 256)), block(256);
    hipLaunchKernelGGL(k_pack_sun, grid, block, 0, (hipStream_t)stream, lin, sun, rg, N);
    return (int)hipGetLastError();
}

int launch_field_psum(const uint32_t *lin, int *S, int X, int Y, int Z, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const size_t nx = (size_t)(Y + 1) * (Z + 1), ny = (size_t)(X + 1) * (Z + 1), nz = (size_t)(X + 1) * (Y + 1);
    hipLaunchKernelGGL(k_psum_x, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, s, lin, S, X, Y, Z);
    hipLaunchKernelGGL(k_psum_yz, dim3((unsigned)((ny + 255) / 256)), dim3(256), 0, s, S, X, Y, Z, 1);
    hipLaunchKernelGGL(k_psum_yz, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, S, X, Y, Z, 2);
    return (int)hipGetLastError();
}

int launch_field_box(const uint32_t *lin, const int *S, uint32_t *prim_copy, int X, int Y, int Z, int pad, int cap,
                     int oct, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    const int sx = oct & 1 ? -1 : 1, sy = oct & 2 ? -1 : 1, sz = oct & 4 ? -1 : 1;
    hipLaunchKernelGGL(k_oct_box, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, lin, S,
                       prim_copy, X, Y, Z, pad, cap, sx, sy, sz);
    return (int)hipGetLastError();
}

int launch_sun_pad(const uint32_t *lin, int8_t *sunp, int X, int Y, int Z, int SB, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    hipLaunchKernelGGL(k_sun_pad, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, lin, sunp, X, Y,
                       Z, SB);
    return (int)hipGetLastError();
}

int launch_sun_exit(const int8_t *sunp, int8_t *sunx, uint8_t *flags, int X, int Y, int Z, int SB, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int SXp = X + 2 * SB, SYp = Y + 2 * SB, SZp = Z + 2 * SB;
    const size_t SXpYp = (size_t)SXp * SYp, np = SXpYp * SZp;
    const size_t nx = (size_t)Y * Z, ny = (size_t)X * Z, nz = (size_t)X * Y;
    for (int o = 0; o < 8; o++) {
        const int sx = o & 1 ? 1 : -1, sy = o & 2 ? 1 : -1, sz = o & 4 ? 1 : -1;
        const int8_t *ch = sz > 0 ? sunp : sunp + np;          // R for up-going rays, G otherwise
        hipLaunchKernelGGL(k_ox_x, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, s, ch, flags, X, Y, Z, SB, SXp,
                           SXpYp, sx);
        hipLaunchKernelGGL(k_ox_y, dim3((unsigned)((ny + 255) / 256)), dim3(256), 0, s, flags, X, Y, Z, sy);
        hipLaunchKernelGGL(k_ox_z, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, ch, flags, sunx + o * np, X,
                           Y, Z, SB, SXp, SXpYp, sz);
        const size_t n = (size_t)X * Y * Z;
        hipLaunchKernelGGL(k_exit_face_bits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, sunx + o * np, X, Y,
                           Z, SB, SXp, SXpYp, sx, sy, sz);
    }
    return (int)hipGetLastError();
}

int launch_sun_cone(const int8_t *sunp, int8_t *sunc, int X, int Y, int Z, int SB, int oct, int kx, int ky,
                    void *stream) {
    if (!(oct & 4) || kx < 0 || ky < 0 || kx > SB || ky > SB) return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const int SXp = X + 2 * SB, SYp = Y + 2 * SB;
    const size_t SXpYp = (size_t)SXp * SYp, n = (size_t)X * Y;
    const int sx = oct & 1 ? 1 : -1, sy = oct & 2 ? 1 : -1;
    for (int z = Z - 1; z >= 0; z--)          // R channel (up-going rays), top layer first
        hipLaunchKernelGGL(k_sun_cone_layer, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, sunp, sunc, X, Y, z,
                           SB, SXp, SXpYp, sx, sy, kx, ky);
    const size_t nc = n * Z;
    hipLaunchKernelGGL(k_exit_face_bits, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, sunc, X, Y, Z, SB, SXp,
                       SXpYp, sx, sy, 1);
    return (int)hipGetLastError();
}

int launch_sun_doom(const int8_t *sunp, int8_t *sunc, int X, int Y, int Z, int SB, const int plan[7], void *stream) {
    const int sx = plan[0], sy = plan[1], xlo = plan[2], xhi = plan[3], ylo = plan[4], yhi = plan[5], hmax = plan[6];
    // the block's staged window (k_doom_layer): xlo, ylo >= -1, xhi, yhi <= kDoomXhi; codes down to -128
    if (xlo < -1 || ylo < -1 || xhi > kDoomXhi || yhi > kDoomXhi || xlo > xhi || ylo > yhi || SB < 1 || hmax < 1 ||
        hmax > kDoomHCap || doom_cross(hmax, xhi, yhi) > 120)
        return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const int SXp = X + 2 * SB, SYp = Y + 2 * SB, SZp = Z + 2 * SB;
    const size_t SXpYp = (size_t)SXp * SYp, np = SXpYp * SZp;
    const size_t G = (size_t)X * Y * kDoomQ * kDoomQ;
    uint8_t *d[2] = {nullptr, nullptr};
    hipError_t e = hipMallocAsync((void **)&d[0], 2 * G, s);
    if (e != hipSuccess) return (int)e;
    d[1] = d[0] + G;
    e = hipMemsetAsync(d[0], 0xFF, G, s);                 // above the top layer: leaves the grid
    if (e == hipSuccess) {
        const dim3 grid((unsigned)((X + kDoomT - 1) / kDoomT), (unsigned)((Y + kDoomT - 1) / kDoomT));
        for (int z = Z - 1, k = 0; z >= 0; z--, k ^= 1)
            hipLaunchKernelGGL(k_doom_layer, grid, dim3(256), 0, s, sunp, np, sunc, d[k], d[k ^ 1], X, Y, z, SB, SXp,
                               SXpYp, sx, sy, xlo, xhi, ylo, yhi, hmax);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(d[0], s);
    return (int)(e != hipSuccess ? e : f);
}

int launch_field_unpack(const uint16_t *rg, const uint8_t *bcol, const uint32_t *prim_copy, uint32_t *out, int X,
                        int Y, int Z, int pad, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rg, bcol,
                       prim_copy, out, X, Y, Z, pad);
    return (int)hipGetLastError();
}

int launch_footprint(const uint32_t *lin, uint8_t *c2d, int X, int Y, int Z, void *stream) {
    const size_t N = (size_t)X * Y;
    hipLaunchKernelGGL(k_footprint, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, lin, c2d,
                       X, Y, Z);
    return (int)hipGetLastError();
}

int launch_field_vis(uint32_t *lin, uint8_t *bcol, int X, int Y, int Z, void *stream) {
    const size_t N = (size_t)X * Y * Z;
    hipLaunchKernelGGL(k_vis, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, lin, bcol, N);
    return (int)hipGetLastError();
}

int launch_field_octant(uint32_t *field, int X, int Y, int Z, int cap, int oct, uint8_t *ga, uint8_t *gb,
                        void *stream) {
    const size_t N = (size_t)X * Y * Z;
    dim3 grid((unsigned)((N + 255) / 256)), block(256);
    hipStream_t s = (hipStream_t)stream;
    const int sx = oct & 1 ? -1 : 1, sy = oct & 2 ? -1 : 1, sz = oct & 4 ? -1 : 1;
    hipLaunchKernelGGL(k_oct_x, grid, block, 0, s, (const uint32_t *)field, ga, X, Y, Z, cap, sx);
    hipLaunchKernelGGL(k_oct_yz, grid, block, 0, s, ga, gb, field, X, Y, Z, cap, 1, sy);
    hipLaunchKernelGGL(k_oct_yz, grid, block, 0, s, gb, ga, field, X, Y, Z, cap, 2, sz);
    return (int)hipGetLastError();
}

}  // namespace vx
