// vx_field.cpp — host-side asset producers.
//
// vx_field_build: map.bin from a palette-index voxel grid, restating the
// distance-field half of src/gen/sdf.cpp (lines 405-470).  The reference runs
// a serial x->y->z sweep (voxmap.h:50-55) whose only cross-cell dependency is
// the diagonal neighbour mid = sdf(x-1, y-1, z-1) clamped (sdf.cpp:439-444).
// For x >= 1 that neighbour lies in plane x-1, so plane x depends only on
// plane x-1: planes are swept in order and the Y*Z cells of a plane run in
// parallel (identical results to the serial sweep).  Plane 0 keeps the serial
// (y, z) order because its clamped neighbour is in the same plane.
//
// vol() (sdf.cpp:63-83) reads the table produced by the recurrence of
// sdf.cpp:407-422 through clamped indices; the recurrence makes the table
// equal to bin on the three 0-planes, and the clamped lower corner means vol()
// only ever sums the table's 3-D differences at cells with x, y, z >= 1.  So
// vol() = number of blocks of the box inside [1,X-1]x[1,Y-1]x[1,Z-1]; we
// compute exactly that from an ordinary prefix sum of bin restricted to
// x, y, z >= 1 (tests compare against the literal oracle restatement).
#include <algorithm>
#include <barrier>
#include <cstring>
#include <thread>
#include <vector>

#include "vx_internal.h"

namespace vx {

namespace {
struct Field {
    int X, Y, Z;
    std::vector<int32_t> pre;   // prefix sum of bin' (bin with 0-planes cleared)
    std::vector<uint8_t> sdf;   // 2 per cell: [0] up (R), [1] down (G)
    const uint8_t *color;
    size_t idx(int x, int y, int z) const { return (size_t)x + (size_t)X * ((size_t)y + (size_t)Y * (size_t)z); }
    int P(int x, int y, int z) const {  // clamped prefix read, as csum() clamps
        x = std::clamp(x, 0, X - 1);
        y = std::clamp(y, 0, Y - 1);
        z = std::clamp(z, 0, Z - 1);
        return pre[idx(x, y, z)];
    }
    int vol(int x0, int y0, int z0, int x1, int y1, int z1) const {
        x0--; y0--; z0--;
        return P(x1, y1, z1) - P(x0, y1, z1) - P(x1, y0, z1) - P(x1, y1, z0) + P(x0, y0, z1) + P(x0, y1, z0) +
               P(x1, y0, z0) - P(x0, y0, z0);
    }
    void cell(int x, int y, int z) {
        const size_t i = idx(x, y, z);
        if (color[i] != 0) return;  // blocks keep 0
        for (int o = 0; o < 2; o++) {
            int mn = 1, mx = o == 0 ? Z : z;
            if (x + y + z > 0) {
                const int mid = sdf[2 * idx(std::max(x - 1, 0), std::max(y - 1, 0), std::max(z - 1, 0)) + o];
                mn = std::max(mn, mid - 1);
                mx = std::min(mx, mid + 1);
            }
            int r = mn;
            while (r < mx && vol(x - r, y - r, z - o * r, x + r, y + r, z + (1 - o) * r) == 0) r++;
            sdf[2 * i + o] = (uint8_t)r;
        }
    }
};
}  // namespace

int field_build(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba, int n_threads) {
    if (!color || !rgba || X <= 0 || Y <= 0 || Z <= 0 || X > 65535 || Y > 65535 || Z > 255)
        return set_error(VX_EINVAL, "vx_field_build: bad arguments (need 0<X,Y<=65535, 0<Z<=255)");
    Field f;
    f.X = X; f.Y = Y; f.Z = Z;
    f.color = color;
    const size_t N = (size_t)X * Y * Z;
    if (N > (size_t)INT32_MAX) return set_error(VX_EINVAL, "vx_field_build: grid too large for int32 volume sums");
    try {
        f.pre.assign(N, 0);
        f.sdf.assign(2 * N, 0);
    } catch (...) {
        return set_error(VX_ENOMEM, "vx_field_build: out of host memory");
    }
    // prefix sum of bin' = bin on x,y,z >= 1, else 0: three separable passes
    for (int z = 0; z < Z; z++)
        for (int y = 0; y < Y; y++) {
            int run = 0;
            for (int x = 0; x < X; x++) {
                const size_t i = f.idx(x, y, z);
                run += (x >= 1 && y >= 1 && z >= 1 && color[i] != 0) ? 1 : 0;
                f.pre[i] = run;
            }
        }
    for (int z = 0; z < Z; z++)
        for (int y = 1; y < Y; y++)
            for (int x = 0; x < X; x++) f.pre[f.idx(x, y, z)] += f.pre[f.idx(x, y - 1, z)];
    for (int z = 1; z < Z; z++)
        for (int y = 0; y < Y; y++)
            for (int x = 0; x < X; x++) f.pre[f.idx(x, y, z)] += f.pre[f.idx(x, y, z - 1)];

    // plane 0: the reference's serial order
    for (int y = 0; y < Y; y++)
        for (int z = 0; z < Z; z++) f.cell(0, y, z);
    // planes 1..X-1: plane-wavefront, cells of a plane in parallel
    int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::min(nt, 64);
    const int plane = Y * Z;
    if (nt <= 1 || X == 1) {
        for (int x = 1; x < X; x++)
            for (int k = 0; k < plane; k++) f.cell(x, k / Z, k % Z);
    } else {
        std::barrier sync(nt);
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; t++)
            pool.emplace_back([&, t] {
                const int lo = (int)((long long)plane * t / nt), hi = (int)((long long)plane * (t + 1) / nt);
                for (int x = 1; x < X; x++) {
                    for (int k = lo; k < hi; k++) f.cell(x, k / Z, k % Z);
                    sync.arrive_and_wait();
                }
            });
        for (auto &th : pool) th.join();
    }
    // map.bin texels: R = up, G = down, B = remapped palette index, A = 0
    // (sdf.cpp:462-470); the remap turns air into pal_size (sdf.cpp:229-233)
    for (size_t i = 0; i < N; i++) {
        rgba[4 * i + 0] = f.sdf[2 * i + 0];
        rgba[4 * i + 1] = f.sdf[2 * i + 1];
        rgba[4 * i + 2] = color[i] ? color[i] : (uint8_t)VX_PAL_SIZE;
        rgba[4 * i + 3] = 0;
    }
    return VX_OK;
}

// ---- synthetic noise texture in the layout of noise.cpp:34-41 ----------
// RGB = white noise, A = tileable 10-octave value-noise fBm mapped like
// noise.cpp:29 (128 + clamp(300 n, -128, 127)).  Used only when a scene is
// created without a noise texture; the reference's own res/noise.bin.gz ships
// as voxmap_amd/data/noise.bin.gz and is what the tests, smoke() and bench.py
// load (SHA-256 pinned, tests/test_reference_pins.py).
static inline uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}

int noise_synth(uint32_t seed, int w, int h, uint8_t *out) {
    if (!out || w <= 0 || h <= 0 || (w & (w - 1)) || (h & (h - 1)))
        return set_error(VX_EINVAL, "vx_noise_synth: w, h must be powers of two");
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            double n = 0.0;
            for (int o = 0; o < 10; o++) {
                const int cells = 4 << o;              // lattice cells across the torus
                const int cx = std::min(cells, w), cy = std::min(cells, h);
                const double fx = (double)x * cx / w, fy = (double)y * cy / h;
                const int ix = (int)fx, iy = (int)fy;
                const double tx = fx - ix, ty = fy - iy;
                const double sx = tx * tx * (3 - 2 * tx), sy = ty * ty * (3 - 2 * ty);
                auto lat = [&](int i, int j) {
                    return (hash3((uint32_t)(i % cx), (uint32_t)(j % cy), seed * 16u + (uint32_t)o) >> 8) /
                               (double)(1u << 24) * 2.0 - 1.0;
                };
                const double v = (lat(ix, iy) * (1 - sx) + lat(ix + 1, iy) * sx) * (1 - sy) +
                                 (lat(ix, iy + 1) * (1 - sx) + lat(ix + 1, iy + 1) * sx) * sy;
                n += 0.45 * v / (double)(1 << o);
            }
            const size_t i = 4 * ((size_t)y * w + x);
            const uint32_t wn = hash3((uint32_t)x, (uint32_t)y, seed ^ 0xA5A5A5A5u);
            out[i + 0] = (uint8_t)(wn & 0xff);
            out[i + 1] = (uint8_t)((wn >> 8) & 0xff);
            out[i + 2] = (uint8_t)((wn >> 16) & 0xff);
            out[i + 3] = (uint8_t)(128 + std::clamp((int)(300 * n), -128, 127));
        }
    return VX_OK;
}

}  // namespace vx

namespace vx {

// ---- 2D mode mesh (sdf.cpp:362-401) --------------------------------------
// c2d (x fastest, X*Y): the vis colour of each column's top block with z >= 1
// (sdf.cpp:201-204: z2d starts at 0 and only z > z2d replaces it), 0 where
// there is none or it is not a meshed index.  Greedy quads per colour
// c = 1..pal_size-1 in ascending order (sdf.cpp:367; colour 0 never occurs
// after the remap, air = pal_size is never meshed), cells visited x-major
// then y (forXY, voxmap.h:45-49), each quad grown along x while the mask
// holds (:378), then along y while the whole row of w cells holds (:380-385),
// its cells then cleared (:391-395).  origin[i] = x0 | y0 << 16 of the quad
// covering cell i (the quad's corner is v_cellPos, render.vert:27).
void mesh2d(const uint8_t *c2d, int X, int Y, std::vector<Quad2d> &quads, uint32_t *origin) {
    quads.clear();
    std::vector<uint8_t> mask((size_t)X * Y);
    auto at = [&](int x, int y) -> uint8_t & { return mask[(size_t)y * X + x]; };
    for (int color = 1; color < VX_PAL_SIZE; color++) {
        bool any = false;
        for (size_t i = 0; i < mask.size(); i++) any |= (mask[i] = c2d[i] == color) != 0;
        if (!any) continue;
        for (int x = 0; x < X; x++)
            for (int y = 0; y < Y; y++) {
                if (!at(x, y)) continue;
                int w = 1, h = 1;
                while (x + w < X && at(x + w, y)) w++;
                for (; y + h < Y; h++) {
                    bool row = true;
                    for (int k = 0; k < w && row; k++) row = at(x + k, y + h) != 0;
                    if (!row) break;
                }
                quads.push_back({x, y, w, h, color});
                for (int l = 0; l < h; l++)
                    for (int k = 0; k < w; k++) {
                        at(x + k, y + l) = 0;
                        if (origin) origin[(size_t)(y + l) * X + (x + k)] = (uint32_t)x | ((uint32_t)y << 16);
                    }
            }
    }
}

// vert2d records (sdf.cpp:154-173): quad2d(x, y, w, 0, 0, h) = tri2d((0,0),
// (w,0), (0,h)) + tri2d((0,h), (w,0), (w,h)); each vertex i16 x, y, 0, dx, dy,
// 0, u8 colour, 0, id (2 for glass = pal_size - 1, :388), 0 -- 16 bytes.
size_t vertex2d_bytes(const std::vector<Quad2d> &quads, uint8_t *out, size_t cap) {
    const size_t need = quads.size() * 6 * 16;
    if (!out || cap < need) return need;
    uint8_t *p = out;
    auto i16 = [&](int v) { *p++ = (uint8_t)(v & 0xff); *p++ = (uint8_t)((v >> 8) & 0xff); };
    for (const Quad2d &q : quads) {
        const int d[6][2] = {{0, 0}, {q.w, 0}, {0, q.h}, {0, q.h}, {q.w, 0}, {q.w, q.h}};
        for (int v = 0; v < 6; v++) {
            i16(q.x); i16(q.y); i16(0);
            i16(d[v][0]); i16(d[v][1]); i16(0);
            *p++ = (uint8_t)q.color;
            *p++ = 0;
            *p++ = (uint8_t)(q.color == VX_GLASS ? 2 : 0);
            *p++ = 0;
        }
    }
    return need;
}

}  // namespace vx

extern "C" int vx_vertex2d(const uint8_t *rgba, int X, int Y, int Z, void *out, size_t cap, size_t *out_size) {
    using namespace vx;
    if (!rgba || !out_size || X <= 0 || Y <= 0 || Z <= 0 || X > 65535 || Y > 65535)
        return set_error(VX_EINVAL, "vx_vertex2d: bad arguments");
    // footprint: each column's top block (R == 0, sdf.cpp:430) with z >= 1 (sdf.cpp:201-204)
    const size_t n = (size_t)X * Y;
    std::vector<uint8_t> c2d(n, 0);
    for (size_t i = 0; i < n; i++)
        for (int z = Z - 1; z >= 1; z--) {
            const uint8_t *t = rgba + 4 * (i + n * (size_t)z);
            if (t[0] == 0) {
                c2d[i] = (t[2] >= 1 && t[2] < VX_PAL_SIZE) ? t[2] : 0;
                break;
            }
        }
    std::vector<Quad2d> quads;
    mesh2d(c2d.data(), X, Y, quads, nullptr);
    *out_size = vertex2d_bytes(quads, nullptr, 0);
    if (!out) return VX_OK;
    if (cap < *out_size) return set_error(VX_EINVAL, "vx_vertex2d: output buffer too small");
    vertex2d_bytes(quads, static_cast<uint8_t *>(out), cap);
    return VX_OK;
}
