// vx_host.cpp — the host-only half of the C ABI (include/voxmap.h): every
// entry point and check that runs without a GPU.  It holds all handling of
// untrusted input -- the map / noise containers (.bin, .bin.gz, .blob: the
// reference's D.fetch path, utils.js:10-30, render.js:52-58), scene
// descriptions, frame parameters -- plus the camera/sun helpers (map.js:349-402,
// math.js:16-49), the field builder front end and the multi-GPU deal.  No HIP:
// tests/test_sanitizers.py builds this file with vx_codec.cpp, vx_field.cpp and
// vx_frame.cpp under -fsanitize=address,undefined and drives it with corrupt,
// truncated and hostile inputs.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "vx_internal.h"

namespace vx {
static thread_local std::string g_err;
const char *last_error() { return g_err.c_str(); }
int set_error(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
}  // namespace vx


using namespace vx;

static int read_file(const char *path, std::vector<unsigned char> &buf) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return set_error(VX_EIO, std::string("cannot open ") + path);
    buf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    if (f.bad()) return set_error(VX_EIO, std::string("read error on ") + path);
    return VX_OK;
}

static int load_asset(const char *path, const void *bytes, size_t size, int format, const char *key,
                      size_t expect, const char *what, std::vector<unsigned char> &out) {
    std::vector<unsigned char> raw;
    const unsigned char *src = static_cast<const unsigned char *>(bytes);
    size_t n = size;
    if (path) {
        int rc = read_file(path, raw);
        if (rc) return rc;
        src = raw.data();
        n = raw.size();
        if (format == VX_FORMAT_AUTO) format = format_from_path(path);
    } else if (format == VX_FORMAT_AUTO) {
        // sniff: gzip magic, else raw if the size matches, else assume blob
        format = (n >= 2 && src[0] == 0x1f && src[1] == 0x8b) ? VX_FORMAT_BIN_GZ
                 : (n == expect)                               ? VX_FORMAT_BIN
                                                               : VX_FORMAT_BLOB;
    }
    int rc = decode_container(src, n, format, key, out, expect);
    if (rc) return set_error(rc, std::string(what) + ": " + last_error());
    if (out.size() != expect)
        return set_error(VX_ESIZE, std::string(what) + ": decoded " + std::to_string(out.size()) +
                                       " bytes, expected " + std::to_string(expect));
    return VX_OK;
}


FieldLayout vx::field_layout(int X, int Y, int Z, int cap) {
    FieldLayout L;
    L.pad = cap;
    L.Xp = X + 2 * cap;
    L.Yp = Y + 2 * cap;
    L.Zp = Z + 2 * cap;
    L.texels = (size_t)L.Xp * L.Yp * L.Zp;
    return L;
}

int vx::scene_inputs(const vx_scene_desc *d, SceneInputs &in) {
    if (!d) return set_error(VX_EINVAL, "vx_scene_create: null argument");
    const int X = d->X ? d->X : 1024, Y = d->Y ? d->Y : 256, Z = d->Z ? d->Z : 32;
    const int NW = d->noise_w ? d->noise_w : 1024, NH = d->noise_h ? d->noise_h : 1024;
    if (X <= 0 || Y <= 0 || Z <= 0 || X > 65535 || Y > 65535 || Z > 255)
        return set_error(VX_EINVAL, "vx_scene_create: dims out of range");
    int cap = d->dist_cap ? d->dist_cap : VX_DEFAULT_DIST_CAP;
    if (cap < 1 || cap > 255) return set_error(VX_EINVAL, "dist_cap must be in [1,255]");
    // the default cap's border: a field that fits with the ABI <= 8 default (32)
    // but not with 64 takes 32 instead of failing
    auto fits = [&](int c) {
        const FieldLayout Lc = field_layout(X, Y, Z, c);
        return Lc.texels < (1ull << 31) && (unsigned long long)Lc.Xp * Lc.Yp < (1ull << 23);
    };
    if (!d->dist_cap && !fits(cap) && fits(VX_FALLBACK_DIST_CAP)) cap = VX_FALLBACK_DIST_CAP;
    const FieldLayout L = field_layout(X, Y, Z, cap);
    // 32-bit buffer byte offsets and 24-bit index products in the kernels
    if (L.texels >= (1ull << 31) || (unsigned long long)L.Xp * L.Yp >= (1ull << 23))
        return set_error(VX_EINVAL, "vx_scene_create: field too large (padded grid must be < 2^31 cells)");
    // the AO pair array (4 B per cell, X + 1 per row) and the noise quad planes
    // (4 planes of 4 B per texel) are addressed with 32-bit byte offsets
    if (4ull * ((unsigned long long)X + 1) * Y * Z >= (1ull << 32))
        return set_error(VX_EINVAL, "vx_scene_create: field too large (4*(X+1)*Y*Z must be < 2^32)");
    if ((NW & (NW - 1)) || (NH & (NH - 1))) return set_error(VX_EINVAL, "noise dims must be powers of two");
    if (16ull * (unsigned long long)NW * NH >= (1ull << 32))
        return set_error(VX_EINVAL, "vx_scene_create: noise too large (16*w*h must be < 2^32)");
    // CHUNK of the greedy mesh whose quads give the fragments' G-buffer split
    // (voxmap.h:9: CHUNK = Z); offsets within a chunk are stored in 8 bits
    const int chunk = d->mesh_chunk ? d->mesh_chunk : Z;
    if (chunk < 1 || chunk > 255) return set_error(VX_EINVAL, "mesh_chunk must be in [1,255] (0: Z)");
    if (!!d->map_path == !!d->map_bytes) return set_error(VX_EINVAL, "set exactly one of map_path / map_bytes");
    const size_t field_bytes = (size_t)X * Y * Z * 4, noise_bytes = (size_t)NW * NH * 4;

    std::vector<unsigned char> &field = in.field, &noise = in.noise;
    const bool from_grid = d->map_format == VX_FORMAT_GRID;
    int rc = VX_OK;
    if (from_grid) {   // palette grid: the field is built on the device below
        if (!d->map_bytes || d->map_size != (size_t)X * Y * Z)
            return set_error(VX_ESIZE, "map grid: need map_bytes of X*Y*Z palette indices");
    } else {
        rc = load_asset(d->map_path, d->map_bytes, d->map_size, d->map_format, d->key_jwk_k, field_bytes, "map",
                        field);
        if (rc) return rc;
    }
    // the padded int8 sun march (march_pad) needs every R/G value <= Z: a step
    // then moves at most Z + 1 cells per axis and lands in the -1 border of
    // Z + 2 cells, and no value reads as a negative int8.  sdf.cpp and the GPU
    // builder cap R at Z and G at z (sdf.cpp:437); a hand-made map.bin may
    // not, and then the bounds-checked u8 march runs instead.
    int max_rg = 0;
    if (!from_grid) {
        const size_t n = (size_t)X * Y * Z;
        unsigned char m = 0;
        for (size_t i = 0; i < n; i++) m = std::max(m, std::max(field[4 * i], field[4 * i + 1]));
        max_rg = m;
    }
    if (d->noise_path || d->noise_bytes) {
        rc = load_asset(d->noise_path, d->noise_bytes, d->noise_size, d->noise_format, d->key_jwk_k, noise_bytes,
                        "noise", noise);
        if (rc) return rc;
    } else {
        noise.resize(noise_bytes);
        rc = noise_synth(d->noise_seed, NW, NH, noise.data());
        if (rc) return rc;
    }
    in.X = X; in.Y = Y; in.Z = Z; in.NW = NW; in.NH = NH; in.cap = cap; in.chunk = chunk;
    in.from_grid = from_grid;
    in.max_rg = max_rg;
    return VX_OK;
}

int vx::check_frame(const vx_frame_params *p, int w, int h, int fmt) {
    if (!p) return set_error(VX_EINVAL, "null scene/params");
    if (w <= 0 || h <= 0 || w > 32768 || h > 32768) return set_error(VX_EINVAL, "frame size out of range");
    if (fmt != VX_PIXEL_RGBA32F && fmt != VX_PIXEL_RGBA8) return set_error(VX_EINVAL, "unknown pixel format");
    for (int i = 0; i < 3; i++)
        if (!std::isfinite(p->cam_fract[i]) || !std::isfinite(p->ray_fwd[i]) || !std::isfinite(p->ray_right[i]) ||
            !std::isfinite(p->ray_up[i]) || !std::isfinite(p->sun_dir[i]))
            return set_error(VX_EINVAL, "non-finite frame parameter");
    // u_fractPos is fract(position) (render.js:289-290); the primary traversal
    // relies on 0 <= o < 1 and on camera-relative cells below 2^22
    for (int i = 0; i < 3; i++) {
        if (!(p->cam_fract[i] >= 0.0f && p->cam_fract[i] < 1.0f))
            return set_error(VX_EINVAL, "cam_fract must be in [0, 1)");
        if (p->cam_cell[i] <= -(1 << 22) || p->cam_cell[i] >= (1 << 22))
            return set_error(VX_EINVAL, "cam_cell out of range (|cell| < 2^22)");
    }
    if (p->shadow_samples > VX_MAX_SHADOW_SAMPLES)
        return set_error(VX_EINVAL, "shadow_samples must be <= VX_MAX_SHADOW_SAMPLES (16)");
    if (p->shadow_samples > 1 && !(p->sun_radius >= 0.0f && p->sun_radius <= 0.5f))
        return set_error(VX_EINVAL, "sun_radius must be in [0, 0.5] for soft shadows");
    return VX_OK;
}


extern "C" {

const char *vx_last_error(void) { return last_error(); }
int vx_abi_version(void) { return VX_ABI_VERSION; }

// ---- camera / sun (map.js:349-402, math.js:16-49,106-178) ----------------
static void mat_mul(const double a[16], const double b[16], double r[16]) {   // column-major a*b (math.js:51-102)
    for (int c = 0; c < 4; c++)
        for (int rr = 0; rr < 4; rr++) {
            double acc = 0.0;
            for (int k = 0; k < 4; k++) acc += a[k * 4 + rr] * b[c * 4 + k];
            r[c * 4 + rr] = acc;
        }
}
static void rot_x(double t, double m[16]) {   // math.js:144-154
    const double c = std::cos(t), s = std::sin(t);
    const double v[16] = {1, 0, 0, 0, 0, c, s, 0, 0, -s, c, 0, 0, 0, 0, 1};
    std::memcpy(m, v, sizeof v);
}
static void rot_z(double t, double m[16]) {   // math.js:168-178
    const double c = std::cos(t), s = std::sin(t);
    const double v[16] = {c, s, 0, 0, -s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    std::memcpy(m, v, sizeof v);
}
static void translation(double x, double y, double z, double m[16]) {   // math.js:137-142
    const double v[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, x, y, z, 1};
    std::memcpy(m, v, sizeof v);
}
static void set_cam(const double pos[3], vx_frame_params *p) {
    for (int i = 0; i < 3; i++) {
        const double fl = std::floor(pos[i]);
        p->cam_cell[i] = (int)fl;               // render.js:289 position.map(floor)
        p->cam_fract[i] = (float)(pos[i] - fl); // render.js:290 position.map(fract)
        if (p->cam_fract[i] >= 1.0f) {          // fract within 2^-25 of 1 rounds up in fp32:
            p->cam_cell[i] += 1;                // the same point as cell + 1, fract 0
            p->cam_fract[i] = 0.0f;
        }
    }
}

int vx_frame_from_orbit(const double sbj[3], const double rot[3], int w, int h, vx_frame_params *p) {
    if (!sbj || !rot || !p || w <= 0 || h <= 0) return set_error(VX_EINVAL, "vx_frame_from_orbit: bad arguments");
    // map.js:373-380: orbit = T(sbj) Rz(rz) Rx(rx) T(0,0,R), R = sbj.z; pos = orbit * (0,0,0,1)
    double T1[16], Rz[16], Rx[16], T2[16], m1[16], m2[16], orbit[16];
    translation(sbj[0], sbj[1], sbj[2], T1);
    rot_z(rot[2], Rz);
    rot_x(rot[0], Rx);
    translation(0, 0, sbj[2], T2);
    mat_mul(T1, Rz, m1);
    mat_mul(m1, Rx, m2);
    mat_mul(m2, T2, orbit);
    const double pos[3] = {orbit[12], orbit[13], orbit[14]};
    set_cam(pos, p);
    // map.js:382-391 + math.js:37-42: P = projection(f, aspect) with x scale f/sqrt(a),
    // y scale f*sqrt(a); view = Rx(-rx) Rz(-rz) T(-pos).  Eye ray for NDC (nx, ny):
    // (nx*sqrt(a)/f, ny/(f*sqrt(a)), -1); world = Rz(rz) Rx(rx) eye.
    const double f = 1.0 / std::tan(60.0 * M_PI / 360.0);
    const double sa = std::sqrt((double)w / (double)h);
    double RzRx[16];
    mat_mul(Rz, Rx, RzRx);
    auto apply = [&](double ex, double ey, double ez, float out[3]) {
        for (int r = 0; r < 3; r++) out[r] = (float)(RzRx[0 * 4 + r] * ex + RzRx[1 * 4 + r] * ey + RzRx[2 * 4 + r] * ez);
    };
    apply(0, 0, -1, p->ray_fwd);
    apply(sa / f, 0, 0, p->ray_right);
    apply(0, 1.0 / (f * sa), 0, p->ray_up);
    return VX_OK;
}

int vx_frame_from_matrix(const float m[16], const double cam_pos[3], vx_frame_params *p) {
    if (!m || !cam_pos || !p) return set_error(VX_EINVAL, "vx_frame_from_matrix: null argument");
    // invert the column-major u_matrix (double Gauss-Jordan), unproject NDC
    // points on the far side of the near plane, subtract the camera position.
    double a[4][8];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            a[r][c] = m[c * 4 + r];
            a[r][4 + c] = r == c ? 1.0 : 0.0;
        }
    for (int c = 0; c < 4; c++) {
        int piv = c;
        for (int r = c + 1; r < 4; r++)
            if (std::fabs(a[r][c]) > std::fabs(a[piv][c])) piv = r;
        if (std::fabs(a[piv][c]) < 1e-300) return set_error(VX_EINVAL, "u_matrix is singular");
        for (int k = 0; k < 8; k++) std::swap(a[c][k], a[piv][k]);
        const double d = a[c][c];
        for (int k = 0; k < 8; k++) a[c][k] /= d;
        for (int r = 0; r < 4; r++)
            if (r != c) {
                const double fct = a[r][c];
                for (int k = 0; k < 8; k++) a[r][k] -= fct * a[c][k];
            }
    }
    auto unproj = [&](double x, double y, double out[3]) {
        double v[4];
        for (int r = 0; r < 4; r++) v[r] = a[r][4] * x + a[r][5] * y + a[r][6] * 1.0 + a[r][7] * 1.0;
        for (int r = 0; r < 3; r++) out[r] = v[r] / v[3] - cam_pos[r];
    };
    double c0[3], cx[3], cy[3];
    unproj(0, 0, c0);
    unproj(1, 0, cx);
    unproj(0, 1, cy);
    // scale so the forward component has unit length along the eye axis
    const double len = std::sqrt(c0[0] * c0[0] + c0[1] * c0[1] + c0[2] * c0[2]);
    if (!(len > 0)) return set_error(VX_EINVAL, "degenerate u_matrix");
    for (int i = 0; i < 3; i++) {
        p->ray_fwd[i] = (float)(c0[i] / len);
        p->ray_right[i] = (float)((cx[i] - c0[i]) / len);
        p->ray_up[i] = (float)((cy[i] - c0[i]) / len);
    }
    set_cam(cam_pos, p);
    return VX_OK;
}

void vx_sun_from_hour(double hour, float sun[3]) {   // map.js:399-402
    sun[0] = (float)(std::sin(hour) * std::sqrt(3.0 / 4.0));
    sun[1] = (float)(std::sin(hour) * std::sqrt(1.0 / 4.0));
    sun[2] = (float)std::fabs(std::cos(hour));
}

int vx_sun_samples(const float sun[3], float radius, int n, float out[][3]) {
    if (!sun || !out) return set_error(VX_EINVAL, "vx_sun_samples: null argument");
    sun_samples(sun, radius, n, out);
    return VX_OK;
}

int vx_decode(const void *in, size_t n, int format, const char *key, void *out, size_t out_cap, size_t *out_size) {
    if (!in || !out_size) return set_error(VX_EINVAL, "vx_decode: null argument");
    std::vector<unsigned char> buf;
    int rc = decode_container(static_cast<const unsigned char *>(in), n, format, key, buf, 0);
    if (rc) return rc;
    *out_size = buf.size();
    if (!out) return VX_OK;   // size query
    if (out_cap < buf.size()) return set_error(VX_EINVAL, "vx_decode: output buffer too small");
    std::memcpy(out, buf.data(), buf.size());
    return VX_OK;
}

int vx_blob_encrypt(const void *in, size_t n, const char *key, void *out, size_t out_cap, size_t *out_size) {
    if (!in || !out_size) return set_error(VX_EINVAL, "vx_blob_encrypt: null argument");
    std::vector<unsigned char> buf;
    int rc = encrypt_blob(static_cast<const unsigned char *>(in), n, key, buf);
    if (rc) return rc;
    *out_size = buf.size();
    if (!out) return VX_OK;   // size query
    if (out_cap < buf.size()) return set_error(VX_EINVAL, "vx_blob_encrypt: output buffer too small");
    std::memcpy(out, buf.data(), buf.size());
    return VX_OK;
}

int vx_field_build(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba_out, int n_threads) {
    return field_build(color, X, Y, Z, rgba_out, n_threads);
}

int vx_noise_synth(uint32_t seed, int w, int h, uint8_t *rgba_out) { return noise_synth(seed, w, h, rgba_out); }

int vx_mgpu_bands(int h, int band_rows, int nranks, int rank, int *ids, int cap) {
    if (h <= 0 || band_rows <= 0 || nranks <= 0 || rank < 0 || rank >= nranks)
        return set_error(VX_EINVAL, "vx_mgpu_bands: bad arguments");
    const int nb = (h + band_rows - 1) / band_rows;
    int n = 0;
    for (int b = rank; b < nb; b += nranks) {
        if (ids && n < cap) ids[n] = b;
        n++;
    }
    return n;
}

// The band height of the deal: the multiple of 8 up to max_rows whose
// round-robin deal gives the busiest rank the fewest rows (ties: the tallest
// band, the fewest sends).  4320 rows over 8 ranks: 32-row bands, 544 rows for
// the busiest rank against a mean of 540 (64-row bands: 576).
int vx_mgpu_band_rows(int h, int nranks, int max_rows) {
    if (h <= 0 || nranks <= 0) return set_error(VX_EINVAL, "vx_mgpu_band_rows: bad arguments");
    if (max_rows <= 0) max_rows = 64;
    max_rows = max_rows < VX_TILE_ALIGN_Y ? VX_TILE_ALIGN_Y : max_rows - max_rows % VX_TILE_ALIGN_Y;
    int best = VX_TILE_ALIGN_Y;
    long long best_rows = -1;
    for (int r = VX_TILE_ALIGN_Y; r <= max_rows; r += VX_TILE_ALIGN_Y) {
        const int nb = (h + r - 1) / r;
        long long busiest = 0;
        for (int k = 0; k < nranks && k < nb; k++) {           // rank k owns bands k, k + nranks, ...
            long long rows = 0;
            for (int b = k; b < nb; b += nranks) rows += (b + 1) * (long long)r <= h ? r : h - (long long)b * r;
            busiest = rows > busiest ? rows : busiest;
        }
        if (best_rows < 0 || busiest <= best_rows) {
            best = r;
            best_rows = busiest;
        }
    }
    return best;
}

int vx_mgpu_transfers(int w, int h, int band_rows, int pixel_format, int nranks, int rank, vx_mgpu_xfer *out,
                      int cap) {
    if (w <= 0 || h <= 0 || band_rows <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || cap < 0 ||
        (pixel_format != VX_PIXEL_RGBA8 && pixel_format != VX_PIXEL_RGBA32F))
        return set_error(VX_EINVAL, "vx_mgpu_transfers: bad arguments");
    const uint64_t row_bytes = (uint64_t)w * (pixel_format == VX_PIXEL_RGBA32F ? 16u : 4u);
    const int nb = (h + band_rows - 1) / band_rows;
    int n = 0;
    for (int b = 0; b < nb; b++) {
        const int owner = b % nranks;
        if (owner == 0 || (rank != 0 && owner != rank)) continue;
        if (out && n < cap) {
            vx_mgpu_xfer &x = out[n];
            x.band = b;
            x.src = owner;
            x.dst = 0;
            x.rows = (b + 1) * band_rows <= h ? band_rows : h - b * band_rows;
            x.offset = (uint64_t)b * band_rows * row_bytes;
            x.bytes = (uint64_t)x.rows * row_bytes;
        }
        n++;
    }
    return n;
}

}  // extern "C"
