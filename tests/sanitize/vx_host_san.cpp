// Host half of the C ABI under AddressSanitizer + UndefinedBehaviorSanitizer
// (SURVEY §5 "HIP host code under ASan/UBSan in CPU tests").  Built by
// tests/test_sanitizers.py from voxmap_amd/csrc/vx_host.cpp, vx_codec.cpp,
// vx_field.cpp and vx_frame.cpp with -fsanitize=address,undefined
// -fno-sanitize-recover=all, so any out-of-bounds access, leak, overflow or
// bad shift aborts the run.  It feeds the untrusted-input paths -- the
// reference's D.fetch chain (utils.js:10-30: AES-CBC, then gzip), scene
// descriptions, frame parameters -- every truncation and a spread of
// corruptions of valid containers, plus the field builder and the 2D mesher on
// random and edge-size grids.  Exit 0 and "SAN_OK" = every check held.
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../voxmap_amd/csrc/vx_internal.h"

static int failures = 0;
#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                                          \
        }                                                                        \
    } while (0)

static const char *kKey = "q83vEjRWeJCrze8SNFZ4kKvN7xI0VniQq83vEjRWeJA";   // base64url of 32 test bytes

static std::vector<unsigned char> gzip_of(const std::vector<unsigned char> &raw) {
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    deflateInit2(&zs, 6, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY);
    std::vector<unsigned char> out(deflateBound(&zs, raw.size()) + 64);
    zs.next_in = const_cast<unsigned char *>(raw.data());
    zs.avail_in = (uInt)raw.size();
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    deflate(&zs, Z_FINISH);
    out.resize(zs.total_out);
    deflateEnd(&zs);
    return out;
}

static std::vector<unsigned char> read_all(const char *path) {
    std::vector<unsigned char> b;
    FILE *f = std::fopen(path, "rb");
    if (!f) return b;
    unsigned char tmp[65536];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + n);
    std::fclose(f);
    return b;
}

static int decode(const std::vector<unsigned char> &in, int fmt, const char *key, std::vector<unsigned char> &out) {
    size_t sz = 0;
    const unsigned char dummy = 0;
    int rc = vx_decode(in.empty() ? &dummy : in.data(), in.size(), fmt, key, nullptr, 0, &sz);
    if (rc) return rc;
    out.assign(sz, 0);
    return vx_decode(in.empty() ? &dummy : in.data(), in.size(), fmt, key, out.data(), out.size(), &sz);
}

static void codec(const char *asset_dir) {
    std::mt19937 rng(7);
    std::vector<unsigned char> raw(40000);
    for (size_t i = 0; i < raw.size(); i++) raw[i] = (unsigned char)((i * 131) ^ (rng() & 7));
    const std::vector<unsigned char> gz = gzip_of(raw);
    std::vector<unsigned char> out;
    CHECK(decode(gz, VX_FORMAT_BIN_GZ, nullptr, out) == VX_OK && out == raw);
    // every truncation of the gzip member fails cleanly (no read past the input)
    for (size_t n = 0; n < gz.size(); n += (n < 64 ? 1 : 97)) {
        std::vector<unsigned char> t(gz.begin(), gz.begin() + n);
        CHECK(decode(t, VX_FORMAT_BIN_GZ, nullptr, out) != VX_OK);
    }
    // corrupt bytes anywhere: the decoder may fail or (in stored data) succeed, never misbehave
    for (int k = 0; k < 400; k++) {
        std::vector<unsigned char> c = gz;
        c[rng() % c.size()] ^= (unsigned char)(1u << (rng() % 8));
        (void)decode(c, VX_FORMAT_BIN_GZ, nullptr, out);
    }
    // random garbage
    for (int k = 0; k < 200; k++) {
        std::vector<unsigned char> g(rng() % 300);
        for (auto &b : g) b = (unsigned char)rng();
        (void)decode(g, VX_FORMAT_BIN_GZ, nullptr, out);
        (void)decode(g, VX_FORMAT_BLOB, kKey, out);
        (void)decode(g, VX_FORMAT_BIN, nullptr, out);
    }
    // a stream that inflates past a known size is rejected (scene inputs pass the size)
    {
        std::vector<unsigned char> big(1 << 20, 0);
        std::vector<unsigned char> v;
        CHECK(vx::decode_container(gzip_of(big).data(), gzip_of(big).size(), VX_FORMAT_BIN_GZ, nullptr, v, 4096) ==
              VX_ESIZE);
    }
    // blob: round trip, wrong key, truncations, flipped bytes, bad key strings
    size_t bsz = 0;
    CHECK(vx_blob_encrypt(gz.data(), gz.size(), kKey, nullptr, 0, &bsz) == VX_OK);
    std::vector<unsigned char> blob(bsz);
    CHECK(vx_blob_encrypt(gz.data(), gz.size(), kKey, blob.data(), blob.size(), &bsz) == VX_OK);
    CHECK(bsz % 16 == 0 && bsz > gz.size());
    CHECK(decode(blob, VX_FORMAT_BLOB, kKey, out) == VX_OK && out == raw);
    CHECK(decode(blob, VX_FORMAT_BLOB, "A0bcdEfghIjklmnopqrstuvwxyzABCDEFGHIJKLMNOP", out) != VX_OK);
    CHECK(decode(blob, VX_FORMAT_BLOB, nullptr, out) == VX_ECRYPTO);
    for (const char *bad : {"", "short", "!!!!", "q83vEjRWeJCrze8SNFZ4kKvN7xI0VniQq83vEjRWeJAAAAA", "q83v=E"})
        CHECK(decode(blob, VX_FORMAT_BLOB, bad, out) == VX_ECRYPTO);
    for (size_t n = 0; n < blob.size(); n += (n < 48 ? 1 : 61)) {
        std::vector<unsigned char> t(blob.begin(), blob.begin() + n);
        CHECK(decode(t, VX_FORMAT_BLOB, kKey, out) != VX_OK);
    }
    for (int k = 0; k < 200; k++) {
        std::vector<unsigned char> c = blob;
        c[rng() % c.size()] ^= (unsigned char)(1u << (rng() % 8));
        (void)decode(c, VX_FORMAT_BLOB, kKey, out);
    }
    CHECK(vx_blob_encrypt(gz.data(), gz.size(), kKey, blob.data(), 3, &bsz) == VX_EINVAL);   // too small
    CHECK(decode(gz, 99, nullptr, out) == VX_EINVAL);
    // the reference's own plaintext assets through the same decoder
    const std::string dir = asset_dir;
    std::vector<unsigned char> n = read_all((dir + "/voxmap_amd/data/noise.bin.gz").c_str());
    CHECK(!n.empty() && decode(n, VX_FORMAT_BIN_GZ, nullptr, out) == VX_OK && out.size() == 4194304);
    std::vector<unsigned char> v = read_all((dir + "/tests/golden/vertex2d.bin.gz").c_str());
    CHECK(!v.empty() && decode(v, VX_FORMAT_BIN_GZ, nullptr, out) == VX_OK && out.size() == 19116 * 16);
}

static void scene_inputs(const char *asset_dir) {
    const int X = 24, Y = 12, Z = 6;
    std::vector<unsigned char> grid((size_t)X * Y * Z, 0);
    for (size_t i = 0; i < grid.size(); i++) grid[i] = (i % 7 == 0) ? (unsigned char)(1 + i % 21) : 0;
    std::vector<unsigned char> field(4 * grid.size());
    CHECK(vx_field_build(grid.data(), X, Y, Z, field.data(), 2) == VX_OK);
    vx_scene_desc d;
    vx::SceneInputs in;
    auto base = [&]() {
        std::memset(&d, 0, sizeof d);
        d.map_bytes = field.data();
        d.map_size = field.size();
        d.map_format = VX_FORMAT_BIN;
        d.X = X; d.Y = Y; d.Z = Z;
        d.noise_w = 16; d.noise_h = 16;
    };
    base();
    CHECK(vx::scene_inputs(&d, in) == VX_OK && in.field == field && in.noise.size() == 16 * 16 * 4);
    CHECK(vx::scene_inputs(nullptr, in) == VX_EINVAL);
    base(); d.X = 0x10000; CHECK(vx::scene_inputs(&d, in) == VX_EINVAL);
    base(); d.Z = 256; CHECK(vx::scene_inputs(&d, in) == VX_EINVAL);
    base(); d.dist_cap = 300; CHECK(vx::scene_inputs(&d, in) == VX_EINVAL);
    base(); d.noise_w = 12; CHECK(vx::scene_inputs(&d, in) == VX_EINVAL);
    base(); d.map_path = "/nonexistent"; CHECK(vx::scene_inputs(&d, in) == VX_EINVAL);    // both set
    base(); d.map_bytes = nullptr; d.map_path = "/nonexistent/map.bin"; CHECK(vx::scene_inputs(&d, in) == VX_EIO);
    base(); d.map_size = field.size() - 1; CHECK(vx::scene_inputs(&d, in) == VX_ESIZE);
    base(); d.map_format = VX_FORMAT_GRID; CHECK(vx::scene_inputs(&d, in) == VX_ESIZE);   // needs X*Y*Z bytes
    base(); d.map_format = VX_FORMAT_GRID; d.map_bytes = grid.data(); d.map_size = grid.size();
    CHECK(vx::scene_inputs(&d, in) == VX_OK && in.from_grid);
    // .bin.gz / .blob containers and AUTO sniffing, with truncations
    const std::vector<unsigned char> gz = gzip_of(field);
    size_t bsz = 0;
    vx_blob_encrypt(gz.data(), gz.size(), kKey, nullptr, 0, &bsz);
    std::vector<unsigned char> blob(bsz);
    vx_blob_encrypt(gz.data(), gz.size(), kKey, blob.data(), blob.size(), &bsz);
    for (int fmt : {VX_FORMAT_BIN_GZ, VX_FORMAT_AUTO}) {
        base(); d.map_bytes = gz.data(); d.map_size = gz.size(); d.map_format = fmt;
        CHECK(vx::scene_inputs(&d, in) == VX_OK && in.field == field);
        for (size_t n = 0; n < gz.size(); n += 7) {
            d.map_size = n;
            CHECK(vx::scene_inputs(&d, in) != VX_OK);
        }
    }
    for (int fmt : {VX_FORMAT_BLOB, VX_FORMAT_AUTO}) {
        base(); d.map_bytes = blob.data(); d.map_size = blob.size(); d.map_format = fmt; d.key_jwk_k = kKey;
        CHECK(vx::scene_inputs(&d, in) == VX_OK && in.field == field);
        d.key_jwk_k = nullptr;
        CHECK(vx::scene_inputs(&d, in) == VX_ECRYPTO);
        d.key_jwk_k = kKey;
        for (size_t n = 1; n < blob.size(); n += 5) {
            d.map_size = n;
            CHECK(vx::scene_inputs(&d, in) != VX_OK);
        }
    }
    // a field whose R/G exceed Z is accepted (the kernels fall back to the checked march)
    std::vector<unsigned char> hot = field;
    hot[0] = 200;
    base(); d.map_bytes = hot.data();
    CHECK(vx::scene_inputs(&d, in) == VX_OK && in.max_rg == 200);
    // the real noise texture through its path (AUTO by extension)
    base();
    const std::string np = std::string(asset_dir) + "/voxmap_amd/data/noise.bin.gz";
    d.noise_path = np.c_str(); d.noise_w = 1024; d.noise_h = 1024;
    CHECK(vx::scene_inputs(&d, in) == VX_OK && in.noise.size() == 4194304);
    d.noise_w = 512; d.noise_h = 512;
    CHECK(vx::scene_inputs(&d, in) == VX_ESIZE);            // size mismatch after a clean inflate
}

static void frames() {
    vx_frame_params p;
    std::memset(&p, 0, sizeof p);
    const double sbj[3] = {381.5, 128.1, 40.0}, rot[3] = {1.1, 0.0, 0.6};
    CHECK(vx_frame_from_orbit(sbj, rot, 3840, 2160, &p) == VX_OK);
    vx_sun_from_hour(1.0, p.sun_dir);
    CHECK(vx::check_frame(&p, 3840, 2160, VX_PIXEL_RGBA8) == VX_OK);
    CHECK(vx::check_frame(nullptr, 1, 1, VX_PIXEL_RGBA8) == VX_EINVAL);
    CHECK(vx::check_frame(&p, 0, 10, VX_PIXEL_RGBA8) == VX_EINVAL);
    CHECK(vx::check_frame(&p, 40000, 10, VX_PIXEL_RGBA8) == VX_EINVAL);
    CHECK(vx::check_frame(&p, 10, 10, 7) == VX_EINVAL);
    const float bad[] = {NAN, INFINITY, -INFINITY, 1.0f, -1e-9f};
    for (int i = 0; i < 3; i++)
        for (float b : bad) {
            vx_frame_params q = p;
            q.cam_fract[i] = b;
            CHECK(vx::check_frame(&q, 8, 8, VX_PIXEL_RGBA32F) == VX_EINVAL);
            q = p;
            q.ray_fwd[i] = b;
            if (!std::isfinite(b)) CHECK(vx::check_frame(&q, 8, 8, VX_PIXEL_RGBA32F) == VX_EINVAL);
            q = p;
            q.sun_dir[i] = b;
            if (!std::isfinite(b)) CHECK(vx::check_frame(&q, 8, 8, VX_PIXEL_RGBA32F) == VX_EINVAL);
        }
    vx_frame_params q = p;
    q.cam_cell[1] = 1 << 22;
    CHECK(vx::check_frame(&q, 8, 8, VX_PIXEL_RGBA8) == VX_EINVAL);
    q = p;
    q.shadow_samples = 17;
    CHECK(vx::check_frame(&q, 8, 8, VX_PIXEL_RGBA8) == VX_EINVAL);
    q.shadow_samples = 4;
    q.sun_radius = NAN;
    CHECK(vx::check_frame(&q, 8, 8, VX_PIXEL_RGBA8) == VX_EINVAL);
    // projection matrices: a singular one is rejected, a regular one works
    float m[16] = {0};
    const double cp[3] = {1, 2, 3};
    CHECK(vx_frame_from_matrix(m, cp, &q) == VX_EINVAL);
    for (int i = 0; i < 4; i++) m[5 * i] = 1.0f;       // identity: invertible
    CHECK(vx_frame_from_matrix(m, cp, &q) == VX_OK);
    float samples[20][3];
    for (int n = -1; n <= 20; n++) CHECK(vx_sun_samples(p.sun_dir, 0.05f, n, samples) == VX_OK);
    CHECK(vx_sun_samples(nullptr, 0.05f, 4, samples) == VX_EINVAL);
    // the frame constants the kernels read, from odd sizes and extreme suns
    vx::FrameConsts fc;
    const float suns[][3] = {{0.7288f, 0.4208f, 0.5403f}, {0.0f, 0.0f, 1.0f}, {1e-30f, -1.0f, 0.0f}, {0, 0, 0}};
    for (const auto &s : suns) {
        vx_frame_params r = p;
        std::memcpy(r.sun_dir, s, sizeof s);
        r.shadow_samples = 16;
        r.sun_radius = 0.03f;
        vx::frame_consts(r, 7, 3, 1024, 256, 32, 64, fc);
    }
}

static void fields() {
    std::mt19937 rng(11);
    const int dims[][3] = {{1, 1, 1}, {1, 7, 3}, {9, 1, 2}, {5, 4, 255}, {33, 17, 12}, {64, 40, 20}};
    for (const auto &dm : dims) {
        const int X = dm[0], Y = dm[1], Z = dm[2];
        const size_t N = (size_t)X * Y * Z;
        std::vector<unsigned char> g(N), f(4 * N);
        for (int fill : {0, 1, 2}) {
            for (size_t i = 0; i < N; i++)
                g[i] = fill == 0 ? 0 : fill == 1 ? (unsigned char)(1 + rng() % 21) : (rng() % 4 ? 0 : 1 + rng() % 21);
            CHECK(vx_field_build(g.data(), X, Y, Z, f.data(), 1 + (int)(rng() % 4)) == VX_OK);
            size_t sz = 0;
            CHECK(vx_vertex2d(f.data(), X, Y, Z, nullptr, 0, &sz) == VX_OK && sz % 16 == 0);
            std::vector<unsigned char> v(sz + 1);
            CHECK(vx_vertex2d(f.data(), X, Y, Z, v.data(), v.size(), &sz) == VX_OK);
            if (sz) CHECK(vx_vertex2d(f.data(), X, Y, Z, v.data(), sz - 1, &sz) != VX_OK);   // too small
            // hostile B values (air 22, out-of-palette bytes) in the mesher
            for (size_t i = 0; i < N; i++)
                if (rng() % 5 == 0) f[4 * i + 2] = (unsigned char)rng();
            CHECK(vx_vertex2d(f.data(), X, Y, Z, nullptr, 0, &sz) == VX_OK);
        }
    }
    std::vector<unsigned char> f(64);
    CHECK(vx_field_build(f.data(), 0, 4, 4, f.data(), 1) == VX_EINVAL);
    CHECK(vx_field_build(f.data(), 4, 4, 256, f.data(), 1) == VX_EINVAL);
    std::vector<unsigned char> noise(64 * 32 * 4);
    CHECK(vx_noise_synth(3, 64, 32, noise.data()) == VX_OK);
    CHECK(vx_noise_synth(3, 60, 32, noise.data()) == VX_EINVAL);
}

static void mgpu() {
    int ids[4];
    CHECK(vx_mgpu_bands(4320, 64, 8, 3, ids, 4) == 9);          // count beyond cap, no write past it
    CHECK(vx_mgpu_bands(4320, 64, 8, 8, ids, 4) == VX_EINVAL);
    vx_mgpu_xfer xs[2];
    CHECK(vx_mgpu_transfers(7680, 4320, 64, VX_PIXEL_RGBA8, 8, 0, xs, 2) == 59);
    CHECK(xs[1].band == 2 && xs[1].src == 2 && xs[1].offset == 2ull * 64 * 7680 * 4);
    CHECK(vx_mgpu_transfers(7680, 4320, 64, VX_PIXEL_RGBA8, 8, 9, xs, 2) == VX_EINVAL);
    CHECK(vx_mgpu_transfers(33, 1000, 24, VX_PIXEL_RGBA32F, 5, 4, xs, 0) == 8);
}

int main(int argc, char **argv) {
    const char *root = argc > 1 ? argv[1] : ".";
    codec(root);
    scene_inputs(root);
    frames();
    fields();
    mgpu();
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("SAN_OK\n");
    return 0;
}
