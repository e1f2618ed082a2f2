// vxrender — C++ host over the C ABI (include/voxmap.h): the stand-alone
// replacement of the reference's browser host for one frame or a timed run.
//
//   loadEncryptedTextures (render.js:190-206)  -> vx_scene_create (.bin/.bin.gz/.blob + key, or a palette grid)
//   updateState camera / sun (map.js:349-402)  -> vx_frame_from_orbit, vx_sun_from_hour
//   drawScene + gl.drawArrays (render.js:267)  -> vx_render into a device framebuffer
//   canvas.toDataURL (map.js:185)              -> the RGBA8 frame written as .ppm / .rgba
//   --ranks N: one frame across N GPUs (devices D..D+N-1): one process per GPU
//   forked before any HIP call, rank 0's RCCL unique id passed through a pipe,
//   vx_mgpu_render gathers the bands into rank 0's frame (include/voxmap.h)
//
// usage: vxrender --map FILE [--format bin|gz|blob|grid] [--key JWK_K] [--noise FILE]
//                 [--dims X,Y,Z] [--size W,H] [--camera K0|K1|K2 | --orbit sx,sy,sz,rx,ry,rz]
//                 [--hour H] [--time T] [--flags N] [--full] [--samples N] [--radius R]
//                 [--frames N] [--device D] [--ranks N] [--out FILE.ppm|FILE.rgba]
// The key may also come from the VOXMAP_KEY environment variable (never a file in the repository).
#include <hip/hip_runtime.h>

#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/voxmap.h"

namespace {

[[noreturn]] void die(const std::string &msg) {
    std::fprintf(stderr, "vxrender: %s\n", msg.c_str());
    std::exit(2);
}

void check(int rc, const char *what) {
    if (rc != VX_OK) die(std::string(what) + ": " + vx_last_error());
}

std::vector<double> parse_list(const char *s, size_t n) {
    std::vector<double> v;
    const char *p = s;
    while (*p) {
        char *end;
        v.push_back(std::strtod(p, &end));
        if (end == p) break;
        p = *end == ',' ? end + 1 : end;
    }
    if (v.size() != n) die(std::string("expected ") + std::to_string(n) + " comma-separated numbers: " + s);
    return v;
}

std::vector<unsigned char> read_all(const std::string &path) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) die("cannot open " + path);
    std::vector<unsigned char> b;
    unsigned char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    std::fclose(f);
    return b;
}

}  // namespace

int main(int argc, char **argv) {
    std::string map, noise, key, out, format = "auto";
    int dims[3] = {1024, 256, 32}, w = 3840, h = 2160, frames = 1, device = 0, samples = 0, ranks = 0;
    double sbj[3] = {381.5, 128.1, 40.0}, rot[3] = {1.1, 0.0, 0.6};   // camera K1 (voxmap_amd/presets.py)
    double hour = 1.0, time = 123.0, radius = 0.03;
    unsigned flags = 0;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) die("missing value after " + a);
            return argv[++i];
        };
        if (a == "--map") map = next();
        else if (a == "--format") format = next();
        else if (a == "--key") key = next();
        else if (a == "--noise") noise = next();
        else if (a == "--dims") { auto v = parse_list(next(), 3); for (int k = 0; k < 3; k++) dims[k] = (int)v[k]; }
        else if (a == "--size") { auto v = parse_list(next(), 2); w = (int)v[0]; h = (int)v[1]; }
        else if (a == "--orbit") { auto v = parse_list(next(), 6); for (int k = 0; k < 3; k++) { sbj[k] = v[k]; rot[k] = v[3 + k]; } }
        else if (a == "--camera") {
            const std::string c = next();
            if (c == "K0") { sbj[0] = 381.5; sbj[1] = 128.1; sbj[2] = 128.0; rot[0] = 1e-4; rot[1] = 0; rot[2] = -0.002; }
            else if (c == "K1") { sbj[0] = 381.5; sbj[1] = 128.1; sbj[2] = 40.0; rot[0] = 1.1; rot[1] = 0; rot[2] = 0.6; }
            else if (c == "K2") { sbj[0] = 0.0; sbj[1] = 128.1; sbj[2] = 12.0; rot[0] = 1.45; rot[1] = 0; rot[2] = -M_PI / 2; }
            else die("unknown camera " + c);
        }
        else if (a == "--hour") hour = std::atof(next());
        else if (a == "--time") time = std::atof(next());
        else if (a == "--flags") flags = (unsigned)std::strtoul(next(), nullptr, 0);
        else if (a == "--full") flags |= VX_FLAG_FULL_QUALITY;
        else if (a == "--samples") samples = std::atoi(next());
        else if (a == "--radius") radius = std::atof(next());
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--ranks") ranks = std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--help" || a == "-h") {
            std::printf("usage: vxrender --map FILE [--format bin|gz|blob|grid] [--key K] [--noise FILE] "
                        "[--dims X,Y,Z] [--size W,H] [--camera K0|K1|K2 | --orbit sx,sy,sz,rx,ry,rz] [--hour H] "
                        "[--time T] [--flags N] [--full] [--samples N] [--radius R] [--frames N] [--device D] "
                        "[--ranks N] [--out FILE.ppm|FILE.rgba]\n(ABI version %d)\n", vx_abi_version());
            return 0;
        } else die("unknown option " + a);
    }
    if (map.empty()) die("--map is required (see --help)");
    if (key.empty() && std::getenv("VOXMAP_KEY")) key = std::getenv("VOXMAP_KEY");
    if (ranks < 0 || ranks > 64) die("--ranks must be in 0..64");

    // --ranks N: fork the rank processes now, before anything touches the GPU
    int rank = 0, nranks = 1, uid_pipe[2] = {-1, -1};
    if (ranks >= 1) {
        nranks = ranks;
        if (pipe(uid_pipe) != 0) die("pipe failed");
        std::vector<pid_t> kids;
        for (int r = 0; r < nranks; r++) {
            const pid_t pid = fork();
            if (pid < 0) die("fork failed");
            if (pid == 0) { rank = r; kids.clear(); break; }
            kids.push_back(pid);
        }
        if (!kids.empty()) {                         // the parent: wait for every rank
            close(uid_pipe[0]); close(uid_pipe[1]);
            int rc = 0;
            for (pid_t k : kids) {
                int stw = 0;
                if (waitpid(k, &stw, 0) < 0 || !WIFEXITED(stw) || WEXITSTATUS(stw) != 0) rc = 2;
            }
            return rc;
        }
        device += rank;
    }

    const std::vector<unsigned char> bytes = read_all(map);
    vx_scene_desc d = {};
    d.map_bytes = bytes.data();
    d.map_size = bytes.size();
    d.map_format = format == "bin" ? VX_FORMAT_BIN : format == "gz" ? VX_FORMAT_BIN_GZ
                 : format == "blob" ? VX_FORMAT_BLOB : format == "grid" ? VX_FORMAT_GRID : VX_FORMAT_AUTO;
    if (d.map_format == VX_FORMAT_AUTO) {   // by extension, as vx_scene_create does for paths
        if (map.size() > 5 && map.compare(map.size() - 5, 5, ".blob") == 0) d.map_format = VX_FORMAT_BLOB;
        else if (map.size() > 3 && map.compare(map.size() - 3, 3, ".gz") == 0) d.map_format = VX_FORMAT_BIN_GZ;
        else if (bytes.size() == (size_t)dims[0] * dims[1] * dims[2]) d.map_format = VX_FORMAT_GRID;
        else d.map_format = VX_FORMAT_BIN;
    }
    d.key_jwk_k = key.empty() ? nullptr : key.c_str();
    if (!noise.empty()) d.noise_path = noise.c_str();
    d.X = dims[0]; d.Y = dims[1]; d.Z = dims[2];
    d.device = device;

    const auto t0 = std::chrono::steady_clock::now();
    vx_scene *scene = nullptr;
    check(vx_scene_create(&d, &scene), "vx_scene_create");
    const double scene_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    vx_frame_params p = {};
    check(vx_frame_from_orbit(sbj, rot, w, h, &p), "vx_frame_from_orbit");
    vx_sun_from_hour(hour, p.sun_dir);
    p.time = (float)std::fmod(time, 1000.0);   // render.js:293
    p.quality = 1;                              // 3D mode (render.js:287)
    p.flags = flags;
    p.shadow_samples = samples;
    p.sun_radius = samples > 1 ? (float)radius : 0.0f;

    const size_t bytes_out = (size_t)w * h * 4;
    void *d_out = nullptr;
    hipStream_t stream = nullptr;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreate(&stream) != hipSuccess ||
        hipMalloc(&d_out, bytes_out) != hipSuccess)
        die("device framebuffer allocation failed");
    vx_mgpu *mg = nullptr;
    if (ranks >= 1) {                                // rank 0 makes the RCCL id, the others read it
        unsigned char uid[VX_MGPU_UID_BYTES];
        if (rank == 0) {
            check(vx_mgpu_unique_id(uid), "vx_mgpu_unique_id");
            for (int r = 1; r < nranks; r++)
                if (write(uid_pipe[1], uid, sizeof uid) != (ssize_t)sizeof uid) die("pipe write failed");
        } else {
            size_t got = 0;
            while (got < sizeof uid) {
                const ssize_t n = read(uid_pipe[0], uid + got, sizeof uid - got);
                if (n <= 0) die("pipe read failed");
                got += (size_t)n;
            }
        }
        close(uid_pipe[0]); close(uid_pipe[1]);
        check(vx_mgpu_create(scene, uid, nranks, rank, &mg), "vx_mgpu_create");
    }
    const int band_rows = vx_mgpu_band_rows(h, nranks > 0 ? nranks : 1, 64);   // the balanced deal
    auto draw = [&](vx_stats *s) {
        if (mg) check(vx_mgpu_render(mg, &p, w, h, band_rows, VX_PIXEL_RGBA8, d_out, stream, s), "vx_mgpu_render");
        else check(vx_render(scene, &p, w, h, VX_PIXEL_RGBA8, d_out, 1, stream, s), "vx_render");
    };
    vx_stats st = {};
    draw(&st);                                        // counters (this rank's pixels)
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, stream);
    for (int f = 0; f < frames; f++) draw(nullptr);
    (void)hipEventRecord(e1, stream);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= (float)frames;
    const double rays = (double)(st.pixels + st.shadow_rays + st.reflect_rays);
    if (rank == 0)
        std::printf("{\"size\": [%d, %d], \"field\": [%d, %d, %d], \"flags\": %u, \"shadow_samples\": %d, "
                    "\"ranks\": %d, \"scene_build_s\": %.3f, \"ms_per_frame\": %.4f, \"fps\": %.1f, "
                    "\"rank0_pixels\": %llu, \"rank0_mrays_per_s\": %.1f, \"rank0_alg_gbps\": %.1f, "
                    "\"rank0_rays_per_frame\": %.0f}\n",
                    w, h, dims[0], dims[1], dims[2], flags, samples, nranks, scene_s, ms, 1000.0 / ms,
                    (unsigned long long)st.pixels, rays / ms / 1e3, (double)st.alg_bytes / ms / 1e6, rays);
    std::fflush(stdout);
    if (mg) vx_mgpu_destroy(mg);

    if (!out.empty() && rank == 0) {
        std::vector<unsigned char> rgba(bytes_out);
        if (hipMemcpy(rgba.data(), d_out, bytes_out, hipMemcpyDeviceToHost) != hipSuccess) die("readback failed");
        FILE *f = std::fopen(out.c_str(), "wb");
        if (!f) die("cannot write " + out);
        if (out.size() > 4 && out.compare(out.size() - 4, 4, ".ppm") == 0) {
            std::fprintf(f, "P6\n%d %d\n255\n", w, h);
            for (size_t i = 0; i < (size_t)w * h; i++) std::fwrite(&rgba[4 * i], 1, 3, f);
        } else {
            std::fwrite(rgba.data(), 1, rgba.size(), f);
        }
        std::fclose(f);
    }
    (void)hipFree(d_out);
    (void)hipStreamDestroy(stream);
    vx_scene_destroy(scene);
    return 0;
}
