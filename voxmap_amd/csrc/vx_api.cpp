// vx_api.cpp — the C ABI (include/voxmap.h) over the HIP kernels.
//
// Replaces the WebGL host of the reference (src/web/render.js): texture
// upload (render.js:134-206) becomes vx_scene_create (field + noise resident
// in HBM, A channel filled on the GPU), drawScene (render.js:267-298) becomes
// vx_render / vx_render_tiles.  The camera/sun helpers restate map.js:349-402
// and math.js:16-49 in double precision, as the JS computes them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "vx_internal.h"

using namespace vx;

struct vx_scene {
    int device = 0;
    int X = 0, Y = 0, Z = 0;
    int noise_w = 0, noise_h = 0;
    uint32_t *d_prim = nullptr;   // 8 padded octant copies (vx_internal.h FieldLayout)
    uint8_t *d_sun = nullptr;     // R, G channels
    int8_t *d_sunp = nullptr;     // R, G channels, int8, -1 border (Z <= 126)
    int8_t *d_sunx = nullptr;     // 8 orthant-exit copies of the march channel (launch_sun_exit)
    // cone copies of the march channel, built on first use for a frame's sun
    // samples {octant, kx, ky} (exit_plan) and kept: the sun moves slowly
    // (map.js:399-402), so one serves many frames
    struct Cone {
        int oct = -1, kx = -1, ky = -1;
        bool doom = false;            // the doom table is in (launch_sun_doom, window `plan`)
        int plan[7] = {0, 0, 0, 0, 0, 0, 0};
        int8_t *d = nullptr;
        hipEvent_t ready = nullptr;   // recorded on the build's stream after the build
        unsigned long long used = 0;
        bool ready_seen = false;      // the build's `ready` event observed complete
    } cones[2];
    unsigned long long cone_tick = 0;
    std::mutex cone_mu;
    // band / tile-id lists (vx_render_tiles / _bands, vx_detile), uploaded once
    // per distinct list and never rewritten while cached (list_acquire)
    struct ListBuf {
        std::vector<int> ids;         // the list d holds (also the upload's source)
        unsigned long long hash = 0;
        int *d = nullptr;
        hipEvent_t ready = nullptr;   // recorded after the upload
        bool ready_seen = false;
        int pins = 0;                 // renders between lookup and enqueue
        unsigned long long used = 0;
    };
    std::vector<std::unique_ptr<ListBuf>> lists;
    std::mutex lists_mu;
    unsigned long long list_tick = 0;
    int SB = 0, SXp = 0, SYp = 0, SZp = 0;
    uint16_t *d_rg = nullptr;     // R | G << 8
    uint32_t *d_rg2 = nullptr;    // AO x-pairs: (R, G) of cells x and x + 1, clamped, (X + 1) per row
    uint8_t *d_bcol = nullptr;    // map.bin's B channel as uploaded (vx_scene_read_field)
    uint16_t *d_qface = nullptr;  // greedy mesh per face: 6 planes of X*Y*Z offsets from the quad origin
    uint32_t *d_qcopy = nullptr;  // per octant, prim layout: entry faces' offsets (CHUNK <= 32), or null
    int chunk = 0;                // its CHUNK (sdf.cpp:284, voxmap.h:9)
    uint32_t *d_fp2d = nullptr;   // 2D mode: per column vis colour + quad corner (KernelArgs::fp2d)
    std::vector<Quad2d> quads2d;  // 2D mode: the footprint's greedy quads (vx_scene_vertex2d)
    uint32_t *d_noise = nullptr;
    uint32_t *d_noise4 = nullptr; // noise quads, 4 planes (A, R, G, B): a channel of texels (x, y), (x+1, y), (x, y+1), (x+1, y+1), wrapped
    unsigned long long *d_stats = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    FieldLayout L;
    unsigned long long *d_blk = nullptr;   // VX_BLOCK_TIMING builds: the last launch's block times
    size_t blk_cap = 0, blk_n = 0;
};

#define VX_HIP(call)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return set_error(VX_EDEVICE, std::string(#call " failed: ") + hipGetErrorString(e_));     \
    } while (0)

int vx::scene_device(const vx_scene *s) { return s->device; }
void *vx::scene_stream(const vx_scene *s) { return (void *)s->stream; }

// 2D mode data (DESIGN.md §3 "2D mode"): the footprint of the field (each
// column's top block with z >= 1, sdf.cpp:201-204) meshed by the greedy 2D
// mesher of sdf.cpp:362-401 on the host, uploaded as {colour, quad corner}
// per column.  Returns a hipError_t as int.
static int build_2d(vx_scene *s, const uint32_t *d_lin) {
    const size_t n = (size_t)s->X * s->Y;
    uint8_t *d_c2d = nullptr;
    hipError_t e = hipMalloc(&d_c2d, n);
    std::vector<uint8_t> c2d(n);
    if (e == hipSuccess) e = (hipError_t)launch_footprint(d_lin, d_c2d, s->X, s->Y, s->Z, s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(c2d.data(), d_c2d, n, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (d_c2d) (void)hipFree(d_c2d);
    if (e != hipSuccess) return (int)e;
    std::vector<uint32_t> origin(n, 0), fp(2 * n);
    mesh2d(c2d.data(), s->X, s->Y, s->quads2d, origin.data());
    for (size_t i = 0; i < n; i++) {
        fp[2 * i] = c2d[i];
        fp[2 * i + 1] = origin[i];
    }
    e = hipMalloc(&s->d_fp2d, fp.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(s->d_fp2d, fp.data(), fp.size() * 4, hipMemcpyHostToDevice);
    return (int)e;
}

extern "C" {


int vx_scene_vertex2d(const vx_scene *s, void *out, size_t cap, size_t *out_size) {
    if (!s || !out_size) return set_error(VX_EINVAL, "vx_scene_vertex2d: null argument");
    *out_size = vertex2d_bytes(s->quads2d, nullptr, 0);
    if (!out) return VX_OK;
    if (cap < *out_size) return set_error(VX_EINVAL, "vx_scene_vertex2d: output buffer too small");
    vertex2d_bytes(s->quads2d, static_cast<uint8_t *>(out), cap);
    return VX_OK;
}

int vx_scene_create(const vx_scene_desc *d, vx_scene **out) {
    if (!d || !out) return set_error(VX_EINVAL, "vx_scene_create: null argument");
    *out = nullptr;
    SceneInputs in;
    int rc = scene_inputs(d, in);           // validation + container decode (vx_host.cpp)
    if (rc) return rc;
    const int X = in.X, Y = in.Y, Z = in.Z, NW = in.NW, NH = in.NH, cap = in.cap;
    const FieldLayout L = field_layout(X, Y, Z, cap);
    const bool from_grid = in.from_grid;
    const int max_rg = in.max_rg;
    std::vector<unsigned char> &field = in.field, &noise = in.noise;
    const size_t field_bytes = (size_t)X * Y * Z * 4, noise_bytes = (size_t)NW * NH * 4;
    VX_HIP(hipSetDevice(d->device));
    vx_scene *s = new vx_scene();
    s->device = d->device;
    s->X = X; s->Y = Y; s->Z = Z;
    s->noise_w = NW; s->noise_h = NH;
    auto fail = [&](int code) { vx_scene_destroy(s); return code; };
    hipError_t e;
    uint8_t *ga = nullptr, *gb = nullptr;
    uint32_t *lin = nullptr;   // the linear RGBA upload, B -> vis colour, A rewritten per octant
    if ((e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreate(&s->ev0)) != hipSuccess || (e = hipEventCreate(&s->ev1)) != hipSuccess ||
        (e = hipMalloc(&lin, field_bytes)) != hipSuccess ||
        (e = hipMalloc(&s->d_noise, noise_bytes)) != hipSuccess ||
        (e = hipMalloc(&s->d_noise4, 4 * noise_bytes)) != hipSuccess ||
        (e = hipMalloc(&s->d_stats, sizeof(unsigned long long) * ST_COUNT * 64)) != hipSuccess ||
        (e = hipMalloc(&s->d_bcol, field_bytes / 4)) != hipSuccess ||
        (e = hipMalloc(&ga, field_bytes / 4)) != hipSuccess || (e = hipMalloc(&gb, field_bytes / 4)) != hipSuccess ||
        (!from_grid &&
         (e = hipMemcpyAsync(lin, field.data(), field_bytes, hipMemcpyHostToDevice, s->stream)) != hipSuccess) ||
        (e = hipMemcpyAsync(s->d_noise, noise.data(), noise_bytes, hipMemcpyHostToDevice, s->stream)) != hipSuccess) {
        if (ga) (void)hipFree(ga);
        if (gb) (void)hipFree(gb);
        if (lin) (void)hipFree(lin);
        return fail(set_error(VX_EDEVICE, std::string("scene upload failed: ") + hipGetErrorString(e)));
    }
    if (from_grid) {   // sdf.cpp:405-470 on the device, into the linear RGBA upload buffer
        uint8_t *d_col = nullptr;
        e = hipMalloc(&d_col, (size_t)X * Y * Z);
        if (e == hipSuccess) e = hipMemcpyAsync(d_col, d->map_bytes, (size_t)X * Y * Z, hipMemcpyHostToDevice, s->stream);
        if (e == hipSuccess) e = (hipError_t)field_build_device(d_col, lin, X, Y, Z, s->stream);
        if (d_col) (void)hipFree(d_col);
        if (e != hipSuccess) {
            (void)hipFree(ga);
            (void)hipFree(gb);
            (void)hipFree(lin);
            return fail(set_error(VX_EDEVICE, std::string("device field build failed: ") + hipGetErrorString(e)));
        }
    }
    // the kernels' arrays: sun channels and AO array from
    // the upload, then per octant its cube sizes into the upload's A channel
    // and from there into that octant's prim copy (border = sentinel)
    const size_t N = (size_t)X * Y * Z;
    int lrc = 0;
    int *psum = nullptr;   // prefix sums of solid cells for the octant boxes
    if ((e = hipMalloc(&s->d_prim, 8 * L.texels * 4)) == hipSuccess &&
        (e = hipMalloc(&s->d_sun, 2 * N)) == hipSuccess && (e = hipMalloc(&s->d_rg, 2 * N)) == hipSuccess &&
        (e = hipMalloc(&s->d_rg2, 4 * (N + (size_t)Y * Z))) == hipSuccess &&
        (e = hipMalloc(&psum, sizeof(int) * (size_t)(X + 1) * (Y + 1) * (Z + 1))) == hipSuccess &&
        (e = hipMemsetD32Async((hipDeviceptr_t)s->d_prim, 0xFFFFFFFF, 8 * L.texels, s->stream)) == hipSuccess) {
        // B -> vis colour first: the boxes and prim copies classify by it
        lrc = launch_field_vis(lin, s->d_bcol, X, Y, Z, s->stream);
        if (!lrc) lrc = build_2d(s, lin);
        if (!lrc) lrc = launch_field_pack(lin, s->d_sun, s->d_rg, X, Y, Z, s->stream);
        if (!lrc) lrc = launch_ao_pairs(s->d_rg, s->d_rg2, X, Y, Z, s->stream);
        if (!lrc) lrc = launch_noise_quads(s->d_noise, s->d_noise4, NW, NH, s->stream);
        if (!lrc) lrc = launch_field_psum(lin, psum, X, Y, Z, s->stream);
        // march copy of the sun channels: int8 inside a border of -1 ("left the grid"), so the
        // march's loaded value carries the exit test (vx_kernels.hip march_fast); values <= Z <= 126
        const size_t sxy = (size_t)(X + 2 * (Z + 2)) * (Y + 2 * (Z + 2));
        // the march's byte offset is 0x4B000000 + x + Xp*y + XpYp*z from fp32 bit patterns
        // (vx_kernels.hip march_pad): the padded plane below 2^23, the sum below 2^32
        if (!lrc && Z <= 126 && max_rg <= Z && sxy < (1u << 23) && sxy * (Z + 2 * (Z + 2) + 3) + 0x4B000000ull < (1ull << 32)) {
            s->SB = Z + 2;
            s->SXp = X + 2 * s->SB; s->SYp = Y + 2 * s->SB; s->SZp = Z + 2 * s->SB;
            const size_t np = (size_t)s->SXp * s->SYp * s->SZp;
            if ((e = hipMalloc(&s->d_sunp, 2 * np)) == hipSuccess &&
                (e = hipMemsetAsync(s->d_sunp, 0xFF, 2 * np, s->stream)) == hipSuccess)
                lrc = launch_sun_pad(lin, s->d_sunp, X, Y, Z, s->SB, s->stream);
#ifndef VX_SUNX
#define VX_SUNX 1
#endif
            // per ray octant, the channel with every cell whose orthant ahead holds no block
            // marked -1: the march exits "lit" there (DESIGN.md §3 "Orthant exit")
            if (e != hipSuccess) lrc = (int)e;
            // the exit tables are an optimisation (the kernel marches the plain
            // channel when a.sunx is null): a copy that does not fit leaves them off
            if (VX_SUNX && !lrc) {
                if (hipMalloc(&s->d_sunx, 8 * np) != hipSuccess) {
                    (void)hipGetLastError();
                    s->d_sunx = nullptr;
                } else if ((e = hipMemsetAsync(s->d_sunx, 0xFF, 8 * np, s->stream)) == hipSuccess) {
                    lrc = launch_sun_exit(s->d_sunp, s->d_sunx, ga, X, Y, Z, s->SB, s->stream);
                } else {
                    lrc = (int)e;
                }
            }
        }
        for (int oct = 0; oct < 8 && !lrc; oct++) {
            lrc = launch_field_octant(lin, X, Y, Z, cap, oct, ga, gb, s->stream);
            if (!lrc) lrc = launch_field_box(lin, psum, s->d_prim + oct * L.texels, X, Y, Z, L.pad, cap, oct, s->stream);
        }
        // the greedy mesh's quad per face (render.vert:25-28: v_cellPos is the quad origin),
        // allocated after the arrays the kernels read every step: placed in front of them
        // it moved their device addresses, and the v1 frame measured 3.3 % slower with the
        // same kernel code (profiles/r04_ab_v1_bisect.txt, r04_ab_alloc_order.txt)
        // Optional: a field whose table does not fit still loads; its
        // frames then need the unit-cell split and the single glass layer
        // (vx_render refuses others), which are the only ones that read no mesh.
        // VOXMAP_TEST_NO_FACE_TABLE=1 makes the allocation fail (tests).
        if (!lrc) {
            const char *no_tab = std::getenv("VOXMAP_TEST_NO_FACE_TABLE");
            if ((no_tab && no_tab[0] == '1') || hipMalloc(&s->d_qface, 3 * field_bytes) != hipSuccess) {
                (void)hipGetLastError();
                s->d_qface = nullptr;
            } else {
                lrc = launch_face_quads(lin, s->d_qface, X, Y, Z, in.chunk, s->stream);
            }
        }
        // the fp32-index walk's companion copy: quad offsets loaded beside
        // every prim word; fields whose walk takes the integer index (or CHUNK > 32) read
        // the face table once after the walk instead.  Optional: not allocated if it does not fit.
        const bool f32_ok = 4.0 * (double)L.Xp * (double)L.Yp < 8388608.0 && 32.0 * (double)L.texels < 4294967296.0 &&
                            L.Zp < (1 << 20);
#ifndef VX_QSPEC
#define VX_QSPEC 1
#endif
        if (VX_QSPEC && !lrc && s->d_qface && in.chunk <= 32 && f32_ok) {
            if (hipMalloc(&s->d_qcopy, 8 * L.texels * 4) != hipSuccess) {
                (void)hipGetLastError();
                s->d_qcopy = nullptr;
            } else {
                lrc = launch_qcopy(s->d_qface, s->d_qcopy, X, Y, Z, L.pad, L.texels, s->stream);
            }
        }
        e = hipStreamSynchronize(s->stream);
    }
    if (psum) (void)hipFree(psum);
    (void)hipFree(ga);
    (void)hipFree(gb);
    (void)hipFree(lin);
    if (lrc != 0 || e != hipSuccess)
        return fail(set_error(VX_EDEVICE, std::string("field preparation failed: ") +
                                              hipGetErrorString(lrc ? (hipError_t)lrc : e)));
    s->L = L;
    s->chunk = in.chunk;
    *out = s;
    return VX_OK;
}

void vx_scene_destroy(vx_scene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->d_prim) (void)hipFree(s->d_prim);
    if (s->d_sun) (void)hipFree(s->d_sun);
    if (s->d_sunp) (void)hipFree(s->d_sunp);
    if (s->d_sunx) (void)hipFree(s->d_sunx);
    for (auto &c : s->cones) {
        if (c.d) (void)hipFree(c.d);
        if (c.ready) (void)hipEventDestroy(c.ready);
    }
    if (s->d_rg) (void)hipFree(s->d_rg);
    if (s->d_rg2) (void)hipFree(s->d_rg2);
    if (s->d_noise4) (void)hipFree(s->d_noise4);
    if (s->d_bcol) (void)hipFree(s->d_bcol);
    if (s->d_qface) (void)hipFree(s->d_qface);
    if (s->d_qcopy) (void)hipFree(s->d_qcopy);
    if (s->d_blk) (void)hipFree(s->d_blk);
    if (s->d_fp2d) (void)hipFree(s->d_fp2d);
    if (s->d_noise) (void)hipFree(s->d_noise);
    if (s->d_stats) (void)hipFree(s->d_stats);
    for (auto &b : s->lists) {
        if (b->d) (void)hipFree(b->d);
        if (b->ready) (void)hipEventDestroy(b->ready);
    }
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

int vx_scene_dims(const vx_scene *s, int dims[3]) {
    if (!s || !dims) return set_error(VX_EINVAL, "vx_scene_dims: null argument");
    dims[0] = s->X; dims[1] = s->Y; dims[2] = s->Z;
    return VX_OK;
}

int vx_scene_read_field(vx_scene *s, void *host_out, size_t cap) { return vx_scene_read_field_copy(s, 0, host_out, cap); }

static int read_copy(vx_scene *s, int octant, void *host_out, size_t cap, bool boxes, const char *what) {
    if (!s || !host_out) return set_error(VX_EINVAL, std::string(what) + ": null argument");
    if (octant < 0 || octant > 7) return set_error(VX_EINVAL, std::string(what) + ": octant must be 0..7");
    const size_t n = (size_t)s->X * s->Y * s->Z * 4;
    if (cap < n) return set_error(VX_EINVAL, std::string(what) + ": buffer too small");
    VX_HIP(hipSetDevice(s->device));
    uint32_t *lin = nullptr;
    VX_HIP(hipMalloc(&lin, n));
    hipError_t e = (hipError_t)launch_field_unpack(boxes ? nullptr : s->d_rg, s->d_bcol,
                                                   s->d_prim + (size_t)octant * s->L.texels, lin, s->X, s->Y, s->Z,
                                                   s->L.pad, s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(host_out, lin, n, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(lin);
    if (e != hipSuccess) return set_error(VX_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
    return VX_OK;
}

#ifdef VX_BLOCK_TIMING
// diagnostics build only: the last untiled launch's per-block (start, end) on the 100 MHz clock
int vx_debug_block_times(vx_scene *s, unsigned long long *out, size_t cap, size_t *n) {
    if (!s || !n) return set_error(VX_EINVAL, "vx_debug_block_times: null argument");
    *n = s->blk_n;
    if (!out || !s->d_blk) return VX_OK;
    VX_HIP(hipDeviceSynchronize());
    VX_HIP(hipMemcpy(out, s->d_blk, 16 * std::min(cap / 2, s->blk_n), hipMemcpyDeviceToHost));
    return VX_OK;
}
#endif

int vx_scene_read_face_quads(vx_scene *s, void *host_out, size_t cap) {
    if (!s || !host_out) return set_error(VX_EINVAL, "vx_scene_read_face_quads: null argument");
    if (!s->d_qface) return set_error(VX_ENOMEM, "vx_scene_read_face_quads: the scene has no face table (it did not fit)");
    const size_t N = (size_t)s->X * s->Y * s->Z;
    if (cap < 12 * N) return set_error(VX_EINVAL, "vx_scene_read_face_quads: buffer too small");
    VX_HIP(hipSetDevice(s->device));
    uint16_t *tmp = nullptr;
    VX_HIP(hipMalloc(&tmp, 12 * N));
    hipError_t e = (hipError_t)launch_face_quads_interleave(s->d_qface, tmp, N, s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(host_out, tmp, 12 * N, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(tmp);
    if (e != hipSuccess) return set_error(VX_EDEVICE, std::string("vx_scene_read_face_quads: ") + hipGetErrorString(e));
    return VX_OK;
}

int vx_scene_read_field_copy(vx_scene *s, int octant, void *host_out, size_t cap) {
    return read_copy(s, octant, host_out, cap, false, "vx_scene_read_field");
}

int vx_scene_read_boxes(vx_scene *s, int octant, void *host_out, size_t cap) {
    return read_copy(s, octant, host_out, cap, true, "vx_scene_read_boxes");
}

static int check_render(const vx_scene *s, const vx_frame_params *p, int w, int h, int fmt) {
    if (!s) return set_error(VX_EINVAL, "null scene/params");
    const int rc = check_frame(p, w, h, fmt);
    if (rc) return rc;
    // a scene without the greedy mesh per face (it did not fit) renders only
    // what reads no mesh: the unit-cell split and the single glass layer
    const unsigned need = VX_FLAG_UNIT_GBUF | VX_FLAG_GLASS_SINGLE;
    if (!s->d_qface && p->quality != 0 && ((p->flags & need) != need || (p->flags & VX_FLAG_GLASS_ORDER)))
        return set_error(VX_EINVAL, "this scene has no face table (it did not fit in device memory): its 3D frames "
                                    "need VX_FLAG_UNIT_GBUF | VX_FLAG_GLASS_SINGLE and not VX_FLAG_GLASS_ORDER");
    return VX_OK;
}

static void fill_stats(vx_stats *st, const unsigned long long *v, float ms, int out_bytes) {
    st->pixels = v[ST_PIXELS];
    st->sky_px = v[ST_SKY];
    st->block_px = v[ST_BLOCK];
    st->glass_px = v[ST_GLASS];
    st->primary_fetches = v[ST_PRIM_FETCH];
    st->shadow_rays = v[ST_SHADOW_RAYS];
    st->shadow_fetches = v[ST_SHADOW_FETCH];
    st->ao_samples = v[ST_AO];
    st->noise_px = v[ST_NOISE_PX];
    st->primary_cap_hits = v[ST_CAP_HITS];
    st->reflect_rays = v[ST_REFL_RAYS];
    st->reflect_fetches = v[ST_REFL_FETCH];
    st->rough_px = v[ST_ROUGH];
    st->primary_wave_iters = v[ST_PRIM_WITERS];
    st->march_wave_iters = v[ST_MARCH_WITERS];
    st->march_lane_slots = v[ST_MARCH_SLOTS];
    st->shadow_rays_resolved = v[ST_SHADOW_RESOLVED];
    // 4 B per field texel read (primary, shadow and reflection
    // rays), 32 B per trilinear AO, 80 B per clouded sky pixel (5 bilinear
    // noise taps), 16 B per rough-normal white() tap (4 texels), plus the
    // framebuffer store.
    st->alg_bytes = 4ull * (st->primary_fetches + st->shadow_fetches + st->reflect_fetches) +
                    32ull * st->ao_samples + 80ull * st->noise_px + 16ull * st->rough_px +
                    (unsigned long long)out_bytes * st->pixels;
    st->kernel_ms = ms;
}

// A tiled launch: tiles of tw x th pixels (multiples of the 32 x 8 kernel
// block), tiles_x per tile row; compact output (tile k at k * th * pitch
// pixels, rows pitch pixels apart) or in place in the w-wide frame.
struct TileSpec {
    int tw = 0, th = 0, pitch = 0, tiles_x = 0, inplace = 0;
    const int *ids = nullptr;   // device list
    int n = 0;
};

// The frame's cone copy {oct, kx, ky}: found in the scene's cache, or built on
// stream st into a free or the least recently used slot.  The caller holds
// s->cone_mu from here until its render is enqueued, so every render that
// reads a slot is enqueued before anyone can recycle it.  A recycle waits for
// the device: it needs a third sun window in the scene's two slots, so it
// happens at most once per sun window change (the sun moves about 1 rad per
// hour, map.js:399), and it keeps no handle of a caller's stream (ADVICE r05:
// a caller may destroy a stream it rendered on; an event per render on the
// reader's stream instead costs +3 % at C3, profiles/r04_ab_event_c3.txt).  A
// cache hit waits for the build's event until the host has seen it complete
// (a no-op on the build's own stream).  t_build: recorded on st just before
// the build's first packet (vx_prepare_sun's timing), if built.
// doom: the copy carries the doom table of window plan (DESIGN.md §3 "Doom
// table"; part of the cache key).
static int cone_copy(vx_scene *s, int oct, int kx, int ky, bool doom, const int plan[7], hipStream_t st,
                     const int8_t **out, bool *built, vx_scene::Cone **used, hipEvent_t t_build) {
    *built = false;
    vx_scene::Cone *slot = nullptr;
    for (auto &c : s->cones)
        if (c.d && c.oct == oct && c.kx == kx && c.ky == ky && c.doom == doom &&
            (!doom || std::memcmp(c.plan, plan, sizeof c.plan) == 0))
            slot = &c;
    if (!slot) {
        slot = &s->cones[0];
        for (auto &c : s->cones)
            if (!c.d || c.used < slot->used) slot = &c;
        if (slot->d) {
            VX_HIP(hipDeviceSynchronize());            // every render that read it is enqueued: done
        } else {
            const size_t np = (size_t)s->SXp * s->SYp * s->SZp;
            VX_HIP(hipMalloc(&slot->d, np));
            if (!slot->ready) VX_HIP(hipEventCreateWithFlags(&slot->ready, hipEventDisableTiming));
        }
        slot->oct = -1;
        if (t_build) VX_HIP(hipEventRecord(t_build, st));
        VX_HIP(hipMemsetAsync(slot->d, 0xFF, (size_t)s->SXp * s->SYp * s->SZp, st));
        int rc = launch_sun_cone(s->d_sunp, slot->d, s->X, s->Y, s->Z, s->SB, oct, kx, ky, st);
        if (rc) return set_error(VX_EDEVICE, std::string("sun cone copy: ") + hipGetErrorString((hipError_t)rc));
        if (doom) {
            rc = launch_sun_doom(s->d_sunp, slot->d, s->X, s->Y, s->Z, s->SB, plan, st);
            if (rc) return set_error(VX_EDEVICE, std::string("sun doom table: ") + hipGetErrorString((hipError_t)rc));
        }
        VX_HIP(hipEventRecord(slot->ready, st));
        slot->ready_seen = false;
        slot->oct = oct; slot->kx = kx; slot->ky = ky;
        slot->doom = doom;
        std::memcpy(slot->plan, plan, sizeof slot->plan);
        *built = true;
    } else if (!slot->ready_seen) {
        const hipError_t q = hipEventQuery(slot->ready);   // wait for the build
        if (q == hipSuccess) slot->ready_seen = true;
        else if (q == hipErrorNotReady) VX_HIP(hipStreamWaitEvent(st, slot->ready, 0));
        else VX_HIP(q);
    }
    slot->used = ++s->cone_tick;
    *out = slot->d;
    *used = slot;
    return VX_OK;
}

// The sun exit copy frame constants fc select (vx_exit_info kind 0/1/2):
// a.sunc (cone) built or found, and the info filled.  A frame's cone copy
// carries the doom table unless the frame asks VX_FLAG_NO_DOOM or
// VX_FLAG_SOFT_BRICK (the LDS brick march reads no doom codes).
static int frame_exit(vx_scene *s, const vx_frame_params *p, const FrameConsts &fc, hipStream_t st,
                      const int8_t **sunc, vx_exit_info *info, bool *built, vx_scene::Cone **used,
                      hipEvent_t t_build = nullptr) {
    *sunc = nullptr;
    *used = nullptr;
    bool b = false;
    vx_exit_info e{0, -1, -1, -1, 0.0f};
    const bool tables = s->d_sunx && !(p->flags & VX_FLAG_NO_EXIT);
    if (tables && p->quality != 0 && !(p->flags & (VX_FLAG_NO_SHADOW | VX_FLAG_PRIMARY_ONLY))) {
        int oct, kx, ky;
        if (!(p->flags & VX_FLAG_NO_CONE) && exit_plan(fc, s->SB, &oct, &kx, &ky)) {
            int plan[7] = {0, 0, 0, 0, 0, 0, 0};
            doom_plan(fc, plan);
            const bool doom = plan[6] >= 1 && !(p->flags & (VX_FLAG_NO_DOOM | VX_FLAG_SOFT_BRICK));
            const int rc = cone_copy(s, oct, kx, ky, doom, plan, st, sunc, &b, used, t_build);
            if (rc) return rc;
            e = vx_exit_info{2, oct, kx, ky, 0.0f};
        } else if (fc.sun_k[0].fast) {
            const float *r = fc.sun_k[0].r;
            e = vx_exit_info{1, (r[0] > 0.0f ? 1 : 0) | (r[1] > 0.0f ? 2 : 0) | (r[2] > 0.0f ? 4 : 0), -1, -1, 0.0f};
        }
    }
    if (built) *built = b;
    if (info) *info = e;
    return VX_OK;
}

// ListRef (list_acquire): the list the launch reads, unpinned once it is enqueued
struct ListRef;
static void list_release(ListRef *lr);
static int do_render(vx_scene *s, const vx_frame_params *p, int w, int h, const TileSpec &ts, int fmt, void *out_dev,
                     void *stream, vx_stats *stats, ListRef *lr = nullptr) {
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    KernelArgs a;
    std::memset(&a, 0, sizeof a);
    a.prim = s->d_prim;
    a.sun = s->d_sun;
    a.sunp = s->d_sunp;
    a.sunx = (p->flags & VX_FLAG_NO_EXIT) ? nullptr : s->d_sunx;
    a.SB = s->SB;
    a.SBf = (float)s->SB;
    a.SXp = s->SXp;
    a.SXpYp = (unsigned)s->SXp * (unsigned)s->SYp;
    a.sunp_texels = (unsigned)s->SXp * (unsigned)s->SYp * (unsigned)s->SZp;
    a.rg = s->d_rg;
    a.rg2 = s->d_rg2;
    a.noise = s->d_noise;
    a.noise4 = s->d_noise4;
    a.fp2d = s->d_fp2d;
    a.qface = s->d_qface;
    a.qcopy = s->d_qcopy;
    a.quad_gbuf = (p->flags & VX_FLAG_UNIT_GBUF) ? 0 : 1;
    a.chunk = s->chunk;
    a.X = s->X; a.Y = s->Y; a.Z = s->Z;
    a.noise_w = s->noise_w; a.noise_h = s->noise_h;
    a.noise_rw = 1.0f / (float)s->noise_w;   // powers of two: exact
    a.noise_rh = 1.0f / (float)s->noise_h;
    a.noise_lw = 0;
    while ((1 << a.noise_lw) < s->noise_w) a.noise_lw++;
    a.w = w; a.h = h;
    a.tile_w = ts.tw;
    a.tile_h = ts.th;
    a.tile_pitch = ts.pitch;
    a.tiles_x = ts.tiles_x;
    a.tile_inplace = ts.inplace;
    a.tile_ids = ts.ids;
    a.n_tiles = ts.n;
    a.out = out_dev;
    a.p = *p;
    a.max_shadow_steps = p->max_shadow_steps > 0 ? p->max_shadow_steps : 2 * s->Z;   // render.frag:12
    frame_consts(*p, w, h, s->X, s->Y, s->Z, a.max_shadow_steps, a.fc);
    // the cone copy the frame reads stays pinned from its lookup until this
    // render is enqueued (a second thread must not recycle it in
    // between)
    std::unique_lock<std::mutex> cone_lock(s->cone_mu);
    vx_scene::Cone *cone = nullptr;
    {
        const int rc = frame_exit(s, p, a.fc, st, &a.sunc, nullptr, nullptr, &cone);
        if (rc) return rc;
    }
    if (!cone) cone_lock.unlock();
    a.Xp = s->L.Xp;
    a.pad = s->L.pad;
    a.XpYp = (unsigned)s->L.Xp * (unsigned)s->L.Yp;
    a.XY = (unsigned)s->X * (unsigned)s->Y;
    a.XYZ = a.XY * (unsigned)s->Z;
    a.copy_texels = (unsigned)s->L.texels;
    a.kcam = (unsigned)(p->cam_cell[0] + s->L.pad) + (unsigned)a.Xp * (unsigned)(p->cam_cell[1] + s->L.pad) +
             a.XpYp * (unsigned)(p->cam_cell[2] + s->L.pad);   // mod 2^32
    {
        // fp32 x/y index: 4*(x + Xp*y) of a fetched cell lies in [0, 4*Xp*Yp),
        // its partial sums 4x in [0, 4Xp) and y in [0, Yp), all exact fp32
        // integers below 2^24; the 24-bit multiply needs 4*Xp*Yp < 2^23, the
        // 32-bit byte offsets all 8 copies below 4 GiB
        const double xy4 = 4.0 * (double)s->L.Xp * (double)s->L.Yp;
        const bool ok = xy4 < 8388608.0 && 32.0 * (double)s->L.texels < 4294967296.0 &&
                        std::abs(p->cam_cell[0]) < (1 << 21) && std::abs(p->cam_cell[1]) < (1 << 21) &&
                        std::abs(p->cam_cell[2]) < (1 << 20) && s->L.Zp < (1 << 20);   // |z| < 2^21 (k_render)
        // (the fp32-index walk loads its quad offsets from the qcopy beside each prim word)
        a.prim_f32 = ok && (s->d_qcopy || !VX_QSPEC) && !(p->flags & VX_FLAG_INT_INDEX) ? 1 : 0;
        a.kx4 = (float)(4 * (p->cam_cell[0] + s->L.pad));
        a.ky = (float)(p->cam_cell[1] + s->L.pad);
        a.kz = 4u * a.XpYp * (unsigned)(p->cam_cell[2] + s->L.pad);
    }

    if (stats) {
        a.stats = s->d_stats;
        VX_HIP(hipMemsetAsync(s->d_stats, 0, sizeof(unsigned long long) * ST_COUNT * 64, st));
    }
#ifdef VX_BLOCK_TIMING
    if (!ts.ids) {
        const size_t nb = (size_t)((w + 31) / 32) * (size_t)((h + 7) / 8);
        if (nb > s->blk_cap) {
            if (s->d_blk) VX_HIP(hipFree(s->d_blk));
            VX_HIP(hipMalloc(&s->d_blk, 16 * nb));
            s->blk_cap = nb;
        }
        s->blk_n = nb;
        a.blk_time = s->d_blk;
    }
#endif
    // events only for the stats launch (kernel_ms): two extra stream packets
    // per frame otherwise widen the gap between back-to-back frames
    if (stats) VX_HIP(hipEventRecord(s->ev0, st));
    int rc = launch_render(a, fmt, st);
    if (rc) return set_error(VX_EDEVICE, std::string("render launch failed: ") + hipGetErrorString((hipError_t)rc));
    if (cone) cone_lock.unlock();   // enqueued: a recycle now waits for this render
    if (lr) list_release(lr);
    if (stats) VX_HIP(hipEventRecord(s->ev1, st));
    if (stats) {
        unsigned long long v[ST_COUNT];
        VX_HIP(hipMemcpyAsync(v, s->d_stats, sizeof v, hipMemcpyDeviceToHost, st));
        VX_HIP(hipStreamSynchronize(st));
        float ms = 0.0f;
        VX_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        fill_stats(stats, v, ms, fmt == VX_PIXEL_RGBA32F ? 16 : 4);
    }
    return VX_OK;
}

int vx_prepare_sun(vx_scene *s, const vx_frame_params *p, void *stream, vx_exit_info *info) {
    if (!s || !p) return set_error(VX_EINVAL, "vx_prepare_sun: null argument");
    int rc = check_frame(p, 64, 64, VX_PIXEL_RGBA8);
    if (rc) return rc;
    VX_HIP(hipSetDevice(s->device));
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    FrameConsts fc;
    const int max_steps = p->max_shadow_steps > 0 ? p->max_shadow_steps : 2 * s->Z;
    frame_consts(*p, 64, 64, s->X, s->Y, s->Z, max_steps, fc);
    const int8_t *sunc = nullptr;
    bool built = false;
    vx_scene::Cone *cone = nullptr;
    {
        // ev0 is recorded inside cone_copy right before the build's first packet:
        // build_ms is the copy's GPU time, not the host's allocation or waits
        std::lock_guard<std::mutex> lock(s->cone_mu);
        rc = frame_exit(s, p, fc, st, &sunc, info, &built, &cone, s->ev0);
        if (rc) return rc;
        if (built) VX_HIP(hipEventRecord(s->ev1, st));
    }
    VX_HIP(hipStreamSynchronize(st));
    if (info && built) {
        float ms = 0.0f;
        VX_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        info->build_ms = ms;
    }
    return VX_OK;
}

int vx_render(vx_scene *s, const vx_frame_params *p, int w, int h, int fmt, void *out, int out_on_device,
              void *stream, vx_stats *stats) {
    int rc = check_render(s, p, w, h, fmt);
    if (rc) return rc;
    if (!out) return set_error(VX_EINVAL, "vx_render: null output");
    VX_HIP(hipSetDevice(s->device));
    const size_t bytes = (size_t)w * h * (fmt == VX_PIXEL_RGBA32F ? 16 : 4);
    if (out_on_device) return do_render(s, p, w, h, TileSpec(), fmt, out, stream, stats);
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    void *d_out = nullptr;
    VX_HIP(hipMallocAsync(&d_out, bytes, st));
    rc = do_render(s, p, w, h, TileSpec(), fmt, d_out, st, stats);
    if (rc == VX_OK) {
        hipError_t e = hipMemcpyAsync(out, d_out, bytes, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = set_error(VX_EDEVICE, std::string("readback failed: ") + hipGetErrorString(e));
    }
    (void)hipFreeAsync(d_out, st);
    (void)hipStreamSynchronize(st);
    return rc;
}

}  // extern "C"

// Tile / band-id lists live on the device, uploaded once per distinct list
// and never rewritten while cached: a render on any stream with a list the
// scene holds reads its buffer as it is, with no upload and no wait; a new
// list gets a new buffer, filled with hipMemcpyAsync on the caller's stream
// (renders of it on other streams wait for that copy's event until the host
// has seen it complete).  So threads may render different lists of one scene
// on their own streams at once, and a list change stalls nothing (VERDICT r05
// item 5: rounds 1-5 rewrote one buffer per kind after a device-wide wait).
// A list is pinned from its lookup until its render is enqueued (ListRef).
// Only when more than kMaxLists distinct lists are cached is the least
// recently used unpinned one freed, after a device wait (its readers may be
// in flight on any stream).
constexpr size_t kMaxLists = 256;

struct ListRef {
    vx_scene *s = nullptr;
    vx_scene::ListBuf *b = nullptr;
    void release() {
        if (!b) return;
        std::lock_guard<std::mutex> g(s->lists_mu);
        b->pins--;
        b = nullptr;
    }
    ~ListRef() { release(); }
};
static void list_release(ListRef *lr) { lr->release(); }

static unsigned long long list_hash(const int *ids, int n) {
    unsigned long long h = 1469598103934665603ull;   // FNV-1a over the ints
    for (int i = 0; i < n; i++) h = (h ^ (unsigned)ids[i]) * 1099511628211ull;
    return h ^ (unsigned long long)n;
}

static int list_acquire(vx_scene *s, hipStream_t st, const int *ids, int n, ListRef &ref) {
    const unsigned long long h = list_hash(ids, n);
    std::lock_guard<std::mutex> g(s->lists_mu);
    vx_scene::ListBuf *b = nullptr;
    for (auto &p : s->lists)
        if (p->hash == h && (int)p->ids.size() == n && std::equal(p->ids.begin(), p->ids.end(), ids)) b = p.get();
    if (b) {
        if (!b->ready_seen) {
            const hipError_t q = hipEventQuery(b->ready);
            if (q == hipSuccess) b->ready_seen = true;
            else if (q == hipErrorNotReady) VX_HIP(hipStreamWaitEvent(st, b->ready, 0));
            else VX_HIP(q);
        }
    } else {
        if (s->lists.size() >= kMaxLists) {
            size_t v = s->lists.size();
            for (size_t i = 0; i < s->lists.size(); i++)
                if (s->lists[i]->pins == 0 && (v == s->lists.size() || s->lists[i]->used < s->lists[v]->used)) v = i;
            if (v != s->lists.size()) {
                VX_HIP(hipDeviceSynchronize());
                vx_scene::ListBuf *c = s->lists[v].get();
                if (c->d) VX_HIP(hipFree(c->d));
                if (c->ready) VX_HIP(hipEventDestroy(c->ready));
                s->lists.erase(s->lists.begin() + (long)v);
            }
        }
        auto nb = std::make_unique<vx_scene::ListBuf>();
        nb->ids.assign(ids, ids + n);
        nb->hash = h;
        VX_HIP(hipMalloc(reinterpret_cast<void **>(&nb->d), sizeof(int) * (size_t)n));
        if (hipEventCreateWithFlags(&nb->ready, hipEventDisableTiming) != hipSuccess) {
            (void)hipFree(nb->d);
            return set_error(VX_EDEVICE, "list upload: event creation failed");
        }
        // the entry's own host copy is the source: it lives as long as the buffer
        hipError_t e = hipMemcpyAsync(nb->d, nb->ids.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(nb->ready, st);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);
            (void)hipFree(nb->d);
            (void)hipEventDestroy(nb->ready);
            return set_error(VX_EDEVICE, std::string("list upload: ") + hipGetErrorString(e));
        }
        s->lists.push_back(std::move(nb));
        b = s->lists.back().get();
    }
    b->pins++;
    b->used = ++s->list_tick;
    ref.s = s;
    ref.b = b;
    return VX_OK;
}

extern "C" {

int vx_render_tiles(vx_scene *s, const vx_frame_params *p, int w, int h, int ts, const int *tile_ids, int n_tiles,
                    int fmt, void *out_device, void *stream, vx_stats *stats) {
    int rc = check_render(s, p, w, h, fmt);
    if (rc) return rc;
    if (ts <= 0 || ts % VX_TILE_ALIGN_X) return set_error(VX_EINVAL, "tile_size must be a positive multiple of 32");
    if (!tile_ids || n_tiles <= 0 || !out_device) return set_error(VX_EINVAL, "vx_render_tiles: empty tile list");
    const int tx = (w + ts - 1) / ts, ty = (h + ts - 1) / ts;
    for (int i = 0; i < n_tiles; i++)
        if (tile_ids[i] < 0 || tile_ids[i] >= tx * ty) return set_error(VX_EINVAL, "tile id out of range");
    if ((unsigned long long)n_tiles * (unsigned long long)ts * (unsigned long long)ts >= (1ull << 32))
        return set_error(VX_EINVAL, "vx_render_tiles: the compact output must hold fewer than 2^32 pixels");
    VX_HIP(hipSetDevice(s->device));
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    ListRef lr;
    rc = list_acquire(s, st, tile_ids, n_tiles, lr);
    if (rc) return rc;
    const int *d_ids = lr.b->d;
    TileSpec t;
    t.tw = t.th = t.pitch = ts;
    t.tiles_x = tx;
    t.ids = d_ids;
    t.n = n_tiles;
    return do_render(s, p, w, h, t, fmt, out_device, st, stats, &lr);
}

int vx_render_bands(vx_scene *s, const vx_frame_params *p, int w, int h, int band_rows, const int *band_ids,
                    int n_bands, int fmt, void *out_device, int inplace, void *stream, vx_stats *stats) {
    int rc = check_render(s, p, w, h, fmt);
    if (rc) return rc;
    if (band_rows <= 0 || band_rows % VX_TILE_ALIGN_Y)
        return set_error(VX_EINVAL, "band_rows must be a positive multiple of 8");
    if (!band_ids || n_bands <= 0 || !out_device) return set_error(VX_EINVAL, "vx_render_bands: empty band list");
    const int nb = (h + band_rows - 1) / band_rows;
    for (int i = 0; i < n_bands; i++)
        if (band_ids[i] < 0 || band_ids[i] >= nb) return set_error(VX_EINVAL, "band id out of range");
    VX_HIP(hipSetDevice(s->device));
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    if (!inplace && (unsigned long long)n_bands * (unsigned long long)band_rows * (unsigned long long)w >= (1ull << 32))
        return set_error(VX_EINVAL, "vx_render_bands: the compact output must hold fewer than 2^32 pixels");
    ListRef lr;
    rc = list_acquire(s, st, band_ids, n_bands, lr);
    if (rc) return rc;
    const int *d_ids = lr.b->d;
    TileSpec t;
    t.tw = (w + VX_TILE_ALIGN_X - 1) / VX_TILE_ALIGN_X * VX_TILE_ALIGN_X;   // one tile spans the row
    t.th = band_rows;
    t.pitch = w;                      // compact bands keep the frame's row pitch
    t.tiles_x = 1;
    t.inplace = inplace ? 1 : 0;
    t.ids = d_ids;
    t.n = n_bands;
    return do_render(s, p, w, h, t, fmt, out_device, st, stats, &lr);
}

int vx_detile(vx_scene *s, int w, int h, int ts, const int *tile_ids, int n_tiles, int fmt, const void *tiles_device,
              void *frame_device, void *stream) {
    if (!s || !tile_ids || !tiles_device || !frame_device || ts <= 0 || n_tiles <= 0)
        return set_error(VX_EINVAL, "vx_detile: bad arguments");
    if (w <= 0 || h <= 0 || w > 32768 || h > 32768) return set_error(VX_EINVAL, "vx_detile: frame size out of range");
    if (fmt != VX_PIXEL_RGBA32F && fmt != VX_PIXEL_RGBA8) return set_error(VX_EINVAL, "vx_detile: unknown pixel format");
    if (ts % VX_TILE_ALIGN_X) return set_error(VX_EINVAL, "vx_detile: tile_size must be a positive multiple of 32");
    {
        const int tx = (w + ts - 1) / ts, ty = (h + ts - 1) / ts;
        for (int i = 0; i < n_tiles; i++)
            if (tile_ids[i] < 0 || tile_ids[i] >= tx * ty) return set_error(VX_EINVAL, "vx_detile: tile id out of range");
    }
    VX_HIP(hipSetDevice(s->device));
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    ListRef lr;
    int rc = list_acquire(s, st, tile_ids, n_tiles, lr);
    if (rc) return rc;
    const int *d_ids = lr.b->d;
    rc = launch_detile(tiles_device, frame_device, w, h, ts, (w + ts - 1) / ts, d_ids, n_tiles, fmt, st);
    if (rc) return set_error(VX_EDEVICE, std::string("detile failed: ") + hipGetErrorString((hipError_t)rc));
    return VX_OK;
}

int vx_field_build_gpu(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba_out, int device) {
    if (!color || !rgba_out || X <= 0 || Y <= 0 || Z <= 0 || X > 65535 || Y > 65535 || Z > 255)
        return set_error(VX_EINVAL, "vx_field_build_gpu: bad arguments (need 0<X,Y<=65535, 0<Z<=255)");
    const size_t N = (size_t)X * Y * Z;
    if (N > (size_t)INT32_MAX) return set_error(VX_EINVAL, "vx_field_build_gpu: grid too large for int32 volume sums");
    VX_HIP(hipSetDevice(device));
    uint8_t *d_col = nullptr;
    uint32_t *d_rgba = nullptr;
    hipStream_t st = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&d_col, N);
    if (e == hipSuccess) e = hipMalloc(&d_rgba, 4 * N);
    if (e == hipSuccess) e = hipMemcpyAsync(d_col, color, N, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = (hipError_t)field_build_device(d_col, d_rgba, X, Y, Z, st);
    if (e == hipSuccess) e = hipMemcpyAsync(rgba_out, d_rgba, 4 * N, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (d_col) (void)hipFree(d_col);
    if (d_rgba) (void)hipFree(d_rgba);
    if (st) (void)hipStreamDestroy(st);
    if (e != hipSuccess) return set_error(VX_EDEVICE, std::string("vx_field_build_gpu: ") + hipGetErrorString(e));
    return VX_OK;
}

}  // extern "C"
