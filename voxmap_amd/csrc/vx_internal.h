// vx_internal.h — shared between the C-ABI host code and the HIP kernels.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string>
#include <vector>
#include "../../include/voxmap.h"

namespace vx {

// Error plumbing: every C entry point returns a VX_E* code and leaves a
// message in a thread-local buffer (vx_last_error).
int set_error(int code, const std::string &msg);
const char *last_error();
// containers (vx_codec.cpp) and host field / noise builders (vx_field.cpp)
int decode_container(const unsigned char *in, size_t n, int format, const char *key,
                     std::vector<unsigned char> &out, size_t expect);
int format_from_path(const char *path);
int encrypt_blob(const unsigned char *in, size_t n, const char *key, std::vector<unsigned char> &out);
int field_build(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba, int n_threads);
int noise_synth(uint32_t seed, int w, int h, uint8_t *out);
// the HIP device ordinal a scene lives on (vx_api.cpp)
int scene_device(const vx_scene *s);
// the scene's own (non-blocking) stream: what vx_render* run on when given stream == NULL
void *scene_stream(const vx_scene *s);

// One sun direction of the march (render.frag:75-142) with the per-frame
// constants its loop needs: sign(r), |r|, RN(1/|r|) (Markstein division).
struct SunRay {
    float r[3], sign[3], abs[3], rcp[3];
    int up;                            // r.z > 0: march reads R, else G (render.frag:89)
    int fast;                          // every 2^-10 <= |r_i|: fast exact march path
};
void sun_ray(const float r[3], SunRay &s);
// ext soft shadows: the sun-disc sample directions
void sun_samples(const float sun[3], float radius, int n, float out[][3]);

// Per-frame constants derived on the host from vx_frame_params with the same
// fp32 operations (same order, IEEE, no contraction) the oracle performs per
// pixel, so the kernel reads bit-identical values.
struct FrameConsts {
    int cam_cell[3];
    float cam_fract[3];
    float cam_cell_f[3];               // (float)cam_cell: exact (|cam_cell| < 2^22, vx_host checks)
    // primary traversal setup, per axis (the kernel's former per-lane fp32 ops):
    // grid slab (float)(0 - cam_cell) - cam_fract, (float)(dim - cam_cell) - cam_fract,
    // and the camera-relative cell range (float)(-cam_cell), (float)(dim - cam_cell - 1)
    float slab_lo[3], slab_hi[3], cell_lo[3], cell_hi[3];
    float fwd[3], right[3], up[3];
    float fw, fh, rcp_w, rcp_h;        // (float)w, (float)h and RN(1/w), RN(1/h)
    float sun[3];                      // u_sunDir
    float sun_sign[3];                 // sign(u_sunDir) (render.frag:94)
    float sun_abs[3], sun_rcp[3];      // |u_sunDir|, RN(1/|u_sunDir|)
    int sun_up;                        // u_sunDir.z > 0: march reads R, else G (render.frag:89)
    int march_fast;                    // every 2^-10 <= |u_sunDir_i|: fast exact march path
    int max_steps;                     // MAX_STEPS = 2*Z (render.frag:12)
    float scatterCol[3], spaceCol[3], shadeCol[3];   // render.frag:168-170, 220
    float shadeFactor[6];              // per normal index (render.frag:228-229)
    float normalCol[6][3];             // per normal index (render.frag:211-217)
    float sf[3];                       // Sf = 1/dims (render.h:24)
    float cloudTime;                   // u_time * 4e-3 (render.frag:183)
    float skyOff[2];                   // 1e-4 * (u_cellPos.xy + u_fractPos.xy) (render.frag:191)
    int quality;
    unsigned flags;
    int n_sun;                         // ext: sun samples per shadow (1 = the reference's hard shadow)
    int soft_sg;                       // ext: axis-sign pattern shared by every sample (bit i: r_i > 0), all
                                       // of them on the fast path and reading one channel; -1 otherwise
    int soft_lg;                       // ext: log2 of the lanes per fragment in the pooled march (2^lg >= n_sun)
    SunRay sun_k[VX_MAX_SHADOW_SAMPLES];   // ext: soft-shadow sample directions
};

// Parameters of one render launch (passed by value to the kernel).
struct KernelArgs {
    const uint32_t *prim;    // 8 padded octant copies: colour | ex << 8 | ey << 16 | ez << 24 (FieldLayout)
    const uint8_t *sun;      // R channel then G channel, X*Y*Z bytes each
    const int8_t *sunp;      // R then G, int8, inside a border of SB cells of -1 (nullptr: Z > 126)
    int SB;                  // border width of sunp (Z + 2: a march step moves <= Z + 1 cells per axis)
    float SBf;               // (float)SB
    int SXp;                 // padded row length of sunp
    unsigned SXpYp, sunp_texels;
    const int8_t *sunx;      // 8 orthant-exit copies of sunp's channel, one per ray octant (bit i: r_i > 0), or nullptr
    const int8_t *sunc;      // the frame's cone-exit copy (every sample of the frame reads it), or nullptr
    const uint16_t *rg;      // R | G << 8 per cell
    const uint32_t *rg2;     // AO x-pairs (X + 1 per row): entry p = (R, G) of cells clamp(p - 1), clamp(p)
    const uint32_t *noise;   // RGBA8 noise texels
    const uint32_t *noise4;  // noise quads, planes A, R, G, B: entry (x, y) = that channel of (x, y), (x+1, y),
                             // (x, y+1), (x+1, y+1), REPEAT-wrapped
    const uint32_t *fp2d;    // 2D mode: 2 words per column (x fastest): vis colour, quad corner x0 | y0 << 16
    const uint16_t *qface;   // greedy mesh per face: plane n (normal index) of X*Y*Z u16, du | dv << 8 (launch_face_quads)
    const uint32_t *qcopy;   // 8 copies in the prim layout: the octant's entry faces' offsets (launch_qcopy), or null
    int quad_gbuf;           // 1: fragments carry the quad-relative split (render.vert:25-28); 0: the unit cell
    int chunk;               // the mesh's CHUNK (glass draw order, face_key)
    unsigned long long *blk_time;   // diagnostics build (VX_BLOCK_TIMING): per block start, end; else null
    int X, Y, Z;
    int noise_w, noise_h;    // powers of two
    float noise_rw, noise_rh;    // 1/noise_w, 1/noise_h (exact)
    int noise_lw;                // log2(noise_w)
    int w, h;                // frame size
    int tile_w, tile_h;      // tiled mode: tile size in pixels (multiples of VX_TILE_ALIGN_X / _Y)
    int tiles_x;             // ceil(w / tile_w)
    int tile_pitch;          // tiled mode, compact: row pitch in pixels (tile_w for tiles, w for bands)
    int tile_inplace;        // tiled mode: 1 = pixels at their frame positions, 0 = compact tile-major
    const int *tile_ids;     // tiled mode: device list of tile ids, else nullptr
    int n_tiles;
    void *out;               // RGBA32F or RGBA8
    unsigned long long *stats;   // device counters (nullptr = no stats)
    vx_frame_params p;
    int max_shadow_steps;
    int Xp;                  // padded row length (FieldLayout)
    int pad;                 // border width of the prim copies (FieldLayout::pad)
    unsigned XpYp;           // padded slice size
    unsigned XY, XYZ;        // X*Y, X*Y*Z
    unsigned copy_texels;    // cells per prim copy (FieldLayout::texels)
    unsigned kcam;           // padded index of the camera cell, mod 2^32
    FrameConsts fc;
    // fp32 x/y primary index (vx_render decides): byte offset
    // from prim = cvt(fma(4Xp, h1 + ky, fma(4, h0, kx4))) + 4XpYp*(int)h2 + kz
    // (mod 2^32), exact while 4*Xp*Yp < 2^23 and the 8 copies < 4 GiB
    int prim_f32;            // 0: the integer index path
    float kx4, ky;           // 4*(camera padded x), camera padded y (ray octant terms added per lane)
    unsigned kz;             // 4*XpYp*(camera padded z), mod 2^32
};

// tile sizes must be multiples of the render kernel's block (32 x 8 pixels)
constexpr int VX_TILE_ALIGN_X = 32, VX_TILE_ALIGN_Y = 8;

void frame_consts(const vx_frame_params &p, int w, int h, int X, int Y, int Z, int max_steps, FrameConsts &fc);

enum StatSlot {
    ST_PIXELS = 0, ST_SKY, ST_BLOCK, ST_GLASS, ST_PRIM_FETCH, ST_SHADOW_RAYS, ST_SHADOW_FETCH,
    ST_AO, ST_NOISE_PX, ST_CAP_HITS, ST_REFL_RAYS, ST_REFL_FETCH, ST_ROUGH, ST_PRIM_WITERS, ST_MARCH_WITERS,
    ST_MARCH_SLOTS, ST_SHADOW_RESOLVED, ST_COUNT
};

// Field data in HBM (vx_kernels.hip): `prim` = 8 copies (one
// per ray octant) of the X x Y x Z grid, u32 colour | air-box extents << 8,
// 16, 24, inside a border of pad = cap sentinel cells; `sun` = R and G
// channels (u8); `rg` = R | G << 8 (u16).
struct FieldLayout {
    int pad, Xp, Yp, Zp;
    size_t texels;           // Xp * Yp * Zp, one prim copy
};
FieldLayout field_layout(int X, int Y, int Z, int cap);

// vx_scene_create's host half (vx_host.cpp): the description checked, the map
// and noise containers decoded and size-checked (or the noise synthesised).
struct SceneInputs {
    int X = 0, Y = 0, Z = 0, NW = 0, NH = 0, cap = 0, chunk = 0;
    bool from_grid = false;           // VX_FORMAT_GRID: field holds nothing, the device builds it
    int max_rg = 0;                   // largest R/G of a decoded map.bin (march_pad needs <= Z)
    std::vector<unsigned char> field, noise;
};
int scene_inputs(const vx_scene_desc *d, SceneInputs &in);
// vx_render*'s frame checks (vx_host.cpp)
int check_frame(const vx_frame_params *p, int w, int h, int fmt);
// padded int8 sun channels (border = -1) from the linear RGBA upload
int launch_sun_pad(const uint32_t *lin, int8_t *sunp, int X, int Y, int Z, int SB, void *stream);
// Sun exit tables (DESIGN.md §3 "Sun exit tables"): copies of sunp's march
// channel with every cell from which the march cannot end unlit set to -1.
// The 8 orthant copies (sunx, 8 * padded texels; flags = X*Y*Z bytes of
// scratch), built with the scene, hold for any direction of their octant:
int launch_sun_exit(const int8_t *sunp, int8_t *sunx, uint8_t *flags, int X, int Y, int Z, int SB, void *stream);
// a cone copy (one padded channel, border pre-filled with -1) holds for every
// up-going direction of octant oct whose slopes |r_x/r_z| <= kx - 1/64,
// |r_y/r_z| <= ky - 1/64 (layer recursion, kx, ky <= SB):
int launch_sun_cone(const int8_t *sunp, int8_t *sunc, int X, int Y, int Z, int SB, int oct, int kx, int ky,
                    void *stream);
// The sun doom table (DESIGN.md §3 "Doom table", oracle vxo_field_doom): in a
// cone copy already holding its exit marks and face bits, every cell from which
// every ray of the sub-cell window {sx, sy, xlo, xhi, ylo, yhi} (doom_plan)
// provably enters a solid cell h <= hmax layers up, and whose march texel is
// >= 1, becomes kDoomBase - doom_cross(h) (-9 .. -128, doom_cross <= kDoomHCap): the boundary crossings
// a march makes from it into the block; the march reads the texel itself from
// the plain channel when it goes on from such a cell.
constexpr int kDoomQ = 8, kDoomHCap = 120, kDoomBase = -8;
// the stop rule's soundness: a march step ends within 0.1024 cell of where its
// segment entered the doomed ray's solid region (T = 1, |r_a| >= 2^-10), inside
// the 1/Q margin the recursion checks (DESIGN.md §3 "Doom table", the stop rule)
static_assert(kDoomQ <= 9, "doom margin 1/Q must exceed the 0.1024-cell step overshoot plus drift");
int launch_sun_doom(const int8_t *sunp, int8_t *sunc, int X, int Y, int Z, int SB, const int plan[7], void *stream);
// the doom table's plan for a frame's samples (all fast, one octant, r_z > 0)
// (oracle vxo_doom_plan): sx, sy, the per-layer sub-cell offsets xlo, xhi,
// ylo, yhi, and hmax, the largest h whose stop rule j + 2 doom_cross(h) <
// MAX_STEPS can hold (hmax < 1: no table)
void doom_plan(const FrameConsts &fc, int plan[7]);
// crossings from a doomed cell with h into its block (oracle vxo_doom_cross):
// h in z, floor(h xhi / Q) + 1 in x, floor(h yhi / Q) + 1 in y
constexpr int doom_cross(int h, int xhi, int yhi) {   // (constexpr: host and device)
    return h + (h * xhi) / kDoomQ + 1 + (h * yhi) / kDoomQ + 1;
}
// which copy a frame's sun march reads: 1 = one cone copy {oct, kx, ky} for every
// sample (all on the fast path, one sign pattern, r_z > 0, slopes <= 4, kx, ky
// <= SB); 0 = each fast sample its octant's orthant copy (oracle vxo_exit_plan)
int exit_plan(const FrameConsts &fc, int SB, int *oct, int *kx, int *ky);
// the greedy mesh per face (sdf.cpp:281-356): 6 planes (normal index) of X*Y*Z u16, du | dv << 8 = the
// face's offset from its quad's origin, 0xFFFF = no face; from the upload after launch_field_vis
int launch_face_quads(const uint32_t *lin, uint16_t *qface, int X, int Y, int Z, int chunk, void *stream);
int launch_face_quads_interleave(const uint16_t *qface, uint16_t *out, size_t N, void *stream);
// per ray octant, the entry faces' offsets (10 bits each) in the prim copies' padded layout (CHUNK <= 32)
int launch_qcopy(const uint16_t *qface, uint32_t *qcopy, int X, int Y, int Z, int pad, size_t texels, void *stream);
// AO x-pair array from rg: (X + 1) * Y * Z u32 (R, G of two x-neighbours, clamped)
int launch_ao_pairs(const uint16_t *rg, uint32_t *rg2, int X, int Y, int Z, void *stream);
// noise quad texture from the RGBA8 noise: 4 planes (A, R, G, B) of each texel's wrapped 2x2 block
int launch_noise_quads(const uint32_t *noise, uint32_t *noise4, int W, int H, void *stream);
// linear RGBA upload -> sun, rg
int launch_field_pack(const uint32_t *lin, uint8_t *sun, uint16_t *rg, int X, int Y, int Z, void *stream);
// prefix sums of solid cells of the upload, (X+1)(Y+1)(Z+1) ints
int launch_field_psum(const uint32_t *lin, int *S, int X, int Y, int Z, void *stream);
// upload with A = an octant's cube sizes (launch_field_octant) -> that octant's prim copy (boxes)
int launch_field_box(const uint32_t *lin, const int *S, uint32_t *prim_copy, int X, int Y, int Z, int pad, int cap,
                     int oct, void *stream);
// RGBA of one octant copy, linear (B from bcol = map.bin's B channel)
int launch_field_unpack(const uint16_t *rg, const uint8_t *bcol, const uint32_t *prim_copy, uint32_t *out, int X,
                        int Y, int Z, int pad, void *stream);
// upload's B -> vis colour in place (1..VX_PAL_SIZE-1 kept, else 0), original B into bcol
int launch_field_vis(uint32_t *lin, uint8_t *bcol, int X, int Y, int Z, void *stream);

// 2D mode (sdf.cpp:362-401; DESIGN.md §3 "2D mode"): the footprint's greedy quads
struct Quad2d {
    int x, y, w, h, color;
};
void mesh2d(const uint8_t *c2d, int X, int Y, std::vector<Quad2d> &quads, uint32_t *origin);
size_t vertex2d_bytes(const std::vector<Quad2d> &quads, uint8_t *out, size_t cap);
// c2d (X*Y, x fastest) of the upload after launch_field_vis: vis colour of each column's top block, z >= 1
int launch_footprint(const uint32_t *lin, uint8_t *c2d, int X, int Y, int Z, void *stream);

// Launchers (vx_kernels.hip).  Return a hipError_t as int.
int launch_render(const KernelArgs &a, int pixel_format, void *stream);
int launch_detile(const void *tiles, void *frame, int w, int h, int tile_size, int tiles_x,
                  const int *tile_ids, int n_tiles, int pixel_format, void *stream);
// map.bin texels (A = 0) from a device palette grid (vx_field_gpu.hip)
int field_build_device(const uint8_t *d_col, uint32_t *d_rgba, int X, int Y, int Z, void *stream);
// A channel of octant copy `oct` (in place in a linear grid upload)
int launch_field_octant(uint32_t *field, int X, int Y, int Z, int cap, int oct, uint8_t *scratch_a,
                        uint8_t *scratch_b, void *stream);

}  // namespace vx
