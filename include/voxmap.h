/*
 * voxmap.h — C ABI of the MI355X-native Voxmap shading path (libvoxmap_hip.so).
 *
 * The reference's boundary for this path is the WebGL2 program interface of
 * P.renderer (src/web/render.js:94-132): uniforms u_quality, u_matrix,
 * u_cellPos, u_fractPos, u_frame, u_time, u_sunDir (src/shaders/render.h:5-11),
 * samplers u_noise / u_map (render.js:138-149, 194-206), and the RGBA8 canvas
 * the fragment shader writes (render.frag:4, map.js:7).  Its caller is
 * drawScene() (render.js:267-298).  Each entry point below names the
 * reference interface it replaces.  Plain C types only: pointers, sizes, ints.
 *
 * Conventions: return 0 = OK, < 0 = VX_E* code; the message of the last error
 * on the calling thread is vx_last_error().  A scene owns device memory on one
 * GPU; vx_render* calls are stream-ordered and may run concurrently on
 * different scenes, and on different streams of one scene -- except calls that
 * ask for stats: those share the scene's counters and events and must be
 * serialised per scene.  The tile / band lists of vx_render_tiles,
 * vx_render_bands and vx_detile are uploaded once per distinct list (on the
 * caller's stream, no device-wide wait) and never rewritten while cached, so
 * threads may render different lists of one scene concurrently.  The scene
 * keeps no stream handle of the caller's: a stream may be destroyed at any
 * time.  No global mutable state besides the thread-local error.
 */
#ifndef VOXMAP_H
#define VOXMAP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 10 (round 6): no signature or layout change; glass blends over the RGBA8
 * canvas byte with clamped source and alpha (render.js:84-86, map.js:7), band /
 * tile lists are cached per distinct list, no caller stream handle is kept,
 * a zeroed dist_cap falls back to VX_FALLBACK_DIST_CAP where 64 does not fit,
 * and the sun march reads the doom table (VX_FLAG_NO_DOOM: without). */
#define VX_ABI_VERSION 10

/* error codes */
#define VX_OK 0
#define VX_EINVAL (-1)   /* bad argument */
#define VX_EIO (-2)      /* file read failure */
#define VX_EFORMAT (-3)  /* gzip stream corrupt / not gzip */
#define VX_ECRYPTO (-4)  /* bad key, bad padding, AES failure */
#define VX_ESIZE (-5)    /* decoded size != expected (X*Y*Z*4, noise w*h*4) */
#define VX_EDEVICE (-6)  /* HIP runtime error */
#define VX_ENOMEM (-7)

/* field / asset container formats (render.js:52-58, utils.js:10-30) */
#define VX_FORMAT_AUTO 0    /* by extension: .blob -> BLOB, .gz -> BIN_GZ, else BIN */
#define VX_FORMAT_BIN 1     /* raw RGBA8 bytes */
#define VX_FORMAT_BIN_GZ 2  /* gzip of raw (makefile:70-71) */
#define VX_FORMAT_BLOB 3    /* AES-256-CBC(PKCS#7, fixed IV) of gzip (encrypt.js:12-46) */
#define VX_FORMAT_GRID 4    /* map only: raw palette-index grid, X*Y*Z bytes, 0 = air (the
                               input of sdf.cpp after its remap); the distance field is
                               built on the GPU */

/* Palette (render.vert:20-22): sdf.cpp builds it as {0 = air} + the map's
 * colours in ascending order (sdf.cpp:188-227), glass sorting last, so the
 * shipped shader has pal_size = 22 entries and glass = pal_size - 1 = 21.
 * map.bin's B channel is the remapped index, and the remap (sdf.cpp:229-233)
 * turns AIR into pal_size (the first zero entry of the zero-initialised pal[]).
 * The mesh (sdf.cpp:284) has faces only for colours < pal_size, and colour 0
 * never survives the remap: a cell is a surface candidate ("meshed") iff
 * 1 <= B <= VX_PAL_SIZE - 1.  Every other B -- air written as 22 by sdf.cpp,
 * 0 in palette grids (VX_FORMAT_GRID) -- is never a surface.  Shadows and AO
 * read R/G only: a block is R == G == 0 (sdf.cpp:430). */
#define VX_PAL_SIZE 22
#define VX_GLASS (VX_PAL_SIZE - 1)

/* output pixel formats */
#define VX_PIXEL_RGBA32F 0  /* 16 B/pixel, parity format */
#define VX_PIXEL_RGBA8 1    /* 4 B/pixel, what the canvas holds (map.js:185 toDataURL) */

/* feature flags (vx_frame_params.flags); 0 = the reference v1 shader */
#define VX_FLAG_NO_SHADOW 0x1u   /* skip the sun march (render.frag:232-235) */
#define VX_FLAG_NO_AO 0x2u       /* skip the trilinear AO sample (render.frag:223-225) */
#define VX_FLAG_NO_CLOUDS 0x4u   /* sky without noise fetches (render.frag:181-203) */
#define VX_FLAG_PRIMARY_ONLY 0x8u /* primary visibility only: v_color of the first surface
                                    (render.vert:30), sky = palette(0); BASELINE config C1 */
/* Extensions (BASELINE "full quality" = shadow + reflection +
 * clouds + rough normals).  The reference has no code for them (README.md:15-22
 * describes an earlier renderer's reflections and rough normals, README.md:56-57
 * lists soft shadows as to-do); DESIGN.md §3 "Extensions" defines them. */
#define VX_FLAG_REFLECT 0x10u    /* glass mirrors the traced scene (Fresnel-weighted) */
#define VX_FLAG_ROUGH 0x20u      /* shading normal jittered by white() noise (render.frag:21) */
#define VX_FLAG_FULL_QUALITY (VX_FLAG_REFLECT | VX_FLAG_ROUGH)
/* Diagnostics: force the integer primary-index path (the fp32 one is chosen
 * whenever it is exact; both give identical frames). */
#define VX_FLAG_INT_INDEX 0x40u
/* Soft shadows (shadow_samples > 1) marched by the pooled wave pass: the
 * marching fragments are compacted by a ballot and their samples dealt over
 * all 64 lanes (DESIGN.md §6 "C5").  Identical frames; off by default because
 * it measures slower on C5. */
#define VX_FLAG_SOFT_POOL 0x80u
/* VX_FLAG_SOFT_POOL plus LDS brick staging (the 8x8x8 march-channel block
 * around each fragment staged per pass; DESIGN.md §6 "C5").  Identical frames;
 * an experiment, off by default (slower on C5). */
#define VX_FLAG_SOFT_BRICK 0x100u
/* Diagnostics: march without the sun exit tables (DESIGN.md §3 "Sun exit
 * tables"), i.e. every step render.frag:92-136 takes.  Identical frames; the
 * shadow fetch counters are the reference's own step counts instead of the
 * steps this build takes. */
#define VX_FLAG_NO_EXIT 0x200u
/* Diagnostics: the orthant exit tables only, no per-sun cone table.  Identical frames. */
#define VX_FLAG_NO_CONE 0x400u
/* Diagnostics (ABI 8): the unit-cell G-buffer split of ABI <= 7.  By default a
 * fragment carries what the raster hands render.frag: v_cellPos = the origin of
 * the greedy quad that covers its face, v_fractPos = the hit point minus that
 * origin (render.vert:25-28, quads sdf.cpp:284-356).  With this
 * flag v_cellPos is the hit cell and v_fractPos the hit's fraction in it: the
 * same point, another fp32 split. */
#define VX_FLAG_UNIT_GBUF 0x800u
/* Glass (ABI 9; DESIGN.md §5 "Glass").  By default every front-facing glass
 * face in front of the opaque surface is blended as the reference's raster
 * does: glass quads after all opaque ones, in vertex.bin order (sdf.cpp:284,
 * 337), depth test LESS with depth writes on, SRC_ALPHA blending
 * (render.js:82-91) -- a pane is blended iff it is nearer than the last surface
 * written when its quad is drawn.  The render kernel shades a pixel whose ray
 * crosses one pane with one blend (the draw order's result) and re-walks the
 * panes in key order only where two or more stack.
 * VX_FLAG_GLASS_ORDER: the whole frame through the general draw-order kernel
 * (diagnostic / A-B: identical frames).  VX_FLAG_GLASS_SINGLE: the nearest
 * pane only, over the surface behind it (the single layer of ABI <= 8;
 * diagnostic, differs where panes stack). */
#define VX_FLAG_GLASS_ORDER 0x1000u
#define VX_FLAG_GLASS_SINGLE 0x8000u
/* Extension (ABI 8): every first surface mirrors the traced scene, as
 * VX_FLAG_REFLECT does for glass: the surface a pixel shows first (and every
 * pane blended in draw order) adds Schlick F * the colour along its mirror ray
 * (DESIGN.md §3 "Extensions"; README.md:18-25 describes a reflection pass over
 * the frame).  What a pane blends over is seen through the glass: not mirrored. */
#define VX_FLAG_REFLECT_ALL 0x2000u
/* Diagnostics (ABI 8): the frame's 32x8-pixel blocks dispatched bottom row first
 * (the launch's tail).  Identical frames. */
#define VX_FLAG_ROWS_BOTTOM_UP 0x4000u
/* Diagnostics: the frame's cone copy without the sun doom table (DESIGN.md §3
 * "Doom table": cells from which every ray of the frame's sun window provably
 * meets a solid cell within a few layers end the march unlit there).
 * Identical frames; the shadow fetch counters count the steps the march takes
 * without it.  VX_FLAG_SOFT_BRICK frames never use the doom table. */
#define VX_FLAG_NO_DOOM 0x20000u
#define VX_MAX_SHADOW_SAMPLES 16
/* ABI 9: the default box cap of the primary traversal (vx_scene_desc.dist_cap
 * = 0).  64 since round 5 (was 32): fewer steps, 2x the octant copies' memory
 * (C3 2.3 GB, C5 20.5 GB of 288 GB); identical frames.  The cap is also the
 * copies' border, and the padded plane must stay below 2^23 cells: a field
 * that fits with 32 but not with 64 (X = Y above ~2770) gets
 * VX_FALLBACK_DIST_CAP when dist_cap = 0 instead of VX_EINVAL. */
#define VX_DEFAULT_DIST_CAP 64
#define VX_FALLBACK_DIST_CAP 32

typedef struct vx_scene vx_scene;

/* Replaces loadTextures()/loadEncryptedTextures() (render.js:134-245):
 * where the field (u_map) and noise (u_noise) come from.  Exactly one of
 * map_path / map_bytes is set; noise may be absent (then a deterministic
 * synthetic noise texture of the same layout is generated). */
typedef struct vx_scene_desc {
    const char *map_path;
    const void *map_bytes;
    size_t map_size;
    int map_format;             /* VX_FORMAT_* */
    const char *key_jwk_k;      /* JWK "k" (base64url AES-256 key) for BLOB; may be NULL */
    const char *noise_path;
    const void *noise_bytes;
    size_t noise_size;
    int noise_format;           /* VX_FORMAT_* */
    int noise_w, noise_h;       /* 0 -> 1024 x 1024 (render.js:141) */
    int X, Y, Z;                /* 0 -> 1024, 256, 32 (render.h:14-16) */
    int device;                 /* HIP device ordinal */
    int dist_cap;               /* air-cube size cap of the primary traversal (and border width), 0 ->
                                   VX_DEFAULT_DIST_CAP */
    uint32_t noise_seed;        /* seed of the synthetic noise when none is given */
    int mesh_chunk;             /* ABI 8: CHUNK of the greedy mesh whose quads give the G-buffer split
                                   (voxmap.h:9, sdf.cpp:284-356); 0 -> Z; at most 255 */
} vx_scene_desc;

/* Replaces the per-frame uniforms set in drawScene() (render.js:287-295).
 * u_matrix is carried as the primary-ray basis (vx_frame_from_matrix /
 * vx_frame_from_orbit derive it); the view ray of pixel (px,py) of a w*h
 * frame is d = fwd + nx*right + ny*up with nx = (2px+1)/w - 1,
 * ny = 1 - (2py+1)/h (fp32, this operation order). */
typedef struct vx_frame_params {
    int quality;                /* u_quality: 0 = MODE_2D (render.js:278,287: the vertex2d footprint
                                   mesh, unlit), 1 = MODE_3D */
    int frame;                  /* u_frame (unused by render.frag, render.h:9) */
    float time;                 /* u_time = t % 1000 seconds (render.js:293) */
    int cam_cell[3];            /* u_cellPos = floor(camera position) */
    float cam_fract[3];         /* u_fractPos = fract(camera position) */
    float sun_dir[3];           /* u_sunDir (map.js:399-402) */
    float ray_fwd[3];
    float ray_right[3];
    float ray_up[3];
    uint32_t flags;             /* VX_FLAG_* */
    int max_shadow_steps;       /* MAX_STEPS (render.frag:12); <= 0 -> 2*Z */
    int shadow_samples;         /* ext soft shadows: <= 1 the reference's hard shadow,
                                   2..VX_MAX_SHADOW_SAMPLES sun-disc samples (vx_sun_samples) */
    float sun_radius;           /* ext: sun-disc radius (tangent-plane, radians) for the samples */
} vx_frame_params;

/* Counters of the work one vx_render call did (algorithmic). */
typedef struct vx_stats {
    uint64_t pixels, sky_px, block_px, glass_px;
    uint64_t primary_fetches;   /* field texels read by the primary march */
    uint64_t shadow_rays, shadow_fetches;
    uint64_t ao_samples, noise_px;
    uint64_t primary_cap_hits;  /* must be 0 */
    uint64_t reflect_rays, reflect_fetches;   /* ext REFLECT: reflection rays traced, texels read */
    uint64_t rough_px;          /* ext ROUGH: fragments with a jittered normal (4 noise texels each) */
    uint64_t primary_wave_iters, march_wave_iters;   /* diagnostic: loop iterations summed over
                                   waves (the primary's entry fetch counts as one); lane
                                   utilisation = fetches / (64 * wave_iters) <= 1 */
    uint64_t march_lane_slots;  /* diagnostic (ABI 6): per march wave iteration, the lanes that
                                   began that march; shadow_fetches / march_lane_slots = the
                                   utilisation of the marching lanes alone */
    uint64_t shadow_rays_resolved;   /* diagnostic (ABI 8): shadow rays counted in shadow_rays whose lit
                                   flag came from one exit-table test of the fragment's first step
                                   instead of a march (soft shadows): rays resolved, not
                                   marched; shadow_rays - this = rays marched */
    uint64_t alg_bytes;         /* 4*(primary+shadow+reflect fetches) + 32*ao + 80*clouded sky
                                   + 16*rough + out bytes */
    double kernel_ms;           /* HIP-event time of the render kernel(s) */
} vx_stats;

/* --- scene lifetime ------------------------------------------------------ */
int vx_scene_create(const vx_scene_desc *desc, vx_scene **out);
void vx_scene_destroy(vx_scene *scene);
/* Copy the device-resident field back (RGBA8 X*Y*Z, x fastest).  The device
 * keeps one copy per ray octant (bit 0/1/2: x/y/z direction negative) holding
 * the colour and the extents of the all-air box ahead of each cell for the
 * primary traversal.  vx_scene_read_field[_copy]: R, G, B are
 * map.bin's, A is the octant's air-cube size (= the smallest box extent);
 * vx_scene_read_field reads octant 0.  vx_scene_read_boxes: 4 bytes per cell,
 * colour, ex, ey, ez (ABI 3). */
int vx_scene_read_field(vx_scene *scene, void *host_out, size_t cap);
int vx_scene_read_field_copy(vx_scene *scene, int octant, void *host_out, size_t cap);
int vx_scene_read_boxes(vx_scene *scene, int octant, void *host_out, size_t cap);
int vx_scene_dims(const vx_scene *scene, int dims[3]);
/* The greedy mesh per face (ABI 8): 6 uint16 per cell, cell x fastest, normal
 * index fastest within a cell (render.vert:14-17): du | dv << 8, the offset of
 * the face from the origin of the quad covering it along the face's in-plane
 * axes u = (d+1)%3, v = (d+2)%3 (d = normal index / 2); 0xFFFF where the mesh
 * has no face.  The fragments' v_cellPos / v_fractPos split comes from it. */
int vx_scene_read_face_quads(vx_scene *scene, void *host_out, size_t cap);
/* The 2D mode mesh of the scene (what sdf.cpp:362-401 writes to
 * out/vertex2d.bin): the greedy quads of each column's top block (z >= 1) as
 * 16-byte vert2d records (sdf.cpp:154-173), six per quad.  out == NULL:
 * size query.  Rendering with quality = 0 draws this mesh (render.js:278). */
int vx_scene_vertex2d(const vx_scene *scene, void *out, size_t cap, size_t *out_size);

/* --- rendering (replaces gl.drawArrays at render.js:297 + the shaders) --- */
/* Render a full w*h frame.  out is RGBA32F or RGBA8, row-major, top row
 * first.  out_on_device != 0: out is a device pointer on the scene's GPU and
 * the call returns without synchronising (stream-ordered); otherwise out is
 * host memory and the call synchronises.  stream: hipStream_t or NULL (the
 * scene's own stream).  stats may be NULL (counting costs one extra pass). */
int vx_render(vx_scene *scene, const vx_frame_params *p, int w, int h, int pixel_format,
              void *out, int out_on_device, void *stream, vx_stats *stats);

/* Render only the listed tile_size x tile_size tiles (tile t covers pixels
 * [(t % tiles_x)*ts, ...) with tiles_x = ceil(w/ts); ts a multiple of 32)
 * into a compact, tile-major device buffer: tile k of the list occupies
 * ts*ts pixels at offset k*ts*ts, row-major inside the tile (n_tiles*ts*ts
 * below 2^32, else VX_EINVAL). */
int vx_render_tiles(vx_scene *scene, const vx_frame_params *p, int w, int h, int tile_size,
                    const int *tile_ids, int n_tiles, int pixel_format, void *out_device,
                    void *stream, vx_stats *stats);

/* Sun exit tables (ABI 7; DESIGN.md §3 "Sun exit tables").  The sun march
 * reads a copy of the march channel in which every cell from which the march
 * cannot end unlit holds the "left the grid" mark, so a march stops there,
 * lit, instead of stepping on to the grid edge (render.frag:92-136): the same
 * lit flag on every pixel, fewer steps.  Orthant copies (valid for any sun of
 * their octant) are built with the scene; a cone copy for the frame's sun
 * samples {octant, kx, ky} is built by the first vx_render* that needs it
 * (stream-ordered; the scene keeps two) -- the sun moves slowly
 * (map.js:399-402), so one copy serves many frames.  vx_prepare_sun builds the
 * copy frame p will read ahead of time (when the sun moves, off a frame's
 * path) and reports which one it is: kind 0 = none (a sun component below
 * 2^-10, a field without the padded march copy, or VX_FLAG_NO_EXIT), 1 = the
 * orthant copies, 2 = a cone copy.  It synchronises `stream` and, like a call
 * with stats, uses the scene's timing events (serialise it per scene). */
typedef struct vx_exit_info {
    int kind, octant, kx, ky;
    float build_ms;             /* vx_prepare_sun: GPU time of the copy it built (0: already built) */
} vx_exit_info;
int vx_prepare_sun(vx_scene *scene, const vx_frame_params *p, void *stream, vx_exit_info *info);

/* Scatter a compact tile-major device buffer back into a w*h frame. */
int vx_detile(vx_scene *scene, int w, int h, int tile_size, const int *tile_ids, int n_tiles,
              int pixel_format, const void *tiles_device, void *frame_device, void *stream);

/* Render the listed full-width bands of a w*h frame: band b covers rows
 * [b*band_rows, (b+1)*band_rows) clipped to h; band_rows a multiple of 8.
 * inplace != 0: out is the w*h frame and each band lands at its own rows
 * (other rows untouched); inplace == 0: compact, band k of the list at
 * k*band_rows*w pixels (same row pitch w; n_bands*band_rows*w below 2^32,
 * else VX_EINVAL).  The multi-GPU path's unit. */
int vx_render_bands(vx_scene *scene, const vx_frame_params *p, int w, int h, int band_rows,
                    const int *band_ids, int n_bands, int pixel_format, void *out_device,
                    int inplace, void *stream, vx_stats *stats);

/* --- one frame across the GPUs of a node (RCCL over xGMI) -----
 * Replaces nothing in the reference (one browser GPU); SURVEY §8(e).  One
 * process (or thread) per GPU, each with its own vx_scene of the same map.
 * Rank 0 makes a unique id and shares its VX_MGPU_UID_BYTES bytes out of band
 * (pipe, file, torch.distributed, MPI); every rank then calls vx_mgpu_create
 * (collective: blocks until all ranks have joined).  vx_mgpu_render
 * (collective, stream-ordered) deals full-width bands round-robin (band b ->
 * rank b % nranks, vx_mgpu_bands), renders each rank's bands in place into its
 * own w*h frame_device and gathers them into rank 0's frame_device with one
 * RCCL group of ncclSend/ncclRecv: rank 0's frame is the finished image, no
 * de-tile pass.  stats: this rank's bands only.  stream NULL: the scene's own
 * stream, for the render and the gather alike (the gather never reads rows a
 * render on another stream has not finished). */
#define VX_MGPU_UID_BYTES 128
typedef struct vx_mgpu vx_mgpu;
int vx_mgpu_unique_id(void *uid_out);
int vx_mgpu_create(vx_scene *scene, const void *uid, int nranks, int rank, vx_mgpu **out);
int vx_mgpu_render(vx_mgpu *m, const vx_frame_params *p, int w, int h, int band_rows, int pixel_format,
                   void *frame_device, void *stream, vx_stats *stats);
/* The gather step of vx_mgpu_render alone (collective, stream-ordered): the
 * bands of ranks 1..n-1 from their frame rows into rank 0's.  vx_mgpu_render
 * = vx_render_bands of this rank's bands (in place) + vx_mgpu_gather; the bench
 * times the two apart (gather and render time reported separately). */
int vx_mgpu_gather(vx_mgpu *m, int w, int h, int band_rows, int pixel_format, void *frame_device, void *stream);
int vx_mgpu_rank(const vx_mgpu *m, int *nranks, int *rank);
void vx_mgpu_destroy(vx_mgpu *m);
/* The deal: the band ids of `rank` (ascending) into ids[0..cap); returns their count. */
int vx_mgpu_bands(int h, int band_rows, int nranks, int rank, int *ids, int cap);
/* ABI 9: the band_rows for an h-row frame over nranks ranks -- the multiple of 8
 * up to max_rows (<= 0: 64) whose deal gives the busiest rank the fewest rows,
 * ties to the tallest band (a pure host function).  C4 (4320 rows) over 8 GPUs:
 * 32, i.e. 544 rows for the busiest rank against a mean of 540. */
int vx_mgpu_band_rows(int h, int nranks, int max_rows);
/* One point-to-point move of the gather (ABI 6): band `band` (rows
 * [band*band_rows, band*band_rows + rows)) goes from rank `src` (its owner) to
 * rank `dst` = 0; the bytes lie at `offset` of the w x h frame on both ranks. */
typedef struct vx_mgpu_xfer {
    int band, src, dst, rows;
    uint64_t offset, bytes;
} vx_mgpu_xfer;
/* The gather's transfer list as `rank` issues it (a pure host function, no
 * GPU): rank 0 receives every band whose owner is not 0, rank r > 0 sends its
 * own bands, in ascending band order.  Writes up to cap entries (out may be
 * NULL) and returns the count.  vx_mgpu_gather issues exactly these, as
 * ncclRecv (rank 0) / ncclSend (the owner) inside one RCCL group. */
int vx_mgpu_transfers(int w, int h, int band_rows, int pixel_format, int nranks, int rank, vx_mgpu_xfer *out,
                      int cap);

/* --- host helpers (map.js / math.js / sdf.cpp / utils.js) ----------------- */
/* map.js:373-391 orbit camera + math.js:37-42 projection (with its sqrt(aspect)
 * quirk): fills cam_cell/cam_fract/ray_* of p.  fov 60, near 1. */
int vx_frame_from_orbit(const double sbj[3], const double rot[3], int w, int h, vx_frame_params *p);
/* Same from a column-major u_matrix (render.js:288) and camera position. */
int vx_frame_from_matrix(const float u_matrix[16], const double cam_pos[3], vx_frame_params *p);
/* map.js:399-402: hour -> sun direction. */
void vx_sun_from_hour(double hour, float sun[3]);
/* The soft-shadow sun directions a frame with shadow_samples = n uses
 * (DESIGN.md §3): n <= 1 -> the sun itself; n is clamped to 16. */
int vx_sun_samples(const float sun[3], float radius, int n, float out[][3]);

/* Decode a field/asset container to raw bytes (render.js:52-58). */
int vx_decode(const void *in, size_t n, int format, const char *key_jwk_k,
              void *out, size_t out_cap, size_t *out_size);
/* AES-256-CBC encrypt with the reference's fixed IV (encrypt.js:12-46). */
int vx_blob_encrypt(const void *in, size_t n, const char *key_jwk_k,
                    void *out, size_t out_cap, size_t *out_size);

/* map.bin from a palette-index grid (x fastest, 0 = air, 1..21 palette
 * indices): sdf.cpp:405-470.  rgba_out holds X*Y*Z*4 bytes: R = up radius,
 * G = down radius, B = the index with air written as VX_PAL_SIZE (sdf.cpp:
 * 229-233, 466-468), A = 0 (sdf.cpp:469). */
int vx_field_build(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba_out, int n_threads);

/* Same output as vx_field_build, computed on GPU `device` (plane-parallel
 * restatement of the same recurrence; host buffers in and out). */
int vx_field_build_gpu(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba_out, int device);

/* vertex2d.bin (sdf.cpp:362-401) of a map.bin field (host; no GPU): the 2D
 * mode mesh vx_scene_vertex2d holds, from RGBA8 texels.  out == NULL: size. */
int vx_vertex2d(const uint8_t *rgba_field, int X, int Y, int Z, void *out, size_t cap, size_t *out_size);

/* Deterministic synthetic noise texture in noise.bin layout (noise.cpp:34-41). */
int vx_noise_synth(uint32_t seed, int w, int h, uint8_t *rgba_out);

const char *vx_last_error(void);
int vx_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
