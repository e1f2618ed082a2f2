/*
 * vxo.h — CPU ORACLE for the Voxmap shading path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a scalar C restatement of the reference's per-pixel path, written
 * from reading the reference as text.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker or the
 * timed CPU baseline — never as part of the product path.
 *
 * PARITY STATUS: "parity unpinned" against reference outputs.  The reference
 * is GLSL ES 3.00 running in a browser and has no tests, golden images or
 * known-answer vectors; compiling/running the reference's
 * C++ was refused by the environment, so it is read as text
 * only.  The oracle is pinned instead by hand-derived known-answer tests
 * (tests/test_oracle_kat.py: empty map, single block shadow footprint,
 * closed-form sky, march() traces) and by the plaintext reference assets
 * (res/noise.bin.gz checksums).
 *
 * Restated reference files (all under /root/reference):
 *   src/shaders/render.frag:12-142   march(), texture helpers
 *   src/shaders/render.frag:147-252  main() shading
 *   src/shaders/render.h:2-24        constants, uniforms
 *   src/shaders/render.vert:14-22    normal()/palette() tables
 *   src/web/render.js:62,138-149,194-206  texel layout and sampler state
 *   src/gen/sdf.cpp:405-470          field definition (see vxo_field.c)
 */
#ifndef VXO_H
#define VXO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int X, Y, Z;              /* field dims (render.h:14-16) */
    const uint8_t *field;     /* RGBA8 X*Y*Z texels, x fastest (render.js:62) */
    const uint8_t *noise;     /* RGBA8 noise texture (render.js:138-149) */
    int noise_w, noise_h;
    const uint8_t *oct_e[8];  /* vxo_field_box per ray octant: 3 extents per cell (primary traversal) */
    const uint32_t *fp2d;     /* 2D mode (quality 0): per column (x fastest) colour, quad corner x0 | y0 << 16
                                 of the sdf.cpp:362-401 mesh (oracle/__init__.py footprint_2d); may be NULL */
    int exit_mode;            /* 0: the reference's literal march, every step of render.frag:92-136 counted.
                                 1: the build's sun exit tables (vxo_field_exit, chosen per frame by
                                 vxo_exit_plan), so the shadow fetch counters equal the kernel's; frames are
                                 identical either way.  2: orthant tables only (VX_FLAG_NO_CONE). */
    const uint8_t *held;      /* a table the caller built (vxo_field_exit) and keeps, for {held_oct, held_kx,
                                 held_ky}: a frame whose plan needs exactly that table reads it instead of
                                 building its own (the CPU baseline's timed frames); NULL = none */
    int held_oct, held_kx, held_ky;
    const uint16_t *qoff;     /* quad-relative G-buffer: per cell and normal index, the offset
                                 (du | dv << 8) of the face from its greedy quad's origin (vxo_face_quads); the
                                 primary records then carry v_cellPos = the quad origin and v_fractPos = the hit
                                 point minus it, as render.vert:25-28 hands them over.  NULL: the unit cell. */
    int chunk;                /* the mesher's CHUNK (voxmap.h:9: Z); <= 0 -> Z */
    int unit_split;           /* 1: the unit-cell split even with qoff set (qoff then serves the glass draw
                                 order only); a frame's flag VXO_FLAG_UNIT_GBUF does the same per frame */
    const uint8_t *held_doom; /* a doom table the caller built (vxo_field_doom) for the plan held_dplan
                                 (sx, sy, xlo, xhi, ylo, yhi), read instead of building one; NULL = none */
    int held_dplan[7];
} vxo_scene;

/* Mirrors include/voxmap.h vx_frame_params field-for-field. */
typedef struct {
    int quality;              /* u_quality (render.h:5) */
    int frame;                /* u_frame (unused by render.frag) */
    float time;               /* u_time (render.h:10) */
    int cam_cell[3];          /* u_cellPos */
    float cam_fract[3];       /* u_fractPos */
    float sun_dir[3];         /* u_sunDir */
    float ray_fwd[3];         /* primary ray basis: d = fwd + nx*right + ny*up */
    float ray_right[3];
    float ray_up[3];
    unsigned flags;
    int max_shadow_steps;     /* MAX_STEPS = 2*Z (render.frag:12); <=0 -> 2*Z */
    int shadow_samples;       /* ext (README "Soft shadows"): <=1 hard, 2..16 sun samples */
    float sun_radius;         /* ext: angular radius of the sun disc, radians */
} vxo_frame;

/* Extension flags (no reference code exists for them, so the
 * build defines them — DESIGN.md §3 "Extensions"): */
#define VXO_FLAG_REFLECT 0x10u  /* glass reflects the traced scene (README.md:15-20) */
#define VXO_FLAG_ROUGH 0x20u    /* per-fragment normal jitter from white() (README.md:22, render.frag:21) */
#define VXO_MAX_SAMPLES 16
/* Glass (DESIGN.md §5 "Glass"), include/voxmap.h VX_FLAG_GLASS_*: by default
 * every front-facing glass face in front of the opaque surface is blended as
 * the reference's raster does -- glass quads drawn after all opaque ones in
 * vertex.bin order (sdf.cpp:284,337), depth test LESS with depth writes on,
 * SRC_ALPHA blending (render.js:82-91); every pane the ray crosses takes part.
 * VXO_FLAG_GLASS_SINGLE: the nearest pane only, over the surface behind it
 * (diagnostic).  VXO_FLAG_GLASS_ORDER selects the kernel's whole-frame path
 * and changes nothing here. */
#define VXO_FLAG_GLASS_ORDER 0x1000u
#define VXO_FLAG_GLASS_SINGLE 0x8000u
#define VXO_FLAG_UNIT_GBUF 0x800u   /* the unit-cell G-buffer split (include/voxmap.h VX_FLAG_UNIT_GBUF) */
#define VXO_FLAG_REFLECT_ALL 0x2000u /* ext: the first surface of every pixel mirrors the scene (as REFLECT glass) */
/* Oracle-only diagnostic: the round-5 blend (unclamped fp32 src and dst, dst
 * not read back from the 8-bit canvas), kept so tests can show which pixels
 * the GL blend stage (blend_canvas) changes.  Not a kernel flag. */
#define VXO_FLAG_BLEND_FLOAT 0x10000u
/* The sun doom table (DESIGN.md §3 "Doom table"), restated from the kernel's
 * launch_sun_doom: where a frame reads a cone exit copy, a cell from which every ray of the frame's sun samples
 * provably enters a solid cell h layers up (h <= the plan's hmax) ends the
 * march unlit at once when the march lands there early enough (landing index
 * j with j + 2 C < MAX, C = vxo_doom_cross(h)); later, the march goes on with
 * the cell's texel and no fetch is counted.  Only cells whose march texel is
 * >= 1 carry it.  hmax = the largest h with 1 + 2 C(h) < MAX and C(h) <=
 * VXO_DOOM_HCAP (the kernel's int8 codes).  VXO_FLAG_NO_DOOM (= VX_FLAG_NO_DOOM) and
 * VX_FLAG_SOFT_BRICK frames read copies without it.  Frames are identical. */
#define VXO_FLAG_NO_DOOM 0x20000u
#define VXO_FLAG_SOFT_BRICK 0x100u
#define VXO_DOOM_Q 8     /* <= 9: the margin 1/Q the stop rule needs (DESIGN.md §3 "Doom table") */
#define VXO_DOOM_HCAP 120
/* plan = {sx, sy, xlo, xhi, ylo, yhi, hmax}: the sub-cell window of the
 * frame's samples (all fast, one octant, r_z > 0), and hmax for its MAX
 * (hmax < 1: no table) */
void vxo_doom_plan(const float dirs[][3], int n, int max_steps, int plan[7]);
/* the boundary crossings a march makes from a doomed cell with h into its
 * block: h in z, floor(h xhi / Q) + 1 in x, floor(h yhi / Q) + 1 in y */
int vxo_doom_cross(int h, int xhi, int yhi);
/* code[z][y][x] = vxo_doom_cross(h, ...) for doomed cells (h <= plan[6]), else 0 */
void vxo_field_doom(const uint8_t *rgba, int X, int Y, int Z, const int plan[7], uint8_t *code);

typedef struct {
    uint64_t pixels, sky_px, block_px, glass_px;
    uint64_t primary_fetches;  /* texels read by the primary march */
    uint64_t shadow_rays, shadow_fetches;
    uint64_t ao_samples, noise_px;
    uint64_t primary_cap_hits; /* primary marches that hit the iteration cap */
    uint64_t reflect_rays, reflect_fetches;  /* ext REFLECT: traced reflection rays, texels */
    uint64_t rough_px;         /* ext ROUGH: fragments whose normal was jittered */
} vxo_stats;

/* march() result (render.frag:64-70) */
typedef struct {
    int cell[3];
    float fract[3];
    float normal[3];
    float min_dist;
    int step;
    int fetches;
} vxo_march_t;

/* G-buffer record: what render.vert hands to render.frag (render.vert:24-31). */
typedef struct {
    int id;                   /* 0 block, 1 sky, 2 glass (sdf.cpp:337, :250-279) */
    int color;                /* palette index (B channel) */
    int normal_idx;           /* 0..5 (render.vert:14-17) */
    int cell[3];              /* v_cellPos */
    float fract[3];           /* v_fractPos */
    float t;                  /* ray parameter of the face (its depth along the view ray) */
    uint64_t key;             /* glass faces: draw order of the covering quad (vxo_face_order) */
} vxo_gbuf;

/* Literal march() (render.frag:75-142). */
void vxo_march(const vxo_scene *s, const int cell[3], const float fract[3],
               const float dir[3], int max_steps, vxo_march_t *res);

/* Primary visibility (replaces raster of vertex.bin).
 * Returns the number of surface records written (0 = sky, 1 = opaque,
 * 2 = glass in g[0] followed by what is behind it in g[1] (g[1].id may be 1). */
int vxo_primary(const vxo_scene *s, const vxo_frame *f, const float dir[3],
                vxo_gbuf g[2], int *fetches, int *cap_hit);

/* Diagnostic: per pixel of a w*h frame, the front-facing glass faces the view
 * ray crosses before its opaque surface (the reference blends each, in draw
 * order; the build blends the first one: DESIGN.md §5).  out: w*h bytes. */
void vxo_glass_layers(const vxo_scene *s, const vxo_frame *f, int w, int h, uint8_t *out, int n_threads);

/* Diagnostic: per pixel of a tw x th block, the fetch counts of its sun
 * marches in shading order (-1 past the last), maxrec ints per pixel. */
void vxo_march_lengths(const vxo_scene *s, const vxo_frame *f, int w, int h, int px0, int py0, int tw, int th,
                       int *out, int maxrec);

/* Shade one fragment (render.frag:147-252).  out_rgba[3] = alpha. */
void vxo_shade(const vxo_scene *s, const vxo_frame *f, const vxo_gbuf *g,
               const float prim_dir[3], float out_rgba[4], vxo_stats *st);

/* Render rows r = row0, row0+row_step, ... of a w*h frame into out (RGBA fp32,
 * row-major, top row first).  Rows not rendered are left untouched.
 * Uses OpenMP over rows when compiled with it; n_threads<=0 -> default. */
void vxo_render(const vxo_scene *s, const vxo_frame *f, int w, int h,
                int row0, int row_step, float *out, vxo_stats *st, int n_threads);

/* Per-pixel ray direction for pixel (px,py) (float, fixed op order). */
void vxo_pixel_dir(const vxo_frame *f, int w, int h, int px, int py, float d[3]);

/* Soft-shadow sun directions (ext): n samples of the sun disc of angular
 * radius `radius` around sun (Vogel spiral, double precision, rounded to
 * float).  n <= 1 gives the sun itself. */
void vxo_sun_samples(const float sun[3], float radius, int n, float out[][3]);

/* render.vert:21 palette(p) for p = 0..21. */
void vxo_palette(float out[22][3]);

/* Deterministic transcendental used by both oracle and kernel. */
float vxo_exp2(float x);

/* --- palette / air encoding ---------------------------------------------
 * sdf.cpp builds the palette as {0} + the map's colours (sdf.cpp:188-227):
 * pal_size = 22 for the shipped shader (render.vert:21), glass = 21.  The
 * remap (sdf.cpp:229-233) writes air as B = pal_size; the mesher meshes only
 * colours < pal_size (sdf.cpp:284) and colour 0 never survives the remap.  So
 * a cell can show a face iff 1 <= B <= 21 ("vis colour" B, else 0). */
#define VXO_PAL_SIZE 22
static inline int vxo_vis(int b) { return (b >= 1 && b < VXO_PAL_SIZE) ? b : 0; }

/* --- greedy mesh per face, vxo_mesh.c (sdf.cpp:281-356) ------------------ */
#define VXO_NO_FACE 0xFFFFu
/* out[6 * cell + nidx] = du | dv << 8: the offset, along the face's in-plane
 * axes u = (d+1)%3 and v = (d+2)%3 (d = nidx / 2), of the face of `cell` with
 * normal index nidx from the origin of the greedy quad covering it;
 * VXO_NO_FACE where the mesh has no such face.  chunk <= 0 -> Z. */
void vxo_face_quads(const uint8_t *rgba, int X, int Y, int Z, int chunk, uint16_t *out);
/* Draw order (vertex.bin emission order) of the quad covering a face, for
 * faces of one colour: smaller is drawn first. */
uint64_t vxo_face_order(const int cell[3], int nidx, uint16_t off, int X, int Y, int Z, int chunk);
/* Diagnostic: per pixel of rows row0::row_step, the sun-march result and AO
 * distance of the first surface (slot 0) and of what a glass pane blends over
 * (slot 1): lit[2*px + k] = lit samples (0/1 for the hard shadow), 255 = no
 * march; amb[2*px + k] = sdf() of :223, NaN = no sample. */
void vxo_render_terms(const vxo_scene *s, const vxo_frame *f, int w, int h, int row0, int row_step,
                      uint8_t *lit, float *amb, int n_threads);

/* --- field (map.bin) definition, vxo_field.c ---------------------------- */
/* Build the RGBA8 field from a palette-index grid (x fastest), restating
 * sdf.cpp:405-470 literally (serial x->y->z order, clamped-index quirks). */
void vxo_field_build(const uint8_t *color, int X, int Y, int Z, uint8_t *rgba);
/* Per-cell size r of the all-air cube ahead of the cell for ray octant oct
 * (bit 0/1/2: x/y/z direction negative), capped: the primary traversal's own
 * data, X*Y*Z bytes into r_out. */
void vxo_field_octant(const uint8_t *rgba, int X, int Y, int Z, int cap, int oct, uint8_t *r_out);
/* Per-cell extents (ex, ey, ez) of the all-air box [c, c + e*s] the primary
 * traversal jumps across: grown from the cube r (r_cube, from
 * vxo_field_octant) to the largest x extent, then y, then z, each <= cap - 1;
 * (0, 0, 0) for non-air cells.  3*X*Y*Z bytes into e_out, x fastest. */
void vxo_field_box(const uint8_t *rgba, int X, int Y, int Z, int cap, int oct, const uint8_t *r_cube,
                   uint8_t *e_out);
/* Sun exit table for sun octant oct (bit i: r_i > 0) and window (kx, ky) (< 0:
 * unbounded, the orthant table): out[c] = 1 marks a cell from which the march
 * cannot end unlit.  X*Y*Z bytes, x fastest; definition in vxo_field.c. */
void vxo_field_exit(const uint8_t *rgba, int X, int Y, int Z, int oct, int kx, int ky, uint8_t *out);
/* Which exit table a frame's sun march reads (the build's rule):
 * sample k of n (directions dirs[k]) uses table {oct[k], kx, ky}, or none
 * (oct[k] = -1: the literal path, some |r_i| < 2^-10).  Returns 1 when every
 * sample shares one cone table (kx, ky >= 0), else 0 (orthant tables, kx = ky
 * = -1).  allow_cone = 0 forces the orthant tables. */
int vxo_exit_plan(const float dirs[][3], int n, int allow_cone, int oct[], int *kx, int *ky);

#ifdef __cplusplus
}
#endif
#endif
