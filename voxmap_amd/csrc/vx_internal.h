// vx_internal.h — shared between the C-ABI host code and the HIP kernels.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string>
#include "../../include/voxmap.h"

namespace vx {

// Error plumbing: every C entry point returns a VX_E* code and leaves a
// message in a thread-local buffer (vx_last_error).
int set_error(int code, const std::string &msg);

// Parameters of one render launch (passed by value to the kernel).
struct KernelArgs {
    const uint32_t *field;   // RGBA8 texels, x fastest (render.js:62)
    const uint32_t *noise;   // RGBA8 noise texels
    int X, Y, Z;
    int noise_w, noise_h;    // powers of two
    int w, h;                // frame size
    int tile_size;           // tiled mode: tile edge in pixels (multiple of 16)
    int tiles_x;             // ceil(w / tile_size)
    const int *tile_ids;     // tiled mode: device list of tile ids, else nullptr
    int n_tiles;
    void *out;               // RGBA32F or RGBA8
    unsigned long long *stats;   // device counters (nullptr = no stats)
    vx_frame_params p;
    int max_shadow_steps;
};

enum StatSlot {
    ST_PIXELS = 0, ST_SKY, ST_BLOCK, ST_GLASS, ST_PRIM_FETCH, ST_SHADOW_RAYS, ST_SHADOW_FETCH,
    ST_AO, ST_NOISE_PX, ST_CAP_HITS, ST_COUNT
};

// Launchers (vx_kernels.hip).  Return a hipError_t as int.
int launch_render(const KernelArgs &a, int pixel_format, void *stream);
int launch_detile(const void *tiles, void *frame, int w, int h, int tile_size, int tiles_x,
                  const int *tile_ids, int n_tiles, int pixel_format, void *stream);
int launch_field_dist(uint32_t *field, int X, int Y, int Z, int cap, uint8_t *scratch_a,
                      uint8_t *scratch_b, void *stream);

}  // namespace vx
