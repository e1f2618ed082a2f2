// vx_render_e56.hip — the render kernel's general shading modes, EXT 5 / 6
// (glass in draw order over the whole frame, REFLECT_ALL; hard / soft
// shadows), a translation unit of their own with a register budget of their
// own: 5 waves/SIMD (96 VGPRs).  Their loop over a pixel's panes and mirror
// walks spills heavily at the 8-wave budget of the other modes;
// the template is the same text, so EXT 0-4 keep their code generation.
#define VX_OCC_ATTR __attribute__((amdgpu_waves_per_eu(5, 5)))
#include "vx_render.h"

namespace vx {
int launch_render_e56(int ext, const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    return ext == 6 ? launch_render_ext<6>(a, fmt, gx, gy, stream) : launch_render_ext<5>(a, fmt, gx, gy, stream);
}
}  // namespace vx
