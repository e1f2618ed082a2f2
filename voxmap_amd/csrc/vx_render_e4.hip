// vx_render_e4.hip — the render kernel's EXT 4 instantiations (soft shadows, LDS bricks: VX_FLAG_SOFT_BRICK),
// a translation unit of their own (vx_render.h).
#include "vx_render.h"

namespace vx {
int launch_render_e4(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    return launch_render_ext<4>(a, fmt, gx, gy, stream);
}
}  // namespace vx
