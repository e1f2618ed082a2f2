// vx_render_e3.hip — the render kernel's EXT 3 instantiations (soft shadows, pooled wave pass: VX_FLAG_SOFT_POOL),
// a translation unit of their own (vx_render.h).
#include "vx_render.h"

namespace vx {
int launch_render_e3(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    return launch_render_ext<3>(a, fmt, gx, gy, stream);
}
}  // namespace vx
