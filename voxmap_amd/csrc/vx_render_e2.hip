// vx_render_e2.hip — the render kernel's EXT 2 instantiations (soft shadows),
// a translation unit of their own (vx_render.h).
#include "vx_render.h"

namespace vx {
int launch_render_e2(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    return launch_render_ext<2>(a, fmt, gx, gy, stream);
}
}  // namespace vx
