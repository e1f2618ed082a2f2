// vx_render_e0.hip — the render kernel's EXT 0 instantiations (the reference's shader, v1),
// a translation unit of their own (vx_render.h).
#include "vx_render.h"

namespace vx {
int launch_render_e0(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    return launch_render_ext<0>(a, fmt, gx, gy, stream);
}
}  // namespace vx
