// vx_render_e1.hip — the render kernel's EXT 1 instantiations (REFLECT / ROUGH with the hard shadow),
// a translation unit of their own (vx_render.h).
#include "vx_render.h"

namespace vx {
int launch_render_e1(const KernelArgs &a, int fmt, unsigned gx, unsigned gy, void *stream) {
    return launch_render_ext<1>(a, fmt, gx, gy, stream);
}
}  // namespace vx
