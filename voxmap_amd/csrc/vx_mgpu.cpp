// vx_mgpu.cpp — one frame shared by the GPUs of a node, RCCL
// over xGMI, no PyTorch: the C++ host (vxrender --ranks N) and any other
// caller of the C ABI can shard a frame with it.
//
// The reference draws one frame per drawScene() (render.js:267-298); every
// pixel is independent (render.frag reads only the replicated u_map / u_noise
// textures), so the frame is cut into full-width bands of band_rows rows,
// dealt round-robin (band b -> rank b % nranks: neighbouring bands cost about
// the same, so the interleave balances sky against geometry).  Every rank
// renders its bands IN PLACE in its own w x h framebuffer (vx_render_bands,
// inplace = 1), then one RCCL group moves them to rank 0: rank r sends each of
// its bands from its frame rows, rank 0 receives each into the same rows of
// its frame.  A band is contiguous in a row-major frame, so the gather lands
// directly in the final image: no tile-major staging, no de-tile pass, no
// extra copy.  All of it is stream-ordered on the caller's stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "vx_internal.h"

static_assert(sizeof(ncclUniqueId) == VX_MGPU_UID_BYTES, "ncclUniqueId size");

struct vx_mgpu {
    vx_scene *scene = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    int h = -1, band_rows = -1;          // the cached deal
    std::vector<int> mine;
};

using namespace vx;

#define VX_NCCL(call)                                                                                 \
    do {                                                                                              \
        ncclResult_t r_ = (call);                                                                     \
        if (r_ != ncclSuccess)                                                                        \
            return set_error(VX_EDEVICE, std::string(#call " failed: ") + ncclGetErrorString(r_));    \
    } while (0)

extern "C" {

int vx_mgpu_unique_id(void *uid) {
    if (!uid) return set_error(VX_EINVAL, "vx_mgpu_unique_id: null argument");
    ncclUniqueId id;
    VX_NCCL(ncclGetUniqueId(&id));
    std::memcpy(uid, &id, sizeof id);
    return VX_OK;
}

int vx_mgpu_create(vx_scene *scene, const void *uid, int nranks, int rank, vx_mgpu **out) {
    if (!scene || !uid || !out || nranks <= 0 || rank < 0 || rank >= nranks)
        return set_error(VX_EINVAL, "vx_mgpu_create: bad arguments");
    *out = nullptr;
    const int dev = scene_device(scene);
    if (hipSetDevice(dev) != hipSuccess) return set_error(VX_EDEVICE, "vx_mgpu_create: hipSetDevice failed");
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    ncclComm_t comm = nullptr;
    VX_NCCL(ncclCommInitRank(&comm, nranks, id, rank));
    vx_mgpu *m = new vx_mgpu();
    m->scene = scene;
    m->comm = comm;
    m->nranks = nranks;
    m->rank = rank;
    m->device = dev;
    *out = m;
    return VX_OK;
}

void vx_mgpu_destroy(vx_mgpu *m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->comm) (void)ncclCommDestroy(m->comm);
    delete m;
}

int vx_mgpu_render(vx_mgpu *m, const vx_frame_params *p, int w, int h, int band_rows, int pixel_format,
                   void *frame_device, void *stream, vx_stats *stats) {
    if (!m || !p || !frame_device) return set_error(VX_EINVAL, "vx_mgpu_render: null argument");
    if (band_rows <= 0 || band_rows % VX_TILE_ALIGN_Y)
        return set_error(VX_EINVAL, "vx_mgpu_render: band_rows must be a positive multiple of 8");
    if (h <= 0 || w <= 0) return set_error(VX_EINVAL, "vx_mgpu_render: frame size out of range");
    if (pixel_format != VX_PIXEL_RGBA8 && pixel_format != VX_PIXEL_RGBA32F)
        return set_error(VX_EINVAL, "vx_mgpu_render: unknown pixel format");
    if (m->h != h || m->band_rows != band_rows) {
        const int n = vx_mgpu_bands(h, band_rows, m->nranks, m->rank, nullptr, 0);
        m->mine.resize(n > 0 ? n : 0);
        if (n > 0) vx_mgpu_bands(h, band_rows, m->nranks, m->rank, m->mine.data(), n);
        m->h = h;
        m->band_rows = band_rows;
    }
    if (hipSetDevice(m->device) != hipSuccess) return set_error(VX_EDEVICE, "vx_mgpu_render: hipSetDevice failed");
    // one stream for the render and the gather: NULL means the scene's own
    // stream (non-blocking), which the legacy null stream would not wait for
    if (!stream) stream = scene_stream(m->scene);
    if (!m->mine.empty()) {
        const int rc = vx_render_bands(m->scene, p, w, h, band_rows, m->mine.data(), (int)m->mine.size(),
                                       pixel_format, frame_device, 1, stream, stats);
        if (rc) return rc;
    } else if (stats) {
        std::memset(stats, 0, sizeof *stats);
    }
    return vx_mgpu_gather(m, w, h, band_rows, pixel_format, frame_device, stream);
}

int vx_mgpu_gather(vx_mgpu *m, int w, int h, int band_rows, int pixel_format, void *frame_device, void *stream) {
    if (!m || !frame_device) return set_error(VX_EINVAL, "vx_mgpu_gather: null argument");
    if (band_rows <= 0 || band_rows % VX_TILE_ALIGN_Y)
        return set_error(VX_EINVAL, "vx_mgpu_gather: band_rows must be a positive multiple of 8");
    if (h <= 0 || w <= 0) return set_error(VX_EINVAL, "vx_mgpu_gather: frame size out of range");
    if (pixel_format != VX_PIXEL_RGBA8 && pixel_format != VX_PIXEL_RGBA32F)
        return set_error(VX_EINVAL, "vx_mgpu_gather: unknown pixel format");
    if (m->nranks == 1) return VX_OK;
    if (hipSetDevice(m->device) != hipSuccess) return set_error(VX_EDEVICE, "vx_mgpu_gather: hipSetDevice failed");
    hipStream_t st = (hipStream_t)(stream ? stream : scene_stream(m->scene));
    // the gather: every band not rank 0's goes from its owner's frame rows to rank 0's
    const int n = vx_mgpu_transfers(w, h, band_rows, pixel_format, m->nranks, m->rank, nullptr, 0);
    std::vector<vx_mgpu_xfer> xs(n > 0 ? n : 0);
    if (n > 0) vx_mgpu_transfers(w, h, band_rows, pixel_format, m->nranks, m->rank, xs.data(), n);
    char *frame = static_cast<char *>(frame_device);
    VX_NCCL(ncclGroupStart());
    for (const vx_mgpu_xfer &x : xs) {
        const ncclResult_t r = m->rank == 0 ? ncclRecv(frame + x.offset, x.bytes, ncclUint8, x.src, m->comm, st)
                                            : ncclSend(frame + x.offset, x.bytes, ncclUint8, x.dst, m->comm, st);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return set_error(VX_EDEVICE, std::string(m->rank == 0 ? "ncclRecv" : "ncclSend") + " failed: " +
                                             ncclGetErrorString(r));
        }
    }
    VX_NCCL(ncclGroupEnd());
    return VX_OK;
}

int vx_mgpu_rank(const vx_mgpu *m, int *nranks, int *rank) {
    if (!m) return set_error(VX_EINVAL, "vx_mgpu_rank: null argument");
    if (nranks) *nranks = m->nranks;
    if (rank) *rank = m->rank;
    return VX_OK;
}

}  // extern "C"
