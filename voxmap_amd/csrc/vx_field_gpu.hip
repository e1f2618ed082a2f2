// vx_field_gpu.hip — map.bin distance field on the GPU (the
// C5 3^3-upscaled 3072x768x96 field has 226 M cells).
//
// Same definition as vx_field.cpp / oracle vxo_field.c (sdf.cpp:405-470):
//   * vol() = number of blocks of a box inside [1,X-1]x[1,Y-1]x[1,Z-1], read
//     from an inclusive prefix sum of bin' (blocks with x, y, z >= 1) through
//     clamped indices (the csum() clamp of sdf.cpp:36-42);
//   * per air cell and channel o (R: box [z, z+r], cap Z; G: box [z-r, z],
//     cap z) the radius r is searched from the diagonal neighbour's value
//     mid = sdf(max(x-1,0), max(y-1,0), max(z-1,0)) within [mid-1, mid+1]
//     (sdf.cpp:436-453); blocks keep 0.
// The reference sweeps x -> y -> z serially (voxmap.h:50-55).  For x >= 1 the
// neighbour lies in plane x - 1, so each plane is one launch of Y*Z
// independent cells, in order.  In plane 0 the neighbour (0, y-1, z-1) is in
// the same plane: cells with max(y, z) = s depend only on shell s - 1, so one
// workgroup walks the shells with a barrier between them.  Results equal the
// serial sweep exactly (integer arithmetic throughout).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vx_internal.h"

namespace vx {
namespace {

struct Grid {
    int X, Y, Z;
    __device__ size_t idx(int x, int y, int z) const {
        return (size_t)x + (size_t)X * ((size_t)y + (size_t)Y * (size_t)z);
    }
};

// inclusive prefix sum of bin' along x, one thread per (y, z) row
__global__ void k_scan_x(const uint8_t *col, int32_t *pre, Grid g) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= g.Y * g.Z) return;
    const int y = r % g.Y, z = r / g.Y;
    const size_t base = g.idx(0, y, z);
    int run = 0;
    const bool yz = y >= 1 && z >= 1;
    for (int x = 0; x < g.X; x++) {
        run += (yz && x >= 1 && col[base + x] != 0) ? 1 : 0;
        pre[base + x] = run;
    }
}
// along y (thread per (x, z)) and along z (thread per (x, y)): coalesced over x
__global__ void k_scan_y(int32_t *pre, Grid g) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)g.X * g.Z) return;
    const int x = (int)(t % g.X), z = (int)(t / g.X);
    int32_t acc = 0;
    for (int y = 0; y < g.Y; y++) {
        const size_t i = g.idx(x, y, z);
        acc += pre[i];
        pre[i] = acc;
    }
}
__global__ void k_scan_z(int32_t *pre, Grid g) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)g.X * g.Y) return;
    const size_t XY = (size_t)g.X * g.Y;
    int32_t acc = 0;
    for (int z = 0; z < g.Z; z++) {
        acc += pre[t + XY * z];
        pre[t + XY * z] = acc;
    }
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int P(const int32_t *pre, const Grid &g, int x, int y, int z) {
    return pre[g.idx(clampi(x, 0, g.X - 1), clampi(y, 0, g.Y - 1), clampi(z, 0, g.Z - 1))];
}

// vol() of sdf.cpp:63-83 over the clamped prefix sum
__device__ int vol(const int32_t *pre, const Grid &g, int x0, int y0, int z0, int x1, int y1, int z1) {
    x0--; y0--; z0--;
    return P(pre, g, x1, y1, z1) - P(pre, g, x0, y1, z1) - P(pre, g, x1, y0, z1) - P(pre, g, x1, y1, z0) +
           P(pre, g, x0, y0, z1) + P(pre, g, x0, y1, z0) + P(pre, g, x1, y0, z0) - P(pre, g, x0, y0, z0);
}

// both channels of one cell (sdf.cpp:430-455); sdf holds (R, G) per cell
__device__ void cell(const uint8_t *col, const int32_t *pre, uint8_t *sdf, const Grid &g, int x, int y, int z) {
    const size_t i = g.idx(x, y, z);
    if (col[i] != 0) return;   // blocks keep 0 (buffer zeroed)
    const size_t nb = g.idx(x > 0 ? x - 1 : 0, y > 0 ? y - 1 : 0, z > 0 ? z - 1 : 0);
    for (int o = 0; o < 2; o++) {
        int mn = 1, mx = o == 0 ? g.Z : z;
        if (x + y + z > 0) {
            const int mid = sdf[2 * nb + o];
            mn = mn > mid - 1 ? mn : mid - 1;
            mx = mx < mid + 1 ? mx : mid + 1;
        }
        int r = mn;
        while (r < mx && vol(pre, g, x - r, y - r, z - o * r, x + r, y + r, z + (1 - o) * r) == 0) r++;
        sdf[2 * i + o] = (uint8_t)r;
    }
}

// plane 0: shells s = max(y, z) in order, one workgroup, barrier between shells
__global__ __launch_bounds__(1024) void k_plane0(const uint8_t *col, const int32_t *pre, uint8_t *sdf, Grid g) {
    const int S = g.Y > g.Z ? g.Y : g.Z;
    for (int s = 0; s < S; s++) {
        // shell cells: (y = s, z = 0..min(s, Z-1)) if s < Y, then (z = s, y = 0..s-1) if s < Z
        const int na = s < g.Y ? (s < g.Z - 1 ? s : g.Z - 1) + 1 : 0;
        const int nbk = s < g.Z ? (s < g.Y ? s : g.Y) : 0;
        for (int k = threadIdx.x; k < na + nbk; k += blockDim.x) {
            if (k < na) cell(col, pre, sdf, g, 0, s, k);
            else cell(col, pre, sdf, g, 0, k - na, s);
        }
        __syncthreads();   // orders this shell's stores before the next shell's loads (one workgroup)
    }
}

// plane x >= 1: Y*Z independent cells
__global__ void k_plane(const uint8_t *col, const int32_t *pre, uint8_t *sdf, Grid g, int x) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= g.Y * g.Z) return;
    cell(col, pre, sdf, g, x, k / g.Z, k % g.Z);   // (y, z) order of the host sweep; any order is exact
}

// map.bin texels: R = up, G = down, B = remapped palette index (air ->
// pal_size, sdf.cpp:229-233), A = 0 (sdf.cpp:462-470)
__global__ void k_texels(const uint8_t *col, const uint8_t *sdf, uint32_t *rgba, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint32_t b = col[i] ? (uint32_t)col[i] : (uint32_t)VX_PAL_SIZE;
    rgba[i] = (uint32_t)sdf[2 * i] | ((uint32_t)sdf[2 * i + 1] << 8) | (b << 16);
}

}  // namespace

int field_build_device(const uint8_t *d_col, uint32_t *d_rgba, int X, int Y, int Z, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)X * Y * Z;
    Grid g{X, Y, Z};
    int32_t *pre = nullptr;
    uint8_t *sdf = nullptr;
    hipError_t e = hipMalloc(&pre, N * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&sdf, 2 * N);
    if (e == hipSuccess) e = hipMemsetAsync(sdf, 0, 2 * N, s);
    if (e == hipSuccess) {
        const int rows = Y * Z;
        hipLaunchKernelGGL(k_scan_x, dim3((rows + 255) / 256), dim3(256), 0, s, d_col, pre, g);
        hipLaunchKernelGGL(k_scan_y, dim3((unsigned)(((size_t)X * Z + 255) / 256)), dim3(256), 0, s, pre, g);
        hipLaunchKernelGGL(k_scan_z, dim3((unsigned)(((size_t)X * Y + 255) / 256)), dim3(256), 0, s, pre, g);
        hipLaunchKernelGGL(k_plane0, dim3(1), dim3(1024), 0, s, d_col, pre, sdf, g);
        for (int x = 1; x < X; x++)
            hipLaunchKernelGGL(k_plane, dim3((rows + 255) / 256), dim3(256), 0, s, d_col, pre, sdf, g, x);
        hipLaunchKernelGGL(k_texels, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, d_col, sdf, d_rgba, N);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    if (pre) (void)hipFree(pre);
    if (sdf) (void)hipFree(sdf);
    return (int)e;
}

}  // namespace vx
