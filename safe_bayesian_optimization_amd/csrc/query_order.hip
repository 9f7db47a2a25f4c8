// query_order.hip -- spatial (Morton) ordering of the query points of a tick.
//
// The predictive sweep skips a k-tile for a workgroup when the tile's
// training points are far from ALL of the workgroup's 128 queries, so the
// work depends on how compact each block of 128 queries is.  Callers pass
// arbitrary query order (a row-major terrain grid gives 1 x 128 strips); the
// tick therefore sorts the queries by a 32-bit Morton code (16 bits per axis
// over the training bounding box, clamped), sweeps them in that order, and
// the acquisition kernel scatters every output back to the caller's index
// (argmax ties still resolve to the lowest caller index).
//
// Raster grids (the node's terrain grid, or a contiguous shard of its rows)
// get blocks that are whole grid patches instead: 8 points along the fast
// axis x 16 rows, patches in raster order, the last R % 16 rows in patches
// of the next power-of-two height (as wide as it takes for 128), partial
// patches padded (a padded sweep position repeats the nearest grid point of
// its column and carries perm = -1, so no output is written for it).  Morton blocks of a grid whose side is not
// a power of two are L-shaped or split; at C4 (1000^2) their boxes average
// 3.2x the patches' area, and the patch blocks keep 6 % fewer k-tiles.  The
// layout is a function of (m, W, c0) alone -- any data gets a valid
// permutation -- so the detection (grid_*_kernel, one host read) is cached
// by the caller per query buffer.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

__device__ __forceinline__ uint32_t spread16(uint32_t v) {
    v &= 0xFFFFu;
    v = (v | (v << 8)) & 0x00FF00FFu;
    v = (v | (v << 4)) & 0x0F0F0F0Fu;
    v = (v | (v << 2)) & 0x33333333u;
    v = (v | (v << 1)) & 0x55555555u;
    return v;
}

__global__ void morton_kernel(const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, float x0,
                              float sx, float y0, float sy, uint32_t *__restrict__ code, int32_t *__restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    float u = (qx[i] - x0) * sx, v = (qy[i] - y0) * sy;
    u = fminf(fmaxf(u, 0.0f), 65535.0f);  // NaN -> 0
    v = fminf(fmaxf(v, 0.0f), 65535.0f);
    code[i] = spread16((uint32_t)u) | (spread16((uint32_t)v) << 1);
    idx[i] = (int32_t)i;
}

__global__ void gather_kernel(const float *__restrict__ qx, const float *__restrict__ qy,
                              const int32_t *__restrict__ perm, int64_t m, float *__restrict__ sx,
                              float *__restrict__ sy) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int32_t p = perm[i];
    sx[i] = qx[p];
    sy[i] = qy[p];
}

// Grid detection, both orientations (o = 0: y is the slow axis, rows of
// constant y; o = 1: x).  g[3 o + 0] = j1 = the first index whose slow
// coordinate differs from point 0's, g[3 o + 1] = j2 = the first one after j1
// differing from point j1's (so W = j2 - j1 points per row, the first row
// holding j1 of them), g[3 o + 2] != 0: the points are not that raster.
__global__ void grid_j1_kernel(const float *__restrict__ qx, const float *__restrict__ qy, int64_t m,
                               unsigned long long *__restrict__ g) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    if (qy[i] != qy[0]) atomicMin(g + 0, (unsigned long long)i);
    if (qx[i] != qx[0]) atomicMin(g + 3, (unsigned long long)i);
}
__global__ void grid_j2_kernel(const float *__restrict__ qx, const float *__restrict__ qy, int64_t m,
                               unsigned long long *__restrict__ g) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const unsigned long long a = g[0], b = g[3];
    if ((unsigned long long)i > a && a < (unsigned long long)m && qy[i] != qy[a]) atomicMin(g + 1, (unsigned long long)i);
    if ((unsigned long long)i > b && b < (unsigned long long)m && qx[i] != qx[b]) atomicMin(g + 4, (unsigned long long)i);
}
// point i of a raster with W per row whose first row starts at column c0:
// row r = (c0 + i) / W starts at max(0, r W - c0) and has the slow value of
// that point; its column c = (c0 + i) % W has the fast value of point j1 + c
// (row 1, a whole row)
__global__ void grid_check_kernel(const float *__restrict__ qx, const float *__restrict__ qy, int64_t m,
                                  unsigned long long *__restrict__ g) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        const unsigned long long j1 = g[3 * o], j2 = g[3 * o + 1];
        if (j2 >= (unsigned long long)m || j2 - j1 < j1) continue;  // no whole second row: not a raster
        const int64_t W = (int64_t)(j2 - j1), c0 = W - (int64_t)j1;
        const float *slow = o ? qx : qy, *fast = o ? qy : qx;
        const int64_t r = (c0 + i) / W, c = (c0 + i) % W;
        const int64_t rs = r * W - c0 > 0 ? r * W - c0 : 0;
        if (slow[i] != slow[rs] || fast[i] != fast[(int64_t)j1 + c]) g[3 * o + 2] = 1;
    }
}

// Sweep position p of the patch layout (see launch_query_grid) -> caller index (or -1) and coordinates.
__global__ void grid_gather_kernel(const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, QueryGrid q,
                                   int32_t *__restrict__ perm, float *__restrict__ sx, float *__restrict__ sy) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= q.ms) return;
    const int64_t W = q.W, c0 = q.c0, R = q.R;
    const int64_t patch = p / kBN, l = p % kBN, nfp = q.nfull * q.npf;
    // whole patch rows, then the last rows (R % kGridPatchSlow of them) in
    // patches q.wl wide and kBN / q.wl tall
    const int64_t cf = patch < nfp ? (patch % q.npf) * kGridPatchFast + l % kGridPatchFast
                                   : (patch - nfp) * q.wl + l % q.wl;
    const int64_t rs = patch < nfp ? (patch / q.npf) * kGridPatchSlow + l / kGridPatchFast
                                   : q.nfull * kGridPatchSlow + l / q.wl;
    const int64_t i = rs * W + cf - c0;
    const bool valid = cf < W && rs < R && i >= 0 && i < m;
    // a padded position repeats the nearest grid point of its own column
    // (the next row before the first row's start c0, the previous row past
    // the last row's end), so the patch's box stays the patch's
    int64_t src = (rs < R ? rs : R - 1) * W + (cf < W ? cf : W - 1) - c0;
    if (src < 0) src += W;
    if (src >= m) src -= W;
    src = src < 0 ? 0 : (src >= m ? m - 1 : src);
    perm[p] = valid ? (int32_t)i : -1;
    sx[p] = qx[src];
    sy[p] = qy[src];
}

}  // namespace

size_t query_grid_bytes(int64_t m) {
    // g[6] + perm + coordinates for up to grid_max_positions(m) sweep positions
    const size_t a = (size_t)grid_max_positions(m);
    return 256 + 4 * a + 2 * 4 * a;
}

hipError_t launch_grid_detect(hipStream_t s, const float *qx, const float *qy, int64_t m, void *work,
                              unsigned long long host_g[6]) {
    auto *g = static_cast<unsigned long long *>(work);
    const unsigned long long init[6] = {~0ull, ~0ull, 0ull, ~0ull, ~0ull, 0ull};
    hipError_t e = hipMemcpyAsync(g, init, sizeof(init), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    const unsigned nb = (unsigned)((m + 255) / 256);
    hipLaunchKernelGGL(grid_j1_kernel, dim3(nb), dim3(256), 0, s, qx, qy, m, g);
    hipLaunchKernelGGL(grid_j2_kernel, dim3(nb), dim3(256), 0, s, qx, qy, m, g);
    hipLaunchKernelGGL(grid_check_kernel, dim3(nb), dim3(256), 0, s, qx, qy, m, g);
    e = hipMemcpyAsync(host_g, g, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

bool grid_layout(const unsigned long long g[6], int64_t m, QueryGrid &q) {
    q = QueryGrid{};
    for (int o = 0; o < 2; ++o) {
        const unsigned long long j1 = g[3 * o], j2 = g[3 * o + 1];
        if (g[3 * o + 2] || j2 >= (unsigned long long)m || j2 - j1 < j1) continue;
        const int64_t W = (int64_t)(j2 - j1), c0 = W - (int64_t)j1;
        const int64_t R = (c0 + m + W - 1) / W;
        const int64_t npf = (W + kGridPatchFast - 1) / kGridPatchFast, nfull = R / kGridPatchSlow;
        // the last R % kGridPatchSlow rows: patches of the next power-of-two height
        const int64_t h = R % kGridPatchSlow;
        int64_t hp = 1;
        while (hp < h) hp <<= 1;
        const int64_t wl = h ? kBN / hp : kBN, npl = h ? (W + wl - 1) / wl : 0;
        const int64_t ms = (nfull * npf + npl) * kBN;
        if (W < kGridPatchFast || ms > grid_max_positions(m)) continue;  // too much padding: Morton instead
        q = QueryGrid{true, W, c0, R, npf, ms, nfull, wl};
        return true;
    }
    return false;
}

hipError_t launch_query_grid(hipStream_t s, const float *qx, const float *qy, int64_t m, const QueryGrid &q,
                             void *work, int32_t **perm_out, float **sqx, float **sqy) {
    char *p = static_cast<char *>(work) + 256;
    const size_t a = (size_t)grid_max_positions(m);
    int32_t *perm = reinterpret_cast<int32_t *>(p);
    float *xs = reinterpret_cast<float *>(perm + a);
    float *ys = xs + a;
    hipLaunchKernelGGL(grid_gather_kernel, dim3((unsigned)((q.ms + 255) / 256)), dim3(256), 0, s, qx, qy, m, q, perm,
                       xs, ys);
    *perm_out = perm;
    *sqx = xs;
    *sqy = ys;
    return hipGetLastError();
}

size_t query_order_bytes(int64_t m) {
    size_t temp = 0;
    (void)rocprim::radix_sort_pairs(nullptr, temp, (uint32_t *)nullptr, (uint32_t *)nullptr, (int32_t *)nullptr,
                              (int32_t *)nullptr, (size_t)m, 0, 32, nullptr);
    const size_t a = (size_t)round_up(m, kBN);  // gathered coordinates padded to whole query blocks
    return 4 * a * 4 + 2 * a * 4 + round_up((int64_t)temp, 256);
}

hipError_t launch_query_order(hipStream_t s, const float *qx, const float *qy, int64_t m, const float bbox[4],
                              void *work, size_t work_bytes, int32_t **perm_out, float **sqx, float **sqy) {
    const size_t a = (size_t)round_up(m, kBN);  // gathered coordinates padded to whole query blocks
    char *p = static_cast<char *>(work);
    uint32_t *code_in = reinterpret_cast<uint32_t *>(p);
    uint32_t *code_out = code_in + a;
    int32_t *idx_in = reinterpret_cast<int32_t *>(code_out + a);
    int32_t *idx_out = idx_in + a;
    float *xs = reinterpret_cast<float *>(idx_out + a);
    float *ys = xs + a;
    void *temp = ys + a;
    size_t temp_bytes = work_bytes - (size_t)(static_cast<char *>(temp) - p);
    const float x0 = bbox[0], y0 = bbox[2];
    const float sx = bbox[1] > bbox[0] ? 65535.0f / (bbox[1] - bbox[0]) : 0.0f;
    const float sy = bbox[3] > bbox[2] ? 65535.0f / (bbox[3] - bbox[2]) : 0.0f;
    const unsigned g = (unsigned)((m + 255) / 256);
    hipLaunchKernelGGL(morton_kernel, dim3(g), dim3(256), 0, s, qx, qy, m, x0, sx, y0, sy, code_in, idx_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(temp, temp_bytes, code_in, code_out, idx_in, idx_out, (size_t)m, 0, 32, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gather_kernel, dim3(g), dim3(256), 0, s, qx, qy, idx_out, m, xs, ys);
    *perm_out = idx_out;
    *sqx = xs;
    *sqy = ys;
    return hipGetLastError();
}

}  // namespace sbo
