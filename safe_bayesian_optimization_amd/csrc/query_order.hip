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

}  // namespace

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
