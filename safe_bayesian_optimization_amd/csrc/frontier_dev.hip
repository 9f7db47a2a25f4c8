// frontier_dev.hip -- device raster of the node's frontier extraction
// (src/safe_bayesian_optimization_node.cpp:418-497).
//
// The O(M) part of FindSafetyContourIndices -- bounds, the per-point pixel
// arithmetic and the last-writer-wins maps (:425-475) -- runs on the grid
// where the tick left it; the host only follows the borders of the
// width x height image (Suzuki-Abe, frontier.cpp) and never sees the M
// points.  Arithmetic is the node's IEEE double sequence (-ffp-contract=off,
// correctly rounded f64 division), so pixels are bit-identical to the host
// restatement.
#include <climits>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

constexpr int kRasterThreads = 256;
constexpr int kMinMaxBlocks = 512;

// static_cast<int>(double) as the node's x86-64 build executes it
// (cvttsd2si): NaN and out-of-range values become INT_MIN.
__device__ __forceinline__ int trunc_to_int(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
    return (int)v;
}

__device__ __forceinline__ void block_minmax4(double (&v)[4]) {
    __shared__ double sh[4][kRasterThreads / 64];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        v[0] = fmin(v[0], __shfl_xor(v[0], o));
        v[1] = fmax(v[1], __shfl_xor(v[1], o));
        v[2] = fmin(v[2], __shfl_xor(v[2], o));
        v[3] = fmax(v[3], __shfl_xor(v[3], o));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int c = 0; c < 4; ++c) sh[c][w] = v[c];
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 1; k < kRasterThreads / 64; ++k) {
            v[0] = fmin(v[0], sh[0][k]);
            v[1] = fmax(v[1], sh[1][k]);
            v[2] = fmin(v[2], sh[2][k]);
            v[3] = fmax(v[3], sh[3][k]);
        }
}

// part[b] = (min x, max x, min y, max y) over a grid-stride slice
__global__ __launch_bounds__(kRasterThreads) void minmax_kernel(const double *__restrict__ Dx,
                                                                const double *__restrict__ Dy, int64_t m,
                                                                double *__restrict__ part) {
    double v[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const double x = Dx[i], y = Dy[i];
        v[0] = fmin(v[0], x); v[1] = fmax(v[1], x);
        v[2] = fmin(v[2], y); v[3] = fmax(v[3], y);
    }
    block_minmax4(v);
    if (threadIdx.x == 0)
        for (int c = 0; c < 4; ++c) part[blockIdx.x * 4 + c] = v[c];
}

// bounds = (min_x, min_y, span_x, span_y) with the node's int truncation (:431-434)
__global__ __launch_bounds__(kRasterThreads) void bounds_kernel(const double *__restrict__ part, int nb,
                                                                double *__restrict__ bounds) {
    double v[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        v[0] = fmin(v[0], part[b * 4 + 0]); v[1] = fmax(v[1], part[b * 4 + 1]);
        v[2] = fmin(v[2], part[b * 4 + 2]); v[3] = fmax(v[3], part[b * 4 + 3]);
    }
    block_minmax4(v);
    if (threadIdx.x == 0) {
        const int min_x = trunc_to_int(v[0]), max_x = trunc_to_int(v[1]);
        const int min_y = trunc_to_int(v[2]), max_y = trunc_to_int(v[3]);
        bounds[0] = (double)min_x;
        bounds[1] = (double)min_y;
        bounds[2] = (double)(int)((unsigned)max_x - (unsigned)min_x);  // the node's int difference
        bounds[3] = (double)(int)((unsigned)max_y - (unsigned)min_y);
    }
}

// pixel of every grid point; last writer (highest index) wins (:450-475)
__global__ __launch_bounds__(kRasterThreads) void raster_kernel(const double *__restrict__ Dx,
                                                                const double *__restrict__ Dy, int64_t m,
                                                                const double *__restrict__ bounds, int width,
                                                                int height, int32_t *__restrict__ owner) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double min_x = bounds[0], min_y = bounds[1], span_x = bounds[2], span_y = bounds[3];
    // scaled by width / height (not width-1): D == max maps past the image and is dropped (:450-453)
    const int x = trunc_to_int((Dx[i] - min_x) / span_x * (double)width);
    const int y = trunc_to_int((Dy[i] - min_y) / span_y * (double)height);
    if (x >= 0 && x < width && y >= 0 && y < height) atomicMax(owner + (int64_t)y * width + x, (int32_t)i);
}

// owner[k] keeps its point only when that point is safe (the pixel is
// foreground); img[k] = 1 for foreground pixels
__global__ __launch_bounds__(kRasterThreads) void safe_owner_kernel(int32_t *__restrict__ owner,
                                                                    const uint8_t *__restrict__ safe, int64_t npx,
                                                                    uint8_t *__restrict__ img) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npx) return;
    int32_t o = owner[k];
    if (o >= 0 && !safe[o]) {
        o = -1;
        owner[k] = -1;
    }
    img[k] = o >= 0 ? 1 : 0;
}

// F[i] = owner[pix[i]]; with lo (and Dx, Dy, hi) given, out = the four
// gathered columns (nf each)
__global__ __launch_bounds__(kRasterThreads) void gather_kernel(const int32_t *__restrict__ pix, int64_t nf,
                                                                const int32_t *__restrict__ owner,
                                                                const double *__restrict__ Dx,
                                                                const double *__restrict__ Dy,
                                                                const double *__restrict__ lo,
                                                                const double *__restrict__ hi,
                                                                int32_t *__restrict__ F, double *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const int32_t f = owner[pix[i]];
    F[i] = f;
    if (lo && f >= 0) {
        out[i] = Dx[f];
        out[nf + i] = Dy[f];
        out[2 * nf + i] = lo[f];
        out[3 * nf + i] = hi[f];
    }
}

}  // namespace

size_t frontier_work_bytes(int64_t) { return sizeof(double) * (kMinMaxBlocks * 4 + 4); }

hipError_t launch_frontier_raster(hipStream_t s, const double *Dx, const double *Dy, const uint8_t *safe, int64_t m,
                                  int width, int height, void *work, int32_t *owner, uint8_t *img) {
    double *part = static_cast<double *>(work);
    double *bounds = part + kMinMaxBlocks * 4;
    const int64_t npx = (int64_t)width * height;
    hipError_t e = hipMemsetAsync(owner, 0xFF, sizeof(int32_t) * (size_t)npx, s);  // -1
    if (e != hipSuccess) return e;
    const int nb = (int)std::min<int64_t>(kMinMaxBlocks, (m + kRasterThreads - 1) / kRasterThreads);
    hipLaunchKernelGGL(minmax_kernel, dim3(nb), dim3(kRasterThreads), 0, s, Dx, Dy, m, part);
    hipLaunchKernelGGL(bounds_kernel, dim3(1), dim3(kRasterThreads), 0, s, part, nb, bounds);
    hipLaunchKernelGGL(raster_kernel, dim3((unsigned)((m + kRasterThreads - 1) / kRasterThreads)), dim3(kRasterThreads),
                       0, s, Dx, Dy, m, bounds, width, height, owner);
    hipLaunchKernelGGL(safe_owner_kernel, dim3((unsigned)((npx + kRasterThreads - 1) / kRasterThreads)),
                       dim3(kRasterThreads), 0, s, owner, safe, npx, img);
    return hipGetLastError();
}

hipError_t launch_frontier_gather(hipStream_t s, const int32_t *pix, int64_t nf, const int32_t *owner,
                                  const double *Dx, const double *Dy, const double *lo, const double *hi, int32_t *F,
                                  double *out) {
    if (nf <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_kernel, dim3((unsigned)((nf + kRasterThreads - 1) / kRasterThreads)),
                       dim3(kRasterThreads), 0, s, pix, nf, owner, Dx, Dy, lo, hi, F, out);
    return hipGetLastError();
}

}  // namespace sbo
