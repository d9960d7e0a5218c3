// Sliding-window evaluation on device: tile gather and overlap-averaged assembly.
//
// Reference: sliding_window_predict (utils/eval_utils.py:26-96): num_rows = ceil((H-wh)/sh)+1
// (same for columns), tile (i, j) starts at (i*sh, j*sw) and is snapped to the border when it would
// cross it; the density map is the per-pixel average of the overlapping tile predictions, placed at
// [start/r, end/r) with integer division by the model reduction r.
#include "ebc_common.h"

namespace {

__device__ __forceinline__ int tile_start(int i, int stride, int win, int full) {
    const int s = i * stride;
    return (s + win > full) ? full - win : s;
}

// tiles [T = rows*cols, C, wh, ww] <- image [C, H, W]
__global__ void tile_gather_kernel(const float* __restrict__ img, float* __restrict__ tiles, int C, int H, int W,
                                   int wh, int ww, int sh, int sw, int rows, int cols, int t0, int nt)
{
    const size_t per = (size_t)C * wh * ww;
    const size_t total = per * nt;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int t = (int)(e / per) + t0;
        const size_t r = e % per;
        const int x = (int)(r % ww), y = (int)((r / ww) % wh), c = (int)(r / ((size_t)ww * wh));
        const int i = t / cols, j = t % cols;
        const int ys = tile_start(i, sh, wh, H), xs = tile_start(j, sw, ww, W);
        tiles[e] = img[((size_t)c * H + ys + y) * W + xs + x];
    }
}

// out [Cp, H/r, W/r] = mean over covering tiles of preds [T, Cp, wh/r, ww/r]
__global__ void tile_assemble_kernel(const float* __restrict__ preds, float* __restrict__ out, int Cp, int H, int W,
                                     int wh, int ww, int sh, int sw, int rows, int cols, int r)
{
    const int Ho = H / r, Wo = W / r, ph = wh / r, pw = ww / r;
    const size_t total = (size_t)Cp * Ho * Wo;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(e % Wo), y = (int)((e / Wo) % Ho), c = (int)(e / ((size_t)Wo * Ho));
        float s = 0.f, n = 0.f;
        for (int i = 0; i < rows; ++i) {
            const int ys = tile_start(i, sh, wh, H) / r, ye = (tile_start(i, sh, wh, H) + wh) / r;
            if (y < ys || y >= ye) continue;
            for (int j = 0; j < cols; ++j) {
                const int xs = tile_start(j, sw, ww, W) / r, xe = (tile_start(j, sw, ww, W) + ww) / r;
                if (x < xs || x >= xe) continue;
                s += preds[(((size_t)(i * cols + j) * Cp + c) * ph + (y - ys)) * pw + (x - xs)];
                n += 1.f;
            }
        }
        out[e] = s / n;
    }
}

inline int grid_for(size_t n) {
    const size_t g = (n + 255) / 256;
    return (int)(g < 8192 ? (g ? g : 1) : 8192);
}

}  // namespace

extern "C" int ebc_tile_gather(const float* image, float* tiles, int C, int H, int W, int wh, int ww, int sh, int sw,
                               int tile_begin, int tile_count, ebc_stream_t stream)
{
    if (wh > H || ww > W || sh <= 0 || sw <= 0 || sh > wh || sw > ww) return EBC_E_ARG;
    const int rows = (H - wh + sh - 1) / sh + 1, cols = (W - ww + sw - 1) / sw + 1;
    if (tile_begin < 0 || tile_begin + tile_count > rows * cols) return EBC_E_ARG;
    if (tile_count == 0) return EBC_OK;
    const size_t n = (size_t)C * wh * ww * tile_count;
    hipLaunchKernelGGL(tile_gather_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, image, tiles, C, H, W,
                       wh, ww, sh, sw, rows, cols, tile_begin, tile_count);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}

extern "C" int ebc_tile_assemble(const float* preds, float* out, int Cp, int H, int W, int wh, int ww, int sh, int sw,
                                 int reduction, ebc_stream_t stream)
{
    if (wh > H || ww > W || sh <= 0 || sw <= 0 || sh > wh || sw > ww || reduction <= 0) return EBC_E_ARG;
    const int rows = (H - wh + sh - 1) / sh + 1, cols = (W - ww + sw - 1) / sw + 1;
    const size_t n = (size_t)Cp * (H / reduction) * (W / reduction);
    hipLaunchKernelGGL(tile_assemble_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, preds, out, Cp, H, W,
                       wh, ww, sh, sw, rows, cols, reduction);
    EBC_CHECK_LAUNCH();
    return EBC_OK;
}
