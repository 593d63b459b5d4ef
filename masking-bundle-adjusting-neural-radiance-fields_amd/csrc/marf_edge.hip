// marf_edge.hip -- edge maps and mask erosion on the GPU.
//
// inputs.compute_edges (reference inputs.py:50-67) runs per image on the host through cv2:
// Sobel 3x3 (CV_64F) in x and y, magnitude, GaussianBlur 5x5 with sigma 0, BORDER_REFLECT_101.
// The reference copies every rendered patch D2H for it at each logging step (model/planar.py:336);
// here one launch covers all B x C channel images in place on the device.
//
// One block = a 16 x 16 output tile of one channel image.  Stage 1: the Sobel magnitude on the
// 20 x 20 window the 5x5 blur needs, each at its reflect-101 coordinate (equal to cv2's blur border,
// because reflect-101 commutes with the symmetric / antisymmetric 3-tap Sobel kernels); the fp32
// inputs are read straight from global (L1/L2 serve the 3x3 reuse).  Stage 2: row pass of the
// blur into LDS, stage 3: column pass to the output.  fp64 throughout; the Sobel sums of fp32
// values are exact in fp64, the blur accumulates left to right like oracle.edge_map.
// Bound: latency / tiny (runs at logging steps only): 4 B in + 8 B out per pixel.
#include "marf_args.h"

namespace marf {

MARF_DEV int refl101(int p, int n) {
    if (n == 1) return 0;
    const int period = 2 * n - 2;
    p = p < 0 ? -p : p;
    p %= period;
    return p >= n ? period - p : p;
}

__global__ __launch_bounds__(256) void k_edge_map(const float* __restrict__ in, double* __restrict__ out, int H, int W) {
    constexpr int T = 16, HW = T + 4;
    __shared__ double mag[HW][HW + 1];
    __shared__ double rowp[HW][T + 1];
    const float* img = in + (size_t)blockIdx.z * H * W;
    const int x0 = blockIdx.x * T - 2, y0 = blockIdx.y * T - 2;
    for (int e = threadIdx.x; e < HW * HW; e += 256) {
        const int ty = e / HW, tx = e % HW;
        const int y = refl101(y0 + ty, H), x = refl101(x0 + tx, W);
        const int ym = refl101(y - 1, H), yp = refl101(y + 1, H);
        const int xm = refl101(x - 1, W), xp = refl101(x + 1, W);
        const float* ru = img + (size_t)ym * W;
        const float* rc = img + (size_t)y * W;
        const float* rd = img + (size_t)yp * W;
        const double sx = (((double)ru[xp] - (double)ru[xm]) + 2.0 * ((double)rc[xp] - (double)rc[xm])) +
                          ((double)rd[xp] - (double)rd[xm]);
        const double sy = (((double)rd[xm] - (double)ru[xm]) + 2.0 * ((double)rd[x] - (double)ru[x])) +
                          ((double)rd[xp] - (double)ru[xp]);
        mag[ty][tx] = sqrt(sx * sx + sy * sy);
    }
    __syncthreads();
    const double g0 = 0.0625, g1 = 0.25, g2 = 0.375;
    for (int e = threadIdx.x; e < HW * T; e += 256) {
        const int ty = e / T, tx = e % T;
        const double* m = &mag[ty][tx];
        rowp[ty][tx] = (((g0 * m[0] + g1 * m[1]) + g2 * m[2]) + g1 * m[3]) + g0 * m[4];
    }
    __syncthreads();
    const int tx = threadIdx.x % T, ty = threadIdx.x / T;
    const int x = blockIdx.x * T + tx, y = blockIdx.y * T + ty;
    if (x < W && y < H) {
        const double v = (((g0 * rowp[ty][tx] + g1 * rowp[ty + 1][tx]) + g2 * rowp[ty + 2][tx]) + g1 * rowp[ty + 3][tx]) +
                         g0 * rowp[ty + 4][tx];
        out[(size_t)blockIdx.z * H * W + (size_t)y * W + x] = v;
    }
}

// erode_images (reference inputs.py:71-85): cv2.erode with a kh x kw MORPH_RECT element, anchor at
// its centre (kw / 2, kh / 2), default border (constant +max for erosion: out-of-image taps never
// win), i.e. the minimum over the in-image part of the window.  One thread per pixel; the window
// reads are L1 hits.
__global__ __launch_bounds__(256) void k_erode_rect(const float* __restrict__ in, float* __restrict__ out, int H, int W,
                                                    int kh, int kw) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float* img = in + (size_t)blockIdx.z * H * W;
    const int ya = max(0, y - kh / 2), yb = min(H, y - kh / 2 + kh);
    const int xa = max(0, x - kw / 2), xb = min(W, x - kw / 2 + kw);
    float m = img[(size_t)y * W + x];
    for (int yy = ya; yy < yb; ++yy)
        for (int xx = xa; xx < xb; ++xx) m = fminf(m, img[(size_t)yy * W + xx]);
    out[(size_t)blockIdx.z * H * W + (size_t)y * W + x] = m;
}

}  // namespace marf

using namespace marf;

hipError_t marf_launch_erode_rect(const float* in, float* out, int n_img, int H, int W, int kh, int kw, hipStream_t s) {
    dim3 grid((W + 15) / 16, (H + 15) / 16, n_img);
    hipLaunchKernelGGL(k_erode_rect, grid, dim3(256), 0, s, in, out, H, W, kh, kw);
    return hipGetLastError();
}

hipError_t marf_launch_edge_map(const float* in, double* out, int n_img, int H, int W, hipStream_t s) {
    dim3 grid((W + 15) / 16, (H + 15) / 16, n_img);
    hipLaunchKernelGGL(k_edge_map, grid, dim3(256), 0, s, in, out, H, W);
    return hipGetLastError();
}
