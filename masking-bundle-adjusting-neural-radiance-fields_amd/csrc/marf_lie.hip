// marf_lie.hip -- sl(3) -> SL(3) exponential (Lie.sl3_to_SL3, warp.py:98-106) and its adjoint,
// plus the per-patch reduction of the warp gradient.
//
// torch.linalg.matrix_exp is reproduced operation for operation in fp32 so that H is
// bit-identical to the reference's: for a batch of >= 2 matrices torch always uses
// the degree-18 optimized Taylor polynomial with scaling & squaring; for a batch of one it picks
// the degree (1, 2, 4, 8, 12, 18) from the 1-norm.  Linear combinations of the matrix powers
// accumulate with fused multiply-add starting from 0 (torch's _compute_linear_combination CPU
// kernel); the small matrix products accumulate with separate multiply and add starting from 0
// (torch's baddbmm small-matrix kernel).  The backward is torch's: exp of the block matrix
// [[A^T, G], [0, A^T]] (same algorithm on 6x6), upper-right block, then the generator adjoint.
//
// One thread per patch: B <= a few thousand 3x3 problems, latency-only work.
#include "marf_args.h"

namespace marf {

#define LMAX 6

struct Mat {
    float a[LMAX * LMAX];
};

MARF_DEV void mm_plain(const float* X, const float* Y, float* R, int n) {
    float tmp[LMAX * LMAX];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            float acc = 0.0f;
            for (int k = 0; k < n; ++k) {
                float p = __fmul_rn(X[i * n + k], Y[k * n + j]);
                acc = __fadd_rn(acc, p);
            }
            tmp[i * n + j] = acc;
        }
    for (int e = 0; e < n * n; ++e) R[e] = tmp[e];
}

MARF_DEV void eye(float* I, int n) {
    for (int e = 0; e < n * n; ++e) I[e] = 0.0f;
    for (int i = 0; i < n; ++i) I[i * n + i] = 1.0f;
}

MARF_DEV void lincomb(const float* const* As, const float* c, int m, float* out, int n) {
    float tmp[LMAX * LMAX];
    for (int e = 0; e < n * n; ++e) {
        float acc = 0.0f;
        for (int j = 0; j < m; ++j) acc = __fmaf_rn(As[j][e], c[j], acc);
        tmp[e] = acc;
    }
    for (int e = 0; e < n * n; ++e) out[e] = tmp[e];
}

MARF_DEV void add_inplace(float* X, const float* Y, int n) {
    for (int e = 0; e < n * n; ++e) X[e] = __fadd_rn(X[e], Y[e]);
}

// Bader-Blanes-Casas coefficients as torch stores them (scalar_t = float).
__constant__ float kB18[5][5] = {
    {0.f, -1.00365581030144618291e-01, -8.02924648241156932449e-03, -8.92138498045333711011e-04, 0.f},
    {0.f, 3.97849749499645077844e-01, 1.36783778460411720168e+00, 4.98289622525382669416e-01,
     -6.37898194594723280150e-04},
    {-1.09676396052962061844e+01, 1.68015813878906206114e+00, 5.71779846478865511061e-02,
     -6.98210122488052056106e-03, 3.34975017086070470649e-05},
    {-9.04316832390810593223e-02, -6.76404519071381882256e-02, 6.75961301770459654925e-02,
     2.95552570429315521194e-02, -1.39180257516060693404e-05},
    {0.f, 0.f, -9.23364619367118555360e-02, -1.69364939002081722752e-02, -1.40086798182036094347e-05}};
__constant__ float kB12[4][4] = {
    {9.0198e-16, 0.46932117595418237389, -0.20099424927047284052, -0.04623946134063071740},
    {5.31597895759871264183, 1.19926790417132231573, 0.01179296240992997031, 0.01108844528519167989},
    {0.18188869982170434744, 0.05502798439925399070, 0.09351590770535414968, 0.00610700528898058230},
    {-2.0861320e-13, -0.13181061013830184015, -0.02027855540589259079, -0.00675951846863086359}};
__constant__ float kTheta[6] = {1.192092800768788e-07, 5.978858893805233e-04, 5.116619363445086e-02,
                                5.800524627688768e-01, 1.461661507209034e+00, 3.010066362817634e+00};

MARF_DEV void T18(const float* A, float* E, int n) {
    float I[LMAX * LMAX], A2[LMAX * LMAX], A3[LMAX * LMAX], A6[LMAX * LMAX];
    float Bs[5][LMAX * LMAX], V[LMAX * LMAX];
    eye(I, n);
    mm_plain(A, A, A2, n);
    mm_plain(A, A2, A3, n);
    mm_plain(A3, A3, A6, n);
    const float* as[5] = {I, A, A2, A3, A6};
    for (int i = 0; i < 5; ++i) lincomb(as, kB18[i], 5, Bs[i], n);
    mm_plain(Bs[0], Bs[4], V, n);  // A9
    add_inplace(Bs[3], V, n);
    add_inplace(Bs[2], Bs[3], n);
    mm_plain(Bs[2], Bs[3], V, n);
    add_inplace(Bs[1], V, n);
    for (int e = 0; e < n * n; ++e) E[e] = Bs[1][e];
}

MARF_DEV void T12(const float* A, float* E, int n) {
    float I[LMAX * LMAX], A2[LMAX * LMAX], A3[LMAX * LMAX];
    float Bs[4][LMAX * LMAX], V[LMAX * LMAX];
    eye(I, n);
    mm_plain(A, A, A2, n);
    mm_plain(A, A2, A3, n);
    const float* as[4] = {I, A, A2, A3};
    for (int i = 0; i < 4; ++i) lincomb(as, kB12[i], 4, Bs[i], n);
    mm_plain(Bs[3], Bs[3], V, n);  // A6
    add_inplace(Bs[2], V, n);
    add_inplace(Bs[1], Bs[2], n);
    mm_plain(Bs[1], Bs[2], V, n);
    add_inplace(Bs[0], V, n);
    for (int e = 0; e < n * n; ++e) E[e] = Bs[0][e];
}

MARF_DEV void T8(const float* A, float* E, int n) {
    // constants evaluated exactly as torch's constexpr scalar_t expressions (float members,
    // double literals)
    const float sqrt_177 = 0.1330413469565007072504e+2;
    const float x3 = 2. / 3.;
    const float x1 = (double)x3 * ((1. + (double)sqrt_177) / 88.);
    const float x2 = (double)x3 * ((1. + (double)sqrt_177) / 352.);
    const float x4 = (-271. + 29. * (double)sqrt_177) / (315. * (double)x3);
    const float x5 = (-11. + 11. * (double)sqrt_177) / (1260. * (double)x3);
    const float x6 = (-99. + 11. * (double)sqrt_177) / (5040. * (double)x3);
    const float x7 = (89. - (double)sqrt_177) / (5040. * (double)x3);
    const float y2 = (857. - 58. * (double)sqrt_177) / 630.;
    float I[LMAX * LMAX], A2[LMAX * LMAX], A4[LMAX * LMAX], A8[LMAX * LMAX], L1[LMAX * LMAX],
        L2[LMAX * LMAX];
    eye(I, n);
    mm_plain(A, A, A2, n);
    {
        const float* as[2] = {A, A2};
        const float c[2] = {x1, x2};
        lincomb(as, c, 2, L1, n);
        mm_plain(A2, L1, A4, n);
    }
    {
        const float* asa[2] = {A2, A4};
        const float ca[2] = {x3, 1.0f};
        lincomb(asa, ca, 2, L1, n);
        const float* asb[4] = {I, A, A2, A4};
        const float cb[4] = {x4, x5, x6, x7};
        lincomb(asb, cb, 4, L2, n);
        mm_plain(L1, L2, A8, n);
    }
    const float* as5[5] = {I, A, A2, A4, A8};
    const float c5[5] = {1.0f, 1.0f, y2, 0.0f, 1.0f};
    lincomb(as5, c5, 5, E, n);
}

MARF_DEV void T4(const float* A, float* E, int n) {
    float I[LMAX * LMAX], A2[LMAX * LMAX], L[LMAX * LMAX], P[LMAX * LMAX];
    eye(I, n);
    mm_plain(A, A, A2, n);
    const float* as3[3] = {I, A, A2};
    const float c3[3] = {(float)(1 / 2.0), (float)(1 / 6.0), (float)(1 / 24.0)};
    lincomb(as3, c3, 3, L, n);
    mm_plain(A2, L, P, n);
    const float* as4[4] = {I, A, A2, P};
    const float c4[4] = {1.0f, 1.0f, 0.0f, 1.0f};
    lincomb(as4, c4, 4, E, n);
}

MARF_DEV void T2(const float* A, float* E, int n) {
    float I[LMAX * LMAX], A2[LMAX * LMAX];
    eye(I, n);
    mm_plain(A, A, A2, n);
    for (int e = 0; e < n * n; ++e) E[e] = __fadd_rn(__fadd_rn(I[e], A[e]), A2[e] / 2.0f);
}

MARF_DEV void T1(const float* A, float* E, int n) {
    for (int e = 0; e < n * n; ++e) E[e] = __fadd_rn(((e / n) == (e % n)) ? 1.0f : 0.0f, A[e]);
}

MARF_DEV float one_norm(const float* A, int n) {
    float best = 0.0f;
    for (int j = 0; j < n; ++j) {
        float s = 0.0f;
        for (int i = 0; i < n; ++i) s = __fadd_rn(s, fabsf(A[i * n + j]));
        if (j == 0 || s > best) best = s;
    }
    return best;
}

MARF_DEV void T18_scale_square(const float* A, float* E, int n, float norm) {
    float q = norm / kTheta[5];
    float l = ceilf(log2f(q));
    int s = l > 0.0f ? (int)l : 0;
    float As[LMAX * LMAX];
    float scale = ldexpf(1.0f, -s);
    for (int e = 0; e < n * n; ++e) As[e] = __fmul_rn(A[e], scale);
    T18(As, E, n);
    for (int p = 0; p < s; ++p) mm_plain(E, E, E, n);
}

// torch.linalg.matrix_exp of one n x n matrix as part of a batch of `batch` matrices.
MARF_DEV void expm(const float* A, float* E, int n, int batch) {
    float norm = one_norm(A, n);
    if (batch > 1) {
        T18_scale_square(A, E, n, norm);
        return;
    }
    if (isnan(norm)) {
        for (int e = 0; e < n * n; ++e) E[e] = __int_as_float(0x7fc00000);
    } else if (norm >= kTheta[4]) {
        T18_scale_square(A, E, n, norm);
    } else if (norm <= kTheta[0]) {
        T1(A, E, n);
    } else if (norm <= kTheta[1]) {
        T2(A, E, n);
    } else if (norm <= kTheta[2]) {
        T4(A, E, n);
    } else if (norm <= kTheta[3]) {
        T8(A, E, n);
    } else {
        T12(A, E, n);
    }
}

// warp.py:101-104: A = [[h5,h3,h1],[h4,-h5-h6,h2],[h7,h8,h6]] (1-based h).
MARF_DEV void sl3_generator(const float* h, float* A) {
    A[0] = h[4];
    A[1] = h[2];
    A[2] = h[0];
    A[3] = h[3];
    A[4] = __fadd_rn(-h[4], -h[5]);
    A[5] = h[1];
    A[6] = h[6];
    A[7] = h[7];
    A[8] = h[5];
}

__global__ void k_sl3_to_SL3(const float* __restrict__ h, float* __restrict__ H, int B, int batch_hint) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float A[9], E[9];
    sl3_generator(h + 8 * b, A);
    expm(A, E, 3, batch_hint);
    for (int e = 0; e < 9; ++e) H[9 * b + e] = E[e];
}

MARF_DEV void sl3_backward_one(const float* h, const float* dH, float* d, int batch_hint) {
    float A[9], M[36], E[36], G[9];
    sl3_generator(h, A);
    for (int e = 0; e < 36; ++e) M[e] = 0.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            M[i * 6 + j] = A[j * 3 + i];
            M[(i + 3) * 6 + (j + 3)] = A[j * 3 + i];
            M[i * 6 + (j + 3)] = dH[i * 3 + j];
        }
    expm(M, E, 6, batch_hint);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) G[i * 3 + j] = E[i * 6 + (j + 3)];
    d[0] = G[2];
    d[1] = G[5];
    d[2] = G[1];
    d[3] = G[3];
    d[4] = __fadd_rn(G[0], -G[4]);
    d[5] = __fadd_rn(G[8], -G[4]);
    d[6] = G[6];
    d[7] = G[7];
}

__global__ void k_sl3_backward(const float* __restrict__ h, const float* __restrict__ dH, float* __restrict__ dh,
                               int B, int batch_hint) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float d[8];
    sl3_backward_one(h + 8 * b, dH + 9 * b, d, batch_hint);
    for (int e = 0; e < 8; ++e) dh[8 * b + e] = d[e];
}

// Per-patch sum (fixed order, fp64) of the per-tile dH partials written by the backward MLP
// kernel, then the Lie adjoint.  One block per patch.
// partial: [B * tiles_per_patch][9] fp32; dH_out: [B][9] (optional); dh: [B][8] (accumulate=0 ->
// overwrite).
// 576 threads = 64 slots x 9 entries: the tile partials of a patch pass through LDS in segments of
// 64 x RD_SEG tiles (every thread loads, all loads in flight together), and thread (t, e) adds entry
// e of tiles t, t + 64, t + 128, ... in that order in fp64 -- the per-slot sums of the former 64-thread
// form, which issued each slot's loads one after another (42 us at C3), in the same order.
constexpr int RD_SEG = 16;
__global__ __launch_bounds__(576) void k_reduce_dH_lie_bwd(const float* __restrict__ partial, int tiles_per_patch,
                                    const float* __restrict__ h, float* __restrict__ dH_out,
                                    float* __restrict__ dh, int batch_hint, const float* __restrict__ gscale,
                                    const float* __restrict__ denom) {
    __shared__ double red[64][9];
    __shared__ float seg[64 * RD_SEG * 9];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int t = tid & 63, e = tid >> 6;
    double acc = 0.0;
    const float* p = partial + (size_t)b * tiles_per_patch * 9;
    for (int i0 = 0; i0 < tiles_per_patch; i0 += 64 * RD_SEG) {
        const int n = min(64 * RD_SEG, tiles_per_patch - i0) * 9;
        __syncthreads();  // the previous segment is consumed
        for (int q = tid; q < n; q += 576) seg[q] = p[(size_t)i0 * 9 + q];
        __syncthreads();
        for (int k = 0; t + 64 * k < n / 9; ++k) acc += (double)seg[(t + 64 * k) * 9 + e];
    }
    red[t][e] = acc;
    __syncthreads();
    // the nine entries are summed on nine threads at once, each in the fixed order i = 0..63
    __shared__ float dHs[9];
    if (tid < 9) {
        double s = 0.0;
        for (int i = 0; i < 64; ++i) s += red[i][tid];
        dHs[tid] = (float)s;
    }
    __syncthreads();
    if (tid == 0) {
        float dHf[9];
        for (int q = 0; q < 9; ++q) dHf[q] = dHs[q];
        // fused step: partials carry the unit-upstream gradient without 1/denominator
        if (gscale)
            for (int q = 0; q < 9; ++q) dHf[q] = dHf[q] * (gscale[0] / denom[0]);
        if (dH_out)
            for (int q = 0; q < 9; ++q) dH_out[9 * b + q] = dHf[q];
        if (dh) {
            float d[8];
            sl3_backward_one(h + 8 * b, dHf, d, batch_hint);
            for (int q = 0; q < 8; ++q) dh[8 * b + q] = d[q];
        }
    }
}

// SE(2) as a sub-algebra of the reference's sl(3) parametrisation (an extension: the reference
// warps with sl(3) only, warp.py:72-80).  se(2) tangent p = (tx, ty, theta) -> the generator
// [[0, -theta, tx], [theta, 0, ty], [0, 0, 0]], which in warp.py:101-104's layout
// A = [[h5, h3, h1], [h4, -h5-h6, h2], [h7, h8, h6]] is h = (tx, ty, -theta, theta, 0, 0, 0, 0);
// marf_sl3_to_SL3 of that h is the SE(2) exponential.  Backward: the adjoint of the embedding.
__global__ void k_se2_to_sl3(const float* __restrict__ p, float* __restrict__ h, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float tx = p[3 * b], ty = p[3 * b + 1], th = p[3 * b + 2];
    float* o = h + 8 * (size_t)b;
    o[0] = tx;
    o[1] = ty;
    o[2] = -th;
    o[3] = th;
    o[4] = 0.f;
    o[5] = 0.f;
    o[6] = 0.f;
    o[7] = 0.f;
}

__global__ void k_se2_to_sl3_bwd(const float* __restrict__ dh, float* __restrict__ dp, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float* d = dh + 8 * (size_t)b;
    dp[3 * b] = d[0];
    dp[3 * b + 1] = d[1];
    dp[3 * b + 2] = d[3] - d[2];
}

}  // namespace marf

// ------------------------------------------------------------------ launch helpers (C++)

hipError_t marf_launch_se2_embed(const float* p, float* h, int B, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(marf::k_se2_to_sl3, dim3((B + 63) / 64), dim3(64), 0, s, p, h, B);
    return hipGetLastError();
}

hipError_t marf_launch_se2_embed_bwd(const float* dh, float* dp, int B, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(marf::k_se2_to_sl3_bwd, dim3((B + 63) / 64), dim3(64), 0, s, dh, dp, B);
    return hipGetLastError();
}

hipError_t marf_launch_sl3(const float* h, float* H, int B, int batch_hint, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(marf::k_sl3_to_SL3, dim3((B + 63) / 64), dim3(64), 0, s, h, H, B, batch_hint);
    return hipGetLastError();
}

hipError_t marf_launch_sl3_bwd(const float* h, const float* dH, float* dh, int B, int batch_hint, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(marf::k_sl3_backward, dim3((B + 63) / 64), dim3(64), 0, s, h, dH, dh, B, batch_hint);
    return hipGetLastError();
}

hipError_t marf_launch_reduce_dH(const float* partial, int tiles_per_patch, int B, const float* h,
                                 float* dH_out, float* dh, int batch_hint, hipStream_t s, const float* gscale,
                                 const float* denom) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(marf::k_reduce_dH_lie_bwd, dim3(B), dim3(576), 0, s, partial, tiles_per_patch, h, dH_out, dh,
                       batch_hint, gscale, denom);
    return hipGetLastError();
}
