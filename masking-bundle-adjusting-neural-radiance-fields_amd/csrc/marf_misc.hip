// marf_misc.hip -- the small kernels around the hot loop:
//   * masked MSE forward/backward            (Graph.mse_loss, model/planar.py:382-391)
//   * Adam                                   (torch.optim.Adam as built in Model.setup_optimizer,
//                                             model/planar.py:86-104)
//   * weight packing fp32 master -> bf16/fp32 MFMA operand layouts (padded, + transposed copy)
//   * standalone pixel grid / warp / posenc  (warp.py:33-81, model/planar.py:451-471) for the
//     module-level API (Warp.get_normalized_pixel_grid, Warp.warp_grid,
//     NeuralImageFunction.positional_encoding)
#include "marf_args.h"

namespace marf {

// ------------------------------------------------------------------ masked MSE

// pred [B][Np][3] (pixel-major, as the MLP writes it), gt [B][3][h*w], mask [B][1][h*w] (or null).
// Per-block partial sums in fp64: num = sum ((pred-gt)*m)^2, msum = sum m.
__global__ void k_mse_partial(const float* __restrict__ pred, const float* __restrict__ gt,
                              const float* __restrict__ mask, int B, int Np, double* __restrict__ part) {
    __shared__ double rn[256], rm[256];
    double num = 0.0, ms = 0.0;
    const long long n = (long long)B * Np;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        int b = (int)(e / Np), p = (int)(e % Np);
        float m = mask ? mask[(size_t)b * Np + p] : 1.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float d = (pred[e * 3 + c] - gt[((size_t)b * 3 + c) * Np + p]) * m;
            float d2 = d * d;
            num += (double)d2;
        }
        ms += (double)m;
    }
    rn[threadIdx.x] = num;
    rm[threadIdx.x] = ms;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            rn[threadIdx.x] += rn[threadIdx.x + o];
            rm[threadIdx.x] += rm[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = rn[0];
        part[2 * blockIdx.x + 1] = rm[0];
    }
}

// loss = f32(num) / (f32(sum m) * 3)   (model/planar.py:390); out[0] = loss, out[1] = denominator.
// denom_override (device scalar, optional): the global 3*sum(mask) when the patches are sharded over
// ranks (each rank then returns its share of the global loss).  Fixed-order tree in fp64.
__global__ __launch_bounds__(256) void k_mse_final(const double* __restrict__ part, int nblk, float* __restrict__ out,
                                                   const float* __restrict__ denom_override) {
    __shared__ double rn[256], rm[256];
    double num = 0.0, ms = 0.0;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        num += part[2 * i];
        ms += part[2 * i + 1];
    }
    rn[threadIdx.x] = num;
    rm[threadIdx.x] = ms;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            rn[threadIdx.x] += rn[threadIdx.x + o];
            rm[threadIdx.x] += rm[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float denom = denom_override ? denom_override[0] : (float)rm[0] * 3.0f;
        out[0] = (float)rn[0] / denom;
        out[1] = denom;
        out[2] = (float)rm[0] * 3.0f;
    }
}

// d pred = ((gout / denom) * (2 * (pred - gt) * m)) * m   (autograd of model/planar.py:388-390)
__global__ void k_mse_backward(const float* __restrict__ pred, const float* __restrict__ gt,
                               const float* __restrict__ mask, int B, int Np, const float* __restrict__ denom,
                               const float* __restrict__ gout, float* __restrict__ d_pred) {
    const long long n = (long long)B * Np;
    const float gs = gout[0] / denom[0];
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        int b = (int)(e / Np), p = (int)(e % Np);
        float m = mask ? mask[(size_t)b * Np + p] : 1.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float md = (pred[e * 3 + c] - gt[((size_t)b * 3 + c) * Np + p]) * m;
            d_pred[e * 3 + c] = (gs * (2.0f * md)) * m;
        }
    }
}

// ------------------------------------------------------------------ Adam

// torch.optim.Adam (foreach form): m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g g;
// p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps).  grad_scale multiplies g first (1 = none).
MARF_DEV void adam_body(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                        float* __restrict__ v, long long n, float w1, float b2, float one_minus_b2, float step_size,
                        float bc2_sqrt, float eps, const float* __restrict__ grad_scale) {
    const float gsc = grad_scale ? grad_scale[0] : 1.0f;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        float gi = g[i] * gsc;
        float mi = m[i];
        mi = mi + w1 * (gi - mi);
        float vi = v[i] * b2;
        vi = vi + one_minus_b2 * gi * gi;
        m[i] = mi;
        v[i] = vi;
        float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] - step_size * (mi / denom);
    }
}
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, long long n, float w1, float b2, float one_minus_b2,
                       float step_size, float bc2_sqrt, float eps, const float* __restrict__ grad_scale) {
    adam_body(p, g, m, v, n, w1, b2, one_minus_b2, step_size, bc2_sqrt, eps, grad_scale);
}
// the step's scalars from a device schedule row (sched[2 s], sched[2 s + 1], s = *index): the same
// update with host-free per-step values, so a captured training iteration can replay it
__global__ void k_adam_sched(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long long n, float w1, float b2, float one_minus_b2,
                             const float* __restrict__ sched, const int* __restrict__ index, float eps,
                             const float* __restrict__ grad_scale) {
    const int s = *index;
    adam_body(p, g, m, v, n, w1, b2, one_minus_b2, sched[2 * s], sched[2 * s + 1], eps, grad_scale);
}

// ------------------------------------------------------------------ packing

// Fragment-major packing (layout: marf_common.h).  Element e of a packed matrix with R rows (tiles
// of TR = 32 or 16 rows) and Kp columns: j = e % FE, lane, ks, rt from the rest; (row, k) from the
// MFMA fragment map of the tile shape.  src(row, k) = W[row][k] (forward) or W[k][row] (transposed).
template <class P>
MARF_DEV void frag_coord(long long e, int nk, bool t16, int& row, int& k) {
    const int j = (int)(e % P::FE);
    long long r = e / P::FE;
    const int lane = (int)(r % 64);
    r /= 64;
    const int ks = (int)(r % nk);
    const int rt = (int)(r / nk);
    if (t16) {
        row = rt * 16 + (lane & 15);
        k = ks * P::KS16 + (lane >> 4) * P::FE + j;
    } else {
        row = rt * 32 + (lane & 31);
        k = ks * P::KS + (lane >> 5) * P::FE + j;
    }
}

template <class P>
__global__ void k_pack(const float* __restrict__ params, char* __restrict__ packed, PackArgs a) {
    typedef typename P::T T;
    const int l = blockIdx.y;
    const PackLayer& L = a.ly[l];
    T* wf = reinterpret_cast<T*>(packed + L.wf_off);
    T* wt = reinterpret_cast<T*>(packed + L.wt_off);
    float* bias = reinterpret_cast<float*>(packed + L.bias_off);
    const float* W = params + L.w_off;
    const float* bsrc = params + L.b_off;
    const long long nf = (long long)L.Mp * L.Kp;
    const long long nt = (long long)L.Kp * L.Mt;
    const bool last16 = L.Mp == 16;  // the 3-output layer runs on 16x16 MFMA
    const int nkf = L.Kp / (last16 ? P::KS16 : P::KS), nkt = L.Mt / P::KS;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < nf + nt + L.Mp; e += (long long)gridDim.x * 256) {
        if (e < nf) {
            int m, k;
            frag_coord<P>(e, nkf, last16, m, k);
            float wv = m < L.M && k < L.K ? W[(size_t)m * L.K + k] : 0.f;
            wf[e] = P::cvt(MARF_DIAG_ROUND(wv, L.diag, 0));
        } else if (e < nf + nt) {
            int kr, m;  // row of W^T = input feature, column = output feature
            frag_coord<P>(e - nf, nkt, false, kr, m);
            float wtv = m < L.M && kr < L.K ? W[(size_t)m * L.K + kr] : 0.f;
            wt[e - nf] = P::cvt(MARF_DIAG_ROUND(wtv, L.diag, 1));
        } else {
            int m = (int)(e - nf - nt);
            bias[m] = m < L.M ? bsrc[m] : 0.f;
        }
    }
}

// ------------------------------------------------------------------ standalone prologue ops

__global__ void k_pixel_grid(GeoDev g, float* __restrict__ xy, int n) {
    for (int p = blockIdx.x * 256 + threadIdx.x; p < n; p += gridDim.x * 256) {
        int r = p / g.w, c = p - r * g.w;
        xy[2 * (size_t)p] = grid_coord(g.x0 + c, g.W, g.norm_w);
        xy[2 * (size_t)p + 1] = grid_coord(g.y0 + r, g.H, g.norm_h);
    }
}

// xy [B or 1][n][2] -> uv [B][n][2] under Hm [B][9]
__global__ void k_warp_points(const float* __restrict__ xy, const float* __restrict__ Hm, float* __restrict__ uv,
                              int B, int n, int xy_shared) {
    const long long tot = (long long)B * n;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < tot; e += (long long)gridDim.x * 256) {
        int b = (int)(e / n);
        long long src = xy_shared ? (e % n) : e;
        float X[3], u, v;
        warp_point(Hm + 9 * b, xy[2 * src], xy[2 * src + 1], u, v, X, 9 * n < 400);
        uv[2 * e] = u;
        uv[2 * e + 1] = v;
    }
}

// coord [n][2] -> enc [n][4L] (model/planar.py:451-471 layout: x: sin_k, cos_k; y: sin_k, cos_k)
__global__ void k_posenc(const float* __restrict__ coord, long long n, int L, const float* progress, float start,
                         float span, int c2f_on, float* __restrict__ enc) {
    const long long tot = n * 2 * L;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < tot; e += (long long)gridDim.x * 256) {
        long long i = e / (2 * L);
        int ck = (int)(e % (2 * L)), c = ck / L, k = ck % L;
        float s, co;
        sincosf(posenc_arg(coord[2 * i + c], k), &s, &co);
        if (c2f_on) {
            float w = c2f_weight(*progress, start, span, L, k);
            s = s * w;
            co = co * w;
        }
        enc[i * 4 * L + c * 2 * L + k] = s;
        enc[i * 4 * L + c * 2 * L + L + k] = co;
    }
}

// Warp.warp_grid autograd (warp.py:70-81): uv = X[:2] / (X[2] + 1e-8), X = H [x, y, 1].
// One block per patch walks its points: d xy per point, and dH = sum over points of
// dX (x, y, 1)^T accumulated in fp64 in a fixed order (deterministic).  With a shared point set the
// per-patch d xy rows are written separately and the caller sums them (autograd of the expand).
__global__ __launch_bounds__(1024) void k_warp_points_bwd(const float* __restrict__ xy, const float* __restrict__ Hm,
                                                          const float* __restrict__ G, float* __restrict__ dxy,
                                                          float* __restrict__ dH, int n, int xy_shared) {
    __shared__ double red[16][9];
    const int b = blockIdx.x;
    const float* H = Hm + 9 * b;
    double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = threadIdx.x; p < n; p += 1024) {
        const long long src = xy_shared ? p : (long long)b * n + p;
        const long long dst = (long long)b * n + p;
        const float x = xy[2 * src], y = xy[2 * src + 1];
        float X[3], u, v;
        warp_point(H, x, y, u, v, X, 9 * n < 400);
        const float gu = G[2 * dst], gv = G[2 * dst + 1];
        const float d = X[2] + 1e-8f;
        const float dX0 = gu / d, dX1 = gv / d;
        const float dd2 = d * d;
        const float dX2 = (-gu * X[0]) / dd2 + (-gv * X[1]) / dd2;
        const float hom[3] = {x, y, 1.f};
        const float dX[3] = {dX0, dX1, dX2};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[3 * r + c] += (double)(dX[r] * hom[c]);
        dxy[2 * dst] = (H[0] * dX0 + H[3] * dX1) + H[6] * dX2;
        dxy[2 * dst + 1] = (H[1] * dX0 + H[4] * dX1) + H[7] * dX2;
    }
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        const double t = wave_total63(acc[e]);
        if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6][e] = t;
    }
    __syncthreads();
    if (threadIdx.x < 9) {
        double t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w][threadIdx.x];
        dH[9 * b + threadIdx.x] = (float)t;
    }
}

// NeuralImageFunction.positional_encoding autograd (model/planar.py:451-471): for coordinate c of
// point i, d c = sum_k (w_k g_sin cos(s_k) - w_k g_cos sin(s_k)) * 2^k pi, s_k = 2^k pi c (the c2f
// weights w_k are constants of the step: progress carries no gradient).
__global__ void k_posenc_bwd(const float* __restrict__ coord, const float* __restrict__ G, long long n, int L,
                             const float* progress, float start, float span, int c2f_on, float* __restrict__ dcoord) {
    const float pi_f = 3.14159265358979323846f;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < 2 * n; e += (long long)gridDim.x * 256) {
        const long long i = e >> 1;
        const int c = (int)(e & 1);
        const float* g = G + i * 4 * L + c * 2 * L;
        float acc = 0.f;
        for (int k = 0; k < L; ++k) {
            float s, co;
            sincosf(posenc_arg(coord[e], k), &s, &co);
            float gs = g[k], gc = g[L + k];
            if (c2f_on) {
                const float w = c2f_weight(*progress, start, span, L, k);
                gs = gs * w;
                gc = gc * w;
            }
            acc += (gs * co + gc * -s) * ldexpf(pi_f, k);
        }
        dcoord[e] = acc;
    }
}


// Prologue probe (measurement only, SURVEY.md §8(d) "achieved prologue GB/s"): the fused step's
// per-pixel input side on its own -- read the target r, g, b and the mask (16 B/px, fp32 planes),
// pixel grid -> warp by the patch's H -> posenc + c2f features -- reduced to one float per block so
// that nothing is optimised away.  bench.py divides 16 B/px by its HIP-event time.
__global__ __launch_bounds__(256) void k_prologue_probe(GeoDev g, C2fDev c, int L, const float* __restrict__ gt,
                                                        const float* __restrict__ mask, float* __restrict__ out) {
    __shared__ float wl[32];
    __shared__ float red[4];
    if (threadIdx.x < 32) {
        float w = 1.0f;
        if (c.on && (int)threadIdx.x < L) w = c2f_weight(*c.progress, c.start, c.span, L, threadIdx.x);
        wl[threadIdx.x] = w;
    }
    __syncthreads();
    const long long n = (long long)g.B * g.Np;
    float acc = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const int b = (int)(i / g.Np), p = (int)(i - (long long)b * g.Np);
        const float* t = gt + (size_t)b * 3 * g.Np + p;
        const float m = mask ? mask[(size_t)b * g.Np + p] : 1.0f;
        const float tsum = (t[0] + t[g.Np] + t[2 * (size_t)g.Np]) * m;
        float x, y, u, v, X[3];
        slot_point<true>(g, b, p, x, y, u, v, X);
        float f = u + v;
        for (int k = 0; k < L; ++k) {
            float s0, c0, s1, c1;
            band_sincos<true>(u, k, s0, c0);
            band_sincos<true>(v, k, s1, c1);
            f += wl[k] * ((s0 + c0) + (s1 + c1));
        }
        acc += f * tsum;
    }
    acc = wave_total63(acc);
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace marf

using namespace marf;

static int grid_for(long long n) {
    long long b = (n + 255) / 256;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t marf_launch_mse(const float* pred, const float* gt, const float* mask, int B, int Np, double* part,
                           float* out, const float* denom_override, hipStream_t s) {
    int nb = grid_for((long long)B * Np);
    if (nb > 1024) nb = 1024;
    hipLaunchKernelGGL(k_mse_partial, dim3(nb), dim3(256), 0, s, pred, gt, mask, B, Np, part);
    hipLaunchKernelGGL(k_mse_final, dim3(1), dim3(256), 0, s, part, nb, out, denom_override);
    return hipGetLastError();
}

hipError_t marf_launch_mse_bwd(const float* pred, const float* gt, const float* mask, int B, int Np,
                               const float* denom, const float* gout, float* d_pred, hipStream_t s) {
    hipLaunchKernelGGL(k_mse_backward, dim3(grid_for((long long)B * Np)), dim3(256), 0, s, pred, gt, mask, B, Np,
                       denom, gout, d_pred);
    return hipGetLastError();
}

hipError_t marf_launch_adam(float* p, const float* g, float* m, float* v, long long n, float w1, float b2,
                            float one_minus_b2, float step_size, float bc2_sqrt, float eps, const float* grad_scale,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_adam, dim3(grid_for(n)), dim3(256), 0, s, p, g, m, v, n, w1, b2, one_minus_b2, step_size,
                       bc2_sqrt, eps, grad_scale);
    return hipGetLastError();
}

hipError_t marf_launch_adam_sched(float* p, const float* g, float* m, float* v, long long n, float w1, float b2,
                                  float one_minus_b2, const float* sched, const int* index, float eps,
                                  const float* grad_scale, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_adam_sched, dim3(grid_for(n)), dim3(256), 0, s, p, g, m, v, n, w1, b2, one_minus_b2, sched,
                       index, eps, grad_scale);
    return hipGetLastError();
}

hipError_t marf_launch_pack(int dtype, const float* params, char* packed, const PackArgs& a, long long max_elems,
                            hipStream_t s) {
    dim3 grid(grid_for(max_elems), a.n_layers);
    if (dtype == 1)
        hipLaunchKernelGGL(k_pack<PrecBF16>, grid, dim3(256), 0, s, params, packed, a);
    else if (dtype == 2)
        hipLaunchKernelGGL(k_pack<PrecF16>, grid, dim3(256), 0, s, params, packed, a);
    else
        hipLaunchKernelGGL(k_pack<PrecF32>, grid, dim3(256), 0, s, params, packed, a);
    return hipGetLastError();
}

hipError_t marf_launch_pixel_grid(const GeoDev& g, float* xy, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_pixel_grid, dim3(grid_for(n)), dim3(256), 0, s, g, xy, n);
    return hipGetLastError();
}

hipError_t marf_launch_warp_points(const float* xy, const float* Hm, float* uv, int B, int n, int xy_shared,
                                   hipStream_t s) {
    hipLaunchKernelGGL(k_warp_points, dim3(grid_for((long long)B * n)), dim3(256), 0, s, xy, Hm, uv, B, n, xy_shared);
    return hipGetLastError();
}

hipError_t marf_launch_posenc(const float* coord, long long n, int L, const float* progress, float start, float span,
                              int c2f_on, float* enc, hipStream_t s) {
    hipLaunchKernelGGL(k_posenc, dim3(grid_for(n * 2 * L)), dim3(256), 0, s, coord, n, L, progress, start, span,
                       c2f_on, enc);
    return hipGetLastError();
}

hipError_t marf_launch_prologue_probe(const GeoDev& g, const C2fDev& c, int L, const float* gt, const float* mask,
                                      float* out, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_prologue_probe, dim3(grid), dim3(256), 0, s, g, c, L, gt, mask, out);
    return hipGetLastError();
}

hipError_t marf_launch_warp_points_bwd(const float* xy, const float* Hm, const float* G, float* dxy, float* dH, int B,
                                       int n, int xy_shared, hipStream_t s) {
    hipLaunchKernelGGL(k_warp_points_bwd, dim3(B), dim3(1024), 0, s, xy, Hm, G, dxy, dH, n, xy_shared);
    return hipGetLastError();
}

hipError_t marf_launch_posenc_bwd(const float* coord, const float* G, long long n, int L, const float* progress,
                                  float start, float span, int c2f_on, float* dcoord, hipStream_t s) {
    hipLaunchKernelGGL(k_posenc_bwd, dim3(grid_for(2 * n)), dim3(256), 0, s, coord, G, n, L, progress, start, span,
                       c2f_on, dcoord);
    return hipGetLastError();
}
