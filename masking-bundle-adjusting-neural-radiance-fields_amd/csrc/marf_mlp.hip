// marf_mlp.hip -- the planar render loop's hot path on gfx950:
//
//   k_mlp_fwd : per tile of TP pixel slots, fused
//                 pixel grid -> sl(3) warp -> posenc + c2f  (warp.py:33-81, model/planar.py:451-471)
//                 -> Linear+ReLU x (n-1) -> Linear -> sigmoid   (model/planar.py:429-449)
//               Activations stay in one LDS tile between layers (in place: each wave keeps its
//               outputs in MFMA accumulators until every wave has read the layer input); the
//               weights stream from L2.  Optionally saves every layer input (pixel-major rows) and
//               the ReLU masks (1 bit / feature) for the backward pass.
//   k_mlp_bwd : per tile, the dgrad chain sigmoid' -> W_l^T ... with ReLU masks, saving dz_l for the
//               weight-gradient kernel, then the posenc / projective-warp adjoint fused into the
//               last step, reduced to one dH[3x3] partial per tile (or d coords per point).
//
// Orientation: Z^T[out x px] = W[out x in] . A^T[in x px]: the weights are the MFMA A operand
// (lane = output row, 8 contiguous k), the activations the B operand read from LDS
// (lane = pixel, 8 contiguous features), the accumulator holds a pixel per lane and features in
// registers, so 4 consecutive features per lane are written back with one 8-byte LDS store.
//
// 256 threads = 4 waves per block.  Output row tiles (32) of a layer are dealt round-robin to the
// 4 waves; each wave covers all PT = TP/32 pixel tiles, RT*PT = 8 accumulator tiles (128 VGPRs).
#include "marf_gemm.h"

namespace marf {

// ======================================================================== forward

// SK: the net has skip layers (their posenc prologue is compiled in only then: it costs the plain
// nets registers and spills)
template <class P, int TP, bool SK>
__global__ __launch_bounds__(256, 2) void k_mlp_fwd(FwdArgs a) {
    typedef typename P::T T;
    constexpr int PT = TP / 32;
    constexpr int RT = 8 / PT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* act = reinterpret_cast<T*>(smem);
    __shared__ float wsh[32];

    const NetDev& net = a.net;
    const int lda = a.lda;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int b, p0;
    long long slot0;
    tile_origin(a.geo, blockIdx.x, TP, b, p0, slot0);

    c2f_weights_lds(a.c2f, net.L, wsh);
    __syncthreads();
    tile_prologue<P, TP>(net, a.geo, a.c2f.on, wsh, act, lda, b, p0);
    __syncthreads();
    TileStore<T> st;
    st.clear();
    if (a.feat[0])
        save_tile<P>(st, act, lda, TP, net.Kp[0], reinterpret_cast<T*>(a.feat[0]) + slot0 * net.Kp[0], net.Kp[0] / P::KS);

    // ---- hidden layers
    const int nl = net.n_layers;
    for (int l = 0; l < nl - 1; ++l) {
        const int K = net.Kp[l], M = net.Mp[l], n_rt = M / 32;
        f32x16 acc[RT][PT];
        gemm_tile<P, RT, PT>(acc, reinterpret_cast<const T*>(net.Wf[l]), K, n_rt, act, lda, wave, lane, net.bias[l], st);
        __syncthreads();  // every wave has consumed the layer input
        relu_epilogue<P, RT, PT>(acc, act, lda, n_rt, wave, lane, a.mask[l + 1], blockIdx.x, net.diag[l + 1]);
        __syncthreads();
        if (SK && ((net.skip >> (l + 1)) & 1u)) {  // skip layer: [feature ; posenc] (model/planar.py:440-441)
            tile_prologue<P, TP>(net, a.geo, a.c2f.on, wsh, act, lda, b, p0, M);
            __syncthreads();
        }
        st.clear();
        if (a.feat[l + 1]) {
            const int Kn = net.Kp[l + 1];  // (M + Kp0 for a skip layer)
            if (l + 1 < nl - 1)
                save_tile<P>(st, act, lda, TP, Kn, reinterpret_cast<T*>(a.feat[l + 1]) + slot0 * Kn, Kn / P::KS);
            else  // input of the last (16x16) layer: plain copy
                copy_tile_out<P>(act, lda, TP, M, reinterpret_cast<T*>(a.feat[l + 1]) + slot0 * M, M);
        }
    }

    // ---- last layer (3 outputs, rows padded to 16): 16x16 MFMA, TP/4 pixels per wave, sigmoid
    {
        const int l = nl - 1;
        const int K = net.Kp[l];
        const T* W = reinterpret_cast<const T*>(net.Wf[l]);
        constexpr int NJ = TP / 64;
        f32x4 acc[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = (f32x4){};
        const int ko = P::kofs16(lane);
        for (int k0 = 0; k0 < K; k0 += P::KS16) {
            typename P::frag wa = P::load_frag(W + ((size_t)(k0 / P::KS16) * 64 + lane) * P::FE);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int px = wave * (TP / 4) + j * 16 + (lane & 15);
                typename P::frag bb = P::load_frag(act + (size_t)px * lda + k0 + ko);
                acc[j] = P::mma16(wa, bb, acc[j]);
            }
        }
        if (lane < 16) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int px = wave * (TP / 4) + j * 16 + lane;
                const int p = p0 + px;
                if (p < a.geo.Np) {
                    float* o = a.rgb + ((size_t)b * a.geo.Np + p) * 3;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        float z = acc[j][c] + net.bias[l][c];
                        o[c] = 1.0f / (1.0f + expf(-z));
                    }
                }
            }
        }
    }
}

// ======================================================================== backward

template <class P, int TP>
__global__ __launch_bounds__(256, 2) void k_mlp_bwd(BwdArgs a) {
    typedef typename P::T T;
    constexpr int PT = TP / 32;
    constexpr int RT = 8 / PT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* act = reinterpret_cast<T*>(smem);
    __shared__ float wsh[32];
    __shared__ float red[4 * TP * 2];
    __shared__ float red9[4 * 9];

    const NetDev& net = a.net;
    const int lda = a.lda;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int b, p0;
    long long slot0;
    tile_origin(a.geo, blockIdx.x, TP, b, p0, slot0);
    const int nl = net.n_layers;

    c2f_weights_lds(a.c2f, net.L, wsh);
    float* dsk = nullptr;  // skip nets: the posenc gradient of the skip layers
    if (net.skip) {
        dsk = reinterpret_cast<float*>(smem + skip_lds_off<P, TP>(net, lda));
        for (int e = threadIdx.x; e < TP * net.Kp[0]; e += 256) dsk[e] = 0.f;
    }

    // ---- sigmoid backward: g = d_rgb * (1 - y) * y   (torch sigmoid_backward)
    if ((int)threadIdx.x < TP) {
        const int i = threadIdx.x, p = p0 + i;
        float g[3] = {0.f, 0.f, 0.f};
        if (p < a.geo.Np) {
            const size_t o = ((size_t)b * a.geo.Np + p) * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float y = a.rgb[o + c];
                g[c] = (a.d_rgb[o + c] * (1.0f - y)) * y;
            }
        }
        *reinterpret_cast<float4*>(a.glast + (slot0 + i) * 4) = make_float4(g[0], g[1], g[2], 0.f);
        T* row = act + (size_t)i * lda;
        const int Kl = net.Mt[nl - 1];
        for (int c = 0; c < Kl; ++c) row[c] = P::cvt(c < 3 ? g[c] : 0.f);
    }
    __syncthreads();

    // ---- dgrad chain, l = nl-1 .. 1 : dfeat_l = W_l^T dz_{l+1}; dz_l = dfeat_l * relu'(feat_l)
    TileStore<T> st;
    st.clear();
    for (int l = nl - 1; l >= 1; --l) {
        const int R = net.Kp[l], Kk = net.Mt[l], n_rt = R / 32;
        f32x16 acc[RT][PT];
        const uint4 mw = *mask_record(const_cast<uint64_t*>(a.mask[l]), blockIdx.x, wave, lane);
        gemm_tile<P, RT, PT>(acc, reinterpret_cast<const T*>(net.Wt[l]), Kk, n_rt, act, lda, wave, lane, nullptr, st);
        __syncthreads();
        dgrad_epilogue<P, RT, PT>(acc, net, l, act, lda, wave, lane, mw, dsk);
        __syncthreads();
        save_tile<P>(st, act, lda, TP, R, reinterpret_cast<T*>(a.dz[l]) + slot0 * R, net.Mt[l - 1] / P::KS);
    }

    // ---- layer 0 dgrad + posenc / warp adjoint
    warp_adjoint<P, TP>(net, a.geo, a.c2f.on, wsh, smem, lda, wave, lane, b, p0, red, red9, a.dH_partial, a.d_coords, st,
                        nullptr, dsk);
}

}  // namespace marf

// ------------------------------------------------------------------ host launchers

using namespace marf;

template <class P, int TP, bool SK>
static hipError_t launch_fwd_sk(const FwdArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    {
        hipError_t e = ensure_dynamic_lds((const void*)k_mlp_fwd<P, TP, SK>, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_mlp_fwd<P, TP, SK>), dim3(n_tiles), dim3(256), lds, s, a);
    return hipGetLastError();
}

template <class P, int TP>
static hipError_t launch_fwd_t(const FwdArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    return a.net.skip ? launch_fwd_sk<P, TP, true>(a, lds, n_tiles, s) : launch_fwd_sk<P, TP, false>(a, lds, n_tiles, s);
}

template <class P, int TP>
static hipError_t launch_bwd_t(const BwdArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    {
        hipError_t e = ensure_dynamic_lds((const void*)k_mlp_bwd<P, TP>, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_mlp_bwd<P, TP>), dim3(n_tiles), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t marf_launch_mlp_fwd(const FwdArgs& a, int dtype, int TP, size_t lds, int n_tiles, hipStream_t s) {
    if (dtype == 1) return TP == 128 ? launch_fwd_t<PrecBF16, 128>(a, lds, n_tiles, s) : launch_fwd_t<PrecBF16, 64>(a, lds, n_tiles, s);
    if (dtype == 2) return TP == 128 ? launch_fwd_t<PrecF16, 128>(a, lds, n_tiles, s) : launch_fwd_t<PrecF16, 64>(a, lds, n_tiles, s);
    return TP == 128 ? launch_fwd_t<PrecF32, 128>(a, lds, n_tiles, s) : launch_fwd_t<PrecF32, 64>(a, lds, n_tiles, s);
}

hipError_t marf_launch_mlp_bwd(const BwdArgs& a, int dtype, int TP, size_t lds, int n_tiles, hipStream_t s) {
    if (dtype == 1) return TP == 128 ? launch_bwd_t<PrecBF16, 128>(a, lds, n_tiles, s) : launch_bwd_t<PrecBF16, 64>(a, lds, n_tiles, s);
    if (dtype == 2) return TP == 128 ? launch_bwd_t<PrecF16, 128>(a, lds, n_tiles, s) : launch_bwd_t<PrecF16, 64>(a, lds, n_tiles, s);
    return TP == 128 ? launch_bwd_t<PrecF32, 128>(a, lds, n_tiles, s) : launch_bwd_t<PrecF32, 64>(a, lds, n_tiles, s);
}
