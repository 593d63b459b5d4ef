// marf_step.hip -- the fused training step of the planar render loop on gfx950.
//
// One block = one tile of TP pixel slots of the crop grid.  Because the target and the mask are
// known when Graph.forward runs (model/planar.py:329-336 -> compute_loss :355-391), the tile's whole
// forward AND backward run in one pass, activations resident in one LDS tile:
//
//   grid -> sl(3) warp -> posenc + c2f                 (warp.py:33-81, model/planar.py:451-471)
//   (Linear + ReLU) x (n-1) -> Linear -> sigmoid       (model/planar.py:429-449)      -> rgb
//   masked MSE: loss partial, d rgb = 2 (p - g) m m    (model/planar.py:382-391), unit upstream
//                                                       gradient and no 1/denominator: both
//                                                       multiply every gradient and are applied
//                                                       in the reduction kernels (gout / denom)
//   sigmoid' -> last-layer weight gradient (16x16 MFMA over the tile's pixels, feat_{n-1} is
//   still in LDS) -> dgrad chain W_l^T with the ReLU masks -> dz_l saved for the hidden-layer
//   weight gradients -> layer-0 dgrad -> posenc / warp adjoint -> dH[3x3] partial per tile.
//
// HBM traffic per pixel (bf16, C3: L=16, 4 x 256 hidden): writes feat_0..feat_{n-2} and
// dz_1..dz_{n-1} (192 + 3*512 + 4*512 B), the ReLU masks (4 * 32 B, read back by the same wave)
// and rgb (12 B); reads target + mask (16 B).  Against the separate forward / loss / backward
// kernels this drops the last layer's input (written and read back, 1 KB), rgb / d rgb round
// trips and a second prologue.
#include "marf_gemm.h"

namespace marf {

// Transposed LDS read (gfx950 ds_read_b64_tr_b16): per 16-lane group, a 4 x 16 block of bf16 is
// read row-major (lane gi addresses row gi >> 2, columns 4 (gi & 3) ..) and delivered
// column-major: lane gi receives column gi of the 4 rows.
MARF_DEV i16x4 tr_read16(const u16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(p));
}

#define STAMP(i) MARF_STAMP(sp, i)

// BL: every forward bias staged in LDS at the start (sum of the hidden widths <= MARF_STEP_NBIAS):
// a GEMM's accumulator init reads LDS instead of loading from global behind the previous GEMM's
// stores (vmcnt retires in issue order), and no bias registers are live across the prologue.
constexpr int MARF_STEP_NBIAS = 1024;

// NW = waves per block: 4 (two blocks per CU) or 8 (one 512-thread block per CU, two waves per
// SIMD: the 512-wide C5 net at TP = 128, where every weight fragment a wave loads from L2 feeds 4
// pixel tiles' MFMAs instead of 2 -- half the weight-fragment traffic per MFMA of TP = 64)
// SK: the net has skip layers (their prologue / posenc-gradient code is compiled in only then: it
// costs the plain nets registers and spills)
template <class P, int TP, bool BL, int NW, bool SK>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void k_mlp_step(StepArgs a) {
    typedef typename P::T T;
    constexpr int PT = TP / 32;
    constexpr int RT = 8 / PT;
    static_assert(TP % (16 * NW) == 0, "last layer: whole 16-pixel groups per wave");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* act = reinterpret_cast<T*>(smem);
    __shared__ float wsh[32];
    __shared__ float red[(NW * 64 > 2 * TP ? NW * 64 : 2 * TP) * 2];
    __shared__ float red9[NW * 9];
    __shared__ __attribute__((aligned(16))) float gl[TP][4];  // sigmoid' gradient per slot (fp32)
    __shared__ __attribute__((aligned(16))) T gT[8][TP];      // the same, channel-major, split hi / lo
    __shared__ float lsum[2][TP];                              // per-slot ((p-g) m)^2 and m
    __shared__ __attribute__((aligned(16))) float bsh[BL ? MARF_STEP_NBIAS : 4];  // forward biases

    const NetDev& net = a.net;
    const int lda = a.lda;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int b, p0;
    long long slot0;
    tile_origin(a.geo, blockIdx.x, TP, b, p0, slot0);
    const int nl = net.n_layers;
    const int Np = a.geo.Np;
#ifdef MARF_STAMPS
    unsigned long long* sp = a.stamps ? a.stamps + (size_t)blockIdx.x * 32 : nullptr;
#endif

    STAMP(0);
    // the band weights first: vmcnt retires loads in issue order, so the barrier below must not
    // wait behind the tile's HBM target loads (those stay in flight through the prologue)
    const float cw = (int)threadIdx.x < net.L ? a.c2f_w[threadIdx.x] : 0.f;
    if constexpr (BL) {
        for (int l = 0, off = 0; l < nl - 1; off += net.Mp[l], ++l)
            for (int e = threadIdx.x; e < net.Mp[l]; e += 64 * NW) bsh[off + e] = net.bias[l][e];
    }
    // target + mask of the tile's slots: loaded now, parked in gl until the loss needs them.
    // Straight-line (every thread loads, padding slots a clamped valid pixel, zeroed after) so the
    // compiler counts them and the barrier below waits for the band weights only.
    float4 tg;
    {
        const int ti = threadIdx.x & (TP - 1);
        const int pc = min(p0 + ti, Np - 1);
        const float* gb = a.gt + (size_t)b * 3 * Np + pc;
        const float* mb = a.mask ? a.mask + (size_t)b * Np + pc : gb;
        tg = make_float4(gb[0], gb[Np], gb[2 * (size_t)Np], mb[0]);
        if (!a.mask) tg.w = 1.0f;
        if (p0 + ti >= Np) tg = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if ((int)threadIdx.x < net.L) wsh[threadIdx.x] = cw;
    __syncthreads();
    STAMP(19);
    tile_prologue<P, TP, true, NW>(net, a.geo, a.c2f.on, wsh, act, lda, b, p0);
    if ((int)threadIdx.x < TP) *reinterpret_cast<float4*>(&gl[threadIdx.x][0]) = tg;
    __syncthreads();
    STAMP(1);
    // every saved tile streams out during the GEMM that reads it next (TileStore)
    TileStore<T> st;
    save_tile<P, NW>(st, act, lda, TP, net.Kp[0], reinterpret_cast<T*>(a.feat[0]) + slot0 * net.Kp[0],
                     net.Kp[0] / P::KS, MARF_DIAG_SAVE(net));

    // ---- hidden layers (forward); the last one is peeled so the last layer's weight fragments
    //      can be in flight behind its epilogue without pinning registers through the loop
    int boff = 0;  // offset of layer l's bias in bsh
    auto bias_of = [&](int l) -> const float* {
        if constexpr (BL) return bsh + boff;
        else return net.bias[l];
    };
    auto hidden = [&](int l) {
        const int K = net.Kp[l], M = net.Mp[l], n_rt = M / 32;
        f32x16 acc[RT][PT];
        gemm_tile<P, RT, PT, NW>(acc, reinterpret_cast<const T*>(net.Wf[l]), K, n_rt, act, lda, wave, lane, bias_of(l), st);
        boff += M;
        __syncthreads();  // every wave has consumed the layer input
        STAMP(2 + 2 * l);
        relu_epilogue<P, RT, PT, NW>(acc, act, lda, n_rt, wave, lane, a.mask_bits[l + 1], blockIdx.x, net.diag[l + 1]);
        __syncthreads();
        if (l < 3) STAMP(3 + 2 * l);
        if (SK && ((net.skip >> (l + 1)) & 1u)) {  // skip layer: [feature ; posenc] (model/planar.py:440-441)
            tile_prologue<P, TP, true, NW>(net, a.geo, a.c2f.on, wsh, act, lda, b, p0, M);
            __syncthreads();
        }
        st.clear();
        if (l + 1 < nl - 1) {  // the last layer's input never leaves LDS
            const int Kn = net.Kp[l + 1];  // (M + Kp0 for a skip layer)
            save_tile<P, NW>(st, act, lda, TP, Kn, reinterpret_cast<T*>(a.feat[l + 1]) + slot0 * Kn, Kn / P::KS,
                             MARF_DIAG_SAVE(net));
        }
    };
    for (int l = 0; l < nl - 2; ++l) hidden(l);
    constexpr int NWL = 8;  // prefetched last-layer k-steps (16x16 fragments)
    typename P::frag wl[NWL];
    {
        const int l = nl - 2;
        const int K = net.Kp[l], M = net.Mp[l], n_rt = M / 32;
        f32x16 acc[RT][PT];
        gemm_tile<P, RT, PT, NW>(acc, reinterpret_cast<const T*>(net.Wf[l]), K, n_rt, act, lda, wave, lane, bias_of(l), st);
        __syncthreads();
        STAMP(2 + 2 * l);
        const T* W = reinterpret_cast<const T*>(net.Wf[nl - 1]);
        const int nk16 = net.Kp[nl - 1] / P::KS16;
#pragma unroll
        for (int u = 0; u < NWL; ++u) wl[u] = P::load_frag(W + ((size_t)(u < nk16 ? u : 0) * 64 + lane) * P::FE);
        relu_epilogue<P, RT, PT, NW>(acc, act, lda, n_rt, wave, lane, a.mask_bits[l + 1], blockIdx.x, net.diag[l + 1]);
        __syncthreads();
        st.clear();
    }

    // ---- last layer (3 outputs, rows padded to 16): 16x16 MFMA, TP/NW pixels per wave, sigmoid,
    //      rgb, masked-MSE partial and d rgb, sigmoid backward -> gl
    const int Kl = net.Kp[nl - 1];
    {
        const T* W = reinterpret_cast<const T*>(net.Wf[nl - 1]);
        constexpr int NJ = TP / NW / 16;
        f32x4 acc[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = (f32x4){};
        const int ko = P::kofs16(lane);
        const int nk16 = Kl / P::KS16;
#pragma unroll
        for (int u = 0; u < NWL; ++u) {
            if (u < nk16) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int px = wave * (TP / NW) + j * 16 + (lane & 15);
                    typename P::frag bb = P::load_frag(act + (size_t)px * lda + u * P::KS16 + ko);
                    acc[j] = P::mma16(wl[u], bb, acc[j]);
                }
            }
        }
        for (int u = NWL; u < nk16; ++u) {
            typename P::frag wa = P::load_frag(W + ((size_t)u * 64 + lane) * P::FE);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int px = wave * (TP / NW) + j * 16 + (lane & 15);
                typename P::frag bb = P::load_frag(act + (size_t)px * lda + u * P::KS16 + ko);
                acc[j] = P::mma16(wa, bb, acc[j]);
            }
        }
        if (lane < 16) {
            const float* bl = net.bias[nl - 1];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int px = wave * (TP / NW) + j * 16 + lane;
                const int p = p0 + px;
                float g[3] = {0.f, 0.f, 0.f};
                float sq = 0.f, mv = 0.f;
                const float4 tv = *reinterpret_cast<const float4*>(&gl[px][0]);  // prefetched target, mask
                const float tgt[3] = {tv.x, tv.y, tv.z};
                if (p < Np) {
                    const float m = tv.w;
                    float* o = a.rgb ? a.rgb + ((size_t)b * Np + p) * 3 : nullptr;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const float z = acc[j][c] + bl[c];
                        const float y = 1.0f / (1.0f + expf(-z));
                        if (o) o[c] = y;
                        // model/planar.py:388-390 and its autograd: x = (p - g) m, d = 2 x m
                        const float x = (y - tgt[c]) * m;
                        sq += x * x;
                        const float d = (2.0f * x) * m;
                        g[c] = (d * (1.0f - y)) * y;  // torch sigmoid_backward
                    }
                    mv = m;
                }
                *reinterpret_cast<float4*>(&gl[px][0]) = make_float4(g[0], g[1], g[2], 0.f);
#pragma unroll
                for (int c = 0; c < 3; ++c) {  // g = hi + lo (bf16 pair: ~16 significant bits)
                    const T hi = P::cvt(g[c]);
                    gT[c][px] = hi;
                    gT[4 + c][px] = P::cvt(g[c] - P::tof(hi));
                }
                gT[3][px] = P::cvt(0.f);
                gT[7][px] = P::cvt(0.f);
                lsum[0][px] = sq;
                lsum[1][px] = mv;
            }
        }
    }
    __syncthreads();

    STAMP(9);
    // ---- masked-MSE partial of the tile (fp64, fixed order) and the last bias gradient
    if (wave == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (int px = lane; px < TP; px += 64) {
            s0 += (double)lsum[0][px];
            s1 += (double)lsum[1][px];
        }
        s0 = wave_total63(s0);
        s1 = wave_total63(s1);
        if (lane == 63) {
            a.loss_partial[2 * (size_t)blockIdx.x] = s0;
            a.loss_partial[2 * (size_t)blockIdx.x + 1] = s1;
        }
    } else if (wave == 1) {
        float s[3] = {0.f, 0.f, 0.f};
        for (int px = lane; px < TP; px += 64)
#pragma unroll
            for (int c = 0; c < 3; ++c) s[c] += gl[px][c];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float t = wave_total63(s[c]);
            if (lane == 63) a.blast_partial[(size_t)blockIdx.x * 3 + c] = t;
        }
    }

    // ---- last-layer weight gradient of the tile: dW[c][k] = sum_px g[px][c] feat[px][k]
    //      16x16 MFMA, A = g^T (rows 0-2: bf16 hi parts of the 3 channels, rows 4-6: lo parts),
    //      B = feat (pixels x features, transposed LDS read for bf16); hi + lo rows are added
    //      after the K loop.  Column tiles of 16 features dealt round-robin to the waves.
    {
        float* wout = a.wlast_partial + (size_t)blockIdx.x * 3 * Kl;
        for (int ct = wave; ct < Kl / 16; ct += NW) {
            f32x4 acc = (f32x4){};
            if constexpr (sizeof(T) == 2) {
                const int g = lane >> 4, gi = lane & 15;
#pragma unroll
                for (int k0 = 0; k0 < TP; k0 += 32) {
                    typename P::frag fa;
                    if (gi < 8) fa = *reinterpret_cast<const typename P::frag*>(&gT[gi][k0 + 8 * g]);
                    else fa = (typename P::frag){};
                    const int r0 = k0 + 8 * g + (gi >> 2);
                    const u16* base = reinterpret_cast<const u16*>(act) + (size_t)r0 * lda + ct * 16 + 4 * (gi & 3);
                    i16x4 v[2] = {tr_read16(base), tr_read16(base + 4 * lda)};
                    acc = P::mma16(fa, *reinterpret_cast<typename P::frag*>(v), acc);
                }
            } else {
                const int kk = lane >> 4, n = lane & 15;
                for (int k0 = 0; k0 < TP; k0 += 4) {
                    const float fa = n < 8 ? P::tof(gT[n][k0 + kk]) : 0.f;
                    const float fb = P::tof(act[(size_t)(k0 + kk) * lda + ct * 16 + n]);
                    acc = P::mma16(fa, fb, acc);
                }
            }
            // accumulator: lane l, reg r -> row 4 (l >> 4) + r, column l & 15: hi rows in lanes
            // 0-15, lo rows in lanes 16-31
            float lo[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) lo[c] = __shfl_down(acc[c], 16, 64);
            if (lane < 16) {
#pragma unroll
                for (int c = 0; c < 3; ++c) wout[(size_t)c * Kl + ct * 16 + lane] = acc[c] + lo[c];
            }
        }
    }
    __syncthreads();  // feat_{n-1} consumed

    // ---- d (last-layer input) operand: act[px][0 .. Mt) = g
    if ((int)threadIdx.x < TP) {
        const int i = threadIdx.x;
        T* row = act + (size_t)i * lda;
        const int Kt = net.Mt[nl - 1];
        for (int c = 0; c < Kt; ++c) row[c] = P::cvt(c < 3 ? MARF_DIAG_ROUND(gl[i][c], net.diag[nl - 1], 3) : 0.f);
    }
    STAMP(10);
    __syncthreads();

    // ---- dgrad chain, l = n-1 .. 1 : dfeat_l = W_l^T dz_{l+1}; dz_l = dfeat_l * relu'(feat_l)
    st.clear();
    float* dsk = nullptr;  // skip nets: the posenc gradient of the skip layers
    if (SK && net.skip) {
        dsk = reinterpret_cast<float*>(smem + skip_lds_off<P, TP>(net, lda));
        for (int e = threadIdx.x; e < TP * net.Kp[0]; e += 64 * NW) dsk[e] = 0.f;
    }
    for (int l = nl - 1; l >= 1; --l) {
        const int R = net.Kp[l], Kk = net.Mt[l], n_rt = R / 32;
        f32x16 acc[RT][PT];
        const uint4 mw = *mask_record(a.mask_bits[l], blockIdx.x, wave, lane, NW);  // in flight behind the GEMM
        gemm_tile<P, RT, PT, NW>(acc, reinterpret_cast<const T*>(net.Wt[l]), Kk, n_rt, act, lda, wave, lane, nullptr, st);
        __syncthreads();
        dgrad_epilogue<P, RT, PT, NW>(acc, net, l, act, lda, wave, lane, mw, dsk);
        __syncthreads();
        if (l <= 4) STAMP(15 - l);  // 14 .. 11
        save_tile<P, NW>(st, act, lda, TP, R, reinterpret_cast<T*>(a.dz[l]) + slot0 * R, net.Mt[l - 1] / P::KS,
                         MARF_DIAG_SAVE(net));
    }

    // ---- layer-0 dgrad + posenc / warp adjoint -> dH partial
#ifdef MARF_STAMPS
    warp_adjoint<P, TP, true, NW>(net, a.geo, a.c2f.on, wsh, smem, lda, wave, lane, b, p0, red, red9, a.dH_partial, nullptr, st, sp,
                                  dsk);
#else
    warp_adjoint<P, TP, true, NW>(net, a.geo, a.c2f.on, wsh, smem, lda, wave, lane, b, p0, red, red9, a.dH_partial, nullptr, st,
                                  nullptr, dsk);
#endif
    STAMP(15);
}

// The step's c2f band weights, once (model/planar.py:462-470; 1 without c2f).
// (+ an optional int copy riding along: the step kernel's layer-0 column map, one launch fewer)
__global__ void k_c2f_weights(C2fDev c, int L, float* __restrict__ out, const int* __restrict__ csrc,
                              int* __restrict__ cdst, int cn) {
    if ((int)threadIdx.x < L) out[threadIdx.x] = c.on ? c2f_weight(*c.progress, c.start, c.span, L, threadIdx.x) : 1.0f;
    for (int i = threadIdx.x; i < cn; i += blockDim.x) cdst[i] = csrc[i];
}

// Loss of the fused step from the per-tile partials (fp64, fixed-order tree):
// out[0] = f32(sum x^2) / denom, out[1] = denom (= denom_override or 3 * f32(sum m)),
// out[2] = local 3 * f32(sum m)  (model/planar.py:390, as k_mse_final).
__global__ __launch_bounds__(256) void k_loss_final(const double* __restrict__ part, int n, float* __restrict__ out,
                                                    const float* __restrict__ denom_override) {
    __shared__ double rn[256], rm[256];
    double num = 0.0, ms = 0.0;
    // unrolled so 8 partial loads are in flight per thread (latency-bound single block); the
    // per-thread summation order is unchanged
#pragma unroll 8
    for (int i = threadIdx.x; i < n; i += 256) {
        num += part[2 * (size_t)i];
        ms += part[2 * (size_t)i + 1];
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
        const float denom = denom_override ? denom_override[0] : (float)rm[0] * 3.0f;
        out[0] = (float)rn[0] / denom;
        out[1] = denom;
        out[2] = (float)rm[0] * 3.0f;
    }
}

}  // namespace marf

using namespace marf;

template <class P, int TP, bool BL, int NW, bool SK>
static hipError_t launch_step_sk(const StepArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    {
        hipError_t e = ensure_dynamic_lds((const void*)k_mlp_step<P, TP, BL, NW, SK>, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_mlp_step<P, TP, BL, NW, SK>), dim3(n_tiles), dim3(64 * NW), lds, s, a);
    return hipGetLastError();
}

template <class P, int TP, bool BL, int NW>
static hipError_t launch_step_t(const StepArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    return a.net.skip ? launch_step_sk<P, TP, BL, NW, true>(a, lds, n_tiles, s)
                      : launch_step_sk<P, TP, BL, NW, false>(a, lds, n_tiles, s);
}

template <class P, int TP, int NW>
static hipError_t launch_step_b(const StepArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    int nb = 0;
    for (int l = 0; l + 1 < a.net.n_layers; ++l) nb += a.net.Mp[l];
    if (nb <= MARF_STEP_NBIAS) return launch_step_t<P, TP, true, NW>(a, lds, n_tiles, s);
    return launch_step_t<P, TP, false, NW>(a, lds, n_tiles, s);
}

template <class P>
static hipError_t launch_step_p(const StepArgs& a, int TP, int NW, size_t lds, int n_tiles, hipStream_t s) {
    if (TP == 128 && NW == 8) return launch_step_b<P, 128, 8>(a, lds, n_tiles, s);
    if (NW != 4) return hipErrorInvalidValue;
    return TP == 128 ? launch_step_b<P, 128, 4>(a, lds, n_tiles, s) : launch_step_b<P, 64, 4>(a, lds, n_tiles, s);
}

// TP pixel slots per block tile, NW waves per block (4, or 8 for the 16-bit recipes at TP = 128)
hipError_t marf_launch_mlp_step(const StepArgs& a, int dtype, int TP, int NW, size_t lds, int n_tiles, hipStream_t s) {
    if (dtype == 1) return launch_step_p<PrecBF16>(a, TP, NW, lds, n_tiles, s);
    if (dtype == 2) return launch_step_p<PrecF16>(a, TP, NW, lds, n_tiles, s);
    if (NW != 4) return hipErrorInvalidValue;
    return TP == 128 ? launch_step_b<PrecF32, 128, 4>(a, lds, n_tiles, s) : launch_step_b<PrecF32, 64, 4>(a, lds, n_tiles, s);
}

hipError_t marf_launch_c2f_weights(const C2fDev& c, int L, float* out, hipStream_t s, const int* csrc, int* cdst,
                                   int cn) {
    hipLaunchKernelGGL(k_c2f_weights, dim3(1), dim3(64), 0, s, c, L, out, csrc, cdst, cn);
    return hipGetLastError();
}

hipError_t marf_launch_loss_final(const double* part, int n, float* out, const float* denom_override, hipStream_t s) {
    hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(256), 0, s, part, n, out, denom_override);
    return hipGetLastError();
}
