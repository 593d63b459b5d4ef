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
#include "marf_args.h"

namespace marf {

template <class P>
MARF_DEV void copy_tile_out(const typename P::T* act, int lda, int rows, int cols, typename P::T* dst, int ldd) {
    // LDS [rows][lda] -> global [rows][ldd], first `cols` columns. bf16: 16-byte chunks.
    // The (row, chunk) walk is incremental: one division per call, none per element.
    typedef typename P::T T;
    if (sizeof(T) == 2) {
        const int nch = cols / 8;
        const int step = blockDim.x, dr = step / nch, dc = step - dr * nch;
        int r = threadIdx.x / nch, c = threadIdx.x - r * nch;
        for (; r < rows;) {
            uint4 v = *reinterpret_cast<const uint4*>(act + (size_t)r * lda + 8 * c);
            *reinterpret_cast<uint4*>(dst + (size_t)r * ldd + 8 * c) = v;
            r += dr;
            c += dc;
            if (c >= nch) {
                c -= nch;
                ++r;
            }
        }
    } else {
        for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
            int r = e / cols, c = e - r * cols;
            dst[(size_t)r * ldd + c] = act[(size_t)r * lda + c];
        }
    }
}

// acc[i][PT] += W[rows (wave + 4 i)*32 .., k] . act[px, k]^T over k < K for the NA row tiles this
// wave owns (i < NA).  NA is dispatched once per layer (wave-uniform), so the body is branch-free.
//
// Schedule: the weight fragments stream from L2 through a static 4-deep register ring (slot u is
// reloaded for k-step k+4 right after its MFMAs issue: three k-steps of latency cover, no register
// moves), the activation fragments of step k+1 are read from LDS while step k's MFMAs run (two
// statically named buffers).  Loads past the last k-step are clamped to it (harmless L2 hits).
template <class P, int NA, int RT, int PT>
MARF_DEV void gemm_rows(f32x16 (&acc)[RT][PT], const typename P::T* __restrict__ W, int K,
                        const typename P::T* act, int lda, int wave, int lane) {
    typedef typename P::frag F;
    const int ko = P::kofs(lane);
    const int rl = lane & 31;
    const int nk = K / P::KS;
    const typename P::T* wrow[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) wrow[i] = W + (size_t)((wave + 4 * i) * 32 + rl) * K + ko;
    const typename P::T* brow = act + (size_t)rl * lda + ko;
    auto ldA = [&](F (&dst)[NA], int k) {
        const int kc = (k < nk ? k : nk - 1) * P::KS;
#pragma unroll
        for (int i = 0; i < NA; ++i) dst[i] = P::load_frag(wrow[i] + kc);
    };
    auto ldB = [&](F (&dst)[PT], int k) {
        const int kc = (k < nk ? k : nk - 1) * P::KS;
#pragma unroll
        for (int j = 0; j < PT; ++j) dst[j] = P::load_frag(brow + (size_t)j * 32 * lda + kc);
    };
    auto mma = [&](const F (&a)[NA], const F (&b)[PT]) {
#pragma unroll
        for (int j = 0; j < PT; ++j)
#pragma unroll
            for (int i = 0; i < NA; ++i) acc[i][j] = P::mma32(a[i], b[j], acc[i][j]);
    };
    F A0[NA], A1[NA], A2[NA], A3[NA], B0[PT], B1[PT];
    if constexpr (sizeof(F) * NA > 32) {
        // wide row blocks (bf16, NA > 2): a 2-deep ring keeps the kernel inside 256 VGPRs
        ldA(A0, 0);
        ldA(A1, 1);
        ldB(B0, 0);
        int k = 0;
        for (; k + 2 <= nk; k += 2) {
            ldB(B1, k + 1);
            __builtin_amdgcn_sched_barrier(0);
            mma(A0, B0);
            __builtin_amdgcn_sched_barrier(0);
            ldA(A0, k + 2);
            ldB(B0, k + 2);
            __builtin_amdgcn_sched_barrier(0);
            mma(A1, B1);
            __builtin_amdgcn_sched_barrier(0);
            ldA(A1, k + 3);
        }
        if (k < nk) mma(A0, B0);
        return;
    }
    ldA(A0, 0);
    ldA(A1, 1);
    ldA(A2, 2);
    ldA(A3, 3);
    ldB(B0, 0);
    int k = 0;
    // sched_barrier pins the issue order: left alone, the scheduler sinks every weight load to
    // the loop end (one MFMA of latency cover) and folds the two B buffers into one.
    for (; k + 4 <= nk; k += 4) {
        ldB(B1, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(A0, B0);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A0, k + 4);
        ldB(B0, k + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(A1, B1);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A1, k + 5);
        ldB(B1, k + 3);
        __builtin_amdgcn_sched_barrier(0);
        mma(A2, B0);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A2, k + 6);
        ldB(B0, k + 4);
        __builtin_amdgcn_sched_barrier(0);
        mma(A3, B1);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A3, k + 7);
    }
    // remainder (nk % 4 steps): A0..A2 hold steps k..k+2, B0 holds step k
    if (k < nk) {
        ldB(B1, k + 1);
        mma(A0, B0);
        if (k + 1 < nk) {
            ldB(B0, k + 2);
            mma(A1, B1);
            if (k + 2 < nk) mma(A2, B0);
        }
    }
}

// Accumulators start at the bias of their output row when `bias` is given (so the epilogue does
// not add it), else at zero.
template <class P, int RT, int PT>
MARF_DEV void gemm_tile(f32x16 (&acc)[RT][PT], const typename P::T* __restrict__ W, int K, int n_rt,
                        const typename P::T* act, int lda, int wave, int lane, const float* bias = nullptr) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        f32x16 init = (f32x16){};
        const int rt = wave + 4 * i;
        if (bias && rt < n_rt) {
            const float* bb = bias + rt * 32 + 4 * (lane >> 5);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 bv = *reinterpret_cast<const float4*>(bb + 8 * q);
                init[4 * q] = bv.x;
                init[4 * q + 1] = bv.y;
                init[4 * q + 2] = bv.z;
                init[4 * q + 3] = bv.w;
            }
        }
#pragma unroll
        for (int j = 0; j < PT; ++j) acc[i][j] = init;
    }
    int na = (n_rt - wave + 3) / 4;
    na = na < 0 ? 0 : (na > RT ? RT : na);
    switch (na) {
        case 1: gemm_rows<P, 1, RT, PT>(acc, W, K, act, lda, wave, lane); break;
        case 2: gemm_rows<P, 2, RT, PT>(acc, W, K, act, lda, wave, lane); break;
        case 3: if constexpr (RT >= 3) gemm_rows<P, 3, RT, PT>(acc, W, K, act, lda, wave, lane); break;
        case 4: if constexpr (RT >= 4) gemm_rows<P, 4, RT, PT>(acc, W, K, act, lda, wave, lane); break;
        default: break;
    }
}

// Store 4 consecutive rows (features) of one accumulator group for this lane's pixel.
template <class P>
MARF_DEV void store4(typename P::T* dst, float x0, float x1, float x2, float x3) {
    if (sizeof(typename P::T) == 2) {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        uint2 v;  // one v_cvt_pk_bf16_f32 per pair (RNE)
        v.x = __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){x0, x1}), bf16x2));
        v.y = __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){x2, x3}), bf16x2));
        *reinterpret_cast<uint2*>(dst) = v;
    } else {
        float* d = reinterpret_cast<float*>(dst);
        d[0] = x0;
        d[1] = x1;
        d[2] = x2;
        d[3] = x3;
    }
}

MARF_DEV void tile_origin(const GeoDev& g, int tile, int TP, int& b, int& p0, long long& slot0) {
    int tpp = g.Np_pad / TP;
    b = tile / tpp;
    p0 = (tile - b * tpp) * TP;
    slot0 = (long long)b * g.Np_pad + p0;
}

// ======================================================================== forward

template <class P, int TP>
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
    const int L = net.L;

    if ((int)threadIdx.x < L)
        wsh[threadIdx.x] = a.c2f.on ? c2f_weight(*a.c2f.progress, a.c2f.start, a.c2f.span, L, threadIdx.x) : 1.0f;
    __syncthreads();

    // ---- prologue: grid -> warp -> posenc (+c2f) -> LDS [px][Kp0]
    {
        constexpr int NPART = 256 / TP;
        const int i = threadIdx.x % TP, part = threadIdx.x / TP;
        float x, y, u = 0.f, v = 0.f, X[3];
        slot_point(a.geo, b, p0 + i, x, y, u, v, X);
        T* row = act + (size_t)i * lda;
        if (part == NPART - 1) {
            row[0] = P::cvt(u);
            row[1] = P::cvt(v);
        }
        // band q = c*L + k of coordinate c: sin at 2 + 2cL + k, cos at 2 + 2cL + L + k
        for (int q = part; q < 2 * L; q += NPART) {
            const int c = q >= L, k = q - c * L;
            float s, co;
            band_sincos<sizeof(T) == 2>(c ? v : u, k, s, co);
            if (a.c2f.on) {
                const float w = wsh[k];
                s = s * w;
                co = co * w;
            }
            row[2 + q + c * L] = P::cvt(s);
            row[2 + q + c * L + L] = P::cvt(co);
        }
        for (int f = net.D + part; f < net.Kp[0]; f += NPART) row[f] = P::cvt(0.f);
    }
    __syncthreads();
    if (a.feat[0]) copy_tile_out<P>(act, lda, TP, net.Kp[0], reinterpret_cast<T*>(a.feat[0]) + slot0 * net.Kp[0], net.Kp[0]);

    // ---- hidden layers
    const int nl = net.n_layers;
    for (int l = 0; l < nl - 1; ++l) {
        const int K = net.Kp[l], M = net.Mp[l], n_rt = M / 32;
        f32x16 acc[RT][PT];
        gemm_tile<P, RT, PT>(acc, reinterpret_cast<const T*>(net.Wf[l]), K, n_rt, act, lda, wave, lane, net.bias[l]);
        __syncthreads();  // every wave has consumed the layer input
        uint64_t* mk = a.mask[l + 1];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int rt = wave + 4 * i;
            if (rt >= n_rt) continue;
            const int rbase = rt * 32 + 4 * (lane >> 5);
#pragma unroll
            for (int j = 0; j < PT; ++j) {
                const int px = j * 32 + (lane & 31);
                float o[16];
                uint64_t bal[16];  // the v_cmp results themselves (SGPR pairs)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float z = acc[i][j][r];
                    const bool pos = z > 0.f;
                    o[r] = pos ? z : 0.f;
                    bal[r] = __ballot(pos);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    store4<P>(act + (size_t)px * lda + rbase + 8 * q, o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                if (mk) {
                    // 128 contiguous bytes per (pixel tile, row tile): the 32 ballot dwords are
                    // gathered into lanes 0..31 of one VGPR (v_writelane from the SGPR pairs) and
                    // written with one vector store
                    uint32_t w = 0;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"((uint32_t)bal[r]), "n"(2 * r));
                        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"((uint32_t)(bal[r] >> 32)), "n"(2 * r + 1));
                    }
                    uint32_t* mrow = reinterpret_cast<uint32_t*>(mk + (((slot0 >> 5) + j) * n_rt + rt) * 16);
                    if (lane < 32) mrow[lane] = w;
                }
            }
        }
        __syncthreads();
        if (a.feat[l + 1])
            copy_tile_out<P>(act, lda, TP, M, reinterpret_cast<T*>(a.feat[l + 1]) + slot0 * M, M);
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
            typename P::frag wa = P::load_frag(W + (size_t)(lane & 15) * K + k0 + ko);
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
    __shared__ float red[4][TP][2];
    __shared__ float red9[4][9];

    const NetDev& net = a.net;
    const int lda = a.lda;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int b, p0;
    long long slot0;
    tile_origin(a.geo, blockIdx.x, TP, b, p0, slot0);
    const int L = net.L;
    const int nl = net.n_layers;

    if ((int)threadIdx.x < L)
        wsh[threadIdx.x] = a.c2f.on ? c2f_weight(*a.c2f.progress, a.c2f.start, a.c2f.span, L, threadIdx.x) : 1.0f;

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
    for (int l = nl - 1; l >= 1; --l) {
        const int R = net.Kp[l], Kk = net.Mt[l], n_rt = R / 32;
        f32x16 acc[RT][PT];
        gemm_tile<P, RT, PT>(acc, reinterpret_cast<const T*>(net.Wt[l]), Kk, n_rt, act, lda, wave, lane);
        __syncthreads();
        const uint64_t* mk = a.mask[l];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int rt = wave + 4 * i;
            if (rt >= n_rt) continue;
            const int rbase = rt * 32 + 4 * (lane >> 5);
#pragma unroll
            for (int j = 0; j < PT; ++j) {
                const int px = j * 32 + (lane & 31);
                // the 16 wave-uniform lane masks of this tile (one per accumulator register),
                // fetched with two scalar loads into SGPRs; each element is one v_cndmask
                const uint64_t* mrow = mk + (((slot0 >> 5) + j) * n_rt + rt) * 16;
                u32x16 m0, m1;
                asm volatile(
                    "s_load_dwordx16 %0, %2, 0x0\n\t"
                    "s_load_dwordx16 %1, %2, 0x40\n\t"
                    "s_waitcnt lgkmcnt(0)"
                    : "=&s"(m0), "=&s"(m1)
                    : "s"(mrow)
                    : "memory");
                float o[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint32_t lo = r < 8 ? m0[2 * r] : m1[2 * r - 16];
                    const uint32_t hi = r < 8 ? m0[2 * r + 1] : m1[2 * r - 15];
                    const uint64_t ms = ((uint64_t)hi << 32) | lo;
                    float v;
                    asm volatile("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(v) : "v"(acc[i][j][r]), "s"(ms));
                    o[r] = v;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    store4<P>(act + (size_t)px * lda + rbase + 8 * q, o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
            }
        }
        __syncthreads();
        copy_tile_out<P>(act, lda, TP, R, reinterpret_cast<T*>(a.dz[l]) + slot0 * R, R);
    }

    // ---- layer 0 dgrad: d feat_0 = W_0^T dz_1  -> fp32 LDS [TP][Kp0 + 1]
    {
        const int R = net.Kp[0], Kk = net.Mt[0], n_rt = R / 32;
        f32x16 acc[RT][PT];
        gemm_tile<P, RT, PT>(acc, reinterpret_cast<const T*>(net.Wt[0]), Kk, n_rt, act, lda, wave, lane);
        __syncthreads();
        float* df = reinterpret_cast<float*>(smem);
        const int ldf = R + 1;
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int rt = wave + 4 * i;
            if (rt >= n_rt) continue;
#pragma unroll
            for (int j = 0; j < PT; ++j) {
                const int px = j * 32 + (lane & 31);
#pragma unroll
                for (int r = 0; r < 16; ++r) df[(size_t)px * ldf + rt * 32 + acc_row(lane, r)] = acc[i][j][r];
            }
        }
        __syncthreads();

        // ---- posenc adjoint: d coord_c = df[c] + sum_k w_k f_k (cos(x_k) df_sin - sin(x_k) df_cos)
        constexpr int NPART = 256 / TP;
        const int i = threadIdx.x % TP, part = threadIdx.x / TP;
        float x, y, u = 0.f, v = 0.f, X[3] = {0.f, 0.f, 1.f};
        const bool valid = slot_point(a.geo, b, p0 + i, x, y, u, v, X);
        const float* row = df + (size_t)i * ldf;
        float du = 0.f, dv = 0.f;
        if (part == 0) {
            du += row[0];
            dv += row[1];
        }
        for (int q = part; q < 2 * L; q += NPART) {
            const int c = q >= L, k = q - c * L;
            float s, co;
            band_sincos<sizeof(T) == 2>(c ? v : u, k, s, co);
            float gs = row[2 + q + c * L], gc = row[2 + q + c * L + L];
            if (a.c2f.on) {
                const float w = wsh[k];
                gs = gs * w;
                gc = gc * w;
            }
            float dspec = gs * co - gc * s;
            float d = dspec * ldexpf(3.14159265358979323846f, k);
            if (c == 0) du += d; else dv += d;
        }
        red[part][i][0] = du;
        red[part][i][1] = dv;
        __syncthreads();
        float h9[9];
#pragma unroll
        for (int e = 0; e < 9; ++e) h9[e] = 0.f;
        if ((int)threadIdx.x < TP) {
            du = red[0][i][0];
            dv = red[0][i][1];
            for (int q = 1; q < NPART; ++q) {
                du += red[q][i][0];
                dv += red[q][i][1];
            }
            if (a.geo.mode == 1) {
                if (valid && a.d_coords) {
                    a.d_coords[2 * (size_t)(p0 + i)] = du;
                    a.d_coords[2 * (size_t)(p0 + i) + 1] = dv;
                }
            } else if (valid) {
                // (u, v) = X[:2] / (X[2] + 1e-8): torch div backward, then bmm backward
                float dd = X[2] + 1e-8f;
                float dX0 = du / dd, dX1 = dv / dd;
                float dd2 = dd * dd;
                float dX2 = (-du * X[0]) / dd2 + (-dv * X[1]) / dd2;
                const float hom[3] = {x, y, 1.f};
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    h9[0 + c] = dX0 * hom[c];
                    h9[3 + c] = dX1 * hom[c];
                    h9[6 + c] = dX2 * hom[c];
                }
            }
        }
        if (a.geo.mode == 0) {
#pragma unroll
            for (int e = 0; e < 9; ++e) {
                float s = wave_sum(h9[e]);
                if (lane == 0) red9[wave][e] = s;
            }
            __syncthreads();
            if (threadIdx.x < 9) {
                float s = red9[0][threadIdx.x];
                for (int w = 1; w < 4; ++w) s += red9[w][threadIdx.x];
                a.dH_partial[(size_t)blockIdx.x * 9 + threadIdx.x] = s;
            }
        }
    }
}

}  // namespace marf

// ------------------------------------------------------------------ host launchers

using namespace marf;

template <class P, int TP>
static hipError_t launch_fwd_t(const FwdArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)k_mlp_fwd<P, TP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((k_mlp_fwd<P, TP>), dim3(n_tiles), dim3(256), lds, s, a);
    return hipGetLastError();
}

template <class P, int TP>
static hipError_t launch_bwd_t(const BwdArgs& a, size_t lds, int n_tiles, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)k_mlp_bwd<P, TP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((k_mlp_bwd<P, TP>), dim3(n_tiles), dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t marf_launch_mlp_fwd(const FwdArgs& a, int dtype, int TP, size_t lds, int n_tiles, hipStream_t s) {
    if (dtype == 1) return TP == 128 ? launch_fwd_t<PrecBF16, 128>(a, lds, n_tiles, s) : launch_fwd_t<PrecBF16, 64>(a, lds, n_tiles, s);
    return TP == 128 ? launch_fwd_t<PrecF32, 128>(a, lds, n_tiles, s) : launch_fwd_t<PrecF32, 64>(a, lds, n_tiles, s);
}

hipError_t marf_launch_mlp_bwd(const BwdArgs& a, int dtype, int TP, size_t lds, int n_tiles, hipStream_t s) {
    if (dtype == 1) return TP == 128 ? launch_bwd_t<PrecBF16, 128>(a, lds, n_tiles, s) : launch_bwd_t<PrecBF16, 64>(a, lds, n_tiles, s);
    return TP == 128 ? launch_bwd_t<PrecF32, 128>(a, lds, n_tiles, s) : launch_bwd_t<PrecF32, 64>(a, lds, n_tiles, s);
}
