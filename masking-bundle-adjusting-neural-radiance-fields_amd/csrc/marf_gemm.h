// marf_gemm.h -- device building blocks shared by the per-tile MLP kernels (marf_mlp.hip,
// marf_step.hip): the LDS-resident activation tile GEMM (weights = MFMA A operand streamed from
// L2, activations = B operand read from LDS), its epilogue store and tile addressing.
//
// Orientation: Z^T[out x px] = W[out x in] . A^T[in x px]: lane = output row / 8 contiguous k for
// the weights, lane = pixel / 8 contiguous features for the activations; the accumulator holds a
// pixel per lane and features in registers.  256 threads = 4 waves; output row tiles (32) of a
// layer are dealt round-robin to the 4 waves, each wave covers all PT = TP/32 pixel tiles.
#pragma once
#include <type_traits>

#include "marf_args.h"

namespace marf {

template <class P>
MARF_DEV void copy_tile_out(const typename P::T* act, int lda, int rows, int cols, typename P::T* dst, int ldd,
                            int rmode = 0) {
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
            dst[(size_t)r * ldd + c] = rmode ? diag_round(act[(size_t)r * lda + c], rmode) : act[(size_t)r * lda + c];
        }
    }
}

// Streams an LDS tile [rows][lda] (first `cols` columns) to global [rows][ldd] in 16-byte chunks
// right after the GEMM that reads the tile (gemm_tile flushes it there, before the epilogue
// rewrites the tile).  gemm_rows can also interleave the chunks with its k-steps (JOB 1 / 2), but
// vmcnt retires in issue order, so a store between the weight-fragment loads makes every later
// fragment wait for it: measured slower (C5 80.7 vs 66.7 ms), kept only as the JOB template.
// bf16 tiles only (16-B aligned LDS rows).
//
// Wave-uniform walk: rpi = 64 / nch whole rows per wave step (lane -> row lane / nch, chunk
// lane % nch); wave w of nw copies row groups w, w + nw, ...
template <class T>
struct TileStore {
    T* dst;
    int lda, ldd, rows, rpi, q, nq, wave, nw;
    int lr, lc;  // per lane
    bool active;

    MARF_DEV void clear() {
        active = false;
        q = nq = 0;
    }
    MARF_DEV void init(int lda_, T* d, int ldd_, int rows_, int cols, int wave_, int lane, int nw_ = 4) {
        constexpr int VEC = 16 / sizeof(T);
        const int nch = cols / VEC;  // <= 64 (cols <= 512)
        dst = d;
        lda = lda_;
        ldd = ldd_;
        rows = rows_;
        wave = wave_;
        nw = nw_;
        rpi = 64 / nch;
        lr = lane / nch;
        lc = lane - lr * nch;
        q = 0;
        nq = (rows + nw * rpi - 1) / (nw * rpi);
        active = true;
    }
    MARF_DEV int row() const {
        const int qq = q < nq ? q : nq - 1;
        const int r = (qq * nw + wave) * rpi + lr;
        return r < rows ? r : rows - 1;  // idle lanes / surplus rows repeat the last row's chunk
    }
    MARF_DEV uint4 read(const T* src) const {
        constexpr int VEC = 16 / sizeof(T);
        return *reinterpret_cast<const uint4*>(src + (size_t)row() * lda + VEC * lc);
    }
    MARF_DEV void write(uint4 v) {
        constexpr int VEC = 16 / sizeof(T);
        *reinterpret_cast<uint4*>(dst + (size_t)row() * ldd + VEC * lc) = v;
        ++q;
    }
    MARF_DEV void flush(const T* src) {
        while (q < nq) write(read(src));
    }
};

// acc[i][PT] += W[rows (wave + NW i)*32 .., k] . act[px, k]^T over k < K for the NA row tiles this
// wave owns (i < NA; NW waves per block deal the row tiles round-robin).  NA is dispatched once per layer (wave-uniform), so the body is branch-free.
//
// Schedule: the weight fragments stream from L2 through a static 4-deep register ring (slot u is
// reloaded for k-step k+4 right after its MFMAs issue: three k-steps of latency cover, no register
// moves), the activation fragments of step k+1 are read from LDS while step k's MFMAs run (two
// statically named buffers).  Loads past the last k-step are clamped to it (harmless L2 hits).
// JOB: one TileStore chunk per k-step (1) or per second k-step (2: the job has at most half as many
// chunks as the GEMM k-steps, e.g. a 512-wide tile saved during a 512-deep GEMM at 8 waves, where
// one chunk per k-step would rewrite the last chunk for half the GEMM), read before the B
// prefetch, stored after the A reload.
template <class P, int NA, int RT, int PT, int JOB, int NW = 4>
MARF_DEV void gemm_rows(f32x16 (&acc)[RT][PT], const typename P::T* __restrict__ W, int K,
                        const typename P::T* act, int lda, int wave, int lane, TileStore<typename P::T>& st) {
    typedef typename P::frag F;
    const int ko = P::kofs(lane);
    const int rl = lane & 31;
    const int nk = K / P::KS;
    // fragment-major weights (marf_common.h): fragment (rt, ks) at ((rt * nk + ks) * 64 + lane) * FE
    const typename P::T* wrow[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) wrow[i] = W + ((size_t)(wave + NW * i) * nk * 64 + lane) * P::FE;
    const typename P::T* brow = act + (size_t)rl * lda + ko;
    auto ldA = [&](F (&dst)[NA], int k) {
        const int kc = (k < nk ? k : nk - 1) * 64 * P::FE;
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
    uint4 sv = make_uint4(0, 0, 0, 0);
    // pos: the k-step's position in the 4-step unrolled body (0 in the 2-deep-ring body, which
    // places the job at positions 0 and 1 of its 2-step iterations)
    auto sread = [&](auto posc) {
        if constexpr (JOB == 1 || (JOB == 2 && decltype(posc)::value % 2 == 0)) sv = st.read(act);
    };
    auto swrite = [&](auto posc) {
        if constexpr (JOB == 1 || (JOB == 2 && decltype(posc)::value % 2 == 0)) st.write(sv);
    };
    typedef std::integral_constant<int, 0> J0;
    typedef std::integral_constant<int, 1> J1;
    typedef std::integral_constant<int, 2> J2;
    typedef std::integral_constant<int, 3> J3;
    F A0[NA], A1[NA], A2[NA], A3[NA], B0[PT], B1[PT];
    if constexpr (sizeof(F) * NA > 32) {
        // wide row blocks (bf16, NA > 2): a 2-deep ring keeps the kernel inside 256 VGPRs
        ldA(A0, 0);
        ldA(A1, 1);
        ldB(B0, 0);
        int k = 0;
        for (; k + 2 <= nk; k += 2) {
            sread(J0());
            ldB(B1, k + 1);
            __builtin_amdgcn_sched_barrier(0);
            mma(A0, B0);
            __builtin_amdgcn_sched_barrier(0);
            ldA(A0, k + 2);
            swrite(J0());
            sread(J1());
            ldB(B0, k + 2);
            __builtin_amdgcn_sched_barrier(0);
            mma(A1, B1);
            __builtin_amdgcn_sched_barrier(0);
            ldA(A1, k + 3);
            swrite(J1());
        }
        if (k < nk) mma(A0, B0);
        if constexpr (JOB) st.flush(act);
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
        sread(J0());
        ldB(B1, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(A0, B0);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A0, k + 4);
        swrite(J0());
        sread(J1());
        ldB(B0, k + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(A1, B1);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A1, k + 5);
        swrite(J1());
        sread(J2());
        ldB(B1, k + 3);
        __builtin_amdgcn_sched_barrier(0);
        mma(A2, B0);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A2, k + 6);
        swrite(J2());
        sread(J3());
        ldB(B0, k + 4);
        __builtin_amdgcn_sched_barrier(0);
        mma(A3, B1);
        __builtin_amdgcn_sched_barrier(0);
        ldA(A3, k + 7);
        swrite(J3());
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
    if constexpr (JOB) st.flush(act);
}

// Accumulators start at the bias of their output row when `bias` is given (so the epilogue does
// not add it), else at zero.
template <class P, int RT, int PT, int NW = 4>
MARF_DEV void gemm_tile(f32x16 (&acc)[RT][PT], const typename P::T* __restrict__ W, int K, int n_rt,
                        const typename P::T* act, int lda, int wave, int lane, const float* bias,
                        TileStore<typename P::T>& st) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        f32x16 init = (f32x16){};
        const int rt = wave + NW * i;
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
    int na = (n_rt - wave + NW - 1) / NW;
    na = na < 0 ? 0 : (na > RT ? RT : na);
    // The saved tile's stores go out after the GEMM instead of between its weight-fragment loads:
    // vmcnt retires in issue order, so each fragment wait also waited for the stores issued before
    // it.  Same bits; C5 (8-wave block) 80.7 -> 66.7 ms, plain bf16 at C3 (4-wave) 5.21 -> 5.07 ms
    // (profiles/r4w, r4x).  The stores drain during the epilogue, which loads nothing.
    switch (na) {
        case 1: gemm_rows<P, 1, RT, PT, 0, NW>(acc, W, K, act, lda, wave, lane, st); break;
        case 2: gemm_rows<P, 2, RT, PT, 0, NW>(acc, W, K, act, lda, wave, lane, st); break;
        case 3: if constexpr (RT >= 3) gemm_rows<P, 3, RT, PT, 0, NW>(acc, W, K, act, lda, wave, lane, st); break;
        case 4: if constexpr (RT >= 4) gemm_rows<P, 4, RT, PT, 0, NW>(acc, W, K, act, lda, wave, lane, st); break;
        default: break;
    }
    if (st.active) st.flush(act);
}

// Store 4 consecutive rows (features) of one accumulator group for this lane's pixel.
template <class P>
MARF_DEV void store4(typename P::T* dst, float x0, float x1, float x2, float x3) {
    if constexpr (sizeof(typename P::T) == 2) {
        uint2 v;  // one packed RNE conversion per pair
        v.x = P::pk2(x0, x1);
        v.y = P::pk2(x2, x3);
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


// Save the LDS tile to global: bf16 tiles stream during the GEMM that follows (job handed to
// gemm_tile), fp32 tiles (unaligned LDS rows) are copied right away (job left idle).
template <class P, int NW = 4>
MARF_DEV void save_tile(TileStore<typename P::T>& job, const typename P::T* act, int lda, int rows, int cols,
                        typename P::T* dst, int nk_next, int rmode = 0) {
    if constexpr (sizeof(typename P::T) == 2) {
        const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        job.init(lda, dst, cols, rows, cols, wave, lane, NW);
    } else {
        copy_tile_out<P>(act, lda, rows, cols, dst, cols, rmode);  // (rmode: MARF_DIAG_RT experiments)
        job.clear();
    }
}

// ======================================================================== per-tile phases

// BARF coarse-to-fine weight of every band into LDS (model/planar.py:462-470); 1 without c2f.
MARF_DEV void c2f_weights_lds(const C2fDev& c2f, int L, float* wsh) {
    if ((int)threadIdx.x < L)
        wsh[threadIdx.x] = c2f.on ? c2f_weight(*c2f.progress, c2f.start, c2f.span, L, threadIdx.x) : 1.0f;
}

// Prologue: pixel grid -> sl(3) warp -> posenc (+c2f) of the tile's TP slots -> act [TP][Kp0]
// (warp.py:33-81, model/planar.py:451-471; feature layout [u, v, sin_k(u), cos_k(u), sin_k(v),
// cos_k(v)], zero padded to Kp0).  NPART = 64 NW / TP threads share a pixel: half of them take u,
// half v, each a contiguous run of bands, written as bf16 pairs (one 4-byte LDS store per pair).
// c0: the first column (a skip layer's posenc block, written again at column Mp[l-1]; even).
template <class P, int TP, bool GRID_ONLY = false, int NW = 4>
MARF_DEV void tile_prologue(const NetDev& net, const GeoDev& geo, int c2f_on, const float* wsh,
                            typename P::T* act, int lda, int b, int p0, int c0 = 0) {
    typedef typename P::T T;
    constexpr int NPART = 64 * NW / TP, HALF = NPART / 2;
    const int L = net.L;
    const int i = threadIdx.x % TP, part = threadIdx.x / TP;
    float x, y, u = 0.f, v = 0.f, X[3];
    slot_point<GRID_ONLY>(geo, b, p0 + i, x, y, u, v, X);
    T* row = act + (size_t)i * lda + c0;
    auto put2 = [&](int col, float a0, float a1) {  // col even
        if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint32_t*>(row + col) = P::pk2(a0, a1);
        } else {
            row[col] = a0;
            row[col + 1] = a1;
        }
    };
    if (part == NPART - 1) put2(0, MARF_DIAG_ROUND(u, net.diag[0], 2), MARF_DIAG_ROUND(v, net.diag[0], 2));
    if (L > 0) {
        const int c = part / HALF, sub = part - c * HALF;
        const float cv = c ? v : u;
        const int k0 = sub * L / HALF, k1 = (sub + 1) * L / HALF;
        const int cs = 2 + 2 * c * L, cc = cs + L;  // first sin / cos column of coordinate c
        int k = k0;
        auto band = [&](int kk, float& sv, float& cvv) {
            band_sincos<sizeof(T) == 2>(cv, kk, sv, cvv);
            if (c2f_on) {
                const float w = wsh[kk];
                sv = sv * w;
                cvv = cvv * w;
            }
            sv = MARF_DIAG_ROUND(sv, net.diag[0], 2);
            cvv = MARF_DIAG_ROUND(cvv, net.diag[0], 2);
        };
        if ((k & 1) && k < k1) {  // odd start: single band
            float s0, c0;
            band(k, s0, c0);
            row[cs + k] = P::cvt(s0);
            row[cc + k] = P::cvt(c0);
            ++k;
        }
        for (; k + 1 < k1; k += 2) {
            float s0, c0, s1, c1;
            band(k, s0, c0);
            band(k + 1, s1, c1);
            if ((cs & 1) == 0) {
                put2(cs + k, s0, s1);
            } else {
                row[cs + k] = P::cvt(s0);
                row[cs + k + 1] = P::cvt(s1);
            }
            if (((cc + k) & 1) == 0) {
                put2(cc + k, c0, c1);
            } else {
                row[cc + k] = P::cvt(c0);
                row[cc + k + 1] = P::cvt(c1);
            }
        }
        if (k < k1) {
            float s0, c0;
            band(k, s0, c0);
            row[cs + k] = P::cvt(s0);
            row[cc + k] = P::cvt(c0);
        }
    }
    for (int f = net.D + 2 * part; f < net.Kp[0]; f += 2 * NPART) put2(f, 0.f, 0.f);  // D, Kp0 even
}

// ReLU mask records: one uint4 per lane per (tile, layer) at ((tile * 4 + wave) * 64 + lane), i.e.
// one contiguous 1 KB wave burst.  The RT x PT accumulator tiles of a wave are numbered
// ti = i * PT + j (<= 8); tile ti's 16 bits live in word ti >> 1, bits 16 (1 - (ti & 1)) + 15 - r
// for accumulator register r.  The dgrad epilogue of the backward finds the same (feature, pixel)
// in the same wave / lane / register (gemm_tile deals row tiles identically for W and W^T).
MARF_DEV uint4* mask_record(uint64_t* mk, int tile, int wave, int lane, int nw = 4) {
    return reinterpret_cast<uint4*>(mk) + ((size_t)tile * nw + wave) * 64 + lane;
}

// Hidden-layer epilogue: ReLU of the accumulators (bias already in them) written back to act in
// place, and (mk != null) the ReLU mask record of this wave.  Per element: v_cmp (vcc = z > 0),
// v_cndmask (relu), v_addc (shift the bit into the tile's mask word).
template <class P, int RT, int PT, int NW = 4>
MARF_DEV void relu_epilogue(f32x16 (&acc)[RT][PT], typename P::T* act, int lda, int n_rt, int wave, int lane,
                            uint64_t* mk, int tile, unsigned diag_next = 0) {
    static_assert(RT * PT <= 8, "a wave's ReLU mask record holds 8 accumulator tiles of 16 bits");
    (void)diag_next;  // (the next layer's rounding code: MARF_DIAG_RT builds)
    uint32_t words[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int rt = wave + NW * i;
        if (rt >= n_rt) continue;
        const int rbase = rt * 32 + 4 * (lane >> 5);
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int ti = i * PT + j;
            const int px = j * 32 + (lane & 31);
            float o[16];
            uint32_t bits = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v;
                asm volatile(
                    "v_cmp_lt_f32_e32 vcc, 0, %2\n\t"
                    "v_cndmask_b32_e32 %0, 0, %2, vcc\n\t"
                    "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
                    : "=&v"(v), "+v"(bits)
                    : "v"(acc[i][j][r])
                    : "vcc");
                o[r] = v;
                o[r] = MARF_DIAG_ROUND(o[r], diag_next, 2);
            }
            words[ti >> 1] |= bits << (16 * (1 - (ti & 1)));
#pragma unroll
            for (int q = 0; q < 4; ++q)
                store4<P>(act + (size_t)px * lda + rbase + 8 * q, o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        }
    }
    if (mk) *mask_record(mk, tile, wave, lane, NW) = make_uint4(words[0], words[1], words[2], words[3]);
}

// Dgrad epilogue: dz = acc * relu'(feat) with this wave's mask record `mw` (loaded before the GEMM),
// written to act.  Per element: v_bfe_i32 (0 / -1 from the bit) and v_and.
template <class P, int RT, int PT, int NW = 4>
MARF_DEV void mask_epilogue(f32x16 (&acc)[RT][PT], typename P::T* act, int lda, int n_rt, int wave, int lane,
                            uint4 mw, unsigned diag_out = 0) {
    static_assert(RT * PT <= 8, "a wave's ReLU mask record holds 8 accumulator tiles of 16 bits");
    (void)diag_out;  // (the rounding code of the layer whose output gradient this is: MARF_DIAG_RT)
    const uint32_t words[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int rt = wave + NW * i;
        if (rt >= n_rt) continue;
        const int rbase = rt * 32 + 4 * (lane >> 5);
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int ti = i * PT + j;
            const int px = j * 32 + (lane & 31);
            const uint32_t w = words[ti >> 1];
            float o[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = __builtin_amdgcn_sbfe((int)w, 16 * (1 - (ti & 1)) + 15 - r, 1);
                o[r] = __int_as_float(__float_as_int(acc[i][j][r]) & m);
                o[r] = MARF_DIAG_ROUND(o[r], diag_out, 3);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                store4<P>(act + (size_t)px * lda + rbase + 8 * q, o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        }
    }
}

// Skip layer's dgrad rows past its feature input (rows rt_lo * 32 .. n_rt * 32 = the posenc block,
// model/planar.py:440-441): no ReLU, the gradient of the posenc features, added into the fp32
// accumulator dsk [TP][Kp0] (one (pixel, feature) per lane and register: no two lanes share one).
template <class P, int RT, int PT, int NW = 4>
MARF_DEV void skip_epilogue(const f32x16 (&acc)[RT][PT], float* dsk, int kp0, int rt_lo, int n_rt, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int rt = wave + NW * i;
        if (rt < rt_lo || rt >= n_rt) continue;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int px = j * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = (rt - rt_lo) * 32 + acc_row(lane, r);
                dsk[(size_t)px * kp0 + f] += acc[i][j][r];
            }
        }
    }
}

// LDS byte offset of the skip accumulator dsk: past the activation tile and the fp32 df image
template <class P, int TP>
MARF_DEV int skip_lds_off(const NetDev& net, int lda) {
    const int a = TP * lda * (int)sizeof(typename P::T), d = TP * (net.Kp[0] + 1) * 4;
    return ((a > d ? a : d) + 15) & ~15;
}

// One dgrad layer of the tile kernels: dz_l = (W_l^T dz_{l+1}) * relu'(feat_l) into act (the ReLU
// record of feat_l), and for a skip layer the posenc rows into dsk.  acc holds the GEMM.
template <class P, int RT, int PT, int NW = 4>
MARF_DEV void dgrad_epilogue(f32x16 (&acc)[RT][PT], const NetDev& net, int l, typename P::T* act, int lda, int wave,
                             int lane, uint4 mw, float* dsk) {
    const int R = net.Kp[l];
    if (dsk && ((net.skip >> l) & 1u)) {  // (dsk: null in kernels built without skip support)
        mask_epilogue<P, RT, PT, NW>(acc, act, lda, net.Mp[l - 1] / 32, wave, lane, mw, net.diag[l - 1]);
        skip_epilogue<P, RT, PT, NW>(acc, dsk, net.Kp[0], net.Mp[l - 1] / 32, R / 32, wave, lane);
    } else {
        mask_epilogue<P, RT, PT, NW>(acc, act, lda, R / 32, wave, lane, mw, net.diag[l - 1]);
    }
}

// Layer-0 dgrad (d feat_0 = W_0^T dz_1, act holds dz_1) and the posenc / projective-warp adjoint
// (model/planar.py:451-471, warp.py:74-78 backward): per slot d(u, v), then for the grid geometry
// d(Hx) and one dH[3x3] partial per tile (fixed-order wave + block sums); for explicit coordinates
// d coords.  `red` needs 64 NW * 2 floats, `red9` NW * 9.  smem = the act tile (reused as fp32).
// dsk: the skip layers' posenc gradient ([TP][Kp0] fp32, added to d feat_0), or null.
template <class P, int TP, bool GRID_ONLY = false, int NW = 4>
MARF_DEV void warp_adjoint(const NetDev& net, const GeoDev& geo, int c2f_on, const float* wsh, char* smem, int lda,
                           int wave, int lane, int b, int p0, float* red, float* red9, float* dH_partial,
                           float* d_coords, TileStore<typename P::T>& st, unsigned long long* sp = nullptr,
                           const float* dsk = nullptr) {
    typedef typename P::T T;
    constexpr int PT = TP / 32;
    constexpr int RT = 8 / PT;
    const int L = net.L;
    const T* act = reinterpret_cast<const T*>(smem);
    const int R = net.Kp[0], Kk = net.Mt[0], n_rt = R / 32;
    f32x16 acc[RT][PT];
    gemm_tile<P, RT, PT, NW>(acc, reinterpret_cast<const T*>(net.Wt[0]), Kk, n_rt, act, lda, wave, lane, nullptr, st);
    __syncthreads();
    MARF_STAMP(sp, 16);
    float* df = reinterpret_cast<float*>(smem);
    const int ldf = R + 1;
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int rt = wave + NW * i;
        if (rt >= n_rt) continue;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int px = j * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) df[(size_t)px * ldf + rt * 32 + acc_row(lane, r)] = acc[i][j][r];
        }
    }
    __syncthreads();
    if (dsk) {  // points_enc feeds layer 0 and every skip layer: its gradient is their sum
        for (int e = threadIdx.x; e < TP * R; e += 64 * NW) {
            const int px = e / R, c = e - px * R;
            df[(size_t)px * ldf + c] += dsk[e];
        }
        __syncthreads();
    }
    MARF_STAMP(sp, 17);

    // posenc adjoint: d coord_c = df[c] + sum_k w_k f_k (cos(x_k) df_sin - sin(x_k) df_cos)
    constexpr int NPART = 64 * NW / TP;
    const int i = threadIdx.x % TP, part = threadIdx.x / TP;
    float x, y, u = 0.f, v = 0.f, X[3] = {0.f, 0.f, 1.f};
    const bool valid = slot_point<GRID_ONLY>(geo, b, p0 + i, x, y, u, v, X);
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
        if (c2f_on) {
            const float w = wsh[k];
            gs = gs * w;
            gc = gc * w;
        }
        float dspec = gs * co - gc * s;
        float d = dspec * ldexpf(3.14159265358979323846f, k);
        if (c == 0) du += d; else dv += d;
    }
    red[(part * TP + i) * 2] = du;
    red[(part * TP + i) * 2 + 1] = dv;
    __syncthreads();
    MARF_STAMP(sp, 18);
    float h9[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) h9[e] = 0.f;
    if ((int)threadIdx.x < TP) {
        du = red[i * 2];
        dv = red[i * 2 + 1];
        for (int q = 1; q < NPART; ++q) {
            du += red[(q * TP + i) * 2];
            dv += red[(q * TP + i) * 2 + 1];
        }
        if (geo.mode == 1) {
            if (valid && d_coords) {
                d_coords[2 * (size_t)(p0 + i)] = du;
                d_coords[2 * (size_t)(p0 + i) + 1] = dv;
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
    if (geo.mode == 0) {
#pragma unroll
        for (int e = 0; e < 9; ++e) {
            const float s = wave_total63(h9[e]);
            if (lane == 63) red9[wave * 9 + e] = s;
        }
        __syncthreads();
        if (threadIdx.x < 9) {
            float s = red9[threadIdx.x];
            for (int w = 1; w < NW; ++w) s += red9[w * 9 + threadIdx.x];
            dH_partial[(size_t)blockIdx.x * 9 + threadIdx.x] = s;
        }
    }
}

}  // namespace marf
