// marf_wgrad.hip -- weight gradients of the neural-image MLP, dW_l = sum_px dz_{l+1} (x) feat_l,
// db_l = sum_px dz_{l+1}  (autograd of nn.Linear, model/planar.py:443).
//
// A GEMM whose reduction axis is the pixel axis (K = B*h*w, millions).  Split-K: block (c, o)
// reduces pixel chunk c into a private fp32 partial of output block o; a second kernel sums the
// partials in a fixed order (deterministic, no float atomics).
//
// bf16: v_mfma_f32_32x32x16_bf16 with both operands pixel-minor.  dz and feat arrive pixel-major
// ([S][M], [S][K]), are staged 64 pixels at a time into LDS row-major, and read back with
// ds_read_b64_tr_b16 (gfx950 hardware transpose: per 16-lane group, 4 rows x 16 columns, delivered
// column-major), so a lane receives 8 consecutive pixels of one feature.  LDS rows are padded by
// 64 B so the 4 rows of a transposed read fall in distinct 64-B bank groups.
// fp32: v_mfma_f32_32x32x2_f32, one element per lane, read straight from the row-major tile.
//
// 512 threads = 8 waves as 4 (rows) x 2 (cols); each wave owns RT x CT accumulator tiles.
#include "marf_args.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace marf {

// feat_0 of the step kernel (marf_step2.hip prologue) recomputed on chip instead of read: crop
// grid -> warp -> posenc + c2f, split to the bf16 hi word, in the step kernel's column order
// (16 g + 8 h + j: band group g, coordinate h, j < 4 sin / j >= 4 cos; group nk0 - 1 the raw
// coordinate).  The same device functions and fp32 order give the same bits.
struct Feat0Src {
    GeoDev geo;         // crop grid geometry of the step (Hm: [B][9])
    const float* c2f_w; // [L] band weights of the step, or null (c2f off)
    int L, nk0;
};

struct WgArgs {
    const void* dz;    // [S][ldz] T
    const void* feat;  // [S][ldf] T (unused when feat_0 is recomputed)
    Feat0Src f0;
    long long S;
    int ldz, ldf;      // row strides
    int M, K;          // output rows (<= ldz) and cols (<= ldf)
    int chunk;         // pixels per chunk (multiple of 64)
    int n_chunks;
    int n_oblk_c;      // output blocks along K
    float* partial;    // [n_chunks][M][K]
    float* bpartial;   // [n_chunks][M] (bias), may be null
    // range mode (rng_n > 0, LDS-DMA kernel only): block c of rng_n reduces its share of the pixel
    // rows [s_lo, s_lo + s_len) (whole SP-row stages, split as evenly as they go) into partial
    // part0 + c -- one piece of a pipelined step (marf_abi.hip, step2_forward)
    long long s_lo, s_len;
    int rng_n, part0;
    int t16;           // dz / feat in the step kernel's T16 block layout (t16_off), not row-major
};

template <int RT, int CT>
struct WgGeo {
    static constexpr int BM = 4 * RT * 32;
    static constexpr int BN = 2 * CT * 32;
};

MARF_DEV i16x4 tr_read(const u16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(p));
}

// T16: the layout the split-recipe step kernel saves feat_l / dz_l in (marf_step2.hip store_rt):
// blocks of 32 pixels x 16 features (1 KB, pixel-major inside), the feature blocks of a 32-pixel
// row of tiles consecutive, so each of the step kernel's 16-B lane stores lands in one contiguous
// 1 KB per wave instruction (the row-major layout gave 32 segments of 32 B).  Element (p, f) of an
// [S][ld] tensor (S multiple of 32, ld of 16):
MARF_DEV size_t t16_off(long long p, int f, int ld) {
    return ((size_t)(p >> 5) * (size_t)(ld >> 4) + (size_t)(f >> 4)) * 512 + (size_t)(p & 31) * 16 + (f & 15);
}
// ... and in a stage of the LDS-DMA ring: the same 1 KB blocks, nb per 32-row group, as they
// stand (each DMA instruction copies one block, lanes in address order).  A row permutation that
// took the transposed reads' bank conflicts out (through the lanes' source addresses) cost more in
// the DMA than the conflicts did: hidden layers 2.61 -> 2.84 ms at C3 (profiles/r7e, same box)
MARF_DEV int t16_lds(int r, int c, int nb) {  // byte offset of (stage row r, feature c)
    const int b = c >> 4;
    return ((r >> 5) * nb + b) * 1024 + (r & 31) * 32 + (c & 15) * 2;
}

// the product of pixel chunk `chunk_id` into output block `ob` (the body of one k_wgrad block;
// also a work item of k_wgrad_fused)
template <class P, int RT, int CT, int SP>
MARF_DEV void wgrad_body(const WgArgs& a, int chunk_id, int ob, char* smem) {
    typedef typename P::T T;
    constexpr int BM = WgGeo<RT, CT>::BM, BN = WgGeo<RT, CT>::BN;
    constexpr int PADE = sizeof(T) == 2 ? 32 : 4;  // row padding (elements), keeps rows 16-B aligned
    constexpr int LDZ = BM + PADE, LDF = BN + PADE;
    constexpr int VEC = 16 / sizeof(T);          // elements per 16-byte vector
    constexpr int NVZ = SP * BM / VEC / 512;     // dz vectors per thread and stage
    constexpr int NVF = SP * BN / VEC / 512;     // feat vectors per thread and stage
    T* tz = reinterpret_cast<T*>(smem);          // [SP][LDZ]
    T* tf = tz + SP * LDZ;                        // [SP][LDF]
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int m0 = (ob / a.n_oblk_c) * BM, k0 = (ob % a.n_oblk_c) * BN;
    const long long s_begin = (long long)chunk_id * a.chunk;
    const long long s_end = min(s_begin + a.chunk, a.S);
    const bool do_bias = a.bpartial && (ob % a.n_oblk_c) == 0;
    const T* dz = reinterpret_cast<const T*>(a.dz);
    const T* ft = reinterpret_cast<const T*>(a.feat);

    f32x16 acc[RT][CT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[i][j] = (f32x16){};
    float bsum = 0.f;

    // stage s0 -> registers (16-byte vectors, zero outside the chunk / the matrix)
    uint4 rz[NVZ], rf[NVF];
    auto load_stage = [&](long long s0) {
#pragma unroll
        for (int q = 0; q < NVZ; ++q) {
            const int e = threadIdx.x + 512 * q;
            const int r = e / (BM / VEC), c = (e % (BM / VEC)) * VEC;
            rz[q] = make_uint4(0, 0, 0, 0);
            if (s0 + r < s_end && m0 + c < a.M)
                rz[q] = *reinterpret_cast<const uint4*>(dz + (a.t16 ? t16_off(s0 + r, m0 + c, a.ldz) : (size_t)((s0 + r) * a.ldz + m0 + c)));
        }
#pragma unroll
        for (int q = 0; q < NVF; ++q) {
            const int e = threadIdx.x + 512 * q;
            const int r = e / (BN / VEC), c = (e % (BN / VEC)) * VEC;
            rf[q] = make_uint4(0, 0, 0, 0);
            if (s0 + r < s_end && k0 + c < a.K)
                rf[q] = *reinterpret_cast<const uint4*>(ft + (a.t16 ? t16_off(s0 + r, k0 + c, a.ldf) : (size_t)((s0 + r) * a.ldf + k0 + c)));
        }
    };
    auto store_stage = [&]() {
#pragma unroll
        for (int q = 0; q < NVZ; ++q) {
            const int e = threadIdx.x + 512 * q;
            const int r = e / (BM / VEC), c = (e % (BM / VEC)) * VEC;
            *reinterpret_cast<uint4*>(tz + r * LDZ + c) = rz[q];
        }
#pragma unroll
        for (int q = 0; q < NVF; ++q) {
            const int e = threadIdx.x + 512 * q;
            const int r = e / (BN / VEC), c = (e % (BN / VEC)) * VEC;
            *reinterpret_cast<uint4*>(tf + r * LDF + c) = rf[q];
        }
    };

    if (s_begin < s_end) load_stage(s_begin);
    for (long long s0 = s_begin; s0 < s_end; s0 += SP) {
        __syncthreads();  // previous stage fully consumed
        store_stage();
        __syncthreads();
        if (s0 + SP < s_end) load_stage(s0 + SP);  // next stage in flight behind the MFMAs

        if (do_bias) {
            // db partial: thread t sums column t%BM over rows t/BM, t/BM + 512/BM, ...
            constexpr int RSTEP = 512 / BM > 0 ? 512 / BM : 1;
            const int c = threadIdx.x % BM, r0 = threadIdx.x / BM;
            if (r0 < RSTEP)
                for (int r = r0; r < SP; r += RSTEP) bsum += P::tof(tz[r * LDZ + c]);
        }

        if constexpr (sizeof(T) == 2) {
            const int g = lane >> 4, gi = lane & 15, q = gi >> 2, p4 = gi & 3;
#pragma unroll
            for (int ks = 0; ks < SP; ks += 16) {
                const int r0 = ks + 8 * (g >> 1) + q;  // this lane supplies row r0 (and r0 + 4)
                typename P::frag af[RT], bf[CT];
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    const int c0 = (wr * RT + i) * 32 + 16 * (g & 1) + 4 * p4;
                    const u16* base = reinterpret_cast<const u16*>(tz) + r0 * LDZ + c0;
                    i16x4 lo = tr_read(base), hi = tr_read(base + 4 * LDZ);
                    i16x4 v[2] = {lo, hi};
                    af[i] = *reinterpret_cast<typename P::frag*>(v);
                }
#pragma unroll
                for (int j = 0; j < CT; ++j) {
                    const int c0 = (wc * CT + j) * 32 + 16 * (g & 1) + 4 * p4;
                    const u16* base = reinterpret_cast<const u16*>(tf) + r0 * LDF + c0;
                    i16x4 lo = tr_read(base), hi = tr_read(base + 4 * LDF);
                    i16x4 v[2] = {lo, hi};
                    bf[j] = *reinterpret_cast<typename P::frag*>(v);
                }
#pragma unroll
                for (int i = 0; i < RT; ++i)
#pragma unroll
                    for (int j = 0; j < CT; ++j) acc[i][j] = P::mma32(af[i], bf[j], acc[i][j]);
            }
        } else {
            const int h = lane >> 5, rl = lane & 31;
            for (int ks = 0; ks < SP; ks += 2) {
                typename P::frag af[RT], bf[CT];
#pragma unroll
                for (int i = 0; i < RT; ++i) af[i] = tz[(ks + h) * LDZ + (wr * RT + i) * 32 + rl];
#pragma unroll
                for (int j = 0; j < CT; ++j) bf[j] = tf[(ks + h) * LDF + (wc * CT + j) * 32 + rl];
#pragma unroll
                for (int i = 0; i < RT; ++i)
#pragma unroll
                    for (int j = 0; j < CT; ++j) acc[i][j] = P::mma32(af[i], bf[j], acc[i][j]);
            }
        }
    }

    // ---- epilogue: partial[chunk][m][k]
    float* out = a.partial + (size_t)chunk_id * a.M * a.K;
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) {
            const int k = k0 + (wc * CT + j) * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + (wr * RT + i) * 32 + acc_row(lane, r);
                if (m < a.M && k < a.K) out[(size_t)m * a.K + k] = acc[i][j][r];
            }
        }
    if (do_bias) {
        __syncthreads();
        float* bs = reinterpret_cast<float*>(smem);
        bs[threadIdx.x] = bsum;
        __syncthreads();
        constexpr int RSTEP = 512 / BM > 0 ? 512 / BM : 1;
        if ((int)threadIdx.x < BM && m0 + (int)threadIdx.x < a.M) {
            float s = 0.f;
            for (int r = 0; r < RSTEP; ++r) s += bs[threadIdx.x + r * BM];
            a.bpartial[(size_t)chunk_id * a.M + m0 + threadIdx.x] = s;
        }
    }
}

template <class P, int RT, int CT, int SP>
__global__ __launch_bounds__(512, 1) void k_wgrad(WgArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    wgrad_body<P, RT, CT, SP>(a, blockIdx.x, blockIdx.y, smem);
}

// ---- bf16, 256 x 256 (or 256 x 96) output blocks: LDS-DMA ring
// The same product with the operands streamed HBM -> LDS by global_load_lds_dwordx4 into an
// NBUF-deep ring of SP-pixel stages, NBUF-2 stages in flight behind the one being consumed (the
// register-staged kernel above keeps one stage in flight; at one 8-wave block per CU the HBM
// stream needs more bytes in flight than that).  LDS-DMA writes lane-linear 1 KB per wave
// instruction, so the 512-B operand rows are unpadded and bank conflicts of the transposed reads are
// avoided by an XOR swizzle of the 16-B chunks, applied on the global source address:
// LDS chunk p of row r holds global chunk p ^ 4 (r & 3).  The ring spans the barriers: each thread
// retires its own stage with a counted vmcnt, then a raw s_barrier (no __syncthreads: its fence
// would drain every DMA in flight) publishes the stage to all waves.
// Issued as inline asm: hipcc tracks its own builtin LDS-DMA and waits vmcnt(0) before the next
// ds_read of the same LDS array, which would drain the ring; the asm form is outside its
// bookkeeping, and the kernel counts completion itself.  lds: wave-uniform LDS byte address.
MARF_DEV void glds16(const char* src, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}

constexpr int F0_PATCHES = 4;  // patches a layer-0 weight-gradient chunk may span (host-checked)
// Ring shapes (same-box A/B, profiles/r4g, r4h): the hidden layers read 32-row stages of dz + feat
// through a 4-deep ring (64-row stages, a 5-deep ring and non-temporal loads measured no faster);
// the layer-0 gradient, which recomputes feat_0 and moves only dz over the ring, runs 64-row stages
// 3 deep (0.65 -> 0.53 ms at C3: half the barriers per pixel).
constexpr int WG_SPH = 32, WG_NBUF_H = 4, WG_SP0 = 64, WG_NBUF_0 = 3, WG_NBUF_96 = 4;

MARF_DEV int swz(int r, int c) {  // byte offset of bf16 element (r, c) in a 256-wide swizzled stage
    return r * 512 + ((((c >> 3) ^ (4 * (r & 3)))) << 4) + (c & 7) * 2;
}


template <int N>
MARF_DEV void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// KF = feat row width (bf16): 256 (hidden layers, swizzled like dz) or 96 (layer 0 at L = 16:
// 192-B rows, the stage is one contiguous block copied linearly; rows r..r+3 of a transposed read
// sit 0/192/384/576 B apart, i.e. in four distinct 64-B bank groups, so no swizzle is needed).
template <int KF>
MARF_DEV int foff(int r, int c) {
    if constexpr (KF == 256) return swz(r, c);
    else return r * (KF * 2) + c * 2;
}

// chunk `chunk_id` into output block `ob` (the body of one k_wgrad_dma block; also a work item of
// k_wgrad_fused)
template <class P, int NBUF, int SP, int KF, bool F0 = false, bool T16 = false>
MARF_DEV void wgrad_dma_body(const WgArgs& a, int chunk_id, int ob, char* smem) {
    static_assert(KF == 256 || KF == 96, "feat width");
    static_assert(!F0 || (KF == 96 && SP % 32 == 0), "feat_0 recompute: the 96-wide layer-0 stage, 32-row blocks");
    constexpr int WR = KF == 256 ? 4 : 8, WC = 8 / WR;  // wave grid over the 256 x KF output
    constexpr int RT = 256 / 32 / WR, CT = KF / 32 / WC;
    constexpr int ZB = SP * 512;                 // bytes of the dz stage (SP rows x 256 bf16)
    constexpr int FB = SP * KF * 2;              // bytes of the feat stage
    constexpr int NGZ = ZB / 8192;               // DMA instructions per wave and stage (1 KB each)
    constexpr int NGF = F0 ? 0 : (FB + 8191) / 8192;  // (feat: the last round may be partly idle)
    static_assert(NGZ * 8192 == ZB && FB % 1024 == 0 && NBUF >= 2 && NBUF <= 6, "stage shape");
    constexpr int PER_ST = NGZ + NGF;            // vmcnt units per stage (the same on every wave)
    constexpr int STB = ZB + FB;                 // bytes of one ring slot
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave / WC, wc = wave % WC;
    const int m0 = (ob / a.n_oblk_c) * 256, k0 = (ob % a.n_oblk_c) * KF;
    long long s_begin, s_end;
    int pidx;  // the partial this block writes
    if (a.rng_n > 0) {
        const long long nst = a.s_len / SP;
        s_begin = a.s_lo + (long long)chunk_id * nst / a.rng_n * SP;
        s_end = a.s_lo + (long long)(chunk_id + 1) * nst / a.rng_n * SP;
        pidx = a.part0 + chunk_id;
    } else {
        s_begin = (long long)chunk_id * a.chunk;
        s_end = min(s_begin + a.chunk, a.S);
        pidx = chunk_id;
    }
    const int n_st = s_end > s_begin ? (int)((s_end - s_begin) / SP) : 0;  // host: multiples of SP
    const bool do_bias = a.bpartial != nullptr && k0 == 0;
    const char* dz = reinterpret_cast<const char*>(a.dz) + (size_t)m0 * 2;
    const char* ft = reinterpret_cast<const char*>(a.feat) + (size_t)k0 * 2;
    const size_t ldzb = (size_t)a.ldz * 2, ldfb = (size_t)a.ldf * 2;

    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const unsigned junk = lds0 + NBUF * STB;     // 1 KB sink for the idle feat rounds
    // F0: the patches' homographies and the band weights, staged once (plain loads, drained
    // before the ring starts: no global load inside the ring, whose waits count DMA in order)
    float* f0_h = reinterpret_cast<float*>(smem + NBUF * STB);     // [F0_PATCHES][9]
    float* f0_w = f0_h + 9 * F0_PATCHES;                           // [32]
    float* f0_uv = f0_w + 32;                                      // [NBUF + 1][SP][2] warped coordinates
    int f0_b0 = 0, f0_p0 = 0;
    float f0_inv_w = 0.f;
    if constexpr (F0) {
        const GeoDev& gg = a.f0.geo;
        f0_b0 = (int)(s_begin / gg.Np_pad);
        f0_p0 = (int)(s_begin - (long long)f0_b0 * gg.Np_pad);
        f0_inv_w = 1.0f / (float)gg.w;
        for (int e = threadIdx.x; e < 9 * F0_PATCHES; e += 512) {
            const int bb = min(f0_b0 + e / 9, gg.B - 1);
            f0_h[e] = gg.Hm[9 * (size_t)bb + e % 9];
        }
        if (threadIdx.x < 32) f0_w[threadIdx.x] = (a.f0.c2f_w && (int)threadIdx.x < a.f0.L) ? a.f0.c2f_w[threadIdx.x] : 1.0f;
        wait_vm<0>();
        __syncthreads();
    }
    // F0: the warped coordinates of a stage's SP rows (one thread per row) into uv slot
    // st % (NBUF + 1): stages 0..NBUF-1 before the ring starts, stage st + NBUF in main iteration st
    // (the slot of stage st - 1, whose feat_0 was built before an earlier barrier)
    auto warp_rows = [&](int st, int r) {
        const GeoDev& gg = a.f0.geo;
        // division-free: the chunk's first slot split once (f0_b0, f0_p0); a chunk spans at most
        // F0_PATCHES patches, and p < 2^24 keeps the float quotient within one of the row
        int p = f0_p0 + st * SP + r, bb = f0_b0;
        for (int i = 0; i < F0_PATCHES && p >= gg.Np_pad; ++i) {
            p -= gg.Np_pad;
            ++bb;
        }
        int rr = (int)((float)p * f0_inv_w);
        rr -= rr * gg.w > p;
        rr += (rr + 1) * gg.w <= p;
        const int cc = p - rr * gg.w;
        const float x = grid_coord(gg.x0 + cc, gg.W, gg.norm_w);
        const float y = grid_coord(gg.y0 + rr, gg.H, gg.norm_h);
        float u, v, X[3];
        warp_point(f0_h + 9 * min(bb - f0_b0, F0_PATCHES - 1), x, y, u, v, X, gg.bmm_small);
        f0_uv[((st % (NBUF + 1)) * SP + r) * 2] = u;
        f0_uv[((st % (NBUF + 1)) * SP + r) * 2 + 1] = v;
    };
    if constexpr (F0) {
        if ((int)threadIdx.x < SP * NBUF && (int)threadIdx.x / SP < n_st) warp_rows(threadIdx.x / SP, threadIdx.x % SP);
        __syncthreads();
    }
    // F0: one stage of feat_0 (SP = 32 rows of 96 bf16) into its ring slot: 16 threads per row, each
    // two bands of one coordinate (sin pair + cos pair) and one pair of the raw-coordinate / padding
    // columns 64..95 (the step kernel's s2_split8 hi words: v_cvt_pk_bf16_f32 of the same fp32 values).
    // Stage st's coordinates were warped before a barrier that precedes this call.
    auto compute_f0 = [&](int st, int buf_off) {
#pragma unroll
      for (int rb = 0; rb < SP; rb += 32) {
        const int r = rb + (threadIdx.x >> 4), sub = threadIdx.x & 15;
        const float u = f0_uv[((st % (NBUF + 1)) * SP + r) * 2], v = f0_uv[((st % (NBUF + 1)) * SP + r) * 2 + 1];
        char* row = smem + buf_off + r * (KF * 2);
        const int h = sub >> 3, k0 = 2 * (sub & 7);
        const float cd = h ? v : u;
        float sn[2] = {0.f, 0.f}, cs[2] = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int k = k0 + i;
            if (k < a.f0.L) {
                band_sincos<true>(cd, k, sn[i], cs[i]);
                if (a.f0.c2f_w) {
                    sn[i] = sn[i] * f0_w[k];
                    cs[i] = cs[i] * f0_w[k];
                }
            }
        }
        const int ng = a.f0.nk0 - 1;
        const int g = k0 >> 2, j = k0 & 3;
        if (g < ng) {
            *reinterpret_cast<uint32_t*>(row + 2 * (16 * g + 8 * h + j)) = P::pk2(sn[0], sn[1]);
            *reinterpret_cast<uint32_t*>(row + 2 * (16 * g + 8 * h + 4 + j)) = P::pk2(cs[0], cs[1]);
        }
        // columns 16 ng .. 95: the raw coordinates (16 ng + 8 h) and zeros, one pair per thread
        for (int c = 16 * ng + 2 * sub; c < KF; c += 32) {
            const int hc = (c - 16 * ng) >> 3;
            const float val = (c - 16 * ng) == 8 * hc && hc < 2 ? (hc ? v : u) : 0.f;
            *reinterpret_cast<uint32_t*>(row + 2 * c) = P::pk2(val, 0.f);
        }
      }
    };
    // T16 sources: 1 KB instruction seg = block seg % nb of 32-row group seg / nb, lane L its bytes
    // 16 L .. 16 L + 15 (stage-invariant: computed once per instruction slot q; a stage adds the
    // base of its 32-row group)
    auto t16_lane = [&](int ld, int blk0, int nb, int seg) -> unsigned {
        const int tr = seg / nb, b = seg - tr * nb;
        return ((unsigned)tr * (unsigned)(ld >> 4) + (unsigned)(blk0 + b)) * 1024u + (unsigned)lane * 16u;
    };
    unsigned t16z[NGZ > 0 ? NGZ : 1], t16f[NGF > 0 ? NGF : 1];
    if constexpr (T16) {
#pragma unroll
        for (int q = 0; q < NGZ; ++q) t16z[q] = t16_lane(a.ldz, m0 >> 4, 16, q * 8 + wave);
#pragma unroll
        for (int q = 0; q < NGF; ++q) t16f[q] = t16_lane(a.ldf, k0 >> 4, KF >> 4, q * 8 + wave < (FB >> 10) ? q * 8 + wave : 0);
    }
    auto issue = [&](int st) {
        const unsigned buf = lds0 + (st % NBUF) * STB;
        const long long row0 = s_begin + (long long)st * SP;
        // T16: the stage's first 32-row group (wave-uniform)
        const char* z16 = reinterpret_cast<const char*>(a.dz) + (size_t)(row0 >> 5) * (size_t)(a.ldz >> 4) * 1024;
        const char* f16 = reinterpret_cast<const char*>(a.feat) + (size_t)(row0 >> 5) * (size_t)(a.ldf >> 4) * 1024;
#pragma unroll
        for (int q = 0; q < NGZ; ++q) {
            const int seg = q * 8 + wave;         // 1 KB = 2 rows per wave instruction
            if constexpr (T16) {
                glds16(z16 + t16z[q], __builtin_amdgcn_readfirstlane(buf + seg * 1024));
                continue;
            }
            const int r = seg * 2 + (lane >> 5);
            const int c16 = (lane & 31) ^ (4 * (r & 3));
            glds16(dz + (size_t)(row0 + r) * ldzb + c16 * 16, __builtin_amdgcn_readfirstlane(buf + seg * 1024));
        }
#pragma unroll
        for (int q = 0; q < NGF; ++q) {
            const int seg = q * 8 + wave;
            if constexpr (T16) {
                const bool real = seg * 1024 < FB;
                glds16(f16 + t16f[q], __builtin_amdgcn_readfirstlane(real ? buf + ZB + seg * 1024 : junk));
            } else if constexpr (KF == 256) {
                const int r = seg * 2 + (lane >> 5);
                const int c16 = (lane & 31) ^ (4 * (r & 3));
                glds16(ft + (size_t)(row0 + r) * ldfb + c16 * 16, __builtin_amdgcn_readfirstlane(buf + ZB + seg * 1024));
            } else {
                // rows are contiguous (ldf == KF): the stage is one linear block
                const bool real = seg * 1024 < FB;
                const char* src = ft + (size_t)row0 * ldfb + (real ? seg * 1024 : 0) + lane * 16;
                glds16(src, __builtin_amdgcn_readfirstlane(real ? buf + ZB + seg * 1024 : junk));
            }
        }
        if constexpr (F0) compute_f0(st, (st % NBUF) * STB + ZB);  // after the stage's DMA is in flight
    };

    f32x16 acc[RT][CT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[i][j] = (f32x16){};
    float bsum = 0.f;

    for (int st = 0; st < NBUF - 1 && st < n_st; ++st) issue(st);
    const int g = lane >> 4, gi = lane & 15, q4 = gi >> 2, p4 = gi & 3;
    for (int st = 0; st < n_st; ++st) {
        const int ahead = min(NBUF - 2, n_st - 1 - st);  // stages issued after st, still in flight
        if (ahead >= 4) wait_vm<4 * PER_ST>();
        else if (ahead == 3) wait_vm<3 * PER_ST>();
        else if (ahead == 2) wait_vm<2 * PER_ST>();
        else if (ahead == 1) wait_vm<PER_ST>();
        else wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // every wave is past its reads of buffer (st - 1) % NBUF: refill it
        if (st + NBUF - 1 < n_st) issue(st + NBUF - 1);
        if constexpr (F0) {  // the last wave warps the rows of stage st + NBUF (one lane per row)
            if (wave == 7 && lane < SP && st + NBUF < n_st) warp_rows(st + NBUF, lane);
        }

        const char* tz = smem + (st % NBUF) * STB;
        const char* tf = tz + ZB;
        if (do_bias) {
            const int c = threadIdx.x & 255;
#pragma unroll
            for (int r = 0; r < SP; r += 2) {
                const int rr = r + (threadIdx.x >> 8);
                bsum += P::tof(*reinterpret_cast<const u16*>(tz + (T16 ? t16_lds(rr, c, 16) : swz(rr, c))));
            }
        }
#pragma unroll
        for (int ks = 0; ks < SP; ks += 16) {
            const int r0 = ks + 8 * (g >> 1) + q4;  // rows r0 and r0 + 4 (same r & 3)
            typename P::frag af[RT], bf[CT];
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const int c = (wr * RT + i) * 32 + 16 * (g & 1) + 4 * p4;
                const u16* base = reinterpret_cast<const u16*>(tz + (T16 ? t16_lds(r0, c, 16) : swz(r0, c)));
                const u16* base4 = T16 ? reinterpret_cast<const u16*>(tz + t16_lds(r0 + 4, c, 16)) : base + 4 * 256;
                i16x4 v[2] = {tr_read(base), tr_read(base4)};
                af[i] = *reinterpret_cast<typename P::frag*>(v);
            }
#pragma unroll
            for (int j = 0; j < CT; ++j) {
                const int c = (wc * CT + j) * 32 + 16 * (g & 1) + 4 * p4;
                // (F0: the recomputed feat_0 keeps its own row layout)
                constexpr bool FT = T16 && !F0;
                const u16* base = reinterpret_cast<const u16*>(tf + (FT ? t16_lds(r0, c, KF >> 4) : foff<KF>(r0, c)));
                const u16* base4 = FT ? reinterpret_cast<const u16*>(tf + t16_lds(r0 + 4, c, KF >> 4)) : base + 4 * KF;
                i16x4 v[2] = {tr_read(base), tr_read(base4)};
                bf[j] = *reinterpret_cast<typename P::frag*>(v);
            }
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int j = 0; j < CT; ++j) acc[i][j] = P::mma32(af[i], bf[j], acc[i][j]);
        }
    }

    float* out = a.partial + (size_t)pidx * a.M * a.K + (size_t)m0 * a.K + k0;
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) {
            const int k = (wc * CT + j) * 32 + (lane & 31);
            if (KF != 256 && k0 + k >= a.K) continue;  // (a 64-wide layer-0 partial from the 96-wide stage)
#pragma unroll
            for (int r = 0; r < 16; ++r) out[(size_t)((wr * RT + i) * 32 + acc_row(lane, r)) * a.K + k] = acc[i][j][r];
        }
    if (do_bias) {
        __syncthreads();  // all DMA retired (the last iteration waited vmcnt(0)) and all reads done
        float* bs = reinterpret_cast<float*>(smem);
        bs[threadIdx.x] = bsum;
        __syncthreads();
        if (threadIdx.x < 256)
            a.bpartial[(size_t)pidx * a.M + m0 + threadIdx.x] = bs[threadIdx.x] + bs[threadIdx.x + 256];
    }
}

template <class P, int NBUF, int SP, int KF, bool F0 = false, bool T16 = false>
__global__ __launch_bounds__(512, 1) void k_wgrad_dma(WgArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // (chunk, output block): wider layers (M, K multiples of 256, e.g. 512) split the output in
    // 256 x KF blocks.  The blocks sharing a chunk take ids 8 apart, i.e. the same XCD (blocks are
    // dealt to the 8 XCDs round robin), so the second read of each operand slice hits its L2.
    const int n_ob = (a.M / 256) * a.n_oblk_c;
    int chunk_id, ob;
    if (n_ob > 1 && a.n_chunks % 8 == 0) {
        const int grp = blockIdx.x / (8 * n_ob), rem = blockIdx.x % (8 * n_ob);
        chunk_id = grp * 8 + rem % 8;
        ob = rem / 8;
    } else {
        chunk_id = blockIdx.x % a.n_chunks;
        ob = blockIdx.x / a.n_chunks;
    }
    wgrad_dma_body<P, NBUF, SP, KF, F0, T16>(a, chunk_id, ob, smem);
}

// Last layer (3 outputs): dW[c][k] = sum_px g[px][c] feat[px][k], db[c] = sum_px g[px][c].
// Bandwidth-bound (reads feat_{n-1} once): each thread owns VEC consecutive features (one 16-byte
// load per pixel row) and a pixel lane; a wave covers whole rows so every load instruction is
// contiguous.  Pixel lanes are summed through LDS at the end (fixed order).
template <class P>
__global__ __launch_bounds__(256) void k_wgrad_last(const float* __restrict__ glast, const void* feat_v, long long S,
                                                    int ldf, int K, int chunk, float* partial, float* bpartial) {
    typedef typename P::T T;
    constexpr int VEC = 16 / sizeof(T);
    __shared__ float red[3072];
    __shared__ float redb[256][3];
    const T* feat = reinterpret_cast<const T*>(feat_v);
    const int ngrp = K / VEC;               // feature groups (K is a multiple of 32)
    const int lanes = 256 / ngrp;           // pixel lanes (>= 1 for K <= 256*VEC)
    const int t = threadIdx.x;
    const int fg = t % ngrp, pl = t / ngrp;
    const bool active = pl < lanes;
    const long long s_begin = (long long)blockIdx.x * chunk;
    const long long s_end = min(s_begin + chunk, S);
    float acc[VEC][3];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v][0] = acc[v][1] = acc[v][2] = 0.f;
    float b0 = 0.f, b1 = 0.f, b2 = 0.f;
    if (active) {
        long long s = s_begin + pl;
#pragma unroll 4
        for (; s < s_end; s += lanes) {
            const float4 g = *reinterpret_cast<const float4*>(glast + s * 4);
            const uint4 raw = *reinterpret_cast<const uint4*>(feat + s * ldf + fg * VEC);
            const T* f = reinterpret_cast<const T*>(&raw);
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                const float x = P::tof(f[v]);
                acc[v][0] += g.x * x;
                acc[v][1] += g.y * x;
                acc[v][2] += g.z * x;
            }
            b0 += g.x;
            b1 += g.y;
            b2 += g.z;
        }
    }
    // pixel-lane reduction through LDS, lanes added in a fixed order: red[k][c], K*3 <= 3072
    float* out = partial + (size_t)blockIdx.x * 3 * K;
    for (int lane_id = 0; lane_id < lanes; ++lane_id) {
        if (active && pl == lane_id) {
#pragma unroll
            for (int v = 0; v < VEC; ++v)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float* r = &red[(fg * VEC + v) * 3 + c];
                    *r = lane_id == 0 ? acc[v][c] : *r + acc[v][c];
                }
        }
        __syncthreads();
    }
    for (int e = t; e < K * 3; e += 256) out[(e % 3) * K + e / 3] = red[e];
    redb[t][0] = (active && fg == 0) ? b0 : 0.f;
    redb[t][1] = (active && fg == 0) ? b1 : 0.f;
    redb[t][2] = (active && fg == 0) ? b2 : 0.f;
    __syncthreads();
    if (t < 3) {
        float sb = 0.f;
        for (int i = 0; i < 256; ++i) sb += redb[i][t];
        bpartial[(size_t)blockIdx.x * 3 + t] = sb;
    }
}

// First stage of a reduction over many partials (the fused step writes one per pixel tile): group
// g sums chunks [g*per, (g+1)*per) of partial [n][E] (and bpartial [n][Eb]) into out [G][E]
// (bout [G][Eb]), in chunk order.  Coalesced over the element index.
__global__ __launch_bounds__(256) void k_fold_partials(const float* __restrict__ partial, const float* __restrict__ bpartial,
                                                       int n, int per, long long E, int Eb, float* __restrict__ out,
                                                       float* __restrict__ bout) {
    const long long e = blockIdx.x * 256LL + threadIdx.x;
    const int g = blockIdx.y;
    const int c0 = g * per, c1 = min(n, c0 + per);
    if (e < E) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        int c = c0;
        // 2 x 4 loads in flight; acc[u] still sums chunks u, u+4, u+8, ... in order
#pragma unroll 2
        for (; c + 4 <= c1; c += 4)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] += partial[(size_t)(c + u) * E + e];
        for (int u = 0; c < c1; ++c, ++u) acc[u] += partial[(size_t)c * E + e];
        out[(size_t)g * E + e] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    } else if (e < E + Eb) {
        const int eb = (int)(e - E);
        float s = 0.f;
        for (int c = c0; c < c1; ++c) s += bpartial[(size_t)c * Eb + eb];
        bout[(size_t)g * Eb + eb] = s;
    }
}


// ---- the weight gradients of a step in three launches (marf_launch_wgrad_fused)
//
// The per-layer path is 4 + 5 launches per step (three hidden layers, layer 0, five reductions),
// each with its own ramp and tail, layer 0 (sin / cos bound: it recomputes feat_0) after the hidden
// layers (HBM bound).  Here: every hidden layer's chunks in ONE launch (k_wgrad_dma_layers), layer 0
// in a concurrent launch on a second stream (its blocks take CUs as the hidden-layer blocks free
// them), then every layer's reduction in ONE launch (k_wgrad_reduce_layers).  Each block runs the
// per-layer kernels' own body for its (layer, chunk) and the reduction the arithmetic of
// k_wgrad_reduce, so every partial and every gradient is bit-identical to the per-layer path.
// (One persistent work-queue kernel holding both bodies needed 256 VGPRs and spilled; separate
// kernels keep each body's own allocation.)
constexpr int WF_MAXJ = 6;  // the pixel-per-wave step: at most 5 layers + the last-layer reduction

struct WgLayersArgs {
    WgArgs a[WF_MAXJ];
    int n_chunks;
};

template <class P, int NBUF, int SP, int KF>
__global__ __launch_bounds__(512, 1) void k_wgrad_dma_layers(WgLayersArgs la) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int l = blockIdx.x / la.n_chunks, c = blockIdx.x - l * la.n_chunks;  // layer-major
    wgrad_dma_body<P, NBUF, SP, KF, false, true>(la.a[l], c, 0, smem);  // (the step kernel's T16 tensors)
}

struct WgRedJob {
    const float* partial;
    const float* bpartial;
    int n_chunks, M, K, Mo, Ko, blk0;
    float* dW;
    float* db;
    const int* kmap;
    float post;  // exact power of two the partials carry the inverse of (1, or the fp16x2 recipe's 2^-10)
};
struct WgRedArgs {
    WgRedJob job[WF_MAXJ];
    int n_jobs;
    const float* gscale;
    const float* denom;
};

// k_wgrad_reduce's block (64 outputs x 4 chunk groups) for output block `blk` of one job
MARF_DEV void wgrad_reduce_block(const float* __restrict__ partial, const float* __restrict__ bpartial, int n_chunks,
                                 int M, int K, int Mo, int Ko, float* __restrict__ dW, float* __restrict__ db,
                                 const float* __restrict__ gscale, const float* __restrict__ denom,
                                 const int* __restrict__ kmap, int blk, float (*red)[64], float post = 1.f) {
    const long long n = (long long)Mo * Ko;
    const long long e = blk * 64LL + (threadIdx.x & 63);
    const int g = threadIdx.x >> 6;
    const int c0 = (int)((long long)n_chunks * g / 4), c1 = (int)((long long)n_chunks * (g + 1) / 4);
    float s = 0.f;
    if (e < n + Mo) {
        const float* src;
        size_t stride;
        if (e < n) {
            const int m = (int)(e / Ko), k = (int)(e % Ko);
            // kmap: column of true input feature k in the partial (the step2 layer-0 layout)
            src = partial + (size_t)m * K + (kmap ? kmap[k] : k);
            stride = (size_t)M * K;
        } else {
            src = bpartial + (e - n);
            stride = (size_t)M;
        }
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += src[(size_t)(c + u) * stride];
        }
        for (int u = 0; c < c1; ++c, ++u) acc[u] += src[(size_t)c * stride];
        s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    red[g][threadIdx.x & 63] = s;
    __syncthreads();
    if (g == 0 && e < n + Mo) {
        float t = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
        // fused step: the partials carry the unit-upstream gradient without 1/denominator
        if (gscale) t = t * (gscale[0] / denom[0]);
        if (post != 1.f) t = t * post;  // (exact: a power of two)
        if (e < n) dW[e] = t;
        else db[e - n] = t;
    }
}

__global__ __launch_bounds__(256) void k_wgrad_reduce_layers(WgRedArgs r) {
    __shared__ float red[4][64];
    int j = 0;
    while (j < r.n_jobs - 1 && (int)blockIdx.x >= r.job[j + 1].blk0) ++j;
    const WgRedJob& q = r.job[j];
    wgrad_reduce_block(q.partial, q.bpartial, q.n_chunks, q.M, q.K, q.Mo, q.Ko, q.dW, q.db, r.gscale, r.denom, q.kmap,
                       (int)blockIdx.x - q.blk0, red, q.post);
}

// Fixed-order sum of the chunk partials into the flat fp32 gradient (nn.Linear layout [M][K],
// unpadded [Mo][Ko]), then the bias, optionally times gscale / denom (device scalars).  Block = 64
// outputs x 4 chunk groups; group g sums chunks [g*n/4, (g+1)*n/4) with independent loads in
// flight, the 4 group sums are added in order (wgrad_reduce_block).
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ partial,
                                                      const float* __restrict__ bpartial, int n_chunks, int M, int K,
                                                      int Mo, int Ko, float* __restrict__ dW, float* __restrict__ db,
                                                      const float* __restrict__ gscale, const float* __restrict__ denom,
                                                      const int* __restrict__ kmap, float post) {
    __shared__ float red[4][64];
    wgrad_reduce_block(partial, bpartial, n_chunks, M, K, Mo, Ko, dW, db, gscale, denom, kmap, blockIdx.x, red, post);
}

}  // namespace marf

using namespace marf;

template <class P, int RT, int CT>
static hipError_t launch_wg(const WgArgs& a, int n_chunks, int n_oblk, hipStream_t s) {
    typedef typename P::T T;
    constexpr int SP = 64;  // pixels per stage (128 measured slower: register pressure / spills)
    constexpr int BM = WgGeo<RT, CT>::BM, BN = WgGeo<RT, CT>::BN;
    constexpr int PADE = sizeof(T) == 2 ? 32 : 4;
    size_t lds = (size_t)SP * (BM + PADE + BN + PADE) * sizeof(T);
    if (lds < 512 * sizeof(float)) lds = 512 * sizeof(float);
    {
        hipError_t e = ensure_dynamic_lds((const void*)k_wgrad<P, RT, CT, SP>, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_wgrad<P, RT, CT, SP>), dim3(n_chunks, n_oblk), dim3(512), lds, s, a);
    return hipGetLastError();
}

static bool wgrad_dma_enabled() {
    const char* e = getenv("MARF_WGRAD_DMA");  // A/B switch (read per launch): 0 = register-staged kernel
    return !(e && e[0] == '0');
}

template <class P, int KF, bool F0 = false, bool T16 = false>
static hipError_t launch_wg_dma(WgArgs a, int n_chunks, hipStream_t s) {
    a.n_chunks = n_chunks;
    a.n_oblk_c = (a.K + KF - 1) / KF;
    constexpr int SP = F0 ? WG_SP0 : KF == 256 ? WG_SPH : 32;
    constexpr int NBUF = KF == 256 ? WG_NBUF_H : F0 ? WG_NBUF_0 : WG_NBUF_96;  // ring depth within 160 KB of LDS
    const size_t lds = (size_t)NBUF * SP * (512 + KF * 2) + (KF == 256 ? 0 : 1024) + (F0 ? (9 * F0_PATCHES + 32 + (NBUF + 1) * SP * 2) * 4 : 0);
    {
        hipError_t e = ensure_dynamic_lds((const void*)k_wgrad_dma<P, NBUF, SP, KF, F0, T16>, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_wgrad_dma<P, NBUF, SP, KF, F0, T16>), dim3(n_chunks * (a.M / 256) * a.n_oblk_c), dim3(512), lds, s,
                       a);
    return hipGetLastError();
}

// Picks the output-block shape for an M x K weight gradient: 256x256 (2x4 tiles per wave),
// 256x64 (2x1) or 128x64 (1x1).
hipError_t marf_launch_wgrad(int dtype, const void* dz, int ldz, const void* feat, int ldf, long long S, int M, int K,
                             int chunk, int n_chunks, float* partial, float* bpartial, hipStream_t s,
                             const WgRange* rng, bool t16) {
    WgArgs a;
    memset(&a, 0, sizeof(a));
    a.t16 = t16 ? 1 : 0;
    if (rng) {
        a.s_lo = rng->s_lo;
        a.s_len = rng->s_len;
        a.rng_n = n_chunks = rng->n;
        a.part0 = rng->part0;
        chunk = 64;  // (a multiple of every stage height the range mode splits at)
    }
    a.dz = dz;
    a.feat = feat;
    a.S = S;
    a.ldz = ldz;
    a.ldf = ldf;
    a.M = M;
    a.K = K;
    a.chunk = chunk;
    a.partial = partial;
    a.bpartial = bpartial;
    int cfg;
    if (M >= 256 && K >= 192) cfg = 0;       // 256 x 256 (2 x 4 tiles per wave)
    else if (M >= 256 && K > 64) cfg = 3;    // 256 x 128 (2 x 2): layer 0 at L = 16 reads dz once
    else if (M >= 256) cfg = 1;              // 256 x 64  (2 x 1)
    else cfg = 2;                            // 128 x 64  (1 x 1)
    int BM = cfg == 2 ? 128 : 256, BN = cfg == 0 ? 256 : (cfg == 3 ? 128 : 64);
    int nr = (M + BM - 1) / BM, nc = (K + BN - 1) / BN;
    a.n_oblk_c = nc;
    // LDS-DMA ring: 256-wide dz with a 256-wide (hidden) or 96-wide (layer 0, L = 16) feat
    const bool dma = M % 256 == 0 && ldz % 8 == 0 && ldz >= M && S % 32 == 0 && chunk % 32 == 0 &&
                     (long long)n_chunks * (M / 256) * ((K + 255) / 256) <= 0x7fffffff && wgrad_dma_enabled();
    const bool dma256 = dma && K % 256 == 0 && ldf % 8 == 0 && ldf >= K && S % WG_SPH == 0 && chunk % WG_SPH == 0,
               dma96 = dma && K == 96 && ldf == 96;
    if (rng && (dtype == 0 || !(dma256 || dma96))) return hipErrorInvalidValue;  // range mode: LDS-DMA kernel only
    if (t16 && dtype == 0) return hipErrorInvalidValue;  // (T16: 16-bit tensors of the step kernel only)
    if (dtype == 1) {
        if (dma256) return t16 ? launch_wg_dma<PrecBF16, 256, false, true>(a, n_chunks, s) : launch_wg_dma<PrecBF16, 256>(a, n_chunks, s);
        if (dma96) return t16 ? launch_wg_dma<PrecBF16, 96, false, true>(a, n_chunks, s) : launch_wg_dma<PrecBF16, 96>(a, n_chunks, s);
        if (cfg == 0) return launch_wg<PrecBF16, 2, 4>(a, n_chunks, nr * nc, s);
        if (cfg == 3) return launch_wg<PrecBF16, 2, 2>(a, n_chunks, nr * nc, s);
        if (cfg == 1) return launch_wg<PrecBF16, 2, 1>(a, n_chunks, nr * nc, s);
        return launch_wg<PrecBF16, 1, 1>(a, n_chunks, nr * nc, s);
    }
    if (dtype == 2) {
        if (dma256) return t16 ? launch_wg_dma<PrecF16, 256, false, true>(a, n_chunks, s) : launch_wg_dma<PrecF16, 256>(a, n_chunks, s);
        if (dma96) return t16 ? launch_wg_dma<PrecF16, 96, false, true>(a, n_chunks, s) : launch_wg_dma<PrecF16, 96>(a, n_chunks, s);
        if (cfg == 0) return launch_wg<PrecF16, 2, 4>(a, n_chunks, nr * nc, s);
        if (cfg == 3) return launch_wg<PrecF16, 2, 2>(a, n_chunks, nr * nc, s);
        if (cfg == 1) return launch_wg<PrecF16, 2, 1>(a, n_chunks, nr * nc, s);
        return launch_wg<PrecF16, 1, 1>(a, n_chunks, nr * nc, s);
    }
    if (cfg == 0) return launch_wg<PrecF32, 2, 4>(a, n_chunks, nr * nc, s);
    if (cfg == 3) return launch_wg<PrecF32, 2, 2>(a, n_chunks, nr * nc, s);
    if (cfg == 1) return launch_wg<PrecF32, 2, 1>(a, n_chunks, nr * nc, s);
    return launch_wg<PrecF32, 1, 1>(a, n_chunks, nr * nc, s);
}

// The range mode (WgRange) runs on the LDS-DMA kernel only: true if an M x K gradient with these
// strides takes it (bf16 / fp16; marf_launch_wgrad's dma256 / dma96 conditions).
bool marf_wgrad_range_ok(int dtype, int M, int ldz, int K, int ldf) {
    if (dtype != 1 && dtype != 2) return false;
    if (!(M % 256 == 0 && ldz % 8 == 0 && ldz >= M && wgrad_dma_enabled())) return false;
    return (K % 256 == 0 && ldf % 8 == 0 && ldf >= K) || (K == 96 && ldf == 96);
}

// Layer-0 weight gradient with feat_0 recomputed on chip (step kernel's feat0_recompute); bf16,
// 256-wide layer 0, the 64-wide feat_0 of L <= 12 or the 96-wide one of L = 13..16 (both built in
// the 96-wide stage, whose 192-B rows keep the transposed reads conflict-free; a 64-wide partial
// takes its first 64 columns).  False if the shape does not qualify.
bool marf_wgrad_l0_recompute_ok(int M, int ldz, int ldf0, long long S, int chunk, int n_chunks, long long Np_pad) {
    return M == 256 && ldz % 8 == 0 && ldz >= M && (ldf0 == 96 || ldf0 == 64) && S % WG_SP0 == 0 && chunk % WG_SP0 == 0 &&
           (long long)n_chunks <= 0x7fffffff && Np_pad < (1 << 24) && (chunk + Np_pad - 1) / Np_pad + 1 <= F0_PATCHES;
}

hipError_t marf_launch_wgrad_l0_recompute(const void* dz, int ldz, const GeoDev& geo, const float* c2f_w, int L,
                                          int nk0, int K0, long long S, int M, int chunk, int n_chunks, float* partial,
                                          float* bpartial, hipStream_t s, const WgRange* rng, int dtype) {
    WgArgs a;
    memset(&a, 0, sizeof(a));
    if (rng) {
        a.s_lo = rng->s_lo;
        a.s_len = rng->s_len;
        a.rng_n = n_chunks = rng->n;
        a.part0 = rng->part0;
    }
    a.dz = dz;
    a.feat = nullptr;
    a.f0.geo = geo;
    a.f0.c2f_w = c2f_w;
    a.f0.L = L;
    a.f0.nk0 = nk0;
    a.S = S;
    a.ldz = ldz;
    a.ldf = 96;
    a.M = M;
    a.K = K0;  // partial columns: 96, or the first 64 of the 96-wide stage
    a.t16 = 1;  // dz_1 from the step kernel
    a.chunk = chunk;
    a.partial = partial;
    a.bpartial = bpartial;
    // (dtype 2: the fp16x2 recipe's dz_1 and feat_0 in fp16)
    if (dtype == 2) return launch_wg_dma<PrecF16, 96, true, true>(a, n_chunks, s);
    return launch_wg_dma<PrecBF16, 96, true, true>(a, n_chunks, s);
}

// ---- the fused launch: hidden layers in one launch, layer 0 beside it on `s2`, one reduction launch
bool marf_wgrad_fused_ok(const WgFusedLayer* layers, int n_layers, long long S, int chunk, int n_chunks,
                         long long Np_pad) {
    if (!layers || n_layers < 1 || n_layers > WF_MAXJ || n_chunks < 1 || chunk < 64 || chunk % 64) return false;
    if (const char* e = getenv("MARF_WGRAD_FUSED")) {  // A/B switch (read per launch): 0 = per-layer launches
        if (e[0] == '0') return false;
    }
    int n_l0 = 0;
    for (int i = 0; i < n_layers; ++i) {
        const WgFusedLayer& L = layers[i];
        if (L.Mo > L.M || L.Ko > L.K || !L.partial || !L.bpartial || !L.dW || !L.db) return false;
        switch (L.kind) {
            case 0:  // k_wgrad_dma<PrecBF16, 4, 32, 256>'s one-output-block shape (marf_launch_wgrad's dma256)
                if (!(L.M == 256 && L.K == 256 && L.ldz % 8 == 0 && L.ldz >= L.M && L.ldf % 8 == 0 && L.ldf >= L.K &&
                      S % WG_SPH == 0 && chunk % WG_SPH == 0 && wgrad_dma_enabled()))
                    return false;
                break;
            case 1:  // marf_launch_wgrad_l0_recompute's shape
                if (!marf_wgrad_l0_recompute_ok(L.M, L.ldz, L.K, S, chunk, n_chunks, Np_pad)) return false;
                ++n_l0;
                break;
            case 2:  // layer 0 stored: any shape marf_launch_wgrad takes (its kernel is picked there)
                ++n_l0;
                break;
            case 3:
                if (L.n_parts < 1 || L.n_parts > 1024) return false;  // (the per-layer path folds above 1024)
                break;
            default: return false;
        }
    }
    return n_l0 <= 1;
}

hipError_t marf_launch_wgrad_fused(const WgFusedLayer* layers, int n_layers, long long S, int chunk, int n_chunks,
                                   const GeoDev& f0_geo, const float* c2f_w, int L, int nk0, const float* gscale,
                                   const float* denom, hipStream_t s, hipStream_t s2, hipEvent_t fork,
                                   hipEvent_t join, int dtype, float post) {
    hipError_t e;
    // layer 0 on s2, beside the hidden layers
    const WgFusedLayer* l0 = nullptr;
    for (int i = 0; i < n_layers; ++i)
        if (layers[i].kind == 1 || layers[i].kind == 2) l0 = &layers[i];
    if (l0) {
        if ((e = hipEventRecord(fork, s)) != hipSuccess || (e = hipStreamWaitEvent(s2, fork, 0)) != hipSuccess) return e;
        if (l0->kind == 1)
            e = marf_launch_wgrad_l0_recompute(l0->dz, l0->ldz, f0_geo, c2f_w, L, nk0, l0->K, S, l0->M, chunk, n_chunks, l0->partial,
                                               l0->bpartial, s2, nullptr, dtype);
        else
            e = marf_launch_wgrad(dtype, l0->dz, l0->ldz, l0->feat, l0->ldf, S, l0->M, l0->K, chunk, n_chunks, l0->partial,
                                  l0->bpartial, s2, nullptr, true);
        if (e != hipSuccess) return e;
        if ((e = hipEventRecord(join, s2)) != hipSuccess) return e;
    }
    // every hidden layer's chunks: one launch, layer-major blocks
    WgLayersArgs la;
    memset(&la, 0, sizeof(la));
    la.n_chunks = n_chunks;
    int nh = 0;
    for (int i = 0; i < n_layers; ++i) {
        const WgFusedLayer& Ly = layers[i];
        if (Ly.kind != 0) continue;
        WgArgs& a = la.a[nh++];
        a.dz = Ly.dz;
        a.feat = Ly.feat;
        a.S = S;
        a.ldz = Ly.ldz;
        a.ldf = Ly.ldf;
        a.M = Ly.M;
        a.K = Ly.K;
        a.chunk = chunk;
        a.n_chunks = n_chunks;
        a.n_oblk_c = 1;
        a.partial = Ly.partial;
        a.bpartial = Ly.bpartial;
        a.t16 = 1;
    }
    if (nh) {
        const size_t lds = (size_t)WG_NBUF_H * WG_SPH * (512 + 256 * 2);
        auto go = [&](auto prec) -> hipError_t {
            typedef decltype(prec) P;
            hipError_t er = ensure_dynamic_lds((const void*)k_wgrad_dma_layers<P, WG_NBUF_H, WG_SPH, 256>, lds);
            if (er != hipSuccess) return er;
            hipLaunchKernelGGL((k_wgrad_dma_layers<P, WG_NBUF_H, WG_SPH, 256>), dim3(nh * n_chunks), dim3(512), lds, s, la);
            return hipGetLastError();
        };
        e = dtype == 2 ? go(PrecF16()) : go(PrecBF16());  // (fp16x2: fp16 saved tensors)
        if (e != hipSuccess) return e;
    }
    if (l0 && (e = hipStreamWaitEvent(s, join, 0)) != hipSuccess) return e;
    // every layer's reduction: one launch, in the layers' order
    WgRedArgs r;
    memset(&r, 0, sizeof(r));
    r.n_jobs = n_layers;
    r.gscale = gscale;
    r.denom = denom;
    int blk = 0;
    for (int i = 0; i < n_layers; ++i) {
        const WgFusedLayer& Ly = layers[i];
        WgRedJob& q = r.job[i];
        q.partial = Ly.partial;
        q.bpartial = Ly.bpartial;
        q.n_chunks = Ly.kind == 3 ? Ly.n_parts : n_chunks;
        q.M = Ly.M;
        q.K = Ly.K;
        q.Mo = Ly.Mo;
        q.Ko = Ly.Ko;
        q.dW = Ly.dW;
        q.db = Ly.db;
        q.kmap = Ly.kmap;
        q.post = Ly.kind == 3 ? 1.f : post;  // (the last layer's partials: unscaled in the step kernel)
        q.blk0 = blk;
        blk += (int)(((long long)Ly.Mo * Ly.Ko + Ly.Mo + 63) / 64);
    }
    hipLaunchKernelGGL(k_wgrad_reduce_layers, dim3(blk), dim3(256), 0, s, r);
    return hipGetLastError();
}

hipError_t marf_launch_wgrad_last(int dtype, const float* glast, const void* feat, long long S, int ldf, int K, int chunk,
                                  int n_chunks, float* partial, float* bpartial, hipStream_t s) {
    if (dtype == 1)
        hipLaunchKernelGGL(k_wgrad_last<PrecBF16>, dim3(n_chunks), dim3(256), 0, s, glast, feat, S, ldf, K, chunk,
                           partial, bpartial);
    else if (dtype == 2)
        hipLaunchKernelGGL(k_wgrad_last<PrecF16>, dim3(n_chunks), dim3(256), 0, s, glast, feat, S, ldf, K, chunk,
                           partial, bpartial);
    else
        hipLaunchKernelGGL(k_wgrad_last<PrecF32>, dim3(n_chunks), dim3(256), 0, s, glast, feat, S, ldf, K, chunk,
                           partial, bpartial);
    return hipGetLastError();
}

hipError_t marf_launch_wgrad_reduce(const float* partial, const float* bpartial, int n_chunks, int M, int K, int Mo,
                                    int Ko, float* dW, float* db, hipStream_t s, const float* gscale,
                                    const float* denom, float* scratch, const int* kmap, float post) {
    if (n_chunks > 1024 && scratch) {
        // fold into G <= 256 groups first (n_chunks up to millions of partials)
        const int per = (n_chunks + 255) / 256;
        const int G = (n_chunks + per - 1) / per;
        const long long E = (long long)M * K;
        float* out = scratch;
        float* bout = scratch + (size_t)G * E;
        dim3 grid((unsigned)((E + M + 255) / 256), G);
        hipLaunchKernelGGL(k_fold_partials, grid, dim3(256), 0, s, partial, bpartial, n_chunks, per, E, M, out, bout);
        hipError_t err = hipGetLastError();
        if (err != hipSuccess) return err;
        partial = out;
        bpartial = bout;
        n_chunks = G;
    }
    long long n = (long long)Mo * Ko + Mo;
    int blocks = (int)((n + 63) / 64);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(blocks), dim3(256), 0, s, partial, bpartial, n_chunks, M, K, Mo, Ko, dW, db,
                       gscale, denom, kmap, post);
    return hipGetLastError();
}
