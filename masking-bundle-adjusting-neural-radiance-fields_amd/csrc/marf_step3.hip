// marf_step3.hip -- the fused training step of the split-bf16 recipe at TWO waves per SIMD (gfx950).
//
// Same contract and saved tensors as k_step2 (marf_step2.hip, variant 1): per pixel grid -> sl(3)
// warp -> posenc + c2f -> MLP forward (hi*hi + hi*lo + lo*hi, fp32 accumulation) -> sigmoid ->
// masked-MSE partial -> d rgb -> dgrad chain (W_hi^T dz + W_lo^T dz) -> posenc / warp adjoint
// (model/planar.py:329-391, warp.py:33-81), writing feat_l / dz_l for the weight-gradient kernels.
// What changes is the shape on the CU:
//
//   * one wave owns 16 pixels (not 32) and computes every feature of them with
//     v_mfma_f32_16x16x32_bf16: a 16-row accumulator tile holds, per lane (pixel l & 15, group
//     l >> 4), rows 4 (l >> 4) + 0..3; the pair of row tiles (2s, 2s + 1), packed to bf16 hi + lo,
//     is k-step s of the next layer's B operand as it stands (k order permuted inside the step:
//     position 8 g + j <-> feature 32 s + 4 g + j for j < 4, 32 s + 16 + 4 g + j - 4 otherwise;
//     the weights are packed in the same order, k_pack3).  Half the pixels halve the activation
//     registers (hi + lo of a 256-wide layer: 64 instead of 128), so a wave fits in 256 registers
//     and the 512-thread block (8 waves, one per CU) runs TWO waves per SIMD: while one wave waits
//     (ring, barrier, an epilogue's dependency) the other issues MFMAs.
//   * the weights stream through the same 3-slot LDS ring (one 32 KB slot = 32 rows of one layer,
//     hi then lo, filled by global_load_lds_dwordx4 two stages ahead, 4 pieces per wave).
//   * ReLU masks: 4 bits per lane and row tile, 2 words per lane and layer, in wave-private LDS.
//   * one pixel set per dgrad pass (the two-set dgrad of k_step2 is not needed at two waves per
//     SIMD: the LDS A-fragment reads of a dgrad stage are 2 KB per 2 MFMAs and wave).
//
// Memory ordering as in k_step2: all global traffic inside the tile loop is inline asm (LDS-DMA,
// stores); each wave counts the store instructions it issues per stage and waits for a ring slot
// with the vmcnt that leaves exactly the younger operations in flight.  Every counted store is
// issued by every wave (lanes with nothing to store write a private sink), so the counts hold.
#include <type_traits>

#include "marf_args.h"

namespace marf {
namespace s3 {

constexpr int PX = 16;                        // pixels per wave
constexpr int HM = 256;                       // widest hidden layer
constexpr int NKH = HM / 32;                  // k-steps (32 k) of a hidden-width operand
constexpr int NRT = HM / 16;                  // 16-row tiles of a hidden-width output
constexpr int SLOT = 32768;                   // one ring slot = one program stage
constexpr int LO = 16384;                     // byte offset of the lo fragments in a slot
constexpr int PER_DMA = 4;                    // 1 KB DMA pieces per DMA wave and stage
constexpr int NK0MAX = 5;                     // max layer-0 k-steps (L <= 32: 4 band steps + raw)
constexpr int NML = 4;                        // max ReLU layers (nl <= 5)
// wave-private LDS: g^T image (256 B), transpose scratch (1 KB), mask words [NML][2][64], dW_last [3][256]
constexpr int W_GIMG = 0, W_SCR = 256, W_MASK = 1280, W_WLA = W_MASK + NML * 2 * 64 * 4;
constexpr int WAVE_LDS = W_WLA + 3 * HM * 4;
static_assert(SLOT % (PER_DMA * 1024) == 0, "ring geometry");

}  // namespace s3

union S3Frag {
    bf16x8 f;
    uint4 u;
};

// ------------------------------------------------------------------ inline-asm memory ops

MARF_DEV void s3_glds4(const void* src, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}
typedef uint32_t s3_u32x4 __attribute__((ext_vector_type(4)));
MARF_DEV void s3_st16(void* dst, uint4 u) {
#ifdef S3_AB_NOSTORE  // timing-only A/B builds: no saved-tensor stores
    return;
#endif
    const s3_u32x4 v = {u.x, u.y, u.z, u.w};
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
template <int OFF>
MARF_DEV void s3_st16o(void* base, uint4 u) {  // 16 B at base + OFF bytes (instruction offset)
#ifdef S3_AB_NOSTORE  // timing-only A/B builds: no saved-tensor stores
    return;
#endif
    const s3_u32x4 v = {u.x, u.y, u.z, u.w};
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2\n\ts_nop 1" ::"v"(base), "v"(v), "n"(OFF) : "memory");
}
MARF_DEV void s3_st12(void* dst, float a, float b, float c) {
    typedef float f32x3 __attribute__((ext_vector_type(3)));
    f32x3 v = {a, b, c};
    asm volatile("global_store_dwordx3 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
MARF_DEV void s3_st4(void* dst, float a) {
    asm volatile("global_store_dword %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(a) : "memory");
}
template <int N>
MARF_DEV void s3_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
MARF_DEV i16x4 s3_tr16(const u16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(p));
}

template <int... I, class F>
MARF_DEV void s3_sfor_impl(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>()), ...);
}
template <int N, class F>
MARF_DEV void s3_sfor(F&& f) {
    s3_sfor_impl(std::make_integer_sequence<int, N>(), f);
}

// two floats -> packed bf16 pair (v_cvt_pk_bf16_f32, RNE)
MARF_DEV uint32_t s3_pk(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){a, b}), bf16x2));
}
MARF_DEV float s3_lo16(uint32_t w) { return __uint_as_float(w << 16); }
MARF_DEV float s3_hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
// relu as a signed-integer max with 0: exactly x > 0 ? x : +0 (negative floats and -0 are negative integers)
MARF_DEV float s3_relu(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
// 8 floats -> bf16 hi fragment + lo remainder fragment
MARF_DEV void s3_split8(const float* x, S3Frag& hi, S3Frag& lo) {
    hi.u = make_uint4(s3_pk(x[0], x[1]), s3_pk(x[2], x[3]), s3_pk(x[4], x[5]), s3_pk(x[6], x[7]));
    const uint32_t w[4] = {hi.u.x, hi.u.y, hi.u.z, hi.u.w};
    float r[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r[2 * q] = x[2 * q] - s3_lo16(w[q]);
        r[2 * q + 1] = x[2 * q + 1] - s3_hi16(w[q]);
    }
    lo.u = make_uint4(s3_pk(r[0], r[1]), s3_pk(r[2], r[3]), s3_pk(r[4], r[5]), s3_pk(r[6], r[7]));
}
// per 16-bit half of a packed bf16 pair: (half != 0) at bits 0 and 16
MARF_DEV uint32_t s3_nz_pair(uint32_t w) {
    uint32_t t;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(t) : "v"(w), "s"(0x00010001u));
    return t;
}

// forward epilogue of one 16-row accumulator tile: ReLU, bf16 hi + lo of the 4 values (x0 x1 | x2 x3),
// and the mask nibble (bits 0: x0, 1: x2, 16: x1, 17: x3), taken from the packed hi words: a value
// is passed by the ReLU exactly when its bf16 hi is non-zero, except for 0 < z < 2^-133 (a zero hi,
// as in k_step2)
struct S3Ep {
    uint32_t h0, h1, l0, l1, nib;
};
MARF_DEV S3Ep s3_fwd_ep(const f32x4& acc) {
    S3Ep e;
    const float x0 = s3_relu(acc[0]), x1 = s3_relu(acc[1]), x2 = s3_relu(acc[2]), x3 = s3_relu(acc[3]);
    e.h0 = s3_pk(x0, x1);
    e.h1 = s3_pk(x2, x3);
    e.l0 = s3_pk(x0 - s3_lo16(e.h0), x1 - s3_hi16(e.h0));
    e.l1 = s3_pk(x2 - s3_lo16(e.h1), x3 - s3_hi16(e.h1));
    e.nib = (s3_nz_pair(e.h1) << 1) | s3_nz_pair(e.h0);
    return e;
}
// dgrad epilogue: dz = acc * relu'(z) from mask word mw (row tile with nibble shift SH) -> bf16 pair words
template <int SH>
MARF_DEV uint2 s3_bwd_ep(const f32x4& acc, uint32_t mw) {
    const int m0 = __builtin_amdgcn_sbfe((int)mw, SH, 1), m2 = __builtin_amdgcn_sbfe((int)mw, SH + 1, 1);
    const int m1 = __builtin_amdgcn_sbfe((int)mw, SH + 16, 1), m3 = __builtin_amdgcn_sbfe((int)mw, SH + 17, 1);
    const float x0 = __int_as_float(__float_as_int(acc[0]) & m0), x1 = __int_as_float(__float_as_int(acc[1]) & m1);
    const float x2 = __int_as_float(__float_as_int(acc[2]) & m2), x3 = __int_as_float(__float_as_int(acc[3]) & m3);
    return make_uint2(s3_pk(x0, x1), s3_pk(x2, x3));
}

// ------------------------------------------------------------------ the kernel

// Diagnostic phase timing (MARF_STAMPS builds): wave 0 of each block sums s_memtime deltas per
// phase category (tools/step2_phases.py --kernel step3 prints them).
#ifdef MARF_STAMPS
#define S3T_BEGIN(k) const unsigned long long _t##k = __builtin_amdgcn_s_memtime()
#define S3T_END(k) tacc[k] += __builtin_amdgcn_s_memtime() - _t##k
#else
#define S3T_BEGIN(k) \
    do {         \
    } while (0)
#define S3T_END(k) \
    do {       \
    } while (0)
#endif

// NK0T: layer-0 k-steps (nb + 1 = ceil(L / 8) + 1); FULL: every hidden layer 256 wide.  Both make
// the row-tile and k-step counts compile-time (no guards, no merges of partly written operand
// arrays, which cost registers); <NK0MAX, false> is the generic instantiation.
// NWT: waves per block -- 8 (two per SIMD, 3-slot ring) or 12 (three per SIMD, 2-slot ring: a
// stage lasts long enough for its successor's DMA; 8 of the 12 waves issue it)
template <int NK0T, bool FULL, int NWT>
__global__ __launch_bounds__(64 * NWT, NWT / 4) void k_step3(Step2Args a) {
    using namespace s3;
    constexpr int NW = NWT;
    constexpr int TPX = NW * PX;
    constexpr int NSLOT = NW == 8 ? 3 : 2;
    constexpr int NDW = SLOT / (PER_DMA * 1024);  // waves that issue the ring's DMA
    static_assert(NW == 8 || NW == 12, "waves per block");
    constexpr int NK0 = NK0T;
    constexpr int NTA = 2 * (NK0 - 1) + 1;        // adjoint row tiles (max)
    constexpr int R0F = (16 / NK0) & ~1;           // layer-0 row tiles per stage (FULL)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pxl = lane & 15, grp = lane >> 4;
    const int nl = a.nl, L = a.L;
    const int nk0 = FULL ? NK0 : a.nk0, nb = nk0 - 1;

    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    float* bias_l = reinterpret_cast<float*>(smem + a.lds_bias);
    float* c2f_l = reinterpret_cast<float*>(smem + a.lds_c2f);
    S2Layer* lyr = reinterpret_cast<S2Layer*>(smem + a.lds_layers);
    auto ly_int = [&](int l, int field) -> int {
        return __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(lyr + l)[field]);
    };
    auto ly_ptr = [&](int l, int which) -> u16* {  // which 0: feat, 1: dz
        const uint32_t* q = reinterpret_cast<const uint32_t*>(lyr + l) + 6 + 2 * which;
        const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane(q[0]);
        const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(q[1]);
        return reinterpret_cast<u16*>(lo | (hi << 32));
    };
    char* wpriv = smem + a.lds_wave + wave * a.lds_wave_bytes;
    u16* gimg = reinterpret_cast<u16*>(wpriv + W_GIMG);        // [6][16] g hi / lo of the wave's pixels
    u16* scr = reinterpret_cast<u16*>(wpriv + W_SCR);          // [16 px][32 features] transpose image
    uint32_t* mkl = reinterpret_cast<uint32_t*>(wpriv + W_MASK);  // [layer][word][lane]
    float* wla = reinterpret_cast<float*>(wpriv + W_WLA);      // [3][Kl] dW_last of the wave
    float* dmy = a.dummy + (((size_t)blockIdx.x * NW + wave) * 64 + lane) * 16;  // 64-B store sink per lane
#ifdef MARF_STAMPS
    unsigned long long tacc[16] = {};
#endif

    // ---- constants into LDS (plain loads before the ring starts)
    for (int e = threadIdx.x; e < a.nbias; e += NW * 64) bias_l[e] = a.bias[e];
    if ((int)threadIdx.x < 32) c2f_l[threadIdx.x] = (int)threadIdx.x < L ? a.c2f_w[threadIdx.x] : 0.f;
    for (int e = threadIdx.x; e < nl * (int)(sizeof(S2Layer) / 4); e += NW * 64)
        reinterpret_cast<uint32_t*>(lyr)[e] = reinterpret_cast<const uint32_t*>(a.layers)[e];
    for (int e = lane; e < 3 * a.Kl; e += 64) wla[e] = 0.f;
    for (int e = lane; e < 128; e += 64) reinterpret_cast<uint32_t*>(gimg)[e] = 0u;

    const int tpp = a.geo.Np_pad / TPX;  // block tiles per patch
    const int Np = a.geo.Np;
    const int tbase = a.tile0 + (int)blockIdx.x;
    int my_tiles = 0;
    if (tbase < a.n_tiles) my_tiles = (a.n_tiles - 1 - tbase) / (int)gridDim.x + 1;
    const int nS = a.n_stages;  // stages per tile (render: the forward ones)
    const int total = my_tiles * nS;

    // ---- per-tile input DMA: target r, g, b, mask (TPX floats each) and H (9 floats)
    auto pro_buf = [&](int pb) -> float* { return reinterpret_cast<float*>(smem + a.lds_pro + pb * (4 * TPX + 64) * 4); };
    auto issue_pro = [&](int tile, int pb) {
        const int b = tile / tpp, q0 = (tile - b * tpp) * TPX;
        const unsigned base = lds0 + a.lds_pro + pb * (4 * TPX + 64) * 4;
        const int f = wave * 64 + lane;  // float index in [0, 4 TPX)
        const int ch = f / TPX, q = f - ch * TPX;
        const int p = min(q0 + q, Np - 1);
        const float* src = !a.gt ? a.pro_fallback
                           : ch < 3 ? a.gt + ((size_t)b * 3 + ch) * Np + p
                                    : (a.mask ? a.mask + (size_t)b * Np + p : a.gt + (size_t)b * 3 * Np + p);
        s3_glds4(src, __builtin_amdgcn_readfirstlane(base + wave * 256));
        s3_glds4(a.geo.Hm ? a.geo.Hm + 9 * (size_t)b + (lane < 9 ? lane : 0) : a.pro_fallback,
                 __builtin_amdgcn_readfirstlane(base + 4 * TPX * 4));
    };

    // ---- the weight ring: stage c of this block is program stage c mod nS, in slot c mod 3 (the
    //      counters wrap instead of dividing)
    int c_slot = 0;                   // slot of the next stage_begin
    int dma_stage = 0, dma_ps = 0, dma_slot = 0;  // next DMA: block stage, program stage, slot
    unsigned dma_m0 = 0;
    const char* dma_va = nullptr;
    const bool dma_wave = NDW == NW || wave < NDW;
    const char* const prog_w = a.prog + (dma_wave ? wave : 0) * PER_DMA * 1024 + lane * 16;
    const unsigned lds_w = lds0 + wave * PER_DMA * 1024;
    auto dma_arm = [&]() {
        const int ps = dma_stage < total ? dma_ps : 0;  // past the end: refill from stage 0 (never read)
        dma_m0 = __builtin_amdgcn_readfirstlane(lds_w + dma_slot * SLOT);
        dma_va = prog_w + (size_t)ps * SLOT;
        ++dma_stage;
        dma_ps = dma_ps + 1 == nS ? 0 : dma_ps + 1;
        dma_slot = dma_slot == NSLOT - 1 ? 0 : dma_slot + 1;
    };
    auto dma_piece = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
#ifdef S3_AB_NODMA  // timing-only A/B builds (wrong results): no weight DMA
        return;
#endif
        if (!dma_wave) return;
        const char* va = dma_va;
        const unsigned m = __builtin_amdgcn_readfirstlane(dma_m0);  // an SGPR even under pressure
        unsigned keep;  // m0 is reserved to the compiler: saved and restored around the piece
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off offset:%3\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(va), "s"(m), "n"(j * 1024)
                     : "memory");
    };
    auto dma_burst = [&]() { s3_sfor<PER_DMA>([&](auto jc) { dma_piece(jc); }); };
    // The DMA of stage c was issued right after the barrier of stage c - 2; younger than it are the
    // stores of stage c - 2 (st_prev), the pieces of stage c + 1 and the stores of stage c - 1 (st_cur).
    int st_cur = 0, st_prev = 0;
    auto wait_ring = [&]() {
#ifdef S3_AB_NOWAIT  // timing-only A/B builds (wrong results): no ring wait
        return;
#endif
        if constexpr (NSLOT == 2) {  // (every wave: the next tile's inputs are counted in as well)
            // 2-slot ring: the DMA of stage c went out in stage c - 1; younger: that stage's stores
            const int y = st_cur;
            if (y >= 16) s3_wait_vm<16>();
            else if (y >= 12) s3_wait_vm<12>();
            else if (y >= 8) s3_wait_vm<8>();
            else if (y >= 6) s3_wait_vm<6>();
            else if (y >= 4) s3_wait_vm<4>();
            else if (y >= 2) s3_wait_vm<2>();
            else if (y >= 1) s3_wait_vm<1>();
            else s3_wait_vm<0>();
            return;
        }
        const int y = st_prev + st_cur;
        if (y >= 16) s3_wait_vm<PER_DMA + 16>();
        else if (y >= 12) s3_wait_vm<PER_DMA + 12>();
        else if (y >= 8) s3_wait_vm<PER_DMA + 8>();
        else if (y >= 6) s3_wait_vm<PER_DMA + 6>();
        else if (y >= 4) s3_wait_vm<PER_DMA + 4>();
        else if (y >= 2) s3_wait_vm<PER_DMA + 2>();
        else s3_wait_vm<PER_DMA>();
    };
    auto stage_begin = [&]() -> const char* {
        S3T_BEGIN(0);
        wait_ring();
        st_prev = st_cur;
        st_cur = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        S3T_END(0);
        S3T_BEGIN(1);
#ifndef S3_AB_NOBAR  // timing-only A/B builds (wrong results): no stage barrier
        __builtin_amdgcn_s_barrier();
#endif
        asm volatile("" ::: "memory");
        S3T_END(1);
        S3T_BEGIN(2);
        dma_arm();  // the pieces go out beside the stage's first MFMAs (gemm's PC flag) or in a burst
        S3T_END(2);
        const char* slot = smem + c_slot * SLOT;
        c_slot = c_slot == NSLOT - 1 ? 0 : c_slot + 1;
        return slot;
    };

    if (my_tiles > 0) {
        issue_pro(tbase, 0);
        s3_sfor<NSLOT - 1>([&](auto) {
            dma_arm();
            dma_burst();
        });
    }
    s3_wait_vm<0>();
    __syncthreads();

    double lsq = 0.0, lms = 0.0;
    float bl0 = 0.f, bl1 = 0.f, bl2 = 0.f;

    auto mf = [&](f32x4& acc, const bf16x8& x, const bf16x8& y) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc, 0, 0, 0);
    };
    // one 16-row output tile over NK k-steps (nk live): MODE 1 split forward (hi.hi + hi.lo + lo.hi),
    // MODE 2 split dgrad (hi.B + lo.B).  A fragments of k-step ks at slot + ks KB (hi) and + LO (lo),
    // read two k-steps ahead.
    // PC: this GEMM is its stage's first -- the stage's DMA pieces go out beside its MFMAs (piece j
    // after k-step 2 j of an 8-k-step GEMM; after the last k-step of a shorter one), so the MFMAs
    // start right after the barrier; every store of the stage follows (the ring-wait accounting)
    auto gemm = [&](f32x4& acc, const char* slot, const S3Frag* Bh, const S3Frag* Bl, int nk, auto nk_tag, auto mode_tag,
                    auto pc_tag) {
        constexpr int NK = decltype(nk_tag)::value;
        constexpr int MODE = decltype(mode_tag)::value;
        constexpr bool PC = decltype(pc_tag)::value;
        const bf16x8* ah = reinterpret_cast<const bf16x8*>(slot + lane * 16);
        const bf16x8* al = reinterpret_cast<const bf16x8*>(slot + LO + lane * 16);
        bf16x8 A0[2], A1[2];
        A0[0] = ah[0];
        A1[0] = al[0];
        if constexpr (NK > 1) {
            A0[1] = ah[64];
            A1[1] = al[64];
        }
        // sched_barrier pins the order: left alone the scheduler sinks each LDS read to right before
        // its MFMA (an lgkmcnt(0) wait per MFMA) to save the ring's registers
        __builtin_amdgcn_sched_barrier(0);
        s3_sfor<NK>([&](auto ksc) {
            constexpr int ks = decltype(ksc)::value;
            constexpr int u = ks & 1;
            const bool live = NK != NK0 || ks < nk;
            if (live) {
                if constexpr (MODE == 1) {
                    mf(acc, A0[u], Bh[ks].f);
                    mf(acc, A0[u], Bl[ks].f);
                    __builtin_amdgcn_sched_barrier(0);
                    if constexpr (ks + 2 < NK) A0[u] = ah[(ks + 2) * 64];
                    mf(acc, A1[u], Bh[ks].f);
                } else {
                    mf(acc, A0[u], Bh[ks].f);
                    __builtin_amdgcn_sched_barrier(0);
                    if constexpr (ks + 2 < NK) A0[u] = ah[(ks + 2) * 64];
                    mf(acc, A1[u], Bh[ks].f);
                }
            } else if constexpr (ks + 2 < NK) {
                A0[u] = ah[(ks + 2) * 64];
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ks + 2 < NK) A1[u] = al[(ks + 2) * 64];
            if constexpr (PC && NK == NKH && (ks & 1) == 0) dma_piece(std::integral_constant<int, ks / 2>());
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (PC && NK != NKH) dma_burst();
    };
    typedef std::integral_constant<bool, true> PcOn;
    typedef std::integral_constant<bool, false> PcOff;
    typedef std::integral_constant<int, 1> MFt;
    typedef std::integral_constant<int, 2> MBt;
    typedef std::integral_constant<int, NKH> NKHt;
    typedef std::integral_constant<int, NK0> NK0t;
    typedef std::integral_constant<int, 1> NK1t;

    auto bias_init = [&](int boff, int rt) -> f32x4 {
        const float4 v = *reinterpret_cast<const float4*>(bias_l + boff + rt * 16 + 4 * grp);
        return (f32x4){v.x, v.y, v.z, v.w};
    };
    // a packed k-step (x, y: features 32 s + 4 g + 0..3 of the lane's pixel; z, w: 32 s + 16 + 4 g + 0..3)
    // into a natural-order [S][ld] bf16 row: one v_permlane16_swap per dword pair puts features
    // 32 s + 16 (g & 1) + 8 (g >> 1) + 0..7 in every lane: one 16-B store
    //  (row = the lane's row base + 16 (g & 1) + 8 (g >> 1) elements; k-step S at instruction offset 64 S)
    auto store_ks = [&](u16* row, auto sc, const uint4& u) {
        constexpr int S = decltype(sc)::value;
        const auto xz = __builtin_amdgcn_permlane16_swap(u.x, u.z, false, false);
        const auto yw = __builtin_amdgcn_permlane16_swap(u.y, u.w, false, false);
        s3_st16o<64 * S>(row, make_uint4(xz[0], yw[0], xz[1], yw[1]));
        st_cur += 1;
    };
    const int colg = 16 * (grp & 1) + 8 * (grp >> 1);

    S3Frag Bh[NKH], Bl[NKH], Oh[NKH], Ol[NKH];
    const float pi_f = 3.14159265358979323846f;

    S3T_BEGIN(15);
    for (int ti = 0; ti < my_tiles; ++ti) {
        S3T_BEGIN(3);
        const int tile = tbase + ti * (int)gridDim.x;
        const int pb = ti & 1;
        const int b = tile / tpp;
        const int p0 = (tile - b * tpp) * TPX + PX * wave;
        const long long slot0 = (long long)b * a.geo.Np_pad + p0;
        const long long myslot = slot0 + pxl;
        const int p = p0 + pxl;
        const bool valid = p < Np;
        const float* pro = pro_buf(pb);

        // ---- prologue: pixel grid -> warp (warp.py:33-81) -> posenc + c2f (model/planar.py:451-471)
        float u, v, X[3];
        if (a.geo.mode == 1) {  // explicit coordinates (render only)
            const int pc = min(p, Np - 1);
            u = a.geo.coords[2 * (size_t)pc];
            v = a.geo.coords[2 * (size_t)pc + 1];
            X[0] = u;
            X[1] = v;
            X[2] = 1.0f;
        } else {
            const int r = p / a.geo.w, cc = p - r * a.geo.w;
            const float x = grid_coord(a.geo.x0 + cc, a.geo.W, a.geo.norm_w);
            const float y = grid_coord(a.geo.y0 + r, a.geo.H, a.geo.norm_h);
            warp_point(pro + 4 * TPX, x, y, u, v, X, a.geo.bmm_small);
        }
        {
            // layer-0 operand: band k-step ks, group g: bands 8 ks + 4 (g >> 1) + 0..3 of coordinate
            // g & 1, sin (j < 4) then cos; k-step nb: the raw coordinates (group 0: u, 1: v)
            const float cd = (grp & 1) ? v : u;
#pragma unroll
            for (int ks = 0; ks < NK0 - 1; ++ks) {
                if (ks < nb) {
                    float f[8];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int k = 8 * ks + 4 * (grp >> 1) + i;
                        float sn = 0.f, co = 0.f;
                        if (k < L) {
                            band_sincos<true>(cd, k, sn, co);
                            if (a.c2f_on) {
                                const float w = c2f_l[k];
                                sn = sn * w;
                                co = co * w;
                            }
                        }
                        f[i] = sn;
                        f[4 + i] = co;
                    }
                    s3_split8(f, Bh[ks], Bl[ks]);
                }
            }
            float f[8] = {grp == 0 ? u : (grp == 1 ? v : 0.f), 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            S3Frag rh, rl;
            s3_split8(f, rh, rl);
#pragma unroll
            for (int ks = 0; ks < NK0; ++ks)
                if (ks == nb) {
                    Bh[ks] = rh;
                    Bl[ks] = rl;
                }
            // feat_0 (bf16 hi) in k_step2's column order, which the layer-0 weight gradient and its
            // column map read: band group q (4 bands, sin then cos) of coordinate h at column
            // 16 q + 8 h, the raw coordinates in group ng, zero columns up to ldf0
            if (!a.fwd_only && !a.feat0_recompute) {
                u16* row = ly_ptr(0, 0) + myslot * ly_int(0, 3);
                const int ng = (L + 3) / 4, ldf0 = ly_int(0, 3);
#pragma unroll
                for (int ks = 0; ks < NK0 - 1; ++ks) {
                    if (ks < nb) {
                        const int q = 2 * ks + (grp >> 1);
                        s3_st16(q < ng ? (void*)(row + 16 * q + 8 * (grp & 1)) : (void*)dmy, Bh[ks].u);
                        st_cur += 1;
                    }
                }
                const bool raw = grp < 2, pad = grp >= 2 && 16 * (ng + 1) + 8 * (grp & 1) < ldf0;
                s3_st16(raw ? (void*)(row + 16 * ng + 8 * grp) : (pad ? (void*)(row + 16 * (ng + 1) + 8 * (grp & 1)) : (void*)dmy),
                        raw ? rh.u : make_uint4(0, 0, 0, 0));
                st_cur += 1;
            }
        }

        // ---- forward: layer 0, hidden layers.  Row tile rt of layer l: acc = bias + W . B, epilogue,
        //      the pair (2s, 2s + 1) -> operand k-step s of layer l + 1 (+ feat_{l+1} store, mask words)
        auto fwd_layer = [&](int l, const S3Frag* BH, const S3Frag* BL, int nk, auto nk_tag, int r0) {
            const int nrt = FULL ? (l == 0 ? NRT : NRT) : ly_int(l, 0);
            const bool save = l + 1 < nl - 1 && !a.fwd_only;
            u16* srow = save ? ly_ptr(l + 1, 0) + myslot * ly_int(l + 1, 3) + colg : nullptr;
            const int boff = ly_int(l, 2);
            uint32_t* mk = mkl + l * 2 * 64 + lane;
            const char* slot = nullptr;
            uint32_t mword = 0;
            S3Ep ev;
            s3_sfor<NRT>([&](auto rtc) {
                constexpr int rt = decltype(rtc)::value;
                if (rt < nrt) {
                    const int sub = rt % r0;
                    if (sub == 0) {
                        slot = stage_begin();
                        // the next tile's target / mask / H into the other input buffer
                        if (l == 0 && rt == 0 && ti + 1 < my_tiles) issue_pro(tile + (int)gridDim.x, pb ^ 1);
                    }
                    f32x4 acc = bias_init(boff, rt);
                    S3T_BEGIN(6);
                    if (sub == 0)
                        gemm(acc, slot + sub * nk * 1024, BH, BL, nk, nk_tag, MFt(), PcOn());
                    else
                        gemm(acc, slot + sub * nk * 1024, BH, BL, nk, nk_tag, MFt(), PcOff());
                    S3T_END(6);
                    S3T_BEGIN(7);
                    const S3Ep e = s3_fwd_ep(acc);
                    // the lo words computed here, not deferred to the layer's end, where the compiler
                    // would keep the 64 fp32 values alive (26 registers)
                    asm volatile("" ::"v"(e.l0), "v"(e.l1));
                    mword = (mword << 2) | e.nib;
                    if constexpr (rt & 1) {
                        Oh[rt >> 1].u = make_uint4(ev.h0, ev.h1, e.h0, e.h1);
                        Ol[rt >> 1].u = make_uint4(ev.l0, ev.l1, e.l0, e.l1);
                        if (save) store_ks(srow, std::integral_constant<int, (rt >> 1)>(), Oh[rt >> 1].u);
                    } else {
                        ev = e;
                    }
                    if (rt == nrt - 1 || (rt & 7) == 7) {  // a mask word: row tiles 8 (rt >> 3) .. rt
                        mk[(rt >> 3) * 64] = mword << (2 * (7 - (rt & 7)));
                        mword = 0;
                    }
                    S3T_END(7);
                } else if constexpr ((rt & 1) == 0) {
                    Oh[rt >> 1].u = Ol[rt >> 1].u = make_uint4(0, 0, 0, 0);
                }
            });
#pragma unroll
            for (int k = 0; k < NKH; ++k) {
                Bh[k] = Oh[k];
                Bl[k] = Ol[k];
            }
        };
        S3T_END(3);
        S3T_BEGIN(4);
        fwd_layer(0, Bh, Bl, nk0, NK0t(), FULL ? R0F : a.r0);
        S3T_END(4);
        S3T_BEGIN(5);
        for (int l = 1; l < nl - 1; ++l) fwd_layer(l, Bh, Bl, NKH, NKHt(), 2);
        S3T_END(5);
        S3T_BEGIN(8);

        // ---- last layer: 3 outputs (rows 0..2 of one tile, lanes 0..15), sigmoid, masked MSE, d rgb
        float g[3] = {0.f, 0.f, 0.f};
        {
            f32x4 acc = bias_init(ly_int(nl - 1, 2), 0);
            const char* slot = stage_begin();
            gemm(acc, slot, Bh, Bl, NKH, NKHt(), MFt(), PcOn());
            float* o = (a.rgb && valid && grp == 0) ? a.rgb + ((size_t)b * Np + p) * 3 : dmy;
            float yv[3] = {0.f, 0.f, 0.f};
            if (grp == 0) {
                const float m = valid ? (a.mask ? pro[3 * TPX + PX * wave + pxl] : 1.0f) : 0.f;
                float sqf = 0.f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float z = acc[c];
                    const float yy = 1.0f / (1.0f + expf(-z));
                    yv[c] = yy;
                    const float tg = valid ? pro[c * TPX + PX * wave + pxl] : 0.f;
                    // model/planar.py:388-390 and its autograd: x = (p - g) m, d = 2 x m
                    const float xx = (yy - tg) * m;
                    sqf += xx * xx;
                    const float d = (2.0f * xx) * m;
                    g[c] = (d * (1.0f - yy)) * yy;  // sigmoid backward
                }
                lsq += (double)sqf;
                lms += (double)m;
                bl0 += g[0];
                bl1 += g[1];
                bl2 += g[2];
            }
            s3_st12(o, yv[0], yv[1], yv[2]);
            st_cur += 1;
        }
        S3T_END(8);
        if (a.fwd_only) continue;

        S3T_BEGIN(9);
        // g as a split pair: hi = bf16(g), lo = bf16(g - hi)
        float ghi[3], glo[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            ghi[c] = s3_lo16(s3_pk(g[c], 0.f));
            glo[c] = g[c] - ghi[c];
        }
        // ---- last-layer weight gradient of the wave's 16 pixels: dW[c][k] += sum_px g[c] feat[k]
        //      (feat = the last layer's input, bf16 hi).  v_mfma_f32_16x16x32_bf16 with A = g^T (rows
        //      c, k = pixels 0..15; 16..31 zero) hi and lo, B = feat^T per 16 features through a
        //      transposing LDS round trip (ds_read_b64_tr_b16)
        {
            if (grp == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    gimg[c * 16 + pxl] = (u16)(s3_pk(ghi[c], 0.f) & 0xffff);
                    gimg[(3 + c) * 16 + pxl] = (u16)(s3_pk(glo[c], 0.f) & 0xffff);
                }
            }
            asm volatile("" ::: "memory");
            const int rc = lane & 15, kg = lane >> 4;
            S3Frag gah, gal;
            gah.u = gal.u = make_uint4(0, 0, 0, 0);
            {
                const uint4 th = *reinterpret_cast<const uint4*>(gimg + min(rc, 2) * 16 + 8 * (kg & 1));
                const uint4 tl = *reinterpret_cast<const uint4*>(gimg + (3 + min(rc, 2)) * 16 + 8 * (kg & 1));
                if (rc < 3 && kg < 2) {
                    gah.u = th;
                    gal.u = tl;
                }
            }
            const int q = (lane & 15) >> 2, pq = lane & 3;
            const int nkl = a.Kl / 32;
#pragma unroll
            for (int s = 0; s < NKH; ++s) {
                if (s < nkl) {
                    asm volatile("" ::: "memory");
                    uint2* w2 = reinterpret_cast<uint2*>(scr + pxl * 32);
                    w2[grp] = make_uint2(Bh[s].u.x, Bh[s].u.y);      // features 4 g + 0..3
                    w2[4 + grp] = make_uint2(Bh[s].u.z, Bh[s].u.w);  // features 16 + 4 g + 0..3
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int fb = 0; fb < 2; ++fb) {
                        const u16* b0 = scr + (8 * (kg & 1) + q) * 32 + 16 * fb + 4 * pq;
                        i16x4 vv[2] = {s3_tr16(b0), s3_tr16(b0 + 4 * 32)};
                        const bf16x8 bt = *reinterpret_cast<bf16x8*>(vv);
                        f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gah.f, bt, (f32x4){}, 0, 0, 0);
                        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gal.f, bt, d, 0, 0, 0);
                        if (lane < 16) {
#pragma unroll
                            for (int c = 0; c < 3; ++c) wla[c * a.Kl + 32 * s + 16 * fb + lane] += d[c];
                        }
                    }
                }
            }
        }

        S3T_END(9);
        S3T_BEGIN(10);
        // ---- last-layer dgrad: dfeat = W_{n-1}^T g (one k-step per row tile: lanes 0..15 carry
        //      k = [g hi (3), 0, g lo (3), 0]), mask -> dz_{n-1}; one stage holds every row tile
        S3Frag gB;
        {
            float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (grp == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    f[c] = ghi[c];
                    f[4 + c] = glo[c];
                }
            }
            gB.u = make_uint4(s3_pk(f[0], f[1]), s3_pk(f[2], f[3]), s3_pk(f[4], f[5]), s3_pk(f[6], f[7]));
        }
        auto bwd_pass = [&](int l, int lmask, int nrt, const char* slot_first, bool last) {
            // row tiles of dz: last: every tile from one stage (tile rt at rt KB); else two per stage
            u16* brow = ly_ptr(l, 1) + myslot * ly_int(l, 4) + colg;
            const uint32_t* mk = mkl + lmask * 2 * 64 + lane;
            const char* slot = slot_first;
            uint32_t mw = 0, hv0 = 0, hv1 = 0;
            s3_sfor<NRT>([&](auto rtc) {
                constexpr int rt = decltype(rtc)::value;
                if (rt < nrt) {
                    if constexpr ((rt & 7) == 0) mw = mk[(rt >> 3) * 64];
                    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
                    if (last) {
                        S3T_BEGIN(11);
                        if constexpr (rt == 0)
                            gemm(acc, slot + rt * 1024, &gB, &gB, 1, NK1t(), MBt(), PcOn());
                        else
                            gemm(acc, slot + rt * 1024, &gB, &gB, 1, NK1t(), MBt(), PcOff());
                        S3T_END(11);
                    } else {
                        if constexpr ((rt & 1) == 0) slot = stage_begin();
                        S3T_BEGIN(11);
                        gemm(acc, slot + (rt & 1) * NKH * 1024, Bh, Bh, NKH, NKHt(), MBt(),
                             std::integral_constant<bool, (rt & 1) == 0>());
                        S3T_END(11);
                    }
                    S3T_BEGIN(12);
                    const uint2 hw = s3_bwd_ep<2 * (7 - (rt & 7))>(acc, mw);
                    if constexpr (rt & 1) {
                        Oh[rt >> 1].u = make_uint4(hv0, hv1, hw.x, hw.y);
                        store_ks(brow, std::integral_constant<int, (rt >> 1)>(), Oh[rt >> 1].u);
                    } else {
                        hv0 = hw.x;
                        hv1 = hw.y;
                    }
                    S3T_END(12);
                } else if constexpr ((rt & 1) == 0) {
                    Oh[rt >> 1].u = make_uint4(0, 0, 0, 0);
                }
            });
#pragma unroll
            for (int k = 0; k < NKH; ++k) Bh[k] = Oh[k];
        };
        {
            const char* slot = stage_begin();
            bwd_pass(nl - 1, nl - 2, FULL ? NRT : ly_int(nl - 1, 1), slot, true);
        }
        for (int l = nl - 2; l >= 1; --l) bwd_pass(l, l - 1, FULL ? NRT : ly_int(l, 1), nullptr, false);
        S3T_END(10);
        S3T_BEGIN(13);

        // ---- layer-0 dgrad + posenc adjoint: row tile t, register r of lane group G holds band
        //      4 t + r of coordinate G >> 1, the sin slot for even G, the cos slot for odd G (the raw
        //      coordinates: tile 2 nb, register 0 of groups 0 (u) and 2 (v)).  One v_permlane16_swap
        //      gives each lane its partner group's slot of the same band, so every lane forms the
        //      band's term as k_step2 and torch's autograd of sin / cos do, (g_sin cos - g_cos sin)
        //      2^k pi, accumulated over the bands in increasing k, then the raw coordinate
        float dc = 0.f;
        {
            const int nta = FULL ? NTA : a.nta;
            const float cd = (grp >> 1) ? v : u;
            const bool sinl = (grp & 1) == 0;
            const char* slot = nullptr;
            s3_sfor<NTA>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                if (t < nta) {
                    if constexpr ((t & 1) == 0) slot = stage_begin();
                    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
                    gemm(acc, slot + (t & 1) * NKH * 1024, Bh, Bh, NKH, NKHt(), MBt(), std::integral_constant<bool, (t & 1) == 0>());
                    if (t < 2 * nb) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int k = 4 * t + r;
                            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[r]), __float_as_uint(acc[r]),
                                                                            false, false);
                            const float other = __uint_as_float(sinl ? sw[1] : sw[0]);
                            if (k < L) {
                                float sn, co;
                                band_sincos<true>(cd, k, sn, co);
                                float gs = sinl ? acc[r] : other, gc = sinl ? other : acc[r];
                                if (a.c2f_on) {
                                    const float w = c2f_l[k];
                                    gs = gs * w;
                                    gc = gc * w;
                                }
                                dc += (gs * co - gc * sn) * ldexpf(pi_f, k);
                            }
                        }
                    } else if (t == 2 * nb) {
                        dc += acc[0];  // (read from groups 0 and 2 only)
                    }
                }
            });
        }
        S3T_END(13);
        S3T_BEGIN(14);
        // ---- (u, v) = X[:2] / (X[2] + 1e-8) backward, the bmm backward -> dH partial of the wave
        {
            const float du = dc, dv = __shfl(dc, (lane & 15) + 32, 64);  // groups 0: du, 2: dv
            float h9[9];
#pragma unroll
            for (int e = 0; e < 9; ++e) h9[e] = 0.f;
            if (grp == 0 && valid) {
                const int r = p / a.geo.w, cc = p - r * a.geo.w;
                const float x = grid_coord(a.geo.x0 + cc, a.geo.W, a.geo.norm_w);
                const float y = grid_coord(a.geo.y0 + r, a.geo.H, a.geo.norm_h);
                const float dd = X[2] + 1e-8f;
                const float dX0 = du / dd, dX1 = dv / dd;
                const float dd2 = dd * dd;
                const float dX2 = (-du * X[0]) / dd2 + (-dv * X[1]) / dd2;
                const float hom[3] = {x, y, 1.f};
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    h9[0 + c] = dX0 * hom[c];
                    h9[3 + c] = dX1 * hom[c];
                    h9[6 + c] = dX2 * hom[c];
                }
            }
            float mine = 0.f;
#pragma unroll
            for (int e = 0; e < 9; ++e) {
                const float sm = wave_total63(h9[e]);
                const float sb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm), 63));
                if (lane == e) mine = sb;
            }
            s3_st4(lane < 9 ? (void*)(a.dH_partial + (size_t)(slot0 / PX) * 9 + lane) : (void*)dmy, mine);
            st_cur += 1;
        }
        S3T_END(14);
    }
    S3T_END(15);
#ifdef MARF_STAMPS
    if (a.stamps && threadIdx.x == 0)
        for (int k = 0; k < 16; ++k) a.stamps[(size_t)blockIdx.x * 16 + k] = tacc[k];
#endif

    // ---- per-block partials (fixed order over waves)
    s3_wait_vm<0>();
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);  // the ring is idle now
    {
        const double s0 = wave_total63(lsq), s1 = wave_total63(lms);
        const float t0 = wave_total63(bl0), t1 = wave_total63(bl1), t2 = wave_total63(bl2);
        if (lane == 63) {
            red[wave * 5 + 0] = s0;
            red[wave * 5 + 1] = s1;
            red[wave * 5 + 2] = (double)t0;
            red[wave * 5 + 3] = (double)t1;
            red[wave * 5 + 4] = (double)t2;
        }
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        double s = 0.0;
        float sf = 0.f;
        for (int w = 0; w < NW; ++w) {
            s += red[w * 5 + threadIdx.x];
            sf += (float)red[w * 5 + threadIdx.x];
        }
        if (threadIdx.x < 2) a.loss_partial[2 * (size_t)blockIdx.x + threadIdx.x] = s;
        else a.blast_partial[3 * (size_t)blockIdx.x + threadIdx.x - 2] = sf;
    }
    for (int e = threadIdx.x; e < 3 * a.Kl; e += NW * 64) {
        float s = 0.f;
        for (int w = 0; w < NW; ++w) s += reinterpret_cast<const float*>(smem + a.lds_wave + w * a.lds_wave_bytes + W_WLA)[e];
        a.wlast_partial[(size_t)blockIdx.x * 3 * a.Kl + e] = s;
    }
}

// ------------------------------------------------------------------ weight program packing

// layer-0 operand k index (k-step ks, group g, element j) -> input feature of the reference's
// [x, y, posenc] vector (model/planar.py:451-471: posenc = [sin bands of x, of y, cos ...] as
// 2 + 2 h L + (cos ? L : 0) + band); -1: a zero slot
MARF_DEV int s3_l0_feature(int ks, int g, int j, int L, int nb) {
    if (ks == nb) return (j == 0 && g < 2) ? g : -1;
    const int band = 8 * ks + 4 * (g >> 1) + (j & 3);
    if (band >= L) return -1;
    return 2 + 2 * (g & 1) * L + (j >= 4 ? L : 0) + band;
}
// hidden operand k index (k-step s, group g, element j) -> feature (the accumulator-pair order)
MARF_DEV int s3_kperm(int s, int g, int j) { return 32 * s + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4); }

// One thread per (stage, part, fragment, lane, element).  Stage sequence per tile: layer-0 forward
// (r0 row tiles of nk0 k-steps each), hidden forward (pairs of row tiles), last layer, last-layer
// dgrad (every row tile's single k-step), hidden dgrad l = nl-2 .. 1 (pairs), adjoint (pairs).
// A fragment of row tile rt, k-step ks: lane l holds row 16 rt + (l & 15), k index (ks, l >> 4, j).
__global__ void k_pack3(const float* __restrict__ params, u16* __restrict__ prog, float* __restrict__ bias_out,
                        int* __restrict__ kmap, Pack2Args a) {
    const int per_slot = s3::SLOT / 2;
    const long long total = (long long)a.n_stages * per_slot;
    const int D = a.dims[0];
    const int nb = a.nk0 - 1;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total + a.nbias + D; e += (long long)gridDim.x * 256) {
        if (e >= total + a.nbias) {
            // layer-0 column map of feat_0 (k_step2's column order): true input feature f -> column
            const int f = (int)(e - total - a.nbias), L = a.L, ng = (L + 3) / 4;
            int col;
            if (f < 2) col = 16 * ng + 8 * f;
            else {
                const int q = f - 2, hh = q / (2 * L), rr = q - hh * 2 * L, cosp = rr >= L, k = rr - cosp * L;
                col = 16 * (k / 4) + 8 * hh + 4 * cosp + (k % 4);
            }
            kmap[f] = col;
            continue;
        }
        if (e >= total) {  // padded bias table
            const int be = (int)(e - total);
            float v = 0.f;
            for (int l = 0; l < a.nl; ++l) {
                const int nbias = (l == a.nl - 1) ? 32 : a.Mp[l];
                if (be >= a.boff[l] && be < a.boff[l] + nbias) {
                    const int m = be - a.boff[l];
                    if (m < a.dims[l + 1]) v = params[a.b_off[l] + m];
                }
            }
            bias_out[be] = v;
            continue;
        }
        const int st = (int)(e / per_slot);
        const int w = (int)(e - (long long)st * per_slot);
        const int part = w / 8192;  // 0 hi, 1 lo
        const int idx = (w % 8192) / 512, lane = (w >> 3) & 63, j = w & 7;
        const int r16 = lane & 15, g = lane >> 4;
        int layer = -1, kind = -1, rt = 0, ks = 0;  // kind 0 fwd, 1 last fwd, 2 last dgrad, 3 hidden dgrad, 4 adjoint
        {
            int s = st;
            if (s < a.ns0) {
                layer = 0;
                kind = 0;
                rt = s * a.r0 + idx / a.nk0;
                ks = idx % a.nk0;
                if (idx >= a.r0 * a.nk0 || rt >= a.nrt[0]) kind = -1;
            } else {
                s -= a.ns0;
                for (int l = 1; l < a.nl - 1 && layer < 0; ++l) {
                    if (s < a.nrt[l] / 2) {
                        layer = l;
                        kind = 0;
                        rt = 2 * s + idx / 8;
                        ks = idx % 8;
                    } else {
                        s -= a.nrt[l] / 2;
                    }
                }
                if (layer < 0) {
                    if (s == 0) {
                        layer = a.nl - 1;
                        kind = 1;
                        rt = idx / 8;
                        ks = idx % 8;
                        if (rt > 0) kind = -1;
                    } else if (s == 1) {
                        layer = a.nl - 1;
                        kind = 2;
                        rt = idx;
                        ks = 0;
                        if (rt >= a.nrtb[layer]) kind = -1;
                    } else {
                        s -= 2;
                        for (int l = a.nl - 2; l >= 1 && layer < 0; --l) {
                            if (s < a.nrtb[l] / 2) {
                                layer = l;
                                kind = 3;
                                rt = 2 * s + idx / 8;
                                ks = idx % 8;
                            } else {
                                s -= a.nrtb[l] / 2;
                            }
                        }
                        if (layer < 0 && s < (a.nta + 1) / 2) {
                            layer = 0;
                            kind = 4;
                            rt = 2 * s + idx / 8;
                            ks = idx % 8;
                            if (rt >= a.nta) kind = -1;
                        }
                    }
                }
            }
        }
        float val = 0.f;
        bool have = false;
        if (kind >= 0) {
            const int Mt = a.dims[layer + 1], Kt = a.dims[layer];
            const float* W = params + a.w_off[layer];
            int m = -1, k = -1;  // W[m][k]
            const int row = 16 * rt + r16;
            if (kind == 0 && layer == 0) {
                m = row;
                k = s3_l0_feature(ks, g, j, a.L, nb);
            } else if (kind == 0 || kind == 1) {
                m = row;
                k = s3_kperm(ks, g, j);
            } else if (kind == 2) {  // rows = input features of the last layer, k = [g hi (3), 0, g lo (3), 0]
                if (g == 0 && (j & 3) < 3) {
                    m = j & 3;
                    k = row;
                }
            } else if (kind == 3) {  // W_l^T: row = input feature of layer l, k = its output (permuted)
                m = s3_kperm(ks, g, j);
                k = row;
            } else {  // adjoint: row = layer-0 operand k index 32 ks' + 8 g' + j'
                m = s3_kperm(ks, g, j);
                k = s3_l0_feature(row >> 5, (row >> 3) & 3, row & 7, a.L, nb);
            }
            if (m >= 0 && k >= 0 && m < Mt && k < Kt) {
                val = W[(size_t)m * Kt + k];
                have = true;
            }
        }
        u16 out = 0;
        if (have) {
            const u16 hi = f2bf(val);
            out = part == 0 ? hi : f2bf(val - bf2f(hi));
        }
        prog[e] = out;
    }
}

}  // namespace marf

using namespace marf;

template <int NK0T, bool FULL, int NWT>
static hipError_t launch_step3_t(const Step2Args& a, int grid, hipStream_t s) {
    hipError_t e = ensure_dynamic_lds((const void*)k_step3<NK0T, FULL, NWT>, (size_t)a.lds_total);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_step3<NK0T, FULL, NWT>), dim3(grid), dim3(NWT * 64), (size_t)a.lds_total, s, a);
    return hipGetLastError();
}

// full = every hidden layer 256 wide (the host checks): L <= 8 and L <= 16 get their own code; the
// generic instantiation covers the rest.  8 waves per block (two per SIMD).
bool marf_step3_nw_ok(bool, int, int nw) { return nw == 8; }
hipError_t marf_launch_step3(const Step2Args& a, bool full, int nw, int grid, hipStream_t s) {
    if (nw != 8) return hipErrorInvalidValue;
    if (full && a.nk0 == 2) return launch_step3_t<2, true, 8>(a, grid, s);
    if (full && a.nk0 == 3) return launch_step3_t<3, true, 8>(a, grid, s);
    return launch_step3_t<s3::NK0MAX, false, 8>(a, grid, s);
}

hipError_t marf_launch_pack3(const float* params, void* prog, float* bias_out, int* kmap, const Pack2Args& a,
                             hipStream_t s) {
    const long long total = (long long)a.n_stages * (s3::SLOT / 2) + a.nbias + a.dims[0];
    long long blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_pack3, dim3((unsigned)blocks), dim3(256), 0, s, params, (u16*)prog, bias_out, kmap, a);
    return hipGetLastError();
}

int marf_step3_wave_lds_bytes() { return s3::WAVE_LDS; }
