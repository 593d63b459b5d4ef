// marf_step3.hip -- the fused training step of the split-bf16 recipe at TWO waves per SIMD (gfx950),
// bit-identical to k_step2 (marf_step2.hip, variant 1).
//
// Same contract and saved tensors as k_step2: per pixel grid -> sl(3) warp -> posenc + c2f -> MLP
// forward (hi*hi + hi*lo + lo*hi, fp32 accumulation) -> sigmoid -> masked-MSE partial -> d rgb ->
// dgrad chain (W_hi^T dz + W_lo^T dz) -> posenc / warp adjoint (model/planar.py:329-391,
// warp.py:33-81), writing feat_l / dz_l for the weight-gradient kernels.  Every fp32 operation on
// the way happens in k_step2's order, so rgb, loss and every gradient carry k_step2's bits (and
// with them its seed-3 run).  What changes is the shape on the CU:
//
//   * one wave owns 16 pixels (not 32) on v_mfma_f32_16x16x32_bf16, so a wave's operands fit in
//     256 registers and the 512-thread block (8 waves, one per CU) runs TWO waves per SIMD.
//   * k_step2 accumulates each output over 16-k chunks c with one 32x32x16 MFMA per term: forward
//     hh(c), hl(c), lh(c) (hi.hi, hi.lo, lo.hi), dgrad hd(c), ld(c) (W_hi^T dz, W_lo^T dz).  A
//     16x16x32 MFMA adds its two 16-k halves (lane groups 0-1, then 2-3) in order, each exactly as
//     a 32x32x16 MFMA would (tools/mfma_compose_probe.hip: 0 of 12,288 outputs differ), so two
//     consecutive terms make one MFMA: per pair of chunks (2s, 2s+1)
//       forward  [hh(2s) | hl(2s)], [lh(2s) | hh(2s+1)], [hl(2s+1) | lh(2s+1)]   (3 MFMAs, as k_step2)
//       dgrad    [hd(2s) | ld(2s)], [hd(2s+1) | ld(2s+1)]                          (2 MFMAs, as k_step2)
//     The lane group g of an operand pair holds chunk 2s + (g >> 1) at k_step2's position
//     8 (g & 1) + j, i.e. feature F(s, g, j) = 32 s + 16 (g >> 1) + 8 (j >> 2) + 4 (g & 1) + (j & 3)
//     (k_step2's s2_kperm).  The output row tiles are permuted to match (s3_mrow), so a pair of
//     16-row accumulator tiles packed to bf16 is operand pair s as it stands (H: hi words, L: lo).
//     The B operands of the composite MFMAs are H / L with halves exchanged: one v_permlane32_swap
//     per dword builds B1 = [H.h0 | L.h0] and B3 = [L.h1 | H.h1] (forward; the middle MFMA takes
//     H = [B1.h0 | B3.h1], a select), or D1 = [D.h0 | D.h0] and D2 = [D.h1 | D.h1] (dgrad).  The A
//     operands are the packed hi / lo fragments read with per-lane addresses (3 reads per forward
//     pair, 2 per dgrad pair).
//   * reductions over pixels are k_step2's 32-pixel ones: the waves w and w + 4 (one SIMD) own the
//     two halves of k_step2's wave W = w: the last-layer weight gradient runs as one K = 32-pixel
//     chain, the first half from 0 (stage L), the second half from that partial (stage L + 1,
//     handed over through a per-block global buffer, xbuf); the dH partial and the loss / bias
//     sums gather the pair's 32 pixels in LDS and reduce them with k_step2's DPP tree.
//   * the weights stream through a 3-slot LDS ring (one 32 KB slot = 32 rows of one layer, hi then
//     lo, filled by global_load_lds_dwordx4 two stages ahead, 4 pieces per wave).
//
// Memory ordering as in k_step2: all global traffic inside the tile loop is inline asm (LDS-DMA,
// stores) except the xbuf loads; each wave counts the store instructions it issues per stage and
// waits for a ring slot with the vmcnt that leaves exactly the younger operations in flight.
// Every counted store is issued by every wave (lanes with nothing to store write a private sink).
#include <type_traits>

#include "marf_args.h"

namespace marf {
namespace s3 {

constexpr int PX = 16;                        // pixels per wave
constexpr int NW = 8;                         // waves per block (two per SIMD)
constexpr int TPX = NW * PX;                  // pixel slots per block tile (k_step2's)
constexpr int HM = 256;                       // widest hidden layer
constexpr int NPH = HM / 32;                  // operand pairs (two 16-k chunks) of a hidden-width input
constexpr int NRT = HM / 16;                  // 16-row tiles of a hidden-width output
constexpr int SLOT = 32768;                   // one ring slot = one program stage
constexpr int LO = 16384;                     // byte offset of the lo fragments in a slot
constexpr int PER_DMA = 4;                    // 1 KB DMA pieces per wave and stage
constexpr int NSLOT = 3;
constexpr int NP0MAX = 5;                     // max layer-0 pairs (L <= 32: 8 band chunks + raw)
constexpr int NML = 4;                        // max ReLU layers (nl <= 5)
constexpr int XQ = 12;                        // 16-B pieces of a lane's dW_last partial (16 MFMAs x 3 rows)
// wave-private LDS: g^T image [8][16] (256 B), transpose scratch (1 KB), mask words [NML][2][64],
// dW_last [3][256] (second-half waves; a first-half wave's copy is its pair's exchange buffer)
constexpr int W_GIMG = 0, W_SCR = 256, W_MASK = 1280, W_WLA = W_MASK + NML * 2 * 64 * 4;
constexpr int WAVE_LDS = W_WLA + 3 * HM * 4;
// the pair exchange buffer (bytes): dH terms [9][32] fp32, loss sums [32] fp64 x 2, bias grads [3][32]
constexpr int PB_DH = 0, PB_LSQ = 9 * 32 * 4, PB_LMS = PB_LSQ + 32 * 8, PB_BL = PB_LMS + 32 * 8;
static_assert(PB_BL + 3 * 32 * 4 <= 3 * HM * 4, "pair buffer");
static_assert(SLOT % (PER_DMA * 1024 * NW) == 0, "ring geometry");

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
    const s3_u32x4 v = {u.x, u.y, u.z, u.w};
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
template <int OFF>
MARF_DEV void s3_st16o(void* base, uint4 u) {  // 16 B at base + OFF bytes (instruction offset)
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
// 8 floats -> bf16 hi words + lo remainder words (k_step2's s2_split8)
MARF_DEV void s3_split8(const float* x, uint4& hi, uint4& lo) {
    hi = make_uint4(s3_pk(x[0], x[1]), s3_pk(x[2], x[3]), s3_pk(x[4], x[5]), s3_pk(x[6], x[7]));
    const uint32_t w[4] = {hi.x, hi.y, hi.z, hi.w};
    float r[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r[2 * q] = x[2 * q] - s3_lo16(w[q]);
        r[2 * q + 1] = x[2 * q + 1] - s3_hi16(w[q]);
    }
    lo = make_uint4(s3_pk(r[0], r[1]), s3_pk(r[2], r[3]), s3_pk(r[4], r[5]), s3_pk(r[6], r[7]));
}
// per 16-bit half of a packed bf16 pair: (half != 0) at bits 0 and 16
MARF_DEV uint32_t s3_nz_pair(uint32_t w) {
    uint32_t t;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(t) : "v"(w), "s"(0x00010001u));
    return t;
}

// forward operand pair from its hi / lo words: B1 = [H.h0 | L.h0], B3 = [L.h1 | H.h1] (lo32: lane < 32)
MARF_DEV void s3_fwd_pair(const uint4& H, const uint4& L, bool lo32, S3Frag& B1, S3Frag& B3) {
    const uint32_t h[4] = {H.x, H.y, H.z, H.w}, l[4] = {L.x, L.y, L.z, L.w};
    uint32_t b1[4], b3[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const auto p = __builtin_amdgcn_permlane32_swap(lo32 ? h[q] : l[q], lo32 ? l[q] : h[q], false, false);
        b1[q] = p[0];
        b3[q] = p[1];
    }
    B1.u = make_uint4(b1[0], b1[1], b1[2], b1[3]);
    B3.u = make_uint4(b3[0], b3[1], b3[2], b3[3]);
}
// the hi words H = [B1.h0 | B3.h1] of a forward operand pair (volatile asm: rebuilt at each use, in
// the MFMA gap -- a select the compiler may hoist would keep all of a layer's H words live, 32 VGPRs)
MARF_DEV uint32_t s3_sel32(uint32_t lo_lanes, uint32_t hi_lanes) {
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(hi_lanes), "v"(lo_lanes), "s"(0xffffffffull));
    return r;
}
MARF_DEV uint4 s3_mid(const S3Frag& B1, const S3Frag& B3) {
    return make_uint4(s3_sel32(B1.u.x, B3.u.x), s3_sel32(B1.u.y, B3.u.y), s3_sel32(B1.u.z, B3.u.z),
                      s3_sel32(B1.u.w, B3.u.w));
}
// dgrad operand pair: D1 = [D.h0 | D.h0], D2 = [D.h1 | D.h1]
MARF_DEV void s3_bwd_pair(const uint4& D, S3Frag& D1, S3Frag& D2) {
    const uint32_t d[4] = {D.x, D.y, D.z, D.w};
    uint32_t a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const auto p = __builtin_amdgcn_permlane32_swap(d[q], d[q], false, false);
        a[q] = p[0];
        b[q] = p[1];
    }
    D1.u = make_uint4(a[0], a[1], a[2], a[3]);
    D2.u = make_uint4(b[0], b[1], b[2], b[3]);
}

// forward epilogue of one 16-row accumulator tile: ReLU, bf16 hi + lo of the 4 values (x0 x1 | x2 x3),
// and the mask nibble (bits 0: x0, 1: x2, 16: x1, 17: x3) from the packed hi words (k_step2's mask_pair:
// a value passes the ReLU exactly when its bf16 hi is non-zero, except for 0 < z < 2^-133)
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

// NP0T: layer-0 operand pairs (ceil((ceil(L / 4) + 1) / 2)); FULL: every hidden layer 256 wide.
// Both make the row-tile and pair counts compile-time; <NP0MAX, false> is the generic instantiation.
template <int NP0T, bool FULL>
__global__ __launch_bounds__(512, 2) void k_step3(Step2Args a) {
    using namespace s3;
    constexpr int NP0 = NP0T;
    constexpr int NTA = 2 * NP0;                   // adjoint row tiles (max: ng band tiles + raw)
    constexpr int R0F = (16 / NP0) & ~1;           // layer-0 row tiles per stage (FULL)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pxl = lane & 15, grp = lane >> 4;
    const bool lo32 = lane < 32;
    // k_step2's wave W = wave & 3 (its 32 pixels); this wave holds half (wave >> 2) of them, and its
    // SIMD partner (wave ^ 4) the other half
    const int W = wave & 3, half = wave >> 2, pblk = 2 * W + half;
    const int nl = a.nl, L = a.L;
    const int np0 = FULL ? NP0 : a.nk0;
    const int ng = (L + 3) / 4;                    // k_step2's band chunks (then the raw chunk)
    const bool odd_tail = ((ng + 1) & 1) != 0;     // the last layer-0 pair has no second chunk

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
    u16* gimg = reinterpret_cast<u16*>(wpriv + W_GIMG);        // [8][16]: rows 0-2 g hi, 4-6 g lo
    u16* scr = reinterpret_cast<u16*>(wpriv + W_SCR);          // [16 px][32 features] transpose image
    uint32_t* mkl = reinterpret_cast<uint32_t*>(wpriv + W_MASK);  // [layer][word][lane]
    float* wla = reinterpret_cast<float*>(wpriv + W_WLA);      // [3][Kl] dW_last (second-half waves)
    char* pbuf = smem + a.lds_wave + W * a.lds_wave_bytes + W_WLA;  // the pair's exchange buffer
    float* dmy = a.dummy + (((size_t)blockIdx.x * NW + wave) * 64 + lane) * 16;  // 64-B store sink per lane
#ifdef MARF_STAMPS
    unsigned long long tacc[16] = {};
#endif

    // ---- constants into LDS (plain loads before the ring starts)
    for (int e = threadIdx.x; e < a.nbias; e += NW * 64) bias_l[e] = a.bias[e];
    if ((int)threadIdx.x < 32) c2f_l[threadIdx.x] = (int)threadIdx.x < L ? a.c2f_w[threadIdx.x] : 0.f;
    for (int e = threadIdx.x; e < nl * (int)(sizeof(S2Layer) / 4); e += NW * 64)
        reinterpret_cast<uint32_t*>(lyr)[e] = reinterpret_cast<const uint32_t*>(a.layers)[e];
    if (half == 1)
        for (int e = lane; e < 3 * a.Kl; e += 64) wla[e] = 0.f;
    reinterpret_cast<uint32_t*>(gimg)[lane] = 0u;

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
    const char* const prog_w = a.prog + wave * PER_DMA * 1024 + lane * 16;
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
    // xflush: this wave stored a dW_last partial its partner loads after the next barrier -- wait for
    // every store before it.
    int st_cur = 0, st_prev = 0;
    bool xflush = false;
    auto wait_ring = [&]() {
        if (xflush) {
            s3_wait_vm<0>();
            xflush = false;
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
        __builtin_amdgcn_s_barrier();
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
    // per-lane byte offsets of the composite A operands in a pair's fragments (hi at +0, lo at +LO;
    // fragment lane (row r, group g) holds k positions 8 g .. 8 g + 7 of the pair)
    // (recomputed from the lane id at each GEMM: four live offsets cost more registers than the VALU)
    auto oF1 = [&]() -> unsigned { return (threadIdx.x & 31) * 16; };                                 // [hi(2s) | hi(2s)]
    auto oF2 = [&]() -> unsigned { return (threadIdx.x & 63) * 16 + ((threadIdx.x & 32) ? 0 : LO); };     // [lo(2s) | hi(2s+1)]
    auto oF3 = [&]() -> unsigned {  // [hi(2s+1) | lo(2s+1)] (dgrad: the second MFMA)
        return (threadIdx.x & 32) ? LO + (threadIdx.x & 63) * 16 : ((threadIdx.x & 31) + 32) * 16;
    };
    auto oD1 = [&]() -> unsigned { return (threadIdx.x & 31) * 16 + ((threadIdx.x & 32) ? LO : 0); };  // [hi(2s) | lo(2s)]

    // forward: one 16-row output tile over NP operand pairs (np live; the last layer-0 pair of an odd
    // chunk count has no second chunk: its third MFMA is skipped).  The A fragments of pair s + 1 are
    // read as pair s's MFMAs go out.  PC: this GEMM is its stage's first -- the stage's DMA pieces go
    // out beside its MFMAs (piece j after pair 2 j of an 8-pair GEMM; after a shorter one's last pair)
    auto gemm_f = [&](f32x4& acc, const char* slot, const S3Frag* B1, const S3Frag* B3, int np, auto np_tag,
                      auto pc_tag) {
        constexpr int NP = decltype(np_tag)::value;
        constexpr bool PC = decltype(pc_tag)::value;
        const char* p1 = slot + oF1();
        const char* p2 = slot + oF2();
        const char* p3 = slot + oF3();
        bf16x8 F0 = *reinterpret_cast<const bf16x8*>(p1);
        bf16x8 F1 = *reinterpret_cast<const bf16x8*>(p2);
        bf16x8 F2 = *reinterpret_cast<const bf16x8*>(p3);
        __builtin_amdgcn_sched_barrier(0);
        s3_sfor<NP>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const bool live = NP != NP0 || s < np;
            if (live) {
                S3Frag mid;
                mid.u = s3_mid(B1[s], B3[s]);
                mf(acc, F0, B1[s].f);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (s + 1 < NP) if (NP != NP0 || s + 1 < np) F0 = *reinterpret_cast<const bf16x8*>(p1 + (s + 1) * 1024);
                mf(acc, F1, mid.f);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (s + 1 < NP) if (NP != NP0 || s + 1 < np) F1 = *reinterpret_cast<const bf16x8*>(p2 + (s + 1) * 1024);
                if (!(NP == NP0 && odd_tail && s == np - 1)) mf(acc, F2, B3[s].f);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (s + 1 < NP) if (NP != NP0 || s + 1 < np) F2 = *reinterpret_cast<const bf16x8*>(p3 + (s + 1) * 1024);
            }
            if constexpr (PC && NP == NPH && (s & 1) == 0) dma_piece(std::integral_constant<int, s / 2>());
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (PC && NP != NPH) dma_burst();
    };
    // dgrad: one 16-row output tile over NP operand pairs: [hd(2s) | ld(2s)], [hd(2s+1) | ld(2s+1)]
    auto gemm_b = [&](f32x4& acc, const char* slot, const S3Frag* D1, const S3Frag* D2, auto np_tag, auto pc_tag) {
        constexpr int NP = decltype(np_tag)::value;
        constexpr bool PC = decltype(pc_tag)::value;
        const char* q1 = slot + oD1();
        const char* q2 = slot + oF3();
        bf16x8 G0 = *reinterpret_cast<const bf16x8*>(q1);
        bf16x8 G1 = *reinterpret_cast<const bf16x8*>(q2);
        __builtin_amdgcn_sched_barrier(0);
        s3_sfor<NP>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            mf(acc, G0, D1[s].f);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (s + 1 < NP) G0 = *reinterpret_cast<const bf16x8*>(q1 + (s + 1) * 1024);
            mf(acc, G1, D2[s].f);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (s + 1 < NP) G1 = *reinterpret_cast<const bf16x8*>(q2 + (s + 1) * 1024);
            if constexpr (PC && NP == NPH && (s & 1) == 0) dma_piece(std::integral_constant<int, s / 2>());
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (PC && NP != NPH) dma_burst();
    };
    typedef std::integral_constant<bool, true> PcOn;
    typedef std::integral_constant<bool, false> PcOff;
    typedef std::integral_constant<int, NPH> NPHt;
    typedef std::integral_constant<int, NP0> NP0t;

    auto bias_init = [&](int boff, int rt) -> f32x4 {
        const float4 v = *reinterpret_cast<const float4*>(bias_l + boff + rt * 16 + 4 * grp);
        return (f32x4){v.x, v.y, v.z, v.w};
    };
    // an operand pair's hi words (lane group g: features F(s, g, 0..7)) into a natural-order [S][ld]
    // bf16 row: one v_permlane16_swap per dword pair gives lane group g features 32 s + 8 g + 0..7:
    // one 16-B store at the row base + 8 g elements, pair S at instruction offset 64 S
    auto store_ks = [&](u16* row, auto sc, const uint4& u) {
        constexpr int S = decltype(sc)::value;
        const auto xz = __builtin_amdgcn_permlane16_swap(u.x, u.z, false, false);
        const auto yw = __builtin_amdgcn_permlane16_swap(u.y, u.w, false, false);
        s3_st16o<64 * S>(row, make_uint4(xz[0], yw[0], xz[1], yw[1]));
        st_cur += 1;
    };
    const int colg = 8 * grp;

    S3Frag Bh[NPH], Bl[NPH], Oh[NPH], Ol[NPH];
    const float pi_f = 3.14159265358979323846f;

    // ---- the pair's dH partial: both waves leave their pixels' 9 terms in the pair buffer at the end
    //      of a tile; the first-half wave reduces the 32 pixels with k_step2's DPP tree after the next
    //      barrier (or after the loop) and stores k_step2's per-32-pixel partial
    long long dh_pending = -1;  // (first half) the pending partial's index
    auto flush_dH = [&]() {
        const float* pd = reinterpret_cast<const float*>(pbuf + PB_DH);
        float mine = 0.f;
#pragma unroll
        for (int e = 0; e < 9; ++e) {
            const float v = lo32 ? pd[e * 32 + lane] : 0.f;
            const float sm = wave_total63(v);
            const float sb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm), 63));
            if (lane == e) mine = sb;
        }
        s3_st4(lane < 9 ? (void*)(a.dH_partial + (size_t)dh_pending * 9 + lane) : (void*)dmy, mine);
        st_cur += 1;
        dh_pending = -1;
    };

    S3T_BEGIN(15);
    for (int ti = 0; ti < my_tiles; ++ti) {
        S3T_BEGIN(3);
        const int tile = tbase + ti * (int)gridDim.x;
        const int pb = ti & 1;
        const int b = tile / tpp;
        const int q0 = (tile - b * tpp) * TPX;
        const int p0 = q0 + PX * pblk;
        const long long slot0 = (long long)b * a.geo.Np_pad + p0;
        const long long myslot = slot0 + pxl;
        const int p = p0 + pxl;
        const bool valid = p < Np;
        const float* pro = pro_buf(pb);
        const int pix = PX * pblk + pxl;  // pixel within the block tile

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
            // layer-0 operand pair s, lane group g: k_step2's chunk c = 2 s + (g >> 1) of coordinate
            // g & 1: c < ng: bands 4 c + 0..3, sin then cos; c = ng: the raw coordinate; beyond: zero
            const float cd = (grp & 1) ? v : u;
            u16* row = (!a.fwd_only && !a.feat0_recompute) ? ly_ptr(0, 0) + myslot * ly_int(0, 3) : nullptr;
            const int ldf0 = row ? ly_int(0, 3) : 0;
            s3_sfor<NP0>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if (s < np0) {
                    const int c = 2 * s + (grp >> 1);
                    float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                    if (c < ng) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int k = 4 * c + i;
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
                    } else if (c == ng) {
                        f[0] = cd;
                    }
                    uint4 H, Lw;
                    s3_split8(f, H, Lw);
                    // feat_0 (bf16 hi) in k_step2's column order: chunk c of coordinate h at column
                    // 16 c + 8 h, zero columns up to ldf0
                    if (row) {
                        const bool st = c <= ng || 16 * c + 8 * (grp & 1) < ldf0;
                        s3_st16(st ? (void*)(row + 16 * c + 8 * (grp & 1)) : (void*)dmy, H);
                        st_cur += 1;
                    }
                    s3_fwd_pair(H, Lw, lo32, Bh[s], Bl[s]);
                }
            });
        }

        // ---- forward: layer 0, hidden layers.  Row tile rt of layer l: acc = bias + W . B, epilogue,
        //      the pair (2s, 2s + 1) -> operand pair s of layer l + 1 (+ feat_{l+1} store, mask words)
        auto fwd_layer = [&](int l, int np, auto np_tag, int r0) {
            const int nrt = FULL ? NRT : ly_int(l, 0);
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
                        if (l == 0 && rt == 0) {
                            // the next tile's target / mask / H into the other input buffer; the
                            // previous tile's dH partial (its terms are in the pair buffer)
                            if (ti + 1 < my_tiles) issue_pro(tile + (int)gridDim.x, pb ^ 1);
                            if (half == 0 && dh_pending >= 0) flush_dH();
                        }
                    }
                    f32x4 acc = bias_init(boff, rt);
                    S3T_BEGIN(6);
                    if (sub == 0)
                        gemm_f(acc, slot + sub * np * 1024, Bh, Bl, np, np_tag, PcOn());
                    else
                        gemm_f(acc, slot + sub * np * 1024, Bh, Bl, np, np_tag, PcOff());
                    S3T_END(6);
                    S3T_BEGIN(7);
                    const S3Ep e = s3_fwd_ep(acc);
                    asm volatile("" ::"v"(e.l0), "v"(e.l1));
                    mword = (mword << 2) | e.nib;
                    if constexpr (rt & 1) {
                        const uint4 H = make_uint4(ev.h0, ev.h1, e.h0, e.h1);
                        const uint4 Lw = make_uint4(ev.l0, ev.l1, e.l0, e.l1);
                        if (save) store_ks(srow, std::integral_constant<int, (rt >> 1)>(), H);
                        s3_fwd_pair(H, Lw, lo32, Oh[rt >> 1], Ol[rt >> 1]);
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
            for (int k = 0; k < NPH; ++k) {
                Bh[k] = Oh[k];
                Bl[k] = Ol[k];
            }
        };
        S3T_END(3);
        S3T_BEGIN(4);
        fwd_layer(0, np0, NP0t(), FULL ? R0F : a.r0);
        S3T_END(4);
        S3T_BEGIN(5);
        for (int l = 1; l < nl - 1; ++l) fwd_layer(l, NPH, NPHt(), 2);
        S3T_END(5);
        S3T_BEGIN(8);

        // ---- last layer: 3 outputs (rows 0..2 of one tile, lanes 0..15), sigmoid, masked MSE, d rgb
        float g[3] = {0.f, 0.f, 0.f};
        {
            f32x4 acc = bias_init(ly_int(nl - 1, 2), 0);
            const char* slot = stage_begin();
            gemm_f(acc, slot, Bh, Bl, NPH, NPHt(), PcOn());
            float* o = (a.rgb && valid && grp == 0) ? a.rgb + ((size_t)b * Np + p) * 3 : dmy;
            float yv[3] = {0.f, 0.f, 0.f};
            if (grp == 0) {
                const float m = valid ? (a.mask ? pro[3 * TPX + pix] : 1.0f) : 0.f;
                float sqf = 0.f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float z = acc[c];
                    const float yy = 1.0f / (1.0f + expf(-z));
                    yv[c] = yy;
                    const float tg = valid ? pro[c * TPX + pix] : 0.f;
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
        // g as a split pair: hi = bf16(g), lo = bf16(g - hi) (k_step2's Bg)
        float ghi[3], glo[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            ghi[c] = s3_lo16(s3_pk(g[c], 0.f));
            glo[c] = g[c] - ghi[c];
        }
        // ---- last-layer weight gradient, k_step2's chain: per 16 features one 16x16x32 MFMA with
        //      A = g^T (rows 0-2 hi, 4-6 lo; k = the 32 pixels of the pair), B = feat^T (the last layer's
        //      input, bf16 hi, through a transposing LDS round trip); the first-half wave runs pixels
        //      0..15 from 0, the second-half wave pixels 16..31 from that partial, then
        //      dW[c][f] += (row c) + (row 4 + c)
        if (grp == 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                gimg[c * 16 + pxl] = (u16)(s3_pk(ghi[c], 0.f) & 0xffff);
                gimg[(4 + c) * 16 + pxl] = (u16)(s3_pk(glo[c], 0.f) & 0xffff);
            }
        }
        asm volatile("" ::: "memory");
        S3Frag ga;  // A: this wave's half of k (lane groups 2 half, 2 half + 1), zero elsewhere
        {
            const int rc = lane & 15, kg = lane >> 4;
            const uint4 t = *reinterpret_cast<const uint4*>(gimg + (rc & 7) * 16 + 8 * (kg & 1));
            ga.u = ((kg >> 1) == half && rc < 8 && (rc & 3) < 3) ? t : make_uint4(0, 0, 0, 0);
        }
        float* const xb = a.xbuf + (((size_t)blockIdx.x * 4 + W) * XQ) * 128 + (lane & 31) * 4;  // [q][32 lanes][4]
        auto dw_last = [&](float* xv) {  // xv: the pair's partial (second half: in; first half: 12-float staging)
            const int q = (lane & 15) >> 2, pq = lane & 3, kg = lane >> 4;
            s3_sfor<NPH>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                __builtin_amdgcn_sched_barrier(0);  // one pair at a time (the scheduler would hoist every read)
                const uint4 hv = s3_mid(Bh[s], Bl[s]);
                asm volatile("" ::: "memory");
                uint2* w2 = reinterpret_cast<uint2*>(scr + pxl * 32);  // natural feature order of the pair
                w2[4 * (grp >> 1) + (grp & 1)] = make_uint2(hv.x, hv.y);
                w2[4 * (grp >> 1) + 2 + (grp & 1)] = make_uint2(hv.z, hv.w);
                asm volatile("" ::: "memory");
#pragma unroll
                for (int fb = 0; fb < 2; ++fb) {
                    const u16* b0 = scr + (8 * (kg & 1) + q) * 32 + 16 * fb + 4 * pq;
                    i16x4 vv[2] = {s3_tr16(b0), s3_tr16(b0 + 4 * 32)};
                    const bf16x8 bt = *reinterpret_cast<bf16x8*>(vv);
                    const int m = 2 * s + fb;
                    if (half == 0) {
                        // rows 0..2 of lanes 0..31 (hi rows of group 0, lo rows of group 1): 3 floats per
                        // MFMA, stored 16 B per lane every 4 MFMAs
                        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga.f, bt, (f32x4){}, 0, 0, 0);
                        const int mm = m & 3;
                        xv[3 * mm] = d[0];
                        xv[3 * mm + 1] = d[1];
                        xv[3 * mm + 2] = d[2];
                        if (mm == 3) {
#pragma unroll
                            for (int k = 0; k < 3; ++k) {
                                const int qd = 3 * (m >> 2) + k;
                                s3_st16(lo32 ? (void*)(xb + qd * 128) : (void*)dmy,
                                        make_uint4(__float_as_uint(xv[4 * k]), __float_as_uint(xv[4 * k + 1]),
                                                   __float_as_uint(xv[4 * k + 2]), __float_as_uint(xv[4 * k + 3])));
                            }
                        }
                    } else {
                        const f32x4 x0 = lo32 ? (f32x4){xv[3 * m], xv[3 * m + 1], xv[3 * m + 2], 0.f} : (f32x4){};
                        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga.f, bt, x0, 0, 0, 0);
                        float lo[3];
#pragma unroll
                        for (int c = 0; c < 3; ++c) lo[c] = __shfl_down(d[c], 16, 64);
                        if (lane < 16 && 32 * s < a.Kl) {  // (a narrower last-layer input: zero pairs past Kl)
#pragma unroll
                            for (int c = 0; c < 3; ++c) wla[c * a.Kl + 32 * s + 16 * fb + lane] += d[c] + lo[c];
                        }
                    }
                }
            });
        };
        if (half == 0) {
            float xv[12];
            dw_last(xv);
            st_cur += XQ;
            xflush = true;  // the partner loads them after the next barrier
        }

        S3T_END(9);
        S3T_BEGIN(10);
        // ---- last-layer dgrad: dfeat = W_{n-1}^T g as ONE MFMA per row tile, [hd | ld] with B = [gB | gB]
        //      (lane group 0: k = [g hi (3), 0, g lo (3), 0], k_step2's Bg), mask -> dz_{n-1}; one
        //      stage holds every row tile's fragments (tile rt at rt KB)
        S3Frag gB1;
        {
            float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (grp == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    f[c] = ghi[c];
                    f[4 + c] = glo[c];
                }
            }
            const uint32_t w[4] = {s3_pk(f[0], f[1]), s3_pk(f[2], f[3]), s3_pk(f[4], f[5]), s3_pk(f[6], f[7])};
            uint32_t o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = __builtin_amdgcn_permlane32_swap(w[q], w[q], false, false)[0];
            gB1.u = make_uint4(o[0], o[1], o[2], o[3]);
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
                        const bf16x8 A = *reinterpret_cast<const bf16x8*>(slot + rt * 1024 + oD1());
                        mf(acc, A, gB1.f);
                        if constexpr (rt == 0) dma_burst();
                        S3T_END(11);
                    } else {
                        if constexpr ((rt & 1) == 0) slot = stage_begin();
                        S3T_BEGIN(11);
                        gemm_b(acc, slot + (rt & 1) * NPH * 1024, Bh, Bl, NPHt(),
                               std::integral_constant<bool, (rt & 1) == 0>());
                        S3T_END(11);
                    }
                    S3T_BEGIN(12);
                    const uint2 hw = s3_bwd_ep<2 * (7 - (rt & 7))>(acc, mw);
                    if constexpr (rt & 1) {
                        const uint4 H = make_uint4(hv0, hv1, hw.x, hw.y);
                        store_ks(brow, std::integral_constant<int, (rt >> 1)>(), H);
                        s3_bwd_pair(H, Oh[rt >> 1], Ol[rt >> 1]);
                    } else {
                        hv0 = hw.x;
                        hv1 = hw.y;
                    }
                    S3T_END(12);
                } else if constexpr ((rt & 1) == 0) {
                    Oh[rt >> 1].u = Ol[rt >> 1].u = make_uint4(0, 0, 0, 0);
                }
            });
#pragma unroll
            for (int k = 0; k < NPH; ++k) {
                Bh[k] = Oh[k];
                Bl[k] = Ol[k];
            }
        };
        {
            const char* slot = stage_begin();
            if (half == 1) {  // the second half of the pair's dW_last chain, from the partner's partial
                float xv[3 * 2 * NPH];
                typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int qd = 0; qd < XQ; ++qd) {
                    const u32x4v t = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(xb + qd * 128));
                    xv[4 * qd] = __uint_as_float(t[0]);
                    xv[4 * qd + 1] = __uint_as_float(t[1]);
                    xv[4 * qd + 2] = __uint_as_float(t[2]);
                    xv[4 * qd + 3] = __uint_as_float(t[3]);
                }
                dw_last(xv);
            }
            bwd_pass(nl - 1, nl - 2, FULL ? NRT : ly_int(nl - 1, 1), slot, true);
        }
        for (int l = nl - 2; l >= 1; --l) bwd_pass(l, l - 1, FULL ? NRT : ly_int(l, 1), nullptr, false);
        S3T_END(10);
        S3T_BEGIN(13);

        // ---- layer-0 dgrad + posenc adjoint: row tile t < ng, register r of lane group G holds band
        //      4 t + r of coordinate G >> 1, the sin slot for even G, the cos slot for odd G; tile ng
        //      the raw coordinates (register 0 of groups 0 (u) and 2 (v)).  One v_permlane16_swap gives
        //      each lane its partner group's slot of the same band, so every lane forms the band's term
        //      as k_step2 and torch's autograd of sin / cos do, (g_sin cos - g_cos sin) 2^k pi,
        //      accumulated over the bands in increasing k, then the raw coordinate
        float dc = 0.f;
        {
            const int nta = FULL ? ng + 1 : a.nta;
            const float cd = (grp >> 1) ? v : u;
            const bool sinl = (grp & 1) == 0;
            const char* slot = nullptr;
            s3_sfor<NTA>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                if (t < nta) {
                    if constexpr ((t & 1) == 0) slot = stage_begin();
                    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
                    gemm_b(acc, slot + (t & 1) * NPH * 1024, Bh, Bl, NPHt(), std::integral_constant<bool, (t & 1) == 0>());
                    if (t < ng) {
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
                    } else if (t == ng) {
                        dc += acc[0];  // (read from groups 0 and 2 only)
                    }
                }
            });
        }
        S3T_END(13);
        S3T_BEGIN(14);
        // ---- (u, v) = X[:2] / (X[2] + 1e-8) backward, the bmm backward -> the pixel's dH terms
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
            if (grp == 0) {
                float* pd = reinterpret_cast<float*>(pbuf + PB_DH);
#pragma unroll
                for (int e = 0; e < 9; ++e) pd[e * 32 + 16 * half + pxl] = h9[e];
            }
            if (half == 0) dh_pending = ((long long)b * a.geo.Np_pad + q0 + 32 * W) / 32;
        }
        S3T_END(14);
    }
    S3T_END(15);
#ifdef MARF_STAMPS
    if (a.stamps && threadIdx.x == 0)
        for (int k = 0; k < 16; ++k) a.stamps[(size_t)blockIdx.x * 16 + k] = tacc[k];
#endif

    // ---- per-block partials (fixed order over k_step2's waves W = 0..3)
    s3_wait_vm<0>();
    __syncthreads();
    if (half == 0 && dh_pending >= 0) flush_dH();
    if (grp == 0) {
        reinterpret_cast<double*>(pbuf + PB_LSQ)[16 * half + pxl] = lsq;
        reinterpret_cast<double*>(pbuf + PB_LMS)[16 * half + pxl] = lms;
        float* pl = reinterpret_cast<float*>(pbuf + PB_BL);
        pl[16 * half + pxl] = bl0;
        pl[32 + 16 * half + pxl] = bl1;
        pl[64 + 16 * half + pxl] = bl2;
    }
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);  // the ring is idle now
    if (half == 0) {
        const double* pl2 = reinterpret_cast<const double*>(pbuf + PB_LSQ);
        const double* pm2 = reinterpret_cast<const double*>(pbuf + PB_LMS);
        const float* pl = reinterpret_cast<const float*>(pbuf + PB_BL);
        const double s0 = wave_total63(lo32 ? pl2[lane] : 0.0), s1 = wave_total63(lo32 ? pm2[lane] : 0.0);
        const float t0 = wave_total63(lo32 ? pl[lane] : 0.f), t1 = wave_total63(lo32 ? pl[32 + lane] : 0.f);
        const float t2 = wave_total63(lo32 ? pl[64 + lane] : 0.f);
        if (lane == 63) {
            red[W * 5 + 0] = s0;
            red[W * 5 + 1] = s1;
            red[W * 5 + 2] = (double)t0;
            red[W * 5 + 3] = (double)t1;
            red[W * 5 + 4] = (double)t2;
        }
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        double s = 0.0;
        float sf = 0.f;
        for (int w = 0; w < 4; ++w) {
            s += red[w * 5 + threadIdx.x];
            sf += (float)red[w * 5 + threadIdx.x];
        }
        if (threadIdx.x < 2) a.loss_partial[2 * (size_t)blockIdx.x + threadIdx.x] = s;
        else a.blast_partial[3 * (size_t)blockIdx.x + threadIdx.x - 2] = sf;
    }
    for (int e = threadIdx.x; e < 3 * a.Kl; e += NW * 64) {
        float s = 0.f;
        for (int w = 0; w < 4; ++w)
            s += reinterpret_cast<const float*>(smem + a.lds_wave + (w + 4) * a.lds_wave_bytes + W_WLA)[e];
        a.wlast_partial[(size_t)blockIdx.x * 3 * a.Kl + e] = s;
    }
}

// ------------------------------------------------------------------ weight program packing

// output feature of row r of 16-row output tile rt (the pair of tiles (2 s, 2 s + 1) packs to operand
// pair s: lane group g of tile 2 s + b holds features 32 s + 16 (g >> 1) + 8 b + 4 (g & 1) + 0..3)
MARF_DEV int s3_mrow(int rt, int r) { return 32 * (rt >> 1) + 16 * (r >> 3) + 8 * (rt & 1) + 4 * ((r >> 2) & 1) + (r & 3); }
// operand pair feature F(s, g, j) = k_step2's s2_kperm(chunk 2 s + (g >> 1), g & 1, j)
MARF_DEV int s3_kfeat(int s, int g, int j) { return 32 * s + 16 * (g >> 1) + 8 * (j >> 2) + 4 * (g & 1) + (j & 3); }
// layer-0 operand pair feature of the reference's [x, y, posenc] vector (model/planar.py:451-471:
// posenc = [sin bands of x, of y, cos ...] at 2 + 2 h L + (cos ? L : 0) + band): k_step2's
// s2_l0_fwd_feature of chunk 2 s + (g >> 1), coordinate g & 1; -1: a zero slot
MARF_DEV int s3_l0_feature(int s, int g, int j, int L, int ng) {
    const int c = 2 * s + (g >> 1), h = g & 1;
    if (c == ng) return j == 0 ? h : -1;
    if (c > ng) return -1;
    const int k = 4 * c + (j & 3);
    if (k >= L) return -1;
    return 2 + 2 * h * L + (j >= 4 ? L : 0) + k;
}
// layer-0 input feature of adjoint row r of tile t (-1: none)
MARF_DEV int s3_adj_feature(int t, int r, int L, int ng) {
    const int G = r >> 2, i = r & 3;
    if (t == ng) return (i == 0 && (G & 1) == 0) ? (G >> 1) : -1;
    if (t > ng) return -1;
    const int k = 4 * t + i;
    if (k >= L) return -1;
    return 2 + 2 * (G >> 1) * L + ((G & 1) ? L : 0) + k;
}

// One thread per (stage, part, fragment, lane, element).  Stage sequence per tile: layer-0 forward
// (r0 row tiles of np0 pairs each), hidden forward (pairs of row tiles), last layer, last-layer
// dgrad (every row tile's fragment), hidden dgrad l = nl-2 .. 1 (pairs), adjoint (pairs).
// A fragment of row tile rt, pair s: lane l holds row r = l & 15, k positions (s, g = l >> 4, j).
__global__ void k_pack3(const float* __restrict__ params, u16* __restrict__ prog, float* __restrict__ bias_out,
                        int* __restrict__ kmap, Pack2Args a) {
    const int per_slot = s3::SLOT / 2;
    const long long total = (long long)a.n_stages * per_slot;
    const int D = a.dims[0];
    const int ng = (a.L + 3) / 4, np0 = a.nk0;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total + a.nbias + D; e += (long long)gridDim.x * 256) {
        if (e >= total + a.nbias) {
            // layer-0 column map of feat_0 (k_step2's column order): true input feature f -> column
            const int f = (int)(e - total - a.nbias), L = a.L, ngc = (L + 3) / 4;
            int col;
            if (f < 2) col = 16 * ngc + 8 * f;
            else {
                const int q = f - 2, hh = q / (2 * L), rr = q - hh * 2 * L, cosp = rr >= L, k = rr - cosp * L;
                col = 16 * (k / 4) + 8 * hh + 4 * cosp + (k % 4);
            }
            kmap[f] = col;
            continue;
        }
        if (e >= total) {  // padded bias table, rows in the output tiles' order (s3_mrow)
            const int be = (int)(e - total);
            float v = 0.f;
            for (int l = 0; l < a.nl; ++l) {
                const bool last = l == a.nl - 1;
                const int nbias = last ? 32 : a.Mp[l];
                if (be >= a.boff[l] && be < a.boff[l] + nbias) {
                    const int mm = be - a.boff[l];
                    const int m = last ? mm : s3_mrow(mm >> 4, mm & 15);
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
        int layer = -1, kind = -1, rt = 0, ps = 0;  // kind 0 fwd, 1 last fwd, 2 last dgrad, 3 hidden dgrad, 4 adjoint
        {
            int s = st;
            if (s < a.ns0) {
                layer = 0;
                kind = 0;
                rt = s * a.r0 + idx / np0;
                ps = idx % np0;
                if (idx >= a.r0 * np0 || rt >= a.nrt[0]) kind = -1;
            } else {
                s -= a.ns0;
                for (int l = 1; l < a.nl - 1 && layer < 0; ++l) {
                    if (s < a.nrt[l] / 2) {
                        layer = l;
                        kind = 0;
                        rt = 2 * s + idx / 8;
                        ps = idx % 8;
                    } else {
                        s -= a.nrt[l] / 2;
                    }
                }
                if (layer < 0) {
                    if (s == 0) {
                        layer = a.nl - 1;
                        kind = 1;
                        rt = idx / 8;
                        ps = idx % 8;
                        if (rt > 0) kind = -1;
                    } else if (s == 1) {
                        layer = a.nl - 1;
                        kind = 2;
                        rt = idx;
                        ps = 0;
                        if (rt >= a.nrtb[layer]) kind = -1;
                    } else {
                        s -= 2;
                        for (int l = a.nl - 2; l >= 1 && layer < 0; --l) {
                            if (s < a.nrtb[l] / 2) {
                                layer = l;
                                kind = 3;
                                rt = 2 * s + idx / 8;
                                ps = idx % 8;
                            } else {
                                s -= a.nrtb[l] / 2;
                            }
                        }
                        if (layer < 0 && s < (a.nta + 1) / 2) {
                            layer = 0;
                            kind = 4;
                            rt = 2 * s + idx / 8;
                            ps = idx % 8;
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
            const float* Wt = params + a.w_off[layer];
            int m = -1, k = -1;  // W[m][k]
            if (kind == 0 && layer == 0) {
                m = s3_mrow(rt, r16);
                k = s3_l0_feature(ps, g, j, a.L, ng);
            } else if (kind == 0) {
                m = s3_mrow(rt, r16);
                k = s3_kfeat(ps, g, j);
            } else if (kind == 1) {
                m = r16;  // the last layer's outputs (rows 0..2)
                k = s3_kfeat(ps, g, j);
            } else if (kind == 2) {  // rows = input features of the last layer, k = [g hi (3), 0, g lo (3), 0]
                if (g == 0 && (j & 3) < 3) {
                    m = j & 3;
                    k = s3_mrow(rt, r16);
                }
            } else if (kind == 3) {  // W_l^T: row = input feature of layer l, k = its output
                m = s3_kfeat(ps, g, j);
                k = s3_mrow(rt, r16);
            } else {  // adjoint: row = layer-0 input slot, k = layer-0 output
                m = s3_kfeat(ps, g, j);
                k = s3_adj_feature(rt, r16, a.L, ng);
            }
            if (m >= 0 && k >= 0 && m < Mt && k < Kt) {
                val = Wt[(size_t)m * Kt + k];
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

template <int NP0T, bool FULL>
static hipError_t launch_step3_t(const Step2Args& a, int grid, hipStream_t s) {
    hipError_t e = ensure_dynamic_lds((const void*)k_step3<NP0T, FULL>, (size_t)a.lds_total);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_step3<NP0T, FULL>), dim3(grid), dim3(s3::NW * 64), (size_t)a.lds_total, s, a);
    return hipGetLastError();
}

// full = every hidden layer 256 wide (the host checks): 2 and 3 layer-0 pairs (L <= 12, L <= 20)
// get their own code; the generic instantiation covers the rest.  8 waves per block.
bool marf_step3_nw_ok(bool, int, int nw) { return nw == 8; }
hipError_t marf_launch_step3(const Step2Args& a, bool full, int nw, int grid, hipStream_t s) {
    if (nw != 8 || a.nk0 < 1 || a.nk0 > s3::NP0MAX) return hipErrorInvalidValue;
    if (full && a.nk0 == 2) return launch_step3_t<2, true>(a, grid, s);
    if (full && a.nk0 == 3) return launch_step3_t<3, true>(a, grid, s);
    return launch_step3_t<s3::NP0MAX, false>(a, grid, s);
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
