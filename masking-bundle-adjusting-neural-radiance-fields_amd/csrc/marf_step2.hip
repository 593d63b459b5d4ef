// marf_step2.hip -- the fused training step in the pixel-per-wave form (gfx950).
//
// Same contract as k_mlp_step (marf_step.hip): per pixel grid -> sl(3) warp -> posenc + c2f ->
// MLP forward -> sigmoid -> masked-MSE partial -> d rgb -> dgrad chain -> posenc / warp adjoint,
// writing the layer inputs feat_l and the pre-activation gradients dz_l that the weight-gradient
// kernels (marf_wgrad.hip) consume (model/planar.py:329-391, warp.py:33-81).  The mapping onto the
// CU is different:
//
//   * one wave owns 32 pixels and computes EVERY feature of them; a 32x32 accumulator tile of
//     layer l (rows = features, column = the lane's pixel) is, after ReLU and bf16 packing, the B
//     operand of layer l+1 as it stands (CDNA "accumulator as the next MFMA's operand": registers
//     8s..8s+7 form k-step s, with the k order permuted inside the step).  Activations never touch
//     LDS; the weights are packed in the matching k order.
//   * the weights (MFMA A operand) stream through a 3-slot LDS ring shared by all waves of the
//     block: one slot = one 32-row tile of one layer's matrix, filled by global_load_lds_dwordx4
//     (issued by every wave, 1 KB per instruction) two stages ahead of its use.  The block is
//     persistent (one per CU) and the per-tile stage sequence repeats, so the stream never stops
//     between pixel tiles.
//   * the ReLU masks of the forward are packed into one word per lane per pair of row tiles and
//     kept in wave-private LDS until the dgrad pass reads them (no mask records in HBM).
//   * split-bf16 mode (MARF_BF16X3): weights and forward activations are carried as bf16 hi + lo
//     pairs, the forward is hi*hi + hi*lo + lo*hi (fp32 accumulation, ~16 significant bits) and
//     the dgrad is W_hi^T dz + W_lo^T dz; dz and the saved tensors stay bf16.  This is the precision
//     recipe that keeps the seed-3 planar run in the reference's basin.
//
// Memory ordering: all global traffic inside the tile loop is inline asm (LDS-DMA, stores) so the
// compiler inserts no vmcnt waits of its own.  Each wave counts the store instructions it issues
// per stage (st_cur / st_prev), and the wait for a ring slot is the vmcnt that leaves exactly the
// operations younger than that slot's DMA in flight (wait_ring).
#include <type_traits>

#include "marf_args.h"

namespace marf {

// ------------------------------------------------------------------ inline-asm memory ops

// LDS-DMA, 4 B per lane (256 B per wave instruction)
MARF_DEV void s2_glds4(const void* src, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}
// Stores outside the compiler's bookkeeping: the s_nop covers the store-data hazard (the data
// registers may be rewritten right after), which hipcc pads only for its own stores.
typedef uint32_t s2_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t s2_u32x4 __attribute__((ext_vector_type(4)));
MARF_DEV void s2_st8(void* dst, uint32_t a, uint32_t b) {
    const s2_u32x2 v = {a, b};
    asm volatile("global_store_dwordx2 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
MARF_DEV void s2_st16(void* dst, uint4 u) {
    const s2_u32x4 v = {u.x, u.y, u.z, u.w};
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
template <int OFF>
MARF_DEV void s2_st16o(void* base, uint4 u) {  // 16 B at base + OFF bytes (instruction offset)
    const s2_u32x4 v = {u.x, u.y, u.z, u.w};
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2\n\ts_nop 1" ::"v"(base), "v"(v), "n"(OFF) : "memory");
}
MARF_DEV void s2_st12(void* dst, float a, float b, float c) {
    typedef float f32x3 __attribute__((ext_vector_type(3)));
    f32x3 v = {a, b, c};
    asm volatile("global_store_dwordx3 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
MARF_DEV void s2_st4(void* dst, float a) {
    asm volatile("global_store_dword %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(a) : "memory");
}
template <int N>
MARF_DEV void s2_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

MARF_DEV i16x4 s2_tr16(const u16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(p));
}

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1
template <int... I, class F>
MARF_DEV void s2_sfor_impl(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>()), ...);
}
template <int N, class F>
MARF_DEV void s2_sfor(F&& f) {
    s2_sfor_impl(std::make_integer_sequence<int, N>(), f);
}

// two floats -> packed bf16 pair (v_cvt_pk_bf16_f32, RNE)
MARF_DEV uint32_t s2_pk(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){a, b}), bf16x2));
}
MARF_DEV float s2_lo16(uint32_t w) { return __uint_as_float(w << 16); }
MARF_DEV float s2_hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

union S2Frag {
    bf16x8 f;
    f16x8 h;  // (the fp16-forward recipe's operands)
    uint4 u;
    uint32_t w[4];
};

// two floats -> packed fp16 pair (v_cvt_pk_f16_f32, RNE)
MARF_DEV uint32_t s2_pkh(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){a, b}), f16x2));
}

// 8 floats -> bf16 hi fragment (+ lo remainder fragment)
template <bool LO>
MARF_DEV void s2_split8(const float* x, S2Frag& hi, S2Frag& lo) {
    hi.u = make_uint4(s2_pk(x[0], x[1]), s2_pk(x[2], x[3]), s2_pk(x[4], x[5]), s2_pk(x[6], x[7]));
    if constexpr (LO) {
        const uint32_t w[4] = {hi.u.x, hi.u.y, hi.u.z, hi.u.w};
        float r[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            r[2 * q] = x[2 * q] - s2_lo16(w[q]);
            r[2 * q + 1] = x[2 * q + 1] - s2_hi16(w[q]);
        }
        lo.u = make_uint4(s2_pk(r[0], r[1]), s2_pk(r[2], r[3]), s2_pk(r[4], r[5]), s2_pk(r[6], r[7]));
    }
}

// ------------------------------------------------------------------ the kernel

// Diagnostic phase timing (MARF_STAMPS builds): wave 0 of each block sums s_memtime deltas per
// phase category; tools/step2_phases.py reads them.
#ifdef MARF_STAMPS
#define S2T_BEGIN(k) const unsigned long long _t##k = __builtin_amdgcn_s_memtime()
#define S2T_END(k) tacc[k] += __builtin_amdgcn_s_memtime() - _t##k
#else
#define S2T_BEGIN(k) \
    do {         \
    } while (0)
#define S2T_END(k) \
    do {       \
    } while (0)
#endif

template <int HM, bool SPLIT, int NW, int MAXR, bool DZ = false>
struct S2Cfg {
    static constexpr int NKH = HM / 16;                    // k-steps of a hidden-width operand
    static constexpr int NRT = HM / 32;                    // row tiles of a hidden-width output
    static constexpr int SLOT = NKH * 1024 * (SPLIT ? 2 : 1);
    static constexpr int LO = NKH * 1024;                  // byte offset of the lo fragments in a slot
    static constexpr int PER_DMA = SLOT / (NW * 1024);     // DMA instructions per wave per stage
    static constexpr int NSLOT = 3, D = 2;
    // pixel sets (tiles) whose dgrad shares each weight stage: the split recipe's dgrad operands are
    // bf16 hi only, so at one wave per SIMD two 32-pixel sets fit the register file there (the
    // forward's hi + lo activations do not); the 8-wave plain variant has 256 registers per wave
    // (DZ: the dgrad operand dz split hi + lo as well: one set, its lo in the lo arrays)
    static constexpr int NS = SPLIT && !DZ ? 2 : 1;
    static constexpr int NK0 = 9;                          // max layer-0 k-steps (L <= 32)
    static constexpr int NTA = 5;                          // max adjoint row tiles (L <= 39)
    static constexpr int TPX = 32 * NW;                    // pixel slots per block tile
    static constexpr int NMW = NRT / 2;                    // mask words per ReLU layer
    static constexpr int MSET = MAXR * NMW * 64;           // mask words of one pixel set (per wave)
    static_assert(PER_DMA * NW * 1024 == SLOT, "slot size");
};

// NK0F: 0 = the generic instantiation (layer-0 k-steps, row tiles per stage and layer widths read at
// run time); > 0 = a full-width net (every hidden layer HM wide) with NK0F layer-0 k-steps and NTAF
// adjoint row tiles, whose layer-0 stages, GEMM lengths and row-tile counts are compile-time (no
// live-k-step branches; 10.4 -> 9.5 ms at C3, profiles/r4r)
// DZ (split recipe, opt-in MARF_STEP2_DZ=1): the hidden dgrad GEMMs also split their dz operand,
// W_hi^T dz_hi + W_lo^T dz_hi + W_hi^T dz_lo (the forward's three terms), one pixel set per dgrad
// pass; dz_1 (the layer-0 adjoint's operand) and the saved dz stay bf16 hi.  DESIGN.md §4: the
// recipe whose emulation reaches fp32's basin rate.
// HF (the fp16x2 recipe, MARF_FP16X2): every MFMA in fp16 -- weights fp16 hi + lo, activations and
// dz single fp16, W_hi a + W_lo a in the forward and W_hi^T dz + W_lo^T dz in the dgrad (2 MFMAs per
// MAC) -- and, since one 32-pixel set's operands then take half the registers, the forward of a
// group's TWO tiles in one pass over the forward stages (every weight fragment read from LDS once
// for both sets, every stage DMA'd once per pair of tiles, as the dgrad already is).  dz carries an
// exact 2^10 gradient scale; the saved tensors are fp16 and the weight gradients run in fp16
// (marf_wgrad.hip PrecF16, the 2^-10 in the reduction).  Compile-time layer-0 instantiations only
// (full-width nets).
template <int HM, bool SPLIT, int NW, int MAXR, int NK0F, int NTAF, bool DZ, bool HF = false>
__device__ __attribute__((always_inline)) inline void k_step2_body(const Step2Args& a) {
    typedef S2Cfg<HM, SPLIT, NW, MAXR, DZ> C;
    constexpr bool SDZ = SPLIT && DZ;
    constexpr int NKH = C::NKH, NRT = C::NRT, NS = C::NS;
    constexpr bool FIX = NK0F > 0;
    static_assert(NK0F <= C::NK0, "layer-0 k-steps");
    static_assert(!HF || (SPLIT && !DZ && NK0F > 0 && NS == 2), "fp16x2: split dgrad, two sets, compile-time layer 0");
    // the hidden dgrad of a group's two pixel sets in one pass per weight stage (compile-time nets;
    // MARF_STEP2_J2=0 at build time keeps one pass per set for A/B)
#ifndef MARF_STEP2_J2
#define MARF_STEP2_J2 1
#endif
    constexpr bool J2 = MARF_STEP2_J2 && NS == 2 && SPLIT && !SDZ && FIX;
    // HF: the dgrad's gradient scale (the saved dz carry it; the host's weight-gradient reduction
    // multiplies by its inverse, marf_abi.hip step2_backward)
    constexpr float kGS = 1024.f;
    constexpr int R0Q = NKH / (FIX ? NK0F : NKH);  // layer-0 row tiles per stage (the host's r0)
    constexpr int R0F = R0Q < 1 ? 1 : (R0Q > NRT ? NRT : R0Q);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, pxl = lane & 31;
    const int nl = a.nl, L = a.L;

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
    u16* trs = reinterpret_cast<u16*>(wpriv);                 // 1 KB transpose scratch
    u16* gts = reinterpret_cast<u16*>(wpriv + 1024);          // 1 KB g^T image [16][32]
    uint32_t* mkl = reinterpret_cast<uint32_t*>(wpriv + 2048);  // ReLU mask words [NS][MAXR][NMW][64]
    float* wla = reinterpret_cast<float*>(wpriv + 2048 + NS * C::MSET * 4);  // [3][Kl] dW_last
    float* dmy = a.dummy + (((size_t)blockIdx.x * NW + wave) * 2 * 64 + lane) * 2;
#ifdef MARF_STAMPS
    unsigned long long tacc[16] = {};
#endif

    // ---- constants into LDS (plain loads: the compiler's waits are harmless before the ring)
    for (int e = threadIdx.x; e < a.nbias; e += NW * 64) bias_l[e] = a.bias[e];
    if ((int)threadIdx.x < 32) c2f_l[threadIdx.x] = (int)threadIdx.x < L ? a.c2f_w[threadIdx.x] : 0.f;
    for (int e = threadIdx.x; e < nl * (int)(sizeof(S2Layer) / 4); e += NW * 64)
        reinterpret_cast<uint32_t*>(lyr)[e] = reinterpret_cast<const uint32_t*>(a.layers)[e];
    for (int e = lane; e < 512; e += 64) reinterpret_cast<uint32_t*>(gts)[e] = 0u;
    for (int e = lane; e < 3 * a.Kl; e += 64) wla[e] = 0.f;

    const int tpp = a.geo.Np_pad / C::TPX;   // block tiles per patch
    const int Np = a.geo.Np;
    // this launch's tiles: tile0 + blockIdx.x + i gridDim.x < n_tiles (one piece of a pipelined step,
    // or all of them)
    const int tbase = a.tile0 + (int)blockIdx.x;
    int my_tiles = 0;
    if (tbase < a.n_tiles) my_tiles = (a.n_tiles - 1 - tbase) / (int)gridDim.x + 1;
    // Stage order of a group of NS tiles: the forward stages of each tile, then ONE pass of the
    // dgrad stages for all of them (render: forward stages only)
    const int nF = a.n_fwd, nB = a.n_stages - a.n_fwd;
    // (HF: one pass of the forward stages per group as well)
    const int total = HF ? ((my_tiles + NS - 1) / NS) * (nF + nB)
                         : (my_tiles / NS) * (NS * nF + nB) + (my_tiles % NS ? (my_tiles % NS) * nF + nB : 0);

    // ---- per-tile input DMA: target r, g, b, mask (TPX floats each) and H (9 floats) of a tile
    auto pro_buf = [&](int pb) -> float* { return reinterpret_cast<float*>(smem + a.lds_pro + pb * (4 * C::TPX + 64) * 4); };
    auto issue_pro = [&](int tile, int pb) {
        const int b = tile / tpp, q0 = (tile - b * tpp) * C::TPX;
        const unsigned base = lds0 + a.lds_pro + pb * (4 * C::TPX + 64) * 4;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int f = ((wave * 2 + i) * 64) + lane;   // float index in [0, 4 TPX)
            const int ch = f / C::TPX, q = f - ch * C::TPX;
            const int p = min(q0 + q, Np - 1);
            const float* src = !a.gt ? a.pro_fallback
                               : ch < 3 ? a.gt + ((size_t)b * 3 + ch) * Np + p
                                        : (a.mask ? a.mask + (size_t)b * Np + p : a.gt + (size_t)b * 3 * Np + p);
            s2_glds4(src, __builtin_amdgcn_readfirstlane(base + (wave * 2 + i) * 256));
        }
        s2_glds4(a.geo.Hm ? a.geo.Hm + 9 * (size_t)b + (lane < 9 ? lane : 0) : a.pro_fallback,
                 __builtin_amdgcn_readfirstlane(base + 4 * C::TPX * 4));
    };

    // ---- HF: the per-group inputs.  The H rows of a group's two tiles go to H buffer (group parity,
    // set) at the previous group's first layer-0 stage; the targets / masks of its two tiles to target
    // buffer (set) at the previous group's first dgrad stage, after its last layer read them.  A
    // group's missing second tile (odd tile count) repeats the first one's inputs.
    auto hf_tile = [&](int ti) -> int { return tbase + min(ti, my_tiles - 1) * (int)gridDim.x; };
    auto proH = [&](int par, int set) -> const float* {
        return reinterpret_cast<const float*>(smem + a.lds_pro + (par * 2 + set) * 256);
    };
    auto proT = [&](int set) -> const float* {
        return reinterpret_cast<const float*>(smem + a.lds_pro + 1024 + set * C::TPX * 16);
    };
    auto issue_h = [&](int ti, int par) {  // 2 vector-memory operations per wave
#pragma unroll
        for (int set = 0; set < 2; ++set) {
            const int b = hf_tile(ti + set) / tpp;
            s2_glds4(a.geo.Hm ? a.geo.Hm + 9 * (size_t)b + (lane < 9 ? lane : 0) : a.pro_fallback,
                     __builtin_amdgcn_readfirstlane(lds0 + a.lds_pro + (par * 2 + set) * 256));
        }
    };
    auto issue_tgt = [&](int ti) {  // 4 vector-memory operations per wave
#pragma unroll
        for (int set = 0; set < 2; ++set) {
            const int tile = hf_tile(ti + set);
            const int b = tile / tpp, q0 = (tile - b * tpp) * C::TPX;
            const unsigned base = lds0 + a.lds_pro + 1024 + set * C::TPX * 16;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int f = ((wave * 2 + i) * 64) + lane;  // float index in [0, 4 TPX)
                const int ch = f / C::TPX, q = f - ch * C::TPX;
                const int p = min(q0 + q, Np - 1);
                const float* src = !a.gt ? a.pro_fallback
                                   : ch < 3 ? a.gt + ((size_t)b * 3 + ch) * Np + p
                                            : (a.mask ? a.mask + (size_t)b * Np + p : a.gt + (size_t)b * 3 * Np + p);
                s2_glds4(src, __builtin_amdgcn_readfirstlane(base + (wave * 2 + i) * 256));
            }
        }
    };

    // ---- the weight ring
    int c_stage = 0;         // global stage counter of this block
    int dma_stage = 0;       // next stage whose DMA is to be issued
    // DMA cursor over the group sequence: index in the group, its length, its tile count, first tile
    int dg_i = 0, dg_n = 0, dg_ns = 0, dg_t = 0;
    auto grp_init = [&](int t) {
        dg_t = t;
        dg_ns = HF ? 1 : min(NS, my_tiles - t);  // (HF: the forward stages once per group)
        dg_n = dg_ns * nF + nB;
        dg_i = 0;
    };
    grp_init(0);
    auto dma_next = [&]() -> int {  // program stage of the next DMA; the cursor advances
        const int i = dg_i;
        const int prog = i < nF ? i : (i < dg_ns * nF ? i - nF : i - (dg_ns - 1) * nF);
        if (++dg_i == dg_n) grp_init(dg_t + NS);
        return prog;
    };
    // The refill of the slot freed at a stage's barrier: PER_DMA pieces of 1 KB per wave, every
    // stage exactly once, all of them before the stage's first store.  Regular stages (one 16-k-step
    // GEMM per pixel set) issue them beside the MFMAs of the first GEMM (dma_piece<j> at fixed
    // k-steps); the others (layer 0, the last-layer dgrad) issue them right after the barrier.  A
    // piece is branch-free: m0 = the stage's LDS base, the VGPR address the stage's source, and the
    // instruction offset (j mod 4) KB moves both (the second half of the pieces from bases 4 KB on).
    // Past the last stage the ring refills the just-freed slot from program stage 0 (never read).
    unsigned dma_m0 = 0;
    const char* dma_va0 = nullptr;
    const char* dma_va1 = nullptr;
    auto dma_arm = [&]() {
        const int ps = dma_stage < total ? dma_next() : 0;
        dma_m0 = __builtin_amdgcn_readfirstlane(lds0 + (dma_stage % C::NSLOT) * C::SLOT + wave * C::PER_DMA * 1024);
        dma_va0 = a.prog + (size_t)ps * C::SLOT + wave * C::PER_DMA * 1024 + lane * 16;
        if constexpr (C::PER_DMA > 4) dma_va1 = dma_va0 + 4096;
        ++dma_stage;
    };
    auto dma_piece = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        static_assert(j < C::PER_DMA && C::PER_DMA <= 8, "piece index");
        const char* va = j < 4 ? dma_va0 : dma_va1;
        const unsigned m = dma_m0 + (j < 4 ? 0u : 4096u);
        unsigned keep;  // m0 is reserved to the compiler: saved and restored around the piece
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off offset:%3\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(va), "s"(m), "n"((j & 3) * 1024)
                     : "memory");
    };
    auto dma_burst = [&]() { s2_sfor<C::PER_DMA>([&](auto jc) { dma_piece(jc); }); };
    // vm-op accounting for the ring waits: st_cur counts the store instructions a wave issued since
    // the last stage_begin (all of them after that stage's DMA pieces), st_prev the count of the
    // stage before.  The DMA of stage c was issued during stage c-2, so st_prev + PER_DMA (the
    // pieces of stage c+1) + st_cur operations are younger than it: vmcnt(that) waits for it (any
    // smaller count is a stricter wait; the operations complete in order).
    int st_cur = 0, st_prev = 0;
    auto wait_ring = [&]() {
        const int y = st_prev + st_cur;
        constexpr int PD = C::PER_DMA;
        if (y >= 8) s2_wait_vm<PD + 8>();
        else if (y >= 6) s2_wait_vm<PD + 6>();
        else if (y >= 4) s2_wait_vm<PD + 4>();
        else if (y >= 2) s2_wait_vm<PD + 2>();
        else s2_wait_vm<PD>();
    };
    // wait for stage c_stage, publish it to every wave, arm the refill of the slot freed by stage
    // c_stage - 1 (burst: issue it now)
    auto stage_begin = [&](bool burst) -> const char* {
        S2T_BEGIN(0);
        S2T_BEGIN(12);
        wait_ring();
#ifdef MARF_STAMPS  // (the stamp splits the vm / lgkm wait from the barrier)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        S2T_END(12);
        st_prev = st_cur;
        st_cur = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        S2T_END(0);
        S2T_BEGIN(1);
        dma_arm();
        if (burst) dma_burst();
        S2T_END(1);
        const char* slot = smem + (c_stage % C::NSLOT) * C::SLOT;
        ++c_stage;
        return slot;
    };

    if (my_tiles > 0) {
        if constexpr (HF) {
            issue_h(0, 0);
            issue_tgt(0);
        } else {
            issue_pro(tbase, 0);
        }
        dma_arm();
        dma_burst();
        dma_arm();
        dma_burst();
    }
    s2_wait_vm<0>();
    __syncthreads();

    // running per-lane sums over this block's tiles (fixed order -> deterministic)
    double lsq = 0.0, lms = 0.0;
    float bl0 = 0.f, bl1 = 0.f, bl2 = 0.f;

    // ReLU mask words in wave-private LDS: word (set, layer, rt >> 1) of a lane, bit
    // (16 (1 - (rt & 1)) + 15 - r) = accumulator register r (the pair of row tiles is assembled in
    // a register, so each word is written once)
    uint32_t mpend = 0u;

    S2Frag Bh[NKH], Bl[NKH], Oh[NKH], Ol[NKH];

    // (the stores of a row tile into a saved tensor in the T16 block layout (marf_wgrad.hip
    //  t16_off: 32 pixels x 16 features per 1 KB block): k-step ks of the lane's pixel holds
    //  columns 16 ks + 4 h + 0..3 (dwords x, y) and 16 ks + 8 + 4 h + 0..3 (z, w); two
    //  v_permlane32_swap exchange the lane halves' x, y <-> z, w so that lane (p, h) holds columns
    //  16 ks + 8 h + 0..7 contiguously: one 16-B store per lane per k-step, and the 64 lanes' stores
    //  of k-step ks fill feature block ks of the set's 32 pixels, 1 KB contiguous (a row-major
    //  [S][ld] tensor took 32 segments of 32 B per instruction).  row0 = the lane's base in the
    //  set's block row (tensor + (slot0 / 32) * ld * 32 + pixel * 16 + 8 h); row tile rt = blocks
    //  2 rt, 2 rt + 1)
    auto store_rt = [&](u16* row0, auto rtc, const S2Frag& f0, const S2Frag& f1) {
        constexpr int rt = decltype(rtc)::value;
        auto contig = [&](const S2Frag& f) -> uint4 {
            const auto xz = __builtin_amdgcn_permlane32_swap(f.u.x, f.u.z, false, false);
            const auto yw = __builtin_amdgcn_permlane32_swap(f.u.y, f.u.w, false, false);
            return make_uint4(xz[0], yw[0], xz[1], yw[1]);
        };
        u16* blk = row0 + 1024 * rt;  // (2 KB per row tile: past the 12-bit instruction offset)
        s2_st16o<0>(blk, contig(f0));
        s2_st16o<1024>(blk, contig(f1));
        st_cur += 2;
    };

    // one 32-row output tile: acc (+)= A[ks] . B[ks] over NK k-steps from the slot
    //   MODE 0: plain; 1: split forward (hi.hi + hi.lo + lo.hi)
    // With one wave per SIMD the issue is in order, so the filler work of a k-step goes INTO the
    // gaps between its MFMAs (each gap hides ~24 cycles of issue): hook(ks, 0) after the first
    // MFMA, hook(ks, 1) after the second (right after the first in plain mode), the A-ring refill
    // of each register right after the last MFMA that reads it, the DMA piece after the last MFMA.
    // sched_barrier pins that order (left alone the scheduler sinks each LDS read to right before
    // its MFMA, exposing its latency, and bunches the VALU behind the MFMA chain).
    auto nohook = [&](auto, auto) {};
    // the stage's DMA pieces beside the MFMAs of a 16-k-step GEMM: piece j after k-step
    // (j + 1) NK / PER_DMA - 1 (PIECES: this GEMM is its stage's first)
    auto piece_at = [&](auto ksc, auto nk_tag, auto pieces_tag) {
        constexpr int ks = decltype(ksc)::value;
        constexpr int NK = decltype(nk_tag)::value;
        if constexpr (decltype(pieces_tag)::value) {
            static_assert(NK % C::PER_DMA == 0, "pieces per k-step");
            constexpr int per = NK / C::PER_DMA;
            if constexpr (ks % per == per - 1) dma_piece(std::integral_constant<int, ks / per>());
        }
    };
    typedef std::integral_constant<bool, true> PcOn;    // the GEMM issues its stage's DMA pieces
    typedef std::integral_constant<bool, false> PcOff;
    // one accumulation chain (a second, alternating accumulator measured no faster, and any change
    // of the summation order re-rolls the seed-3 basin: DESIGN.md §4)
    auto mf = [&](f32x16& acc, const uint4& x, const S2Frag& y) {
        if constexpr (HF)  // (the fp16x2 recipe: every MFMA in fp16)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, x), y.h, acc, 0, 0, 0);
        else
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, x), y.f, acc, 0, 0, 0);
    };
    // one 32-row output tile: acc (+)= A[ks] . B[ks] over NK k-steps from the slot
    //   MODE 0: plain; 1: split forward (hi.hi + hi.lo + lo.hi); 2: split dgrad (hi.B + lo.B)
    // With one wave per SIMD the issue is in order, so the filler work of a k-step goes INTO the
    // gaps between its MFMAs (each gap hides ~24 cycles of issue): hook(ks, 0) after the first
    // MFMA, hook(ks, 1) after the second (right after the first in plain mode), the A-ring refill
    // of each register right after the last MFMA that reads it, the DMA piece after the last MFMA.
    // sched_barrier pins that order (left alone the scheduler sinks each LDS read to right before
    // its MFMA, exposing its latency, and bunches the VALU behind the MFMA chain).
    auto gemm = [&](f32x16& acc, const char* slot, const S2Frag* Bhi, const S2Frag* Blo, int nk, auto mode_tag,
                    auto nk_tag, auto&& hook, auto pieces_tag) {
        constexpr int MODE = decltype(mode_tag)::value;
        constexpr int NK = decltype(nk_tag)::value;
        typedef std::integral_constant<int, 0> P0;
        typedef std::integral_constant<int, 1> P1;
        const uint4* ah = reinterpret_cast<const uint4*>(slot + lane * 16);
        const uint4* al = reinterpret_cast<const uint4*>(slot + C::LO + lane * 16);
        constexpr int P = NK < 4 ? NK : 4;
        uint4 A0[4], A1[4];
#pragma unroll
        for (int u = 0; u < P; ++u) {
            A0[u] = ah[u * 64];
            if constexpr (MODE != 0) A1[u] = al[u * 64];
        }
        s2_sfor<NK>([&](auto ksc) {
            constexpr int ks = decltype(ksc)::value;
            constexpr int u = ks & 3;
            constexpr bool refill = ks + P < NK;
            const bool live = NK != C::NK0 || ks < nk;
            auto piece = [&]() { piece_at(ksc, nk_tag, pieces_tag); };
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (MODE == 0) {
                if (live) {
                    mf(acc, A0[u], Bhi[ks]);
                    hook(ksc, P0());
                    hook(ksc, P1());
                }
                if constexpr (refill) A0[u] = ah[(ks + P) * 64];
                if (live) piece();
            } else if constexpr (MODE == 2) {
                if (live) {
                    mf(acc, A0[u], Bhi[ks]);
                    hook(ksc, P0());
                }
                if constexpr (refill) A0[u] = ah[(ks + P) * 64];
                __builtin_amdgcn_sched_barrier(0);
                if (live) {
                    mf(acc, A1[u], Bhi[ks]);
                    hook(ksc, P1());
                }
                if constexpr (refill) A1[u] = al[(ks + P) * 64];
                if (live) piece();
            } else {
                if (live) {
                    mf(acc, A0[u], Bhi[ks]);
                    hook(ksc, P0());
                }
                __builtin_amdgcn_sched_barrier(0);
                if (live) {
                    mf(acc, A0[u], Blo[ks]);
                    hook(ksc, P1());
                }
                if constexpr (refill) A0[u] = ah[(ks + P) * 64];
                __builtin_amdgcn_sched_barrier(0);
                if (live) mf(acc, A1[u], Bhi[ks]);
                if constexpr (refill) A1[u] = al[(ks + P) * 64];
                if (live) piece();
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    typedef std::integral_constant<int, SPLIT ? 1 : 0> MFt;
    typedef std::integral_constant<int, SPLIT ? 2 : 0> MBt;
    // the hidden dgrad GEMMs: the forward's split mode when dz is split too (SDZ), else MBt
    typedef std::integral_constant<int, SDZ ? 1 : (SPLIT ? 2 : 0)> MDt;
    typedef std::integral_constant<int, NKH> NKHt;
    typedef std::integral_constant<int, C::NK0> NK0t;
    // layer 0's GEMM length: compile-time NK0F (every k-step live) or NK0 with a run-time count
    typedef std::conditional_t<FIX, std::integral_constant<int, FIX ? NK0F : 1>, NK0t> NK0x;
    const int nk0 = FIX ? NK0F : a.nk0, r0 = FIX ? R0F : a.r0;
    typedef std::integral_constant<int, 1> NK1t;

    auto bias_init = [&](int boff, int rt) -> f32x16 {
        f32x16 acc;
        const float* bb = bias_l + boff + rt * 32 + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = *reinterpret_cast<const float4*>(bb + 8 * q);
            acc[4 * q] = v.x;
            acc[4 * q + 1] = v.y;
            acc[4 * q + 2] = v.z;
            acc[4 * q + 3] = v.w;
        }
        return acc;
    };
    // forward epilogue: ReLU, mask bits, next-layer operand fragments (k-steps 2 rt, 2 rt + 1)
    // row tiles past a narrower layer's width: zero operand fragments (the padded weights are zero,
    // and 0 * stale bits could be NaN)
    auto zero_out = [&](S2Frag& o0, S2Frag& o1, S2Frag& q0, S2Frag& q1) {
        o0.u = o1.u = q0.u = q1.u = make_uint4(0, 0, 0, 0);
    };
    // pipelined epilogues: micro-steps of one 32-row accumulator tile
    struct EpSt {
        uint32_t bits, mw;
        float vp, xo;
        uint32_t hw[8], lw[8];
        float ta, tb;  // split pack in two halves: the f32 values of the hi pair
    } ep;
    f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};
    // forward step e: ReLU + mask bit of register e (frelu); the odd steps then pack the (hi, lo)
    // bf16 pair of registers e-1, e (fpack)
    auto frelu = [&](const f32x16& pa, auto ec) {
        constexpr int e = decltype(ec)::value;
        // relu as a signed-integer max with 0 (negative floats and -0 are negative integers: exactly
        // x > 0 ? x : 0); the mask bits come from the packed bf16 pair (mask_pair)
        float x;
        asm volatile("v_max_i32_e32 %0, 0, %1" : "=&v"(x) : "v"(pa[e]));
        if constexpr (e & 1) ep.xo = x;
        else ep.vp = x;
    };
    // ReLU mask bits of a packed (relu'd) bf16 pair w: per 16-bit half (w_half != 0), shifted into
    // ep.bits as two streams -- after the 8 pairs of a row tile the even elements' bits sit at
    // 7 - j and the odd elements' at 23 - j (pair j).  (w_half != 0) equals z > 0 except for
    // 0 < z < 2^-134, which rounds to a zero bf16 and would otherwise pass a dz of a feature whose
    // forward value is a zero hi + a denormal lo: 2 VALU per pair instead of 2 per element.
    const uint32_t k_pair1 = 0x00010001u;
    auto mask_pair = [&](uint32_t w) {
        uint32_t t;
        asm volatile(
            "v_pk_min_u16 %1, %2, %3\n\t"
            "v_lshl_or_b32 %0, %0, 1, %1"
            : "+v"(ep.bits), "=&v"(t)
            : "v"(w), "s"(k_pair1));
    };
    // (inline asm so that the IR passes cannot sink the packing to its use after the GEMM: it is
    //  meant to run in the MFMA gap where the hook places it; v_cvt_pk_bf16_f32 rounds to nearest
    //  even, as s2_pk)
    auto fpack = [&](auto ec) {
        constexpr int e = decltype(ec)::value;
        if constexpr (e & 1) {
            if constexpr (SPLIT) {
                uint32_t w, wl, t0, t1;
                asm volatile(
                    "v_cvt_pk_bf16_f32 %0, %4, %5\n\t"
                    "v_lshlrev_b32_e32 %2, 16, %0\n\t"
                    "v_and_b32_e32 %3, 0xffff0000, %0\n\t"
                    "v_sub_f32_e32 %2, %4, %2\n\t"
                    "v_sub_f32_e32 %3, %5, %3\n\t"
                    "v_cvt_pk_bf16_f32 %1, %2, %3"
                    : "=&v"(w), "=&v"(wl), "=&v"(t0), "=&v"(t1)
                    : "v"(ep.vp), "v"(ep.xo));
                ep.hw[e >> 1] = w;
                ep.lw[e >> 1] = wl;
                mask_pair(w);
            } else {
                uint32_t w;
                asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(w) : "v"(ep.vp), "v"(ep.xo));
                ep.hw[e >> 1] = w;
                mask_pair(w);
            }
        }
    };
    // the split pack in two halves (the same operations as fpack): A = the hi pair and its f32
    // values, B = the lo pair (the remainders); B of a pair must precede the next frelu (it reads
    // the pair's values, which the next even step overwrites)
    auto fpackA = [&](auto ec) {
        constexpr int e = decltype(ec)::value;
        static_assert(e & 1, "odd step");
        uint32_t w;
        float t0, t1;
        asm volatile(
            "v_cvt_pk_bf16_f32 %0, %3, %4\n\t"
            "v_lshlrev_b32_e32 %1, 16, %0\n\t"
            "v_and_b32_e32 %2, 0xffff0000, %0"
            : "=&v"(w), "=&v"(t0), "=&v"(t1)
            : "v"(ep.vp), "v"(ep.xo));
        ep.hw[e >> 1] = w;
        ep.ta = t0;
        ep.tb = t1;
        mask_pair(w);
    };
    auto fpackB = [&](auto ec) {
        constexpr int e = decltype(ec)::value;
        static_assert(e & 1, "odd step");
        uint32_t wl;
        float r0, r1;
        asm volatile(
            "v_sub_f32_e32 %1, %3, %5\n\t"
            "v_sub_f32_e32 %2, %4, %6\n\t"
            "v_cvt_pk_bf16_f32 %0, %1, %2"
            : "=&v"(wl), "=&v"(r0), "=&v"(r1)
            : "v"(ep.vp), "v"(ep.xo), "v"(ep.ta), "v"(ep.tb));
        ep.lw[e >> 1] = wl;
    };
    auto fstep = [&](const f32x16& pa, auto ec) {
        frelu(pa, ec);
        fpack(ec);
    };
    // The steps E0..15 of an epilogue that run after the GEMM (nothing to hide them beside): the
    // same operations as frelu / fpack in plain C++, so the compiler interleaves the pairs' chains
    // (the volatile asm of the in-gap steps keeps each pair's 6-deep chain in program order), then
    // the mask bits in pair order as mask_pair does.  E0 even.
    auto fsteps_free = [&](const f32x16& pa, auto e0c) {
        constexpr int E0 = decltype(e0c)::value;
        static_assert((E0 & 1) == 0, "whole pairs");
        uint32_t w[8];
        s2_sfor<(16 - E0) / 2>([&](auto jc) {
            constexpr int q = E0 / 2 + decltype(jc)::value;
            const float x0 = __int_as_float(max(__float_as_int(pa[2 * q]), 0));
            const float x1 = __int_as_float(max(__float_as_int(pa[2 * q + 1]), 0));
            const uint32_t hw = s2_pk(x0, x1);
            w[q] = hw;
            ep.hw[q] = hw;
            if constexpr (SPLIT) ep.lw[q] = s2_pk(x0 - s2_lo16(hw), x1 - s2_hi16(hw));
        });
        s2_sfor<(16 - E0) / 2>([&](auto jc) { mask_pair(w[E0 / 2 + decltype(jc)::value]); });
    };
    // forward finish of tile rt: operand fragments of k-steps 2 rt, 2 rt + 1, mask word, 2 stores
    // (last: the layer's last row tile -- an odd row-tile count (a width of 32 mod 64) stores its
    //  mask word without the odd partner's bits)
    auto ffinish = [&](int l, auto rtc, bool save, u16* srow, uint32_t* mks, bool last) {
        constexpr int rt = decltype(rtc)::value;
        Oh[2 * rt].u = make_uint4(ep.hw[0], ep.hw[1], ep.hw[2], ep.hw[3]);
        Oh[2 * rt + 1].u = make_uint4(ep.hw[4], ep.hw[5], ep.hw[6], ep.hw[7]);
        if constexpr (SPLIT) {
            Ol[2 * rt].u = make_uint4(ep.lw[0], ep.lw[1], ep.lw[2], ep.lw[3]);
            Ol[2 * rt + 1].u = make_uint4(ep.lw[4], ep.lw[5], ep.lw[6], ep.lw[7]);
        }
        if constexpr ((rt & 1) == 0) {
            mpend = ep.bits << 8;
            if (last) mks[(l * C::NMW + (rt >> 1)) * 64 + lane] = mpend;
        } else {
            mks[(l * C::NMW + (rt >> 1)) * 64 + lane] = mpend | ep.bits;
        }
        if (save) store_rt(srow, rtc, Oh[2 * rt], Oh[2 * rt + 1]);
    };
    // dgrad step e: dz = acc * relu'(z) with the mask word e.mw
    auto bstep = [&](EpSt& es, const f32x16& pa, auto ec, auto rtc) {
        constexpr int e = decltype(ec)::value;
        constexpr int rt = decltype(rtc)::value;
        // (mask_pair's layout: pair e >> 1, odd elements in the upper stream, even row tiles << 8)
        constexpr int bit = 16 * (e & 1) + 8 * (1 - (rt & 1)) + 7 - (e >> 1);
        float x;
        asm volatile(  // x = relu'(z) ? acc : 0 from the mask bit (in the gap, as fpack)
            "v_bfe_i32 %0, %1, %3, 1\n\t"
            "v_and_b32_e32 %0, %0, %2"
            : "=&v"(x)
            : "v"(es.mw), "v"(pa[e]), "n"(bit));
        if constexpr (e & 1) {
            uint32_t w;
            if constexpr (HF)
                asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(w) : "v"(es.vp), "v"(x));
            else
                asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(w) : "v"(es.vp), "v"(x));
            es.hw[e >> 1] = w;
            if constexpr (SDZ) es.lw[e >> 1] = s2_pk(es.vp - s2_lo16(w), x - s2_hi16(w));
        } else {
            es.vp = x;
        }
    };
    // bstep for all 16 elements at once in plain C++ (the same v_bfe / v_and / v_cvt_pk operations)
    // for epilogues with no MFMA gaps to hide in: the compiler interleaves the elements' chains
    auto bsteps_free = [&](EpSt& es, const f32x16& pa, auto rtc) {
        constexpr int rt = decltype(rtc)::value;
        s2_sfor<8>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int b0 = 16 * 0 + 8 * (1 - (rt & 1)) + 7 - q, b1 = 16 * 1 + 8 * (1 - (rt & 1)) + 7 - q;
            const float x0 = __int_as_float(__builtin_amdgcn_sbfe((int)es.mw, b0, 1) & __float_as_int(pa[2 * q]));
            const float x1 = __int_as_float(__builtin_amdgcn_sbfe((int)es.mw, b1, 1) & __float_as_int(pa[2 * q + 1]));
            es.hw[q] = HF ? s2_pkh(x0, x1) : s2_pk(x0, x1);
            if constexpr (SDZ) es.lw[q] = s2_pk(x0 - s2_lo16(es.hw[q]), x1 - s2_hi16(es.hw[q]));
        });
    };
    auto bfinish = [&](EpSt& es, S2Frag* O, auto rtc, u16* row0) {
        constexpr int rt = decltype(rtc)::value;
        O[2 * rt].u = make_uint4(es.hw[0], es.hw[1], es.hw[2], es.hw[3]);
        O[2 * rt + 1].u = make_uint4(es.hw[4], es.hw[5], es.hw[6], es.hw[7]);
        if constexpr (SDZ) {  // (one pixel set: its lo output in the lo array)
            Ol[2 * rt].u = make_uint4(es.lw[0], es.lw[1], es.lw[2], es.lw[3]);
            Ol[2 * rt + 1].u = make_uint4(es.lw[4], es.lw[5], es.lw[6], es.lw[7]);
        }
        store_rt(row0, rtc, O[2 * rt], O[2 * rt + 1]);
    };
    // ---- the fp16x2 forward (HF): helpers
    // one 32-row output tile of BOTH pixel sets: c_s += A_hi . B_s + A_lo . B_s over NK k-steps (fp16
    // MFMAs), each A fragment read from LDS once for the two sets.  Per k-step the order is (set 0,
    // hi), (set 1, hi), (set 0, lo), (set 1, lo): each set's chain is hi, lo per k-step, as one set
    // alone would run it.  hook(ks, p) runs in the gap after MFMA p (0..3) of k-step ks.
    // (F16 = false: the same pass in bf16 -- the split dgrad of two pixel sets, W_hi^T dz + W_lo^T dz
    //  per set in the split recipe's order, so the same bits as one GEMM pass per set)
    auto gemm2 = [&](f32x16& c0, f32x16& c1, const char* slot, const S2Frag* B0, const S2Frag* B1, auto nk_tag,
                     auto&& hook, auto pieces_tag, auto f16_tag) {
        constexpr int NK = decltype(nk_tag)::value;
        constexpr bool F16 = decltype(f16_tag)::value;
        typedef std::integral_constant<int, 0> P0;
        typedef std::integral_constant<int, 1> P1;
        typedef std::integral_constant<int, 2> P2;
        typedef std::integral_constant<int, 3> P3;
        auto mma = [&](f32x16& c, const uint4& av, const S2Frag& b) {
            if constexpr (F16)
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, av), b.h, c, 0, 0, 0);
            else
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av), b.f, c, 0, 0, 0);
        };
        const uint4* ah = reinterpret_cast<const uint4*>(slot + lane * 16);
        const uint4* al = reinterpret_cast<const uint4*>(slot + C::LO + lane * 16);
        constexpr int P = NK < 4 ? NK : 4;
        uint4 A0[4], A1[4];
#pragma unroll
        for (int u = 0; u < P; ++u) {
            A0[u] = ah[u * 64];
            A1[u] = al[u * 64];
        }
        s2_sfor<NK>([&](auto ksc) {
            constexpr int ks = decltype(ksc)::value;
            constexpr int u = ks & 3;
            constexpr bool refill = ks + P < NK;
            __builtin_amdgcn_sched_barrier(0);
            mma(c0, A0[u], B0[ks]);
            hook(ksc, P0());
            __builtin_amdgcn_sched_barrier(0);
            mma(c1, A0[u], B1[ks]);
            hook(ksc, P1());
            if constexpr (refill) A0[u] = ah[(ks + P) * 64];
            __builtin_amdgcn_sched_barrier(0);
            mma(c0, A1[u], B0[ks]);
            hook(ksc, P2());
            __builtin_amdgcn_sched_barrier(0);
            mma(c1, A1[u], B1[ks]);
            hook(ksc, P3());
            if constexpr (refill) A1[u] = al[(ks + P) * 64];
            piece_at(ksc, nk_tag, pieces_tag);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    typedef std::integral_constant<bool, true> F16t;
    typedef std::integral_constant<bool, false> BF16t;
    // epilogue of a 32-row accumulator tile of set s, per pair q of registers (2q, 2q + 1): ReLU of
    // both (integer max with 0, as frelu), the fp16 operand pair into the next layer's fragment
    // (k-step 2 rt + q / 4, word q mod 4) -- also the saved tensor -- and the ReLU mask bits from the
    // pair rounded to bf16 (mask_pair's layout; bf16 keeps fp32's exponent range, so a bit is set
    // exactly for z > 0 as in the split recipe, where fp16 would drop 0 < z < 2^-25)
    struct Ep2 {
        float x[4][2];
        uint32_t bw[8];
        uint32_t bits, mpend;
    };
    Ep2 e2[2];
    auto mask_pair_to = [&](uint32_t& bits, uint32_t w) {
        uint32_t t;
        asm volatile(
            "v_pk_min_u16 %1, %2, %3\n\t"
            "v_lshl_or_b32 %0, %0, 1, %1"
            : "+v"(bits), "=&v"(t)
            : "v"(w), "s"(k_pair1));
    };
    // pair operation op (0: ReLU of element 2q, 1: of 2q + 1, 2: the two packs, 3: the mask bits) of
    // flattened pair PI = 8 s + q, held in temporary slot j
    auto hop = [&](const f32x16& p0s, const f32x16& p1s, S2Frag* O0, S2Frag* O1, auto rtc, auto pic, auto jc, auto opc) {
        constexpr int rt = decltype(rtc)::value, PI = decltype(pic)::value, j = decltype(jc)::value;
        constexpr int op = decltype(opc)::value;
        if constexpr (PI < 16) {
            constexpr int sset = PI >> 3, q = PI & 7;
            const f32x16& pa = sset ? p1s : p0s;
            Ep2& es = e2[sset];
            if constexpr (op < 2) {
                float x;
                asm volatile("v_max_i32_e32 %0, 0, %1" : "=&v"(x) : "v"(pa[2 * q + op]));
                es.x[j][op] = x;
            } else if constexpr (op == 2) {
                uint32_t w, wb;
                asm volatile(
                    "v_cvt_pk_f16_f32 %0, %2, %3\n\t"
                    "v_cvt_pk_bf16_f32 %1, %2, %3"
                    : "=&v"(w), "=&v"(wb)
                    : "v"(es.x[j][0]), "v"(es.x[j][1]));
                (sset ? O1 : O0)[2 * rt + (q >> 2)].w[q & 3] = w;
                es.bw[q] = wb;
            } else {
                mask_pair_to(es.bits, es.bw[q]);
            }
        }
    };
    typedef std::integral_constant<int, 0> I0;
    typedef std::integral_constant<int, 1> I1;
    typedef std::integral_constant<int, 2> I2;
    typedef std::integral_constant<int, 3> I3;
    // the epilogue of row tile rt (accumulators p0s, p1s) in the gaps of the next GEMM: PPK pairs per
    // k-step, pairs in order (set 0's eight, then set 1's)
    auto hook2 = [&](const f32x16& p0s, const f32x16& p1s, S2Frag* O0, S2Frag* O1, auto rtc, auto ksc, auto pc,
                     auto ppkc) {
        constexpr int ks = decltype(ksc)::value, p = decltype(pc)::value, PPK = decltype(ppkc)::value;
        typedef std::integral_constant<int, PPK * ks> Pa;
        typedef std::integral_constant<int, PPK * ks + 1> Pb;
        if constexpr (PPK == 1) {
            hop(p0s, p1s, O0, O1, rtc, Pa(), I0(), pc);
        } else if constexpr (PPK == 4) {
            // (layer 0's 5-k-step GEMMs: all 16 pairs in the gaps) gap p: op p of pairs 4 ks .. 4 ks + 3
            s2_sfor<4>([&](auto jc) {
                hop(p0s, p1s, O0, O1, rtc, std::integral_constant<int, PPK * ks + decltype(jc)::value>(), jc, pc);
            });
        } else {
            static_assert(PPK == 2, "pairs per k-step");
            if constexpr (p == 0) {
                hop(p0s, p1s, O0, O1, rtc, Pa(), I0(), I0());
                hop(p0s, p1s, O0, O1, rtc, Pa(), I0(), I1());
            } else if constexpr (p == 1) {
                hop(p0s, p1s, O0, O1, rtc, Pa(), I0(), I2());
                hop(p0s, p1s, O0, O1, rtc, Pb(), I1(), I0());
            } else if constexpr (p == 2) {
                hop(p0s, p1s, O0, O1, rtc, Pb(), I1(), I1());
                hop(p0s, p1s, O0, O1, rtc, Pa(), I0(), I3());
            } else {
                hop(p0s, p1s, O0, O1, rtc, Pb(), I1(), I2());
                hop(p0s, p1s, O0, O1, rtc, Pb(), I1(), I3());
            }
        }
    };
    // pairs PI0 .. 15 after the GEMM (no gaps left): plain C++, so the compiler interleaves the
    // pairs' chains; the mask bits in pair order
    auto free_pairs = [&](const f32x16& p0s, const f32x16& p1s, S2Frag* O0, S2Frag* O1, auto rtc, auto pi0c) {
        constexpr int rt = decltype(rtc)::value, PI0 = decltype(pi0c)::value;
        if constexpr (PI0 < 16) {
            s2_sfor<16 - PI0>([&](auto jc) {
                constexpr int PI = PI0 + decltype(jc)::value, sset = PI >> 3, q = PI & 7;
                const f32x16& pa = sset ? p1s : p0s;
                const float x0 = __int_as_float(max(__float_as_int(pa[2 * q]), 0));
                const float x1 = __int_as_float(max(__float_as_int(pa[2 * q + 1]), 0));
                (sset ? O1 : O0)[2 * rt + (q >> 2)].w[q & 3] = s2_pkh(x0, x1);
                e2[sset].bw[q] = s2_pk(x0, x1);
            });
            s2_sfor<16 - PI0>([&](auto jc) {
                constexpr int PI = PI0 + decltype(jc)::value;
                mask_pair_to(e2[PI >> 3].bits, e2[PI >> 3].bw[PI & 7]);
            });
        }
    };
    // finish of row tile rt of set s: the mask word (two row tiles per word) and the stores of the
    // saved tensor -- the fp16 operand fragments themselves (the weight gradients run in fp16)
    auto ffinish2 = [&](int l, auto rtc, auto sc, bool save, u16* srow, bool last) {
        constexpr int rt = decltype(rtc)::value, sset = decltype(sc)::value;
        const S2Frag* O = sset ? Ol : Oh;
        Ep2& es = e2[sset];
        uint32_t* mks = mkl + sset * C::MSET;
        if constexpr ((rt & 1) == 0) {
            es.mpend = es.bits << 8;
            if (last) mks[(l * C::NMW + (rt >> 1)) * 64 + lane] = es.mpend;
        } else {
            mks[(l * C::NMW + (rt >> 1)) * 64 + lane] = es.mpend | es.bits;
        }
        if (save) store_rt(srow, rtc, O[2 * rt], O[2 * rt + 1]);
    };
    f32x16 hacc[4];  // HF: current (0, 1) and previous (2, 3) row tile of sets 0, 1 (alternating)

    const float pi_f = 3.14159265358979323846f;

    // what the dgrad pass keeps of each pixel set's forward: the g operand, the warp's homogeneous
    // point and the tile (-1: no tile; the set's stores go to the sink rows); the rest is recomputed
    struct SetSt {
        S2Frag g;
        float X0, X1, X2;
        int tile;
    };
    SetSt ss[NS];

    S2T_BEGIN(7);
    for (int it = 0; it < my_tiles; it += NS) {
        const int nset = min(NS, my_tiles - it);
        if constexpr (HF) {
            // ---- the fp16x2 forward of the group's two pixel sets (set 1 of a last, single tile
            //      repeats set 0's inputs; its stores go to the sink rows, its loss terms are zero)
            S2T_BEGIN(4);
            const int gp = (it / NS) & 1;
            int tl[2];
            long long sl[2];  // the set's first pixel slot of the wave (a missing set: the sink rows)
            bool real[2];
            float Xs[2][3];
            S2Frag F0[2][NK0F > 0 ? NK0F : 1];
            s2_sfor<2>([&](auto sc) {
                constexpr int sset = decltype(sc)::value;
                real[sset] = it + sset < my_tiles;
                const int tile = hf_tile(it + sset);
                tl[sset] = tile;
                const int b = tile / tpp;
                const int p0 = (tile - b * tpp) * C::TPX + 32 * wave;
                sl[sset] = real[sset] ? (long long)b * a.geo.Np_pad + p0 : a.S + 32 * wave;
                const float* hm = proH(gp, sset);
                float Hm[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) Hm[e] = hm[e];
                const int p = p0 + pxl;
                float x, y, u, v, X[3];
                if (a.geo.mode == 1) {  // explicit coordinates (render only)
                    const int pc = min(p, Np - 1);
                    u = x = a.geo.coords[2 * (size_t)pc];
                    v = y = a.geo.coords[2 * (size_t)pc + 1];
                    X[0] = u;
                    X[1] = v;
                    X[2] = 1.0f;
                } else {
                    const int r = p / a.geo.w, cc = p - r * a.geo.w;
                    x = grid_coord(a.geo.x0 + cc, a.geo.W, a.geo.norm_w);
                    y = grid_coord(a.geo.y0 + r, a.geo.H, a.geo.norm_h);
                    warp_point(Hm, x, y, u, v, X, a.geo.bmm_small);
                }
                Xs[sset][0] = X[0];
                Xs[sset][1] = X[1];
                Xs[sset][2] = X[2];
                const float cd = h ? v : u;
                // posenc + c2f: band groups of 4 (sin, cos) and the raw coordinate, as fp16 operands;
                // feat_0 (the fp16 operand) only when the layer-0 weight gradient does not recompute it
                const bool st0 = !a.fwd_only && !a.feat0_recompute;
                u16* row0 = st0 ? ly_ptr(0, 0) + (sl[sset] >> 5) * ly_int(0, 3) * 32 + pxl * 16 + 8 * h : nullptr;
                s2_sfor<NK0F>([&](auto gc) {
                    constexpr int g = decltype(gc)::value;
                    float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                    if constexpr (g < NK0F - 1) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int k = 4 * g + j;
                            float sn = 0.f, co = 0.f;
                            if (k < L) {
                                band_sincos<true>(cd, k, sn, co);
                                if (a.c2f_on) {
                                    const float w = c2f_l[k];
                                    sn = sn * w;
                                    co = co * w;
                                }
                            }
                            f[j] = sn;
                            f[4 + j] = co;
                        }
                    } else {
                        f[0] = cd;
                    }
                    F0[sset][g].u = make_uint4(s2_pkh(f[0], f[1]), s2_pkh(f[2], f[3]), s2_pkh(f[4], f[5]), s2_pkh(f[6], f[7]));
                    if (st0) s2_st16(row0 + 512 * g, F0[sset][g].u);
                });
                if (st0) {
                    st_cur += NK0F;
                    if (16 * NK0F < ly_int(0, 3)) {
                        s2_st16(row0 + 512 * NK0F, make_uint4(0, 0, 0, 0));
                        st_cur += 1;
                    }
                }
            });
            S2T_END(4);
            // ---- forward, layer 0 then the hidden layers: one stage per 32-row output tile (layer
            //      0: r0 row tiles per stage); the epilogue of row tile rt-1 of both sets runs in the
            //      MFMA gaps of row tile rt, the last row tile's right after its own MFMAs
            auto fwd2_layer = [&](int l, const S2Frag* B0, const S2Frag* B1, auto nk_tag, auto ppk_tag) {
                constexpr int NK = decltype(nk_tag)::value, PPK = decltype(ppk_tag)::value;
                typedef std::integral_constant<bool, NK == NKH> PcL;  // hidden: pieces in the GEMM
                const bool save = l + 1 < nl - 1 && !a.fwd_only;
                u16* srow[2];
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    srow[q] = save ? ly_ptr(l + 1, 0) + (sl[q] >> 5) * ly_int(l + 1, 3) * 32 + pxl * 16 + 8 * h : nullptr;
                const int boff = ly_int(l, 2);
                const char* slotb = nullptr;
                s2_sfor<NRT>([&](auto rtc) {
                    constexpr int rt = decltype(rtc)::value;
                    f32x16& c0 = hacc[(rt & 1) ? 2 : 0];
                    f32x16& c1 = hacc[(rt & 1) ? 3 : 1];
                    f32x16& q0 = hacc[(rt & 1) ? 0 : 2];
                    f32x16& q1 = hacc[(rt & 1) ? 1 : 3];
                    const int sub = l == 0 ? rt % R0F : 0;
                    S2T_BEGIN(15);
                    c0 = bias_init(boff, rt);  // (before the stage wait: the reads overlap it)
                    c1 = c0;
                    S2T_END(15);
                    if (sub == 0) slotb = stage_begin(l == 0);  // layer 0: the pieces in a burst
                    const char* slot = slotb + sub * NK * 1024;
                    if (l == 0 && rt == 0 && it + NS < my_tiles) {
                        issue_h(it + NS, gp ^ 1);  // (the buffer's last reader finished before this barrier)
                        st_cur += 2;
                    }
                    if constexpr (rt == 0) {
                        S2T_BEGIN(8);
                        gemm2(c0, c1, slot, B0, B1, nk_tag, nohook, PcL(), F16t());
                        S2T_END(8);
                    } else {
                        typedef std::integral_constant<int, rt - 1> RP;
                        e2[0].bits = 0;
                        e2[1].bits = 0;
                        S2T_BEGIN(8);
                        gemm2(c0, c1, slot, B0, B1, nk_tag, [&](auto ksc, auto pc) {
                            hook2(q0, q1, Oh, Ol, RP(), ksc, pc, ppk_tag);
                        }, PcL(), F16t());
                        S2T_END(8);
                        S2T_BEGIN(13);
                        free_pairs(q0, q1, Oh, Ol, RP(), std::integral_constant<int, PPK * NK>());
                        S2T_END(13);
                        S2T_BEGIN(10);
                        ffinish2(l, RP(), I0(), save, srow[0], false);
                        ffinish2(l, RP(), I1(), save, srow[1], false);
                        S2T_END(10);
                    }
                    if constexpr (rt == NRT - 1) {
                        S2T_BEGIN(13);
                        e2[0].bits = 0;
                        e2[1].bits = 0;
                        free_pairs(c0, c1, Oh, Ol, rtc, I0());
                        ffinish2(l, rtc, I0(), save, srow[0], true);
                        ffinish2(l, rtc, I1(), save, srow[1], true);
                        S2T_END(13);
                    }
                });
#pragma unroll
                for (int k = 0; k < NKH; ++k) {
                    Bh[k] = Oh[k];
                    Bl[k] = Ol[k];
                }
            };
            S2T_BEGIN(5);
            S2T_BEGIN(14);
            fwd2_layer(0, F0[0], F0[1], std::integral_constant<int, NK0F>(), std::integral_constant<int, 4>());
            S2T_END(14);
            for (int l = 1; l < nl - 1; ++l) fwd2_layer(l, Bh, Bl, NKHt(), I1());
            S2T_END(5);
            S2T_BEGIN(6);

            // ---- last layer of both sets: 3 outputs (rows 0..2 of one tile), sigmoid, masked MSE, d rgb
            float gS[2][3];
            {
                f32x16& c0 = hacc[0];
                f32x16& c1 = hacc[1];
                c0 = bias_init(ly_int(nl - 1, 2), 0);
                c1 = c0;
                const char* slot = stage_begin(false);
                gemm2(c0, c1, slot, Bh, Bl, NKHt(), nohook, PcOn(), F16t());
                s2_sfor<2>([&](auto sc) {
                    constexpr int sset = decltype(sc)::value;
                    const f32x16& acc = sset ? c1 : c0;
                    const int b = tl[sset] / tpp;
                    const int p = (tl[sset] - b * tpp) * C::TPX + 32 * wave + pxl;
                    const bool valid = real[sset] && p < Np;
                    const float* pt = proT(sset);
                    float* o = (a.rgb && valid && h == 0) ? a.rgb + ((size_t)b * Np + p) * 3 : dmy;
                    float yv[3] = {0.f, 0.f, 0.f};
                    gS[sset][0] = gS[sset][1] = gS[sset][2] = 0.f;
                    if (h == 0) {
                        const float m = valid ? (a.mask ? pt[3 * C::TPX + 32 * wave + pxl] : 1.0f) : 0.f;
                        float sqf = 0.f;
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const float z = acc[c];
                            const float yy = 1.0f / (1.0f + expf(-z));
                            yv[c] = yy;
                            const float t = valid ? pt[c * C::TPX + 32 * wave + pxl] : 0.f;
                            // model/planar.py:388-390 and its autograd: x = (p - g) m, d = 2 x m
                            const float xx = (yy - t) * m;
                            sqf += xx * xx;
                            const float d = (2.0f * xx) * m;
                            gS[sset][c] = (d * (1.0f - yy)) * yy;  // sigmoid backward
                        }
                        lsq += (double)sqf;
                        lms += (double)m;
                        bl0 += gS[sset][0];
                        bl1 += gS[sset][1];
                        bl2 += gS[sset][2];
                    }
                    s2_st12(o, yv[0], yv[1], yv[2]);
                    st_cur += 1;
                });
            }
            if (a.fwd_only) {  // render: the program holds the forward stages only
                S2T_END(6);
                continue;
            }
            s2_sfor<2>([&](auto sc) {
                constexpr int sset = decltype(sc)::value;
                // g operand of the last-layer dgrad: lane half 0, k = [g hi (3), 0, g lo (3), 0] as
                // fp16 hi + lo of 2^10 g (GS: an exact power of two that lifts the dgrad's dz out of
                // fp16's subnormal range; the dH partials and the weight gradients divide it out)
                S2Frag Bg;
                {
                    uint32_t wv[4] = {0u, 0u, 0u, 0u};
                    if (h == 0) {
                        u16 hi[3], lo[3];
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const float gs = gS[sset][c] * kGS;
                            hi[c] = f2h(gs);
                            lo[c] = f2h(gs - h2f(hi[c]));
                        }
                        wv[0] = hi[0] | ((uint32_t)hi[1] << 16);
                        wv[1] = hi[2];
                        wv[2] = lo[0] | ((uint32_t)lo[1] << 16);
                        wv[3] = lo[2];
                    }
                    Bg.u = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                }
                // last-layer weight gradient of the set's 32 pixels in fp16 (the operand the forward
                // used): A = (2^10 g)^T as fp16 hi (rows 0-2) + lo (rows 4-6) -- an exact power of two
                // that keeps |g| <= 0.5 in fp16's normal range -- B = feat^T through the LDS transpose
                {
                    constexpr float SC = kGS;
                    if (h == 0) {
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const float gs = gS[sset][c] * SC;
                            const u16 hi = f2h(gs);
                            gts[c * 32 + pxl] = hi;
                            gts[(4 + c) * 32 + pxl] = f2h(gs - h2f(hi));
                        }
                    }
                    // (a compiler barrier: the u16 stores and the f16x8 load below do not alias under
                    //  type-based alias analysis, and without it the second set reused the first set's
                    //  load of the image)
                    asm volatile("" ::: "memory");
                    const f16x8 ga = *reinterpret_cast<const f16x8*>(gts + (lane & 15) * 32 + 8 * (lane >> 4));
                    const int gq = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
                    const S2Frag* Bf = sset ? Bl : Bh;
#pragma unroll
                    for (int ks = 0; ks < NKH; ++ks) {
                        *reinterpret_cast<uint4*>(trs + (pxl * 2 + h) * 8) = Bf[ks].u;
                        asm volatile("" ::: "memory");
                        const u16* b0 = trs + (8 * gq + q) * 16 + (pp & 1) * 8 + 4 * (pp >> 1);
                        i16x4 vv[2] = {s2_tr16(b0), s2_tr16(b0 + 4 * 16)};
                        const f32x4 r4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ga, *reinterpret_cast<f16x8*>(vv), (f32x4){}, 0, 0, 0);
                        float lo[3];
#pragma unroll
                        for (int c = 0; c < 3; ++c) lo[c] = __shfl_down(r4[c], 16, 64);
                        if (lane < 16) {
#pragma unroll
                            for (int c = 0; c < 3; ++c) wla[c * HM + 16 * ks + lane] += (r4[c] + lo[c]) * (1.0f / SC);
                        }
                    }
                }
                SetSt cs;
                cs.g = Bg;
                cs.X0 = Xs[sset][0];
                cs.X1 = Xs[sset][1];
                cs.X2 = Xs[sset][2];
                cs.tile = real[sset] ? tl[sset] : -1;
                ss[sset] = cs;
            });
            S2T_END(6);
        } else {
        for (int si = 0; si < nset; ++si) {
            S2T_BEGIN(4);
            const int ti = it + si;
            const int tile = tbase + ti * (int)gridDim.x;
            const int pb = ti & 1;
            const int b = tile / tpp;
            const int p0 = (tile - b * tpp) * C::TPX + 32 * wave;
            const long long slot0 = (long long)b * a.geo.Np_pad + p0;
            const int p = p0 + pxl;
            const bool valid = p < Np;
            const float* pro = pro_buf(pb);
            uint32_t* mks = mkl + si * C::MSET;

            // ---- prologue: pixel grid -> warp (warp.py:33-81) -> posenc + c2f features (model/planar.py:451-471)
            float Hm[9];
#pragma unroll
            for (int e = 0; e < 9; ++e) Hm[e] = pro[4 * C::TPX + e];
            float x, y, u, v, X[3];
            if (a.geo.mode == 1) {  // explicit coordinates (GeoDev mode 1; render only)
                const int pc = min(p, Np - 1);
                u = x = a.geo.coords[2 * (size_t)pc];
                v = y = a.geo.coords[2 * (size_t)pc + 1];
                X[0] = u;
                X[1] = v;
                X[2] = 1.0f;
            } else {
                const int r = p / a.geo.w, cc = p - r * a.geo.w;
                x = grid_coord(a.geo.x0 + cc, a.geo.W, a.geo.norm_w);
                y = grid_coord(a.geo.y0 + r, a.geo.H, a.geo.norm_h);
                warp_point(Hm, x, y, u, v, X, a.geo.bmm_small);
            }
            const float cd = h ? v : u;
            S2Frag F0h[C::NK0], F0l[C::NK0];
            {
                const int ng = nk0 - 1;  // band groups of 4
#pragma unroll
                for (int g = 0; g < C::NK0 - 1; ++g) {
                    if (g < ng) {
                        float f[8];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int k = 4 * g + j;
                            float s = 0.f, co = 0.f;
                            if (k < L) {
                                band_sincos<true>(cd, k, s, co);
                                if (a.c2f_on) {
                                    const float w = c2f_l[k];
                                    s = s * w;
                                    co = co * w;
                                }
                            }
                            f[j] = s;
                            f[4 + j] = co;
                        }
                        s2_split8<SPLIT>(f, F0h[g], F0l[g]);
                    }
                }
                float f[8] = {cd, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                S2Frag rh, rl;
                s2_split8<SPLIT>(f, rh, rl);
#pragma unroll
                for (int g = 0; g < C::NK0; ++g)
                    if (g == ng) {
                        F0h[g] = rh;
                        F0l[g] = rl;
                    }
                // feat_0 (bf16 hi) for the layer-0 weight gradient: column 16 ks + 8 h + j
                // (every armed DMA piece was issued before the previous store: these count as the
                //  current stage's stores)
                if (!a.fwd_only && !a.feat0_recompute) {  // (T16: k-step g = feature block g)
                    u16* row = ly_ptr(0, 0) + (slot0 >> 5) * ly_int(0, 3) * 32 + pxl * 16 + 8 * h;
#pragma unroll
                    for (int g = 0; g < C::NK0; ++g)
                        if (g < nk0) s2_st16(row + 512 * g, F0h[g].u);
                    st_cur += nk0;
                    if (16 * nk0 < ly_int(0, 3)) {
                        s2_st16(row + 512 * nk0, make_uint4(0, 0, 0, 0));
                        st_cur += 1;
                    }
                }
            }

            S2T_END(4);
            S2T_BEGIN(5);
            // ---- forward, layer 0 then the hidden layers: one stage per 32-row output tile; the
            //      epilogue of tile rt-1 (ReLU, mask bits, bf16 split, stores) runs beside the MFMAs
            //      of tile rt, the last tile's epilogue right after its own MFMAs
            auto fwd_layer = [&](int l, const S2Frag* Bhi, const S2Frag* Blo, int nk, auto nk_tag, auto ms_tag) {
                constexpr int MS = decltype(ms_tag)::value;  // epilogue micro-steps beside each k-step
                typedef std::integral_constant<bool, decltype(nk_tag)::value == NKH> PcL;  // hidden: pieces in the GEMM
                constexpr bool SPLITPK = SPLIT && MS == 1 && decltype(nk_tag)::value == NKH;  // hidden, split recipe
                const int nrt = FIX ? NRT : ly_int(l, 0);
                const bool save = l + 1 < nl - 1 && !a.fwd_only;
                u16* srow = save ? ly_ptr(l + 1, 0) + (slot0 >> 5) * ly_int(l + 1, 3) * 32 + pxl * 16 + 8 * h : nullptr;
                const int boff = ly_int(l, 2);
                const char* slot0 = nullptr;
                s2_sfor<NRT>([&](auto rtc) {
                    constexpr int rt = decltype(rtc)::value;
                    f32x16& cur = (rt & 1) ? acc1 : acc0;
                    f32x16& prv = (rt & 1) ? acc0 : acc1;
                    if (rt < nrt) {
                        // layer 0: r0 row tiles share a stage (their few k-steps fill one slot)
                        const int sub = l == 0 ? rt % r0 : 0;
                        // the bias (a static LDS table) before the stage wait: its reads overlap it
                        S2T_BEGIN(15);
                        cur = bias_init(boff, rt);
                        S2T_END(15);
                        if (sub == 0) slot0 = stage_begin(l == 0);  // layer 0: the pieces in a burst
                        const char* slot = slot0 + sub * nk0 * 1024;
                        // the next tile's target / mask / H into the other input buffer (the tile that
                        // read it last finished before this stage's barrier)
                        if (l == 0 && rt == 0 && ti + 1 < my_tiles) issue_pro(tile + (int)gridDim.x, pb ^ 1);
                        if constexpr (rt == 0) {
                            S2T_BEGIN(8);
                            gemm(cur, slot, Bhi, Blo, nk, MFt(), nk_tag, nohook, PcL());
                            S2T_END(8);
                        } else {
                            ep.bits = 0;
                            S2T_BEGIN(8);
                            gemm(cur, slot, Bhi, Blo, nk, MFt(), nk_tag, [&](auto ksc, auto pc) {
                                constexpr int ks = decltype(ksc)::value, p = decltype(pc)::value;
                                if constexpr (SPLITPK) {
                                    // one step per k-step, the pack of pair (ks-1, ks) split over the
                                    // second gap of ks and the first gap of ks+1 (balanced gaps)
                                    if constexpr (p == 0) {
                                        if constexpr ((ks & 1) == 0 && ks >= 2) fpackB(std::integral_constant<int, ks - 1>());
                                        frelu(prv, ksc);
                                    } else if constexpr (ks & 1) {
                                        fpackA(ksc);
                                    }
                                } else {
                                    s2_sfor<MS>([&](auto jc) {
                                        constexpr int e = ks * MS + decltype(jc)::value;
                                        if constexpr (e < 16) {
                                            if constexpr (p == 0) frelu(prv, std::integral_constant<int, e>());
                                            else fpack(std::integral_constant<int, e>());
                                        }
                                    });
                                }
                            }, PcL());
                            S2T_END(8);
                            S2T_BEGIN(13);
                            if constexpr (SPLITPK) fpackB(std::integral_constant<int, 15>());
                            if constexpr (FIX && !SPLITPK) {  // (nk = NK0F: the count is compile-time)
                                constexpr int E0 = MS * decltype(nk_tag)::value;
                                if constexpr (E0 < 16) fsteps_free(prv, std::integral_constant<int, E0>());
                            } else {
                                s2_sfor<16>([&](auto ec) {  // steps not placed beside a live k-step
                                    if (decltype(ec)::value >= MS * nk) fstep(prv, ec);
                                });
                            }
                            S2T_END(13);
                            S2T_BEGIN(10);
                            ffinish(l, std::integral_constant<int, rt - 1>(), save, srow, mks, false);
                            S2T_END(10);
                        }
                        if (rt == nrt - 1) {
                            S2T_BEGIN(13);
                            ep.bits = 0;
                            if constexpr (FIX) fsteps_free(cur, std::integral_constant<int, 0>());
                            else s2_sfor<16>([&](auto ec) { fstep(cur, ec); });
                            ffinish(l, rtc, save, srow, mks, true);
                            S2T_END(13);
                        }
                    } else {
                        zero_out(Oh[2 * rt], Oh[2 * rt + 1], Ol[2 * rt], Ol[2 * rt + 1]);
                    }
                });
#pragma unroll
                for (int k = 0; k < NKH; ++k) {
                    Bh[k] = Oh[k];
                    if constexpr (SPLIT) Bl[k] = Ol[k];
                }
            };
            S2T_BEGIN(14);  // (phase stamps: layer 0 on its own)
            fwd_layer(0, F0h, F0l, nk0, NK0x(), std::integral_constant<int, 2>());
            S2T_END(14);
            for (int l = 1; l < nl - 1; ++l) fwd_layer(l, Bh, Bl, NKH, NKHt(), std::integral_constant<int, 1>());

            S2T_END(5);
            S2T_BEGIN(6);
            // ---- last layer: 3 outputs (rows 0..2 of one tile), sigmoid, masked MSE, d rgb
            float g[3] = {0.f, 0.f, 0.f};
            {
                f32x16 acc = bias_init(ly_int(nl - 1, 2), 0);
                const char* slot = stage_begin(false);
                gemm(acc, slot, Bh, Bl, NKH, MFt(), NKHt(), nohook, PcOn());
                float* o = (a.rgb && valid && h == 0) ? a.rgb + ((size_t)b * Np + p) * 3 : dmy;
                float yv[3] = {0.f, 0.f, 0.f};
                if (h == 0) {
                    const float m = valid ? (a.mask ? pro[3 * C::TPX + 32 * wave + pxl] : 1.0f) : 0.f;
                    double sq = 0.0;
                    float sqf = 0.f;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const float z = acc[c];
                        const float yy = 1.0f / (1.0f + expf(-z));
                        yv[c] = yy;
                        const float t = valid ? pro[c * C::TPX + 32 * wave + pxl] : 0.f;
                        // model/planar.py:388-390 and its autograd: x = (p - g) m, d = 2 x m
                        const float xx = (yy - t) * m;
                        sqf += xx * xx;
                        const float d = (2.0f * xx) * m;
                        g[c] = (d * (1.0f - yy)) * yy;  // sigmoid backward
                    }
                    sq = (double)sqf;
                    lsq += sq;
                    lms += (double)m;
                    bl0 += g[0];
                    bl1 += g[1];
                    bl2 += g[2];
                }
                s2_st12(o, yv[0], yv[1], yv[2]);
                st_cur += 1;
            }
            if (a.fwd_only) {  // render: the program holds the forward stages only
                S2T_END(6);
                continue;
            }
            // g operand of the last-layer dgrad: lane half 0, k = [g hi (3), 0, g lo (3), 0]
            S2Frag Bg;
            {
                float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                if (h == 0) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        f[c] = g[c];                                        // bf16(g) below
                        f[4 + c] = g[c] - s2_lo16(s2_pk(g[c], 0.f));         // g - bf16(g)
                    }
                }
                S2Frag dumm;
                s2_split8<false>(f, Bg, dumm);
            }
            // ---- last-layer weight gradient of the wave's 32 pixels: dW[c][k] += sum_px g[c] feat[k]
            //      16x16x32 MFMA: A = g^T (rows 0-2 hi, 4-6 lo; K = 32 pixels) from a wave-private
            //      LDS image, B = feat^T per 16-feature k-step through a transposing LDS round trip
            {
                if (h == 0) {
                    const uint32_t w0 = Bg.u.x, w1 = Bg.u.y, w2 = Bg.u.z, w3 = Bg.u.w;
                    gts[0 * 32 + pxl] = (u16)(w0 & 0xffff);
                    gts[1 * 32 + pxl] = (u16)(w0 >> 16);
                    gts[2 * 32 + pxl] = (u16)(w1 & 0xffff);
                    gts[4 * 32 + pxl] = (u16)(w2 & 0xffff);
                    gts[5 * 32 + pxl] = (u16)(w2 >> 16);
                    gts[6 * 32 + pxl] = (u16)(w3 & 0xffff);
                }
                const bf16x8 ga = *reinterpret_cast<const bf16x8*>(gts + (lane & 15) * 32 + 8 * (lane >> 4));
                const int gq = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
                const int nkl = FIX ? NKH : a.Kl / 16;
                const int Klw = FIX ? HM : a.Kl;
#pragma unroll
                for (int ks = 0; ks < NKH; ++ks) {
                    if (ks < nkl) {
                        *reinterpret_cast<uint4*>(trs + (pxl * 2 + h) * 8) = Bh[ks].u;
                        const u16* b0 = trs + (8 * gq + q) * 16 + (pp & 1) * 8 + 4 * (pp >> 1);
                        i16x4 vv[2] = {s2_tr16(b0), s2_tr16(b0 + 4 * 16)};
                        const f32x4 r4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, *reinterpret_cast<bf16x8*>(vv), (f32x4){}, 0, 0, 0);
                        float lo[3];
#pragma unroll
                        for (int c = 0; c < 3; ++c) lo[c] = __shfl_down(r4[c], 16, 64);
                        if (lane < 16) {
#pragma unroll
                            for (int c = 0; c < 3; ++c) wla[c * Klw + 16 * ks + lane] += r4[c] + lo[c];
                        }
                    }
                }
            }
            {
                SetSt cs;
                cs.g = Bg;
                cs.X0 = X[0];
                cs.X1 = X[1];
                cs.X2 = X[2];
                cs.tile = tile;
                if (si == 0) ss[0] = cs;
                else ss[NS - 1] = cs;
            }
            S2T_END(6);
        }
        }  // (the split recipe's forward, one tile at a time)
        if (a.fwd_only) continue;
        if (nset < NS) {  // no tile for the last set: its dgrad runs on zeros into the store sink rows
            SetSt cs;
            cs.g.u = make_uint4(0, 0, 0, 0);
            cs.X0 = cs.X1 = 0.f;
            cs.X2 = 1.f;
            cs.tile = -1;
            ss[NS - 1] = cs;
        }

        S2T_BEGIN(2);
        // ---- the dgrad pass of the group's NS pixel sets: every weight stage is read once for all
        //      of them, one GEMM pass per set.  Items i = NS rt + s in order; the epilogue of item
        //      i-1 (mask, bf16 pack, stores) runs beside the MFMAs of item i, so one accumulator per
        //      parity of i suffices.  Per set the MFMA sequence, epilogue and stores are those of a
        //      single tile.
        long long sl0[NS];  // the sets' first pixel slot of the wave (wave-uniform)
        s2_sfor<NS>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const int tl = ss[s].tile;
            long long v;
            if (tl < 0) {
                v = a.S + 32 * wave;
            } else {
                const int bb = tl / tpp;
                v = (long long)bb * a.geo.Np_pad + (tl - bb * tpp) * C::TPX + 32 * wave;
            }
            sl0[s] = v;
        });
        // operand / output fragments of set s: the forward's arrays (the dgrad needs hi only, so the
        // lo arrays carry the second set; reusing them keeps no extra array live across the pass)
        S2Frag* const Dh[2] = {Bh, Bl};
        S2Frag* const Do[2] = {Oh, Ol};
        EpSt eb;
        auto mks_b = [&](int s) -> const uint32_t* { return mkl + s * C::MSET; };
        // ---- last-layer dgrad: dfeat_{n-1} = W_{n-1}^T g, mask -> dz_{n-1}; one stage holds every
        //      row tile's single k-step (tile rt at rt KB)
        {
            const int lmask = nl - 2;
            const int nrt = FIX ? NRT : ly_int(nl - 1, 1);
            u16* brow[NS];
            s2_sfor<NS>([&](auto sc) {
                brow[decltype(sc)::value] = ly_ptr(nl - 1, 1) + (sl0[decltype(sc)::value] >> 5) * ly_int(nl - 1, 4) * 32 + pxl * 16 + 8 * h;
            });
            S2Frag gB[NS];
            s2_sfor<NS>([&](auto sc) { gB[decltype(sc)::value] = ss[decltype(sc)::value].g; });
            const char* slot = stage_begin(true);  // single-k-step GEMMs: the pieces in a burst
            if constexpr (HF) {
                if (it + NS < my_tiles) {  // the next group's targets (this group's last layer read its own)
                    issue_tgt(it + NS);
                    st_cur += 4;
                }
            }
            s2_sfor<NRT>([&](auto rtc) {
                constexpr int rt = decltype(rtc)::value;
                if (rt < nrt) {
                    s2_sfor<NS>([&](auto sc) {
                        constexpr int s = decltype(sc)::value, i = rt * NS + s;
                        constexpr int sp = (i + NS - 1) % NS, rp = (i - 1 + NS) / NS - 1;  // item i-1
                        f32x16& cur = (i & 1) ? acc1 : acc0;
                        f32x16& prv = (i & 1) ? acc0 : acc1;
                        cur = (f32x16){};
                        if constexpr (i == 0) {
                            gemm(cur, slot, &gB[s], &gB[s], 1, MBt(), NK1t(), nohook, PcOff());
                        } else {
                            eb.mw = mks_b(sp)[(lmask * C::NMW + (rp >> 1)) * 64 + lane];
                            if constexpr (FIX) {  // (2 MFMAs: no gaps worth filling)
                                gemm(cur, slot + rt * 1024, &gB[s], &gB[s], 1, MBt(), NK1t(), nohook, PcOff());
                                bsteps_free(eb, prv, std::integral_constant<int, rp>());
                            } else {
                                gemm(cur, slot + rt * 1024, &gB[s], &gB[s], 1, MBt(), NK1t(), [&](auto, auto pc) {
                                    s2_sfor<8>([&](auto ec) {
                                        bstep(eb, prv, std::integral_constant<int, 8 * decltype(pc)::value + decltype(ec)::value>(),
                                              std::integral_constant<int, rp>());
                                    });
                                }, PcOff());
                            }
                            S2T_BEGIN(11);
                            bfinish(eb, Do[sp], std::integral_constant<int, rp>(), brow[sp]);
                            S2T_END(11);
                        }
                        if (s == NS - 1 && rt == nrt - 1) {
                            eb.mw = mks_b(s)[(lmask * C::NMW + (rt >> 1)) * 64 + lane];
                            if constexpr (FIX) bsteps_free(eb, cur, rtc);
                            else s2_sfor<16>([&](auto ec) { bstep(eb, cur, ec, rtc); });
                            bfinish(eb, Do[s], rtc, brow[s]);
                        }
                    });
                } else {
                    s2_sfor<NS>([&](auto sc) {
                        constexpr int s = decltype(sc)::value;
                        Do[s][2 * rt].u = Do[s][2 * rt + 1].u = make_uint4(0, 0, 0, 0);
                    });
                    if constexpr (SDZ) Ol[2 * rt].u = Ol[2 * rt + 1].u = make_uint4(0, 0, 0, 0);
                }
            });
#pragma unroll
            for (int k = 0; k < NKH; ++k) {
                s2_sfor<NS>([&](auto sc) { Dh[decltype(sc)::value][k] = Do[decltype(sc)::value][k]; });
                if constexpr (SDZ) Bl[k] = Ol[k];
            }
        }
        // ---- hidden dgrad chain l = nl-2 .. 1
        for (int l = nl - 2; l >= 1; --l) {
            const int lmask = l - 1;
            const int nrt = FIX ? NRT : ly_int(l, 1);
            u16* brow[NS];
            s2_sfor<NS>([&](auto sc) {
                brow[decltype(sc)::value] = ly_ptr(l, 1) + (sl0[decltype(sc)::value] >> 5) * ly_int(l, 4) * 32 + pxl * 16 + 8 * h;
            });
            if constexpr (J2) {
                // both sets in ONE pass per stage (gemm2, bf16): each A fragment read from LDS once for
                // the two sets; per set the MFMA sequence, epilogue and stores of the per-set passes
                // below, so the same bits.  The epilogue of row tile rt-1 of both sets (set 0 in
                // k-steps 0-7, set 1 in 8-15) runs in the gaps of row tile rt.
                EpSt ebs[2];
                s2_sfor<NRT>([&](auto rtc) {
                    constexpr int rt = decltype(rtc)::value;
                    f32x16& c0 = hacc[(rt & 1) ? 2 : 0];
                    f32x16& c1 = hacc[(rt & 1) ? 3 : 1];
                    f32x16& q0 = hacc[(rt & 1) ? 0 : 2];
                    f32x16& q1 = hacc[(rt & 1) ? 1 : 3];
                    const char* slot = stage_begin(false);
                    c0 = (f32x16){};
                    c1 = (f32x16){};
                    if constexpr (rt == 0) {
                        S2T_BEGIN(9);
                        gemm2(c0, c1, slot, Dh[0], Dh[1], NKHt(), nohook, PcOn(), std::integral_constant<bool, HF>());
                        S2T_END(9);
                    } else {
                        typedef std::integral_constant<int, rt - 1> RP;
                        ebs[0].mw = mks_b(0)[(lmask * C::NMW + ((rt - 1) >> 1)) * 64 + lane];
                        ebs[1].mw = mks_b(1)[(lmask * C::NMW + ((rt - 1) >> 1)) * 64 + lane];
                        S2T_BEGIN(9);
                        gemm2(c0, c1, slot, Dh[0], Dh[1], NKHt(), [&](auto ksc, auto pc) {
                            constexpr int ks = decltype(ksc)::value, p = decltype(pc)::value;
                            if constexpr (p < 2) {
                                constexpr int sset = ks >> 3;
                                bstep(ebs[sset], sset ? q1 : q0, std::integral_constant<int, 2 * (ks & 7) + p>(), RP());
                            }
                        }, PcOn(), std::integral_constant<bool, HF>());
                        S2T_END(9);
                        S2T_BEGIN(11);
                        bfinish(ebs[0], Do[0], RP(), brow[0]);
                        bfinish(ebs[1], Do[1], RP(), brow[1]);
                        S2T_END(11);
                    }
                    if constexpr (rt == NRT - 1) {
                        ebs[0].mw = mks_b(0)[(lmask * C::NMW + (rt >> 1)) * 64 + lane];
                        ebs[1].mw = mks_b(1)[(lmask * C::NMW + (rt >> 1)) * 64 + lane];
                        bsteps_free(ebs[0], c0, rtc);
                        bsteps_free(ebs[1], c1, rtc);
                        bfinish(ebs[0], Do[0], rtc, brow[0]);
                        bfinish(ebs[1], Do[1], rtc, brow[1]);
                    }
                });
            } else
            s2_sfor<NRT>([&](auto rtc) {
                constexpr int rt = decltype(rtc)::value;
                if (rt < nrt) {
                    const char* slot = stage_begin(false);
                    s2_sfor<NS>([&](auto sc) {
                        constexpr int s = decltype(sc)::value, i = rt * NS + s;
                        constexpr int sp = (i + NS - 1) % NS, rp = (i - 1 + NS) / NS - 1;
                        f32x16& cur = (i & 1) ? acc1 : acc0;
                        f32x16& prv = (i & 1) ? acc0 : acc1;
                        cur = (f32x16){};
                        if constexpr (i == 0) {
                            S2T_BEGIN(9);
                            gemm(cur, slot, Dh[s], SDZ ? Bl : Dh[s], NKH, MDt(), NKHt(), nohook, std::integral_constant<bool, s == 0>());
                            S2T_END(9);
                        } else {
                            eb.mw = mks_b(sp)[(lmask * C::NMW + (rp >> 1)) * 64 + lane];
                            S2T_BEGIN(9);
                            gemm(cur, slot, Dh[s], SDZ ? Bl : Dh[s], NKH, MDt(), NKHt(), [&](auto ksc, auto pc) {
                                if constexpr (decltype(pc)::value == 0) bstep(eb, prv, ksc, std::integral_constant<int, rp>());
                            }, std::integral_constant<bool, s == 0>());
                            S2T_END(9);
                            S2T_BEGIN(11);
                            bfinish(eb, Do[sp], std::integral_constant<int, rp>(), brow[sp]);
                            S2T_END(11);
                        }
                        if (s == NS - 1 && rt == nrt - 1) {
                            eb.mw = mks_b(s)[(lmask * C::NMW + (rt >> 1)) * 64 + lane];
                            if constexpr (FIX) bsteps_free(eb, cur, rtc);
                            else s2_sfor<16>([&](auto ec) { bstep(eb, cur, ec, rtc); });
                            bfinish(eb, Do[s], rtc, brow[s]);
                        }
                    });
                } else {
                    s2_sfor<NS>([&](auto sc) {
                        constexpr int s = decltype(sc)::value;
                        Do[s][2 * rt].u = Do[s][2 * rt + 1].u = make_uint4(0, 0, 0, 0);
                    });
                    if constexpr (SDZ) Ol[2 * rt].u = Ol[2 * rt + 1].u = make_uint4(0, 0, 0, 0);
                }
            });
#pragma unroll
            for (int k = 0; k < NKH; ++k) {
                s2_sfor<NS>([&](auto sc) { Dh[decltype(sc)::value][k] = Do[decltype(sc)::value][k]; });
                if constexpr (SDZ) Bl[k] = Ol[k];
            }
        }
        // ---- layer-0 dgrad + posenc adjoint: row (tile t, register r) = slot 16 t + r of the
        //      lane's coordinate: slot 2k = sin band k, 2k + 1 = cos band k, 2L = the raw coordinate.
        //      The adjoint of item i-1 (8 bands) runs beside the MFMAs of item i.
        float dc[NS], cds[NS];
        s2_sfor<NS>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            dc[s] = 0.f;
            const float dd = ss[s].X2 + 1e-8f;  // warp_point's (u, v), bit for bit
            cds[s] = h ? ss[s].X1 / dd : ss[s].X0 / dd;
        });
        {
            const int nta = FIX ? NTAF : a.nta;
            auto adj_band = [&](float& d, const float cd, const f32x16& pa, int t, auto ic) {
                constexpr int i = decltype(ic)::value;
                const int k = 8 * t + i;
                if (k < L) {
                    float sn, co;
                    band_sincos<true>(cd, k, sn, co);
                    float gs = pa[2 * i], gc = pa[2 * i + 1];
                    if (a.c2f_on) {
                        const float w = c2f_l[k];
                        gs = gs * w;
                        gc = gc * w;
                    }
                    d += (gs * co - gc * sn) * ldexpf(pi_f, k);
                }
            };
            auto adj_raw = [&](float& d, const f32x16& pa, int t) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (16 * t + r == 2 * L) d += pa[r];
            };
            s2_sfor<C::NTA>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                if (t < nta) {
                    const char* slot = stage_begin(false);
                    s2_sfor<NS>([&](auto sc) {
                        constexpr int s = decltype(sc)::value, i = t * NS + s;
                        constexpr int sp = (i + NS - 1) % NS, tp = (i - 1 + NS) / NS - 1;
                        f32x16& cur = (i & 1) ? acc1 : acc0;
                        f32x16& prv = (i & 1) ? acc0 : acc1;
                        cur = (f32x16){};
                        if constexpr (i == 0) {
                            S2T_BEGIN(9);
                            gemm(cur, slot, Dh[s], Dh[s], NKH, MBt(), NKHt(), nohook, std::integral_constant<bool, s == 0>());
                            S2T_END(9);
                        } else {
                            S2T_BEGIN(9);
                            gemm(cur, slot, Dh[s], Dh[s], NKH, MBt(), NKHt(), [&](auto ksc, auto pc) {
                                constexpr int ks = decltype(ksc)::value;
                                if constexpr ((ks & 1) == 0 && decltype(pc)::value == 0)
                                    adj_band(dc[sp], cds[sp], prv, tp, std::integral_constant<int, ks / 2>());
                            }, std::integral_constant<bool, s == 0>());
                            S2T_END(9);
                            adj_raw(dc[sp], prv, tp);
                        }
                        if (s == NS - 1 && t == nta - 1) {
                            s2_sfor<8>([&](auto ic) { adj_band(dc[s], cds[s], cur, t, ic); });
                            adj_raw(dc[s], cur, t);
                        }
                    });
                }
            });
        }
        S2T_END(2);
        if constexpr (HF) {  // (the fp16x2 dgrad carries 2^10 g: exact)
            s2_sfor<NS>([&](auto sc) { dc[decltype(sc)::value] *= 1.0f / kGS; });
        }
        S2T_BEGIN(3);
        // (u, v) = X[:2] / (X[2] + 1e-8) backward, then the bmm backward -> dH partial of the wave
        {
            float mine[NS];
            float* dst[NS];
            s2_sfor<NS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                const SetSt& cs = ss[s];
                const float dother = __shfl_xor(dc[s], 32, 64);
                const float du = h ? dother : dc[s], dv = h ? dc[s] : dother;
                // the set's grid point (as the prologue computed it) and validity
                bool valid = false;
                float x = 0.f, y = 0.f;
                if (cs.tile >= 0) {
                    const int bb = cs.tile / tpp;
                    const int p = (cs.tile - bb * tpp) * C::TPX + 32 * wave + pxl;
                    valid = p < Np;
                    const int r = p / a.geo.w, cc = p - r * a.geo.w;
                    x = grid_coord(a.geo.x0 + cc, a.geo.W, a.geo.norm_w);
                    y = grid_coord(a.geo.y0 + r, a.geo.H, a.geo.norm_h);
                }
                float h9[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) h9[e] = 0.f;
                if (h == 0 && valid) {
                    const float dd = cs.X2 + 1e-8f;
                    const float dX0 = du / dd, dX1 = dv / dd;
                    const float dd2 = dd * dd;
                    const float dX2 = (-du * cs.X0) / dd2 + (-dv * cs.X1) / dd2;
                    const float hom[3] = {x, y, 1.f};
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) {
                        h9[0 + cc] = dX0 * hom[cc];
                        h9[3 + cc] = dX1 * hom[cc];
                        h9[6 + cc] = dX2 * hom[cc];
                    }
                }
                mine[s] = 0.f;
#pragma unroll
                for (int e = 0; e < 9; ++e) {
                    const float sm = wave_total63(h9[e]);
                    const float sb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm), 63));
                    if (lane == e) mine[s] = sb;
                }
                dst[s] = lane < 9 ? a.dH_partial + (size_t)(sl0[s] / 32) * 9 + lane : dmy;
            });
            s2_sfor<NS>([&](auto sc) { s2_st4(dst[decltype(sc)::value], mine[decltype(sc)::value]); });
            st_cur += NS;
        }
        S2T_END(3);
    }
    S2T_END(7);
#ifdef MARF_STAMPS
    if (a.stamps && threadIdx.x == 0)
        for (int k = 0; k < 16; ++k) a.stamps[(size_t)blockIdx.x * 16 + k] = tacc[k];
#endif

    // ---- per-block partials (fixed order over waves)
    s2_wait_vm<0>();
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
        for (int w = 0; w < NW; ++w)
            s += reinterpret_cast<const float*>(smem + a.lds_wave + w * a.lds_wave_bytes + 2048 + NS * C::MSET * 4)[e];
        a.wlast_partial[(size_t)blockIdx.x * 3 * a.Kl + e] = s;
    }
}

// ------------------------------------------------------------------ weight program packing

// true input feature of layer-0 forward k index (16 ks + 8 h + j) in the band-group layout; -1: zero
MARF_DEV int s2_l0_fwd_feature(int ks, int hh, int j, int L, int nk0) {
    const int ng = nk0 - 1;
    if (ks == ng) return j == 0 ? hh : -1;  // raw coordinate
    const int k = 4 * ks + (j & 3);
    if (k >= L) return -1;
    const bool cosp = j >= 4;
    return 2 + 2 * hh * L + (cosp ? L : 0) + k;
}
// true input feature of adjoint row rho of tile t (slot 16 t + r of coordinate hh); -1: none
MARF_DEV int s2_l0_adj_feature(int t, int rho, int L) {
    const int hh = (rho >> 2) & 1, r = (rho & 3) + 4 * (rho >> 3);
    const int sl = 16 * t + r;
    if (sl == 2 * L) return hh;
    if (sl >= 2 * L) return -1;
    const int k = sl >> 1;
    return 2 + 2 * hh * L + ((sl & 1) ? L : 0) + k;
}

template <int HM, bool SPLIT, int NW, int MAXR, int NK0F = 0, int NTAF = 0>
__global__ __launch_bounds__(NW * 64, NW / 4) void k_step2(Step2Args a) {
    k_step2_body<HM, SPLIT, NW, MAXR, NK0F, NTAF, false>(a);
}

// the split recipe with dz split in the dgrad too (opt-in: MARF_STEP2_DZ=1)
template <int HM, bool SPLIT, int NW, int MAXR, int NK0F = 0, int NTAF = 0>
__global__ __launch_bounds__(NW * 64, NW / 4) void k_step2dz(Step2Args a) {
    k_step2_body<HM, SPLIT, NW, MAXR, NK0F, NTAF, true>(a);
}

// the fp16x2 recipe (MARF_FP16X2): split-fp16 weights, fp16 forward and dgrad of two pixel sets per stage
template <int HM, int NW, int MAXR, int NK0F, int NTAF>
__global__ __launch_bounds__(NW * 64, NW / 4) void k_step2h(Step2Args a) {
    k_step2_body<HM, true, NW, MAXR, NK0F, NTAF, false, true>(a);
}

// permuted k (hidden operand from an accumulator): k-step ks, lane half hh, element j
MARF_DEV int s2_kperm(int ks, int hh, int j) { return 16 * ks + 8 * (j >> 2) + 4 * hh + (j & 3); }

// One thread per (stage, part, k-step, lane, element): the packed bf16 value.  Stage sequence per
// pixel tile (the kernel's consumption order): layer-0 forward row tiles, hidden forward row tiles,
// the last layer, last-layer dgrad row tiles, hidden dgrad row tiles (l = nl-2 .. 1), adjoint tiles.
__global__ void k_pack2(const float* __restrict__ params, u16* __restrict__ prog, float* __restrict__ bias_out,
                        int* __restrict__ kmap, Pack2Args a) {
    const int per_slot = a.slot_bytes / 2;
    const long long total = (long long)a.n_stages * per_slot;
    const int D = a.dims[0];
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total + a.nbias + D; e += (long long)gridDim.x * 256) {
        if (e >= total + a.nbias) {
            // layer-0 column map: true input feature f -> column of feat_0 (16 ks + 8 h + j)
            const int f = (int)(e - total - a.nbias), L = a.L, ng = a.nk0 - 1;
            int col;
            if (f < 2) col = 16 * ng + 8 * f;
            else {
                const int q = f - 2, hh = q / (2 * L), rr = q - hh * 2 * L, cosp = rr >= L, k = rr - cosp * L;
                col = 16 * (k / 4) + 8 * hh + 4 * cosp + (k % 4);
            }
            kmap[f] = col;
            continue;
        }
        if (e >= total) {
            // padded bias table
            const int be = (int)(e - total);
            float v = 0.f;
            for (int l = 0; l < a.nl; ++l) {
                const int nb = (l == a.nl - 1) ? 32 : a.Mp[l];
                if (be >= a.boff[l] && be < a.boff[l] + nb) {
                    const int m = be - a.boff[l];
                    if (m < a.dims[l + 1]) v = params[a.b_off[l] + m];
                }
            }
            bias_out[be] = v;
            continue;
        }
        int st = (int)(e / per_slot);
        const int w = (int)(e - (long long)st * per_slot);
        const int part = w / (a.NKH * 512);  // 0 hi, 1 lo
        const int w2 = w - part * a.NKH * 512;
        const int ks = w2 / 512, lane = (w2 >> 3) & 63, j = w2 & 7;
        const int r32 = lane & 31, hh = lane >> 5;
        float val = 0.f;
        bool have = false;
        // decode the stage
        int layer = -1, kind = -1, rt = 0;  // kind 0 fwd, 1 last fwd, 2 last dgrad, 3 hidden dgrad, 4 adjoint
        {
            int s = st;
            if (s < a.ns0) { layer = 0; kind = 0; rt = s; }  // rt = the layer-0 stage here
            else {
                s -= a.ns0;
                for (int l = 1; l < a.nl - 1 && kind < 0; ++l) {
                    if (s < a.nrt[l]) { layer = l; kind = 0; rt = s; }
                    else s -= a.nrt[l];
                }
                if (kind < 0) {
                    if (s == 0) { layer = a.nl - 1; kind = 1; rt = 0; }
                    else {
                        s -= 1;
                        if (s == 0) { layer = a.nl - 1; kind = 2; rt = 0; }  // one stage, tile rt at rt KB
                        else {
                            s -= 1;
                            for (int l = a.nl - 2; l >= 1 && kind < 0; --l) {
                                if (s < a.nrtb[l]) { layer = l; kind = 3; rt = s; }
                                else s -= a.nrtb[l];
                            }
                            if (kind < 0 && s < a.nta) { layer = 0; kind = 4; rt = s; }
                        }
                    }
                }
            }
        }
        if (kind >= 0) {
            const int Mt = a.dims[layer + 1], Kt = a.dims[layer];
            const float* W = params + a.w_off[layer];
            int m = -1, k = -1;  // W[m][k]
            if (kind == 0 && layer == 0) {
                // a layer-0 stage holds r0 row tiles: tile rt r0 + r at fragment slots r nk0 ..
                const int r = ks / a.nk0, kk = ks - r * a.nk0, rtt = rt * a.r0 + r;
                if (r < a.r0 && rtt < a.nrt[0]) {
                    m = 32 * rtt + r32;
                    k = s2_l0_fwd_feature(kk, hh, j, a.L, a.nk0);
                }
            } else if (kind == 0 || kind == 1) {
                m = 32 * rt + r32;
                k = s2_kperm(ks, hh, j);
            } else if (kind == 2) {
                // rows = input features of the last layer (natural), k = [g hi (3), 0, g lo (3), 0];
                // fragment slot ks of the stage holds row tile ks
                if (ks < a.nrtb[layer] && hh == 0 && (j & 3) < 3) {
                    m = j & 3;
                    k = 32 * ks + r32;
                }
            } else if (kind == 3) {
                m = s2_kperm(ks, hh, j);
                k = 32 * rt + r32;
            } else {  // adjoint rows
                m = s2_kperm(ks, hh, j);
                k = s2_l0_adj_feature(rt, r32, a.L);
            }
            if (m >= 0 && k >= 0 && m < Mt && k < Kt) {
                val = W[(size_t)m * Kt + k];
                have = true;
            }
        }
        u16 out = 0;
        if (have) {
            if (a.fwd_f16) {  // the fp16x2 recipe: every stage fp16 hi + lo
                const u16 hi = f2h(val);
                out = part == 0 ? hi : f2h(val - h2f(hi));
            } else {
                const u16 hi = f2bf(val);
                out = part == 0 ? hi : (a.split ? f2bf(val - bf2f(hi)) : (u16)0);
            }
        }
        prog[e] = out;
    }
}

}  // namespace marf

using namespace marf;

template <int HM, bool SPLIT, int NW, int MAXR, int NK0F = 0, int NTAF = 0, bool DZ = false, bool HF = false>
static hipError_t launch_step2_t(const Step2Args& a, int grid, hipStream_t s) {
    const void* k;
    if constexpr (HF) k = (const void*)k_step2h<HM, NW, MAXR, NK0F, NTAF>;
    else if constexpr (DZ) k = (const void*)k_step2dz<HM, SPLIT, NW, MAXR, NK0F, NTAF>;
    else k = (const void*)k_step2<HM, SPLIT, NW, MAXR, NK0F, NTAF>;
    hipError_t e = ensure_dynamic_lds(k, (size_t)a.lds_total);
    if (e != hipSuccess) return e;
    if constexpr (HF)
        hipLaunchKernelGGL((k_step2h<HM, NW, MAXR, NK0F, NTAF>), dim3(grid), dim3(NW * 64), (size_t)a.lds_total, s, a);
    else if constexpr (DZ)
        hipLaunchKernelGGL((k_step2dz<HM, SPLIT, NW, MAXR, NK0F, NTAF>), dim3(grid), dim3(NW * 64), (size_t)a.lds_total, s, a);
    else
        hipLaunchKernelGGL((k_step2<HM, SPLIT, NW, MAXR, NK0F, NTAF>), dim3(grid), dim3(NW * 64), (size_t)a.lds_total, s, a);
    return hipGetLastError();
}

// variant: 0 = plain bf16, 256-wide, 8 waves; 1 = split bf16, 256-wide, 4 waves; 2 = plain bf16,
// 256-wide, 4 waves (diagnostic: the variant-0 arithmetic at one wave per SIMD); 3 = fp16x2 (the fp16
// forward of two pixel sets per stage + the split dgrad), 256-wide, 4 waves
// full_nk0: a full-width net's layer-0 k-step count (its r0 and row-tile counts follow from it; see
// k_step2's NK0F), or 0 for the generic instantiation; the compile-time instantiations cover
// (nk0, nta) = (5, 3): L = 16; (5, 2): L = 13..15; (4, 2): L = 9..12; (3, 2): L = 8
// dz: the split recipe with the dgrad's dz split too (k_step2's DZ; L = 8 and 16 instantiated)
hipError_t marf_launch_step2(const Step2Args& a, int variant, int grid, hipStream_t s, int full_nk0, bool dz) {
    if (variant == 3) {  // fp16x2: the compile-time layer-0 instantiations only
        if (full_nk0 == 5 && a.nta == 3) return launch_step2_t<256, true, 4, 4, 5, 3, false, true>(a, grid, s);
        if (full_nk0 == 5 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 5, 2, false, true>(a, grid, s);
        if (full_nk0 == 4 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 4, 2, false, true>(a, grid, s);
        if (full_nk0 == 3 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 3, 2, false, true>(a, grid, s);
        return hipErrorInvalidValue;
    }
    if (variant == 1 && dz) {
        if (full_nk0 == 5 && a.nta == 3) return launch_step2_t<256, true, 4, 4, 5, 3, true>(a, grid, s);
        if (full_nk0 == 3 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 3, 2, true>(a, grid, s);
        return launch_step2_t<256, true, 4, 4, 0, 0, true>(a, grid, s);
    }
    switch (variant) {
        case 0: return launch_step2_t<256, false, 8, 4>(a, grid, s);
        case 1:
            if (full_nk0 == 5 && a.nta == 3) return launch_step2_t<256, true, 4, 4, 5, 3>(a, grid, s);
            if (full_nk0 == 5 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 5, 2>(a, grid, s);
            if (full_nk0 == 4 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 4, 2>(a, grid, s);
            if (full_nk0 == 3 && a.nta == 2) return launch_step2_t<256, true, 4, 4, 3, 2>(a, grid, s);
            return launch_step2_t<256, true, 4, 4>(a, grid, s);
        case 2: return launch_step2_t<256, false, 4, 4>(a, grid, s);  // diagnostic: bf16 on 4 waves
        default: return hipErrorInvalidValue;
    }
}

hipError_t marf_launch_pack2(const float* params, void* prog, float* bias_out, int* kmap, const Pack2Args& a,
                             hipStream_t s) {
    const long long total = (long long)a.n_stages * (a.slot_bytes / 2) + a.nbias + a.dims[0];
    long long blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_pack2, dim3((unsigned)blocks), dim3(256), 0, s, params, (u16*)prog, bias_out, kmap, a);
    return hipGetLastError();
}
