// marf_common.h -- shared device-side definitions for the MI355X (gfx950) planar BA kernels.
//
// Layout conventions (see DESIGN.md "Data layout in HBM"):
//   * pixel slots s = b * Np_pad + p  (patch b, pixel p row-major in the crop, Np_pad = Np rounded
//     up to MARF_TILE_PAD); slots with p >= Np are padding (never written to user outputs, zero
//     gradient).
//   * saved activations  feat_l : [S][Kp_l]  (storage type T, pixel-major rows)
//   * relu masks         mask_l : uint64 [S/32][Kp_l/32][16]: for pixel tile p (32 slots), row tile t and
//                        accumulator register r, bit `lane` = (feature 32t + acc_row(lane, r) of
//                        slot 32p + (lane & 31)) > 0 -- the wave ballot of that register.
//   * packed weights     Wf_l   : W_l [Mp_l][Kp_l] (forward A operand, zero padded) and
//                        Wt_l   : W_l^T [Kp_l][Mt_l] (backward A operand), both FRAGMENT-MAJOR: for
//                        row tile rt and k-step ks the 64 lanes' MFMA A fragments are one
//                        contiguous 64 * FE-element block at ((rt * nk + ks) * 64 + lane) * FE,
//                        so a wave's weight load is one fully used 1 KB (bf16) burst.  Lane l of
//                        a 32x32 fragment holds row 32 rt + (l & 31), k = ks KS + (l >> 5) FE + j;
//                        the 16-row last layer (16x16 MFMA) row l & 15, k = ks KS16 + (l >> 4) FE + j.
//   * MFMA 32x32 accumulator map (both dtypes): lane l, reg r -> col = l&31,
//     row = (r&3) + 8*(r>>2) + 4*(l>>5).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MARF_TILE_PAD 128  // pixel-count granularity of every per-patch slot range

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

#define MARF_DEV __device__ __forceinline__

// Phase timestamps (diagnostic builds only, -DMARF_STAMPS; tools/phase_stamps.py): wave 0 of a
// block writes s_memtime into slot i of its row sp (32 slots per block).
#ifdef MARF_STAMPS
#define MARF_STAMP(sp, i)                                                           \
    do {                                                                            \
        if ((sp) && threadIdx.x == 0) (sp)[i] = __builtin_amdgcn_s_memtime();       \
    } while (0)
#else
#define MARF_STAMP(sp, i) \
    do {                  \
    } while (0)
#endif

// ------------------------------------------------------------------ bf16 helpers

MARF_DEV u16 f2bf(float x) {
    // hardware v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN (torch's conversion)
    __bf16 b = static_cast<__bf16>(x);
    return __builtin_bit_cast(u16, b);
}
MARF_DEV float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }
// fp16 (IEEE binary16): v_cvt_f16_f32 / v_cvt_pk_f16_f32, round-to-nearest-even
MARF_DEV u16 f2h(float x) { return __builtin_bit_cast(u16, static_cast<_Float16>(x)); }
MARF_DEV float h2f(u16 h) { return static_cast<float>(__builtin_bit_cast(_Float16, h)); }
// Numerics experiments (diagnostic builds, -DMARF_DIAG_RT; tools/recipe_sweep.sh): the fp32
// kernels round chosen operands as a lower-precision recipe would see them.  Per layer l, nibble k
// of NetDev::diag[l] is the mode of operand class k -- 0 the forward weight W_l, 1 the dgrad
// weight W_l^T, 2 layer l's input activation, 3 the gradient at layer l's output (dz) -- with mode
// 0 exact fp32, 1 bf16, 2 bf16 hi + lo (~16 bits), 3 fp16, 4 fp16 hi + lo (~22 bits).
MARF_DEV float diag_round(float x, int mode) {
    if (mode == 1) return bf2f(f2bf(x));
    if (mode == 2) {
        const float h = bf2f(f2bf(x));
        return h + bf2f(f2bf(x - h));
    }
    if (mode == 3) return h2f(f2h(x));
    if (mode == 4) {
        const float h = h2f(f2h(x));
        return h + h2f(f2h(x - h));
    }
    return x;
}
MARF_DEV int diag_mode(unsigned code, int k) { return (int)((code >> (4 * k)) & 15u); }
#ifdef MARF_DIAG_RT
#define MARF_DIAG_ROUND(x, code, k) diag_round((x), diag_mode((code), (k)))
#define MARF_DIAG_SAVE(net) diag_mode((net).diag[0], 4)  // saved-tensor rounding (fifth digit)
#else
#define MARF_DIAG_ROUND(x, code, k) (x)
#define MARF_DIAG_SAVE(net) 0
#endif

// ------------------------------------------------------------------ precision traits

// bf16: v_mfma_f32_32x32x16_bf16. A/B fragment of a 16-deep k-step: lane l holds
// A[row l&31][k0 + 8*(l>>5) + j], B[k0 + 8*(l>>5) + j][col l&31], j = 0..7 (16 bytes).
struct PrecBF16 {
    typedef u16 T;
    static constexpr int KS = 16;       // k per MFMA (32x32 shape)
    static constexpr int KS16 = 32;     // k per MFMA (16x16 shape)
    static constexpr int FE = 8;        // elements per lane per A/B fragment
    typedef bf16x8 frag;
    static constexpr int kDtype = 1;

    MARF_DEV static frag load_frag(const T* p) {  // 8 contiguous bf16 (16-B aligned)
        return *reinterpret_cast<const frag*>(p);
    }
    MARF_DEV static int kofs(int lane) { return 8 * (lane >> 5); }    // 32x32 k offset
    MARF_DEV static int kofs16(int lane) { return 8 * (lane >> 4); }  // 16x16 k offset
    MARF_DEV static f32x16 mma32(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    MARF_DEV static f32x4 mma16(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    MARF_DEV static T cvt(float x) { return f2bf(x); }
    MARF_DEV static float tof(T x) { return bf2f(x); }
    MARF_DEV static uint32_t pk2(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        return __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){a, b}), bf16x2));
    }
};

// fp16: v_mfma_f32_32x32x16_f16 / 16x16x32_f16, the bf16 forms' shapes, fragment layouts and
// rate, with 11 significant bits per operand instead of 8 (MARF_FP16).
struct PrecF16 {
    typedef u16 T;
    static constexpr int KS = 16;
    static constexpr int KS16 = 32;
    static constexpr int FE = 8;
    typedef f16x8 frag;
    static constexpr int kDtype = 2;

    MARF_DEV static frag load_frag(const T* p) { return *reinterpret_cast<const frag*>(p); }
    MARF_DEV static int kofs(int lane) { return 8 * (lane >> 5); }
    MARF_DEV static int kofs16(int lane) { return 8 * (lane >> 4); }
    MARF_DEV static f32x16 mma32(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    MARF_DEV static f32x4 mma16(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    MARF_DEV static T cvt(float x) { return f2h(x); }
    MARF_DEV static float tof(T x) { return h2f(x); }
    MARF_DEV static uint32_t pk2(float a, float b) {  // one v_cvt_pk_f16_f32 (RNE)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        return __builtin_bit_cast(uint32_t, __builtin_convertvector(((f32x2){a, b}), f16x2));
    }
};

// fp32: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain). Lane l holds A[row l&31][k0 + (l>>5)],
// B[k0 + (l>>5)][col l&31].  16x16 form: v_mfma_f32_16x16x4_f32, k0 + (l>>4).
struct PrecF32 {
    typedef float T;
    static constexpr int KS = 2;
    static constexpr int KS16 = 4;
    static constexpr int FE = 1;
    typedef float frag;
    static constexpr int kDtype = 0;

    MARF_DEV static frag load_frag(const T* p) { return *p; }
    MARF_DEV static int kofs(int lane) { return lane >> 5; }
    MARF_DEV static int kofs16(int lane) { return lane >> 4; }
    MARF_DEV static f32x16 mma32(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    MARF_DEV static f32x4 mma16(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    MARF_DEV static T cvt(float x) { return x; }
    MARF_DEV static float tof(T x) { return x; }
};

// Row of the 32x32 accumulator element (lane, reg).
MARF_DEV int acc_row(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ------------------------------------------------------------------ network descriptor

#define MARF_MAX_LAYERS 10

struct NetDev {
    int n_layers;                  // Linear layers
    int L;                         // posenc bands (0 = posenc off)
    int D;                         // input features 2 + 4L (or 2)
    int Kp[MARF_MAX_LAYERS];       // padded input width of layer l (Kp[0] = padded D)
    int Mp[MARF_MAX_LAYERS];       // padded output width of layer l (hidden: mult of 32; last: 16)
    int Mt[MARF_MAX_LAYERS];       // padded k-width of Wt_l (= Mp for hidden, 16 for last)
    const void* Wf[MARF_MAX_LAYERS];  // packed forward weights (T)
    const void* Wt[MARF_MAX_LAYERS];  // packed transposed weights (T)
    const float* bias[MARF_MAX_LAYERS];  // padded fp32 bias [Mp]
    unsigned diag[MARF_MAX_LAYERS];      // numerics-experiment rounding codes (MARF_DIAG_RT builds)
    unsigned skip;                       // bit l: layer l's input is [layer l-1 output ; posenc] (Kp[l] =
                                         // Mp[l-1] + Kp[0], the posenc block at column Mp[l-1])
};

// Geometry of the pixel source.
struct GeoDev {
    int mode;       // 0 = crop grid warped by per-patch H; 1 = explicit coordinates
    int B;          // patches (mode 1: 1)
    int Np;         // valid pixels per patch
    int Np_pad;     // slot stride per patch (multiple of MARF_TILE_PAD)
    int H, W;       // canvas
    int x0, y0, w;  // crop origin and crop width (row-major p = r*w + c)
    float norm_h, norm_w;
    const float* Hm;      // [B][9] (mode 0)
    const float* coords;  // [Np][2] (mode 1)
    int bmm_small;        // torch's small-bmm rounding (3 * Np * 3 < 400)
};

// warp.py:38-43: ((i + 0.5) / max * 2 - 1) * norm in fp32 with IEEE division (the library is
// compiled with -ffp-contract=off so no step is fused).
MARF_DEV float grid_coord(int i, int maxdim, float norm) {
    float t = (float)i + 0.5f;
    t = t / (float)maxdim;
    t = t * 2.0f;
    t = t - 1.0f;
    return t * norm;
}

// warp.py:74-78 as torch-CPU's bmm evaluates it.  For a point set with 3*n*3 >= 400 torch runs the
// BLAS path: acc = x*H0; acc = fma(y, H1, acc); acc += H2.  Below that size torch's small-matrix
// kernel accumulates with separate multiply and add (bmm_small = 1).
MARF_DEV void warp_point(const float* Hm, float x, float y, float& u, float& v, float* X, int bmm_small = 0) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float acc = x * Hm[3 * r + 0];
        if (bmm_small) acc = acc + y * Hm[3 * r + 1];
        else acc = __fmaf_rn(y, Hm[3 * r + 1], acc);
        acc = acc + Hm[3 * r + 2];
        X[r] = acc;
    }
    float d = X[2] + 1e-8f;
    u = X[0] / d;
    v = X[1] / d;
}

// Pixel slot -> (x, y) grid point and warped (u, v).  Returns false for padding slots.
// GRID_ONLY: the caller only runs on the crop grid (the fused step); no coordinate-load branch, so
// no outstanding-load merge that would make the compiler wait vmcnt(0) here.
template <bool GRID_ONLY = false>
MARF_DEV bool slot_point(const GeoDev& g, int b, int p, float& x, float& y, float& u, float& v, float* X) {
    if (p >= g.Np) return false;
    if (!GRID_ONLY && g.mode == 1) {
        u = g.coords[2 * (size_t)p];
        v = g.coords[2 * (size_t)p + 1];
        x = u;
        y = v;
        X[0] = u; X[1] = v; X[2] = 1.0f;
        return true;
    }
    int r = p / g.w, c = p - r * g.w;
    x = grid_coord(g.x0 + c, g.W, g.norm_w);
    y = grid_coord(g.y0 + r, g.H, g.norm_h);
    warp_point(g.Hm + 9 * b, x, y, u, v, X, g.bmm_small);
    return true;
}

// BARF coarse-to-fine weight of band k (model/planar.py:462-467).
MARF_DEV float c2f_weight(float progress, float start, float end_minus_start, int L, int k) {
    const float pi_f = 3.14159265358979323846f;
    float a = progress - start;
    a = a / end_minus_start;
    a = a * (float)L;
    float t = a - (float)k;
    t = fminf(fmaxf(t, 0.0f), 1.0f);
    t = t * pi_f;
    t = cosf(t);
    return (1.0f - t) / 2.0f;
}

// Posenc argument 2^k * fl(c * pi_f32), bit-identical to fl(c * fl(2^k * pi_f32)).
MARF_DEV float posenc_arg(float c, int k) {
    const float pi_f = 3.14159265358979323846f;
    return ldexpf(c * pi_f, k);
}

// sin / cos of the posenc argument x = 2^k * fl(c * pi_f32).
//   exact (fp32 path): ocml sincosf of the fp32 argument, as torch evaluates it.
//   fast (bf16 path, whose features are rounded to bf16 = 2^-9 relative anyway): reduce x to
//   revolutions f = frac(x / 2pi) with a double-float product (|error| < 2^-40 rev for k <= 20),
//   then the hardware v_sin_f32 / v_cos_f32, which take revolutions.  ~10 VALU instead of ~100.
template <bool kFast>
MARF_DEV void band_sincos(float c, int k, float& s, float& co) {
    const float pi_f = 3.14159265358979323846f;
    const float y = c * pi_f;
    if constexpr (kFast) {
        const float r_hi = 0.159154936671257019f;    // fl(1 / 2pi)
        const float r_lo = 6.42063831672591501e-09f;  // 1/2pi - r_hi
        float th = y * r_hi;
        float tl = __fmaf_rn(y, r_hi, -th);          // exact product error
        tl = __fmaf_rn(y, r_lo, tl);
        th = ldexpf(th, k);
        tl = ldexpf(tl, k);
        float f = th - rintf(th);                    // exact
        f = f + tl;
        s = __builtin_amdgcn_sinf(f);
        co = __builtin_amdgcn_cosf(f);
    } else {
        sincosf(ldexpf(y, k), &s, &co);
    }
}

// Wave reductions on the DPP network (no LDS traffic): quad swaps, row rotations, then the gfx9
// row broadcasts; fixed order, the total lands in lane 63.
template <int CTRL, int ROWMASK = 0xf>
MARF_DEV int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK = 0xf>
MARF_DEV float dpp_f(float v) {
    return __int_as_float(dpp_i<CTRL, ROWMASK>(__float_as_int(v)));
}
template <int CTRL, int ROWMASK = 0xf>
MARF_DEV double dpp_d(double v) {
    const long long u = __double_as_longlong(v);
    const int lo = dpp_i<CTRL, ROWMASK>((int)(u & 0xffffffffLL)), hi = dpp_i<CTRL, ROWMASK>((int)(u >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <class V>
MARF_DEV V wave_total63(V v) {
    if constexpr (sizeof(V) == 8) {
        v += dpp_d<0xB1>(v);        // quad_perm [1,0,3,2]
        v += dpp_d<0x4E>(v);        // quad_perm [2,3,0,1]
        v += dpp_d<0x124>(v);       // row_ror:4
        v += dpp_d<0x128>(v);       // row_ror:8   -> every lane holds its row's sum
        v += dpp_d<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
        v += dpp_d<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
    } else {
        v += dpp_f<0xB1>(v);
        v += dpp_f<0x4E>(v);
        v += dpp_f<0x124>(v);
        v += dpp_f<0x128>(v);
        v += dpp_f<0x142, 0xa>(v);
        v += dpp_f<0x143, 0xc>(v);
    }
    return v;
}
