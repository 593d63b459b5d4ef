// marf_args.h -- kernel argument blocks and host launcher prototypes shared by the .hip units.
#pragma once
#include "marf_common.h"

namespace marf {

struct C2fDev {
    const float* progress;  // device scalar (NeuralImageFunction.progress)
    float start, span;      // barf_c2f start, end - start
    int on;
};

struct FwdArgs {
    NetDev net;
    GeoDev geo;
    C2fDev c2f;
    float* rgb;                       // [B][Np][3]
    void* feat[MARF_MAX_LAYERS];      // saved layer inputs [S][Kp_l] (nullptr: do not save)
    uint64_t* mask[MARF_MAX_LAYERS];  // relu masks of feat_l (l >= 1), wave-ballot layout (marf_common.h)
    long long S;
    int lda;                          // LDS row stride (elements)
};

struct BwdArgs {
    NetDev net;
    GeoDev geo;
    C2fDev c2f;
    const float* rgb;                       // [B][Np][3] forward output
    const float* d_rgb;                     // [B][Np][3]
    const uint64_t* mask[MARF_MAX_LAYERS];  // from forward
    void* dz[MARF_MAX_LAYERS];              // out: dz_l (l >= 1) [S][Kp_l] (grad of layer l-1 pre-act)
    float* glast;                           // out: [S][4] grad of the last layer pre-activation
    float* dH_partial;                      // out (geo mode 0): [n_tiles][9]
    float* d_coords;                        // out (geo mode 1): [Np][2] (may be null)
    long long S;
    int lda;
};

// Fused training step of the grid geometry (marf_step.hip): forward, masked MSE with unit upstream
// gradient, dgrad chain and warp adjoint in one pass over each tile.
struct StepArgs {
    NetDev net;
    GeoDev geo;
    C2fDev c2f;
    float* rgb;                             // [B][Np][3] forward output (may be null)
    const float* gt;                        // [B][3][Np] target
    const float* mask;                      // [B][1][Np] or null (plain mean)
    void* feat[MARF_MAX_LAYERS];            // out: inputs of layers 0 .. n-2 [S][Kp_l]
    uint64_t* mask_bits[MARF_MAX_LAYERS];   // scratch: ReLU masks of feat_l, l = 1 .. n-1
    void* dz[MARF_MAX_LAYERS];              // out: dz_l, l = 1 .. n-1 [S][Kp_l]
    float* wlast_partial;                   // out: [n_tiles][3][Kp_{n-1}] last-layer weight gradient
    float* blast_partial;                   // out: [n_tiles][3]
    float* dH_partial;                      // out: [n_tiles][9]
    double* loss_partial;                   // out: [n_tiles][2] = sum ((p - g) m)^2, sum m
    const float* c2f_w;                     // [L] band weights of this step (k_c2f_weights)
    unsigned long long* stamps;             // diagnostic builds (MARF_STAMPS): [n_tiles][32] s_memtime
    long long S;
    int lda;
};

struct PackLayer {
    int M, K;                            // true dims (nn.Linear weight [M][K])
    int Mp, Kp, Mt;                      // padded: Wf [Mp][Kp], Wt [Kp][Mt], bias [Mp]
    long long w_off, b_off;              // offsets in the flat fp32 parameter vector
    long long wf_off, wt_off, bias_off;  // byte offsets in the packed buffer
    unsigned diag;                       // numerics-experiment rounding code (marf_common.h)
};

struct PackArgs {
    int n_layers;
    PackLayer ly[MARF_MAX_LAYERS];
};

// Per-layer constants, copied into LDS at kernel start (kept out of the SGPR file).
struct S2Layer {
    int nrt;     // row tiles of the forward output (Mp / 32; last layer: 1)
    int nrtb;    // row tiles of the dgrad output (Kp / 32; layer 0: the adjoint tiles)
    int boff;    // offset of the padded bias in the bias table
    int ldf;     // row stride of feat_l (elements)
    int ldz;     // row stride of dz_l
    int pad;
    u16* feat;   // feat_l [S][ldf] bf16 (l = 0 .. nl-2)
    u16* dz;     // dz_l [S][ldz] bf16 (l = 1 .. nl-1)
};

struct Step2Args {
    GeoDev geo;                      // Np_pad is a multiple of 32 * NW
    int nl, L, nk0, nta, c2f_on;
    int r0;                          // layer-0 row tiles per stage
    const char* prog;                // weight stage program: n_stages slots of SLOT bytes
    int n_stages;
    int n_fwd;                       // the program's forward stages (the first n_fwd; the rest: dgrad)
    long long S;                     // pixel slots; rows S .. S + 32 NW - 1 of dz_l / dH: store sink
                                     // of a backward pixel set that has no tile (odd tile count)
    const float* bias;               // padded biases
    int nbias;                       // floats in the bias table
    const float* gt;                 // [B][3][Np]
    const float* mask;               // [B][1][Np] or null
    float* rgb;                      // [B][Np][3] or null
    S2Layer layers[MARF_MAX_LAYERS]; // per-layer table (copied into LDS at kernel start)
    float* dH_partial;               // [S / 32 + NW][9]
    double* loss_partial;            // [grid][2]
    float* blast_partial;            // [grid][3]
    float* wlast_partial;            // [grid][3][Kl]
    int Kl;                          // padded input width of the last layer
    const float* c2f_w;              // [L] band weights of this step
    float* dummy;                    // [grid][NW][ST][64][2] store sink
    unsigned long long* stamps;      // diagnostic builds (MARF_STAMPS): [grid][8] cycle totals of wave 0
    int tile0, n_tiles;              // this launch's block tiles [tile0, n_tiles) of 32 * NW pixel slots
    int fwd_only;                    // render: forward stages only, rgb out, nothing saved
    int feat0_recompute;             // feat_0 is recomputed by the layer-0 weight gradient: not stored
    const float* pro_fallback;       // valid device address for the input DMA when gt / H are absent
    // LDS layout (byte offsets; computed on the host)
    int lds_pro, lds_bias, lds_c2f, lds_layers, lds_wave, lds_wave_bytes, lds_total;
};

struct Pack2Args {
    int nl, L, nk0, nta, NKH, split, slot_bytes, n_stages;
    int fwd_f16;                     // forward stages in fp16 hi + lo (the fp16x2 recipe)
    int r0, ns0;                     // layer-0 row tiles per stage, layer-0 stages
    int dims[MARF_MAX_LAYERS + 1];   // true widths
    int nrt[MARF_MAX_LAYERS], nrtb[MARF_MAX_LAYERS];
    long long w_off[MARF_MAX_LAYERS], b_off[MARF_MAX_LAYERS];  // flat parameter offsets
    int boff[MARF_MAX_LAYERS];       // padded bias table offsets
    int Mp[MARF_MAX_LAYERS];
    int nbias;
};

// Raise a kernel's dynamic-LDS limit to at least `lds` bytes before a launch.  The limit set so
// far is tracked per (device, kernel) under a mutex, so a later launch of the same instantiation
// with a larger tile (a wider net) raises it again, and concurrent host threads do not race.
hipError_t ensure_dynamic_lds(const void* kernel, size_t lds);

}  // namespace marf

hipError_t marf_launch_sl3(const float* h, float* H, int B, int batch_hint, hipStream_t s);
hipError_t marf_launch_se2_embed(const float* p, float* h, int B, hipStream_t s);
hipError_t marf_launch_se2_embed_bwd(const float* dh, float* dp, int B, hipStream_t s);
hipError_t marf_launch_sl3_bwd(const float* h, const float* dH, float* dh, int B, int batch_hint, hipStream_t s);
hipError_t marf_launch_reduce_dH(const float* partial, int tiles_per_patch, int B, const float* h, float* dH_out,
                                 float* dh, int batch_hint, hipStream_t s, const float* gscale = nullptr,
                                 const float* denom = nullptr);
hipError_t marf_launch_mlp_fwd(const marf::FwdArgs& a, int dtype, int TP, size_t lds, int n_tiles, hipStream_t s);
hipError_t marf_launch_mlp_bwd(const marf::BwdArgs& a, int dtype, int TP, size_t lds, int n_tiles, hipStream_t s);
// one piece of a pipelined step's weight gradients: n blocks split the pixel rows [s_lo, s_lo + s_len)
// and write split-K partials part0 .. part0 + n - 1
struct WgRange {
    long long s_lo, s_len;
    int n, part0;
};
bool marf_wgrad_range_ok(int dtype, int M, int ldz, int K, int ldf);
bool marf_wgrad_l0_recompute_ok(int M, int ldz, int ldf0, long long S, int chunk, int n_chunks, long long Np_pad);
hipError_t marf_launch_wgrad_l0_recompute(const void* dz, int ldz, const GeoDev& geo, const float* c2f_w, int L,
                                          int nk0, int K0, long long S, int M, int chunk, int n_chunks, float* partial,
                                          float* bpartial, hipStream_t s, const WgRange* rng = nullptr, int dtype = 1);
// t16: dz / feat in the split-recipe step kernel's T16 block layout (marf_wgrad.hip t16_off)
hipError_t marf_launch_wgrad(int dtype, const void* dz, int ldz, const void* feat, int ldf, long long S, int M, int K,
                             int chunk, int n_chunks, float* partial, float* bpartial, hipStream_t s,
                             const WgRange* rng = nullptr, bool t16 = false);
// One layer of the fused weight-gradient launch (marf_launch_wgrad_fused): its split-K partials
// [n_parts][M][K] (+ [n_parts][M] bias) and the fixed-order reduction into dW [Mo][Ko] / db [Mo].
struct WgFusedLayer {
    int kind;                 // 0: 256 x 256 LDS-DMA (hidden layer); 1: layer 0, feat_0 recomputed (256 x 96);
                              // 2: layer 0 stored (marf_launch_wgrad's kernel); 3: reduction only
    const void* dz;           // kinds 0..2: [S][ldz] bf16 (fp16x2: fp16)
    const void* feat;         // kinds 0, 2: [S][ldf] bf16 (fp16x2: fp16)
    int ldz, ldf, M, K;
    float* partial;
    float* bpartial;
    int n_parts;              // partials to reduce (kinds 0..2: the launch's n_chunks)
    int Mo, Ko;
    float* dW;
    float* db;
    const int* kmap;          // layer 0: column of true input feature k in the partial
};
// every kind-0 layer's chunk products in one launch on s, the layer-0 one (kind 1 or 2) beside it on
// s2 (fork / join events), then every layer's reduction in one launch on s; false if a shape does
// not qualify
bool marf_wgrad_fused_ok(const WgFusedLayer* layers, int n_layers, long long S, int chunk, int n_chunks,
                         long long Np_pad);
hipError_t marf_launch_wgrad_fused(const WgFusedLayer* layers, int n_layers, long long S, int chunk, int n_chunks,
                                   const GeoDev& f0_geo, const float* c2f_w, int L, int nk0, const float* gscale,
                                   const float* denom, hipStream_t s, hipStream_t s2, hipEvent_t fork, hipEvent_t join,
                                   int dtype = 1, float post = 1.f);  // dtype 2 / post 2^-10: the fp16x2 recipe
hipError_t marf_launch_wgrad_last(int dtype, const float* glast, const void* feat, long long S, int ldf, int K,
                                  int chunk, int n_chunks, float* partial, float* bpartial, hipStream_t s);
hipError_t marf_launch_wgrad_reduce(const float* partial, const float* bpartial, int n_chunks, int M, int K, int Mo,
                                    int Ko, float* dW, float* db, hipStream_t s, const float* gscale = nullptr,
                                    const float* denom = nullptr, float* scratch = nullptr,
                                    const int* kmap = nullptr, float post = 1.f);
hipError_t marf_launch_mlp_step(const marf::StepArgs& a, int dtype, int TP, int NW, size_t lds, int n_tiles, hipStream_t s);
hipError_t marf_launch_c2f_weights(const marf::C2fDev& c, int L, float* out, hipStream_t s,
                                   const int* csrc = nullptr, int* cdst = nullptr, int cn = 0);
hipError_t marf_launch_loss_final(const double* part, int n, float* out, const float* denom_override, hipStream_t s);
hipError_t marf_launch_step2(const marf::Step2Args& a, int variant, int grid, hipStream_t s, int full_nk0, bool dz = false);
hipError_t marf_launch_pack2(const float* params, void* prog, float* bias_out, int* kmap, const marf::Pack2Args& a,
                             hipStream_t s);
hipError_t marf_launch_edge_map(const float* in, double* out, int n_img, int H, int W, hipStream_t s);
hipError_t marf_launch_erode_rect(const float* in, float* out, int n_img, int H, int W, int kh, int kw, hipStream_t s);
hipError_t marf_launch_mse(const float* pred, const float* gt, const float* mask, int B, int Np, double* part,
                           float* out, const float* denom_override, hipStream_t s);
hipError_t marf_launch_mse_bwd(const float* pred, const float* gt, const float* mask, int B, int Np,
                               const float* denom, const float* gout, float* d_pred, hipStream_t s);
hipError_t marf_launch_adam(float* p, const float* g, float* m, float* v, long long n, float w1, float b2,
                            float one_minus_b2, float step_size, float bc2_sqrt, float eps, const float* grad_scale,
                            hipStream_t s);
hipError_t marf_launch_adam_sched(float* p, const float* g, float* m, float* v, long long n, float w1, float b2,
                                  float one_minus_b2, const float* sched, const int* index, float eps,
                                  const float* grad_scale, hipStream_t s);
hipError_t marf_launch_pack(int dtype, const float* params, char* packed, const marf::PackArgs& a,
                            long long max_elems, hipStream_t s);
hipError_t marf_launch_pixel_grid(const GeoDev& g, float* xy, int n, hipStream_t s);
hipError_t marf_launch_warp_points(const float* xy, const float* Hm, float* uv, int B, int n, int xy_shared,
                                   hipStream_t s);
hipError_t marf_launch_posenc(const float* coord, long long n, int L, const float* progress, float start, float span,
                              int c2f_on, float* enc, hipStream_t s);
hipError_t marf_launch_warp_points_bwd(const float* xy, const float* Hm, const float* G, float* dxy, float* dH, int B,
                                       int n, int xy_shared, hipStream_t s);
hipError_t marf_launch_posenc_bwd(const float* coord, const float* G, long long n, int L, const float* progress,
                                  float start, float span, int c2f_on, float* dcoord, hipStream_t s);
hipError_t marf_launch_prologue_probe(const GeoDev& g, const marf::C2fDev& c, int L, const float* gt,
                                      const float* mask, float* out, int grid, hipStream_t s);
