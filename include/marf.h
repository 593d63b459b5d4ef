/*
 * marf.h -- C ABI of libmarf.so, the MI355X (gfx950) implementation of the planar
 * bundle-adjustment render loop of thomasjaron/masking-bundle-adjusting-neural-radiance-fields
 * (model/planar.py + warp.py).
 *
 * The reference has no FFI: its boundary is the Python module API.  Each entry
 * point below replaces the reference interface named in its comment; the Python host package
 * (masking-bundle-adjusting-neural-radiance-fields_amd/marf_hip.py) binds them with ctypes and
 * keeps the reference's module / autograd contract on top.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Every pointer argument named d_* / device is HIP device
 *     memory owned by the caller (PyTorch's allocator); the library borrows it for the call.
 *   - `stream` is a hipStream_t passed as void*; every call is asynchronous on it, no implicit
 *     device synchronisation, no allocation on the step path.
 *   - Every function returns 0 on success or a negative MARF_ERR_* code; marf_last_error()
 *     returns a thread-local message for the last failure.
 *   - float32 everywhere in the interface; dtype selects the internal MLP arithmetic
 *     (MARF_FP32 = exact fp32 MFMA, MARF_BF16 = bf16 MFMA with fp32 accumulation, MARF_BF16X3 = split
 *     bf16, MARF_FP16 = fp16 MFMA with fp32 accumulation, MARF_FP16X2 = split-fp16 weights).
 */
#ifndef MARF_H
#define MARF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MARF_OK 0
#define MARF_ERR_INVALID -1   /* bad argument / shape (reference: AssertionError) */
#define MARF_ERR_HIP -2       /* HIP runtime error */
#define MARF_ERR_UNSUPPORTED -3

#define MARF_FP32 0
#define MARF_BF16 1
#define MARF_BF16X3 2 /* split bf16: weights and forward activations as bf16 hi + lo pairs (hi*hi + hi*lo + lo*hi
                         forward, hi + lo weights in the dgrad), bf16 dz / saved tensors; fused step and
                         marf_render only (marf_forward / marf_backward return MARF_ERR_UNSUPPORTED) */

#define MARF_FP16 3   /* fp16 MFMA (v_mfma_f32_32x32x16_f16, fp32 accumulation): weights, activations, dz and the
                         saved tensors in IEEE binary16 (11 significant bits); the bf16 rate */
#define MARF_FP16X2 4 /* split-fp16 weights: every MFMA fp16 with the weights as fp16 hi + lo pairs (W_hi a +
                         W_lo a forward, W_hi^T dz + W_lo^T dz dgrad: 2 MFMAs per MAC), activations, dz and
                         the saved tensors single fp16 (dz carrying an exact 2^10 gradient scale); full-width
                         nets (5 layers, every hidden layer 256 wide, 8 <= L <= 16, no skip); fused step and
                         marf_render only */

#define MARF_GEO_GRID 0   /* pixels of the centre crop, warped by a per-patch homography */
#define MARF_GEO_COORDS 1 /* explicit [n][2] coordinates (one point set) */
#define MARF_GEO_CANVAS 2 /* every pixel of the H x W canvas (use_cropped_images off), warped per patch
                             (warp.py:54-68 grid; patch_H / patch_W ignored) */

typedef struct marf_net marf_net; /* opaque: MLP shape + padding plan */

typedef struct {
    int mode;             /* MARF_GEO_GRID, MARF_GEO_CANVAS or MARF_GEO_COORDS */
    int B;                /* patches (GRID / CANVAS) ; must be 1 for COORDS */
    int Np;               /* GRID / CANVAS: computed; COORDS: number of points */
    int H, W;             /* canvas (opt.H, opt.W) */
    int patch_H, patch_W; /* crop (opt.patch_H, opt.patch_W) */
    const float* d_H;     /* GRID: [B][3][3] homographies (from marf_sl3_to_SL3) */
    const float* d_coords;/* COORDS: [Np][2] */
} marf_geometry;

typedef struct {
    const float* d_progress; /* fp32 scalar on device (NeuralImageFunction.progress) */
    double start, end;       /* opt.barf_c2f */
    int on;                  /* 0: barf_c2f is None (no band weighting) */
} marf_c2f;

const char* marf_last_error(void);
int marf_version(void);
/* sha1 of the sources the library was built from (build_lib.py embeds it; the host binding refuses
 * a library whose hash differs from the sources next to it). */
const char* marf_source_hash(void);

/* ---- Lie group (warp.py:95-106 Lie.sl3_to_SL3; torch.linalg.matrix_exp semantics).
 * lie_batch: the batch size torch would see (selects torch's path; pass B unless sharded). */
int marf_sl3_to_SL3(const float* d_h, float* d_H, int B, int lie_batch, void* stream);
int marf_sl3_to_SL3_backward(const float* d_h, const float* d_dH, float* d_dh, int B, int lie_batch, void* stream);
/* SE(2) warps (north_star "sl(3)/SE(2)"; an extension: the reference has sl(3) only, warp.py:72-80).
 * se(2) tangent p = (tx, ty, theta) [B][3] -> the sl(3) parameters h [B][8] of the same generator
 * [[0,-theta,tx],[theta,0,ty],[0,0,0]] in warp.py:101-104's layout; marf_sl3_to_SL3(h) is then the
 * SE(2) exponential and every warp / step entry point takes h unchanged.  Backward: dp = adjoint(dh). */
int marf_se2_to_sl3(const float* d_p, float* d_h, int B, void* stream);
int marf_se2_to_sl3_backward(const float* d_dh, float* d_dp, int B, void* stream);

/* ---- Warp (warp.py:33-68 get_normalized_pixel_grid, one copy [n][2]; warp.py:70-81 warp_grid) */
int marf_pixel_grid(int H, int W, int patch_H, int patch_W, int crop, float* d_xy, void* stream);
int marf_warp_points(const float* d_xy, const float* d_H, float* d_uv, int B, int n, int xy_shared, void* stream);

/* ---- Positional encoding + c2f (model/planar.py:451-471): [n][2] -> [n][4L] */
int marf_posenc(const float* d_coord, long long n, int L, const marf_c2f* c2f, float* d_enc, void* stream);

/* Autograd of Warp.warp_grid's point warp (warp.py:70-81): upstream d_G [B][n][2] -> d xy
 * [B][n][2] (per patch even when xy_shared: the caller sums them) and dH [B][3][3] (per-patch sum
 * over points, fp64 accumulation).  dh then follows from marf_sl3_to_SL3_backward. */
int marf_warp_points_backward(const float* d_xy, const float* d_H, const float* d_G, float* d_dxy, float* d_dH, int B,
                              int n, int xy_shared, void* stream);
/* Autograd of NeuralImageFunction.positional_encoding (model/planar.py:451-471): d_G [n][4L] ->
 * d coord [n][2]; the c2f weights are constants (progress carries no gradient). */
int marf_posenc_backward(const float* d_coord, long long n, int L, const marf_c2f* c2f, const float* d_G, float* d_dcoord,
                         void* stream);

/* Measurement only (no reference counterpart): the fused step's per-pixel input side -- target +
 * mask reads (16 B/px), pixel grid, warp, posenc + c2f -- as a standalone launch of `grid` blocks,
 * one float per block into d_out, so the prologue's HBM rate can be timed. */
int marf_prologue_probe(const marf_geometry* geo, const marf_c2f* c2f, int L, const float* d_gt, const float* d_mask,
                        float* d_out, int grid, void* stream);

/* ---- Neural image MLP (model/planar.py:395-449, NeuralImageFunction)
 * dims[0] = 2 + 4L (input), dims[n_layers] = 3, hidden dims arbitrary (padded internally).
 * Flat fp32 parameter vector layout = NeuralImageFunction.mlp parameters in module order:
 * W0 [dims1][dims0], b0 [dims1], W1, b1, ...  (nn.Linear layout). */
int marf_net_create(int n_layers, const int* dims, int L, int dtype, marf_net** out);
/* As marf_net_create, with the pixels one fused step will process on this GPU (0 = unknown; kept for
 * size-dependent kernel choices: the split recipe runs k_step2 at every size today). */
int marf_net_create_hint(int n_layers, const int* dims, int L, int dtype, long long pixels_hint, marf_net** out);
/* As marf_net_create_hint, with skip connections (model/planar.py:419-420, 440-441; opt.arch.skip):
 * bit l of skip_mask makes layer l's input [previous layer's output ; posenc features] (k_in =
 * dims[l] + dims[0] in the flat parameter layout).  Hidden layers 1 .. n_layers-2 only, dims[l] a
 * multiple of 32; the tile kernels (fp32, bf16, fp16) run such nets, the split-bf16 recipe refuses them. */
int marf_net_create_skip(int n_layers, const int* dims, int L, int dtype, long long pixels_hint, unsigned skip_mask,
                         marf_net** out);
void marf_net_destroy(marf_net* net);
long long marf_net_param_count(const marf_net* net);
size_t marf_net_packed_bytes(const marf_net* net);
/* Name of the kernel that runs this net's fused training step ("k_step2" or "k_mlp_step"),
 * fixed at net creation (no reference counterpart: measurement and test bookkeeping). */
const char* marf_net_step_kernel(const marf_net* net);
/* Layer l's parameters in the flat vector: W_l [dims[l+1]][dims[l]] then b_l, from *off, *len floats. */
int marf_net_layer_count(const marf_net* net);
int marf_net_layer_span(const marf_net* net, int l, long long* off, long long* len);
/* Pipelined weight gradients of the fused step (no reference counterpart: scheduling only; the
 * reference's loss.all.backward() at model/planar.py:196 computes the same sums).  mode 0 = off
 * (default; env MARF_PIPE at net creation), 1 = on at any size, -1 = on for large steps.  When on,
 * marf_step_forward runs the step kernel in pieces of piece_tiles tiles on CUs - wg_blocks blocks
 * and the split-K weight-gradient partials of each finished piece on wg_blocks CUs of a second
 * stream; marf_step_backward then only reduces them.  0 = the default size.  Change it between
 * steps only (the saved-buffer layout of a step depends on it).  Measured slower than the
 * sequential step on MI355X: off by default. */
int marf_net_set_pipeline(marf_net* net, int mode, int wg_blocks, int piece_tiles);
/* fp32 master parameters -> MFMA operand layouts (call after every optimizer step). */
int marf_net_pack(const marf_net* net, const float* d_params, void* d_packed, void* stream);

/* Bytes of the activation cache the backward needs, and of the backward scratch. */
size_t marf_saved_bytes(const marf_net* net, const marf_geometry* geo);
size_t marf_workspace_bytes(const marf_net* net, const marf_geometry* geo);

/* Forward (Graph.forward model/planar.py:329-335 for GRID: grid -> warp -> posenc -> MLP;
 * NeuralImageFunction.forward :429 for COORDS).  rgb: [B][Np][3].  d_saved NULL = inference. */
int marf_forward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                 float* d_rgb, void* d_saved, void* stream);

/* Backward of marf_forward given d loss / d rgb.  Writes (overwrites) d_params (flat, fp32),
 * and d_h [B][8] (GRID, needs d_h_params = the sl(3) warp parameters) or d_coords [Np][2]
 * (COORDS).  Any output pointer may be NULL. */
int marf_backward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                  const float* d_h_params, int lie_batch, const float* d_rgb_out, const float* d_drgb,
                  const void* d_saved, void* d_workspace, float* d_dparams, float* d_dh, float* d_dcoords,
                  void* stream);

/* Forward-only render (Graph.forward / NeuralImageFunction.forward without autograd,
 * model/planar.py:329-335, 429-449; Model.predict_entire_image :211-217) in the net's recipe: for
 * split-bf16 nets the pixel-per-wave kernel on grid, canvas or explicit-coordinate geometry with a
 * workspace of marf_render_workspace_bytes(); otherwise marf_forward (d_ws unused). */
size_t marf_render_workspace_bytes(const marf_net* net, const marf_geometry* geo);
int marf_render(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed, float* d_rgb,
                void* d_ws, void* stream);

/* ---- Fused training step (grid geometry).  Graph.forward + Graph.mse_loss (model/planar.py:329-336,
 * 382-391) and the backward of both, computed in one pass per pixel tile because the target and
 * mask are known at forward time.  marf_step_forward writes rgb [B][Np][3] (may be NULL), the loss
 * d_loss_out[3] (as marf_masked_mse: loss, denominator, local 3*sum(mask)) and keeps in d_saved
 * (marf_step_saved_bytes) everything the gradient needs, computed for a unit upstream gradient.
 * marf_step_backward turns it into d_params (flat, fp32) and d_dh [B][8] for the upstream gradient
 * *d_gout (device scalar, d loss / d loss_rgb), reading the denominator from d_loss_out[1]. */
size_t marf_step_saved_bytes(const marf_net* net, const marf_geometry* geo);
int marf_step_forward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                      const float* d_gt, const float* d_mask, const float* d_denom_override, float* d_rgb,
                      float* d_loss_out, void* d_saved, void* stream);
int marf_step_backward(const marf_net* net, const marf_geometry* geo, const void* d_saved, const float* d_h_params,
                       int lie_batch, const float* d_gout, const float* d_loss_out, float* d_dparams, float* d_dh,
                       void* stream);
/* As marf_step_backward; layer_events[l] (hipEvent_t, n_layers entries, NULL entries skipped) is
 * recorded on the stream as soon as layer l's gradient in d_dparams is final.  The layers finish
 * last layer first, layer 0 last (the order a bucketed all-reduce consumes them). */
int marf_step_backward_ev(const marf_net* net, const marf_geometry* geo, const void* d_saved, const float* d_h_params,
                          int lie_batch, const float* d_gout, const float* d_loss_out, float* d_dparams, float* d_dh,
                          void* const* layer_events, void* stream);

/* ---- MLP-gradient exchange of the patch-sharded step (the reference is
 * single-GPU, options.py:117-120, so this replaces no reference call: it is the one collective the
 * sharding adds).  RCCL over xGMI, librccl.so opened at first use.  marf_comm_unique_id fills 128
 * bytes on one rank (the host shares them with the others); marf_comm_create joins rank `rank` of
 * `nranks` on `device`.  marf_allreduce_grads sums a flat fp32 gradient in place on `stream`;
 * marf_allreduce_grads_layers sums each layer's span (marf_net_layer_span) on the communicator's
 * own stream after its marf_step_backward_ev event, so the exchange overlaps the remaining weight
 * gradients, and makes `stream` wait for the last one.  A NULL entry of layer_events waits for the
 * work queued on `stream` before the call.  marf_comm_create leaves the calling thread's current
 * device unchanged.  After an error from either all-reduce call the ranks' collective sequences may
 * disagree: destroy the communicator (every rank) rather than reuse it. */
typedef struct marf_comm marf_comm;
int marf_comm_unique_id(void* out, size_t cap);
int marf_comm_create(const void* unique_id, int nranks, int rank, int device, marf_comm** out);
void marf_comm_destroy(marf_comm* comm);
int marf_allreduce_grads(marf_comm* comm, float* d_flat, size_t n, void* stream);
int marf_allreduce_grads_layers(marf_comm* comm, const marf_net* net, float* d_dparams, void* const* layer_events,
                                void* stream);

/* ---- Masked MSE (Graph.mse_loss, model/planar.py:382-391).  pred [B][Np][3] (MLP layout),
 * gt [B][3][Np], mask [B][1][Np] or NULL (plain mean).  d_out[3]: loss, denominator used,
 * local 3*sum(mask).  d_denom_override: optional device scalar (global denominator of a patch
 * shard).  d_ws: marf_mse_workspace_bytes(). */
size_t marf_mse_workspace_bytes(void);
int marf_masked_mse(const float* d_pred, const float* d_gt, const float* d_mask, int B, int Np,
                    const float* d_denom_override, float* d_out, void* d_ws, void* stream);
int marf_masked_mse_backward(const float* d_pred, const float* d_gt, const float* d_mask, int B, int Np,
                             const float* d_denom, const float* d_gout, float* d_dpred, void* stream);

/* ---- Edge maps (inputs.compute_edges, reference inputs.py:50-67: cv2.Sobel 3x3 CV_64F in x and y,
 * magnitude, cv2.GaussianBlur 5x5 sigma 0, BORDER_REFLECT_101), per channel image on the device.
 * d_img [n_img][H][W] fp32 -> d_out [n_img][H][W] fp64. */
int marf_edge_map(const float* d_img, int n_img, int H, int W, double* d_out, void* stream);

/* ---- Mask erosion (erode_images, reference inputs.py:71-85: cv2.erode with a kh x kw MORPH_RECT
 * element, default anchor and border).  d_img [n_img][H][W] fp32 -> d_out (a different buffer). */
int marf_erode_rect(const float* d_img, int n_img, int H, int W, int kh, int kw, float* d_out, void* stream);

/* ---- Adam (torch.optim.Adam, model/planar.py:98-99): one parameter segment, step >= 1.
 * d_grad_scale: optional device scalar multiplying the gradient (NULL = 1). */
int marf_adam_step(float* d_p, const float* d_g, float* d_m, float* d_v, long long n, double lr, double beta1,
                   double beta2, double eps, long long step, const float* d_grad_scale, void* stream);
/* The same update with the step's scalars read on the device, so a captured training iteration
 * (Model.captured_step) replays it without host values: marf_adam_schedule fills h_out[2 i],
 * h_out[2 i + 1] with step_size = lr / (1 - beta1^k) and sqrt(1 - beta2^k) for k = first_step + i,
 * exactly as marf_adam_step computes them (host only); marf_adam_step_sched reads row *d_index of
 * that table (uploaded by the caller) on the stream. */
int marf_adam_schedule(double lr, double beta1, double beta2, long long first_step, long long count, float* h_out);
int marf_adam_step_sched(float* d_p, const float* d_g, float* d_m, float* d_v, long long n, double beta1, double beta2,
                         double eps, const float* d_sched, const int* d_index, const float* d_grad_scale, void* stream);

/* ---- Profiling: HIP events recorded around each kernel on its launch stream (off by default).
 * marf_profile_read drains the recorded pairs (synchronising on them) and returns, per kernel
 * name, the summed duration (ms) and launch count; names is a [cap][name_len] char array. */
int marf_profile_enable(int on);
/* Restrict the timing to the kernels named in `names` (comma-separated profile names, e.g.
 * "mlp_step"; NULL or "" = every kernel), so a timed region pays for the event pairs of the kernels
 * it reports only (each pair adds a few microseconds between launches). */
int marf_profile_filter(const char* names);
int marf_profile_reset(void);
int marf_profile_read(char* names, int name_len, double* total_ms, long long* count, int cap);

/* ---- Diagnostics: device buffer [n_tiles][32] (u64) receiving the fused step's per-phase
 * s_memtime stamps; only a library built with -DMARF_STAMPS writes it (tools/phase_stamps.py). */
void marf_debug_set_stamps(void* d_stamps);

#ifdef __cplusplus
}
#endif
#endif /* MARF_H */
