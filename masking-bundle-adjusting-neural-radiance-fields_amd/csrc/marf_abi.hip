// marf_abi.hip -- extern "C" entry points of libmarf.so (declared in include/marf.h).
// Host-side validation, buffer planning and kernel launches; no device allocation here: every
// buffer is owned by the caller (PyTorch's caching allocator).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/marf.h"
#include "marf_args.h"
#include "marf_prof.h"

using namespace marf;

static thread_local std::string g_err;
static unsigned long long* g_stamps = nullptr;  // diagnostic phase stamps (MARF_STAMPS builds)

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

static int check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(MARF_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return MARF_OK;
}

#define HIPCHK(expr, what)                          \
    do {                                            \
        int _rc = check_hip((expr), (what));        \
        if (_rc != MARF_OK) return _rc;             \
    } while (0)

static inline long long rup(long long x, long long m) { return (x + m - 1) / m * m; }

// step2 plan (the pixel-per-wave fused step, marf_step2.hip), filled by plan_step2_net
struct Step2NetPlan {
    int variant;           // -1: not available for this net; 0: bf16 (8 waves); 1: split bf16 (4 waves);
                           // 2: bf16 on 4 waves (diagnostic); 3: fp16x2 (split-fp16 weights, fp16
                           // activations and dz, two pixel sets per forward and dgrad stage; 4 waves,
                           // compile-time layer 0 only)
    bool dz;               // variant 1 with the dgrad's dz split too (MARF_STEP2_DZ=1 at net creation)
    int NW, NS, HM, MAXR, NMW, slot, nk0, nta, n_stages, nbias, Kl, ldf0;
    int PX, TPX;           // pixels per wave, pixel slots per block tile
    int nslot;             // weight-ring slots in LDS
    int nk0w;              // k_step2's layer-0 k-steps: feat_0's column layout (weight gradient, kmap)
    int n_fwd;             // the program's forward stages
    int r0, ns0;           // layer-0 row tiles per stage (their k-steps share one slot) and its stages
    int nrt[MARF_MAX_LAYERS], nrtb[MARF_MAX_LAYERS], boff[MARF_MAX_LAYERS];
    size_t prog_off, bias_off, kmap_off, end_off;
};

struct marf_net {
    int n_layers, L, D, dtype;
    unsigned skip;  // bit l: layer l's input is [feature ; posenc] (model/planar.py:419-420, 440-441)
    int kin[MARF_MAX_LAYERS];  // true input width of layer l (dims[l], + D for a skip layer)
    int kdt;  // kernel arithmetic of the generic kernels: 0 fp32, 1 bf16 (MARF_BF16 and MARF_BF16X3), 2 fp16
    Step2NetPlan s2;
    int dims[MARF_MAX_LAYERS + 1];
    int Kp[MARF_MAX_LAYERS], Mp[MARF_MAX_LAYERS], Mt[MARF_MAX_LAYERS];
    long long w_off[MARF_MAX_LAYERS], b_off[MARF_MAX_LAYERS], param_count;
    long long wf_off[MARF_MAX_LAYERS], wt_off[MARF_MAX_LAYERS], bias_off[MARF_MAX_LAYERS];
    size_t packed_bytes;
    int TP, lda, Kmax;
    int sTP, sNW;  // the fused step's tile (pixel slots) and waves per block (k_mlp_step)
    size_t lds_fwd, lds_bwd, lds_step;
    int elem;  // bytes per stored element
    unsigned diag[MARF_MAX_LAYERS];  // numerics-experiment rounding codes (MARF_DIAG_PREC; MARF_DIAG_RT builds)
    int pipe_mode, pipe_wg, pipe_piece;  // pipelined weight gradients (marf_net_set_pipeline)
};

// MARF_DIAG_PREC = "WTAD[S],WTAD,..." per layer (digits: marf_common.h diag_round modes; the last
// entry repeats): the rounding a lower-precision recipe would apply, emulated by the fp32 kernels of
// a MARF_DIAG_RT build (tools/recipe_sweep.sh); an optional fifth digit of the first entry rounds
// every saved tensor the weight gradients read (feat_l, dz_l).  Read once at net creation; other
// builds ignore it.
static void parse_diag(marf_net* n) {
    const char* e = getenv("MARF_DIAG_PREC");
    unsigned code = 0;
    for (int l = 0; l < n->n_layers; ++l) {
        if (e && *e) {
            code = 0;
            for (int k = 0; k < 5 && e[k] >= '0' && e[k] <= '9'; ++k) code |= (unsigned)(e[k] - '0') << (4 * k);
            while (*e && *e != ',') ++e;
            if (*e == ',') ++e;
        }
        n->diag[l] = code;
    }
}

// the split recipes: every path runs k_step2's weight program (no tile-kernel arithmetic for them)
static bool split_recipe(int dtype) { return dtype == MARF_BF16X3 || dtype == MARF_FP16X2; }

static bool step2_env_enabled() {
    const char* e = getenv("MARF_STEP2");  // plain bf16 on the pixel-per-wave kernel: opt-in ("1")
    return e && e[0] == '1';
}

static int device_cus();

// Which pixel-per-wave variant (marf_step2.hip) runs this net, its weight-program shape and the
// byte layout of the program / bias table / layer-0 column map appended to the packed buffer.
// Full-width nets (every hidden layer 256 wide) at L = 8, 9..12, 13..15 and 16 run k_step2's
// compile-time instantiations, every other net the generic k_step2 (the same arithmetic, so the same
// bits: test_step2_bits_unchanged).  (Round 4's k_step3, the same bits at two waves per SIMD, was
// slower than these instantiations at every size measured but 2 patches, profiles/r4s, and is gone.)
static void plan_step2_net(marf_net* n, long long pixels_hint) {
    Step2NetPlan& q = n->s2;
    memset(&q, 0, sizeof(q));
    q.variant = -1;
    const int nl = n->n_layers;
    if (n->kdt != 1 || nl < 2 || nl > 5 || n->L > 32 || n->skip) return;  // (skip nets: the tile kernels)
    for (int l = 0; l < nl - 1; ++l)
        if (n->Mp[l] > 256) return;
    // decided once, here: the split recipe always runs this kernel; plain bf16 only on request
    // (MARF_STEP2=1 at net creation), otherwise it runs the tile kernel and needs no program
    if (!split_recipe(n->dtype) && !step2_env_enabled()) return;
    q.HM = 256;
    q.variant = n->dtype == MARF_BF16X3 ? 1 : (n->dtype == MARF_FP16X2 ? 3 : 0);
    (void)pixels_hint;  // (kernel choice by size: none left to make)
    {
        const char* e = getenv("MARF_STEP2_NW4");  // diagnostic: plain bf16 on 4 waves per block
        if (q.variant == 0 && e && e[0] == '1') q.variant = 2;
    }
    q.NW = q.variant == 0 ? 8 : 4;
    q.nslot = 3;
    {  // the split recipe with dz split in the dgrad too (k_step2's DZ; numerics option)
        const char* e = getenv("MARF_STEP2_DZ");
        q.dz = q.variant == 1 && e && e[0] == '1';
    }
    q.NS = (q.variant == 1 && !q.dz) || q.variant == 3 ? 2 : 1;  // pixel sets per dgrad pass (S2Cfg::NS)
    q.PX = 32;
    q.TPX = 32 * q.NW;
    q.MAXR = 4;
    q.NMW = q.HM / 64;
    q.slot = (q.HM / 16) * 1024 * (q.variant == 1 || q.variant == 3 ? 2 : 1);
    q.nk0 = (n->L + 3) / 4 + 1;
    q.nk0w = q.nk0;
    q.nta = (2 * n->L + 1 + 15) / 16;
    q.ldf0 = (int)rup(16 * q.nk0, 32);
    q.Kl = n->Kp[nl - 1];
    int st = 0, bo = 0;
    for (int l = 0; l < nl; ++l) {
        q.nrt[l] = l == nl - 1 ? 1 : n->Mp[l] / 32;
        q.nrtb[l] = l == 0 ? q.nta : n->Kp[l] / 32;
        q.boff[l] = bo;
        bo += l == nl - 1 ? 32 : n->Mp[l];
    }
    q.nbias = bo;
    q.r0 = std::max(1, std::min(q.nrt[0], (q.HM / 16) / q.nk0));
    q.ns0 = (q.nrt[0] + q.r0 - 1) / q.r0;
    st += q.ns0;
    for (int l = 1; l < nl - 1; ++l) st += q.nrt[l];
    q.n_fwd = st + 1;
    st += 2;  // last layer forward, last-layer dgrad (every row tile in one stage)
    for (int l = nl - 2; l >= 1; --l) st += q.nrtb[l];
    st += q.nta;
    q.n_stages = st;
    q.prog_off = rup((long long)n->packed_bytes, 4096);
    q.bias_off = q.prog_off + (size_t)st * q.slot;
    q.kmap_off = rup((long long)(q.bias_off + (size_t)q.nbias * 4), 256);
    q.end_off = rup((long long)(q.kmap_off + (size_t)n->D * 4), 256);
    if (q.variant == 3) {  // fp16x2: full-width nets with a compile-time layer-0 instantiation only
        bool full = q.Kl == 256 && nl == 5 && q.r0 == std::max(1, std::min(8, 16 / q.nk0)) &&
                    ((q.nk0 == 5 && (q.nta == 3 || q.nta == 2)) || (q.nk0 == 4 && q.nta == 2) || (q.nk0 == 3 && q.nta == 2));
        for (int l = 0; l < nl - 1; ++l) full = full && n->Mp[l] == 256;
        if (!full) q.variant = -1;
    }
}

extern "C" {

const char* marf_last_error(void) { return g_err.c_str(); }
// (for the other translation units: marf_comm.hip)
int marf_set_error(int code, const char* msg) { return fail(code, "%s", msg); }

// Diagnostic builds only: device buffer [n_tiles][32] for the fused step's phase stamps.
void marf_debug_set_stamps(void* d_stamps) { g_stamps = (unsigned long long*)d_stamps; }
int marf_version(void) { return 1; }

#ifndef MARF_SOURCE_HASH
#define MARF_SOURCE_HASH "0000000000000000000000000000000000000000"
#endif
// the marker is searched for in the binary by build_lib.embedded_hash
static const char k_source_hash[] = "MARF_SOURCE_HASH=" MARF_SOURCE_HASH;
const char* marf_source_hash(void) { return k_source_hash + 17; }

// ------------------------------------------------------------------ Lie / warp / posenc

int marf_sl3_to_SL3(const float* d_h, float* d_H, int B, int lie_batch, void* stream) {
    if (B < 0 || (B > 0 && (!d_h || !d_H))) return fail(MARF_ERR_INVALID, "sl3_to_SL3: bad arguments");
    MarfProfScope ps("lie_exp", (hipStream_t)stream);
    HIPCHK(marf_launch_sl3(d_h, d_H, B, lie_batch > 0 ? lie_batch : B, (hipStream_t)stream), "sl3_to_SL3");
    return MARF_OK;
}

int marf_sl3_to_SL3_backward(const float* d_h, const float* d_dH, float* d_dh, int B, int lie_batch, void* stream) {
    if (B < 0 || (B > 0 && (!d_h || !d_dH || !d_dh))) return fail(MARF_ERR_INVALID, "sl3_to_SL3_backward: bad arguments");
    HIPCHK(marf_launch_sl3_bwd(d_h, d_dH, d_dh, B, lie_batch > 0 ? lie_batch : B, (hipStream_t)stream),
           "sl3_to_SL3_backward");
    return MARF_OK;
}

int marf_se2_to_sl3(const float* d_p, float* d_h, int B, void* stream) {
    if (B < 0 || (B > 0 && (!d_p || !d_h))) return fail(MARF_ERR_INVALID, "se2_to_sl3: bad arguments");
    HIPCHK(marf_launch_se2_embed(d_p, d_h, B, (hipStream_t)stream), "se2_to_sl3");
    return MARF_OK;
}

int marf_se2_to_sl3_backward(const float* d_dh, float* d_dp, int B, void* stream) {
    if (B < 0 || (B > 0 && (!d_dh || !d_dp))) return fail(MARF_ERR_INVALID, "se2_to_sl3_backward: bad arguments");
    HIPCHK(marf_launch_se2_embed_bwd(d_dh, d_dp, B, (hipStream_t)stream), "se2_to_sl3_backward");
    return MARF_OK;
}

static int make_geo(const marf_geometry* g, GeoDev& d, int TP_pad) {
    if (!g) return fail(MARF_ERR_INVALID, "geometry is NULL");
    memset(&d, 0, sizeof(d));
    d.mode = g->mode == MARF_GEO_CANVAS ? MARF_GEO_GRID : g->mode;  // the kernels see a window
    if (g->mode == MARF_GEO_CANVAS) {
        // warp.py:54-68: every canvas pixel, row-major (no centre-crop integer halving)
        if (g->B <= 0 || g->H <= 0 || g->W <= 0 || (long long)g->H * g->W > (1LL << 30))
            return fail(MARF_ERR_INVALID, "canvas geometry: B=%d H=%d W=%d", g->B, g->H, g->W);
        if (!g->d_H) return fail(MARF_ERR_INVALID, "canvas geometry needs d_H");
        int mx = std::max(g->H, g->W);
        d.B = g->B;
        d.y0 = 0;
        d.x0 = 0;
        d.w = g->W;
        d.Np = g->H * g->W;
        d.H = g->H;
        d.W = g->W;
        d.norm_h = (float)((double)g->H / (double)mx);
        d.norm_w = (float)((double)g->W / (double)mx);
        d.Hm = g->d_H;
    } else if (g->mode == MARF_GEO_GRID) {
        if (g->B <= 0 || g->H <= 0 || g->W <= 0 || g->patch_H <= 1 || g->patch_W <= 1 || g->patch_H > g->H ||
            g->patch_W > g->W)
            return fail(MARF_ERR_INVALID, "grid geometry: B=%d H=%d W=%d patch=%dx%d", g->B, g->H, g->W, g->patch_H,
                        g->patch_W);
        if (!g->d_H) return fail(MARF_ERR_INVALID, "grid geometry needs d_H");
        // warp.py:14-19: crop window = centre +- half (integer division, as the reference)
        int y0 = g->H / 2 - g->patch_H / 2, y1 = g->H / 2 + g->patch_H / 2;
        int x0 = g->W / 2 - g->patch_W / 2, x1 = g->W / 2 + g->patch_W / 2;
        d.B = g->B;
        d.y0 = y0;
        d.x0 = x0;
        d.w = x1 - x0;
        d.Np = (y1 - y0) * (x1 - x0);
        d.H = g->H;
        d.W = g->W;
        int mx = std::max(g->H, g->W);
        d.norm_h = (float)((double)g->H / (double)mx);
        d.norm_w = (float)((double)g->W / (double)mx);
        d.Hm = g->d_H;
    } else if (g->mode == MARF_GEO_COORDS) {
        if (g->B != 1 || g->Np <= 0 || !g->d_coords)
            return fail(MARF_ERR_INVALID, "coords geometry: B must be 1, Np > 0, coords given");
        d.B = 1;
        d.Np = g->Np;
        d.coords = g->d_coords;
        d.w = 1;
    } else {
        return fail(MARF_ERR_INVALID, "unknown geometry mode %d", g->mode);
    }
    d.Np_pad = (int)rup(d.Np, TP_pad);
    d.bmm_small = (d.mode == MARF_GEO_GRID && 9LL * d.Np < 400) ? 1 : 0;
    return MARF_OK;
}

int marf_pixel_grid(int H, int W, int patch_H, int patch_W, int crop, float* d_xy, void* stream) {
    if (H <= 0 || W <= 0 || !d_xy) return fail(MARF_ERR_INVALID, "pixel_grid: bad arguments");
    GeoDev g;
    memset(&g, 0, sizeof(g));
    int mx = std::max(H, W);
    g.H = H;
    g.W = W;
    g.norm_h = (float)((double)H / (double)mx);
    g.norm_w = (float)((double)W / (double)mx);
    int h = H;
    if (crop) {
        if (patch_H <= 0 || patch_W <= 0 || patch_H > H || patch_W > W)
            return fail(MARF_ERR_INVALID, "pixel_grid: bad crop %dx%d", patch_H, patch_W);
        g.y0 = H / 2 - patch_H / 2;
        g.x0 = W / 2 - patch_W / 2;
        h = (H / 2 + patch_H / 2) - g.y0;
        g.w = (W / 2 + patch_W / 2) - g.x0;
    } else {
        g.w = W;
    }
    HIPCHK(marf_launch_pixel_grid(g, d_xy, h * g.w, (hipStream_t)stream), "pixel_grid");
    return MARF_OK;
}

int marf_warp_points(const float* d_xy, const float* d_H, float* d_uv, int B, int n, int xy_shared, void* stream) {
    if (B <= 0 || n < 0 || !d_xy || !d_H || !d_uv) return fail(MARF_ERR_INVALID, "warp_points: bad arguments");
    if (n == 0) return MARF_OK;
    HIPCHK(marf_launch_warp_points(d_xy, d_H, d_uv, B, n, xy_shared, (hipStream_t)stream), "warp_points");
    return MARF_OK;
}

static C2fDev make_c2f(const marf_c2f* c) {
    C2fDev d;
    memset(&d, 0, sizeof(d));
    if (c && c->on && c->d_progress) {
        d.on = 1;
        d.progress = c->d_progress;
        d.start = (float)c->start;
        d.span = (float)(c->end - c->start);
    }
    return d;
}

int marf_posenc(const float* d_coord, long long n, int L, const marf_c2f* c2f, float* d_enc, void* stream) {
    if (n < 0 || L <= 0 || L > 32 || !d_coord || !d_enc) return fail(MARF_ERR_INVALID, "posenc: bad arguments");
    if (n == 0) return MARF_OK;
    C2fDev c = make_c2f(c2f);
    HIPCHK(marf_launch_posenc(d_coord, n, L, c.progress, c.start, c.span, c.on, d_enc, (hipStream_t)stream), "posenc");
    return MARF_OK;
}

int marf_warp_points_backward(const float* d_xy, const float* d_H, const float* d_G, float* d_dxy, float* d_dH, int B,
                              int n, int xy_shared, void* stream) {
    if (B <= 0 || n < 0 || !d_xy || !d_H || !d_G || !d_dxy || !d_dH)
        return fail(MARF_ERR_INVALID, "warp_points_backward: bad arguments");
    HIPCHK(marf_launch_warp_points_bwd(d_xy, d_H, d_G, d_dxy, d_dH, B, n, xy_shared, (hipStream_t)stream),
           "warp_points_backward");
    return MARF_OK;
}

int marf_posenc_backward(const float* d_coord, long long n, int L, const marf_c2f* c2f, const float* d_G, float* d_dcoord,
                         void* stream) {
    if (n < 0 || L <= 0 || L > 32 || !d_coord || !d_G || !d_dcoord)
        return fail(MARF_ERR_INVALID, "posenc_backward: bad arguments");
    if (n == 0) return MARF_OK;
    C2fDev c = make_c2f(c2f);
    HIPCHK(marf_launch_posenc_bwd(d_coord, d_G, n, L, c.progress, c.start, c.span, c.on, d_dcoord, (hipStream_t)stream),
           "posenc_backward");
    return MARF_OK;
}

// Measurement only: the fused step's input side (target + mask reads, grid, warp, posenc) as its
// own launch, so that the prologue's HBM rate can be timed.  d_out: `grid` floats.
int marf_prologue_probe(const marf_geometry* geo, const marf_c2f* c2f, int L, const float* d_gt, const float* d_mask,
                        float* d_out, int grid, void* stream) {
    GeoDev g;
    int rc = make_geo(geo, g, MARF_TILE_PAD);
    if (rc != MARF_OK) return rc;
    if (g.mode != MARF_GEO_GRID || L < 0 || L > 32 || !d_gt || !d_out || grid <= 0)
        return fail(MARF_ERR_INVALID, "prologue_probe: bad arguments");
    MarfProfScope ps("prologue_probe", (hipStream_t)stream);
    HIPCHK(marf_launch_prologue_probe(g, make_c2f(c2f), L, d_gt, d_mask, d_out, grid, (hipStream_t)stream),
           "prologue_probe");
    return MARF_OK;
}

// ------------------------------------------------------------------ network

int marf_net_create(int n_layers, const int* dims, int L, int dtype, marf_net** out) {
    return marf_net_create_skip(n_layers, dims, L, dtype, 0, 0u, out);
}

int marf_net_create_hint(int n_layers, const int* dims, int L, int dtype, long long pixels_hint, marf_net** out) {
    return marf_net_create_skip(n_layers, dims, L, dtype, pixels_hint, 0u, out);
}

int marf_net_create_skip(int n_layers, const int* dims, int L, int dtype, long long pixels_hint, unsigned skip_mask,
                         marf_net** out) {
    if (!out || !dims) return fail(MARF_ERR_INVALID, "net_create: NULL argument");
    *out = nullptr;
    if (n_layers < 2 || n_layers > MARF_MAX_LAYERS)
        return fail(MARF_ERR_UNSUPPORTED, "net_create: n_layers=%d (supported 2..%d)", n_layers, MARF_MAX_LAYERS);
    if (dtype != MARF_FP32 && dtype != MARF_BF16 && dtype != MARF_BF16X3 && dtype != MARF_FP16 && dtype != MARF_FP16X2)
        return fail(MARF_ERR_INVALID, "net_create: dtype %d", dtype);
    if (L < 0 || L > 32) return fail(MARF_ERR_UNSUPPORTED, "net_create: L=%d (supported 0..32)", L);
    int D = L > 0 ? 2 + 4 * L : 2;
    if (dims[0] != D) return fail(MARF_ERR_INVALID, "net_create: dims[0]=%d but 2+4L=%d", dims[0], D);
    if (dims[n_layers] != 3) return fail(MARF_ERR_INVALID, "net_create: output dim %d != 3", dims[n_layers]);
    marf_net* n = new marf_net;
    memset(n, 0, sizeof(*n));
    n->n_layers = n_layers;
    n->L = L;
    n->D = D;
    n->dtype = dtype;
    n->kdt = dtype == MARF_FP32 ? 0 : (dtype == MARF_FP16 ? 2 : 1);
    n->elem = n->kdt != 0 ? 2 : 4;
    for (int i = 0; i <= n_layers; ++i) {
        if (dims[i] <= 0) {
            delete n;
            return fail(MARF_ERR_INVALID, "net_create: dims[%d]=%d", i, dims[i]);
        }
        n->dims[i] = dims[i];
    }
    // skip layers: hidden layers 1 .. n-2 whose input is [previous output ; posenc]; the posenc
    // block sits at column Mp[l-1] of the layer's padded input, so the previous width must be a
    // multiple of 32 (true column k -> padded column k, the padding after them)
    if (skip_mask >> n_layers) {
        delete n;
        return fail(MARF_ERR_INVALID, "net_create: skip mask 0x%x names layers beyond %d", skip_mask, n_layers - 1);
    }
    n->skip = skip_mask;
    for (int l = 0; l < n_layers; ++l) {
        const bool sk = (skip_mask >> l) & 1u;
        if (sk && (l == 0 || l == n_layers - 1)) {
            delete n;
            return fail(MARF_ERR_UNSUPPORTED, "net_create: skip connection into layer %d (hidden layers 1..%d only)", l,
                        n_layers - 2);
        }
        if (sk && dims[l] % 32) {
            delete n;
            return fail(MARF_ERR_UNSUPPORTED, "net_create: skip layer %d needs an input width multiple of 32 (got %d)", l,
                        dims[l]);
        }
        n->kin[l] = dims[l] + (sk ? D : 0);
    }
    n->Kp[0] = (int)rup(D, 32);
    int hmax = 0;
    for (int l = 0; l < n_layers - 1; ++l) {
        n->Mp[l] = (int)rup(dims[l + 1], 32);
        n->Mt[l] = n->Mp[l];
        n->Kp[l + 1] = n->Mp[l] + (((skip_mask >> (l + 1)) & 1u) ? n->Kp[0] : 0);
        hmax = std::max(hmax, n->Mp[l]);
    }
    n->Mp[n_layers - 1] = 16;
    n->Mt[n_layers - 1] = n->kdt != 0 ? 16 : 4;
    n->Kmax = 0;
    for (int l = 0; l < n_layers; ++l) n->Kmax = std::max(n->Kmax, n->Kp[l]);
    if (hmax > 512 || n->Kmax > 512) {
        delete n;
        return fail(MARF_ERR_UNSUPPORTED, "net_create: hidden width %d / layer input %d > 512", hmax, n->Kmax);
    }
    n->TP = (n->kdt != 0 && n->Kmax <= 256) ? 128 : 64;
    n->lda = n->kdt != 0 ? n->Kmax + 8 : n->Kmax + 1;
    size_t act = (size_t)n->TP * n->lda * n->elem;
    size_t df = (size_t)n->TP * (n->Kp[0] + 1) * 4;
    // skip nets: the posenc gradient of the skip layers, accumulated beside the tile (fp32 [TP][Kp0])
    const size_t dsk = n->skip ? (size_t)n->TP * n->Kp[0] * 4 : 0;
    n->lds_fwd = act;
    n->lds_bwd = std::max(act, df) + dsk;
    n->lds_step = n->lds_bwd;
    // The fused step of a 16-bit net wider than 256: one 512-thread block per CU at TP = 128
    // (MARF_STEP_NW=4 at net creation keeps two 4-wave blocks at TP = 64, for A/B runs)
    n->sTP = n->TP;
    n->sNW = 4;
    {
        const char* e = getenv("MARF_STEP_NW");
        const bool nw8 = !(e && e[0] == '4');
        const size_t act8 = (size_t)128 * n->lda * n->elem, df8 = (size_t)128 * (n->Kp[0] + 1) * 4;
        const size_t dsk8 = n->skip ? (size_t)128 * n->Kp[0] * 4 : 0;
        if (nw8 && n->kdt != 0 && n->Kmax > 256 && std::max(act8, df8) + dsk8 + 16 * 1024 <= 160 * 1024) {
            n->sTP = 128;
            n->sNW = 8;
            n->lds_step = std::max(act8, df8) + dsk8;
        }
    }
    // the 4-wave tile kernels' static __shared__ beside the dynamic tile (k_mlp_step: wsh, red, red9,
    // gl, gT, lsum, bsh; the separate forward / backward kernels hold less): checked here, so a shape
    // whose step would fail ensure_dynamic_lds at launch is refused at creation instead
    const size_t static4 = 128 + (size_t)std::max(4 * 64, 2 * n->TP) * 2 * 4 + 4 * 9 * 4 + (size_t)n->TP * 16 +
                           8 * (size_t)n->TP * n->elem + 2 * (size_t)n->TP * 4 + 16 + 512;
    if (n->lds_bwd + static4 > 160 * 1024) {
        delete n;
        return fail(MARF_ERR_UNSUPPORTED, "net_create: tile does not fit LDS (%zu B dynamic + %zu B static)", n->lds_bwd,
                    static4);
    }
    long long off = 0;
    size_t boff = 0;
    for (int l = 0; l < n_layers; ++l) {
        n->w_off[l] = off;
        off += (long long)dims[l + 1] * n->kin[l];
        n->b_off[l] = off;
        off += dims[l + 1];
        n->wf_off[l] = (long long)boff;
        boff += rup((long long)n->Mp[l] * n->Kp[l] * n->elem, 256);
        n->wt_off[l] = (long long)boff;
        boff += rup((long long)n->Kp[l] * n->Mt[l] * n->elem, 256);
        n->bias_off[l] = (long long)boff;
        boff += rup((long long)n->Mp[l] * 4, 256);
    }
    n->param_count = off;
    n->packed_bytes = boff;
    parse_diag(n);
    plan_step2_net(n, pixels_hint);
    {  // defaults of the pipelined weight gradients (marf_net_set_pipeline changes them)
        const char* e = getenv("MARF_PIPE");
        n->pipe_mode = e && *e ? atoi(e) : 0;  // off: measured slower
        e = getenv("MARF_PIPE_WG");
        n->pipe_wg = e && *e ? atoi(e) : 0;
        e = getenv("MARF_PIPE_PIECE");
        n->pipe_piece = e && *e ? atoi(e) : 0;
    }
    if (n->s2.variant >= 0) n->packed_bytes = n->s2.end_off;
    if (dtype == MARF_FP16X2 && n->s2.variant < 0) {
        delete n;
        return fail(MARF_ERR_UNSUPPORTED,
                    "net_create: fp16x2 needs 5 layers, every hidden layer 256 wide, 8 <= L <= 16 and no skip layers");
    }
    if (dtype == MARF_BF16X3 && n->s2.variant < 0) {
        delete n;
        return fail(MARF_ERR_UNSUPPORTED,
                    "net_create: split-bf16 needs <= 5 layers, hidden widths <= 256, L <= 32 and no skip layers");
    }
    *out = n;
    return MARF_OK;
}

void marf_net_destroy(marf_net* net) { delete net; }

int marf_net_set_pipeline(marf_net* net, int mode, int wg_blocks, int piece_tiles) {
    if (!net) return fail(MARF_ERR_INVALID, "net_set_pipeline: NULL net");
    if (mode < -1 || mode > 1 || wg_blocks < 0 || piece_tiles < 0)
        return fail(MARF_ERR_INVALID, "net_set_pipeline: mode %d, wg_blocks %d, piece_tiles %d", mode, wg_blocks,
                    piece_tiles);
    net->pipe_mode = mode;
    net->pipe_wg = wg_blocks;
    net->pipe_piece = piece_tiles;
    return MARF_OK;
}
long long marf_net_param_count(const marf_net* net) { return net ? net->param_count : -1; }
size_t marf_net_packed_bytes(const marf_net* net) { return net ? net->packed_bytes : 0; }
int marf_net_layer_count(const marf_net* net) { return net ? net->n_layers : 0; }
int marf_net_layer_span(const marf_net* net, int l, long long* off, long long* len) {
    if (!net || l < 0 || l >= net->n_layers || !off || !len) return fail(MARF_ERR_INVALID, "net_layer_span: bad arguments");
    *off = net->w_off[l];
    *len = (long long)net->dims[l + 1] * net->kin[l] + net->dims[l + 1];  // W_l then b_l
    return MARF_OK;
}
const char* marf_net_step_kernel(const marf_net* net) {
    if (!net) return "";
    if (net->s2.variant == 3) return "k_step2h";
    if (net->s2.variant >= 0) return "k_step2";
    return "k_mlp_step";
}

int marf_net_pack(const marf_net* net, const float* d_params, void* d_packed, void* stream) {
    if (!net || !d_params || !d_packed) return fail(MARF_ERR_INVALID, "net_pack: NULL argument");
    PackArgs a;
    memset(&a, 0, sizeof(a));
    a.n_layers = net->n_layers;
    long long mx = 0;
    for (int l = 0; l < net->n_layers; ++l) {
        PackLayer& p = a.ly[l];
        p.M = net->dims[l + 1];
        p.K = net->kin[l];
        p.Mp = net->Mp[l];
        p.Kp = net->Kp[l];
        p.Mt = net->Mt[l];
        p.w_off = net->w_off[l];
        p.b_off = net->b_off[l];
        p.wf_off = net->wf_off[l];
        p.wt_off = net->wt_off[l];
        p.bias_off = net->bias_off[l];
        p.diag = net->diag[l];
        mx = std::max(mx, (long long)p.Mp * p.Kp + (long long)p.Kp * p.Mt + p.Mp);
    }
    MarfProfScope ps("pack_weights", (hipStream_t)stream);
    // the tile kernels' layouts (Wf / Wt / bias): every path of a split-bf16 net runs k_step2's
    // program instead (marf_forward / marf_backward refuse it), so it packs that one only
    if (!split_recipe(net->dtype))
        HIPCHK(marf_launch_pack(net->kdt, d_params, (char*)d_packed, a, mx, (hipStream_t)stream), "net_pack");
    if (net->s2.variant >= 0) {
        const Step2NetPlan& q = net->s2;
        Pack2Args b;
        memset(&b, 0, sizeof(b));
        b.nl = net->n_layers;
        b.L = net->L;
        b.nk0 = q.nk0;
        b.nta = q.nta;
        b.NKH = q.HM / 16;
        b.split = q.variant == 1 || q.variant == 3;
        b.fwd_f16 = q.variant == 3;
        b.slot_bytes = q.slot;
        b.n_stages = q.n_stages;
        b.r0 = q.r0;
        b.ns0 = q.ns0;
        for (int l = 0; l <= net->n_layers; ++l) b.dims[l] = net->dims[l];
        for (int l = 0; l < net->n_layers; ++l) {
            b.nrt[l] = q.nrt[l];
            b.nrtb[l] = q.nrtb[l];
            b.w_off[l] = net->w_off[l];
            b.b_off[l] = net->b_off[l];
            b.boff[l] = q.boff[l];
            b.Mp[l] = net->Mp[l];
        }
        b.nbias = q.nbias;
        char* pk = (char*)d_packed;
        HIPCHK(marf_launch_pack2(d_params, pk + q.prog_off, (float*)(pk + q.bias_off), (int*)(pk + q.kmap_off), b,
                                 (hipStream_t)stream),
               "net_pack step2");
    }
    return MARF_OK;
}

static void fill_netdev(const marf_net* n, const void* packed, NetDev& d) {
    memset(&d, 0, sizeof(d));
    d.n_layers = n->n_layers;
    d.L = n->L;
    d.D = n->D;
    for (int l = 0; l < n->n_layers; ++l) {
        d.Kp[l] = n->Kp[l];
        d.Mp[l] = n->Mp[l];
        d.Mt[l] = n->Mt[l];
        d.Wf[l] = (const char*)packed + n->wf_off[l];
        d.Wt[l] = (const char*)packed + n->wt_off[l];
        d.bias[l] = (const float*)((const char*)packed + n->bias_off[l]);
        d.diag[l] = n->diag[l];
    }
    d.skip = n->skip;
}

// ------------------------------------------------------------------ buffer plans

struct SavedPlan {
    size_t feat[MARF_MAX_LAYERS], mask[MARF_MAX_LAYERS], total;
};

static void plan_saved(const marf_net* n, long long S, SavedPlan& p) {
    size_t off = 0;
    for (int l = 0; l < n->n_layers; ++l) {
        p.feat[l] = off;
        off += rup((long long)S * n->Kp[l] * n->elem, 256);
    }
    p.mask[0] = 0;
    for (int l = 1; l < n->n_layers; ++l) {
        p.mask[l] = off;
        off += rup(S / n->TP * 4096, 256);  // mask records: one uint4 per lane per wave per tile
    }
    p.total = off;
}

struct WsPlan {
    size_t dz[MARF_MAX_LAYERS], glast, dH, part, bpart, total;
    int chunk, n_chunks, n_tiles;
    int chunk_last, n_chunks_last;  // finer split for the bandwidth-bound last-layer wgrad
};

static void plan_ws(const marf_net* n, long long S, int n_tiles, WsPlan& p) {
    size_t off = 0;
    p.dz[0] = 0;
    for (int l = 1; l < n->n_layers; ++l) {
        p.dz[l] = off;
        off += rup((long long)S * n->Kp[l] * n->elem, 256);
    }
    p.glast = off;
    off += rup(S * 16, 256);
    p.dH = off;
    off += rup((long long)n_tiles * 9 * 4, 256);
    long long chunk = rup((S + 255) / 256, 64);
    if (chunk < 64) chunk = 64;
    p.chunk = (int)chunk;
    p.n_chunks = (int)((S + chunk - 1) / chunk);
    p.n_tiles = n_tiles;
    long long mxo = 0, mxm = 0;
    for (int l = 0; l < n->n_layers - 1; ++l) {
        mxo = std::max(mxo, (long long)n->Mp[l] * n->Kp[l]);
        mxm = std::max(mxm, (long long)n->Mp[l]);
    }
    long long cl = rup((S + 1023) / 1024, 64);
    if (cl < 64) cl = 64;
    p.chunk_last = (int)cl;
    p.n_chunks_last = (int)((S + cl - 1) / cl);
    long long part_elems = std::max((long long)p.n_chunks * mxo, (long long)p.n_chunks_last * 3 * n->Kp[n->n_layers - 1]);
    long long bpart_elems = std::max((long long)p.n_chunks * mxm, (long long)p.n_chunks_last * 3);
    p.part = off;
    off += rup(part_elems * 4, 256);
    p.bpart = off;
    off += rup(bpart_elems * 4, 256);
    p.total = off;
}

size_t marf_saved_bytes(const marf_net* net, const marf_geometry* geo) {
    GeoDev g;
    if (!net || make_geo(geo, g, MARF_TILE_PAD) != MARF_OK) return 0;
    SavedPlan p;
    plan_saved(net, (long long)g.B * g.Np_pad, p);
    return p.total;
}

size_t marf_workspace_bytes(const marf_net* net, const marf_geometry* geo) {
    GeoDev g;
    if (!net || make_geo(geo, g, MARF_TILE_PAD) != MARF_OK) return 0;
    long long S = (long long)g.B * g.Np_pad;
    WsPlan p;
    plan_ws(net, S, (int)(S / net->TP), p);
    return p.total;
}

// ------------------------------------------------------------------ forward / backward

int marf_forward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                 float* d_rgb, void* d_saved, void* stream) {
    if (!net || !d_packed || !d_rgb) return fail(MARF_ERR_INVALID, "forward: NULL argument");
    if (split_recipe(net->dtype))  // the generic kernels have no split arithmetic
        return fail(MARF_ERR_UNSUPPORTED, "forward: split-recipe nets run marf_step_forward / marf_render only");
    FwdArgs a;
    memset(&a, 0, sizeof(a));
    int rc = make_geo(geo, a.geo, MARF_TILE_PAD);
    if (rc) return rc;
    fill_netdev(net, d_packed, a.net);
    a.c2f = make_c2f(c2f);
    a.rgb = d_rgb;
    a.S = (long long)a.geo.B * a.geo.Np_pad;
    a.lda = net->lda;
    if (d_saved) {
        SavedPlan p;
        plan_saved(net, a.S, p);
        for (int l = 0; l < net->n_layers; ++l) a.feat[l] = (char*)d_saved + p.feat[l];
        for (int l = 1; l < net->n_layers; ++l) a.mask[l] = (uint64_t*)((char*)d_saved + p.mask[l]);
    }
    int n_tiles = (int)(a.S / net->TP);
    {
        MarfProfScope ps("mlp_fwd", (hipStream_t)stream);
        HIPCHK(marf_launch_mlp_fwd(a, net->kdt, net->TP, net->lds_fwd, n_tiles, (hipStream_t)stream), "forward");
    }
    return MARF_OK;
}

int marf_backward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                  const float* d_h_params, int lie_batch, const float* d_rgb_out, const float* d_drgb,
                  const void* d_saved, void* d_workspace, float* d_dparams, float* d_dh, float* d_dcoords,
                  void* stream) {
    if (!net || !d_packed || !d_rgb_out || !d_drgb || !d_saved || !d_workspace)
        return fail(MARF_ERR_INVALID, "backward: NULL argument");
    if (split_recipe(net->dtype))
        return fail(MARF_ERR_UNSUPPORTED, "backward: split-recipe nets run marf_step_backward only");
    hipStream_t s = (hipStream_t)stream;
    BwdArgs a;
    memset(&a, 0, sizeof(a));
    int rc = make_geo(geo, a.geo, MARF_TILE_PAD);
    if (rc) return rc;
    if (a.geo.mode == MARF_GEO_GRID && d_dh && !d_h_params)
        return fail(MARF_ERR_INVALID, "backward: d_dh requested without the warp parameters");
    fill_netdev(net, d_packed, a.net);
    a.c2f = make_c2f(c2f);
    a.rgb = d_rgb_out;
    a.d_rgb = d_drgb;
    a.S = (long long)a.geo.B * a.geo.Np_pad;
    a.lda = net->lda;
    const int n_tiles = (int)(a.S / net->TP);
    SavedPlan sp;
    plan_saved(net, a.S, sp);
    WsPlan wp;
    plan_ws(net, a.S, n_tiles, wp);
    char* ws = (char*)d_workspace;
    const char* sv = (const char*)d_saved;
    for (int l = 1; l < net->n_layers; ++l) {
        a.mask[l] = (const uint64_t*)(sv + sp.mask[l]);
        a.dz[l] = ws + wp.dz[l];
    }
    a.glast = (float*)(ws + wp.glast);
    a.dH_partial = (float*)(ws + wp.dH);
    a.d_coords = d_dcoords;
    if (a.geo.mode == MARF_GEO_COORDS && !d_dcoords) {
        // d coords not wanted: route them to the partial buffer is not possible -> use glast tail
        a.d_coords = nullptr;
    }
    {
        MarfProfScope ps("mlp_bwd_dgrad", s);
        HIPCHK(marf_launch_mlp_bwd(a, net->kdt, net->TP, net->lds_bwd, n_tiles, s), "backward dgrad");
    }

    if (d_dparams) {
        float* part = (float*)(ws + wp.part);
        float* bpart = (float*)(ws + wp.bpart);
        const int nl = net->n_layers;
        for (int l = 0; l < nl - 1; ++l) {
            {
                MarfProfScope ps(l == 0 ? "wgrad_l0" : "wgrad_hidden", s);
                HIPCHK(marf_launch_wgrad(net->kdt, ws + wp.dz[l + 1], net->Kp[l + 1], sv + sp.feat[l], net->Kp[l],
                                         a.S, net->Mp[l], net->Kp[l], wp.chunk, wp.n_chunks, part, bpart, s),
                       "backward wgrad");
            }
            {
                MarfProfScope ps("wgrad_reduce", s);
                HIPCHK(marf_launch_wgrad_reduce(part, bpart, wp.n_chunks, net->Mp[l], net->Kp[l], net->dims[l + 1],
                                                net->kin[l], d_dparams + net->w_off[l], d_dparams + net->b_off[l], s),
                       "backward wgrad reduce");
            }
        }
        const int l = nl - 1;
        {
            MarfProfScope ps("wgrad_last", s);
            HIPCHK(marf_launch_wgrad_last(net->kdt, a.glast, sv + sp.feat[l], a.S, net->Kp[l], net->Kp[l],
                                          wp.chunk_last, wp.n_chunks_last, part, bpart, s),
                   "backward wgrad last");
        }
        HIPCHK(marf_launch_wgrad_reduce(part, bpart, wp.n_chunks_last, 3, net->Kp[l], 3, net->dims[l],
                                        d_dparams + net->w_off[l], d_dparams + net->b_off[l], s),
               "backward wgrad last reduce");
    }
    if (a.geo.mode == MARF_GEO_GRID && d_dh) {
        MarfProfScope ps("warp_bwd", s);
        HIPCHK(marf_launch_reduce_dH(a.dH_partial, a.geo.Np_pad / net->TP, a.geo.B, d_h_params, nullptr, d_dh,
                                     lie_batch > 0 ? lie_batch : a.geo.B, s),
               "backward warp");
    }
    return MARF_OK;
}

// ------------------------------------------------------------------ fused training step

struct StepPlan {
    size_t feat[MARF_MAX_LAYERS], dz[MARF_MAX_LAYERS], mask[MARF_MAX_LAYERS];
    size_t wlast, blast, dH, loss, c2f, part, bpart, total;
    int n_tiles, chunk, n_chunks;
};

static void plan_step(const marf_net* n, long long S, StepPlan& p) {
    size_t off = 0;
    const int nl = n->n_layers;
    p.n_tiles = (int)(S / n->sTP);
    for (int l = 0; l < nl - 1; ++l) {
        p.feat[l] = off;
        off += rup((long long)S * n->Kp[l] * n->elem, 256);
    }
    p.dz[0] = p.mask[0] = 0;
    for (int l = 1; l < nl; ++l) {
        p.dz[l] = off;
        off += rup((long long)S * n->Kp[l] * n->elem, 256);
        p.mask[l] = off;
        off += rup(S / n->sTP * n->sNW * 1024, 256);  // one uint4 per lane per wave per tile
    }
    p.wlast = off;
    off += rup((long long)p.n_tiles * 3 * n->Kp[nl - 1] * 4, 256);
    p.blast = off;
    off += rup((long long)p.n_tiles * 3 * 4, 256);
    p.dH = off;
    off += rup((long long)p.n_tiles * 9 * 4, 256);
    p.loss = off;
    off += rup((long long)p.n_tiles * 2 * 8, 256);
    p.c2f = off;
    off += 256;
    long long chunk = rup((S + 255) / 256, 64);
    if (chunk < 64) chunk = 64;
    p.chunk = (int)chunk;
    p.n_chunks = (int)((S + chunk - 1) / chunk);
    long long mxo = 0, mxm = 0;
    for (int l = 0; l < nl - 1; ++l) {
        mxo = std::max(mxo, (long long)n->Mp[l] * n->Kp[l]);
        mxm = std::max(mxm, (long long)n->Mp[l]);
    }
    p.part = off;  // also the fold scratch of the last-layer reduction: 256 groups x (3 Kp + 3)
    off += rup(std::max((long long)p.n_chunks * mxo, 256LL * (3 * n->Kp[nl - 1] + 3)) * 4, 256);
    p.bpart = off;
    off += rup((long long)p.n_chunks * mxm * 4, 256);
    p.total = off;
}

// ---- the pixel-per-wave fused step (marf_step2.hip)

// a pipelined step (plan_pipe, below)
#define MARF_PIPE_MAXP 64
struct PipePlan {
    int on;
    int G, R, P;    // step-kernel blocks per piece, weight-gradient blocks per piece, pieces
    int piece;      // tiles per piece (the last one may have fewer)
    int wg_last;    // weight-gradient blocks of the last piece (every CU)
    int n_parts;    // split-K partials per layer: (P - 1) R + wg_last
};

struct Step2BufPlan {
    size_t feat[MARF_MAX_LAYERS], dz[MARF_MAX_LAYERS];
    size_t dH, loss, blast, wlast, dummy, c2f, kmap, part, bpart, total;
    size_t partl[MARF_MAX_LAYERS], bpartl[MARF_MAX_LAYERS];  // per-layer split-K partials (pipelined / fused)
    int grid, n_tiles;
    int nblk;  // per-block partial sets of the step kernel (all pieces' blocks)
    long long S;
    PipePlan pipe;
    bool fused_res;  // partl / bpartl reserved for the fused weight gradients (step2_backward takes
                     // that path only then)
};

// Can the fused weight gradients (marf_launch_wgrad_fused) run this net?  A superset of what
// marf_wgrad_fused_ok accepts (every hidden layer one 256 x 256 output block, the A/B switch
// MARF_WGRAD_FUSED not "0", read once per process so the buffer plan at allocation and at the
// backward agree): only then does plan_step2_bufs reserve every layer's partials at once.
static bool step2_fused_wgrad_possible(const marf_net* n) {
    static const bool env_off = [] {
        const char* e = getenv("MARF_WGRAD_FUSED");
        return e && e[0] == '0';
    }();
    if (env_off) return false;
    for (int l = 1; l < n->n_layers - 1; ++l)
        if (n->Mp[l] != 256 || n->Kp[l] != 256) return false;
    return true;
}

static int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        cus[dev] = c;
    }
    return cus[dev];
}

static bool use_step2(const marf_net* n) { return n->s2.variant >= 0; }

// split-K chunk of the weight gradients over S pixel slots (k_wgrad / k_wgrad_dma)
static long long wgrad_chunk(long long S) {
    long long chunk = rup((S + 255) / 256, 64);
    return chunk < 64 ? 64 : chunk;
}

// The layer-0 weight gradient recomputes feat_0 (grid -> warp -> posenc + c2f, bf16 hi) instead of
// reading it, so the step kernel does not store it (MARF_F0_RECOMPUTE=0: store and read, for A/B).
static bool l0_recompute(const marf_net* n, const GeoDev& g, long long S) {
    const char* e = getenv("MARF_F0_RECOMPUTE");
    if (e && e[0] == '0') return false;
    if ((n->s2.variant != 1 && n->s2.variant != 3) || g.mode != MARF_GEO_GRID) return false;
    const long long chunk = wgrad_chunk(S);
    return marf_wgrad_l0_recompute_ok(n->Mp[0], n->Kp[1], n->s2.ldf0, S, (int)chunk, (int)((S + chunk - 1) / chunk),
                                      g.Np_pad);
}

// ---- pipelined weight gradients (large steps of the pixel-per-wave kernel)
//
// The hidden / layer-0 weight gradients re-read the saved feat_l / dz_l: HBM-bound, about a fifth
// of the step when they follow the whole step kernel.  Their split-K partials do not depend on the
// upstream gradient (it scales the reduction), so they need not wait for the backward: the step
// kernel runs in pieces of whole tiles on G = CUs - R blocks (one per CU, persistent), and after
// each piece the R-block weight-gradient launches of its pixel rows go to a second stream, where
// they take the R CUs the step kernel leaves free (neither kernel fits beside the other on a CU:
// LDS), so the re-read of piece j overlaps the step of piece j + 1.  The last piece's weight
// gradients run on every CU.  Partial (piece j, block b) is j R + b: the reduction order is fixed
// and the result deterministic (it differs from the one-launch step by fp32 summation order only).

static void plan_pipe(const marf_net* n, const GeoDev& g, long long S, int n_tiles, PipePlan& pp) {
    memset(&pp, 0, sizeof(pp));
    const Step2NetPlan& q = n->s2;
    const int mode = n->pipe_mode;  // 0 off (default), 1 on at any size, -1 large steps only
    if (mode == 0 || q.variant < 0 || q.variant == 3 || g.mode != MARF_GEO_GRID) return;  // (fp16x2: not piecewise)
    const int cus = device_cus();
    int R = n->pipe_wg > 0 ? n->pipe_wg : std::max(1, cus * 7 / 64);  // 28 of 256 CUs
    R = std::max(1, std::min(R, cus / 2));
    const int G = cus - R;
    if (mode < 0 && n_tiles < 16 * cus) return;
    int piece = n->pipe_piece;
    if (piece <= 0) {  // about 8 pieces, each a whole number of tile groups per block
        const int k = std::max(1, (int)std::lround((double)n_tiles / (8.0 * q.NS * G)));
        piece = k * q.NS * G;
    }
    piece = (int)rup(piece, q.NS);
    int P = (n_tiles + piece - 1) / piece;
    if (P < 2) {
        if (mode != 1) return;
        piece = (int)rup((n_tiles + 1) / 2, q.NS);
        P = (n_tiles + piece - 1) / piece;
        if (P < 2) return;
    }
    if (P > MARF_PIPE_MAXP) return;
    // every weight gradient on the range-capable LDS-DMA kernel
    const int nl = n->n_layers;
    for (int l = 1; l < nl - 1; ++l)
        if (!marf_wgrad_range_ok(n->kdt, n->Mp[l], n->Kp[l + 1], n->Kp[l], n->Kp[l])) return;
    if (!marf_wgrad_range_ok(n->kdt, n->Mp[0], n->Kp[1], q.ldf0, q.ldf0)) return;
    if (l0_recompute(n, g, S)) {  // the recomputing kernel's ranges may span only a few patches
        const long long mx = rup((long long)piece * q.TPX / R + 32, 32);
        if (!marf_wgrad_l0_recompute_ok(n->Mp[0], n->Kp[1], q.ldf0, S, (int)mx, P * cus, g.Np_pad)) return;
    }
    pp.on = 1;
    pp.G = G;
    pp.R = R;
    pp.P = P;
    pp.piece = piece;
    pp.wg_last = cus;
    pp.n_parts = (P - 1) * R + cus;
}

// the second stream and the events of the pipeline, per device (created once); `use` is held by a
// caller across its whole record / wait sequence, so two host threads never interleave on the events
struct PipeStreams {
    hipStream_t s2;
    hipEvent_t ev[MARF_PIPE_MAXP + 1];
    std::mutex use;
};
static int pipe_streams(PipeStreams** out) {
    static std::mutex mu;
    static PipeStreams ps[64];
    int dev = 0;
    HIPCHK(hipGetDevice(&dev), "pipeline: hipGetDevice");
    if (dev < 0 || dev >= 64) return fail(MARF_ERR_UNSUPPORTED, "pipeline: device %d", dev);
    std::lock_guard<std::mutex> lk(mu);
    PipeStreams& p = ps[dev];
    if (!p.s2) {
        HIPCHK(hipStreamCreateWithFlags(&p.s2, hipStreamNonBlocking), "pipeline: stream");
        for (int i = 0; i <= MARF_PIPE_MAXP; ++i)
            HIPCHK(hipEventCreateWithFlags(&p.ev[i], hipEventDisableTiming), "pipeline: event");
    }
    *out = &p;
    return MARF_OK;
}

// render = a forward-only launch: no saved tensors, no dH / weight-gradient partials
static void plan_step2_bufs(const marf_net* n, const GeoDev& g, Step2BufPlan& p, bool render = false) {
    const Step2NetPlan& q = n->s2;
    const int nl = n->n_layers;
    const long long Ssave = render ? 0 : 1;
    p.S = (long long)g.B * g.Np_pad;
    p.n_tiles = (int)(p.S / q.TPX);
    int cap = device_cus();
    if (const char* e = getenv("MARF_STEP2_GRID")) cap = std::max(1, atoi(e));  // diagnostic override
    p.grid = std::max(1, std::min(p.n_tiles, cap));
    memset(&p.pipe, 0, sizeof(p.pipe));
    p.fused_res = false;
    if (!render) plan_pipe(n, g, p.S, p.n_tiles, p.pipe);
    if (p.pipe.on) p.grid = p.pipe.G;
    p.nblk = p.pipe.on ? p.pipe.P * p.pipe.G : p.grid;
    size_t off = 0;
    // (fp16x2: feat_l carries the 32 NW sink rows too -- a group's missing second set runs its
    //  forward and stores there)
    const long long Sfeat = p.S + (q.variant == 3 ? q.TPX : 0);
    for (int l = 0; l < nl - 1; ++l) {
        p.feat[l] = off;
        off += rup(Ssave * Sfeat * (l == 0 ? q.ldf0 : n->Kp[l]) * 2, 256);
    }
    p.dz[0] = 0;
    // dz_l and the dH partials carry 32 NW sink rows past S: the dgrad pass of a pixel set that has
    // no tile (an odd tile count with two sets per dgrad pass) stores there
    const long long Ssink = p.S + q.TPX;
    for (int l = 1; l < nl; ++l) {
        p.dz[l] = off;
        off += rup(Ssave * Ssink * n->Kp[l] * 2, 256);
    }
    p.dH = off;
    off += rup(Ssave * Ssink / q.PX * 9 * 4, 256);
    p.loss = off;
    off += rup((long long)p.nblk * 2 * 8, 256);
    p.blast = off;
    off += rup((long long)p.nblk * 3 * 4, 256);
    p.wlast = off;
    off += rup((long long)p.nblk * 3 * q.Kl * 4, 256);
    p.dummy = off;
    off += rup((long long)p.grid * q.NW * 4096, 256);  // 64 B per lane
    p.c2f = off;
    off += 256;
    p.kmap = off;  // the layer-0 column map, copied from the packed buffer by the forward
    off += rup((long long)n->D * 4, 256);
    // split-K partials of the hidden / layer-0 weight gradients (as plan_step)
    long long chunk = rup((p.S + 255) / 256, 64);
    if (chunk < 64) chunk = 64;
    const long long n_chunks = (p.S + chunk - 1) / chunk;
    long long mxo = 0, mxm = 0;
    for (int l = 0; l < nl - 1; ++l) {
        mxo = std::max(mxo, (long long)n->Mp[l] * (l == 0 ? q.ldf0 : n->Kp[l]));
        mxm = std::max(mxm, (long long)n->Mp[l]);
    }
    if (p.pipe.on) {  // every layer's partials live from the forward to the backward's reduction
        const long long np = p.pipe.n_parts;
        for (int l = 0; l < nl - 1; ++l) {
            p.partl[l] = off;
            off += rup(np * n->Mp[l] * (l == 0 ? q.ldf0 : n->Kp[l]) * 4, 256);
            p.bpartl[l] = off;
            off += rup(np * n->Mp[l] * 4, 256);
        }
        p.part = off;  // the fold scratch of the last-layer reduction
        off += rup(256LL * (3 * q.Kl + 3) * 4, 256);
        p.bpart = 0;
    } else {
        p.part = off;
        off += rup(Ssave * std::max(n_chunks * mxo, 256LL * (3 * q.Kl + 3)) * 4, 256);
        p.bpart = off;
        off += rup(Ssave * n_chunks * mxm * 4, 256);
        // the fused weight gradients keep every layer's partials at once (layer 0: part); the
        // per-layer path reuses part / bpart for every layer, so nothing more is reserved for it
        p.fused_res = !render && step2_fused_wgrad_possible(n);
        p.partl[0] = p.part;
        p.bpartl[0] = p.bpart;
        for (int l = 1; l < nl - 1; ++l) {
            p.partl[l] = p.part;
            p.bpartl[l] = p.bpart;
            if (!p.fused_res) continue;
            p.partl[l] = off;
            off += rup(Ssave * n_chunks * n->Mp[l] * n->Kp[l] * 4, 256);
            p.bpartl[l] = off;
            off += rup(Ssave * n_chunks * n->Mp[l] * 4, 256);
        }
    }
    p.total = off;
}

// the weight-gradient launches of piece j of a pipelined step (second stream)
static int wgrad_piece(const marf_net* net, const GeoDev& g, const Step2BufPlan& p, char* sv, int j, hipStream_t s2) {
    const Step2NetPlan& q = net->s2;
    const PipePlan& pp = p.pipe;
    const int nl = net->n_layers;
    const long long TPX = q.TPX;
    const long long t0 = (long long)j * pp.piece, t1 = std::min<long long>(p.n_tiles, t0 + pp.piece);
    WgRange r;
    r.s_lo = t0 * TPX;
    r.s_len = (t1 - t0) * TPX;
    r.n = j == pp.P - 1 ? pp.wg_last : pp.R;
    r.part0 = j * pp.R;
    const bool f0 = l0_recompute(net, g, p.S);
    for (int l = 0; l < nl - 1; ++l) {
        const int K = l == 0 ? q.ldf0 : net->Kp[l];
        float* part = (float*)(sv + p.partl[l]);
        float* bpart = (float*)(sv + p.bpartl[l]);
        MarfProfScope ps(l == 0 ? "wgrad_l0" : "wgrad_hidden", s2);
        if (l == 0 && f0)
            HIPCHK(marf_launch_wgrad_l0_recompute(sv + p.dz[1], net->Kp[1], g, (const float*)(sv + p.c2f), net->L, q.nk0w,
                                                  q.ldf0, p.S, net->Mp[0], 32, r.n, part, bpart, s2, &r),
                   "step_forward pipelined wgrad_l0");
        else
            HIPCHK(marf_launch_wgrad(1, sv + p.dz[l + 1], net->Kp[l + 1], sv + p.feat[l], K, p.S, net->Mp[l], K, 32, r.n,
                                     part, bpart, s2, &r, true),
                   "step_forward pipelined wgrad");
    }
    return MARF_OK;
}

static hipError_t launch_s2(const marf_net* n, const Step2Args& a, int grid, hipStream_t s) {
    const Step2NetPlan& q = n->s2;
    // the compile-time layer-0 instantiations: split recipe, every hidden layer 256 wide, the
    // layer-0 row tiles per stage the kernel derives from nk0, a 256-wide last-layer input
    bool full = (q.variant == 1 || q.variant == 3) && q.nk0 >= 1 && q.r0 == std::max(1, std::min(8, 16 / q.nk0)) && q.Kl == 256;
    for (int l = 0; l < n->n_layers - 1; ++l) full = full && n->Mp[l] == 256;
    if (const char* e = getenv("MARF_STEP2_GENERIC")) full = full && e[0] != '1';  // (A/B: the generic kernel)
    return marf_launch_step2(a, q.variant, grid, s, full ? q.nk0 : 0, q.dz);
}

static int step2_forward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                         const float* d_gt, const float* d_mask, const float* d_denom_override, float* d_rgb,
                         float* d_loss_out, void* d_saved, hipStream_t s, bool render = false) {
    const Step2NetPlan& q = net->s2;
    Step2Args a;
    memset(&a, 0, sizeof(a));
    int rc = make_geo(geo, a.geo, q.TPX);
    if (rc) return rc;
    Step2BufPlan p;
    plan_step2_bufs(net, a.geo, p, render);
    char* sv = (char*)d_saved;
    const char* pk = (const char*)d_packed;
    const int nl = net->n_layers;
    a.nl = nl;
    a.L = net->L;
    a.nk0 = q.nk0;
    a.nta = q.nta;
    a.r0 = q.r0;
    C2fDev cf = make_c2f(c2f);
    a.c2f_on = cf.on;
    a.prog = pk + q.prog_off;
    a.n_stages = q.n_stages;
    // the program's forward prefix: the layer-0 and hidden row tiles + the last layer
    a.n_fwd = q.n_fwd;
    a.S = p.S;
    if (render) {
        a.fwd_only = 1;
        a.n_stages = a.n_fwd;
        a.pro_fallback = a.geo.mode == MARF_GEO_COORDS ? a.geo.coords : a.geo.Hm;
    }
    a.bias = (const float*)(pk + q.bias_off);
    a.nbias = q.nbias;
    a.feat0_recompute = !render && l0_recompute(net, a.geo, p.S) ? 1 : 0;
    a.gt = d_gt;
    a.mask = d_mask;
    a.rgb = d_rgb;
    for (int l = 0; l < nl; ++l) {
        S2Layer& y = a.layers[l];
        y.nrt = q.nrt[l];
        y.nrtb = q.nrtb[l];
        y.boff = q.boff[l];
        y.ldf = l == 0 ? q.ldf0 : net->Kp[l];
        y.ldz = net->Kp[l];
        y.feat = l < nl - 1 && !render ? (u16*)(sv + p.feat[l]) : nullptr;
        y.dz = l >= 1 && !render ? (u16*)(sv + p.dz[l]) : nullptr;
    }
    a.dH_partial = (float*)(sv + p.dH);
    a.loss_partial = (double*)(sv + p.loss);
    a.blast_partial = (float*)(sv + p.blast);
    a.wlast_partial = (float*)(sv + p.wlast);
    a.Kl = q.Kl;
    a.c2f_w = (const float*)(sv + p.c2f);
    a.dummy = (float*)(sv + p.dummy);
    a.stamps = g_stamps;
    a.n_tiles = p.n_tiles;
    // LDS layout
    const int TPX = q.TPX;
    int off = q.nslot * q.slot;
    a.lds_pro = off;
    // input buffers: two of (targets + mask + H) per tile; fp16x2: four H rows + two target sets
    off += q.variant == 3 ? 1024 + 2 * 4 * TPX * 4 : 2 * (4 * TPX + 64) * 4;
    a.lds_bias = off;
    off += (int)rup(q.nbias * 4, 16);
    a.lds_c2f = off;
    off += 128;
    a.lds_layers = off;
    off += (int)sizeof(S2Layer) * MARF_MAX_LAYERS;
    a.lds_wave = off;
    // per wave: transpose + g^T scratch, ReLU mask words of each pixel set of a dgrad pass, dW_last
    a.lds_wave_bytes = (int)rup(2048 + q.NS * q.MAXR * q.NMW * 256 + 12 * q.Kl, 16);
    off += q.NW * a.lds_wave_bytes;
    a.lds_total = off;
    if (off > 160 * 1024) return fail(MARF_ERR_UNSUPPORTED, "step2: LDS plan %d B exceeds 160 KB", off);
    // the band weights and the layer-0 column map (packed buffer -> saved buffer) in one launch
    HIPCHK(marf_launch_c2f_weights(cf, net->L, (float*)(sv + p.c2f), s, (const int*)(pk + q.kmap_off),
                                   (int*)(sv + p.kmap), net->D),
           "step_forward c2f / kmap");
    if (render) {
        MarfProfScope ps("mlp_fwd", s);
        HIPCHK(launch_s2(net, a, p.grid, s), "render step2");
        return MARF_OK;
    }
    double* const loss0 = a.loss_partial;
    if (!p.pipe.on) {
        MarfProfScope ps("mlp_step", s);
        HIPCHK(launch_s2(net, a, p.grid, s), "step_forward step2");
    } else {
        // pieces of the step kernel on stream s, each followed by its weight gradients on s2
        const PipePlan& pp = p.pipe;
        PipeStreams* st = nullptr;
        rc = pipe_streams(&st);
        if (rc) return rc;
        std::lock_guard<std::mutex> hold(st->use);
        float* const blast0 = a.blast_partial;
        float* const wlast0 = a.wlast_partial;
        for (int j = 0; j < pp.P; ++j) {
            a.tile0 = j * pp.piece;
            a.n_tiles = std::min(p.n_tiles, (j + 1) * pp.piece);
            a.loss_partial = loss0 + (size_t)j * pp.G * 2;
            a.blast_partial = blast0 + (size_t)j * pp.G * 3;
            a.wlast_partial = wlast0 + (size_t)j * pp.G * 3 * q.Kl;
            {
                MarfProfScope ps("mlp_step", s);
                HIPCHK(launch_s2(net, a, pp.G, s), "step_forward step2 piece");
            }
            HIPCHK(hipEventRecord(st->ev[j], s), "pipeline: record");
            HIPCHK(hipStreamWaitEvent(st->s2, st->ev[j], 0), "pipeline: wait");
            rc = wgrad_piece(net, a.geo, p, sv, j, st->s2);
            if (rc) return rc;
        }
        HIPCHK(hipEventRecord(st->ev[MARF_PIPE_MAXP], st->s2), "pipeline: record");
        HIPCHK(hipStreamWaitEvent(s, st->ev[MARF_PIPE_MAXP], 0), "pipeline: join");
    }
    {
        MarfProfScope ps("loss_final", s);
        HIPCHK(marf_launch_loss_final(loss0, p.nblk, d_loss_out, d_denom_override, s), "step_forward loss");
    }
    return MARF_OK;
}

// record layer l's "gradient final" event, if the caller passed one
static int mark_layer(const void* const* ev, int l, hipStream_t s) {
    if (ev && ev[l]) HIPCHK(hipEventRecord((hipEvent_t)ev[l], s), "step_backward: layer event");
    return MARF_OK;
}

static int step2_backward(const marf_net* net, const marf_geometry* geo, const void* d_saved,
                          const float* d_h_params, int lie_batch, const float* d_gout, const float* d_loss_out,
                          float* d_dparams, float* d_dh, hipStream_t s, const void* const* ev) {
    const Step2NetPlan& q = net->s2;
    GeoDev g;
    int rc = make_geo(geo, g, q.TPX);
    if (rc) return rc;
    Step2BufPlan p;
    plan_step2_bufs(net, g, p);
    const char* sv = (const char*)d_saved;
    float* part = (float*)(sv + p.part);
    float* bpart = (float*)(sv + p.bpart);
    const float* denom = d_loss_out + 1;
    const int nl = net->n_layers;
    // the saved tensors' precision (fp16x2: fp16, carrying the dgrad's 2^10 gradient scale)
    const int sdt = q.variant == 3 ? 2 : 1;
    const float post = q.variant == 3 ? 1.0f / 1024.0f : 1.0f;
    // The fused weight gradients (marf_launch_wgrad_fused): the hidden layers in one launch, layer 0
    // beside it on the side stream, every reduction in one launch -- the same partials and sums as
    // the per-layer launches below (bit-identical).  The layer events follow it, in the per-layer order.
    if (d_dparams && !p.pipe.on && p.fused_res) {
        const long long chunk = wgrad_chunk(p.S);
        const int n_chunks = (int)((p.S + chunk - 1) / chunk);
        const int* kmap = (const int*)(sv + p.kmap);
        const bool f0 = l0_recompute(net, g, p.S);
        WgFusedLayer Lf[MARF_MAX_LAYERS];
        memset(Lf, 0, sizeof(Lf));
        int nf = 0;
        {
            const int l = nl - 1;  // the last layer: the step kernel's per-block partials
            WgFusedLayer& x = Lf[nf++];
            x.kind = 3;
            x.partial = (float*)(sv + p.wlast);
            x.bpartial = (float*)(sv + p.blast);
            x.n_parts = p.nblk;
            x.M = 3;
            x.K = q.Kl;
            x.Mo = 3;
            x.Ko = net->dims[l];
            x.dW = d_dparams + net->w_off[l];
            x.db = d_dparams + net->b_off[l];
        }
        for (int l = nl - 2; l >= 0; --l) {
            WgFusedLayer& x = Lf[nf++];
            x.kind = l > 0 ? 0 : (f0 ? 1 : 2);
            x.dz = sv + p.dz[l + 1];
            x.ldz = net->Kp[l + 1];
            x.feat = (l == 0 && f0) ? nullptr : sv + p.feat[l];
            x.ldf = x.K = l == 0 ? q.ldf0 : net->Kp[l];
            x.M = net->Mp[l];
            x.partial = (float*)(sv + p.partl[l]);
            x.bpartial = (float*)(sv + p.bpartl[l]);
            x.n_parts = n_chunks;
            x.Mo = net->dims[l + 1];
            x.Ko = net->dims[l];
            x.dW = d_dparams + net->w_off[l];
            x.db = d_dparams + net->b_off[l];
            x.kmap = l == 0 ? kmap : nullptr;
        }
        if (marf_wgrad_fused_ok(Lf, nf, p.S, (int)chunk, n_chunks, g.Np_pad)) {
            PipeStreams* st = nullptr;
            rc = pipe_streams(&st);
            if (rc) return rc;
            {
                std::lock_guard<std::mutex> hold(st->use);
                const char* dse = getenv("MARF_DH_SIDE");  // A/B switch (per launch): 0 = after the reductions on s
                float* dh_side = (dse && dse[0] == '0') ? nullptr : d_dh;
                if (dh_side) {  // s2 joins the step here (the fused launch forks it again for layer 0)
                    HIPCHK(hipEventRecord(st->ev[2], s), "step_backward: fork");
                    HIPCHK(hipStreamWaitEvent(st->s2, st->ev[2], 0), "step_backward: fork");
                }
                {
                    MarfProfScope ps("wgrad_fused", s);
                    HIPCHK(marf_launch_wgrad_fused(Lf, nf, p.S, (int)chunk, n_chunks, g, (const float*)(sv + p.c2f),
                                                   net->L, q.nk0w, d_gout, denom, s, st->s2, st->ev[0], st->ev[1], sdt, post),
                           "step_backward fused weight gradients");
                }
                if (dh_side) {
                    // the warp gradient (one block: the dH partials' fixed-order sum + the Lie
                    // backward) reads only the step kernel's partials and the upstream gradient: it
                    // follows layer 0 on the side stream (ahead of it, it would hold layer 0 back
                    // until the hidden layers free a CU) and runs beside the reductions
                    MarfProfScope ps("warp_bwd_side", st->s2);
                    HIPCHK(marf_launch_reduce_dH((const float*)(sv + p.dH), g.Np_pad / q.PX, g.B, d_h_params, nullptr,
                                                 dh_side, lie_batch > 0 ? lie_batch : g.B, st->s2, d_gout, denom),
                           "step_backward warp");
                    HIPCHK(hipEventRecord(st->ev[3], st->s2), "step_backward: join");
                }
                for (int l = nl - 1; l >= 0; --l) {  // (ahead of the warp gradient's join: the
                    rc = mark_layer(ev, l, s);        //  layers' all-reduces do not wait for it)
                    if (rc) return rc;
                }
                if (dh_side) {
                    HIPCHK(hipStreamWaitEvent(s, st->ev[3], 0), "step_backward: join");
                    d_dh = nullptr;
                }
            }
            d_dparams = nullptr;  // done
        }
    }
    // the layers finish in reverse order (last layer first, layer 0 last), each marked by its event,
    // so that a bucketed all-reduce of finished layers overlaps the remaining weight gradients
    if (d_dparams) {
        const int l = nl - 1;
        MarfProfScope ps("wgrad_last_reduce", s);
        HIPCHK(marf_launch_wgrad_reduce((const float*)(sv + p.wlast), (const float*)(sv + p.blast), p.nblk, 3, q.Kl, 3,
                                        net->dims[l], d_dparams + net->w_off[l], d_dparams + net->b_off[l], s, d_gout,
                                        denom, part),
               "step_backward last reduce");
        rc = mark_layer(ev, l, s);
        if (rc) return rc;
    }
    if (d_dparams && p.pipe.on) {  // the split-K partials were computed beside the step kernel
        const int* kmap = (const int*)(sv + p.kmap);
        for (int l = nl - 2; l >= 0; --l) {
            const int K = l == 0 ? q.ldf0 : net->Kp[l];
            MarfProfScope ps("wgrad_reduce", s);
            HIPCHK(marf_launch_wgrad_reduce((const float*)(sv + p.partl[l]), (const float*)(sv + p.bpartl[l]),
                                            p.pipe.n_parts, net->Mp[l], K, net->dims[l + 1], net->dims[l],
                                            d_dparams + net->w_off[l], d_dparams + net->b_off[l], s, d_gout, denom,
                                            nullptr, l == 0 ? kmap : nullptr),
                   "step_backward wgrad reduce (pipelined)");
            rc = mark_layer(ev, l, s);
            if (rc) return rc;
        }
    } else if (d_dparams) {
        const long long chunk = wgrad_chunk(p.S);
        const int n_chunks = (int)((p.S + chunk - 1) / chunk);
        const int* kmap = (const int*)(sv + p.kmap);
        const bool f0 = l0_recompute(net, g, p.S);
        for (int l = nl - 2; l >= 0; --l) {
            const int K = l == 0 ? q.ldf0 : net->Kp[l];
            {
                MarfProfScope ps(l == 0 ? "wgrad_l0" : "wgrad_hidden", s);
                if (l == 0 && f0)
                    HIPCHK(marf_launch_wgrad_l0_recompute(sv + p.dz[1], net->Kp[1], g, (const float*)(sv + p.c2f), net->L,
                                                          q.nk0w, q.ldf0, p.S, net->Mp[0], (int)chunk, n_chunks, part, bpart, s,
                                                          nullptr, sdt),
                           "step_backward wgrad_l0 (feat_0 recomputed)");
                else
                    HIPCHK(marf_launch_wgrad(sdt, sv + p.dz[l + 1], net->Kp[l + 1], sv + p.feat[l], K, p.S, net->Mp[l], K,
                                             (int)chunk, n_chunks, part, bpart, s, nullptr, true),
                           "step_backward wgrad");
            }
            {
                MarfProfScope ps("wgrad_reduce", s);
                HIPCHK(marf_launch_wgrad_reduce(part, bpart, n_chunks, net->Mp[l], K, net->dims[l + 1], net->dims[l],
                                                d_dparams + net->w_off[l], d_dparams + net->b_off[l], s, d_gout, denom,
                                                nullptr, l == 0 ? kmap : nullptr, post),
                       "step_backward wgrad reduce");
            }
            rc = mark_layer(ev, l, s);
            if (rc) return rc;
        }
    }
    if (d_dh) {
        MarfProfScope ps("warp_bwd", s);
        HIPCHK(marf_launch_reduce_dH((const float*)(sv + p.dH), g.Np_pad / q.PX, g.B, d_h_params, nullptr, d_dh,
                                     lie_batch > 0 ? lie_batch : g.B, s, d_gout, denom),
               "step_backward warp");
    }
    return MARF_OK;
}

size_t marf_render_workspace_bytes(const marf_net* net, const marf_geometry* geo) {
    if (!net || !geo || !use_step2(net)) return 0;
    GeoDev g;
    if (make_geo(geo, g, net->s2.TPX) != MARF_OK) return 0;
    Step2BufPlan p;
    plan_step2_bufs(net, g, p, true);
    return p.total;
}

int marf_render(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed, float* d_rgb,
                void* d_ws, void* stream) {
    if (!net || !geo || !d_packed || !d_rgb) return fail(MARF_ERR_INVALID, "render: NULL argument");
    if (!use_step2(net)) return marf_forward(net, geo, c2f, d_packed, d_rgb, nullptr, stream);
    if (!d_ws) return fail(MARF_ERR_INVALID, "render: workspace (marf_render_workspace_bytes) missing");
    if (geo->mode == MARF_GEO_GRID || geo->mode == MARF_GEO_CANVAS) {
        if (!geo->d_H) return fail(MARF_ERR_INVALID, "render: grid geometry needs d_H");
    } else if (geo->mode == MARF_GEO_COORDS) {
        if (geo->Np <= 0 || !geo->d_coords) return fail(MARF_ERR_INVALID, "render: coords geometry needs points");
    }
    return step2_forward(net, geo, c2f, d_packed, nullptr, nullptr, nullptr, d_rgb, nullptr, d_ws,
                         (hipStream_t)stream, true);
}

size_t marf_step_saved_bytes(const marf_net* net, const marf_geometry* geo) {
    GeoDev g;
    if (!net || !geo || geo->mode == MARF_GEO_COORDS) return 0;
    if (use_step2(net)) {
        if (make_geo(geo, g, net->s2.TPX) != MARF_OK) return 0;
        Step2BufPlan p2;
        plan_step2_bufs(net, g, p2);
        return p2.total;
    }
    if (make_geo(geo, g, MARF_TILE_PAD) != MARF_OK) return 0;
    StepPlan p;
    plan_step(net, (long long)g.B * g.Np_pad, p);
    return p.total;
}

int marf_step_forward(const marf_net* net, const marf_geometry* geo, const marf_c2f* c2f, const void* d_packed,
                      const float* d_gt, const float* d_mask, const float* d_denom_override, float* d_rgb,
                      float* d_loss_out, void* d_saved, void* stream) {
    if (!net || !d_packed || !d_gt || !d_loss_out || !d_saved) return fail(MARF_ERR_INVALID, "step_forward: NULL argument");
    if (!geo || geo->mode == MARF_GEO_COORDS) return fail(MARF_ERR_INVALID, "step_forward: needs a pixel-grid geometry");
    hipStream_t s = (hipStream_t)stream;
    if (use_step2(net))
        return step2_forward(net, geo, c2f, d_packed, d_gt, d_mask, d_denom_override, d_rgb, d_loss_out, d_saved, s);
    StepArgs a;
    memset(&a, 0, sizeof(a));
    int rc = make_geo(geo, a.geo, MARF_TILE_PAD);
    if (rc) return rc;
    fill_netdev(net, d_packed, a.net);
    a.c2f = make_c2f(c2f);
    a.rgb = d_rgb;
    a.gt = d_gt;
    a.mask = d_mask;
    a.S = (long long)a.geo.B * a.geo.Np_pad;
    a.lda = net->lda;
    StepPlan p;
    plan_step(net, a.S, p);
    char* sv = (char*)d_saved;
    const int nl = net->n_layers;
    for (int l = 0; l < nl - 1; ++l) a.feat[l] = sv + p.feat[l];
    for (int l = 1; l < nl; ++l) {
        a.dz[l] = sv + p.dz[l];
        a.mask_bits[l] = (uint64_t*)(sv + p.mask[l]);
    }
    a.wlast_partial = (float*)(sv + p.wlast);
    a.blast_partial = (float*)(sv + p.blast);
    a.dH_partial = (float*)(sv + p.dH);
    a.loss_partial = (double*)(sv + p.loss);
    a.c2f_w = (const float*)(sv + p.c2f);
    a.stamps = g_stamps;
    if (net->L > 0) HIPCHK(marf_launch_c2f_weights(a.c2f, net->L, (float*)(sv + p.c2f), s), "step_forward c2f");
    {
        MarfProfScope ps("mlp_step", s);
        HIPCHK(marf_launch_mlp_step(a, net->kdt, net->sTP, net->sNW, net->lds_step, p.n_tiles, s), "step_forward");
    }
    {
        MarfProfScope ps("loss_final", s);
        HIPCHK(marf_launch_loss_final(a.loss_partial, p.n_tiles, d_loss_out, d_denom_override, s), "step_forward loss");
    }
    return MARF_OK;
}

int marf_step_backward(const marf_net* net, const marf_geometry* geo, const void* d_saved, const float* d_h_params,
                       int lie_batch, const float* d_gout, const float* d_loss_out, float* d_dparams, float* d_dh,
                       void* stream) {
    return marf_step_backward_ev(net, geo, d_saved, d_h_params, lie_batch, d_gout, d_loss_out, d_dparams, d_dh, nullptr,
                                 stream);
}

int marf_step_backward_ev(const marf_net* net, const marf_geometry* geo, const void* d_saved, const float* d_h_params,
                          int lie_batch, const float* d_gout, const float* d_loss_out, float* d_dparams, float* d_dh,
                          void* const* layer_events, void* stream) {
    const void* const* ev = (const void* const*)layer_events;
    if (!net || !d_saved || !d_gout || !d_loss_out) return fail(MARF_ERR_INVALID, "step_backward: NULL argument");
    if (!geo || geo->mode == MARF_GEO_COORDS) return fail(MARF_ERR_INVALID, "step_backward: needs a pixel-grid geometry");
    if (d_dh && !d_h_params) return fail(MARF_ERR_INVALID, "step_backward: d_dh requested without the warp parameters");
    hipStream_t s = (hipStream_t)stream;
    if (use_step2(net))
        return step2_backward(net, geo, d_saved, d_h_params, lie_batch, d_gout, d_loss_out, d_dparams, d_dh, s, ev);
    GeoDev g;
    int rc = make_geo(geo, g, MARF_TILE_PAD);
    if (rc) return rc;
    const long long S = (long long)g.B * g.Np_pad;
    StepPlan p;
    plan_step(net, S, p);
    const char* sv = (const char*)d_saved;
    float* part = (float*)(sv + p.part);
    float* bpart = (float*)(sv + p.bpart);
    const float* denom = d_loss_out + 1;
    const int nl = net->n_layers;
    if (d_dparams) {  // last layer first, then l = nl-2 .. 0, each marked by its event (as step2_backward)
        {
            const int l = nl - 1;
            MarfProfScope ps("wgrad_last_reduce", s);
            HIPCHK(marf_launch_wgrad_reduce((const float*)(sv + p.wlast), (const float*)(sv + p.blast), p.n_tiles, 3,
                                            net->Kp[l], 3, net->dims[l], d_dparams + net->w_off[l],
                                            d_dparams + net->b_off[l], s, d_gout, denom, part),
                   "step_backward last reduce");
            rc = mark_layer(ev, l, s);
            if (rc) return rc;
        }
        for (int l = nl - 2; l >= 0; --l) {
            {
                MarfProfScope ps(l == 0 ? "wgrad_l0" : "wgrad_hidden", s);
                HIPCHK(marf_launch_wgrad(net->kdt, sv + p.dz[l + 1], net->Kp[l + 1], sv + p.feat[l], net->Kp[l], S,
                                         net->Mp[l], net->Kp[l], p.chunk, p.n_chunks, part, bpart, s),
                       "step_backward wgrad");
            }
            {
                MarfProfScope ps("wgrad_reduce", s);
                HIPCHK(marf_launch_wgrad_reduce(part, bpart, p.n_chunks, net->Mp[l], net->Kp[l], net->dims[l + 1],
                                                net->kin[l], d_dparams + net->w_off[l], d_dparams + net->b_off[l], s,
                                                d_gout, denom),
                       "step_backward wgrad reduce");
            }
            rc = mark_layer(ev, l, s);
            if (rc) return rc;
        }
    }
    if (d_dh) {
        MarfProfScope ps("warp_bwd", s);
        HIPCHK(marf_launch_reduce_dH((const float*)(sv + p.dH), g.Np_pad / net->sTP, g.B, d_h_params, nullptr, d_dh,
                                     lie_batch > 0 ? lie_batch : g.B, s, d_gout, denom),
               "step_backward warp");
    }
    return MARF_OK;
}

// ------------------------------------------------------------------ loss / optimizer

size_t marf_mse_workspace_bytes(void) { return 1024 * 2 * sizeof(double); }

int marf_masked_mse(const float* d_pred, const float* d_gt, const float* d_mask, int B, int Np,
                    const float* d_denom_override, float* d_out, void* d_ws, void* stream) {
    if (B <= 0 || Np <= 0 || !d_pred || !d_gt || !d_out || !d_ws) return fail(MARF_ERR_INVALID, "masked_mse: bad args");
    MarfProfScope ps("loss_fwd", (hipStream_t)stream);
    HIPCHK(marf_launch_mse(d_pred, d_gt, d_mask, B, Np, (double*)d_ws, d_out, d_denom_override, (hipStream_t)stream),
           "masked_mse");
    return MARF_OK;
}

int marf_masked_mse_backward(const float* d_pred, const float* d_gt, const float* d_mask, int B, int Np,
                             const float* d_denom, const float* d_gout, float* d_dpred, void* stream) {
    if (B <= 0 || Np <= 0 || !d_pred || !d_gt || !d_denom || !d_gout || !d_dpred)
        return fail(MARF_ERR_INVALID, "masked_mse_backward: bad args");
    MarfProfScope ps("loss_bwd", (hipStream_t)stream);
    HIPCHK(marf_launch_mse_bwd(d_pred, d_gt, d_mask, B, Np, d_denom, d_gout, d_dpred, (hipStream_t)stream),
           "masked_mse_backward");
    return MARF_OK;
}

int marf_edge_map(const float* d_img, int n_img, int H, int W, double* d_out, void* stream) {
    if (n_img < 0 || H <= 0 || W <= 0 || (n_img > 0 && (!d_img || !d_out))) return fail(MARF_ERR_INVALID, "edge_map: bad args");
    if (n_img > 65535) return fail(MARF_ERR_INVALID, "edge_map: more than 65535 channel images");
    if (n_img == 0) return MARF_OK;
    MarfProfScope ps("edge_map", (hipStream_t)stream);
    HIPCHK(marf_launch_edge_map(d_img, d_out, n_img, H, W, (hipStream_t)stream), "edge_map");
    return MARF_OK;
}

int marf_erode_rect(const float* d_img, int n_img, int H, int W, int kh, int kw, float* d_out, void* stream) {
    if (n_img < 0 || H <= 0 || W <= 0 || kh <= 0 || kw <= 0 || (n_img > 0 && (!d_img || !d_out)))
        return fail(MARF_ERR_INVALID, "erode_rect: bad args");
    if (n_img > 65535) return fail(MARF_ERR_INVALID, "erode_rect: more than 65535 channel images");
    if (d_img == d_out) return fail(MARF_ERR_INVALID, "erode_rect: in-place erosion is not supported");
    if (n_img == 0) return MARF_OK;
    HIPCHK(marf_launch_erode_rect(d_img, d_out, n_img, H, W, kh, kw, (hipStream_t)stream), "erode_rect");
    return MARF_OK;
}

}  // extern "C"

// torch.optim.Adam's per-step scalars: bias corrections in python float64, step_size = lr / bc1,
// bc2 ** 0.5, handed to the kernel as float
static void adam_scalars(double lr, double beta1, double beta2, long long step, float& step_size, float& bc2_sqrt) {
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    step_size = (float)(lr / bc1);
    bc2_sqrt = (float)std::sqrt(bc2);
}

extern "C" {

int marf_adam_step(float* d_p, const float* d_g, float* d_m, float* d_v, long long n, double lr, double beta1,
                   double beta2, double eps, long long step, const float* d_grad_scale, void* stream) {
    if (n < 0 || step < 1 || (n > 0 && (!d_p || !d_g || !d_m || !d_v))) return fail(MARF_ERR_INVALID, "adam: bad args");
    float step_size, bc2_sqrt;
    adam_scalars(lr, beta1, beta2, step, step_size, bc2_sqrt);
    MarfProfScope ps("adam", (hipStream_t)stream);
    HIPCHK(marf_launch_adam(d_p, d_g, d_m, d_v, n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                            step_size, bc2_sqrt, (float)eps, d_grad_scale, (hipStream_t)stream),
           "adam");
    return MARF_OK;
}

int marf_adam_schedule(double lr, double beta1, double beta2, long long first_step, long long count, float* h_out) {
    if (first_step < 1 || count < 0 || (count > 0 && !h_out)) return fail(MARF_ERR_INVALID, "adam_schedule: bad args");
    for (long long i = 0; i < count; ++i) adam_scalars(lr, beta1, beta2, first_step + i, h_out[2 * i], h_out[2 * i + 1]);
    return MARF_OK;
}

int marf_adam_step_sched(float* d_p, const float* d_g, float* d_m, float* d_v, long long n, double beta1, double beta2,
                         double eps, const float* d_sched, const int* d_index, const float* d_grad_scale, void* stream) {
    if (n < 0 || (n > 0 && (!d_p || !d_g || !d_m || !d_v || !d_sched || !d_index)))
        return fail(MARF_ERR_INVALID, "adam_step_sched: bad args");
    MarfProfScope ps("adam", (hipStream_t)stream);
    HIPCHK(marf_launch_adam_sched(d_p, d_g, d_m, d_v, n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                                  d_sched, d_index, (float)eps, d_grad_scale, (hipStream_t)stream),
           "adam_step_sched");
    return MARF_OK;
}

}  // extern "C"
