"""oracle.py -- CPU restatement of the reference's planar BA training step.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / CPU baseline.
The product (masking-bundle-adjusting-neural-radiance-fields_amd/) never imports it.

numpy (fp32 arithmetic, BLAS sgemm for the MLP) on top of the plain-C prologue in
marf_oracle.c (bit-exact grid / Lie exp / warp).  Every function cites the reference
file:line it restates; parity of this restatement with the reference is pinned by
tests/test_oracle_golden.py against fixtures generated from the reference itself
(tests/golden/make_golden.py).

Reference step (model/planar.py:187-209 + :154-158):
    zero_grad; Graph.forward (:329-336) -> Graph.compute_loss (:355-380)
    -> Model.summarize_loss (:172-185) -> backward -> Adam.step
    -> progress = it/max_iter (:208) -> warp_param[0] = 0 if fix_first (:157-158)
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libmarf_oracle.so")
_lib = None
_FP = ctypes.POINTER(ctypes.c_float)
_DP = ctypes.POINTER(ctypes.c_double)


def lib():
    """Load (building with gcc if needed) the C half of the oracle."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _f(a):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_FP)


def _d(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_DP)


# ------------------------------------------------------------------ Lie / warp

def sl3_to_SL3(h):
    """Lie.sl3_to_SL3, warp.py:98-106 (torch matrix_exp, fp32, batch-dependent path)."""
    h = np.ascontiguousarray(h, np.float32).reshape(-1, 8)
    H = np.zeros((h.shape[0], 3, 3), np.float32)
    lib().oracle_sl3_to_SL3(_f(h), _f(H), ctypes.c_int(h.shape[0]))
    return H


def sl3_to_SL3_backward(h, dH):
    """Autograd of sl3_to_SL3: matrix_exp backward + generator adjoint."""
    h = np.ascontiguousarray(h, np.float32).reshape(-1, 8)
    dH = np.ascontiguousarray(dH, np.float32).reshape(-1, 3, 3)
    dh = np.zeros_like(h)
    lib().oracle_sl3_to_SL3_backward(_f(h), _f(dH), _f(dh), ctypes.c_int(h.shape[0]))
    return dh


def expm(A):
    """torch.linalg.matrix_exp restatement for a batch [n_batch, n, n] (n <= 6)."""
    A = np.ascontiguousarray(A, np.float32)
    E = np.zeros_like(A)
    lib().oracle_expm(_f(A), _f(E), ctypes.c_int(A.shape[-1]), ctypes.c_int(A.shape[0]))
    return E


def pixel_grid(H, W, ph, pw, crop=True):
    """Warp.get_normalized_pixel_grid, warp.py:33-68 (one copy; the reference
    repeats it B times).  Returns [h*w, 2] (x, y), row-major pixels."""
    if crop:
        h = (H // 2 + ph // 2) - (H // 2 - ph // 2)
        w = (W // 2 + pw // 2) - (W // 2 - pw // 2)
    else:
        h, w = H, W
    xy = np.zeros((h * w, 2), np.float32)
    lib().oracle_pixel_grid(ctypes.c_int(H), ctypes.c_int(W), ctypes.c_int(ph), ctypes.c_int(pw),
                            ctypes.c_int(1 if crop else 0), _f(xy))
    return xy


def warp_points(xy, Hm):
    """Warp.warp_grid, warp.py:70-81, for a batch of point sets xy [B, n, 2]."""
    xy = np.ascontiguousarray(xy, np.float32)
    Hm = np.ascontiguousarray(Hm, np.float32).reshape(-1, 9)
    B, n = xy.shape[0], xy.shape[1]
    uv = np.zeros_like(xy)
    lib().oracle_warp_points(_f(xy), _f(Hm), _f(uv), ctypes.c_int(B), ctypes.c_int(n))
    return uv


def c2f_weights(progress, c2f, L):
    """BARF coarse-to-fine band weights, model/planar.py:462-467.  None if c2f off."""
    if c2f is None or L == 0:
        return None
    w = np.zeros(L, np.float32)
    lib().oracle_c2f_weights(ctypes.c_float(progress), ctypes.c_double(c2f[0]),
                             ctypes.c_double(c2f[1]), ctypes.c_int(L), _f(w))
    return w


def posenc_features(coord, L, w):
    """cat([coord, positional_encoding(coord)]), model/planar.py:432-434, 451-471.
    coord [..., 2] -> [..., 2 + 4L].  L == 0 means posenc disabled (feat = coord)."""
    shp = coord.shape[:-1]
    c = np.ascontiguousarray(coord, np.float32).reshape(-1, 2)
    if L == 0:
        return c.reshape(*shp, 2).copy()
    out = np.zeros((c.shape[0], 2 + 4 * L), np.float32)
    lib().oracle_posenc(_f(c), ctypes.c_int(c.shape[0]), ctypes.c_int(L),
                        _f(w) if w is not None else None, _f(out))
    return out.reshape(*shp, 2 + 4 * L)


def prologue_backward(xy, Hm, dfeat, L, w, want_dH=True):
    """Adjoint of posenc + projective warp for points xy[B,n,2] under Hm[B,3,3]:
    returns dH [B,3,3] (float64 sums over points) and d(uv) [B,n,2]."""
    B, n = xy.shape[0], xy.shape[1]
    D = 2 + 4 * L
    dH = np.zeros((B, 9), np.float64)
    duv = np.zeros((B, n, 2), np.float32)
    xy = np.ascontiguousarray(xy, np.float32)
    dfeat = np.ascontiguousarray(dfeat, np.float32).reshape(B, n, D)
    Hm = np.ascontiguousarray(Hm, np.float32).reshape(B, 9)
    for b in range(B):
        dHb = np.zeros(9, np.float64)
        duvb = np.zeros((n, 2), np.float32)
        lib().oracle_prologue_backward(_f(np.ascontiguousarray(xy[b])), _f(np.ascontiguousarray(Hm[b])),
                                       _f(np.ascontiguousarray(dfeat[b])), ctypes.c_int(n),
                                       ctypes.c_int(L), _f(w) if w is not None else None,
                                       _d(dHb), _f(duvb))
        dH[b] = dHb
        duv[b] = duvb
    return dH.reshape(B, 3, 3), duv


# ------------------------------------------------------------------------ MLP

def mlp_forward(f0, params, skip=()):
    """NeuralImageFunction.forward MLP part, model/planar.py:437-448; a layer li in `skip` takes
    cat([feat, points_enc]) (:440-441).  params: [(W [out,in], b [out]), ...] fp32.  Returns (acts,
    rgb) with acts[l] the input of layer l (acts[0] = f0, acts[l>0] post-ReLU, concatenated with f0
    for a skip layer)."""
    f0 = np.asarray(f0, np.float32)
    acts = []
    x = f0
    n = len(params)
    for li, (W, b) in enumerate(params):
        if li in skip:
            x = np.concatenate([x, f0], axis=-1)
        acts.append(x)
        z = x @ W.T + b
        if li != n - 1:
            x = np.maximum(z, np.float32(0))
        else:
            x = np.float32(1) / (np.float32(1) + np.exp(-z))
    return acts, x.astype(np.float32)


def mlp_backward(acts, rgb, d_rgb, params, skip=()):
    """Autograd of mlp_forward: returns ([(dW, db)], d_f0); a skip layer's input gradient splits into
    the previous layer's (ReLU-masked) and the posenc features', which autograd adds to layer 0's."""
    g = (d_rgb * (np.float32(1) - rgb) * rgb).astype(np.float32)
    grads = [None] * len(params)
    d_enc = None
    D = acts[0].shape[-1]
    for li in range(len(params) - 1, -1, -1):
        W, _ = params[li]
        a = acts[li]
        grads[li] = ((g.T @ a).astype(np.float32), g.sum(0, dtype=np.float64).astype(np.float32))
        d = (g @ W).astype(np.float32)
        if li in skip:
            de = d[:, -D:]
            d_enc = de if d_enc is None else (d_enc + de).astype(np.float32)
            d, a = d[:, :-D], a[:, :-D]
        if li > 0:
            g = (d * (a > 0)).astype(np.float32)
        else:
            g = d
    if d_enc is not None:
        g = (d_enc + g).astype(np.float32)
    return grads, g


def masked_mse(pred, gt, mask):
    """Graph.mse_loss with masks, model/planar.py:388-390.  pred/gt [B,3,h,w],
    mask [B,1,h,w].  Returns (loss fp32, denom fp32 = 3*sum(mask))."""
    diff = (pred - gt) * mask
    denom = np.float32(mask.sum(dtype=np.float64)) * np.float32(3)
    num = np.float32((diff.astype(np.float64) ** 2).sum())
    return np.float32(num / denom), denom


def masked_mse_backward(pred, gt, mask, denom, gout):
    """d loss / d pred, scaled by the upstream gradient gout (F7: f32(1-alpha)+1)."""
    gs = np.float32(np.float32(gout) / denom)
    md = ((pred - gt) * mask).astype(np.float32)
    return ((gs * (np.float32(2) * md)) * mask).astype(np.float32)


# ------------------------------------------------------------------------ Adam

class Adam:
    """torch.optim.Adam (betas (0.9, 0.999), eps 1e-8, no weight decay), the
    optimizer built by Model.setup_optimizer, model/planar.py:86-104."""

    def __init__(self, lr_groups, betas=(0.9, 0.999), eps=1e-8):
        self.lr_groups = lr_groups  # list of learning rates, one per param group
        self.b1, self.b2 = betas
        self.eps = eps
        self.state = {}

    def step(self, groups):
        """groups: list (aligned with lr_groups) of lists of (key, param, grad)."""
        for lr, items in zip(self.lr_groups, groups):
            for key, p, g in items:
                if g is None:
                    continue
                st = self.state.setdefault(key, [np.zeros_like(p), np.zeros_like(p), 0])
                m, v = st[0], st[1]
                st[2] += 1
                t = st[2]
                m += (g - m) * np.float32(1 - self.b1)
                v *= np.float32(self.b2)
                v += np.float32(1 - self.b2) * g * g
                bc1 = 1 - self.b1 ** t
                bc2 = 1 - self.b2 ** t
                step_size = lr / bc1
                denom = (np.sqrt(v) / np.float32(bc2 ** 0.5)) + np.float32(self.eps)
                p -= np.float32(step_size) * (m / denom)


# ---------------------------------------------------------------- full step

class PlanarStep:
    """One Model.train_iteration of the planar graph, restated on the CPU.

    cfg keys: H, W, patch_H, patch_W, L (0 = posenc off), c2f (None or [s, e]),
    max_iter, lr, lr_warp, fix_first, use_edges, alpha_initial, alpha_final, crop (default True).
    params: list of (W, b) fp32 (modified in place); warp: [B, 8] fp32.
    """

    def __init__(self, cfg, params, warp, rgb, mask):
        self.cfg = cfg
        self.params = [(np.array(W, np.float32), np.array(b, np.float32)) for W, b in params]
        self.warp = np.array(warp, np.float32)
        self.rgb = np.asarray(rgb, np.float32)  # [B,3,h,w]
        self.mask = np.asarray(mask, np.float32)  # [B,1,h,w]
        self.B = self.warp.shape[0]
        # use_cropped_images off (cfg crop False): every canvas pixel (warp.py:54-68)
        self.xy = pixel_grid(cfg["H"], cfg["W"], cfg["patch_H"], cfg["patch_W"], crop=cfg.get("crop", True))
        self.h, self.w = self.rgb.shape[2], self.rgb.shape[3]
        self.progress = np.float32(0.0)
        self.it = 0
        self.adam = Adam([cfg["lr"], cfg["lr_warp"]])

    def forward(self):
        """Graph.forward (model/planar.py:329-335) -> rgb [B, N, 3] and the caches."""
        cfg = self.cfg
        L = cfg["L"]
        Hm = sl3_to_SL3(self.warp)
        xyB = np.broadcast_to(self.xy, (self.B,) + self.xy.shape).copy()
        uv = warp_points(xyB, Hm)
        w = c2f_weights(self.progress, cfg["c2f"], L)
        f0 = posenc_features(uv, L, w).reshape(-1, 2 + 4 * L)
        acts, rgb = mlp_forward(f0, self.params, cfg.get("skip", ()))
        return dict(Hm=Hm, xyB=xyB, uv=uv, w=w, acts=acts, rgb=rgb)

    def alpha(self):
        c = self.cfg
        if not c.get("use_edges", True):
            return 0
        return c["alpha_initial"] + (c["alpha_final"] - c["alpha_initial"]) * (self.it / c["max_iter"])

    def step(self):
        """Returns dict(loss_rgb, grads, dh) and applies Adam + progress + fix_first."""
        cfg = self.cfg
        fw = self.forward()
        B, h, w = self.B, self.h, self.w
        pred = fw["rgb"].reshape(B, h, w, 3).transpose(0, 3, 1, 2)
        loss, denom = masked_mse(pred, self.rgb, self.mask)
        alpha = self.alpha()
        # summarize_loss: d all / d rgb = f32(1 - alpha) + 1
        gout = np.float32(np.float32(1 - alpha) + np.float32(1.0))
        dpred = masked_mse_backward(pred, self.rgb, self.mask, denom, gout)
        d_rgb = dpred.transpose(0, 2, 3, 1).reshape(-1, 3)
        grads, df0 = mlp_backward(fw["acts"], fw["rgb"], d_rgb, self.params, cfg.get("skip", ()))
        L = cfg["L"]
        dH, _ = prologue_backward(fw["xyB"], fw["Hm"], df0.reshape(B, -1, 2 + 4 * L), L, fw["w"])
        dh = sl3_to_SL3_backward(self.warp, dH.astype(np.float32))
        self.it += 1
        mlp_items = []
        for li, ((W, b), (dW, db)) in enumerate(zip(self.params, grads)):
            mlp_items += [(f"W{li}", W, dW), (f"b{li}", b, db)]
        self.adam.step([mlp_items, [("warp", self.warp, dh)]])
        self.progress = np.float32(self.it / cfg["max_iter"])
        if cfg.get("fix_first", True):
            self.warp[0] = 0
        return dict(loss_rgb=loss, grads=grads, dh=dh, rgb=fw["rgb"], dH=dH)


# ---------------------------------------------------------------- edge stencil
# inputs.compute_edges (reference inputs.py:50-67): per image, cv2.Sobel(i, CV_64F, 1, 0, ksize=3)
# and (0, 1), magnitude sqrt(sx^2 + sy^2), cv2.GaussianBlur(., (5, 5), 0).  cv2 is absent here, so
# this restates OpenCV's documented semantics (parity unpinned against cv2 itself):
#   * default border BORDER_REFLECT_101 (…dcb|abcd|cba…) for both filters;
#   * Sobel ksize 3 = separable [-1, 0, 1] (derivative) x [1, 2, 1] (smoothing);
#   * GaussianBlur ksize 5 with sigma 0 takes OpenCV's fixed small-kernel table
#     [1, 4, 6, 4, 1] / 16 (getGaussianKernel: sigma <= 0 and odd ksize <= 7), row pass then
#     column pass.
# Evaluation order (fp64): Sobel sums of fp32 inputs are exact in fp64; the blur accumulates left to
# right, ((((g0 m0 + g1 m1) + g2 m2) + g3 m3) + g4 m4), which the HIP kernel follows.
EDGE_GAUSS5 = np.array([0.0625, 0.25, 0.375, 0.25, 0.0625], np.float64)


def _reflect101(idx, n):
    idx = np.asarray(idx)
    if n == 1:
        return np.zeros_like(idx)
    period = 2 * n - 2
    idx = np.abs(idx) % period
    return np.where(idx >= n, period - idx, idx)


def edge_map(img):
    """[N, H, W] float32 images -> [N, H, W] float64 edge maps (inputs.compute_edges per channel)."""
    a = np.asarray(img, np.float32).astype(np.float64)
    N, H, W = a.shape
    ry = _reflect101(np.arange(-1, H + 1), H)
    rx = _reflect101(np.arange(-1, W + 1), W)
    e = a[:, ry][:, :, rx]                     # [N, H+2, W+2]
    c = e[:, 1:-1]
    up, dn = e[:, :-2], e[:, 2:]
    sx = ((up[:, :, 2:] - up[:, :, :-2]) + 2.0 * (c[:, :, 2:] - c[:, :, :-2])) + (dn[:, :, 2:] - dn[:, :, :-2])
    sy = ((dn[:, :, :-2] - up[:, :, :-2]) + 2.0 * (dn[:, :, 1:-1] - up[:, :, 1:-1])) + (dn[:, :, 2:] - up[:, :, 2:])
    m = np.sqrt(sx * sx + sy * sy)
    g = EDGE_GAUSS5
    mx = m[:, :, _reflect101(np.arange(-2, W + 2), W)]
    r = g[0] * mx[:, :, 0:W]
    for j in range(1, 5):
        r = r + g[j] * mx[:, :, j:j + W]
    ry5 = r[:, _reflect101(np.arange(-2, H + 2), H)]
    out = g[0] * ry5[:, 0:H]
    for j in range(1, 5):
        out = out + g[j] * ry5[:, j:j + H]
    return out


def erode_rect(img, kh=5, kw=5):
    """erode_images (reference inputs.py:71-85): cv2.erode with a kh x kw MORPH_RECT element, anchor
    at its centre, default border (constant +max for erosion): min over the in-image window part.
    [N, H, W] float32 -> float32."""
    a = np.asarray(img, np.float32)
    N, H, W = a.shape
    pad = np.full((N, H + kh - 1, W + kw - 1), np.inf, np.float32)
    pad[:, kh // 2:kh // 2 + H, kw // 2:kw // 2 + W] = a
    out = np.full_like(a, np.inf)
    for dy in range(kh):
        for dx in range(kw):
            out = np.minimum(out, pad[:, dy:dy + H, dx:dx + W])
    return out
