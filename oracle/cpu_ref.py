"""cpu_ref.py -- op-for-op torch-CPU (fp32) restatement of the reference's planar training step.

TEST INFRASTRUCTURE ONLY.  Only tests/ and bench.py's cpu_baseline leg may import this module:
tests/test_cpu_ref.py pins it to the fixtures generated from the reference (tests/golden/), and
bench.py times it on the GPU box's host cores as the CPU baseline (SURVEY.md §8(d) "CPU baseline").
The product (masking-bundle-adjusting-neural-radiance-fields_amd/) never imports it.

Where oracle.py restates the step in numpy + C with hand-written adjoints, this module runs the same
aten ops the reference runs, in the same order, and lets torch autograd take the backward:
    Warp.get_normalized_pixel_grid(crop=True)     warp.py:33-53
    Warp.warp_grid + to_hom + Lie.sl3_to_SL3      warp.py:27-31, 70-81, 98-106
    NeuralImageFunction.forward / positional_encoding (+ BARF c2f)   model/planar.py:429-471
    Graph.compute_loss / mse_loss                 model/planar.py:355-391
    Model.summarize_loss                          model/planar.py:172-185 (log10 weights all 0)
    Model.train_iteration + fix_first             model/planar.py:187-209, 154-158
    Model.setup_optimizer (Adam, two groups)      model/planar.py:86-104
The edge term carries no gradient in the reference, so it is left out of the loss sum
here: the parameters, rgb and loss.rgb are unaffected.
"""
import math

import numpy as np
import torch


def sl3_to_SL3(h):
    """h [..., 8] -> expm of the trace-free generator (warp.py:98-106 layout)."""
    h1, h2, h3, h4, h5, h6, h7, h8 = h.unbind(-1)
    A = torch.stack([torch.stack([h5, h3, h1], -1),
                     torch.stack([h4, -h5 - h6, h2], -1),
                     torch.stack([h7, h8, h6], -1)], -2)
    return torch.linalg.matrix_exp(A)


def pixel_grid(H, W, ph, pw, crop=True, dtype=torch.float32):
    """Pixel-centre coordinates in [-1, 1] scaled by the aspect norms, x fastest: [h*w, 2]."""
    norm_h, norm_w = H / max(H, W), W / max(H, W)
    if crop:
        ys = torch.arange(H // 2 - ph // 2, H // 2 + ph // 2, dtype=dtype)
        xs = torch.arange(W // 2 - pw // 2, W // 2 + pw // 2, dtype=dtype)
    else:
        ys = torch.arange(H, dtype=dtype)
        xs = torch.arange(W, dtype=dtype)
    y = ((ys + 0.5) / H * 2 - 1) * norm_h
    x = ((xs + 0.5) / W * 2 - 1) * norm_w
    Y, X = torch.meshgrid(y, x, indexing="ij")
    return torch.stack([X, Y], -1).view(-1, 2)


def warp_grid(xy, h):
    """[B, n, 2] points through the homographies of h [B, 8] (perspective divide with +1e-8)."""
    hom = torch.cat([xy, torch.ones_like(xy[..., :1])], -1)
    Xw = hom @ sl3_to_SL3(h).transpose(-2, -1)
    return Xw[..., :2] / (Xw[..., 2:] + 1e-8)


def positional_encoding(coord, L, progress=None, c2f=None):
    """[..., 2] -> [..., 4L]: per coordinate sin bands then cos bands, BARF c2f weighting."""
    freq = (2 ** torch.arange(L, dtype=coord.dtype) * np.pi).to(coord.device)
    spec = coord[..., None] * freq
    enc = torch.stack([spec.sin(), spec.cos()], -2).view(*coord.shape[:-1], -1)
    if c2f is not None:
        start, end = c2f
        a = (progress - start) / (end - start) * L
        k = torch.arange(L, dtype=coord.dtype, device=coord.device)
        wgt = (1 - (a - k).clamp_(min=0, max=1).mul_(np.pi).cos_()) / 2
        enc = (enc.view(-1, L) * wgt).view(enc.shape)
    return enc


class CpuRefStep:
    """One reference training iteration per step() on torch CPU tensors.

    cfg keys as oracle.PlanarStep: H, W, patch_H, patch_W, L (0 = posenc off), c2f (None or
    [start, end]), max_iter, lr, lr_warp, fix_first, use_edges, alpha_initial, alpha_final.
    params: [(W [out, in], b [out]), ...]; warp [B, 8]; rgb [B, 3, h, w]; mask [B, 1, h, w].
    dtype / device: torch.float32 on the CPU is the reference's arithmetic; float64 gives the
    near-exact values the fp32 implementations are measured against (tests).
    """

    def __init__(self, cfg, params, warp, rgb, mask, dtype=torch.float32, device="cpu"):
        self.cfg = cfg
        self.mlp = torch.nn.ModuleList()
        for W, b in params:
            lin = torch.nn.Linear(W.shape[1], W.shape[0])
            lin.weight.data.copy_(torch.as_tensor(np.asarray(W, np.float32)))
            lin.bias.data.copy_(torch.as_tensor(np.asarray(b, np.float32)))
            self.mlp.append(lin)
        self.mlp.to(device=device, dtype=dtype)

        def T(a):
            return torch.as_tensor(np.asarray(a, np.float32)).to(device=device, dtype=dtype)
        self.progress = torch.nn.Parameter(torch.tensor(0.0, dtype=dtype, device=device))
        self.warp = torch.nn.Parameter(T(warp).clone())
        self.rgb = T(rgb)
        self.mask = T(mask)
        self.B, _, self.h, self.w = self.rgb.shape
        self.xy = pixel_grid(cfg["H"], cfg["W"], cfg["patch_H"], cfg["patch_W"], crop=True, dtype=dtype).to(device)
        self.it = 0
        self.optim = torch.optim.Adam([dict(params=list(self.mlp.parameters()) + [self.progress], lr=cfg["lr"]),
                                       dict(params=[self.warp], lr=cfg["lr_warp"])])

    def render(self, coord):
        L = self.cfg["L"]
        points_enc = coord
        if L > 0:
            enc = positional_encoding(coord, L, self.progress.data, self.cfg["c2f"])
            points_enc = torch.cat([coord, enc], -1)
        feat = points_enc
        skip = self.cfg.get("skip", ())
        for li, lin in enumerate(self.mlp):
            if li in skip:  # model/planar.py:440-441
                feat = torch.cat([feat, points_enc], -1)
            feat = lin(feat)
            if li != len(self.mlp) - 1:
                feat = torch.relu(feat)
        return feat.sigmoid_()

    def step(self):
        c = self.cfg
        self.optim.zero_grad()
        uv = warp_grid(self.xy.repeat(self.B, 1, 1), self.warp)
        rgb = self.render(uv)
        pred = rgb.view(self.B, self.h, self.w, 3).permute(0, 3, 1, 2)
        alpha = (c["alpha_initial"] + (c["alpha_final"] - c["alpha_initial"]) * (self.it / c["max_iter"])
                 if c.get("use_edges", False) else 0)
        loss_rgb = (((pred.contiguous() - self.rgb) * self.mask) ** 2).sum() / (self.mask.sum() * 3)
        render = (1 - alpha) * loss_rgb
        (render + loss_rgb).backward()
        self.optim.step()
        self.it += 1
        self.progress.data.fill_(self.it / c["max_iter"])
        if c.get("fix_first", True):
            self.warp.data[0] = 0
        return dict(loss_rgb=float(loss_rgb.detach()), rgb=rgb.detach().reshape(-1, 3).cpu().numpy(),
                    grads=[(lin.weight.grad.cpu().numpy().copy(), lin.bias.grad.cpu().numpy().copy())
                           for lin in self.mlp],
                    dh=self.warp.grad.cpu().numpy().copy())


def set_threads():
    """Every core this process may run on, capped by OMP_NUM_THREADS when that
    is set: the GPU box's affinity mask lists the whole host while the job's CPU share is what
    OMP_NUM_THREADS holds there (16), and oversubscribing it slows torch down.  Returns the count."""
    import os
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    torch.set_num_threads(n)
    return n


def psnr(loss_rgb):
    return -10 * math.log10(loss_rgb)
