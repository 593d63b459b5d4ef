"""Warp / Lie with the reference's API (warp.py:5-108), computed by libmarf.so on the GPU.

  Warp(opt).get_normalized_pixel_grid(crop)  -> [B, h*w, 2]      (HIP pixel-grid kernel)
  Warp(opt).warp_grid(xy_grid, warp)         -> [B, N, 2]        (HIP Lie exp + warp kernels, autograd)
  Warp(opt).warp_corners(warp_param)         -> [B, 4, 2]
  Lie().sl3_to_SL3(h)                        -> [..., 3, 3]      (HIP, torch.matrix_exp bit-exact)
  Lie().se2_to_SE2(p)                        -> [..., 3, 3]      (extension: se(2) tangent (tx, ty, theta))

The training forward does not call these: Graph.forward runs grid, warp, posenc and MLP fused in
one kernel (marf_hip.render_train).  These entry points exist for drop-in callers and logging.
"""
import torch

import marf_hip


def _centre_window(full, crop):
    """[start, stop) of a centred crop, integer halves as warp.py:14-19 computes them."""
    half_full, half_crop = full // 2, crop // 2
    return (half_full - half_crop, half_full + half_crop)


class Warp:
    """Pixel grid + homography warp of the planar patches (warp.py:5-93)."""

    def __init__(self, opt):
        self.max_h, self.max_w = opt.H, opt.W
        self.crop_h, self.crop_w = opt.patch_H, opt.patch_W
        self.y_crop = _centre_window(opt.H, opt.patch_H)
        self.x_crop = _centre_window(opt.W, opt.patch_W)
        longest = max(opt.H, opt.W)
        self.norm_h, self.norm_w = opt.H / longest, opt.W / longest
        self.batch_size, self.device = opt.batch_size, opt.device
        self.warp_type, self.dof = opt.warp.type, opt.warp.dof

    def to_hom(self, matrix):
        return torch.cat([matrix, torch.ones_like(matrix[..., :1])], dim=-1)

    def get_normalized_pixel_grid(self, crop=False):
        xy = marf_hip.pixel_grid(self.max_h, self.max_w, self.crop_h, self.crop_w, crop, self.device)
        return xy.unsqueeze(0).expand(self.batch_size, -1, -1)  # [B, HW, 2] (broadcast view)

    def warp_grid(self, xy_grid, warp):
        if self.warp_type == "homography":
            assert self.dof == 8
            H = lie.sl3_to_SL3(warp)  # differentiable: HIP matrix_exp adjoint
        elif self.warp_type == "se2":  # extension (the reference has no SE(2) warp)
            assert self.dof == 3
            H = lie.se2_to_SE2(warp)
        else:
            raise AssertionError(f"unsupported warp type {self.warp_type}")
        return marf_hip.warp_points(xy_grid, H)  # differentiable in xy and H

    def warp_corners(self, warp_param):
        """The four crop-window corners (in the reference's corner order) warped per patch."""
        def norm(i, full, scale):
            return ((i + 0.5) / full * 2 - 1) * scale
        ys = [norm(i, self.max_h, self.norm_h) for i in self.y_crop]
        xs = [norm(i, self.max_w, self.norm_w) for i in self.x_crop]
        pts = torch.tensor([[xs[0], ys[0]], [xs[0], ys[1]], [xs[1], ys[1]], [xs[1], ys[0]]],
                           dtype=torch.float32, device=warp_param.device)
        return self.warp_grid(pts.unsqueeze(0), warp_param)


class Lie:
    def sl3_to_SL3(self, h):
        return marf_hip.sl3_to_SL3(h)

    def se2_to_SE2(self, p):
        """se(2) tangent (tx, ty, theta) -> SE(2) (extension; exp of the embedded sl(3) generator)."""
        return marf_hip.se2_to_SE2(p)


lie = Lie()
