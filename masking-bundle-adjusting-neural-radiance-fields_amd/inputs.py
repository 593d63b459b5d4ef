"""Input data (inputs.py of the reference, restated without torchvision / cv2 / kornia).

Same file formats and same numbers:
  * images   i.png   (480x360 RGBA) -> RGB, PIL thumbnail to (patch_W, patch_H) with LANCZOS,
             uint8 / 255 in fp32, CHW                          (inputs.py:16-33)
  * masks    i-m.png -> L, same resize, inverted: (x < 0.5)      (inputs.py:30-31, 119)
  * edges    Sobel 3x3 (float64) -> magnitude -> Gaussian 5x5 (sigma from ksize, as cv2), reflect-101
             borders                                            (inputs.py:50-69)
  * erosion  5x5 rectangular min filter                         (inputs.py:71-85)
  * H_0_i.mat 3x3 text homographies, normalised like kornia.geometry.conversions
             .normalize_homography with the reference's (width, height) argument order
             (inputs.py:87-105)
These run on the host once per run (edges: at logging steps); they are not on the GPU hot path.
"""
import os

import numpy as np
import PIL.Image
import torch

from util import EasyDict as edict


def _to_tensor(a):
    """torchvision.transforms.functional.to_tensor: uint8 HWC -> fp32 CHW / 255; float kept."""
    if a.ndim == 2:
        a = a[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).contiguous()
    if t.dtype == torch.uint8:
        return t.to(torch.float32).div(255)
    return t


def load_images(fps, opt, mode="RGB", invert_gray=False):
    if not fps:
        return None
    if not isinstance(fps, list):
        raise TypeError("Function requires list of input filepaths!")
    out = []
    for fp in fps:
        im = PIL.Image.open(fp).convert(mode)
        if opt.use_cropped_images:
            im.thumbnail((opt.patch_W, opt.patch_H), PIL.Image.Resampling.LANCZOS)
        t = _to_tensor(np.array(im, dtype=np.uint8, copy=True)).to(opt.device)
        if mode == "L" and invert_gray:
            t = (t < 0.5).float()
        out.append(t)
    return torch.stack(out)


def load_single_image(fp, device, mode="RGB"):
    if not fp or not device:
        raise ValueError("Function requires file pointer as string and device to store tensor to.")
    im = PIL.Image.open(fp).convert(mode)
    return _to_tensor(np.array(im, dtype=np.uint8, copy=True)).to(device)


def compute_edges(images_tensor, device):
    """inputs.compute_edges (reference inputs.py:50-67): [B, C, H, W] -> [B, C, H, W] float64 edge
    images (cv2.Sobel 3x3 CV_64F x / y, magnitude, cv2.GaussianBlur 5x5 sigma 0, reflect-101), in one
    HIP launch on the device (marf_edge_map); C == 1 stays one channel, as cv2 + to_tensor give."""
    import marf_hip
    return marf_hip.edge_map(images_tensor.to(device))


def erode_images(images_tensor, device, kernel=(5, 5)):
    """erode_images (reference inputs.py:71-85): cv2.erode with a kernel = (width, height) MORPH_RECT
    element, default anchor / border, per channel image; one HIP launch (marf_erode_rect)."""
    import marf_hip
    return marf_hip.erode_rect(images_tensor.to(device), kernel)


def _normal_transform_pixel(height, width, eps=1e-14):
    tr = torch.tensor([[1.0, 0.0, -1.0], [0.0, 1.0, -1.0], [0.0, 0.0, 1.0]])
    wd = eps if width == 1 else width - 1.0
    hd = eps if height == 1 else height - 1.0
    tr[0, 0] = tr[0, 0] * 2.0 / wd
    tr[1, 1] = tr[1, 1] * 2.0 / hd
    return tr[None]


def normalize_homography(dst_pix_trans_src_pix, dsize_src, dsize_dst):
    """kornia.geometry.conversions.normalize_homography restated (dsize = (height, width))."""
    src_h, src_w = dsize_src
    dst_h, dst_w = dsize_dst
    H = dst_pix_trans_src_pix
    src_norm = _normal_transform_pixel(src_h, src_w).to(H)
    src_pix_trans_src_norm = torch.linalg.inv(src_norm)
    dst_norm = _normal_transform_pixel(dst_h, dst_w).to(H)
    return dst_norm @ (H @ src_pix_trans_src_norm)


def load_homography(fps, width, height, device, append_zero=True):
    if not fps:
        return None
    if not isinstance(fps, list):
        raise TypeError("Function requires a list of input file paths!")
    hs = [torch.eye(3, dtype=torch.float32)] if append_zero else []
    for fp in fps:
        hs.append(torch.tensor(np.loadtxt(fp), dtype=torch.float32))
    gt = torch.stack(hs)
    # the reference passes (width, height) where (height, width) is expected; kept as is
    return normalize_homography(gt, (width, height), (width, height)).to(device)


def prepare_images(opt, fps_images=None, fps_masks=None, fp_gt=None, fps_hom=None, edges=True):
    inputs = edict()
    inputs.gt = load_single_image(fp_gt, opt.device) if fp_gt and os.path.exists(fp_gt) else None
    inputs.rgb = load_images(fps_images, opt)
    inputs.gt_hom = load_homography(fps_hom, opt.W, opt.H, opt.device) if fps_hom else None
    inputs.masks = load_images(fps_masks, opt, mode="L", invert_gray=True)
    inputs.masks_eroded = erode_images(inputs.masks, opt.device, kernel=(5, 5)) if inputs.masks is not None else None
    inputs.gray = load_images(fps_images, opt, mode="L")
    inputs.edges = compute_edges(inputs.gray, opt.device) if edges else None
    return inputs
