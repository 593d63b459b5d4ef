"""Bit images of the split-bf16 fused training step on fixed cases (helper module, not a test file).

The bf16x3 recipe carries the seed-3 end-to-end contract through its exact fp32 summation order
(DESIGN.md §4), so every change to the step kernel must keep its bits.  `case_bits(case)` runs one
fused step (rgb, loss, every MLP gradient, the warp gradient), the optimizer, and two more
Model.train_iteration calls (losses, final warps and weights) and returns the sha1 of every
tensor's bytes.  tests/golden/step2_bits.json holds those digests as the library of the commit
named in it computed them (tools/make_step2_bits.py, run on an MI355X); test_gpu_parity.py
compares the current library against it.  The cases cover every compile-time instantiation of
k_step2 (L = 8, 9..12, 13..15, 16), the generic one (narrow widths), one tile per block, and the
headline C3 batch (64 patches of 256x256, L = 16).
"""
import hashlib
import os
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
BITS_JSON = os.path.join(GOLDEN, "step2_bits.json")
DEV = "cuda:0"

CASES = {
    # name: (patches, crop, L, hidden widths); None = the cat_batch3 C1 problem (5 x 180x240, L=8)
    "c1": None,
    "c3x2": (2, 256, 16, [256] * 4),
    "c3x3-L10": (3, 256, 10, [256] * 4),
    "L16-1tile": (2, 100, 16, [256] * 4),
    "narrow": (2, 64, 8, [128, 96, 128]),
    "L13": (2, 128, 13, [256] * 4),
    "L15": (2, 128, 15, [256] * 4),
    "c3x64": (64, 256, 16, [256] * 4),
}


class _Loader:
    def set_postfix(self, **kw):
        pass


def _opt(out, **over):
    import options
    from util import EasyDict as edict
    opt = options.load_options("options/planar.yaml")
    base = {"model": "planar", "yaml": "planar", "seed": 3, "barf_c2f": [0, 0.4], "precision": "bf16x3"}
    base.update(over)
    opt = options.override_options(opt, edict(base))
    opt.device = DEV
    opt.output_path = out
    opt.freq.vis = 10 ** 9
    return opt


def build_case(case, out="/tmp/marf_bits", precision="bf16x3"):
    """The product model of `case` (bf16x3 unless precision says otherwise) and its var bundle
    (seeded; identical on every run)."""
    from model import planar
    from util import EasyDict as edict
    if CASES[case] is None:
        imgs = np.load(os.path.join(GOLDEN, "cat_batch3_c1.npz"), allow_pickle=False)
        opt = _opt(out, precision=precision)
        torch.manual_seed(3)
        m = planar.Model(opt)
        rgb = torch.from_numpy(imgs["rgb"].astype(np.float32) / np.float32(255)).to(DEV)
        mask = torch.from_numpy(imgs["mask"].astype(np.float32)).to(DEV)
        m.images = edict(rgb=rgb, masks=mask, masks_eroded=mask, edges=None, gt_hom=None, gt=None)
        m.build_networks()
    else:
        B, crop, L, hidden = CASES[case]
        opt = _opt(out, H=512, W=512, patch_H=crop, patch_W=crop, batch_size=B, use_edges=False, precision=precision,
                   arch={"layers": [None] + list(hidden) + [3], "skip": [], "posenc": {"L_2D": L}})
        torch.manual_seed(3)
        m = planar.Model(opt)
        rng = np.random.default_rng(3)
        yy, xx = np.meshgrid(np.linspace(0, 1, crop), np.linspace(0, 1, crop), indexing="ij")
        rgb = np.stack([[0.5 + 0.4 * np.sin(2 * np.pi * (rng.uniform(1, 4) * xx + rng.uniform(1, 4) * yy)
                                            + rng.uniform(0, 6)) for _ in range(3)] for _ in range(B)]).astype(np.float32)
        mask = (rng.random((B, 1, crop, crop)) < 0.85).astype(np.float32)
        warp = (rng.standard_normal((B, 8)) * 0.01).astype(np.float32)
        m.images = edict(rgb=torch.from_numpy(rgb).to(DEV), masks=torch.from_numpy(mask).to(DEV),
                         masks_eroded=torch.from_numpy(mask).to(DEV), edges=None, gt_hom=None, gt=None)
        m.build_networks()
        m.graph.warp_param.weight.data.copy_(torch.from_numpy(warp).to(DEV))
        m.graph.neural_image.progress.data.fill_(0.2)
    m.setup_optimizer()
    m.timer = edict(start=time.time(), it_mean=None)
    return m, edict(idx=torch.arange(m.batch_size), images=m.images)


def _digest(t):
    a = t.detach().contiguous().cpu()
    return hashlib.sha1(a.view(torch.uint8).numpy().tobytes() if a.numel() else b"").hexdigest()


def run_case(m, var):
    """The tensors of one fused step, the optimizer, and two more training iterations."""
    m.optim.zero_grad()
    v = m.graph.forward(var, mode="train")
    loss = m.summarize_loss(m.graph.compute_loss(v, mode="train"))
    loss.all.backward()
    out = {"rgb": v.rgb_prediction.detach().clone(), "loss": loss.rgb.detach().reshape(1).clone(),
           "dh": m.graph.warp_param.weight.grad.detach().clone()}
    for i, lay in enumerate(m.graph.neural_image.mlp):
        out[f"dW{i}"] = lay.weight.grad.detach().clone()
        out[f"db{i}"] = lay.bias.grad.detach().clone()
    m.optim.step()
    m.graph.warp_param.weight.data[0] = 0
    losses = []
    for _ in range(2):
        losses.append(m.train_iteration(var, _Loader()).rgb.detach().reshape(1).clone())
        m.graph.warp_param.weight.data[0] = 0
    out["losses"] = torch.cat(losses)
    out["warp"] = m.graph.warp_param.weight.detach().clone()
    for i, lay in enumerate(m.graph.neural_image.mlp):
        out[f"W{i}"] = lay.weight.detach().clone()
    return out


def case_bits(case):
    """{"kernel": the step kernel's name, "bits": {tensor: sha1 of its bytes}} of `case`."""
    m, var = build_case(case)
    kernel = m.graph.neural_image.engine(torch.device(DEV)).net.step_kernel
    out = run_case(m, var)
    return {"kernel": kernel, "bits": {k: _digest(v) for k, v in out.items()}}
