"""Import harness for the upstream reference (test infrastructure only).

Runs ONLY in the survey/build container, where the reference is mounted read-only
at /root/reference.  It is never imported by the product, by `-m gpu` tests, by
`smoke()` or by `bench.py` (the reference does not exist on the GPU box).

The reference's hot path (`warp.py`, `model/planar.py`) needs only torch, but its
module imports pull in packages that are absent here (torchvision, tensorboard,
cv2, kornia, easydict, imageio, visdom, termcolor, ipdb).  None of them is on the
gradient path, so they are registered as inert stub modules before
the import.  `inputs.compute_edges` (cv2, non-differentiable) is
replaced by a float64 zero tensor of the same shape, which leaves every parameter
and every RGB value bit-identical.

Nothing is written under /root/reference: bytecode writing is disabled.
"""
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("MARF_REFERENCE", "/root/reference")


class EasyDict(dict):
    """Minimal recursive attribute dict (stands in for the absent `easydict`)."""

    def __init__(self, d=None, **kwargs):
        super().__init__()
        d = dict(d or {}, **kwargs)
        for k, v in d.items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, EasyDict):
            v = EasyDict(v)
        elif isinstance(v, (list, tuple)):
            v = type(v)(EasyDict(x) if isinstance(x, dict) else x for x in v)
        super().__setitem__(k, v)

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def pop(self, k, *default):
        return super().pop(k, *default)

    def update(self, d=None, **kw):
        for k, v in dict(d or {}, **kw).items():
            self[k] = v


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


def install_stubs():
    if "easydict" not in sys.modules:
        _stub("easydict", EasyDict=EasyDict)
    tv = _stub("torchvision")
    tvt = _stub("torchvision.transforms")
    tvf = _stub("torchvision.transforms.functional")
    tvu = _stub("torchvision.utils")
    tv.transforms, tv.utils, tvt.functional = tvt, tvu, tvf
    import torch.utils  # noqa: F401
    tb = _stub("torch.utils.tensorboard", SummaryWriter=object)
    torch.utils.tensorboard = tb
    _stub("imageio")
    _stub("visdom")
    _stub("cv2")
    k = _stub("kornia")
    kg = _stub("kornia.geometry")
    kgc = _stub("kornia.geometry.conversions")
    k.geometry, kg.conversions = kg, kgc
    _stub("termcolor", colored=lambda s, *a, **kw: s)
    _stub("ipdb")


_mods = None


def import_reference():
    """Return (warp, planar, options, inputs) modules of the reference."""
    global _mods
    if _mods is not None:
        return _mods
    if not os.path.isdir(REF):
        raise RuntimeError(f"reference not found at {REF}")
    sys.dont_write_bytecode = True
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import importlib
    warp = importlib.import_module("warp")
    inputs = importlib.import_module("inputs")
    options = importlib.import_module("options")
    planar = importlib.import_module("model.planar")

    def compute_edges_zero(images_tensor, device):  # gradient-neutral stand-in (F6)
        return torch.zeros(images_tensor.shape, dtype=torch.float64, device=images_tensor.device)

    inputs.compute_edges = compute_edges_zero
    _mods = (warp, planar, options, inputs)
    return _mods


def make_opt(overrides=None, seed=3):
    """options/planar.yaml + overrides, processed like options.process_options
    (options.py:99-120) minus the output-dir creation and the interactive prompts."""
    _, _, options, _ = import_reference()
    opt = options.load_options(os.path.join(REF, "options", "planar.yaml"))
    over = {"model": "planar", "yaml": "planar", "seed": seed, "barf_c2f": [0, 0.4]}
    over.update(overrides or {})
    opt = options.override_options(opt, EasyDict(over), key_stack=[])
    opt = EasyDict(opt)
    opt.device = "cpu"
    return opt


def seed_all(seed):
    import random
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def load_images_pil(paths, opt, mode="RGB", invert_gray=False):
    """PIL-only restatement of inputs.load_images (inputs.py:16-33) with
    torchvision.to_tensor replaced by its numpy equivalent (uint8 / 255 in fp32)."""
    import PIL.Image
    out = []
    for p in paths:
        im = PIL.Image.open(p).convert(mode)
        if opt.use_cropped_images:
            im.thumbnail((opt.patch_W, opt.patch_H), PIL.Image.Resampling.LANCZOS)
        a = np.array(im, dtype=np.uint8, copy=True)
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(a).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
        if mode == "L" and invert_gray:
            t = (t < 0.5).float()
        out.append(t)
    return torch.stack(out)
