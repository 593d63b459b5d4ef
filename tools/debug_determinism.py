"""GPU determinism check of the training step: the same Graph step (forward, fused masked MSE,
backward) run four times on identical inputs must give bit-identical rgb, MLP gradients and
warp gradient.  MARF_LIB selects a library variant (e.g. one built with -fslp-vectorize).

    python tools/debug_determinism.py [precision] [L]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]
from test_gpu_parity import make_opt  # noqa: E402
from model import planar  # noqa: E402
from util import EasyDict as edict  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
L = int(sys.argv[2]) if len(sys.argv) > 2 else 16
B = 8
opt = make_opt(None, H=512, W=512, patch_H=256, patch_W=256, batch_size=B, precision=prec, use_edges=False,
               arch={"layers": [None, 256, 256, 256, 256, 3], "skip": [], "posenc": {"L_2D": L}})
torch.manual_seed(0)
graph = planar.Graph(opt).to("cuda:0")
graph.neural_image.progress.data.fill_(0.2)
rng = np.random.default_rng(2)
graph.warp_param.weight.data.copy_(torch.from_numpy((rng.standard_normal((B, 8)) * 0.01).astype(np.float32)))
gt = torch.from_numpy(rng.random((B, 3, 256, 256)).astype(np.float32)).cuda()
mask = torch.from_numpy((rng.random((B, 1, 256, 256)) < 0.85).astype(np.float32)).cuda()
var = edict(images=edict(rgb=gt, masks=mask, masks_eroded=mask, edges=None))
graph.need_edges = False
snaps = []
for it in range(4):
    for p in graph.parameters():
        p.grad = None
    v = graph.forward(var, mode="train")
    loss = graph.compute_loss(v, mode="train")
    (loss.render + loss.rgb).backward()
    torch.cuda.synchronize()
    snaps.append([v.rgb_prediction.detach().clone(), graph.warp_param.weight.grad.clone()] +
                 [p.grad.clone() for p in graph.neural_image.mlp.parameters()])
names = ["rgb", "dh"] + [n for n, _ in graph.neural_image.mlp.named_parameters()]
bad = 0
for i in range(1, 4):
    for n, a, b in zip(names, snaps[0], snaps[i]):
        if not torch.equal(a, b):
            bad += 1
            d = (a != b).nonzero()
            print(f"run {i} vs 0: {n} differs in {d.shape[0]} elements, max |diff| {float((a - b).abs().max()):.3e}")
print(f"{prec} L={L} lib={os.environ.get('MARF_LIB', 'default')}: "
      + ("bit-identical over 4 runs" if bad == 0 else f"{bad} differing tensors"))
sys.exit(1 if bad else 0)
