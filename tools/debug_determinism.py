"""GPU debug: run the fused backward twice on identical inputs and report which library buffers
differ (workspace regions / saved activations / outputs)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import marf_hip  # noqa
from test_gpu_parity import make_opt  # noqa
from model import planar  # noqa
from util import EasyDict as edict  # noqa

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
L = int(sys.argv[2]) if len(sys.argv) > 2 else 16
B = 4
opt = make_opt(None, H=512, W=512, patch_H=256, patch_W=256, batch_size=B, precision=prec,
               arch={"layers": [None, 256, 256, 256, 256, 3], "skip": [], "posenc": {"L_2D": L}})
torch.manual_seed(0)
graph = planar.Graph(opt).to("cuda:0")
graph.neural_image.progress.data.fill_(0.2)
rng = np.random.default_rng(2)
gt = torch.from_numpy(rng.random((B, 3, 256, 256)).astype(np.float32)).cuda()
mask = torch.from_numpy((rng.random((B, 1, 256, 256)) < 0.85).astype(np.float32)).cuda()
var = edict(images=edict(rgb=gt, masks=mask, masks_eroded=mask, edges=None))
graph.need_edges = False
snaps = []
for it in range(4):
    for p in graph.parameters():
        p.grad = None
    v = graph.forward(var)
    loss = graph.mse_loss(v.rgb_prediction_map, gt, mask)
    loss.backward()
    torch.cuda.synchronize()
    snaps.append(dict(ws=marf_hip._BUFS.bufs["planar_ws"].clone(), saved=marf_hip._BUFS.bufs["planar_saved"].clone(),
                      dh=graph.warp_param.weight.grad.clone(), rgb=v.rgb_prediction.detach().clone()))
S = B * 65536
Kp = [(2 + 4 * L + 31) // 32 * 32, 256, 256, 256, 256]
esz = 2 if prec == "bf16" else 4
off = 0
regions = {}
for l in range(1, 5):
    n = S * Kp[l] * esz
    regions[f"dz{l}"] = (off, off + n)
    off += (n + 255) // 256 * 256
regions["glast"] = (off, off + S * 16)
off += (S * 16 + 255) // 256 * 256
TP = 128 if prec == "bf16" else 64
regions["dH"] = (off, off + (S // TP) * 36)
for i in range(1, 4):
    a, b = snaps[0], snaps[i]
    print(f"run {i} vs 0: rgb equal {torch.equal(a['rgb'], b['rgb'])} dh equal {torch.equal(a['dh'], b['dh'])} "
          f"saved equal {torch.equal(a['saved'], b['saved'])}")
    for name, (s0, s1) in regions.items():
        d = (a["ws"][s0:s1] != b["ws"][s0:s1]).nonzero()
        print(f"   {name}: {d.numel()} differing bytes" + (f", first at +{int(d[0])}" if d.numel() else ""))
    if name == "dH":
        pa = a["ws"][s0:s1].view(torch.float32).view(-1, 9)
        pb = b["ws"][s0:s1].view(torch.float32).view(-1, 9)
        rows = (pa != pb).any(1).nonzero().flatten()
        print("   differing dH tiles:", rows[:20].tolist(), "count", rows.numel())
    if name == "dH" and rows.numel():
        r = int(rows[0])
        print("   tile", r, "run0", pa[r].tolist())
        print("   tile", r, "runi", pb[r].tolist())
