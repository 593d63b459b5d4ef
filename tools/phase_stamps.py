"""Per-phase timing of the fused step kernel from in-kernel s_memtime stamps (wave 0 of every
block).  Needs the diagnostic library: python masking-bundle-adjusting-neural-radiance-fields_amd/build_lib.py --stamps
Run on the GPU box:  MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so python tools/phase_stamps.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd"))
os.environ.setdefault("MARF_LIB", os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd", "lib",
                                               "libmarf_stamps.so"))
import bench  # noqa: E402
import marf_hip  # noqa: E402
from model import planar  # noqa: E402
from util import EasyDict as edict  # noqa: E402

# (name, from slot, to slot)
PHASES = [("start+c2f", 0, 19), ("prologue", 19, 1), ("L0 gemm", 1, 2), ("L0 epi", 2, 3), ("L1 gemm", 3, 4),
          ("L1 epi", 4, 5), ("L2 gemm", 5, 6), ("L2 epi", 6, 7), ("L3 gemm", 7, 8), ("L3 epi+last+loss", 8, 9),
          ("lossred+dWlast", 9, 10), ("dg4", 10, 11), ("dg3", 11, 12), ("dg2", 12, 13), ("dg1", 13, 14),
          ("adj gemm0", 14, 16), ("adj df scatter", 16, 17), ("adj posenc", 17, 18), ("adj warp+dH", 18, 15)]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    dev = torch.device("cuda", 0)
    opt = bench.make_opt(cfg, "bf16", bench.CONFIGS[cfg][2])
    opt.device = str(dev)
    torch.manual_seed(3)
    m = planar.Model(opt)
    B = bench.CONFIGS[cfg][2]
    rgb, mask, warp = bench.synthetic_inputs(B, opt.patch_H, opt.patch_W, dev)
    m.images = edict(rgb=rgb, masks=mask, masks_eroded=mask, edges=None, gt_hom=None, gt=None)
    m.build_networks()
    m.graph.warp_param.weight.data.copy_(warp)
    m.graph.neural_image.progress.data.fill_(0.2)
    var = edict(idx=torch.arange(B), images=m.images)
    n_tiles = B * ((opt.patch_H * opt.patch_W + 127) // 128)
    st = torch.zeros(n_tiles * 32, dtype=torch.int64, device=dev)
    lib = marf_hip.lib()
    for it in range(3):
        lib.marf_debug_set_stamps(st.data_ptr() if it == 2 else None)
        v = m.graph.forward(var, mode="train")
        torch.cuda.synchronize()
    lib.marf_debug_set_stamps(None)
    s = st.view(n_tiles, 32).cpu().numpy().astype(np.float64)
    print(f"tiles {n_tiles}; mean tile life {(s[:, 15] - s[:, 0]).mean():.0f} ticks")
    for nm, a, b in PHASES:
        d = s[:, b] - s[:, a]
        print(f"  {nm:22s} mean {d.mean():9.0f}  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f}")


if __name__ == "__main__":
    main()
