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

NAMES = ["prologue", "L0 gemm", "L0 epi", "L1 gemm", "L1 epi", "L2 gemm", "L2 epi", "L3 gemm", "L3 epi+last+loss",
         "lossred+dWlast", "dg4", "dg3", "dg2", "dg1", "adjoint"]


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
    st = torch.zeros(n_tiles * 16, dtype=torch.int64, device=dev)
    lib = marf_hip.lib()
    for it in range(3):
        lib.marf_debug_set_stamps(st.data_ptr() if it == 2 else None)
        v = m.graph.forward(var, mode="train")
        torch.cuda.synchronize()
    lib.marf_debug_set_stamps(None)
    s = st.view(n_tiles, 16).cpu().numpy().astype(np.float64)
    d = np.diff(s, axis=1)
    t0 = s[:, 0].min()
    print(f"tiles {n_tiles}; kernel span {(s[:, 15].max() - t0):.0f} ticks; mean tile life {(s[:, 15] - s[:, 0]).mean():.0f}")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:22s} mean {d[:, i].mean():9.0f}  p10 {np.percentile(d[:, i], 10):9.0f}  p90 {np.percentile(d[:, i], 90):9.0f}")


if __name__ == "__main__":
    main()
