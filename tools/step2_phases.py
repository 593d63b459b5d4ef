"""Per-phase cycle split of the pixel-per-wave fused step (diagnostic build with MARF_STAMPS):
    MARF_LIB=.../libmarf_stamps.so python tools/step2_phases.py [--precision bf16x3]
Wave 0 of each block sums s_memtime deltas per category over its tiles; printed as the mean over
blocks, in cycles per tile and as a share of the tile loop."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd"))
import bench  # noqa: E402

NAMES = ["stage wait+barrier", "DMA issue", "backward (BWL..BW0)", "dH tail", "prologue", "forward (FW0..FWH)",
         "last layer + dW_last", "tile loop total", "  in fwd GEMM bodies", "  in dgrad GEMM bodies",
         "  fwd tile finish (frag regs, mask, stores)", "  dgrad tile finish (frag regs, stores)",
         "  stage vmcnt/lgkmcnt wait (of wait+barrier)", "  fwd epilogue steps outside GEMM bodies",
         "  forward layer 0 (of forward)", "  fwd bias init"]


NAMES3 = ["stage vmcnt/lgkmcnt wait", "barrier", "DMA issue", "prologue", "forward layer 0", "forward hidden layers",
          "  in fwd GEMM bodies", "  fwd epilogue + stores", "last layer + loss", "dW_last",
          "dgrad (last + hidden)", "  in dgrad GEMM bodies", "  dgrad epilogue + stores", "layer-0 adjoint",
          "dH tail", "tile loop total"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16x3")
    ap.add_argument("--kernel", default="step2", choices=["step2", "step3"],
                    help="step3: the two-waves-per-SIMD kernel (marf_step3.hip, MARF_STEP3=1)")
    args = ap.parse_args()
    names, total_col = (NAMES3, 15) if args.kernel == "step3" else (NAMES, 7)
    os.environ["MARF_STEP3"] = "1" if args.kernel == "step3" else "0"  # (C3's size alone picks k_step2)
    import marf_hip
    from model import planar
    from util import EasyDict as edict
    dev = torch.device("cuda", 0)
    opt = bench.make_opt("c3", args.precision, 64)
    opt.device = str(dev)
    torch.manual_seed(3)
    m = planar.Model(opt)
    rgb, mask, warp = bench.synthetic_inputs(64, 256, 256, dev)
    m.images = edict(rgb=rgb, masks=mask, masks_eroded=mask, edges=None, gt_hom=None, gt=None)
    m.build_networks()
    m.graph.warp_param.weight.data.copy_(warp)
    m.graph.neural_image.progress.data.fill_(0.2)
    m.graph.need_edges = False
    var = edict(images=m.images)
    stamps = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
    marf_hip.lib().marf_debug_set_stamps(marf_hip._ptr(stamps))
    for _ in range(3):
        v = m.graph.forward(var)
        m.graph.compute_loss(v).rgb.backward()
    torch.cuda.synchronize()
    st = stamps.view(-1, 16).cpu().numpy().astype(np.float64)[:, :16]
    st = st[st[:, total_col] > 0]
    tiles = 4194304 // 128 / len(st)
    mean = st.mean(0) / tiles
    for n, v in zip(names, mean):
        print(f"{n:24s} {v:10.0f} cycles/tile  {100 * v / mean[total_col]:5.1f} %")


if __name__ == "__main__":
    main()
