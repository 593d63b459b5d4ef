"""Full 3000-iteration seed-3 cat_batch3 runs of the REFERENCE itself (torch CPU fp32), to pin
what "final PSNR within 0.05 dB / warps within 1e-2 of the reference" can mean for any arithmetic
that is not bit-identical to torch-CPU.

Run in the build container only (needs /root/reference; ~40 min per run on 4 threads):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ref_runs.py <tag> [perturb_ulps]

tag "base": the unperturbed run (PSNR every freq.scalar = 20 iterations, final warps).
tag "ulp1": every MLP weight and bias multiplied by (1 + 2^-23) after init (a 1-ulp perturbation),
the same loop otherwise: how far the reference drifts from itself.
Writes tests/golden/ref_c1_3000_<tag>.npz (data only: trajectories and final warps).
"""
import os
import sys
import time

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as R  # noqa: E402
from make_golden import load_cat_batch3  # noqa: E402


def main():
    tag = sys.argv[1]
    threads = int(os.environ.get("REF_THREADS", "4"))
    torch.set_num_threads(threads)
    _, planar, _, _ = R.import_reference()
    opt = R.make_opt()
    rgb, mask = load_cat_batch3(opt)
    R.seed_all(opt.seed)
    graph = planar.Graph(opt)
    if tag == "ulp1":
        with torch.no_grad():
            for p in graph.neural_image.mlp.parameters():
                p.mul_(1 + 2.0 ** -23)
    optim = torch.optim.Adam([
        dict(params=graph.neural_image.parameters(), lr=opt.optim.lr),
        dict(params=graph.warp_param.parameters(), lr=opt.optim.lr_warp)])
    B, _, h, w = rgb.shape
    var = R.EasyDict(idx=torch.arange(B))
    var.images = R.EasyDict(rgb=torch.from_numpy(rgb), masks=torch.from_numpy(mask),
                            masks_eroded=torch.from_numpy(mask),
                            edges=torch.zeros(B, 1, h, w, dtype=torch.float64))
    fake_model = R.EasyDict(opt=opt)
    psnr, warps, its = [], [], []
    t0 = time.time()
    for it in range(opt.max_iter):
        optim.zero_grad()
        var = graph.forward(var, mode="train")
        loss = graph.compute_loss(var, mode="train")
        loss = planar.Model.summarize_loss(fake_model, loss)
        loss.all.backward()
        optim.step()
        graph.neural_image.progress.data.fill_((it + 1) / opt.max_iter)
        if opt.warp.fix_first:
            graph.warp_param.weight.data[0] = 0
        if (it + 1) % opt.freq.scalar == 0:
            psnr.append(float(-10 * torch.log10(loss.rgb.detach())))
            warps.append(graph.warp_param.weight.detach().numpy().copy())
            its.append(it + 1)
            if (it + 1) % 300 == 0:
                print(f"[{tag}] it {it + 1}: PSNR {psnr[-1]:.4f} ({time.time() - t0:.0f} s)", flush=True)
    np.savez_compressed(os.path.join(HERE, f"ref_c1_3000_{tag}.npz"), its=np.array(its), psnr=np.array(psnr),
                        warps=np.stack(warps).astype(np.float32))
    print(f"[{tag}] final PSNR {psnr[-1]:.4f}, mean of last 10 logged {np.mean(psnr[-10:]):.4f}")


if __name__ == "__main__":
    main()
