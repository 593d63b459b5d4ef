"""3000-iteration cat_batch3 runs over several network-init seeds, fp32 vs bf16 (GPU).

The seed=3 trajectory is bimodal under perturbation: either patch 1's perspective row converges
(final PSNR ~26 dB) or it stalls in a second basin (23-25 dB).  A single seed therefore cannot say
whether a precision mode trains as well as fp32; the fraction of converged inits can.

    python tools/seed_sweep.py --seeds 0 1 2 3 4 5 6 7 --precisions fp32 bf16
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402,F401  (sets sys.path for the package and the checker)
import test_gpu_parity as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=list(range(8)))
    ap.add_argument("--precisions", nargs="+", default=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--perturb", type=int, nargs="+", default=[0],
                    help="ulp-perturbation draws of the init (0 = none); each seed runs every draw")
    ap.add_argument("--out", default="gpurun_out/seed_sweep.json")
    a = ap.parse_args()
    res = []
    for prec in a.precisions:
        for s, pt in [(s, pt) for s in a.seeds for pt in a.perturb]:
            t0 = time.time()
            with tempfile.TemporaryDirectory() as d:
                psnr, w = T._run_c1(prec, d, iters=a.iters, seed=s, perturb=pt)
            r = dict(precision=prec, seed=s, perturb=pt, psnr=float(psnr[-1]), psnr_mean10=float(np.mean(psnr[-10:])),
                     warps=w.tolist(), secs=round(time.time() - t0, 1), lib=os.environ.get("MARF_LIB", "default"),
                     warp_err=float(np.abs(w[1:] - T.REF_WARPS_3000).max()), psnr_traj=[float(x) for x in psnr])
            res.append(r)
            print(f"{prec:5s} seed {s} perturb {pt}: final PSNR {r['psnr']:.3f} dB (mean of last 10 logged {r['psnr_mean10']:.3f}) "
                  f"max |warp - ref| {r['warp_err']:.3e} in {r['secs']} s [{r['lib']}]", flush=True)
            os.makedirs(os.path.dirname(a.out), exist_ok=True)
            json.dump(res, open(a.out, "w"))
    for prec in a.precisions:
        p = np.array([r["psnr_mean10"] for r in res if r["precision"] == prec])
        print(f"{prec}: mean {p.mean():.3f} dB  median {np.median(p):.3f}  min {p.min():.3f}  max {p.max():.3f}  "
              f">=25.5 dB: {int((p >= 25.5).sum())}/{len(p)}")


if __name__ == "__main__":
    main()
