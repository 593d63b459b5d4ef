"""GPU check of the pixel-per-wave fused step (marf_step2.hip) against the tile kernel and fp32.

    python tools/step2_check.py
Prints per case: rgb / loss / gradient agreement of bf16 step2 vs the bf16 tile kernel, and of
bf16 / bf16x3 step2 vs the fp32 path, from the same state.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402,F401
import test_gpu_parity as T  # noqa: E402


def run(precision, step2, geo, seed=0, B=2, L=16, layers=(256, 256, 256, 256), prog=0.2, nw4=False):
    from model import planar
    from util import EasyDict as edict
    os.environ["MARF_STEP2"] = "1" if step2 else "0"
    os.environ["MARF_STEP2_NW4"] = "1" if nw4 else "0"
    H, W, ph, pw = geo
    opt = T.make_opt(None, H=H, W=W, patch_H=ph, patch_W=pw, batch_size=B, precision=precision,
                     arch={"layers": [None] + list(layers) + [3], "skip": [], "posenc": {"L_2D": L}})
    torch.manual_seed(seed)
    graph = planar.Graph(opt).to(T.DEV)
    graph.neural_image.progress.data.fill_(prog)
    graph.need_edges = False
    rng = np.random.default_rng(seed + 5)
    h, w = (ph // 2) * 2, (pw // 2) * 2
    gt = T.t(rng.random((B, 3, h, w)).astype(np.float32))
    mask = T.t((rng.random((B, 1, h, w)) < 0.85).astype(np.float32))
    with torch.no_grad():
        graph.warp_param.weight.copy_(T.t((rng.standard_normal((B, 8)) * 0.02).astype(np.float32)))
    var = edict(images=edict(rgb=gt, masks=mask, masks_eroded=mask, edges=None))
    v = graph.forward(var)
    loss = graph.compute_loss(v).rgb
    loss.backward()
    torch.cuda.synchronize()
    return (v.rgb_prediction.detach().clone(), float(loss), [p.grad.clone() for p in graph.neural_image.mlp.parameters()],
            graph.warp_param.weight.grad.clone())


def cmp(tag, a, b):
    ra, la, ga, wa = a
    rb, lb, gb, wb = b
    out = [f"rgb max {float((ra - rb).abs().max()):.2e}", f"loss rel {abs(la - lb) / abs(lb):.2e}"]
    cs = []
    for x, y in zip(ga, gb):
        cos = float((x * y).sum() / (x.norm() * y.norm() + 1e-30))
        rel = float((x - y).abs().max() / (y.abs().max() + 1e-30))
        cs.append((round(cos, 5), round(rel, 4)))
    wcos = float((wa * wb).sum() / (wa.norm() * wb.norm() + 1e-30))
    wrel = float((wa - wb).abs().max() / (wb.abs().max() + 1e-30))
    print(f"{tag}: " + ", ".join(out) + f"; grads (cos, maxrel) {cs}; warp cos {wcos:.5f} maxrel {wrel:.3e}", flush=True)


def main():
    T._need_gpu()
    for geo, B, L, layers in (((36, 48, 18, 24), 3, 8, (64, 64)), ((360, 480, 180, 240), 2, 8, (256,) * 4),
                              ((512, 512, 256, 256), 2, 16, (256,) * 4)):
        kw = dict(B=B, L=L, layers=layers)
        f32 = run("fp32", False, geo, **kw)
        old = run("bf16", False, geo, **kw)
        spl = run("bf16x3", True, geo, **kw)
        nw4 = run("bf16", True, geo, nw4=True, **kw)
        os.environ["MARF_STEP2_GRID"] = "7"
        few4 = run("bf16", True, geo, nw4=True, **kw)
        fews = run("bf16x3", True, geo, **kw)
        del os.environ["MARF_STEP2_GRID"]
        print(f"== geo {geo} B {B} L {L} layers {layers}")
        cmp("tile bf16 vs fp32", old, f32)
        cmp("step2 bf16x3 vs fp32", spl, f32)
        cmp("step2 bf16 (4 waves) vs fp32", nw4, f32)
        cmp("step2 bf16 (4 waves) grid 7 vs fp32", few4, f32)
        cmp("step2 bf16x3 grid 7 vs fp32", fews, f32)


if __name__ == "__main__":
    main()
