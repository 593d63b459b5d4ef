"""SE(2) warps: the north_star's "sl(3)/SE(2) Lie-exp patch warp".  The reference has the sl(3)
homography only (warp.py:72-80), so this warp type is an extension and its parity against the
reference is unpinned; it is pinned instead to exact mathematics:

  * se2_to_SE2(p) == torch.linalg.matrix_exp of the se(2) generator [[0,-th,tx],[th,0,ty],[0,0,0]]
    (CPU fp32), bit for bit -- the sl(3) kernel's matrix_exp is torch's, and the generator embeds in
    the reference's sl(3) layout exactly;
  * the closed form [[R(th), V(th) t], [0, 0, 1]] in float64 to 1e-5 (the accuracy of torch's fp32
    matrix_exp itself: its batch-of-one Taylor degree is off by ~1e-6 on |theta| ~ 0.3);
  * its gradient against float64 autograd to 1e-5 relative;
  * a training step with warp.type se2 equals the homography step on the embedded parameters bit for
    bit (rgb, MLP gradients), and the se(2) gradient is the embedding's adjoint of the sl(3) one.
"""
import numpy as np
import pytest
import torch

from test_gpu_parity import DEV, make_opt, t

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import marf_hip
    marf_hip.lib()
    yield


def generator(p):
    """[..., 3] (tx, ty, theta) -> the se(2) generator [..., 3, 3] (any dtype / device)."""
    tx, ty, th = p.unbind(-1)
    z = torch.zeros_like(th)
    return torch.stack([torch.stack([z, -th, tx], -1), torch.stack([th, z, ty], -1), torch.stack([z, z, z], -1)], -2)


def closed_form(p):
    tx, ty, th = p[:, 0], p[:, 1], p[:, 2]
    c, s = np.cos(th), np.sin(th)
    small = np.abs(th) < 1e-8
    a = np.where(small, 1.0, np.sin(th) / np.where(small, 1.0, th))
    b = np.where(small, 0.0, (1 - np.cos(th)) / np.where(small, 1.0, th))
    M = np.zeros((p.shape[0], 3, 3))
    M[:, 0, 0], M[:, 0, 1], M[:, 1, 0], M[:, 1, 1] = c, -s, s, c
    M[:, 0, 2] = a * tx - b * ty
    M[:, 1, 2] = b * tx + a * ty
    M[:, 2, 2] = 1
    return M


@pytest.mark.parametrize("B", [1, 5, 64])
def test_se2_exp_bitexact_and_closed_form(B):
    import marf_hip
    rng = np.random.default_rng(B)
    p = rng.standard_normal((B, 3)).astype(np.float32) * np.array([0.3, 0.3, 0.8], np.float32)
    H = marf_hip.se2_to_SE2(t(p)).cpu()
    ref = torch.linalg.matrix_exp(generator(torch.from_numpy(p)))  # torch CPU fp32, same batch
    assert torch.equal(H, ref)
    assert np.abs(H.numpy().astype(np.float64) - closed_form(p.astype(np.float64))).max() <= 1e-5


def test_se2_exp_gradient_vs_float64():
    import marf_hip
    rng = np.random.default_rng(7)
    B = 16
    p = rng.standard_normal((B, 3)).astype(np.float32) * 0.5
    g = rng.standard_normal((B, 3, 3)).astype(np.float32)
    pg = t(p).requires_grad_()
    (marf_hip.se2_to_SE2(pg) * t(g)).sum().backward()
    p64 = torch.from_numpy(p.astype(np.float64)).requires_grad_()
    (torch.linalg.matrix_exp(generator(p64)) * torch.from_numpy(g.astype(np.float64))).sum().backward()
    ref = p64.grad.numpy()
    err = np.abs(pg.grad.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= 1e-5, err


def test_warp_grid_se2_is_rigid():
    """Warp.warp_grid with an se2 warp moves points rigidly: pairwise distances are kept."""
    import warp as warp_mod
    opt = make_opt(warp={"type": "se2", "dof": 3}, batch_size=2)
    w = warp_mod.Warp(opt)
    xy = w.get_normalized_pixel_grid(crop=True)[:, ::997]  # [2, n, 2]
    p = t(np.array([[0.1, -0.05, 0.4], [0.0, 0.2, -1.1]], np.float32))
    uv = w.warp_grid(xy, p)
    d0 = torch.cdist(xy.double(), xy.double())
    d1 = torch.cdist(uv.double(), uv.double())
    assert (d0 - d1).abs().max().item() <= 1e-5


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_se2_step_equals_embedded_homography_step(precision, tmp_path):
    import marf_hip
    from model import planar
    from util import EasyDict as edict
    B = 3
    rng = np.random.default_rng(11)
    gt = t(rng.random((B, 3, 64, 64)).astype(np.float32))
    mask = t((rng.random((B, 1, 64, 64)) < 0.9).astype(np.float32))
    var = edict(images=edict(rgb=gt, masks=mask, masks_eroded=mask, edges=None))
    p = t((rng.standard_normal((B, 3)) * np.array([0.05, 0.05, 0.2])).astype(np.float32))
    arch = {"layers": [None, 128, 128, 3], "skip": [], "posenc": {"L_2D": 8}}
    out = {}
    for kind in ("se2", "homography"):
        opt = make_opt(tmp_path, H=128, W=128, patch_H=64, patch_W=64, batch_size=B, precision=precision, arch=arch,
                       warp={"type": kind, "dof": 3 if kind == "se2" else 8})
        torch.manual_seed(0)
        graph = planar.Graph(opt).to(DEV)
        graph.neural_image.progress.data.fill_(0.3)
        graph.need_edges = False
        with torch.no_grad():
            graph.warp_param.weight.copy_(p if kind == "se2" else marf_hip.se2_to_sl3(p))
        v = graph.forward(var)
        graph.compute_loss(v).rgb.backward()
        out[kind] = (v.rgb_prediction.detach().clone(), [q.grad.clone() for q in graph.neural_image.mlp.parameters()],
                     graph.warp_param.weight.grad.clone())
    rgb_s, g_s, dp = out["se2"]
    rgb_h, g_h, dh = out["homography"]
    assert torch.equal(rgb_s, rgb_h)
    assert all(torch.equal(a, b) for a, b in zip(g_s, g_h))
    # the embedding's adjoint: d tx = dh1, d ty = dh2, d theta = dh4 - dh3
    adj = torch.stack([dh[:, 0], dh[:, 1], dh[:, 3] - dh[:, 2]], -1)
    assert torch.equal(dp, adj)
