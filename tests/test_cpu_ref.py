"""The torch-CPU restatement (oracle/cpu_ref.py, the bench's CPU baseline) against the fixtures
generated from the reference: the same small cases and C1 steps that pin oracle.py."""
import numpy as np
import pytest

import cpu_ref
from test_oracle_golden import reference_init


def _case(g, tag):
    H, W, ph, pw, B, L, c0, c1, max_iter, prog, use_edges = g[f"{tag}_cfg"]
    layers = g[f"{tag}_layers"]
    params = [(g[f"{tag}_init_neural_image.mlp.{i}.weight"], g[f"{tag}_init_neural_image.mlp.{i}.bias"])
              for i in range(len(layers) - 1)]
    c = dict(H=int(H), W=int(W), patch_H=int(ph), patch_W=int(pw), L=int(L), c2f=None if c0 < 0 else [c0, c1],
             max_iter=int(max_iter), lr=1e-3, lr_warp=1e-3, fix_first=True, use_edges=bool(use_edges),
             alpha_initial=0.0, alpha_final=1.0,
             skip=tuple(int(x) for x in g[f"{tag}_skip"]) if f"{tag}_skip" in g.files else ())
    st = cpu_ref.CpuRefStep(c, params, g[f"{tag}_warp0"], g[f"{tag}_rgb"], g[f"{tag}_mask"])
    if prog >= 0:
        st.progress.data.fill_(float(prog))
    return st, len(layers) - 1


@pytest.mark.parametrize("fix,tag", [("step_small", "a"), ("step_small", "b"), ("step_small", "c"),
                                     ("step_small", "d"), ("step_skip", "s1"), ("step_skip", "s2")])
def test_small_step_vs_reference(golden, fix, tag):
    g = golden(fix)
    st, nl = _case(g, tag)
    r = st.step()
    np.testing.assert_allclose(r["rgb"].reshape(g[f"{tag}_rgb0"].shape), g[f"{tag}_rgb0"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(r["loss_rgb"], g[f"{tag}_loss"][0], rtol=1e-6)
    for i in range(nl):
        for j, name in enumerate(("weight", "bias")):
            ref = g[f"{tag}_grad0_neural_image.mlp.{i}.{name}"]
            assert np.abs(r["grads"][i][j] - ref).max() / (np.abs(ref).max() + 1e-12) < 1e-5, (tag, i, name)
    ref = g[f"{tag}_grad0_warp_param.weight"]
    assert np.abs(r["dh"] - ref).max() / (np.abs(ref).max() + 1e-12) < 1e-5
    losses = [r["loss_rgb"]]
    traj = [st.warp.detach().numpy().copy()]
    for _ in range(5):
        losses.append(st.step()["loss_rgb"])
        traj.append(st.warp.detach().numpy().copy())
    np.testing.assert_allclose(losses, g[f"{tag}_loss"], rtol=1e-5)
    np.testing.assert_allclose(np.stack(traj), g[f"{tag}_warp_traj"], atol=1e-6, rtol=0)


def test_c1_first_steps_vs_reference(golden):
    g = golden("step_c1")
    imgs = golden("cat_batch3_c1")
    rgb = imgs["rgb"].astype(np.float32) / np.float32(255)
    mask = imgs["mask"].astype(np.float32)
    params = reference_init([256, 256, 256, 256, 3], 34, [0, 0.4], 3, 5)
    cfg = dict(H=360, W=480, patch_H=180, patch_W=240, L=8, c2f=[0, 0.4], max_iter=3000, lr=1e-3, lr_warp=1e-3,
               fix_first=True, use_edges=True, alpha_initial=0.0, alpha_final=1.0)
    cpu_ref.set_threads()
    st = cpu_ref.CpuRefStep(cfg, params, np.zeros((5, 8), np.float32), rgb, mask)
    r = st.step()
    np.testing.assert_allclose(r["loss_rgb"], 0.050604186952114105, rtol=1e-6)
    np.testing.assert_allclose(r["rgb"][g["rgb0_idx"]], g["rgb0"], atol=1e-6)
    np.testing.assert_allclose(r["dh"], g["grad0_warp"], atol=1e-5 * np.abs(g["grad0_warp"]).max())
    losses = [r["loss_rgb"]]
    for _ in range(3):
        losses.append(st.step()["loss_rgb"])
    np.testing.assert_allclose(losses, g["loss"][:4], rtol=1e-6)


def test_api_autograd_vs_reference(golden):
    """cpu_ref's warp_grid / positional_encoding under torch autograd against the reference's."""
    import torch
    z = golden("api")
    xy = torch.from_numpy(z["wg_xy"]).requires_grad_()
    h = torch.from_numpy(z["wg_h"]).requires_grad_()
    uv = cpu_ref.warp_grid(xy, h)
    np.testing.assert_allclose(uv.detach().numpy(), z["wg_uv"], atol=1e-6, rtol=0)
    uv.backward(torch.from_numpy(z["wg_G"]))
    np.testing.assert_allclose(xy.grad.numpy(), z["wg_dxy"], rtol=1e-5, atol=1e-6 * np.abs(z["wg_dxy"]).max())
    np.testing.assert_allclose(h.grad.numpy(), z["wg_dh"], rtol=1e-5, atol=1e-6 * np.abs(z["wg_dh"]).max())
    for tag in ("pe_L8_c2f", "pe_L10_c2f", "pe_L16_c2f", "pe_L10_off"):
        L, prog, on = z[f"{tag}_cfg"]
        c = torch.from_numpy(z[f"{tag}_coord"]).requires_grad_()
        enc = cpu_ref.positional_encoding(c, int(L), torch.tensor(float(prog)), [0, 0.4] if on else None)
        np.testing.assert_allclose(enc.detach().numpy(), z[f"{tag}_enc"], atol=1e-7, rtol=0)
        enc.backward(torch.from_numpy(z[f"{tag}_G"]))
        np.testing.assert_allclose(c.grad.numpy(), z[f"{tag}_dcoord"], rtol=1e-5,
                                   atol=1e-6 * np.abs(z[f"{tag}_dcoord"]).max())
