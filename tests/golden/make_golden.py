"""Generate the golden fixtures in tests/golden/ from the reference itself.

Run in the build container only (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Every number stored here is produced by the reference's own code
(warp.Lie / warp.Warp / model.planar.Graph / NeuralImageFunction, torch CPU fp32,
torch.optim.Adam), imported through ref_harness.py.  The fixtures are data only
(inputs and expected outputs); no reference source is copied.
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as R  # noqa: E402

torch.set_num_threads(8)


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


# --------------------------------------------------------------------- Lie exp

def make_lie():
    warp, _, _, _ = R.import_reference()
    lie = warp.Lie()
    rng = np.random.default_rng(11)
    out = {}
    h64 = rng.normal(0, 0.1, (64, 8)).astype(np.float32)
    out["h_b64"], out["H_b64"] = h64, np32(lie.sl3_to_SL3(torch.from_numpy(h64)))
    hbig = rng.normal(0, 1.5, (16, 8)).astype(np.float32)
    out["h_big"], out["H_big"] = hbig, np32(lie.sl3_to_SL3(torch.from_numpy(hbig)))
    # batch of exactly one takes torch's degree-selection path
    hb1 = np.concatenate([rng.normal(0, s, (4, 8)) for s in (1e-9, 1e-5, 3e-3, 0.05, 0.2, 0.6, 2.0)]).astype(np.float32)
    out["h_b1"] = hb1
    out["H_b1"] = np.stack([np32(lie.sl3_to_SL3(torch.from_numpy(hb1[i:i + 1])))[0] for i in range(len(hb1))])
    # backward through matrix_exp (autograd), batch 5 and batch 1
    for tag, B in (("b5", 5), ("b1", 1)):
        h = rng.normal(0, 0.1, (B, 8)).astype(np.float32)
        dH = rng.normal(0, 1.0, (B, 3, 3)).astype(np.float32)
        ht = torch.from_numpy(h).requires_grad_()
        lie.sl3_to_SL3(ht).backward(torch.from_numpy(dH))
        out[f"bwd_h_{tag}"], out[f"bwd_dH_{tag}"], out[f"bwd_dh_{tag}"] = h, dH, np32(ht.grad)
    np.savez_compressed(os.path.join(HERE, "lie.npz"), **out)


# -------------------------------------------------------------------- prologue

def make_prologue():
    warp, planar, _, _ = R.import_reference()
    out = {}
    rng = np.random.default_rng(12)
    for tag, geo, B in (("c1", (360, 480, 180, 240), 5), ("c3", (512, 512, 256, 256), 3)):
        H, W, ph, pw = geo
        opt = R.make_opt({"H": H, "W": W, "patch_H": ph, "patch_W": pw, "batch_size": B})
        wp = warp.Warp(opt)
        xy = wp.get_normalized_pixel_grid(crop=True)
        full = wp.get_normalized_pixel_grid(crop=False)
        h = rng.normal(0, 0.05, (B, 8)).astype(np.float32)
        h[0] = 0
        uv = wp.warp_grid(xy, torch.from_numpy(h))
        N = xy.shape[1]
        idx = np.unique(np.concatenate([[0, N - 1], rng.integers(0, N, 1024)])).astype(np.int64)
        fidx = np.unique(np.concatenate([[0, full.shape[1] - 1], rng.integers(0, full.shape[1], 512)]))
        out[f"{tag}_geo"] = np.array([H, W, ph, pw, B], np.int64)
        out[f"{tag}_h"] = h
        out[f"{tag}_H"] = np32(warp.Lie().sl3_to_SL3(torch.from_numpy(h)))
        out[f"{tag}_idx"] = idx
        out[f"{tag}_xy"] = np32(xy[0, idx])
        out[f"{tag}_uv"] = np32(uv[:, idx])
        out[f"{tag}_full_idx"] = fidx
        out[f"{tag}_full_xy"] = np32(full[0, fidx])
        out[f"{tag}_corners"] = np32(wp.warp_corners(torch.from_numpy(h)))
        # posenc (+ c2f) at the sampled warped coordinates
        for L, c2f, plist in ((8, [0, 0.4], (0.0, 0.125, 0.2, 0.39, 1.0)), (16, [0, 0.4], (0.2,)),
                              (8, None, (0.0,)), (10, [0, 0.4], (0.3,))):
            o2 = R.make_opt({"H": H, "W": W, "patch_H": ph, "patch_W": pw, "batch_size": B,
                             "arch": {"posenc": {"L_2D": L}}, "barf_c2f": c2f})
            ni = planar.NeuralImageFunction(o2)
            for p in plist:
                ni.progress.data.fill_(p)
                enc = ni.positional_encoding(uv[:, idx[:256]])
                key = f"{tag}_enc_L{L}_{'c2f' if c2f else 'full'}_p{p}"
                out[key] = np32(enc)
    np.savez_compressed(os.path.join(HERE, "prologue.npz"), **out)


# ---------------------------------------------------------------- training step

def ref_train(opt, rgb, mask, warp_init=None, progress=None, steps=1, keep_full=True):
    """Mirror of Model.setup_optimizer + Model.train_iteration + the fix_first
    line of Model.train (model/planar.py:86-104, 187-209, 154-158), calling the
    reference's Graph and Model.summarize_loss."""
    _, planar, _, _ = R.import_reference()
    R.seed_all(opt.seed)
    graph = planar.Graph(opt)
    init = {k: np32(v) for k, v in graph.state_dict().items()}
    if warp_init is not None:
        graph.warp_param.weight.data.copy_(torch.from_numpy(warp_init))
    if progress is not None:
        graph.neural_image.progress.data.fill_(progress)
    optim = torch.optim.Adam([
        dict(params=graph.neural_image.parameters(), lr=opt.optim.lr),
        dict(params=graph.warp_param.parameters(), lr=opt.optim.lr_warp)])
    B, _, h, w = rgb.shape
    var = R.EasyDict(idx=torch.arange(B))
    var.images = R.EasyDict(rgb=torch.from_numpy(rgb), masks=torch.from_numpy(mask),
                            masks_eroded=torch.from_numpy(mask),
                            edges=torch.zeros(B, 1, h, w, dtype=torch.float64))
    fake_model = R.EasyDict(opt=opt)
    res = {"init": init, "loss": [], "warp": [], "progress": []}
    it = 0
    for s in range(steps):
        optim.zero_grad()
        var = graph.forward(var, mode="train")
        loss = graph.compute_loss(var, mode="train")
        loss = planar.Model.summarize_loss(fake_model, loss)
        loss.all.backward()
        if s == 0:
            res["rgb0"] = np32(var.rgb_prediction)
            res["grads0"] = {k: np32(p.grad) for k, p in graph.named_parameters() if p.grad is not None}
            res["loss_all0"] = float(loss.all)
        optim.step()
        it += 1
        graph.neural_image.progress.data.fill_(it / opt.max_iter)
        if opt.warp.fix_first:
            graph.warp_param.weight.data[0] = 0
        res["loss"].append(float(loss.rgb))
        res["warp"].append(np32(graph.warp_param.weight))
        res["progress"].append(float(graph.neural_image.progress))
    res["final"] = {k: np32(v) for k, v in graph.state_dict().items()}
    return res


def synth_images(B, h, w, seed):
    g = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    rgb = np.stack([np.stack([0.5 + 0.4 * np.sin(2 * np.pi * (f * xx + (c + 1) * yy) + b)
                              for c, f in enumerate((1.0, 2.0, 3.0))]) for b in range(B)])
    rgb = (rgb + 0.05 * g.standard_normal(rgb.shape)).clip(0, 1).astype(np.float32)
    mask = (g.random((B, 1, h, w)) < 0.85).astype(np.float32)
    return rgb, mask


def make_step_small():
    out = {}
    cases = {
        # tag: (overrides, progress)
        "a": ({"arch": {"layers": [None, 64, 64, 3], "posenc": {"L_2D": 8}}, "barf_c2f": [0, 0.4]}, 0.3),
        "b": ({"arch": {"layers": [None, 32, 32, 3], "posenc": None}, "barf_c2f": None}, None),
        "c": ({"arch": {"layers": [None, 48, 40, 3], "posenc": {"L_2D": 16}}, "barf_c2f": [0, 0.4]}, 0.2),
        "d": ({"arch": {"layers": [None, 64, 64, 64, 3], "posenc": {"L_2D": 8}}, "barf_c2f": None,
               "use_edges": False}, None),
    }
    rng = np.random.default_rng(13)
    for tag, (over, prog) in cases.items():
        geo = {"H": 36, "W": 48, "patch_H": 18, "patch_W": 24, "batch_size": 3, "max_iter": 50}
        geo.update(over)
        opt = R.make_opt(geo)
        rgb, mask = synth_images(3, 18, 24, seed=100 + ord(tag))
        warp0 = rng.normal(0, 0.03, (3, 8)).astype(np.float32)
        res = ref_train(opt, rgb, mask, warp_init=warp0, progress=prog, steps=6)
        L = opt.arch.posenc.L_2D if opt.arch.posenc else 0
        c2f = opt.barf_c2f
        out[f"{tag}_cfg"] = np.array([36, 48, 18, 24, 3, L, -1 if c2f is None else c2f[0],
                                      -1 if c2f is None else c2f[1], 50,
                                      -1 if prog is None else prog, 1 if opt.use_edges else 0], np.float64)
        out[f"{tag}_layers"] = np.array([2 + 4 * L] + list(opt.arch.layers[1:]), np.int64)
        out[f"{tag}_rgb"], out[f"{tag}_mask"], out[f"{tag}_warp0"] = rgb, mask, warp0
        for k, v in res["init"].items():
            out[f"{tag}_init_{k}"] = v
        for k, v in res["grads0"].items():
            out[f"{tag}_grad0_{k}"] = v
        for k, v in res["final"].items():
            out[f"{tag}_final_{k}"] = v
        out[f"{tag}_rgb0"] = res["rgb0"]
        out[f"{tag}_loss"] = np.array(res["loss"], np.float64)
        out[f"{tag}_warp_traj"] = np.stack(res["warp"])
        out[f"{tag}_loss_all0"] = np.array(res["loss_all0"])
    np.savez_compressed(os.path.join(HERE, "step_small.npz"), **out)


def make_step_skip():
    """arch.skip (model/planar.py:419-420, 440-441): the reference's Graph with skip layers, 6 steps,
    the same fields as step_small."""
    out = {}
    cases = {
        # tag: (overrides, progress)
        "s1": ({"arch": {"layers": [None, 64, 64, 64, 3], "skip": [2], "posenc": {"L_2D": 8}}, "barf_c2f": [0, 0.4]},
               0.3),
        "s2": ({"arch": {"layers": [None, 64, 64, 64, 64, 3], "skip": [1, 3], "posenc": {"L_2D": 4}}, "barf_c2f": None,
                "use_edges": False}, None),
    }
    rng = np.random.default_rng(17)
    for tag, (over, prog) in cases.items():
        geo = {"H": 36, "W": 48, "patch_H": 18, "patch_W": 24, "batch_size": 3, "max_iter": 50}
        geo.update(over)
        opt = R.make_opt(geo)
        rgb, mask = synth_images(3, 18, 24, seed=200 + ord(tag[1]))
        warp0 = rng.normal(0, 0.03, (3, 8)).astype(np.float32)
        res = ref_train(opt, rgb, mask, warp_init=warp0, progress=prog, steps=6)
        L = opt.arch.posenc.L_2D if opt.arch.posenc else 0
        c2f = opt.barf_c2f
        out[f"{tag}_cfg"] = np.array([36, 48, 18, 24, 3, L, -1 if c2f is None else c2f[0],
                                      -1 if c2f is None else c2f[1], 50,
                                      -1 if prog is None else prog, 1 if opt.use_edges else 0], np.float64)
        out[f"{tag}_layers"] = np.array([2 + 4 * L] + list(opt.arch.layers[1:]), np.int64)
        out[f"{tag}_skip"] = np.array(opt.arch.skip, np.int64)
        out[f"{tag}_rgb"], out[f"{tag}_mask"], out[f"{tag}_warp0"] = rgb, mask, warp0
        for k, v in res["init"].items():
            out[f"{tag}_init_{k}"] = v
        for k, v in res["grads0"].items():
            out[f"{tag}_grad0_{k}"] = v
        for k, v in res["final"].items():
            out[f"{tag}_final_{k}"] = v
        out[f"{tag}_rgb0"] = res["rgb0"]
        out[f"{tag}_loss"] = np.array(res["loss"], np.float64)
        out[f"{tag}_warp_traj"] = np.stack(res["warp"])
    np.savez_compressed(os.path.join(HERE, "step_skip.npz"), **out)


def load_cat_batch3(opt):
    D = os.path.join(R.REF, "data", "planar", opt.dataset)
    rgb = R.load_images_pil([f"{D}/{i}.png" for i in range(opt.batch_size)], opt)
    mask = R.load_images_pil([f"{D}/{i}-m.png" for i in range(opt.batch_size)], opt, mode="L",
                             invert_gray=True)
    return rgb.numpy(), mask.numpy()


def checks(a):
    a = np.asarray(a, np.float64)
    return np.array([a.sum(), np.abs(a).sum(), (a * a).sum(), a.ravel()[0], a.ravel()[-1]])


def make_step_c1(steps=10):
    """Real C1: cat_batch3, yaml + --seed=3 --barf_c2f=[0,0.4] (README.md:31)."""
    opt = R.make_opt()
    rgb, mask = load_cat_batch3(opt)
    res = ref_train(opt, rgb, mask, steps=steps)
    out = {"rgb_checks": checks(rgb), "mask_checks": checks(mask), "mask_sum": mask.sum(dtype=np.float64)}
    rng = np.random.default_rng(14)
    idx = np.unique(rng.integers(0, 5 * 43200, 4096))
    out["rgb0_idx"] = idx
    out["rgb0"] = res["rgb0"].reshape(-1, 3)[idx]
    out["rgb0_checks"] = checks(res["rgb0"])
    for k, v in res["init"].items():
        out[f"init_checks_{k}"] = checks(v)
    for k, v in res["grads0"].items():
        out[f"grad0_checks_{k}"] = checks(v)
        out[f"grad0_sample_{k}"] = v.ravel()[:: max(1, v.size // 512)]
    out["grad0_warp"] = res["grads0"]["warp_param.weight"]
    for k, v in res["final"].items():
        out[f"final_checks_{k}"] = checks(v)
    out["loss"] = np.array(res["loss"], np.float64)
    out["warp_traj"] = np.stack(res["warp"])
    np.savez_compressed(os.path.join(HERE, "step_c1.npz"), **out)
    # also save the loaded images (small) so GPU-box tests need no PIL decode parity
    np.savez_compressed(os.path.join(HERE, "cat_batch3_c1.npz"),
                        rgb=(rgb * 255).round().astype(np.uint8), mask=mask.astype(np.uint8))


# ----------------------------------------------------- module API (autograd, render, metric)

def make_api():
    """Gradients through Warp.warp_grid (warp.py:70-81) and positional_encoding
    (model/planar.py:451-471), the full-canvas render of Model.predict_entire_image
    (model/planar.py:211-217) from the seed-3 init, and Model.homography_error
    (model/planar.py:219-223)."""
    warp, planar, _, _ = R.import_reference()
    out = {}
    rng = np.random.default_rng(15)
    opt = R.make_opt()
    W = warp.Warp(opt)
    xy = W.get_normalized_pixel_grid(crop=True)[:, ::97].clone()  # [5, 446, 2] strided crop grid
    xy = xy + torch.from_numpy(rng.normal(0, 0.01, xy.shape).astype(np.float32))
    h = torch.from_numpy(rng.normal(0, 0.05, (5, 8)).astype(np.float32))
    G = torch.from_numpy(rng.normal(0, 1, xy.shape).astype(np.float32))
    xy_t, h_t = xy.clone().requires_grad_(), h.clone().requires_grad_()
    uv = W.warp_grid(xy_t, h_t)
    uv.backward(G)
    out.update(wg_xy=np32(xy), wg_h=np32(h), wg_G=np32(G), wg_uv=np32(uv), wg_dxy=np32(xy_t.grad), wg_dh=np32(h_t.grad))
    for L, prog, c2f in ((8, 0.3, [0, 0.4]), (10, 0.15, [0, 0.4]), (16, 0.2, [0, 0.4]), (10, 0.0, None)):
        o = R.make_opt({"arch": {"posenc": {"L_2D": L}}, "barf_c2f": c2f})
        R.seed_all(3)
        nif = planar.NeuralImageFunction(o)
        nif.progress.data.fill_(prog)
        c = torch.from_numpy(rng.uniform(-1, 1, (2, 300, 2)).astype(np.float32)).requires_grad_()
        enc = nif.positional_encoding(c)
        Ge = torch.from_numpy(rng.normal(0, 1, enc.shape).astype(np.float32))
        enc.backward(Ge)
        tag = f"pe_L{L}_{'c2f' if c2f else 'off'}"
        out.update({f"{tag}_cfg": np.array([L, prog, 1 if c2f else 0], np.float64), f"{tag}_coord": np32(c),
                    f"{tag}_enc": np32(enc), f"{tag}_G": np32(Ge), f"{tag}_dcoord": np32(c.grad)})
    # predict_entire_image: the seed-3 Graph, unwarped full 360x480 canvas, at two progress values
    R.seed_all(opt.seed)
    graph = planar.Graph(opt)
    full = W.get_normalized_pixel_grid()[:1]
    idx = np.arange(0, 360 * 480, 37)
    out["pred_idx"] = idx
    for prog in (0.0, 0.5):
        graph.neural_image.progress.data.fill_(prog)
        with torch.no_grad():
            rgb = graph.neural_image.forward(full)
        img = rgb.view(opt.H, opt.W, 3).permute(2, 0, 1)
        out[f"pred_p{prog}_sample"] = np32(rgb.view(-1, 3)[idx])
        out[f"pred_p{prog}_checks"] = checks(np32(img))
    # homography_error on fixed tensors
    ph = torch.from_numpy(rng.normal(0, 0.1, (5, 8)).astype(np.float32))
    gh = torch.from_numpy(np.eye(3, dtype=np.float32)[None] + rng.normal(0, 0.05, (5, 3, 3)).astype(np.float32))
    fake = R.EasyDict(lie=warp.Lie())
    out["he_pred"], out["he_gt"] = np32(ph), np32(gh)
    out["he_err"] = np.array(float(planar.Model.homography_error(fake, ph, gh)), np.float64)
    np.savez_compressed(os.path.join(HERE, "api.npz"), **out)


def make_step_c1_L10(steps=4):
    """BASELINE config 1 as written (L=10): cat_batch3, seed 3, c2f [0, 0.4], 4 iterations."""
    opt = R.make_opt({"arch": {"posenc": {"L_2D": 10}}})
    rgb, mask = load_cat_batch3(opt)
    res = ref_train(opt, rgb, mask, steps=steps)
    out = {}
    rng = np.random.default_rng(16)
    idx = np.unique(rng.integers(0, 5 * 43200, 4096))
    out["rgb0_idx"], out["rgb0"] = idx, res["rgb0"].reshape(-1, 3)[idx]
    for k, v in res["init"].items():
        out[f"init_checks_{k}"] = checks(v)
    for k, v in res["grads0"].items():
        out[f"grad0_checks_{k}"] = checks(v)
    out["grad0_warp"] = res["grads0"]["warp_param.weight"]
    out["loss"] = np.array(res["loss"], np.float64)
    out["warp_traj"] = np.stack(res["warp"])
    np.savez_compressed(os.path.join(HERE, "step_c1_L10.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["lie", "prologue", "small", "c1"]
    if "lie" in which:
        make_lie()
    if "prologue" in which:
        make_prologue()
    if "small" in which:
        make_step_small()
    if "c1" in which:
        make_step_c1()
    if "api" in which:
        make_api()
    if "c1L10" in which:
        make_step_c1_L10()
    if "skip" in which:
        make_step_skip()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
