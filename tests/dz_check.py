"""Numerics check of the split-dz step (k_step2dz) against its emulation (numerics experiment).

    python tests/dz_check.py kernel <out.npz>      (product library: bf16x3 with and without MARF_STEP2_DZ)
    MARF_LIB=lib/libmarf_<diag_rt>.so python tests/dz_check.py emul <out.npz>
                                                   (MARF_DIAG_RT build: fp32 kernels rounding as each recipe)
    python tests/dz_check.py compare kernel.npz emul.npz

One fused step of the C3-shaped two-patch case of tests/test_gpu_parity.py; the MLP gradients and
d warp of each recipe.  A correct split-dz kernel sits as close to its emulation as the benchmarked
recipe sits to its own."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import conftest  # noqa: E402,F401  (the package / oracle paths, as under pytest)

EMUL = {"x3": "22211,2221,2221,2221,2222", "dz": "22211,2222,2222,2222,2222"}


def grads(precision, env):
    import tempfile
    import pathlib
    for k, v in env.items():
        os.environ[k] = v
    import test_gpu_parity as T
    m, var, _ = T._synthetic_setup(precision, pathlib.Path(tempfile.mkdtemp()), 2, 256, 16, [256] * 4)
    T.one_step_grads(m, var)
    g = [p.grad.detach().cpu().numpy().copy() for p in m.graph.neural_image.mlp.parameters()]
    return g + [m.graph.warp_param.weight.grad.detach().cpu().numpy().copy()]


def main():
    mode = sys.argv[1]
    if mode == "compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        for ka, kb in (("x3", "x3"), ("dz", "dz"), ("x3", "dz")):
            n = len([k for k in a.files if k.startswith(ka + "_")])
            errs = []
            for i in range(n):
                ga, gb = a[f"{ka}_{i}"], b[f"{kb}_{i}"]
                errs.append(float(np.abs(ga - gb).max() / (np.abs(gb).max() + 1e-30)))
            print(f"kernel {ka} vs emulated {kb}: MLP max rel {max(errs[:-1]):.3e}  d warp {errs[-1]:.3e}")
        return
    out = {}
    for name in ("x3", "dz"):
        if mode == "kernel":
            g = grads("bf16x3", {"MARF_STEP2_DZ": "1" if name == "dz" else "0"})
        else:
            g = grads("fp32", {"MARF_DIAG_PREC": EMUL[name]})
        for i, a in enumerate(g):
            out[f"{name}_{i}"] = a
    np.savez(sys.argv[2], **out)


if __name__ == "__main__":
    main()
