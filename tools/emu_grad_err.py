"""Per-step gradient error of emulated precision recipes (GPU): the fp32 kernels of a MARF_DIAG_RT
build (MARF_LIB) round each operand class as a recipe would (MARF_DIAG_PREC codes, marf_common.h
diag_round), and one fused step on a C3-shaped problem is compared with the reference's ops in
float64 (tests/test_gpu_parity.py _compare_step): which rounding sets the error of d warp and of the
MLP gradients.

    MARF_LIB=.../libmarf_rtg.so python tools/emu_grad_err.py name=CODE [name=CODE ...]
"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402,F401
import test_gpu_parity as T  # noqa: E402


def main():
    shape = os.environ.get("EMU_SHAPE", "c3x2")
    args = dict(c3x2=(2, 256, 16, [256] * 4), c1=(5, 128, 8, [256] * 4))[shape]
    for spec in sys.argv[1:]:
        name, code = spec.split("=", 1)
        os.environ["MARF_DIAG_PREC"] = code
        with tempfile.TemporaryDirectory() as d:
            m, var, inputs = T._synthetic_setup("fp32", d, *args)
            o = T._compare_step(m, var, inputs, name, 5)
        print(f"{shape} {name:10s} {code:28s} rgb {o['rgb']:.3g} grad_err {o['grad_err']:.3g} (ref32 {o['grad_err_ref32']:.3g}) "
              f"dh_err {o['dh_err']:.3g} (ref32 {o['dh_err_ref32']:.3g}) dh_cos {o['dh_cos']:.6f}", flush=True)


if __name__ == "__main__":
    main()
