"""Gradient errors of the two split-bf16 step kernels against the float64 reference ops on the same
state (tests/test_gpu_parity.py _compare_step): k_step2 (MARF_STEP3=0) and k_step3 (MARF_STEP3=1),
at the C3 shape (L=16) and a C1-like shape (L=8), several seeds.   python tools/s3_err.py"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402,F401
import test_gpu_parity as T  # noqa: E402

for (B, crop, L) in ((2, 256, 16), (4, 180, 8)):
    for seed in (3, 4, 5):
        row = []
        for k in ("0", "1"):
            os.environ["MARF_STEP3"] = k
            with tempfile.TemporaryDirectory() as d:
                m, var, inputs = T._synthetic_setup("bf16x3", d, B, crop, L, [256] * 4, seed=seed)
                o = T._compare_step(m, var, inputs, "bf16x3", 5)
            row.append(o)
        print(f"B={B} crop={crop} L={L} seed={seed}: " + " | ".join(
            f"step{'3' if i else '2'} rgb {o['rgb']:.2e} grad {o['grad_err']:.2e} (ref32 {o['grad_err_ref32']:.2e}) "
            f"dh {o['dh_err']:.2e} (ref32 {o['dh_err_ref32']:.2e})" for i, o in enumerate(row)), flush=True)
