"""train.py end to end on the GPU box (SURVEY.md §8(a) a12 + the CLI of the reference's train.py:11-31):
the pre-decoded cat_batch3 inputs (--dataset_npz), seed 3, c2f [0, 0.4], a few hundred iterations
in the benchmarked bf16x3 recipe and in fp32.  Checks that the run completes, writes its options
and scalar log, and that the logged PSNR follows the reference's early trajectory."""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, PKG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["bf16x3", "fp32"])
def test_train_py_dataset_npz(precision, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "train.py", "--group=smoke", "--model=planar", "--yaml=planar", f"--name={precision}",
           "--seed=3", "--barf_c2f=[0,0.4]", f"--dataset_npz={os.path.join(GOLDEN, 'cat_batch3_c1.npz')}",
           f"--precision={precision}", "--max_iter=300", f"--output_root={tmp_path}"]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = tmp_path / "smoke" / precision
    assert (out / "options.yaml").exists()
    rows = [json.loads(x) for x in (out / "metrics.jsonl").read_text().splitlines()]
    psnr = {row["step"]: row["train/PSNR"] for row in rows}
    assert sorted(psnr)[:3] == [20, 40, 60] and max(psnr) == 300, sorted(psnr)
    # the reference's own run passes 19.5 dB at iteration 300 (tests/golden/ref_c1_3000_base.npz)
    import numpy as np
    ref = np.load(os.path.join(GOLDEN, "ref_c1_3000_base.npz"))
    ref300 = float(ref["psnr"][list(ref["its"]).index(300)])
    print(precision, {k: round(v, 3) for k, v in sorted(psnr.items())}, "reference at 300:", ref300)
    assert psnr[300] > psnr[20] + 2.0
    assert abs(psnr[300] - ref300) < 0.5, (psnr[300], ref300)
