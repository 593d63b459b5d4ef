"""train.py end to end on the GPU box (SURVEY.md §8(a) a12 + the CLI of the reference's train.py:11-31):
the pre-decoded cat_batch3 inputs (--dataset_npz), seed 3, c2f [0, 0.4], the full 3000 iterations
(progress = it / max_iter drives the c2f schedule, so a shorter run is a different experiment) in
the benchmarked bf16x3 recipe and in fp32, frames every 100 iterations.  Checks that the run
completes, writes its options, scalar log and frames, and that the final logged PSNR and the mean of
the last 10 logged values are each within 0.05 dB of the nearest of the reference's own three runs
(tests/psnr_rule.py)."""
import json
import os
import subprocess
import sys

import pytest

import psnr_rule
from conftest import GOLDEN, PKG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["bf16x3", "fp32"])
def test_train_py_dataset_npz(precision, tmp_path):
    """bf16x3 runs the default step kernel of the recipe, the one bench.py measures."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    env.pop("MARF_STEP3", None)
    cmd = [sys.executable, "train.py", "--group=smoke", "--model=planar", "--yaml=planar", f"--name={precision}",
           "--seed=3", "--barf_c2f=[0,0.4]", f"--dataset_npz={os.path.join(GOLDEN, 'cat_batch3_c1.npz')}",
           f"--precision={precision}", f"--output_root={tmp_path}"]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=270, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = tmp_path / "smoke" / f"{precision}_seed3"  # the run name gains _seed<N> (options.py:99-104)
    assert (out / "options.yaml").exists()
    rows = [json.loads(x) for x in (out / "metrics.jsonl").read_text().splitlines()]
    psnr = {row["step"]: row["train/PSNR"] for row in rows}
    assert sorted(psnr)[:3] == [20, 40, 60] and max(psnr) == 3000, sorted(psnr)[-3:]
    frames = sorted(int(f.split(".")[0]) for f in os.listdir(out / "vis"))  # frame 0 + one per 100 iterations
    assert frames == list(range(31)), frames
    print(precision, {k: round(v, 3) for k, v in sorted(psnr.items()) if k % 300 == 0})
    last10 = [psnr[k] for k in sorted(psnr)[-10:]]
    ok, msg = psnr_rule.psnr_check(psnr[3000], sum(last10) / 10)
    print(precision, msg)
    assert ok, msg
