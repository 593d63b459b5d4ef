"""Host data path: PNG -> LANCZOS thumbnail -> tensors, inverted masks, and the
text homographies, against the images the reference's own loader produced (tests/golden/
cat_batch3_c1.npz, written by tests/golden/make_golden.py from inputs.load_images,
reference inputs.py:16-33).  Reads the reference's data files in place, so it runs only where
/root/reference is present (this container); no kernels run."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

DATA = "/root/reference/data/planar/cat_batch3"
pytestmark = pytest.mark.skipif(not os.path.isdir(DATA), reason="reference data not present")


def _opt():
    from util import EasyDict as edict
    return edict(use_cropped_images=True, patch_W=240, patch_H=180, H=360, W=480, device="cpu")


def test_load_images_matches_reference_loader():
    import inputs
    opt = _opt()
    z = np.load(os.path.join(GOLDEN, "cat_batch3_c1.npz"))
    rgb = inputs.load_images([f"{DATA}/{i}.png" for i in range(5)], opt)
    mask = inputs.load_images([f"{DATA}/{i}-m.png" for i in range(5)], opt, mode="L", invert_gray=True)
    assert rgb.dtype == torch.float32 and tuple(rgb.shape) == (5, 3, 180, 240)
    assert tuple(mask.shape) == (5, 1, 180, 240)
    np.testing.assert_array_equal((rgb.numpy() * 255).round().astype(np.uint8), z["rgb"])
    np.testing.assert_array_equal(mask.numpy().astype(np.uint8), z["mask"])
    assert set(np.unique(mask.numpy()).tolist()) <= {0.0, 1.0}


def test_load_homography_text_format():
    """load_homography (reference inputs.py:87-105): identity row for patch 0, the .mat text
    matrices, kornia normalize_homography with the reference's (width, height) passed as
    (height, width): N = [[2/(height-1), 0, -1], [0, 2/(width-1), -1], [0, 0, 1]]."""
    import inputs
    fps = [f"{DATA}/H_0_{i}.mat" for i in range(1, 5)]
    H = inputs.load_homography(fps, 480, 360, "cpu").numpy().astype(np.float64)
    raw = np.concatenate([np.eye(3)[None], np.stack([np.loadtxt(f) for f in fps]).astype(np.float32)])
    N = np.array([[2 / (360 - 1), 0, -1], [0, 2 / (480 - 1), -1], [0, 0, 1]])
    ref = N @ raw @ np.linalg.inv(N)
    assert H.shape == (5, 3, 3)
    np.testing.assert_allclose(H, ref, rtol=1e-5, atol=1e-6)
