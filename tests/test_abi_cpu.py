"""CPU-side checks of the C-ABI boundary: libmarf.so builds, loads and exports exactly the entry
points include/marf.h declares; host-side planning calls that need no GPU behave."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "marf.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(marf_[A-Za-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import build_lib
    path = build_lib.build(verbose=False)
    return ctypes.CDLL(path)


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("marf_sl3_to_SL3", "marf_forward", "marf_backward", "marf_masked_mse", "marf_adam_step",
              "marf_pixel_grid", "marf_warp_points", "marf_posenc", "marf_net_create", "marf_last_error"):
        assert s in syms
    assert len(syms) >= 20


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_signatures_cover_header():
    import marf_hip
    assert set(marf_hip._SIGS) == set(declared_symbols())


def test_net_planning_without_gpu(lib):
    import marf_hip
    n = marf_hip.Net([34, 256, 256, 256, 256, 3], 8, marf_hip.MARF_BF16)
    assert n.param_count == 34 * 256 + 256 + 3 * (256 * 256 + 256) + 256 * 3 + 3 == 207107
    assert n.packed_bytes > 0
    g = marf_hip.grid_geometry(5, 360, 480, 180, 240, None)
    g.d_H = 1  # planning reads no device memory
    assert n.saved_bytes(g) > 5 * 43200 * 4 * 512
    assert n.workspace_bytes(g) > 0
    n32 = marf_hip.Net([66, 256, 256, 256, 256, 3], 16, marf_hip.MARF_FP32)
    assert n32.param_count == 215299


def test_net_create_rejects_bad_shapes(lib):
    import marf_hip
    with pytest.raises(RuntimeError, match="dims"):
        marf_hip.Net([35, 256, 3], 8, marf_hip.MARF_FP32)
    with pytest.raises(RuntimeError, match="output dim"):
        marf_hip.Net([34, 256, 4], 8, marf_hip.MARF_FP32)
    with pytest.raises(RuntimeError, match="512"):
        marf_hip.Net([34, 1024, 3], 8, marf_hip.MARF_BF16)


def test_skip_net_planning(lib):
    """marf_net_create_skip (opt.arch.skip, model/planar.py:419-420): a skip layer's weight is
    [out, in + 2+4L] in the flat parameter vector (torch's nn.Linear shapes, in layer order);
    skip into layer 0 or the output layer, a non-multiple-of-32 previous width and the split-bf16
    recipe are refused."""
    import marf_hip
    n = marf_hip.Net([34, 64, 64, 64, 3], 8, marf_hip.MARF_FP32, skip=[2])
    assert n.param_count == (34 * 64 + 64) + (64 * 64 + 64) + ((64 + 34) * 64 + 64) + (64 * 3 + 3)
    assert [s for _, s in n.layer_spans] == [35 * 64, 65 * 64, 99 * 64, 65 * 3]  # W_l then b_l
    assert n.step_kernel != "step2"
    for dt in (marf_hip.MARF_BF16, marf_hip.MARF_FP16):
        assert marf_hip.Net([18, 64, 64, 64, 64, 3], 4, dt, skip=[1, 3]).param_count == \
            (18 * 64 + 64) + (82 * 64 + 64) + (64 * 64 + 64) + (82 * 64 + 64) + (64 * 3 + 3)
    with pytest.raises(RuntimeError, match="skip connection"):
        marf_hip.Net([34, 64, 64, 3], 8, marf_hip.MARF_FP32, skip=[0])
    with pytest.raises(RuntimeError, match="skip connection"):
        marf_hip.Net([34, 64, 64, 3], 8, marf_hip.MARF_FP32, skip=[2])
    with pytest.raises(RuntimeError, match="multiple of 32"):
        marf_hip.Net([34, 60, 64, 3], 8, marf_hip.MARF_FP32, skip=[1])
    with pytest.raises(RuntimeError, match="skip"):
        marf_hip.Net([66, 256, 256, 256, 256, 3], 16, marf_hip.MARF_BF16X3, skip=[2])
    with pytest.raises(RuntimeError, match="512"):
        marf_hip.Net([66, 512, 512, 512, 3], 16, marf_hip.MARF_BF16, skip=[2])  # 512 + 96 inputs


def test_product_refuses_cpu_tensors(lib):
    import torch
    import marf_hip
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        marf_hip.sl3_to_SL3(torch.zeros(2, 8))


def test_split_recipe_kernel_choice(lib, monkeypatch):
    """marf_net_create_hint: the split recipe runs k_step2 at every size (its compile-time
    instantiations for full-width nets at L = 8, 9..12, 13..15, 16; the generic one otherwise), plain
    bf16 / fp32 the tile kernel k_mlp_step unless MARF_STEP2=1."""
    import marf_hip
    monkeypatch.delenv("MARF_STEP2", raising=False)
    c1 = 5 * 180 * 240
    c3 = 64 * 256 * 256
    full16 = [66, 256, 256, 256, 256, 3]
    for L in (8, 10, 13, 15, 16):
        dims = [2 + 4 * L, 256, 256, 256, 256, 3]
        for px in (c1, c3, 0):
            assert marf_hip.Net(dims, L, marf_hip.MARF_BF16X3, pixels_hint=px).step_kernel == "k_step2", (L, px)
    for px in (c1, c3, 0):
        assert marf_hip.Net([66, 128, 128, 3], 16, marf_hip.MARF_BF16X3, pixels_hint=px).step_kernel == "k_step2"
    assert marf_hip.Net(full16, 16, marf_hip.MARF_FP32, pixels_hint=c1).step_kernel == "k_mlp_step"
    assert marf_hip.Net(full16, 16, marf_hip.MARF_BF16, pixels_hint=c3).step_kernel == "k_mlp_step"
    monkeypatch.setenv("MARF_STEP2", "1")
    assert marf_hip.Net(full16, 16, marf_hip.MARF_BF16, pixels_hint=c3).step_kernel == "k_step2"
    monkeypatch.delenv("MARF_STEP2")
    spans = marf_hip.Net(full16, 16, marf_hip.MARF_BF16X3).layer_spans
    assert spans[0] == (0, 256 * 66 + 256) and sum(n for _, n in spans) == 215299


def test_bench_traffic_only_from_the_loaded_library(lib, tmp_path, monkeypatch):
    """bench.py reports PMC traffic only for an entry measured on the library it runs (same
    marf_source_hash) and on the same kernel (symbol prefix); anything else is null."""
    import json
    import sys
    import marf_hip
    sys.path.insert(0, ROOT)
    import bench
    have = marf_hip.lib().marf_source_hash().decode()
    (tmp_path / "profiles").mkdir()
    entry = {"source_hash": have, "source": "test", "kernels": {
        "mlp_step": {"symbol": "k_step2<256, true, 4, 4>", "hbm_read_bytes": 1.0, "hbm_write_bytes": 2.0, "pmc_avg_ns": 1.0}}}
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps({"c3/bf16x3": entry}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic("c3", "bf16x3", "mlp_step", "k_step2")[0] == 3.0
    assert bench.pmc_traffic("c3", "bf16x3", "mlp_step", "k_mlp_step") is None  # another kernel
    assert bench.pmc_traffic("c3", "bf16", "mlp_step", "k_step2") is None       # no entry
    entry["source_hash"] = "0" * 40
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps({"c3/bf16x3": entry}))
    assert bench.pmc_traffic("c3", "bf16x3", "mlp_step", "k_step2") is None     # another build


def test_fp16x2_recipe_planning(lib):
    """MARF_FP16X2 (the fp16-forward split recipe, k_step2h): full-width nets at L = 8..16 plan the
    two-set kernel with the same parameter layout as every recipe; other nets are refused at
    creation with the reason (no silent fallback to another kernel or recipe)."""
    import marf_hip
    for L in (8, 10, 13, 16):
        n = marf_hip.Net([2 + 4 * L, 256, 256, 256, 256, 3], L, marf_hip.MARF_FP16X2)
        assert n.step_kernel == "k_step2h", L
        assert n.layer_spans == marf_hip.Net([2 + 4 * L, 256, 256, 256, 256, 3], L, marf_hip.MARF_BF16X3).layer_spans
    for dims, L in (([34, 64, 64, 3], 8), ([18, 256, 256, 256, 256, 3], 4), ([66, 256, 128, 256, 256, 3], 16),
                    ([66, 256, 256, 256, 3], 16)):
        with pytest.raises(RuntimeError, match="fp16x2"):
            marf_hip.Net(dims, L, marf_hip.MARF_FP16X2)


def test_adam_schedule_matches_the_step_scalars(lib):
    """marf_adam_schedule (the device table a captured iteration's Adam reads, host only): row k-1
    = (lr / (1 - beta1^k), sqrt(1 - beta2^k)) in float64, rounded to float32 -- torch.optim.Adam's
    python-float bias corrections (model/planar.py:98-99), as marf_adam_step computes them."""
    import ctypes
    import math
    import numpy as np
    n = 3000
    buf = (ctypes.c_float * (2 * n))()
    assert lib.marf_adam_schedule(ctypes.c_double(1e-3), ctypes.c_double(0.9), ctypes.c_double(0.999),
                                  ctypes.c_longlong(1), ctypes.c_longlong(n), buf) == 0
    got = np.ctypeslib.as_array(buf).reshape(n, 2)
    for k in (1, 2, 3, 10, 100, 2999, 3000):
        ss = np.float32(1e-3 / (1 - 0.9 ** k))
        b2 = np.float32(math.sqrt(1 - 0.999 ** k))
        assert got[k - 1, 0] == ss and got[k - 1, 1] == b2, k
    assert lib.marf_adam_schedule(ctypes.c_double(1e-3), ctypes.c_double(0.9), ctypes.c_double(0.999),
                                  ctypes.c_longlong(0), ctypes.c_longlong(1), buf) != 0
