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


def test_product_refuses_cpu_tensors(lib):
    import torch
    import marf_hip
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        marf_hip.sl3_to_SL3(torch.zeros(2, 8))
