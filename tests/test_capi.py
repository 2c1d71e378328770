"""The C-ABI library loads and exports every symbol include/screenfit.h
declares (no compute calls; CPU)."""

import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "screenfit.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(sf_\w+)\s*\(",
                                 text, flags=re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("sf_create", "sf_destroy", "sf_set_basis", "sf_kl_fit",
              "sf_set_grid", "sf_kl_eval", "sf_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from ska_sdp_screen_fitting_amd._lib import EXPORTED, LIB_PATH
    assert os.path.exists(LIB_PATH), "build with __graft_entry__.build()"
    lib = ctypes.CDLL(LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert sorted(EXPORTED) == declared_symbols()


def test_version_and_errors_without_device():
    from ska_sdp_screen_fitting_amd._lib import load_library
    lib = load_library()
    assert b"gfx950" in lib.sf_version()
    h = ctypes.c_void_p()
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except ImportError:
        has_gpu = False
    if has_gpu:
        pytest.skip("a GPU is present")
    rc = lib.sf_create(0, ctypes.byref(h))
    assert rc == -19  # SF_ENODEV: no silent CPU fallback
    assert lib.sf_last_error()


def test_null_arguments_rejected():
    from ska_sdp_screen_fitting_amd._lib import load_library
    lib = load_library()
    assert lib.sf_create(0, None) == -22
    assert lib.sf_set_basis(None, None, 3, 100.0, 5 / 3) == -22
    assert lib.sf_kl_eval(None, None, 1, None, 1, 0) == -22


def test_missing_library_fails_loudly(tmp_path):
    from ska_sdp_screen_fitting_amd._lib import ScreenFitError, load_library
    with pytest.raises(ScreenFitError):
        load_library(str(tmp_path / "nope.so"))


def test_device_operands_are_checked_on_the_host():
    """Host-side operand checks of the Python binding (no GPU needed for
    these paths): host arrays and CPU tensors never reach a kernel."""
    import numpy as np
    from ska_sdp_screen_fitting_amd._lib import _dev
    torch = pytest.importorskip("torch")
    with pytest.raises(TypeError):
        _dev(np.zeros(4), np.float64, 4, "coef")
    with pytest.raises(ValueError):
        _dev(torch.zeros(4, dtype=torch.float64), np.float64, 4, "coef")
    assert _dev(None, np.float64, 4, "resid") is None
    assert _dev(1234, np.float64, 4, "raw") == 1234
