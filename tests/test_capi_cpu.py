"""CPU: the HIP library loads, exports every symbol the C ABI header declares, and reports
errors through status codes (no compute without a GPU)."""
import ctypes as C

import numpy as np
import pytest


def test_library_exports_every_declared_symbol(pkg):
    L = pkg.lib()
    names = pkg.declared_symbols()
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_version_and_error_string(pkg):
    L = pkg.lib()
    assert L.aiy_version() >= 100
    assert isinstance(L.aiy_last_error(), bytes)


def test_unsorted_grid_rejected_before_device(pkg):
    a = np.array([0.0, 2.0, 1.0])
    with pytest.raises(pkg.AiyError) as e:
        pkg.vfi_sweep(np.zeros((2, 3)), a, np.ones(2), np.eye(2), 0.04, 1.0, 0.96, 5.0)
    assert e.value.status == "AIY_BAD_ARG"


def test_nonfinite_grid_rejected(pkg):
    a = np.array([0.0, np.nan, 1.0])
    with pytest.raises(pkg.AiyError) as e:
        pkg.vfi_sweep(np.zeros((2, 3)), a, np.ones(2), np.eye(2), 0.04, 1.0, 0.96, 5.0)
    assert e.value.status == "AIY_NON_FINITE"


def test_no_device_is_loud(pkg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    a = np.linspace(0, 1, 5)
    with pytest.raises(pkg.AiyError) as e:
        pkg.vfi_sweep(np.zeros((2, 5)), a, np.ones(2), np.eye(2), 0.04, 1.0, 0.96, 5.0)
    assert e.value.status == "AIY_NO_DEVICE"
