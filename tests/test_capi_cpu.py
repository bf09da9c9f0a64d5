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


def test_interpolating_entry_points_need_strict_grids(pkg):
    """interp1 / griddedInterpolant reject repeated points (MATLAB errors); the library returns
    AIY_BAD_ARG before any device work instead of dividing by a(k+1) - a(k) = 0."""
    a = np.array([0.0, 1.0, 1.0, 2.0])
    P = np.eye(2)
    with pytest.raises(pkg.AiyError) as e:
        pkg.sim_capital(np.zeros((2, 4)), a, P, 1, 0.5, np.full(9, 0.3))
    assert e.value.status == "AIY_BAD_ARG"
    with pytest.raises(pkg.AiyError) as e:
        pkg.dist_stationary(a, P, policy_k=np.zeros((2, 4)), lam0=np.full((2, 4), 0.125),
                            tol=0.0, max_iter=1)
    assert e.value.status == "AIY_BAD_ARG"


def test_ks_multi_device_validates_before_sharding(pkg):
    """ks_vfi_solve(n_devices > 1) checks NULL arguments and k_size >= 3 up front (the sharded
    path does not stage through the checked single-device code)."""
    L = pkg.lib()
    it, rel = C.c_int64(0), C.c_double(0)
    V = np.zeros((2, 4, 4), order="F")
    ko = np.zeros_like(V)
    kg = np.array([0.0, 1.0])
    Kg = np.linspace(30, 50, 4)
    rc = L.aiy_last_error  # noqa: F841  (keeps the handle)
    rc = L.ks_vfi_solve(V.ctypes.data_as(C.c_void_p), ko.ctypes.data_as(C.c_void_p),
                        kg.ctypes.data_as(C.c_void_p), Kg.ctypes.data_as(C.c_void_p), None,
                        None, None, C.c_int64(2), C.c_int64(4), C.c_int64(50), C.c_double(1e-6),
                        C.c_int64(10), C.c_int(2), C.byref(it), C.byref(rel))
    assert rc == 6  # AIY_BAD_ARG (NULL B / P / params)
    B, P, prm = np.array([0, 1, 0, 1.0]), np.eye(4), np.asarray(pkg.ks_params(), np.float64)
    rc = L.ks_vfi_solve(V.ctypes.data_as(C.c_void_p), ko.ctypes.data_as(C.c_void_p),
                        kg.ctypes.data_as(C.c_void_p), Kg.ctypes.data_as(C.c_void_p),
                        B.ctypes.data_as(C.c_void_p), P.ctypes.data_as(C.c_void_p),
                        prm.ctypes.data_as(C.c_void_p), C.c_int64(2), C.c_int64(4), C.c_int64(50),
                        C.c_double(1e-6), C.c_int64(10), C.c_int(2), C.byref(it), C.byref(rel))
    assert rc == 1  # AIY_BAD_SHAPE (k_size < 3)
