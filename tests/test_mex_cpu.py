"""CPU: the MEX/mkoctfile gateways (compiled against the stub mx API) validate their arguments
the way a MATLAB caller sees it — errors come back as mexErrMsgIdAndTxt identifiers — and report
the library status when no device is present."""
import numpy as np
import pytest

from tests import mexstub
from oracle import np_oracle as no


@pytest.fixture(scope="module")
def cal():
    if not mexstub.LIB.exists():
        pytest.skip("libmexstub.so not built")
    return no.calib_aiyagari(Na=20)


def test_usage_error(cal):
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)))
    assert e.value.id == "aiy:usage"


def test_shape_errors(cal):
    with pytest.raises(mexstub.MexError) as e:  # P not N x N
        mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)), cal["a_grid"], cal["s"],
                     np.eye(6), 0.04, 1.0, 0.96, 5.0)
    assert e.value.id == "aiy:shape"
    with pytest.raises(mexstub.MexError) as e:  # a_grid length != size(v_old, 2)
        mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)), cal["a_grid"][:-1], cal["s"],
                     cal["P"], 0.04, 1.0, 0.96, 5.0)
    assert e.value.id == "aiy:shape"
    with pytest.raises(mexstub.MexError) as e:  # scalar expected
        mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)), cal["a_grid"], cal["s"],
                     cal["P"], np.array([0.04, 0.05]), 1.0, 0.96, 5.0)
    assert e.value.id == "aiy:type"


def test_library_status_surfaces_as_mex_error(cal):
    import torch
    a = cal["a_grid"][::-1].copy()  # unsorted grid: rejected by the library before any device work
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)), a, cal["s"], cal["P"], 0.04,
                     1.0, 0.96, 5.0)
    assert e.value.id == "aiy:BAD_ARG"
    if not torch.cuda.is_available():
        with pytest.raises(mexstub.MexError) as e:
            mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)), cal["a_grid"], cal["s"],
                         cal["P"], 0.04, 1.0, 0.96, 5.0)
        assert e.value.id == "aiy:NO_DEVICE"


def test_ks_shape_check(cal):
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_vfi_solve_mex", 2, np.zeros((10, 4, 4)), np.zeros((10, 4, 4)),
                     np.linspace(0, 1, 11), np.linspace(30, 50, 4), np.array([0, 1, 0, 1.0]),
                     np.eye(4), np.zeros(13), 50.0, 1e-6, 10.0, 1.0)
    assert e.value.id == "aiy:shape"


def test_ks_egm_shape_and_usage(cal):
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_egm_solve_mex", 1, np.zeros((10, 4, 4)), np.linspace(0, 1, 11),
                     np.linspace(30, 50, 4), np.array([0, 1, 0, 1.0]), np.eye(4), np.zeros(13),
                     1e-6, 10.0)
    assert e.value.id == "aiy:shape"
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_egm_solve_mex", 1, np.zeros((10, 4, 4)))
    assert e.value.id == "aiy:usage"
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_egm_solve_mex", 1, np.zeros((11, 4, 4)), np.linspace(0, 1, 11),
                     np.linspace(30, 50, 4), np.array([0, 1, 0, 1.0]), np.eye(4), np.zeros(13),
                     1e-6, 10.0, 2.0)
    assert e.value.id == "aiy:type"


def test_ks_panel_gateways_validate(cal):
    """F3/F2 gateways: argument counts and shapes are checked before the library is called."""
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_shocks_mex", 2, 10.0, 5.0, np.zeros(3), np.zeros(13))
    assert e.value.id == "aiy:shape"   # uniforms must hold (T-1) + pop + (T-1)*pop draws
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_shocks_mex", 2, 10.5, 5.0, np.zeros(3), np.zeros(13))
    assert e.value.id == "aiy:shape"
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_simulate_capital_mex", 2, np.zeros((10, 4, 4)), np.linspace(0, 1, 10),
                     np.linspace(30, 50, 4), np.zeros(5), np.ones((5, 3)), np.ones(4))
    assert e.value.id == "aiy:shape"   # epsi_shock columns != numel(k_population)
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("ks_simulate_capital_mex", 2, np.zeros((10, 4, 4)))
    assert e.value.id == "aiy:usage"
    with pytest.raises(mexstub.MexError) as e:   # zi_shock codes other than 0/1: BAD_ARG
        mexstub.call("ks_simulate_capital_mex", 2, np.zeros((10, 4, 4)), np.linspace(0, 1, 10),
                     np.linspace(30, 50, 4), np.full(5, 3.0), np.ones((5, 3)), np.ones(3))
    assert e.value.id == "aiy:BAD_ARG"


def test_ge_batch_gateway_validation(cal):
    v = np.zeros((7, 20))
    U = np.full((99, 2), 0.5)
    args = [np.array([0.01, 0.02]), v, cal["a_grid"], cal["s"], cal["P"], 0.36, 0.08, 0.96, 5.0,
            1.0, 1e-5, 1000.0, 1.0, float(cal["a_grid"][0]), U, 1.0]
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_ge_batch_mex", 3, *args[:-1])
    assert e.value.id == "aiy:usage"
    bad = list(args)
    bad[14] = np.full((99, 3), 0.5)          # one column of uniforms per candidate rate
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_ge_batch_mex", 3, *bad)
    assert e.value.id == "aiy:shape"
    bad = list(args)
    bad[12] = 1.5                              # z1 must be an integer
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_ge_batch_mex", 3, *bad)
    assert e.value.id == "aiy:type"
    bad = list(args)
    a = cal["a_grid"].copy()
    a[3] = a[2]                                # repeated grid point: interp1 would error
    bad[2] = a
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_ge_batch_mex", 3, *bad)
    assert e.value.id == "aiy:BAD_ARG"


def test_sim_gateway_layout_is_explicit_when_ambiguous(cal):
    P = np.eye(7)
    pol = np.zeros((7, 7))                     # Na == N: N x Na and Na x N look alike
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_sim_capital_mex", 1, pol, np.arange(7.0), P, 1.0, 0.0, np.full(9, 0.5))
    assert e.value.id == "aiy:shape" and "layout" in str(e.value)


def test_lifecycle_lock_balanced_and_release_registered(cal):
    """Every call leaves the lock count where it found it, errors included, and the first call
    that reaches the library registers the exit function; `clear mex` runs it, which frees the
    host-tier caches (B3)."""
    L = mexstub.lib()
    d0 = L.stub_lock_depth()
    for _ in range(2):
        try:
            mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)), cal["a_grid"][::-1].copy(),
                         cal["s"], cal["P"], 0.04, 1.0, 0.96, 5.0)
        except mexstub.MexError:
            pass
        try:
            mexstub.call("aiy_vfi_sweep_mex", 3, np.zeros((7, 20)))
        except mexstub.MexError:
            pass
    assert L.stub_lock_depth() == d0
    assert L.stub_clear_mex() >= 1
    import ctypes as C
    from tests.conftest import load_pkg
    lib = load_pkg().lib()
    lib.aiy_host_cache_bytes.restype = C.c_int64
    assert lib.aiy_host_cache_bytes() == 0


def test_step_gateways_validate(cal):
    """The step-level gateways (one EGM pass, one labour sweep): usage, shapes, and
    the library status without a device."""
    import torch
    pc = np.ones((20, 7))  # Na x N
    with pytest.raises(mexstub.MexError) as e:
        mexstub.call("aiy_egm_step_mex", 3, pc, cal["a_grid"])
    assert e.value.id == "aiy:usage"
    with pytest.raises(mexstub.MexError) as e:  # s length != N
        mexstub.call("aiy_egm_step_mex", 3, pc, cal["a_grid"], cal["s"][:-1], cal["P"], 0.04, 1.0,
                     0.96, 5.0, 0.0)
    assert e.value.id == "aiy:shape"
    with pytest.raises(mexstub.MexError) as e:  # P not N x N
        mexstub.call("aiy_labor_egm_step_mex", 4, pc, cal["a_grid"], cal["s"], np.eye(5), 0.04,
                     1.0, 0.96, 5.0, 1.0, 1.0, 0.0)
    assert e.value.id == "aiy:shape"
    L = np.linspace(0.01, 1.5, 10)
    with pytest.raises(mexstub.MexError) as e:  # trailing v_new of the wrong shape
        mexstub.call("aiy_labor_vfi_sweep_mex", 4, np.zeros((7, 20)), cal["a_grid"], cal["s"],
                     cal["P"], L, 0.04, 1.0, 0.96, 5.0, 1.0, 2.0, np.zeros((7, 19)))
    assert e.value.id == "aiy:shape"
    if not torch.cuda.is_available():
        for name, n, args in (
                ("aiy_egm_step_mex", 3, (pc, cal["a_grid"], cal["s"], cal["P"], 0.04, 1.0, 0.96,
                                         5.0, 0.0)),
                ("aiy_labor_egm_step_mex", 4, (pc, cal["a_grid"], cal["s"], cal["P"], 0.04, 1.0,
                                               0.96, 5.0, 1.0, 1.0, 0.0)),
                ("aiy_labor_vfi_sweep_mex", 5, (np.zeros((7, 20)), cal["a_grid"], cal["s"],
                                                cal["P"], L, 0.04, 1.0, 0.96, 5.0, 1.0, 2.0))):
            with pytest.raises(mexstub.MexError) as e:
                mexstub.call(name, n, *args)
            assert e.value.id == "aiy:NO_DEVICE"
