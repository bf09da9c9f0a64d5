"""MI355X-native (gfx950, fp64) solver for the hot path of kostastril/Aiyagari-Replication.

The MATLAB scripts' inner loops (Bellman sweeps, EGM steps, the Monte-Carlo capital supply,
the Krusell-Smith improvement/Howard steps) run as hand-written HIP kernels behind the C ABI
in include/aiyagari_hip.h.  This package is the Python host mirror of that boundary.
There is no CPU fallback: importing works without a GPU, calling a solver without the HIP
library or a device raises.
"""
from . import calibration
from .dist import dist_stationary, dist_stationary_dev, dist_update_dev
from .egm import (egm_solve, egm_solve_dev, egm_step, egm_step_dev, labor_egm_solve,
                  labor_egm_step)
from ._capi import AiyError, LIB_PATH, declared_symbols, lib
from . import ge
from . import ge_batch
from . import ks_dist
from . import ks_panel
from . import stats
from .ks import ks_egm_solve, ks_howard, ks_params, ks_policy_improve, ks_vfi_solve
from .sim import sim_capital, sim_capital_dev
from . import vfi
from .vfi import Workspace, labor_vfi_solve, labor_vfi_sweep, solve_batch_dev, vfi_solve, vfi_sweep

__all__ = ["ge", "ge_batch", "ks_dist", "ks_panel", "stats", "ks_egm_solve", "ks_howard", "ks_params", "ks_policy_improve", "ks_vfi_solve", "dist_stationary", "dist_stationary_dev", "dist_update_dev", "egm_solve", "egm_solve_dev", "egm_step", "egm_step_dev", "labor_egm_solve", "labor_egm_step",
           "AiyError", "LIB_PATH", "Workspace", "calibration", "declared_symbols", "lib",
           "labor_vfi_solve", "sim_capital", "sim_capital_dev", "labor_vfi_sweep", "vfi_solve", "vfi_sweep"]
