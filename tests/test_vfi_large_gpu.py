"""A1 beyond the benched size: Na = 40,000 (Aiyagari_VFI.m:70-83), where a row has 79 superblocks of
512 candidates, more than the 64 the tree kernel's level-0 bounds hold per load — the
superblock walk refills them (`load512(g)`, g = 64), a path Na <= 32,768 never takes.  The
last of a chain of hinted sweeps from v = 0 is compared bit for bit with the C oracle's
exhaustive sweep of the device's own v_old, for the default geometry."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu

NA = 40000


def test_vfi_na40000_refilled_level0_bounds(pkg, gpu):
    import torch
    cal = no.calib_aiyagari(Na=NA, shocks="rouwenhorst")
    N = cal["N"]
    dev = torch.device("cuda:0")
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a, s, P = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    assert (NA + 511) // 512 > 64
    ws = pkg.Workspace(N, NA)
    va = torch.zeros((N, NA), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((N, NA), dtype=torch.int32, device=dev)
    pk, pc = torch.empty_like(va), torch.empty_like(va)
    n = 6
    ws.vfi_sweeps(va, vb, a, s, P, r, w, cal["beta"], cal["sigma"], n, idx, pk, pc, hint=None,
                  mode=1)
    torch.cuda.synchronize()
    v_new, v_old = (vb, va) if n & 1 else (va, vb)
    vo = v_old.cpu().numpy()
    v, ix, k, c = corc.vfi_sweep(vo, cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"],
                                 cal["sigma"])
    assert np.array_equal(v_new.cpu().numpy().view(np.uint64), v.view(np.uint64))
    assert np.array_equal(idx.cpu().numpy(), ix)
    assert np.array_equal(pk.cpu().numpy().view(np.uint64), k.view(np.uint64))
    assert np.array_equal(pc.cpu().numpy().view(np.uint64), c.view(np.uint64))
