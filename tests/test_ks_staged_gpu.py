"""GPU, one process: the staged direct schedule's single-launch sweep (ks_dev_staged_sweep,
DESIGN.md §6) equals the fused single-device sweep bit for bit, whatever the split of the own
columns — in particular a shard with NO interior column (every own column boundary, only copy
and boundary block rows).  That is the round-5 g37 failure: a copy-only interior launch whose
empty column list fell back from list mode to the plain node-range sweep, ran no copy rows, and
left the boundary launch reading a halo that was never filled (Krusell_Smith_VFI.m:172-192).
Every column the staged launch must not read in place is NaN, so a missed copy shows."""
import ctypes as C
import math
import mmap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
B_MIXED = np.array([0.6, 0.84, 0.1, 0.95])  # forecast index one to three K points away


def _case(pkg, nK, K0, K1, k_size, split, with_flags):
    import torch
    from oracle import np_oracle as no
    kd = pkg.ks_dist
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=k_size, K_size=nK)
    nk = kg.size
    dev = "cuda:0"
    sh = kd.HipShard(kg, Kg, B_MIXED, P, pkg.ks_params(), K0, K1, 0, 4)
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    ko = torch.ones_like(V)
    dV = torch.empty_like(V)
    sh.improve(V, ko)                      # k_opt and segment hints of the own nodes
    sh.slopes(V, dV)                       # slopes of every column the shard reads
    Vr, dVr = torch.full_like(V, math.nan), torch.full_like(V, math.nan)
    sh.howard_fused(V, dV, ko, Vr, dVr)    # the reference: fused sweep on full arrays
    # staged: own columns in local buffers, every other column NaN; the forecast columns the
    # shard reads but does not own come from the "peer" arrays (V, dV) through the halo
    own = [s * nK + K for s in range(4) for K in range(K0, K1)]
    owner = [0 if c in own else 1 for c in range(4 * nK)]
    remote, interior, boundary = kd.staged_plan(own, sh.kp_idx, owner, nK, 0)
    if split == "all_boundary":           # the g37 case: no interior column at all
        interior, boundary = [], own
    Vs, dVs = torch.full_like(V, math.nan), torch.full_like(V, math.nan)
    fl = lambda t: t.view(-1, nk)
    for c in own:
        fl(Vs)[c].copy_(fl(V)[c])
        fl(dVs)[c].copy_(fl(dV)[c])
    nr = len(remote)
    hV = torch.full((max(nr, 1), nk), math.nan, dtype=torch.float64, device=dev)
    hdV = torch.full_like(hV, math.nan)
    cb = 8 * nk
    slot = {c: i for i, c in enumerate(remote)}
    tab = torch.tensor([(hV.data_ptr() + cb * slot[c]) if c in slot else Vs.data_ptr() + cb * c
                        for c in range(4 * nK)] +
                       [(hdV.data_ptr() + cb * slot[c]) if c in slot else dVs.data_ptr() + cb * c
                        for c in range(4 * nK)], dtype=torch.int64, device=dev)
    arr = lambda xs: torch.tensor(xs or [0], dtype=torch.int64, device=dev)
    src = arr([V.data_ptr() + cb * c for c in remote] + [dV.data_ptr() + cb * c for c in remote])
    dst = arr([hV.data_ptr() + cb * i for i in range(nr)] + [hdV.data_ptr() + cb * i for i in range(nr)])
    sh.set_split(interior, boundary)
    sh.set_columns(tab)
    Vo, dVo = torch.full_like(V, math.nan), torch.full_like(V, math.nan)
    page = host = None
    check, lib = pkg._capi.check, pkg._capi.lib
    try:
        if with_flags:   # self-satisfied hand-off: wait on, and publish into, slot 0
            page = mmap.mmap(-1, 16384)
            host = C.c_char.from_buffer(page)
            hp = C.addressof(host)
            dptr = C.c_void_p()
            check(lib().aiy_host_register(C.c_void_p(hp), C.c_int64(16384), C.byref(dptr)))
            C.c_uint64.from_address(hp).value = 4
            sh.staged_sweep(Vs, dVs, ko, Vo, dVo, src, dst, 2 * nr, flags=dptr.value, mask=1,
                            wait_v=4, slot=0, pub_v=5, err=dptr.value + 8192)
        else:
            sh.staged_sweep(Vs, dVs, ko, Vo, dVo, src, dst, 2 * nr)
        torch.cuda.synchronize()
        if with_flags:
            assert C.c_uint64.from_address(hp).value == 5          # published
            assert C.c_uint64.from_address(hp + 8192).value == 0   # no timeout
            check(lib().aiy_host_unregister(C.c_void_p(hp)))
    finally:
        sh.set_columns(None)
        del host
        if page is not None:
            page.close()
    for c in own:
        assert torch.equal(fl(Vo)[c], fl(Vr)[c]), c
        assert torch.equal(fl(dVo)[c], fl(dVr)[c]), c
    sh.close()
    return len(interior), len(boundary), nr


@pytest.mark.parametrize("nK,K0,K1,k_size,split,flags", [
    (6, 2, 4, 100, "all_boundary", False),   # g37: every own column boundary, halo > 0
    (6, 2, 4, 100, "all_boundary", True),
    (6, 2, 4, 100, "plan", False),           # interior and boundary columns
    (12, 4, 8, 300, "plan", True),           # two k blocks per column, copy rows of 2 blocks
    (6, 0, 6, 100, "plan", False),           # one shard owns everything: no halo, no boundary
])
def test_staged_sweep_equals_fused(pkg, gpu, nK, K0, K1, k_size, split, flags):
    n_int, n_bnd, nr = _case(pkg, nK, K0, K1, k_size, split, flags)
    if split == "all_boundary":
        assert n_int == 0 and nr > 0
    if K1 - K0 == nK:
        assert nr == 0 and n_bnd == 0
