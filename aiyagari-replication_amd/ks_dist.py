"""E3 / BASELINE config 5 — the Krusell-Smith VFI (Krusell_Smith_VFI.m:141-204) sharded over
ranks, one process per GPU, torch.distributed (RCCL over xGMI on GPUs, gloo on CPU).

Rank r owns the aggregate-capital range K in [K0, K1) for all four s (the (K, Z) slices of
SURVEY §8(e) E3).  Policy improvement is local given V.  A Jacobi Howard sweep reads, for each
owned node, the value columns at the forecast K'_idx for all s', so after every sweep the
owned value slices are all-gathered (one collective of 4·(K1-K0)·k doubles per rank); the
relative-difference stop is an all-reduce MAX of one double.  The kernels are the ones of the
single-device solve (ks_vfi_solve), in the same order, so any number of ranks reproduces it
bit for bit.

Arrays are torch tensors of shape (4, K, k), the memory of MATLAB's k x K x S `value`."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._capi import check, i64, lib, ptr, stream_handle, vp


def shard_range(nK: int, rank: int, world: int):
    return nK * rank // world, nK * (rank + 1) // world


class HipShard:
    """The device-tier handle (ks_dev_*) for this rank's K range."""

    def __init__(self, k_grid, K_grid, B, P, params, K0, K1):
        kg = np.ascontiguousarray(k_grid, np.float64)
        Kg = np.ascontiguousarray(K_grid, np.float64)
        self.K0, self.K1 = K0, K1
        h = vp()
        check(lib().ks_dev_create(ptr(kg), ptr(Kg), ptr(np.ascontiguousarray(B, np.float64)),
                                  ptr(np.asfortranarray(P, dtype=np.float64)),
                                  ptr(np.ascontiguousarray(params, np.float64)), i64(kg.size),
                                  i64(Kg.size), i64(K0), i64(K1), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().ks_dev_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def improve(self, V, kopt):
        check(lib().ks_dev_improve(self._h, ptr(V), ptr(kopt), stream_handle(None)))

    def howard(self, V, kopt, Vout):
        check(lib().ks_dev_howard(self._h, ptr(V), ptr(kopt), ptr(Vout), stream_handle(None)))

    def reldiff(self, V, Vold):
        import torch
        out = torch.zeros(2, dtype=torch.int64, device=V.device)
        check(lib().ks_dev_reldiff(self._h, ptr(V), ptr(Vold), ptr(out), stream_handle(None)))
        o = out.cpu()
        return float(o[0:1].view(torch.float64)[0]) if int(o[1]) != 0 else math.nan


def _exchange(V, K0, K1, rank, world, nK):
    """All-gather the owned (4, K1-K0, k) slices of V into every rank's V (in place)."""
    import torch
    import torch.distributed as dist
    ranges = [shard_range(nK, q, world) for q in range(world)]
    kmax = max(b - a for a, b in ranges)
    mine = torch.zeros((4, kmax, V.shape[2]), dtype=V.dtype, device=V.device)
    mine[:, :K1 - K0, :] = V[:, K0:K1, :]
    if dist.get_backend() == "nccl":
        out = torch.empty((world,) + tuple(mine.shape), dtype=V.dtype, device=V.device)
        dist.all_gather_into_tensor(out, mine)
    else:  # gloo: stage through host memory
        parts = [torch.empty_like(mine, device="cpu") for _ in range(world)]
        dist.all_gather(parts, mine.cpu())
        out = torch.stack(parts).to(V.device)
    for q, (a, b) in enumerate(ranges):
        if q != rank:
            V[:, a:b, :] = out[q, :, :b - a, :]


def _allreduce_max(x: float, device):
    import torch
    import torch.distributed as dist
    t = torch.tensor([-1.0 if math.isnan(x) else x], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = float(t[0])
    return math.nan if v < 0 else v


def ks_vfi_solve_dist(value, k_opt, shard, nK, howard_steps=50, tol=1e-6, max_vfi=10000,
                      rank=0, world=1):
    """Krusell_Smith_VFI.m:141-204 for the current B.  value, k_opt: (4, K, k) tensors on this
    rank's device, full arrays on every rank (in/out).  `shard` owns [K0, K1) (HipShard, or any
    object with the same improve / howard / reldiff methods).  Returns (iters, rel_diff)."""
    V = value
    V2 = V.clone()
    K0, K1 = shard.K0, shard.K1
    rel, it = math.nan, 0
    for it in range(1, max_vfi + 1):
        Vold = V.clone()                                   # value_old = value (:145)
        if (it - 1) % 5 == 0:                              # policy improvement (:148-168)
            shard.improve(V, k_opt)
        for _ in range(howard_steps):                      # Jacobi Howard sweeps (:172-192)
            shard.howard(V, k_opt, V2)
            V2[:, :K0, :] = V[:, :K0, :]
            V2[:, K1:, :] = V[:, K1:, :]
            V, V2 = V2, V
            if world > 1:
                _exchange(V, K0, K1, rank, world, nK)
        rel = shard.reldiff(V, Vold)                       # :195
        if world > 1:
            rel = _allreduce_max(rel, V.device)
        if rel < tol:
            break
    if world > 1:                                          # every rank leaves with all of k_opt
        _exchange(k_opt, K0, K1, rank, world, nK)
    if V is not value:
        value.copy_(V)
    return it, rel
