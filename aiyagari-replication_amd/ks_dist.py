"""E3 / BASELINE config 5 — the Krusell-Smith VFI (Krusell_Smith_VFI.m:141-204) sharded over
ranks, one process per GPU, torch.distributed (RCCL over xGMI on GPUs, gloo on CPU).

Rank r owns the aggregate-capital range K in [K0, K1) for all four s (the (K, Z) slices of
SURVEY §8(e) E3).  Policy improvement is local given V.  A Jacobi Howard sweep reads, for each
owned node, the value columns at the forecast K'_idx(s, K) for all s' (Krusell_Smith_VFI.m:
335-349) and nothing else.  So after every sweep a rank receives exactly the columns its
nodes forecast into that other ranks own (the halo, `halo_plan`; point-to-point isend/irecv
pairs, RCCL over xGMI on GPUs) — with the near-identity ALM that is one or two neighbour
columns, not the whole array.  `exchange="allgather"` keeps the plain all-gather of every
owned slice for comparison.  The relative-difference stop is an all-reduce MAX of one double;
the full value and k_opt arrays are all-gathered once, at the end.  The kernels are the ones
of the single-device solve (ks_vfi_solve), in the same order, so any number of ranks
reproduces it bit for bit.

Arrays are torch tensors of shape (4, K, k), the memory of MATLAB's k x K x S `value`."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._capi import check, i64, lib, ptr, stream_handle, vp


def shard_range(nK: int, rank: int, world: int):
    return nK * rank // world, nK * (rank + 1) // world


def forecast_index(K_grid, B, params):
    """K'_idx(s, K), 0-based, shape (4, nK): ks_forecast_index of the C ABI (host-only, the
    same ks_slices the kernels use, so the halo is exactly what they read)."""
    Kg = np.ascontiguousarray(K_grid, np.float64)
    out = np.zeros(4 * Kg.size, np.int32)
    check(lib().ks_forecast_index(ptr(Kg), ptr(np.ascontiguousarray(B, np.float64)),
                                  ptr(np.ascontiguousarray(params, np.float64)), i64(Kg.size),
                                  ptr(out)))
    return out.reshape(4, Kg.size)


def halo_plan(kp_idx, nK: int, world: int):
    """plan[q][p] = sorted K columns rank q reads that rank p owns (p != q; [] on the
    diagonal): the forecast targets K'_idx(s, K) of q's nodes, all s (:343-349)."""
    ranges = [shard_range(nK, q, world) for q in range(world)]
    owner = np.empty(nK, np.int64)
    for q, (a, b) in enumerate(ranges):
        owner[a:b] = q
    plan = [[[] for _ in range(world)] for _ in range(world)]
    for q, (a, b) in enumerate(ranges):
        need = np.unique(np.asarray(kp_idx)[:, a:b])
        for c in need:
            if owner[c] != q:
                plan[q][int(owner[c])].append(int(c))
    return plan


class HaloExchange:
    """Per-sweep exchange of the halo columns (4 x len x k slabs of V) between ranks."""

    def __init__(self, plan, rank: int, world: int, device, nk: int, dtype):
        import torch
        self.rank, self.world = rank, world
        self.sends, self.recvs = [], []
        for p in range(world):
            if p == rank:
                continue
            if plan[p][rank]:   # what p reads from me
                self.sends.append((p, torch.tensor(plan[p][rank], device=device)))
            if plan[rank][p]:   # what I read from p
                cols = torch.tensor(plan[rank][p], device=device)
                self.recvs.append((p, cols, torch.empty((4, len(plan[rank][p]), nk),
                                                        dtype=dtype, device=device)))
        self.columns = sum(len(c) for _, c, _ in self.recvs)

    def __call__(self, V):
        import torch
        import torch.distributed as dist
        nccl = dist.get_backend() == "nccl"
        ops, staged = [], []
        for p, cols in self.sends:
            buf = V.index_select(1, cols)
            ops.append(dist.P2POp(dist.isend, buf if nccl else buf.cpu(), p))
        for p, cols, buf in self.recvs:
            rb = buf if nccl else torch.empty(buf.shape, dtype=buf.dtype)
            staged.append((cols, rb))
            ops.append(dist.P2POp(dist.irecv, rb, p))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for cols, rb in staged:
            V.index_copy_(1, cols, rb.to(V.device))


class HipShard:
    """The device-tier handle (ks_dev_*) for this rank's K range."""

    def __init__(self, k_grid, K_grid, B, P, params, K0, K1):
        kg = np.ascontiguousarray(k_grid, np.float64)
        Kg = np.ascontiguousarray(K_grid, np.float64)
        self.K0, self.K1 = K0, K1
        self.kp_idx = forecast_index(Kg, B, params)
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
                      rank=0, world=1, exchange="halo", poison=False):
    """Krusell_Smith_VFI.m:141-204 for the current B.  value, k_opt: (4, K, k) tensors on this
    rank's device, full arrays on every rank (in/out).  `shard` owns [K0, K1) (HipShard, or any
    object with the same improve / howard / reldiff methods and a kp_idx table).  exchange:
    "halo" (point-to-point, only the columns read) or "allgather".  poison (tests): NaN every
    column this rank neither owns nor reads, proving the halo is sufficient.
    Returns (iters, rel_diff)."""
    import torch
    import torch.distributed as dist
    V = value
    K0, K1 = shard.K0, shard.K1
    halo = None
    if world > 1:
        dist.barrier()   # first collective on every rank before any point-to-point
        if exchange == "halo":
            plan = halo_plan(shard.kp_idx, nK, world)
            halo = HaloExchange(plan, rank, world, V.device, V.shape[2], V.dtype)
            if poison:
                keep = set(range(K0, K1)) | {c for p in range(world) for c in plan[rank][p]}
                for c in range(nK):
                    if c not in keep:
                        V[:, c, :] = math.nan
        elif exchange != "allgather":
            raise ValueError(f"exchange must be 'halo' or 'allgather', not {exchange!r}")
    V2 = V.clone()
    rel, it = math.nan, 0
    for it in range(1, max_vfi + 1):
        Vold = V.clone()                                   # value_old = value (:145)
        if (it - 1) % 5 == 0:                              # policy improvement (:148-168)
            shard.improve(V, k_opt)
        for _ in range(howard_steps):                      # Jacobi Howard sweeps (:172-192)
            shard.howard(V, k_opt, V2)
            if halo is None:
                V2[:, :K0, :] = V[:, :K0, :]
                V2[:, K1:, :] = V[:, K1:, :]
            V, V2 = V2, V
            if halo is not None:
                halo(V)
            elif world > 1:
                _exchange(V, K0, K1, rank, world, nK)
        rel = shard.reldiff(V, Vold)                       # :195
        if world > 1:
            rel = _allreduce_max(rel, V.device)
        if rel < tol:
            break
    if world > 1:                                          # every rank leaves with all of both
        _exchange(k_opt, K0, K1, rank, world, nK)
        if halo is not None:
            _exchange(V, K0, K1, rank, world, nK)
    if V is not value:
        value.copy_(V)
    return it, rel
