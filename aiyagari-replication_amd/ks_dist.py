"""E3 / BASELINE config 5 — the Krusell-Smith VFI (Krusell_Smith_VFI.m:141-204) sharded over
ranks, one process per GPU, torch.distributed (RCCL over xGMI on GPUs, gloo on CPU).

Rank r owns the aggregate-capital range K in [K0, K1) for all four s, or — with more ranks
than K points — for the two s of one aggregate state z (the (K, Z) slices of SURVEY §8(e) E3,
`shard_slices`).  Policy improvement is local given V.  A Jacobi Howard sweep reads, for each
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


def shard_slices(nK: int, rank: int, world: int):
    """(K0, K1, s0, s1): the rank's shard, K in [K0, K1) of the s blocks [s0, s1).  Up to nK
    ranks split the K range (all four s each); up to 2·nK ranks split the (K, Z) slices —
    s = 0, 1 share one aggregate state z, s = 2, 3 the other — half the ranks per z, each half
    splitting the K range (the reference's K = 4 grid then uses 8 ranks)."""
    if world <= nK:
        K0, K1 = shard_range(nK, rank, world)
        return K0, K1, 0, 4
    if world > 2 * nK:
        raise ValueError(f"{world} ranks exceed the 2·K_size = {2 * nK} (K, Z) slices")
    h = (world + 1) // 2
    if rank < h:
        K0, K1 = shard_range(nK, rank, h)
        return K0, K1, 0, 2
    K0, K1 = shard_range(nK, rank - h, world - h)
    return K0, K1, 2, 4


def owned_columns(nK: int, rank: int, world: int):
    """Flat value columns c = s·nK + K (rows of V viewed as (4·nK, k)) the rank owns."""
    K0, K1, s0, s1 = shard_slices(nK, rank, world)
    return [s * nK + K for s in range(s0, s1) for K in range(K0, K1)]


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
    """plan[q][p] = sorted flat columns (s'·nK + K') rank q reads that rank p owns (p != q;
    [] on the diagonal): for every node q owns, the forecast column K'_idx(s, K) of all four
    s' (Krusell_Smith_VFI.m:343-349)."""
    owner = np.empty(4 * nK, np.int64)
    for q in range(world):
        owner[owned_columns(nK, q, world)] = q
    kp = np.asarray(kp_idx)
    plan = [[[] for _ in range(world)] for _ in range(world)]
    for q in range(world):
        K0, K1, s0, s1 = shard_slices(nK, q, world)
        targets = np.unique(kp[s0:s1, K0:K1])
        need = sorted({sn * nK + int(t) for t in targets for sn in range(4)})
        for c in need:
            if owner[c] != q:
                plan[q][int(owner[c])].append(c)
    return plan


class HaloExchange:
    """Per-sweep exchange of the halo columns (rows of V viewed as (4·nK, k)) between ranks:
    one batched set of point-to-point sends/receives (RCCL over xGMI on GPUs)."""

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
                self.recvs.append((p, cols, torch.empty((len(plan[rank][p]), nk),
                                                        dtype=dtype, device=device)))
        self.columns = sum(len(c) for _, c, _ in self.recvs)

    def __call__(self, V):
        import torch
        import torch.distributed as dist
        nccl = dist.get_backend() == "nccl"
        flat = V.view(-1, V.shape[-1])
        ops, staged = [], []
        for p, cols in self.sends:
            buf = flat.index_select(0, cols)
            ops.append(dist.P2POp(dist.isend, buf if nccl else buf.cpu(), p))
        for p, cols, buf in self.recvs:
            rb = buf if nccl else torch.empty(buf.shape, dtype=buf.dtype)
            staged.append((cols, rb))
            ops.append(dist.P2POp(dist.irecv, rb, p))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for cols, rb in staged:
            flat.index_copy_(0, cols, rb.to(V.device))


class HipShard:
    """The device-tier handle (ks_dev_*) for this rank's shard: K in [K0, K1) of the s blocks
    [s0, s1) (all four by default; one z's pair for (K, Z) slices)."""

    def __init__(self, k_grid, K_grid, B, P, params, K0, K1, s0=0, s1=4):
        kg = np.ascontiguousarray(k_grid, np.float64)
        Kg = np.ascontiguousarray(K_grid, np.float64)
        self.K0, self.K1, self.s0, self.s1 = K0, K1, s0, s1
        self.kp_idx = forecast_index(Kg, B, params)
        h = vp()
        check(lib().ks_dev_create_slice(ptr(kg), ptr(Kg), ptr(np.ascontiguousarray(B, np.float64)),
                                        ptr(np.asfortranarray(P, dtype=np.float64)),
                                        ptr(np.ascontiguousarray(params, np.float64)),
                                        i64(kg.size), i64(Kg.size), i64(K0), i64(K1), i64(s0),
                                        i64(s1), C.byref(h)))
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


def _exchange(V, rank, world, nK):
    """All-gather every rank's owned columns of V (rows of the (4·nK, k) view) into every
    rank's V, in place."""
    import torch
    import torch.distributed as dist
    cols = [owned_columns(nK, q, world) for q in range(world)]
    m = max(len(c) for c in cols)
    flat = V.view(-1, V.shape[-1])
    mine = torch.zeros((m, flat.shape[1]), dtype=V.dtype, device=V.device)
    mine[:len(cols[rank])] = flat.index_select(0, torch.tensor(cols[rank], device=V.device))
    if dist.get_backend() == "nccl":
        out = torch.empty((world, m, flat.shape[1]), dtype=V.dtype, device=V.device)
        dist.all_gather_into_tensor(out, mine)
    else:  # gloo: stage through host memory
        parts = [torch.empty_like(mine, device="cpu") for _ in range(world)]
        dist.all_gather(parts, mine.cpu())
        out = torch.stack(parts).to(V.device)
    for q in range(world):
        if q != rank:
            flat.index_copy_(0, torch.tensor(cols[q], device=V.device), out[q, :len(cols[q])])


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
    nk = V.shape[-1]
    own = torch.tensor(owned_columns(nK, rank, world), device=V.device)
    halo = None
    if world > 1:
        dist.barrier()   # first collective on every rank before any point-to-point
        if exchange == "halo":
            plan = halo_plan(shard.kp_idx, nK, world)
            halo = HaloExchange(plan, rank, world, V.device, V.shape[2], V.dtype)
            if poison:
                keep = set(owned_columns(nK, rank, world)) | \
                    {c for p in range(world) for c in plan[rank][p]}
                flat = V.view(-1, nk)
                for c in range(4 * nK):
                    if c not in keep:
                        flat[c] = math.nan
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
            if halo is None:  # V2 holds the shard's new nodes; carry the rest over, then gather
                fresh = V2.view(-1, nk).index_select(0, own)
                V2.copy_(V)
                V2.view(-1, nk).index_copy_(0, own, fresh)
            V, V2 = V2, V
            if halo is not None:
                halo(V)
            elif world > 1:
                _exchange(V, rank, world, nK)
        rel = shard.reldiff(V, Vold)                       # :195
        if world > 1:
            rel = _allreduce_max(rel, V.device)
        if rel < tol:
            break
    if world > 1:                                          # every rank leaves with all of both
        _exchange(k_opt, rank, world, nK)
        if halo is not None:
            _exchange(V, rank, world, nK)
    if V is not value:
        value.copy_(V)
    return it, rel
