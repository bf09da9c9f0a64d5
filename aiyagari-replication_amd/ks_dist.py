"""E3 / BASELINE config 5 — the Krusell-Smith VFI (Krusell_Smith_VFI.m:141-204) sharded over
ranks, one process per GPU, torch.distributed (RCCL over xGMI on GPUs, gloo on CPU).

Rank r owns the aggregate-capital range K in [K0, K1) for all four s, or — with more ranks
than K points — for the two s of one aggregate state z (the (K, Z) slices of SURVEY §8(e) E3,
`shard_slices`).  Policy improvement is local given V.  A Jacobi Howard sweep reads, for each
owned node, the value columns at the forecast K'_idx(s, K) for all s' (Krusell_Smith_VFI.m:
335-349) and nothing else.  So after every sweep a rank receives exactly the columns its
nodes forecast into that other ranks own (the halo, `halo_plan`; point-to-point isend/irecv
pairs, RCCL over xGMI on GPUs) — with the near-identity ALM that is one or two neighbour
columns, not the whole array; with `depth = m` the halo is exchanged once per block of m
sweeps and a ghost rectangle of neighbouring columns is swept redundantly in between.
`exchange="direct"` (DirectPeers) drops the copies altogether: each rank maps its neighbours'
column buffers through IPC handles and reads the forecast columns in place, with a
stream-ordered counter hand-off per sweep.  `exchange="allgather"` keeps the plain all-gather
of every owned slice for comparison.  The relative-difference stop is an all-reduce MAX of one double;
the full value and k_opt arrays are all-gathered once, at the end.  The kernels are the ones
of the single-device solve (ks_vfi_solve), in the same order, so any number of ranks
reproduces it bit for bit.

Arrays are torch tensors of shape (4, K, k), the memory of MATLAB's k x K x S `value`."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._capi import check, i64, lib, ptr, stream_handle, vp


def shard_range(nK: int, rank: int, world: int, bounds=None):
    if bounds is not None:
        return int(bounds[rank]), int(bounds[rank + 1])
    return nK * rank // world, nK * (rank + 1) // world


def shard_slices(nK: int, rank: int, world: int, bounds=None):
    """(K0, K1, s0, s1): the rank's shard, K in [K0, K1) of the s blocks [s0, s1).  Up to nK
    ranks split the K range (all four s each) — evenly, or at `bounds` (world + 1 increasing
    K boundaries from 0 to nK, e.g. `balanced_bounds`); up to 2·nK ranks split the (K, Z)
    slices — s = 0, 1 share one aggregate state z, s = 2, 3 the other — half the ranks per z,
    each half splitting the K range evenly (the reference's K = 4 grid then uses 8 ranks)."""
    if world <= nK:
        K0, K1 = shard_range(nK, rank, world, bounds)
        return K0, K1, 0, 4
    if world > 2 * nK:
        raise ValueError(f"{world} ranks exceed the 2·K_size = {2 * nK} (K, Z) slices")
    h = (world + 1) // 2
    if rank < h:
        K0, K1 = shard_range(nK, rank, h)
        return K0, K1, 0, 2
    K0, K1 = shard_range(nK, rank - h, world - h)
    return K0, K1, 2, 4


def owned_columns(nK: int, rank: int, world: int, bounds=None):
    """Flat value columns c = s·nK + K (rows of V viewed as (4·nK, k)) the rank owns."""
    K0, K1, s0, s1 = shard_slices(nK, rank, world, bounds)
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


def _need_plan(need, nK: int, world: int, bounds=None):
    """plan[q][p] = sorted flat columns of need[q] that rank p owns (p != q; [] on the
    diagonal)."""
    owner = np.empty(4 * nK, np.int64)
    for q in range(world):
        owner[owned_columns(nK, q, world, bounds)] = q
    plan = [[[] for _ in range(world)] for _ in range(world)]
    for q in range(world):
        for c in sorted(set(int(c) for c in need[q])):
            if owner[c] != q:
                plan[q][int(owner[c])].append(c)
    return plan


def halo_plan(kp_idx, nK: int, world: int, bounds=None):
    """plan[q][p] = sorted flat columns (s'·nK + K') rank q reads that rank p owns (p != q;
    [] on the diagonal): for every node q owns, the forecast column K'_idx(s, K) of all four
    s' (Krusell_Smith_VFI.m:343-349)."""
    kp = np.asarray(kp_idx)
    need = []
    for q in range(world):
        K0, K1, s0, s1 = shard_slices(nK, q, world, bounds)
        targets = np.unique(kp[s0:s1, K0:K1])
        need.append([sn * nK + int(t) for t in targets for sn in range(4)])
    return _need_plan(need, nK, world, bounds)


def ghost_rects(kp_idx, nK: int, K0: int, K1: int, s0: int, s1: int, depth: int):
    """R_0 = the shard (K0, K1, s0, s1); R_j = the smallest rectangle (K range x all four s)
    holding R_{j-1} and every column its nodes read (the forecast columns K'_idx(s, K) of all
    s', Krusell_Smith_VFI.m:343-349).  A rank holding R_L current at sweep t can run sweep
    t + i on R_{L-i} (its reads lie in R_{L-i+1}), so after L sweeps its own nodes are current
    without any exchange in between: the communication-avoiding ("ghost zone") schedule."""
    kp = np.asarray(kp_idx)
    rects = [(K0, K1, s0, s1)]
    for _ in range(depth):
        Ka, Kb, sa, sb = rects[-1]
        t = kp[sa:sb, Ka:Kb]
        rects.append((min(Ka, int(t.min())), max(Kb, int(t.max()) + 1), 0, 4))
    return rects


def rect_columns(rect, nK: int):
    Ka, Kb, sa, sb = rect
    return [s * nK + K for s in range(sa, sb) for K in range(Ka, Kb)]


def ghost_plan(kp_idx, nK: int, world: int, depth: int, bounds=None):
    """Exchange plan for a block of `depth` sweeps: rank q receives every column of its
    R_depth (ghost_rects) that another rank owns."""
    need = [rect_columns(ghost_rects(kp_idx, nK, *shard_slices(nK, q, world, bounds), depth)[depth],
                         nK) for q in range(world)]
    return _need_plan(need, nK, world, bounds)


def ghost_cost(kp_idx, nK: int, K0: int, K1: int, depth: int, w_slopes: float = 0.4):
    """Column-sweeps of one block of `depth` sweeps on the K range [K0, K1) (all four s): the
    fused Howard sweeps on R_{depth-1} .. R_0 plus the block's slopes launch over R_{depth-1},
    weighted by `w_slopes` (a slopes column costs ~0.4 of a sweep column on gfx950:
    DESIGN.md §6, 13.3 µs for 14 columns vs 32.5 µs for 12.5)."""
    rects = ghost_rects(kp_idx, nK, K0, K1, 0, 4, depth)
    w = [b - a for a, b, _, _ in rects[:depth]]
    return sum(w) + w_slopes * w[-1]


def balanced_bounds(kp_idx, nK: int, world: int, depth: int, w_slopes: float = 0.4):
    """K boundaries [0 = b_0 < b_1 < ... < b_world = nK] of contiguous K ranges that minimise
    the largest `ghost_cost` over the ranks (exact DP over the split points).  With the
    near-identity ALM the ghost rectangles of the top ranks grow up to three K points per level
    (the forecast moves further there), so even splits leave those ranks 30 % more work;
    balanced ranges give them fewer own columns.  Any partition gives bit-identical results."""
    if world > nK:
        raise ValueError("balanced_bounds splits the K range: world <= K_size")
    cost = {}

    def c(a, b):
        if (a, b) not in cost:
            cost[(a, b)] = ghost_cost(kp_idx, nK, a, b, depth, w_slopes)
        return cost[(a, b)]

    INF = float("inf")
    # best[p][b]: smallest max cost splitting [0, b) into p ranges; arg for the split point
    best = [[INF] * (nK + 1) for _ in range(world + 1)]
    arg = [[0] * (nK + 1) for _ in range(world + 1)]
    best[0][0] = 0.0
    for p in range(1, world + 1):
        for b in range(p, nK - (world - p) + 1):
            for a in range(p - 1, b):
                if best[p - 1][a] == INF:
                    continue
                m = max(best[p - 1][a], c(a, b))
                if m < best[p][b] - 1e-12:
                    best[p][b], arg[p][b] = m, a
    bounds = [nK]
    for p in range(world, 0, -1):
        bounds.append(arg[p][bounds[-1]])
    return bounds[::-1]


def _runs(cols):
    """sorted columns -> [(c0, c1)) contiguous runs (rows of the flat (4·nK, k) view)"""
    out = []
    for c in cols:
        if out and out[-1][1] == c:
            out[-1][1] = c + 1
        else:
            out.append([c, c + 1])
    return [(a, b) for a, b in out]


class HaloExchange:
    """Exchange of halo columns (rows of V viewed as (4·nK, k)) between ranks: one batched set
    of point-to-point sends/receives (RCCL over xGMI on GPUs).  A column is contiguous in V and
    a plan's columns from one peer are a few contiguous runs (one per s), so every send and
    receive works on a view of V itself: no gather/scatter kernels on the exchange path."""

    def __init__(self, plan, rank: int, world: int, device, nk: int, dtype):
        self.rank, self.world = rank, world
        self.sends, self.recvs = [], []
        for p in range(world):
            if p == rank:
                continue
            self.sends += [(p, a, b) for a, b in _runs(plan[p][rank])]   # what p reads from me
            self.recvs += [(p, a, b) for a, b in _runs(plan[rank][p])]   # what I read from p
        self.columns = sum(b - a for _, a, b in self.recvs)

    def __call__(self, V):
        import torch
        import torch.distributed as dist
        nccl = dist.get_backend() == "nccl"
        flat = V.view(-1, V.shape[-1])
        ops, staged = [], []
        for p, a, b in self.sends:
            ops.append(dist.P2POp(dist.isend, flat[a:b] if nccl else flat[a:b].cpu(), p))
        for p, a, b in self.recvs:
            rb = flat[a:b] if nccl else torch.empty((b - a, flat.shape[1]), dtype=V.dtype)
            if not nccl:
                staged.append((a, b, rb))
            ops.append(dist.P2POp(dist.irecv, rb, p))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for a, b, rb in staged:
            flat[a:b].copy_(rb.to(V.device))


class HipShard:
    """The device-tier handle (ks_dev_*) for this rank's shard: K in [K0, K1) of the s blocks
    [s0, s1) (all four by default; one z's pair for (K, Z) slices)."""

    def __init__(self, k_grid, K_grid, B, P, params, K0, K1, s0=0, s1=4):
        kg = np.ascontiguousarray(k_grid, np.float64)
        Kg = np.ascontiguousarray(K_grid, np.float64)
        self.K0, self.K1, self.s0, self.s1 = K0, K1, s0, s1
        self.kp_idx = forecast_index(Kg, B, params)
        self._keep = (kg, Kg, np.ascontiguousarray(B, np.float64),
                      np.asfortranarray(P, dtype=np.float64),
                      np.ascontiguousarray(params, np.float64))
        self._args = tuple(ptr(x) for x in self._keep) + (i64(kg.size), i64(Kg.size))
        h = vp()
        check(lib().ks_dev_create_slice(*self._args, i64(K0), i64(K1), i64(s0), i64(s1),
                                        C.byref(h)))
        self._h = h
        self._ghosts = []

    def close(self):
        for g in getattr(self, "_ghosts", []):  # they use this handle's hint array
            g.close()
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

    def ghost(self, K0, K1, s0, s1):
        """A shard over the rectangle (K0, K1, s0, s1) of other ranks' columns that shares this
        shard's segment hints (ks_dev_share_hints; close it before this one)."""
        g = HipShard.__new__(HipShard)
        g.K0, g.K1, g.s0, g.s1, g.kp_idx = K0, K1, s0, s1, self.kp_idx
        h = vp()
        check(lib().ks_dev_create_slice(*self._args, i64(K0), i64(K1), i64(s0), i64(s1),
                                        C.byref(h)))
        g._h, g._args, g._keep, g._ghosts = h, self._args, self._keep, []
        self._ghosts.append(g)
        check(lib().ks_dev_share_hints(h, self._h))
        return g

    def hints(self, kopt):
        check(lib().ks_dev_hints(self._h, ptr(kopt), stream_handle(None)))

    def slopes(self, V, dV):
        """pchip slopes of every column this shard's sweep reads, into dV (full array)."""
        check(lib().ks_dev_slopes(self._h, ptr(V), ptr(dV), stream_handle(None)))

    def howard_fused(self, V, dV, kopt, Vout, dVout):
        """One Howard sweep on this shard's nodes writing the next sweep's slopes too."""
        check(lib().ks_dev_howard_fused(self._h, ptr(V), ptr(dV), ptr(kopt), ptr(Vout),
                                        ptr(dVout), stream_handle(None)))

    # the direct schedule (ks_vfi_solve_sharded depth = 0): forecast columns read in place
    def set_columns(self, table):
        """table: device int64 tensor of 4·nK value-column then 4·nK slope-column addresses
        (None: back to the caller's arrays; a no-op on a closed shard)."""
        if table is None and not getattr(self, "_h", None):
            return
        check(lib().ks_dev_set_columns(self._h, ptr(table)))

    def slopes_own(self, V, dV):
        check(lib().ks_dev_slopes_own(self._h, ptr(V), ptr(dV), stream_handle(None)))

    def improve_direct(self, kopt):
        check(lib().ks_dev_improve_direct(self._h, ptr(kopt), stream_handle(None)))

    def set_split(self, interior, boundary):
        """The staged schedule's split of the own columns (ks_dev_set_split)."""
        ii = np.ascontiguousarray(interior, np.int32)
        bb = np.ascontiguousarray(boundary, np.int32)
        check(lib().ks_dev_set_split(self._h, ptr(ii), C.c_int32(ii.size), ptr(bb),
                                     C.c_int32(bb.size)))

    def staged_sweep(self, V, dV, kopt, Vout, dVout, src=None, dst=None, n_halo=0, flags=None,
                     mask=0, wait_v=0, slot=0, pub_v=0, timeout_s=30.0, err=None):
        """One staged sweep in one launch (ks_dev_staged_sweep): src / dst device int64 tensors
        of column addresses; flags / err device addresses (ints) of a mapped host page, or None."""
        check(lib().ks_dev_staged_sweep(
            self._h, ptr(V), ptr(dV), ptr(kopt), ptr(Vout), ptr(dVout), ptr(src), ptr(dst),
            C.c_int32(n_halo), C.c_void_p(flags), C.c_uint64(mask), C.c_uint64(wait_v),
            C.c_int32(slot), C.c_uint64(pub_v), C.c_double(timeout_s), C.c_void_p(err),
            stream_handle(None)))

    def reldiff(self, V, Vold):
        import torch
        out = torch.zeros(2, dtype=torch.int64, device=V.device)
        check(lib().ks_dev_reldiff(self._h, ptr(V), ptr(Vold), ptr(out), stream_handle(None)))
        o = out.cpu()
        return float(o[0:1].view(torch.float64)[0]) if int(o[1]) != 0 else math.nan


def column_table(owners_V, owners_dV, owner, nk):
    """The direct schedule's column table of one shard: column c of value / slopes lives in the
    buffers of shard owner[c] (owners_V[q] / owners_dV[q]: that shard's (4, K, k) tensors).
    Returns a device int64 tensor of 4·nK + 4·nK addresses."""
    import torch
    C = len(owner)
    dev = owners_V[0].device
    addr = [owners_V[owner[c]].data_ptr() + 8 * c * nk for c in range(C)] + \
           [owners_dV[owner[c]].data_ptr() + 8 * c * nk for c in range(C)]
    return torch.tensor(addr, dtype=torch.int64, device=dev)


def staged_plan(own, kp_idx, owner, nK: int, rank: int):
    """The staged direct schedule's plan for one rank: (remote, interior, boundary) — the sorted
    forecast columns s'·nK + K'_idx(s, K) its own columns read that other ranks own (its halo),
    and its own columns split into those whose four forecast columns are all its own and the
    rest (Krusell_Smith_VFI.m:343-349: node (k, K, s) reads column K'_idx(s, K) of every s')."""
    kp = np.asarray(kp_idx)
    targets = {c: [sn * nK + int(kp[c // nK, c % nK]) for sn in range(4)] for c in own}
    remote = sorted({t for c in own for t in targets[c] if owner[t] != rank})
    interior = [c for c in own if all(owner[t] == rank for t in targets[c])]
    inner = set(interior)
    boundary = [c for c in own if c not in inner]
    return remote, interior, boundary


class DirectPeers:
    """The direct schedule (ks_vfi_solve_sharded depth = 0) under one process per
    GPU, staged.  Every rank keeps its own columns of value and slopes in three buffers (version
    v in buffer (v - 1) mod 3); the other ranks map them through IPC handles (exchanged once).
    Per Howard sweep ONE launch (ks_dev_staged_sweep): it publishes the previous version in the
    rank's counter slot of a host page every rank maps, copies the forecast columns peers own
    into a local halo once those peers have published the version it reads (the wait runs in
    the copy blocks), sweeps the interior columns (all forecast columns own) without waiting and
    the boundary columns after the copies.  Stream-ordered, the host never blocks.  Neighbours =
    the owners of the columns this rank reads and the ranks that read its columns (the latter
    so a buffer is not overwritten while it is read: with three buffers that wait is one
    version old and already satisfied by the previous sweep's copy rows)."""

    # the host page: counter slot q at byte 128·q (q < 64), rank q's timeout word at 8192 + 128·q
    PAGE = 16384

    def __init__(self, shard, nK, rank, world, V, bounds=None, timeout_s=30.0):
        import torch
        import torch.distributed as dist
        from multiprocessing import shared_memory
        if world > 32:
            raise ValueError("DirectPeers: at most 32 ranks")
        self.shard, self.nK, self.rank, self.world = shard, nK, rank, world
        self.nk = V.shape[-1]
        self.timeout_s = float(timeout_s)
        # three buffers (version v in buffer (v - 1) mod 3): a sweep writes the
        # buffer its neighbours finished reading two versions ago, so only its copy rows wait.
        # NaN outside the own columns: a read of a local copy instead of the owner's would show
        self.V = [torch.full_like(V, math.nan) for _ in range(3)]
        self.dV = [torch.full_like(V, math.nan) for _ in range(3)]
        self.own = owned_columns(nK, rank, world, bounds)
        plan = halo_plan(shard.kp_idx, nK, world, bounds)
        self.nbr = sorted({p for p in range(world) if p != rank and (plan[rank][p] or plan[p][rank])})
        self.mask = sum(1 << p for p in self.nbr)
        # IPC handles of the six buffers, every rank's (a failure on any rank is raised on
        # every rank, after the same collectives, so no rank is left inside one)
        mine, fail_msg = [], None
        try:
            for t in self.V + self.dV:
                h = (C.c_char * 64)()
                off = C.c_int64()
                check(lib().aiy_ipc_get_handle(ptr(t), h, C.byref(off)))
                mine.append((bytes(h), off.value))
        except Exception as e:  # noqa: BLE001 (re-raised collectively below)
            fail_msg = repr(e)
        allh = [None] * world
        dist.all_gather_object(allh, (mine, fail_msg))
        self._opened = []
        self._shm = None
        addr = []   # addr[q] = (V0, V1, V2, dV0, dV1, dV2) device addresses of rank q's buffers
        if not any(m for _, m in allh):
            try:
                for q in range(world):
                    if q == rank:
                        addr.append(tuple(t.data_ptr() for t in self.V + self.dV))
                        continue
                    # the caching allocator may put several of a rank's buffers in ONE segment
                    # (one handle): each distinct segment is opened once and closed once, the
                    # buffers are offsets into it (duplicate opens of one handle are
                    # runtime-dependent)
                    base = {}
                    row = []
                    for hb, off in allh[q][0]:
                        if hb not in base:
                            p_ = vp()
                            check(lib().aiy_ipc_open(C.create_string_buffer(hb, 64), i64(0),
                                                     C.byref(p_)))
                            base[hb] = p_.value
                            self._opened.append((p_.value, 0))
                        row.append(base[hb] + off)
                    addr.append(tuple(row))
            except Exception as e:  # noqa: BLE001
                fail_msg = repr(e)
        _agree_or_raise(fail_msg, V.device, "DirectPeers: IPC mapping", self._unmap)
        owner = [0] * (4 * nK)
        for q in range(world):
            for c in owned_columns(nK, q, world, bounds):
                owner[c] = q
        cb = 8 * self.nk
        # staged reads: the forecast columns peers own are copied into a
        # local halo once per sweep (after the wait, beside the interior launch), so no kernel
        # reads a peer's memory; the own columns split into interior (every forecast column
        # owned) and boundary (at least one copied)
        self.remote, interior, boundary = staged_plan(self.own, shard.kp_idx, owner, nK, rank)
        shard.set_split(interior, boundary)
        nr = len(self.remote)
        self.hV = torch.empty((max(nr, 1), self.nk), dtype=V.dtype, device=V.device)
        self.hdV = torch.empty_like(self.hV)
        slot = {c: i for i, c in enumerate(self.remote)}
        hv, hdv = self.hV.data_ptr(), self.hdV.data_ptr()

        def col(c, b, slope):
            if owner[c] != rank and c in slot:
                return (hdv if slope else hv) + cb * slot[c]
            return addr[owner[c]][(3 if slope else 0) + b] + cb * c
        self.tab = [torch.tensor([col(c, b, False) for c in range(4 * nK)] +
                                 [col(c, b, True) for c in range(4 * nK)],
                                 dtype=torch.int64, device=V.device) for b in range(3)]
        # the copies of one sweep: the owners' buffer-b value then slope columns -> the halo
        dev_arr = lambda xs: torch.tensor(xs or [0], dtype=torch.int64, device=V.device)
        self._src = [dev_arr([addr[owner[c]][b] + cb * c for c in self.remote] +
                             [addr[owner[c]][3 + b] + cb * c for c in self.remote])
                     for b in range(3)]
        self._dst = dev_arr([hv + cb * i for i in range(nr)] + [hdv + cb * i for i in range(nr)])
        self._ncopy = 2 * nr
        self._col_bytes = cb
        p3 = lambda ts: (C.c_void_p * 3)(*[t.data_ptr() for t in ts])  # host arrays of 3
        self._tabs, self._Vs, self._dVs = p3(self.tab), p3(self.V), p3(self.dV)
        self._srcs = p3(self._src)
        # the counter page: rank 0 creates it, every rank maps and registers it
        name, fail_msg = [None], None
        if rank == 0:
            try:
                self._shm = shared_memory.SharedMemory(create=True, size=self.PAGE)
                self._shm.buf[:self.PAGE] = bytes(self.PAGE)
                name[0] = self._shm.name
            except Exception as e:  # noqa: BLE001 (agreed below)
                fail_msg = repr(e)
        dist.broadcast_object_list(name, src=0)
        if rank != 0 and name[0] is not None:
            try:
                self._shm = shared_memory.SharedMemory(name=name[0])
                try:  # the creator unlinks it; keep this process's tracker from doing so too
                    from multiprocessing import resource_tracker
                    resource_tracker.unregister(self._shm._name, "shared_memory")
                except Exception:  # noqa: BLE001
                    pass
            except Exception as e:  # noqa: BLE001
                fail_msg = repr(e)
        elif name[0] is None:
            fail_msg = fail_msg or "rank 0 could not create the counter page"

        def _drop_page():
            self._unmap()
            if self._shm is not None:
                self._shm.close()
                if rank == 0:
                    self._shm.unlink()
                self._shm = None
        _agree_or_raise(fail_msg, V.device, "DirectPeers: counter page", _drop_page)
        self._host = C.c_char.from_buffer(self._shm.buf)
        self._hostp = C.addressof(self._host)
        dp = vp()
        fail_msg = None
        try:
            check(lib().aiy_host_register(C.c_void_p(self._hostp), i64(self.PAGE), C.byref(dp)))
        except Exception as e:  # noqa: BLE001
            fail_msg = repr(e)
            self._hostp_reg = False
        _agree_or_raise(fail_msg, V.device, "DirectPeers: host page", self.close)
        self._flags = dp.value
        self._err = self._flags + 8192 + 128 * rank     # this rank's error word (host-mapped)
        self._err_host = self._hostp + 8192 + 128 * rank
        self.n = 0     # sweeps this rank has published (identical schedule on every rank)
        dist.barrier()

    def error(self):
        return C.c_uint64.from_address(self._err_host).value

    def publish(self):
        self.n += 1
        check(lib().aiy_flag_set(C.c_void_p(self._flags), C.c_int32(self.rank),
                                 C.c_uint64(self.n), stream_handle(None)))

    def wait(self):
        check(lib().aiy_flags_wait(C.c_void_p(self._flags), C.c_uint64(self.mask),
                                   C.c_uint64(self.n), C.c_double(self.timeout_s),
                                   C.c_void_p(self._err), stream_handle(None)))

    def own_runs(self):
        return _runs(self.own)

    # the schedule (every rank calls the same sequence)
    def start(self, V):
        """Own columns of V into buffer 0, their slopes, and publish the next version (every
        rank restarts its buffer cycle here, after a barrier, so the version -> buffer map is
        the same on every rank)."""
        import torch
        import torch.distributed as dist
        torch.cuda.synchronize()
        dist.barrier()                 # peers finished with every buffer of a past schedule
        nk = self.nk
        for a, b in self.own_runs():
            self.V[0].view(-1, nk)[a:b].copy_(V.view(-1, nk)[a:b])
        self.cur = 0
        self.shard.slopes_own(self.V[0], self.dV[0])
        self.publish()

    def improve(self, kopt):
        """Policy improvement (:148-168) of the own nodes: after the wait, the peers' forecast
        columns are copied into the halo (stream-ordered), the own ones read in place."""
        self.wait()
        check(lib().ks_dev_halo_copy(ptr(self._src[self.cur]), ptr(self._dst),
                                     C.c_int32(self._ncopy), i64(self._col_bytes),
                                     stream_handle(None)))
        self.shard.set_columns(self.tab[self.cur])
        self.shard.improve_direct(kopt)

    def sweeps(self, kopt, n):
        """n Jacobi Howard sweeps (:172-192), ONE launch each (ks_dev_direct_sweeps /
        ks_dev_staged_sweep): publish the previous version, copy the peers' forecast columns once
        they have published theirs, interior columns meanwhile, boundary columns after the
        copies; then one publish of the last version."""
        if n <= 0:
            return
        check(lib().ks_dev_direct_sweeps(
            self.shard._h, self._tabs, self._Vs, self._dVs, ptr(kopt), C.c_int32(self.cur),
            i64(n), self._srcs, ptr(self._dst), C.c_int32(self._ncopy), i64(self._col_bytes),
            C.c_void_p(self._flags), C.c_int32(self.rank), C.c_uint64(self.mask),
            C.c_uint64(self.n), C.c_double(self.timeout_s), C.c_void_p(self._err),
            stream_handle(None)))
        self.n += n
        self.cur = (self.cur + n) % 3

    def current(self):
        return self.V[self.cur]

    def check(self):
        """Raise on every rank if a wait of any rank timed out (call after a host
        synchronisation; collective)."""
        e = self.error()
        msg = f"rank {self.rank} timed out waiting for rank {e - 1}'s sweep" if e else None
        _agree_or_raise(msg, self.V[0].device, "DirectPeers")

    def _unmap(self):
        for p_, off in self._opened:
            lib().aiy_ipc_close(C.c_void_p(p_), i64(off))
        self._opened = []

    def close(self):
        import torch
        import torch.distributed as dist
        if getattr(self, "_shm", None) is None:
            return
        torch.cuda.synchronize()
        self.shard.set_columns(None)   # its table points into the mappings released below
        dist.barrier()     # nobody reads a peer buffer or the page any more
        self._unmap()
        if getattr(self, "_hostp_reg", True):
            lib().aiy_host_unregister(C.c_void_p(self._hostp))
        del self._host
        self._shm.close()
        dist.barrier()
        if self.rank == 0:
            self._shm.unlink()
        self._shm = None


def _agree_or_raise(msg, device, what, cleanup=None):
    """Collective: if `msg` is set on any rank, every rank (after `cleanup`) raises."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1.0 if msg else 0.0], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if float(t[0]) > 0:
        if cleanup is not None:
            cleanup()
        raise RuntimeError(f"{what}: {msg or 'failed on another rank'}")


def _solve_direct(V, k_opt, shard, nK, howard_steps, tol, max_vfi, rank, world, bounds,
                  peers=None):
    """ks_vfi_solve_dist's loop on the direct schedule (DirectPeers); V, k_opt: full arrays on
    every rank (in), own columns current on return (the caller all-gathers)."""
    import torch
    import torch.distributed as dist
    if peers is not None and peers.shard is not shard:
        # the peers' neighbour mask and column tables were built from ITS shard's forecast
        # index (kp_idx, fixed by B at HipShard construction): with another shard (a new ALM B)
        # the solve would sweep the old B and skip waits it needs
        raise ValueError("DirectPeers was built for another shard (a different ALM B): build "
                         "one DirectPeers per shard")
    dp = peers if peers is not None else DirectPeers(shard, nK, rank, world, V, bounds)
    try:
        nk = dp.nk
        runs = dp.own_runs()
        flat = lambda t: t.view(-1, nk)
        Vold = torch.empty_like(V)
        dp.start(V)
        rel, it = math.nan, 0
        for it in range(1, max_vfi + 1):
            for a, b in runs:                  # value_old = value (:145), own columns
                flat(Vold)[a:b].copy_(flat(dp.current())[a:b])
            if (it - 1) % 5 == 0:              # policy improvement (:148-168)
                dp.improve(k_opt)
            dp.sweeps(k_opt, howard_steps)     # Jacobi Howard sweeps (:172-192)
            rel = shard.reldiff(dp.current(), Vold)   # :195 (host sync)
            dp.check()
            rel = _allreduce_max(rel, V.device)
            if rel < tol:
                break
        for a, b in runs:
            flat(V)[a:b].copy_(flat(dp.current())[a:b])
        return it, rel
    finally:
        # the shard must not keep the peers' column table past this solve, also on the error
        # path: a later halo/improve call would read it after DirectPeers.close()
        shard.set_columns(None)
        if peers is None:
            dp.close()


def _exchange(V, rank, world, nK, bounds=None):
    """All-gather every rank's owned columns of V (rows of the (4·nK, k) view) into every
    rank's V, in place."""
    import torch
    import torch.distributed as dist
    cols = [owned_columns(nK, q, world, bounds) for q in range(world)]
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


class HowardSweeps:
    """The Jacobi Howard sweeps of one rank (Krusell_Smith_VFI.m:172-192) with their exchanges.

    depth = 1: after every sweep the rank receives its halo (the forecast columns its nodes
    read, `halo_plan`), one batched point-to-point exchange per sweep.
    depth = m > 1 (communication-avoiding): before each block of L <= m sweeps the rank receives
    every foreign column of its ghost rectangle R_L (`ghost_rects`), then sweep i of the block
    runs on R_{L-i} — other ranks' columns are swept redundantly, with the same kernels on the
    same inputs, so every value is bit-identical to the single-device solve — and only the
    last sweep is confined to the rank's own nodes.  One exchange per block instead of per
    sweep; after a policy improvement the rank also receives k_opt on R_{m-1} (the ghost
    sweeps read it) and rebuilds the segment hints there.  After the last sweep the plain halo
    is exchanged, so the state between calls is the depth-1 schedule's.
    exchange = "allgather": every rank's owned slice to every rank after every sweep."""

    def __init__(self, shard, nK, rank, world, V, depth=1, exchange="halo", bounds=None):
        self.shard, self.nK, self.rank, self.world = shard, nK, rank, world
        self.bounds = bounds
        self.depth = max(1, int(depth)) if (world > 1 and exchange == "halo") else 1
        self.exchange = exchange
        self.halo = None
        self.blocks = {}     # L -> exchange before a block of L sweeps
        self.rects = [(shard.K0, shard.K1, shard.s0, shard.s1)]
        self.shards = [shard]
        self.kx = None
        self.dV = None
        nk = V.shape[-1]
        self.nk = nk
        if world > 1:
            if exchange == "halo":
                self.plan = halo_plan(shard.kp_idx, nK, world, bounds)
                self.halo = HaloExchange(self.plan, rank, world, V.device, nk, V.dtype)
                if self.depth > 1:
                    self.rects = ghost_rects(shard.kp_idx, nK, *self.rects[0], self.depth)
                    self.shards += [shard.ghost(*r) for r in self.rects[1:self.depth]]
                    for L in range(1, self.depth + 1):
                        self.blocks[L] = HaloExchange(ghost_plan(shard.kp_idx, nK, world, L, bounds),
                                                      rank, world, V.device, nk, V.dtype)
                    self.kx = self.blocks[self.depth - 1]   # k_opt on R_{m-1}
            elif exchange != "allgather":
                raise ValueError(f"exchange must be 'halo' or 'allgather', not {exchange!r}")
        if exchange == "allgather" or world == 1:
            import torch
            self.own = torch.tensor(owned_columns(nK, rank, world, bounds), device=V.device)

    def read_columns(self):
        """Every column this rank ever reads or sweeps (own, halo and ghost columns)."""
        cols = set(owned_columns(self.nK, self.rank, self.world, self.bounds))
        if self.halo is not None:
            cols |= {c for p in range(self.world) for c in self.plan[self.rank][p]}
        if self.depth > 1:
            cols |= set(rect_columns(self.rects[self.depth], self.nK))
        return cols

    def kopt_columns(self):
        """Every column of k_opt this rank's sweeps read."""
        cols = set(owned_columns(self.nK, self.rank, self.world, self.bounds))
        if self.depth > 1:
            cols |= set(rect_columns(self.rects[self.depth - 1], self.nK))
        return cols

    def improve(self, V, kopt):
        """Policy improvement (:148-168) on the rank's nodes; with ghost sweeps, k_opt of the
        ghost rectangle from its owners and the hints there."""
        self.shard.improve(V, kopt)
        if self.kx is not None:
            self.kx(kopt)
            self.shards[-1].hints(kopt)

    def _slope_bufs(self, V):
        if self.dV is None:
            import torch
            self.dV = [torch.empty_like(V), torch.empty_like(V)]
        return self.dV

    def run(self, V, V2, kopt, n):
        """n sweeps from V (current on the rank's nodes and halo); returns (V, V2) with V the
        newest buffer, current on the rank's nodes and halo.  One launch per sweep (the fused
        Howard + next-slopes kernel) whenever the columns a sweep reads were all written by
        the previous sweep: on one rank, and inside a ghost block; with a halo exchange after
        every sweep (depth 1 on several ranks) the received columns need their slopes rebuilt,
        so the sweep is slopes + Howard there."""
        if self.depth == 1 and self.world == 1:
            if n:
                dV, dV2 = self._slope_bufs(V)
                self.shard.slopes(V, dV)
                for _ in range(n):
                    self.shard.howard_fused(V, dV, kopt, V2, dV2)
                    V, V2 = V2, V
                    dV, dV2 = dV2, dV
            return V, V2
        if self.depth == 1:
            for _ in range(n):
                self.shard.howard(V, kopt, V2)
                if self.halo is None and self.world > 1:  # allgather: carry the rest over
                    fresh = V2.view(-1, self.nk).index_select(0, self.own)
                    V2.copy_(V)
                    V2.view(-1, self.nk).index_copy_(0, self.own, fresh)
                V, V2 = V2, V
                if self.halo is not None:
                    self.halo(V)
                elif self.world > 1:
                    _exchange(V, self.rank, self.world, self.nK, self.bounds)
            return V, V2
        done = 0
        dV, dV2 = self._slope_bufs(V)
        while done < n:
            L = min(self.depth, n - done)
            self.blocks[L](V)                     # R_L current at this sweep
            self.shards[L - 1].slopes(V, dV)      # what R_{L-1} reads (inside R_L)
            for i in range(1, L + 1):
                self.shards[L - i].howard_fused(V, dV, kopt, V2, dV2)   # R_{L-i} at sweep + i
                V, V2 = V2, V
                dV, dV2 = dV2, dV
            done += L
        if n:
            self.halo(V)
        return V, V2

    def close(self):
        owned = getattr(self.shard, "_ghosts", None)
        for g in self.shards[1:]:
            g.close()
            if owned is not None and g in owned:  # one solve per ALM step: do not accumulate
                owned.remove(g)
        self.shards = self.shards[:1]


def ks_vfi_solve_dist(value, k_opt, shard, nK, howard_steps=50, tol=1e-6, max_vfi=10000,
                      rank=0, world=1, exchange="halo", poison=False, depth=1, bounds=None,
                      peers=None):
    """Krusell_Smith_VFI.m:141-204 for the current B.  value, k_opt: (4, K, k) tensors on this
    rank's device, full arrays on every rank (in/out).  `shard` owns [K0, K1) of [s0, s1)
    (HipShard, or any object with the same improve / howard / reldiff / ghost / hints methods
    and a kp_idx table).  exchange: "halo" (point-to-point, only the columns read; `depth`
    sweeps per exchange, HowardSweeps), "allgather", or "direct" (forecast columns read in the
    owners' buffers through IPC mappings, DirectPeers; `peers`: a DirectPeers kept across
    solves, else one is made and closed per call).  bounds: the K partition the shards were
    made with (`shard_slices(..., bounds)`; None = even ranges).  poison (tests): NaN every column this
    rank neither owns nor reads, proving the exchanges are sufficient.
    Returns (iters, rel_diff)."""
    import torch
    import torch.distributed as dist
    V = value
    nk = V.shape[-1]
    if world > 1:
        dist.barrier()   # first collective on every rank before any point-to-point
    if exchange == "direct":
        if world == 1:
            exchange = "halo"
        else:
            it, rel = _solve_direct(V, k_opt, shard, nK, howard_steps, tol, max_vfi, rank, world,
                                    bounds, peers)
            _exchange(k_opt, rank, world, nK, bounds)   # every rank leaves with all of both
            _exchange(V, rank, world, nK, bounds)
            return it, rel
    hs = HowardSweeps(shard, nK, rank, world, V, depth=depth, exchange=exchange, bounds=bounds)
    if poison and world > 1 and exchange == "halo":
        keep = hs.read_columns()
        flat = V.view(-1, nk)
        kkeep, kflat = hs.kopt_columns(), k_opt.view(-1, nk)
        for c in range(4 * nK):
            if c not in keep:
                flat[c] = math.nan
            if c not in kkeep:
                kflat[c] = math.nan
    V2 = V.clone()
    rel, it = math.nan, 0
    try:
        for it in range(1, max_vfi + 1):
            Vold = V.clone()                                   # value_old = value (:145)
            if (it - 1) % 5 == 0:                              # policy improvement (:148-168)
                hs.improve(V, k_opt)
            V, V2 = hs.run(V, V2, k_opt, howard_steps)         # Jacobi Howard sweeps (:172-192)
            rel = shard.reldiff(V, Vold)                       # :195
            if world > 1:
                rel = _allreduce_max(rel, V.device)
            if rel < tol:
                break
    finally:
        hs.close()
    if world > 1:                                          # every rank leaves with all of both
        _exchange(k_opt, rank, world, nK, bounds)
        if exchange == "halo":
            _exchange(V, rank, world, nK, bounds)
    if V is not value:
        value.copy_(V)
    return it, rel
