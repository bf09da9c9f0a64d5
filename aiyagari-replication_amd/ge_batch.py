"""E2 / BASELINE config 4 — the general-equilibrium r search with many candidate interest
rates solved at once across ranks (one process per GPU, torch.distributed over RCCL).

The reference loop (Aiyagari_VFI.m:131-206) is a 10-step bisection: r = (r_low + r_high)/2,
solve, simulate K_s, compare with K_d, halve the bracket.  Its steps are sequential, but the
points it *may* visit are known in advance: the midpoints of the bisection tree.  A round
evaluates every node of the next L levels of that tree (2^L - 1 candidate rates, each node
computed from its parent bracket exactly as the sequential loop would, bit for bit), spread
round-robin over the ranks; one all-gather of (K_s, K_d) per round (the only collective,
8 bytes x 2 per candidate) lets every rank walk the path the sequential loop would take, with
its early stop |K_s - K_d| < 1e-5.  The all-gather is one float64 tensor collective
(all_gather_into_tensor over RCCL).  Two rounds of L = 6 cover the reference's 10 steps.

Path independence: a node's result must not depend on which nodes were solved before it on
the same rank.  Every candidate therefore starts its VFI from the same value function (the
solution at r0, "warm from r0"), and its Monte-Carlo supply uses the uniforms block of its
tree depth (the block the sequential loop would use at that step).  The sequential twin
`bisection(..., warm="r0")` gives the identical trace (tests/test_ge_batch_*.py); the
reference's own chained warm start (previous step's v_old) differs from it at the
convergence-tolerance level and is reproduced by ge.aiyagari_vfi.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Node:
    depth: int        # 1-based bisection step
    r: float
    lo: float
    hi: float


def subtree(lo: float, hi: float, depth0: int, levels: int) -> list[Node]:
    """The 2^levels - 1 midpoints below bracket (lo, hi), breadth-first, each computed as the
    sequential loop computes it: r = (lo + hi)/2 of its own bracket (Aiyagari_VFI.m:143)."""
    out, frontier = [], [(lo, hi)]
    for lev in range(levels):
        nxt = []
        for (a, b) in frontier:
            m = (a + b) / 2
            out.append(Node(depth0 + lev, m, a, b))
            nxt += [(a, m), (m, b)]
        frontier = nxt
    return out


@dataclass
class Trace:
    r_history: list = field(default_factory=list)
    k_supply: list = field(default_factory=list)
    k_demand: list = field(default_factory=list)
    iters: list = field(default_factory=list)
    r: float = math.nan
    rounds: int = 0
    candidates: int = 0


def walk(nodes: list[Node], res: dict, lo: float, hi: float, steps: int, tr: Trace, tol: float):
    """Follow the sequential loop's path through an evaluated subtree (Aiyagari_VFI.m:195-204).
    Returns (lo, hi, stopped)."""
    by_key = {(n.lo, n.hi): n for n in nodes}
    for _ in range(steps):
        n = by_key[(lo, hi)]
        Ks, Kd, it = res[(n.lo, n.hi)]
        tr.r_history.append(n.r); tr.k_supply.append(Ks); tr.k_demand.append(Kd)
        tr.iters.append(it)
        tr.r = n.r
        if abs(Ks - Kd) < tol:
            return lo, hi, True
        if Ks > Kd:
            hi = n.r
        else:
            lo = n.r
    return lo, hi, False


def multisection(evaluate, r_low, r_high, max_steps=10, levels=6, tol=1e-5, rank=0, world=1,
                 allgather=None) -> Trace:
    """evaluate(node) -> (K_s, K_d, iters) for the nodes this rank owns (index % world == rank),
    or, when `evaluate` has an `many` attribute, evaluate.many(nodes) -> list of triples for all
    of them at once (the batched device path); allgather(mine, n_nodes) -> list over ranks of
    lists (None when world == 1; torch_allgather: one tensor all-gather per round)."""
    tr = Trace()
    lo, hi, done, step = r_low, r_high, False, 0
    while not done and step < max_steps:
        L = min(levels, max_steps - step)
        nodes = subtree(lo, hi, step + 1, L)
        own = [q for q in range(len(nodes)) if q % world == rank]
        if hasattr(evaluate, "many"):
            mine = list(zip(own, evaluate.many([nodes[q] for q in own]))) if own else []
        else:
            mine = [(q, evaluate(nodes[q])) for q in own]
        if world > 1:
            parts = allgather(mine, len(nodes))
            allres = [x for part in parts for x in part]
        else:
            allres = mine
        res = {(nodes[q].lo, nodes[q].hi): v for q, v in allres}
        lo, hi, done = walk(nodes, res, lo, hi, L, tr, tol)
        step += L
        tr.rounds += 1
        tr.candidates += len(nodes)
    return tr


def bisection(evaluate, r_low, r_high, max_steps=10, tol=1e-5) -> Trace:
    """The sequential twin (the reference loop's control flow) over the same evaluator."""
    tr = Trace()
    lo, hi = r_low, r_high
    for step in range(max_steps):
        n = Node(step + 1, (lo + hi) / 2, lo, hi)
        Ks, Kd, it = evaluate(n)
        tr.r_history.append(n.r); tr.k_supply.append(Ks); tr.k_demand.append(Kd)
        tr.iters.append(it)
        tr.r = n.r
        tr.candidates += 1
        if abs(Ks - Kd) < tol:
            break
        if Ks > Kd:
            hi = n.r
        else:
            lo = n.r
    tr.rounds = len(tr.r_history)
    return tr


def torch_allgather(mine, n_nodes):
    """The round's one collective (Aiyagari_VFI.m:193-204's decision inputs): every rank's
    (q, K_s, K_d, iters) rows as one float64 tensor [ceil(n_nodes / world), 4] (padding rows
    q = -1), gathered with all_gather_into_tensor — RCCL on GPU ranks (the tensor lives on the
    rank's current device), gloo on CPU.  All four fields are exact in float64 (q, iters are
    small integers).  Returns the list over ranks of [(q, (K_s, K_d, iters)), ...]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    rows = -(-n_nodes // world)
    if len(mine) > rows:
        raise ValueError(f"{len(mine)} results on one rank, at most {rows} expected")
    dev = (torch.device("cuda", torch.cuda.current_device())
           if dist.get_backend() == "nccl" else torch.device("cpu"))
    buf = torch.full((rows, 4), -1.0, dtype=torch.float64)
    for n, (q, (ks, kd, it)) in enumerate(mine):
        buf[n] = torch.tensor([q, ks, kd, it], dtype=torch.float64)
    out = torch.empty((world * rows, 4), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, buf.to(dev))
    got = out.cpu().view(world, rows, 4).tolist()
    return [[(int(q), (ks, kd, int(it))) for q, ks, kd, it in part if q >= 0] for part in got]


# ------------------------------------------------------------------------------ evaluators
def mc_stream(T=10000, steps=10, seed=5489):
    """MATLAB's fresh-session rand stream split as the VFI script consumes it: randi(N),
    randi(Na), then one block of T-1 uniforms per simulation (initial solve, then step d)."""
    u = np.random.RandomState(seed).random_sample(2 + (T - 1) * (steps + 1))
    head = u[:2]
    blocks = [u[2 + b * (T - 1): 2 + (b + 1) * (T - 1)] for b in range(steps + 1)]
    return head, blocks


def vfi_evaluator(cal, solve, simulate, v_start, T=10000, tol=1e-5, max_iter=1000):
    """Node evaluator for Aiyagari_VFI.m: VFI from v_start (path-independent warm start), MC
    supply with the uniforms block of the node's depth, K_d (:195).
    solve(v_old, r, w) -> dict(policy_k, iters); simulate(policy_k, z1, k1, uniforms) -> K_s."""
    from . import calibration as cb
    N, Na, a = cal["N"], cal["Na"], cal["a_grid"]
    head, blocks = mc_stream(T)
    z1 = int(math.ceil(N * head[0]))
    k1 = a[int(math.ceil(Na * head[1])) - 1]

    def evaluate(node):
        r = node.r
        R = solve(v_start, r, cb.wage(r, cal["alpha"], cal["delta"]))
        Ks = simulate(R["policy_k"], z1, k1, blocks[node.depth])
        Kd = cb.capital_demand(r, cal["labor"], cal["alpha"], cal["delta"])
        return (float(Ks), float(Kd), int(R["iters"]))
    return evaluate


def hip_vfi_evaluator(cal, v_start, T=10000, tol=1e-5, max_iter=1000):
    """The evaluator on this rank's GPU through the C ABI (host tier)."""
    from .sim import sim_capital
    from .vfi import vfi_solve

    def solve(v, r, w):
        return vfi_solve(v, cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"],
                         tol, max_iter)

    def simulate(pk, z1, k1, u):
        return sim_capital(pk, cal["a_grid"], cal["P"], z1, k1, u)
    return vfi_evaluator(cal, solve, simulate, v_start, T, tol, max_iter)


def ge_batch_call(r, v_start, cal, z1, k1, blocks, tol=1e-5, max_iter=1000, n_devices=1):
    """aiy_ge_batch (C ABI): K_s, K_d and iteration count at every rate in `r`, each
    from v_start, with uniforms blocks[c] (T-1 draws) for candidate c; z1 1-based."""
    import ctypes as C
    from ._capi import check, d, i64, ip, lib, ptr
    r = np.ascontiguousarray(r, np.float64)
    n = r.size
    N, Na = cal["N"], cal["Na"]
    U = np.asfortranarray(np.stack([np.asarray(b, np.float64) for b in blocks], axis=1))
    T = U.shape[0] + 1
    v = np.asfortranarray(v_start, dtype=np.float64)
    a = np.ascontiguousarray(cal["a_grid"], np.float64)
    s = np.ascontiguousarray(cal["s"], np.float64)
    P = np.asfortranarray(cal["P"], dtype=np.float64)
    Ks, Kd, it = np.empty(n), np.empty(n), np.empty(n, np.int64)
    check(lib().aiy_ge_batch(ptr(r), i64(n), ptr(v), ptr(a), ptr(s), ptr(P), i64(N), i64(Na),
                             d(cal["alpha"]), d(cal["delta"]), d(cal["beta"]), d(cal["sigma"]),
                             d(cal["labor"]), d(tol), i64(max_iter), i64(z1), d(k1), i64(T),
                             ptr(U), ip(n_devices), ptr(Ks), ptr(Kd), ptr(it)))
    return Ks, Kd, it


def hip_batch_evaluator(cal, v_start, T=10000, tol=1e-5, max_iter=1000, n_devices=1):
    """The node evaluator on the batched device path: all of a round's nodes of this rank in
    one aiy_ge_batch call (one batched solve and one batched launch of the chains per GPU).
    Same per-node arithmetic as vfi_evaluator, so the traces are identical."""
    N, Na, a = cal["N"], cal["Na"], cal["a_grid"]
    head, blocks = mc_stream(T)
    z1 = int(math.ceil(N * head[0]))
    k1 = a[int(math.ceil(Na * head[1])) - 1]

    def many(nodes):
        Ks, Kd, it = ge_batch_call([n.r for n in nodes], v_start, cal, z1, k1,
                                   [blocks[n.depth] for n in nodes], tol, max_iter, n_devices)
        return [(float(Ks[q]), float(Kd[q]), int(it[q])) for q in range(len(nodes))]

    def evaluate(node):
        return many([node])[0]
    evaluate.many = many
    return evaluate


def auto_levels(world: int) -> int:
    """Tree levels per round so that one round's 2^L - 1 candidates fit the ranks (one each)."""
    return max(1, int(math.floor(math.log2(world + 1))))


def aiyagari_vfi_multisection(Na=400, levels=None, rank=0, world=1, allgather=None, r0=0.04,
                              shocks="tauchen", batched=True):
    """Config 4: the GE of Aiyagari_VFI.m with candidate rates spread over `world` ranks.
    Every rank solves r0 once (the common warm start), then the rounds; batched=True evaluates
    each rank's nodes of a round in one batched device call (else one solve after another).
    levels=None picks auto_levels(world); BASELINE's 64-candidate configuration is levels=6."""
    levels = auto_levels(world) if levels is None else levels
    from . import calibration as cb
    from .vfi import vfi_solve
    cal = cb.aiyagari(Na=Na, shocks=shocks)
    R0 = vfi_solve(np.zeros((cal["N"], Na)), cal["a_grid"], cal["s"], cal["P"], r0,
                   cb.wage(r0, cal["alpha"], cal["delta"]), cal["beta"], cal["sigma"])
    ev = (hip_batch_evaluator if batched else hip_vfi_evaluator)(cal, R0["v_old"])
    lo, hi = -0.05, 1 / cal["beta"] - 1
    return multisection(ev, lo, hi, levels=levels, rank=rank, world=world,
                        allgather=allgather if allgather else (torch_allgather if world > 1 else None))
