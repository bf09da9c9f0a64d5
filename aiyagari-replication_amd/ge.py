"""A11 — the general-equilibrium bisection on r that drives the hot path (host side, like the
reference scripts' L4 loop), for all four Aiyagari scripts:

  aiyagari_vfi          Aiyagari_VFI.m:63-206
  aiyagari_labor_vfi    Aiyagari_Endogenous_Labor_VFI.m:59-256
  aiyagari_egm          Aiyagari_EGM.m:58-253     (w frozen at r = 0.04 inside the loop, :61)
  aiyagari_labor_egm    Aiyagari_Endogenous_Labor_EGM.m:54-251 (same quirk, :55)

Each: initial solve at r = 0.04 → Monte-Carlo capital supply (MATLAB's fresh-session rand
stream: randi(N), randi(Na), then 9,999 draws per simulation) → 10 bisection steps on
[-0.05, 1/beta - 1], warm-starting the solver, restarting the chain from the same (z1, k1).
Every solve and every simulation runs on the GPU through the C ABI.  With supply="histogram"
the Monte-Carlo estimator is replaced by K = Σ λ·a at the stationary histogram (A10, new).
"""
from __future__ import annotations

import math
import time

import numpy as np

from . import calibration as cb
from .dist import dist_stationary
from .egm import egm_solve, labor_egm_solve
from .sim import sim_capital
from .vfi import labor_vfi_solve, vfi_solve


def matlab_rand(n: int, seed: int = 5489) -> np.ndarray:
    """MATLAB's `rand` stream in a fresh session: MT19937 seeded 5489, 53-bit doubles."""
    return np.random.RandomState(seed).random_sample(n)


class _Stream:
    def __init__(self, T, steps):
        self.u = matlab_rand(2 + (T - 1) * (steps + 1))
        self.pos = 0

    def take(self, n):
        out = self.u[self.pos:self.pos + n]
        self.pos += n
        return out


def _bisect(cal, solve_at, supply_of, max_r_iter=10, r_tol=1e-5):
    """Aiyagari_VFI.m:133-206: r_mid each step, K_d = labor (alpha/(r+delta))^(1/(1-alpha))."""
    r_low, r_high = -0.05, 1 / cal["beta"] - 1
    out = dict(r_history=[], k_supply=[], k_demand=[], iters=[])
    r = math.nan
    for _ in range(max_r_iter):
        r_guess = (r_low + r_high) / 2
        r = r_guess
        it = solve_at(r)
        Ks = supply_of()
        Kd = cb.capital_demand(r_guess, cal["labor"], cal["alpha"], cal["delta"])
        out["r_history"].append(r); out["k_supply"].append(Ks); out["k_demand"].append(Kd)
        out["iters"].append(it)
        if abs(Ks - Kd) < r_tol:
            break
        elif Ks > Kd:
            r_high = r_guess
        else:
            r_low = r_guess
    out["r"] = r
    return out


def aiyagari_vfi(Na=400, rho=0.75, sigma_e=0.75, shocks="tauchen", T=10000, tol=1e-5,
                 max_iter=1000, supply="mc", r0=0.04):
    """The whole of Aiyagari_VFI.m's computation (no plots)."""
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=rho, sigma_e=sigma_e, shocks=shocks)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    st = _Stream(T, 10)
    z1 = int(math.ceil(N * st.take(1)[0]))                  # randi(N)  (1-based)
    k1 = a[int(math.ceil(Na * st.take(1)[0])) - 1]          # a_grid(randi(grid_size))
    state = {"v_old": np.zeros((N, Na))}

    def solve_at(r):
        R = vfi_solve(state["v_old"], a, s, P, r, cb.wage(r, cal["alpha"], cal["delta"]),
                      cal["beta"], cal["sigma"], tol, max_iter)
        state.update(v_old=R["v_old"], R=R)
        return R["iters"]

    def supply_of():
        R = state["R"]
        if supply == "mc":
            return sim_capital(R["policy_k"], a, P, z1, k1, st.take(T - 1))
        _, K, _, _ = dist_stationary(a, P, policy_idx=R["idx"], tol=1e-13, max_iter=100000)
        return K

    it0 = solve_at(r0)
    supply_of()
    out = _bisect(cal, solve_at, supply_of)
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    out["cal"] = cal
    return out


def aiyagari_labor_vfi(Na=400, T=10000, tol=1e-5, max_iter=1000, supply="mc", r0=0.04,
                       labor_choice=None, psi=1.0, eta=2.0):
    """Aiyagari_Endogenous_Labor_VFI.m (rho = .6, sigma_e = .2, 10 labour levels)."""
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    L = (0.01 + (1.5 - 0.01) * cb.linspace01(10)) if labor_choice is None else np.asarray(labor_choice)
    st = _Stream(T, 10)
    z1 = int(math.ceil(N * st.take(1)[0]))
    k1 = a[int(math.ceil(Na * st.take(1)[0])) - 1]
    state = {"v_old": np.zeros((N, Na)), "v_new": None, "pol": None}

    def solve_at(r):
        R = labor_vfi_solve(state["v_old"], a, s, P, L, r, cb.wage(r, cal["alpha"], cal["delta"]),
                            cal["beta"], cal["sigma"], psi, eta, tol, max_iter,
                            v_new=state["v_new"], policies=state["pol"])
        state.update(v_old=R["v_old"], v_new=R["v_new"], R=R,
                     pol=(R["policy_k"], R["policy_l"], R["policy_c"], R["lin"]))
        return R["iters"]

    def supply_of():
        R = state["R"]
        if supply == "mc":
            return sim_capital(R["policy_k"], a, P, z1, k1, st.take(T - 1))
        idx = (R["lin"] - 1) // len(L) + 1
        _, K, _, _ = dist_stationary(a, P, policy_idx=idx, tol=1e-13, max_iter=100000)
        return K

    it0 = solve_at(r0)
    supply_of()
    out = _bisect(cal, solve_at, supply_of)
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    return out


def _egm_common(labor, Na, T, tol, max_iter, supply, phi=1.0, theta=1.0):
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=0.6 if labor else 0.75, sigma_e=0.2 if labor else 0.75)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    r0 = 0.04
    w = cb.wage(r0, cal["alpha"], cal["delta"])  # frozen: the GE loop never updates w (:61)
    pc = np.tile(((1 + r0) * a + w * np.mean(s))[:, None], (1, N))  # :64
    st = _Stream(T, 10)
    z1 = int(math.ceil(N * st.take(1)[0]))
    k1 = a[int(math.ceil(Na * st.take(1)[0])) - 1]
    state = {"pc": pc}

    def solve_at(r):
        if labor:
            R = labor_egm_solve(state["pc"], a, s, P, r, w, cal["beta"], cal["sigma"], phi, theta,
                                cal["amin"], tol, max_iter)
        else:
            R = egm_solve(state["pc"], a, s, P, r, w, cal["beta"], cal["sigma"], cal["amin"], tol,
                          max_iter)
        state.update(pc=R["policy_c"], R=R)
        return R["iters"]

    def supply_of():
        R = state["R"]
        if supply == "mc":
            return sim_capital(R["policy_k"], a, P, z1, k1, st.take(T - 1), vfi_layout=False)
        _, K, _, _ = dist_stationary(a, P, policy_k=R["policy_k"], tol=1e-13, max_iter=100000,
                                     vfi_layout=False)
        return K

    it0 = solve_at(r0)
    supply_of()
    out = _bisect(cal, solve_at, supply_of)
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    return out


def aiyagari_egm(Na=400, T=10000, tol=1e-5, max_iter=1000, supply="mc"):
    """Aiyagari_EGM.m."""
    return _egm_common(False, Na, T, tol, max_iter, supply)


def aiyagari_labor_egm(Na=400, T=10000, tol=1e-5, max_iter=1000, supply="mc", phi=1.0,
                       theta=1.0):
    """Aiyagari_Endogenous_Labor_EGM.m."""
    return _egm_common(True, Na, T, tol, max_iter, supply, phi, theta)


def aiyagari_vfi_overlapped(Na=400, rho=0.75, sigma_e=0.75, shocks="tauchen", T=10000, tol=1e-5,
                            max_iter=1000, r0=0.04, max_r_iter=10, r_tol=1e-5, lookahead=2):
    """Aiyagari_VFI.m's computation (as `aiyagari_vfi`, supply = MC) with the bisection run
    speculatively ahead of its serial Monte-Carlo chains.  Step j needs K_s(r_j) only to pick
    the next midpoint, and both candidates warm-start from the same v_old(r_j): so every solve
    that finishes starts its own chain at once AND the solves at both of its possible next
    midpoints, up to `lookahead` bisection levels ahead of the step still waiting for its
    chain (each on its own stream and workspace, one host thread per call; ctypes drops the
    GIL); a chain's K_s selects one subtree and the other is discarded.  Every solve and chain
    is the one the sequential loop runs, on the same inputs and uniform block, so r_history /
    k_supply / iters are identical (tests/test_ge_gpu.py).  Default lookahead = 2: with the
    speculative-segment chain (~0.66 ms per 10^4 steps) shorter than a warm small-grid solve
    (~0.7-1.5 ms), the second level keeps the next solves running while the chosen solve's
    chain runs (16.4-17.5 vs 16.9-19.7 ms, profiles/r06_g20_ge_lookahead.txt); deeper trees
    keep more than ~4 streams busy, which this runtime serves slower (profiles/
    r06_g14_hw_queues.txt; round 5, with 1.6 ms chains, lookahead 1 won: r05_g32)."""
    import concurrent.futures as cf

    import torch

    from .sim import sim_capital_dev
    from .vfi import Workspace

    if lookahead < 1:
        raise ValueError("lookahead >= 1")
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=rho, sigma_e=sigma_e, shocks=shocks)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    st = _Stream(T, max_r_iter)
    z1 = int(math.ceil(N * st.take(1)[0]))
    k1 = float(a[int(math.ceil(Na * st.take(1)[0])) - 1])
    dev = torch.device("cuda", torch.cuda.current_device())
    tt = lambda x: torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev)
    a_t, s_t, P_t = tt(a), tt(s), tt(P)
    U = tt(st.u[st.pos:])  # block j (the j-th chain's T-1 draws) = U[j(T-1) : (j+1)(T-1)]

    timeline = []  # (kind, r, j, host start, host end) of every solve and chain (diagnostics)

    def solve(slot, v_init, r, j=-1):
        t_a = time.perf_counter()
        stream = streams.get()  # (a bounded set: every stream its own hardware queue)
        with torch.cuda.stream(stream):
            slot.va.copy_(v_init)
            slot.vb.zero_()
            it, which = slot.ws.vfi_solve(
                slot.va, slot.vb, a_t, s_t, P_t, r, cb.wage(r, cal["alpha"], cal["delta"]),
                cal["beta"], cal["sigma"], tol, max_iter, slot.idx, slot.pk, slot.pc,
                stream=stream)
        _wait_polled(stream)
        streams.put(stream)
        slot.v_old = slot.vb if which == 0 else slot.va
        timeline.append(("solve", r, j, t_a - t0, time.perf_counter() - t0, it))
        return it

    def chain(sim, slot, j):
        t_a = time.perf_counter()
        stream = streams.get()
        with torch.cuda.stream(stream):
            sim_capital_dev(sim.ws, slot.pk, a_t, P_t, z1 - 1, k1, U[j * (T - 1):(j + 1) * (T - 1)],
                            sim.k, sim.status, stream=stream)
            sim.kh.copy_(sim.k, non_blocking=True)
            sim.sh.copy_(sim.status, non_blocking=True)
        # a chain runs ~1.6 ms: poll its event instead of a blocking synchronize (a thread
        # parked in a synchronize slowed the other threads' launches 2-3x)
        _wait_polled(stream, nap=_CHAIN_NAP)
        streams.put(stream)
        if int(sim.sh[0]) != 0:
            raise RuntimeError("find() empty in the capital-supply chain (Aiyagari_VFI.m:106)")
        timeline.append(("chain", None, j, t_a - t0, time.perf_counter() - t0, 0))
        return float(sim.kh[0])

    class _Node:  # bisection step j at r (bracket lo, hi before the step)
        def __init__(self, j, lo, hi, parent):
            self.j, self.lo, self.hi, self.parent = j, lo, hi, parent
            self.r = (lo + hi) / 2
            self.slot = self.it = self.Ks = None
            self.kids = None        # (lo child, hi child) once spawned
            self.refs = 0           # outstanding futures using this node's slot (its solve,
            #                         its chain, its children's solves reading its v_old)
            self.alive = True
            self.chained = False
            self.err = None         # a solve's or chain's exception

    # solve slots and chain resources persist across calls (per device and grid): a new
    # workspace allocates its scratch with hipMalloc / hipMemset on first use, which would
    # synchronise the device in the middle of the speculative pipeline
    key = (dev.index, N, Na)
    pools = _GE_POOLS.setdefault(key, ([], []))
    all_slots, all_sims = [], []
    free_slots, free_sims = pools[0], pools[1]
    # streams: as many as solves and chains can run at once (2^lookahead + 2 solves, as many
    # chains) and no more — the runtime deals streams over its hardware queues (GPU_MAX_HW_QUEUES)
    # and a kernel queued behind a 2.7 ms chain on a shared queue waits for it
    import queue
    nstreams = 2 * (2 ** lookahead + 2)
    spool = _GE_STREAMS.setdefault(dev.index, [])
    while len(spool) < nstreams:
        spool.append(torch.cuda.Stream(device=dev))
    streams = queue.Queue()
    for x in spool[:nstreams]:
        streams.put(x)

    def get(free, pool_all, make):
        if free:
            x = free.pop()
            # a pooled workspace caches its feasible prefixes keyed on (r, w) and the
            # raw addresses of a and s, not their contents; a later call with another
            # calibration at the same Na can get a_t / s_t at the same addresses and repeat an
            # r, so every reuse drops the cache (host-side flags only, no device work)
            x.ws.invalidate()
        else:
            x = make()
        pool_all.append(x)
        return x

    out = dict(r_history=[], k_supply=[], k_demand=[], iters=[])
    fut = {}
    try:
        _run_tree(locals())
    finally:
        # every slot and chain resource goes back to the pools, also on an error
        free_slots[:] = list({id(x): x for x in free_slots + all_slots}.values())
        free_sims[:] = list({id(x): x for x in free_sims + all_sims}.values())
    out["r"] = out["r_history"][-1]
    out["iters"] = [out.pop("it0")] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    out["cal"] = cal
    out["lookahead"] = lookahead
    out["solves"] = len(all_slots)
    out["timeline"] = sorted(timeline, key=lambda e: e[3])
    return out


def _run_tree(env):
    """The speculative tree of aiyagari_vfi_overlapped (its closure state passed in `env`)."""
    import concurrent.futures as cf
    solve, chain, get = env["solve"], env["chain"], env["get"]
    _Node, cal, dev = env["_Node"], env["cal"], env["dev"]
    N, Na, r0 = env["N"], env["Na"], env["r0"]
    free_slots, all_slots = env["free_slots"], env["all_slots"]
    free_sims, all_sims = env["free_sims"], env["all_sims"]
    out, fut = env["out"], env["fut"]
    max_r_iter, r_tol, lookahead = env["max_r_iter"], env["r_tol"], env["lookahead"]
    import torch
    with cf.ThreadPoolExecutor(max_workers=16) as pool:
        root = get(free_slots, all_slots, lambda: _GESlot(N, Na, dev))
        it0 = solve(root, torch.zeros((N, Na), dtype=torch.float64, device=dev), r0)
        r_low, r_high = -0.05, 1 / cal["beta"] - 1
        sim0 = get(free_sims, all_sims, lambda: _GESim(N, Na, dev))
        fut[pool.submit(chain, sim0, root, 0)] = ("chain0", None, sim0)  # (K_s at r0 unused)

        def submit_solve(node, v_init):
            node.slot = get(free_slots, all_slots, lambda: _GESlot(N, Na, dev))
            node.refs += 1  # (its own solve: a node killed meanwhile keeps its slot until then)
            fut[pool.submit(solve, node.slot, v_init, node.r, node.j)] = ("solve", node, None)

        def spawn(node):  # both next midpoints of a solved node, from its v_old
            node.kids = (_Node(node.j + 1, node.lo, node.r, node),
                         _Node(node.j + 1, node.r, node.hi, node))
            for kid in node.kids:
                node.refs += 1
                submit_solve(kid, node.slot.v_old)

        def release(node):  # the slot back to the pool when nothing reads it any more
            if node.slot is not None and node.refs == 0 and (not node.alive or node.j < cur.j):
                free_slots.append(node.slot)
                node.slot = None

        def kill(node):
            if node is None:
                return
            node.alive = False
            release(node)
            if node.kids:
                for kid in node.kids:
                    kill(kid)

        def advance(node):  # a solved live node: its chain, and its children within the window
            if not node.alive or node.slot is None or node.it is None:
                return
            if not node.chained:
                node.chained = True
                node.refs += 1
                sim = get(free_sims, all_sims, lambda: _GESim(N, Na, dev))
                fut[pool.submit(chain, sim, node.slot, node.j)] = ("chain", node, sim)
            if node.kids is None and node.j < max_r_iter and node.j - cur.j < lookahead:
                spawn(node)
            elif node.kids:
                for kid in node.kids:
                    advance(kid)

        cur = _Node(1, r_low, r_high, None)
        submit_solve(cur, root.v_old)
        done = False
        try:
            while fut and not done:
                finished, _ = cf.wait(list(fut), return_when=cf.FIRST_COMPLETED)
                for f in finished:
                    kind, node, sim = fut.pop(f)
                    try:
                        res, err = f.result(), None
                    except Exception as e:  # kept on the node: raised only if the path needs it
                        res, err = None, e
                    if sim is not None:
                        free_sims.append(sim)
                    if kind == "chain0":
                        if err is not None:  # the sequential script runs this chain too
                            raise err
                        continue
                    if kind == "solve":
                        node.it, node.err = res, err
                        node.refs -= 1
                        if node.parent is not None:
                            node.parent.refs -= 1
                            release(node.parent)
                        if not node.alive or err is not None:
                            release(node)
                            continue
                        advance(node)
                        continue
                    node.Ks, node.err = res, err  # a chain
                    node.refs -= 1
                    release(node)
                # decisions: the current step's chain, then (already chained) the steps after it
                while not done and (cur.Ks is not None or cur.err is not None):
                    if cur.err is not None:  # a failure on the sequential loop's own path
                        raise cur.err
                    Kd = cb.capital_demand(cur.r, cal["labor"], cal["alpha"], cal["delta"])
                    out["r_history"].append(cur.r); out["k_supply"].append(cur.Ks)
                    out["k_demand"].append(Kd); out["iters"].append(cur.it)
                    if cur.j == max_r_iter or abs(cur.Ks - Kd) < r_tol:
                        done = True
                        break
                    nxt, other = ((cur.kids[0], cur.kids[1]) if cur.Ks > Kd
                                  else (cur.kids[1], cur.kids[0]))
                    kill(other)
                    prev, cur = cur, nxt
                    release(prev)
                    advance(cur)
        finally:
            # speculative work still running finishes before the slots go back to the pools;
            # its results and errors (killed nodes, steps past the last) are ignored
            for f in list(fut):
                try:
                    f.result()
                except Exception:
                    pass
    out["it0"] = it0


def _wait_polled(stream, nap=0.0):
    """Wait for the work queued so far on `stream` by polling an event (hipEventQuery), not
    parking the thread in a blocking synchronize: concurrent host threads blocked in the runtime
    slowed one another's launches (tools/ge_concurrency.py)."""
    import torch
    ev = torch.cuda.Event()
    ev.record(stream)
    while not ev.query():
        time.sleep(nap)


class _GESlot:
    """One speculative solve's resources (aiyagari_vfi_overlapped): workspace and buffers;
    state only — the calls that use it pass every input explicitly (a slot outlives a call)."""

    def __init__(self, N, Na, dev):
        import torch

        from .vfi import Workspace
        self.ws = Workspace(N, Na)
        self.va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
        self.vb = torch.zeros_like(self.va)
        self.idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
        self.pk, self.pc = torch.empty_like(self.va), torch.empty_like(self.va)
        self.v_old = None
        # the zero fills above are on the creating thread's current stream: done before this
        # slot's own stream touches the buffers (no cross-stream order otherwise)
        torch.cuda.current_stream(dev).synchronize()


class _GESim:
    """One Monte-Carlo chain's resources: workspace and outputs."""

    def __init__(self, N, Na, dev):
        import torch

        from .vfi import Workspace
        self.ws = Workspace(N, Na)
        # the chain's workgroup reserves its CU so no speculative solve block shares it (a
        # co-resident block slows the serial wave; opt-in per workspace since ADVICE r5)
        self.ws.set_cu_exclusive(True)
        self.ws.set_sim(_GE_SIM_MODE)
        self.k = torch.zeros(1, dtype=torch.float64, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.kh = torch.zeros(1, dtype=torch.float64).pin_memory()  # host copies (pinned)
        self.sh = torch.zeros(1, dtype=torch.int32).pin_memory()
        torch.cuda.current_stream(dev).synchronize()


# host poll interval of a Monte-Carlo chain's completion (seconds; AIY_GE_CHAIN_NAP for A/B):
# 20 us, not 200 — the step after a chain waits for its K_s (GE wall 25.1 -> 22.9 ms median over
# three alternating rounds; busy polling 23.6)
import os as _os  # noqa: E402
_CHAIN_NAP = float(_os.environ.get("AIY_GE_CHAIN_NAP", "2e-5"))  # profiles/r06_g15_ge_chain_nap.txt
# the chains' variant (aiy_ws_set_sim; an A/B knob, results identical): -1 by size
_GE_SIM_MODE = int(_os.environ.get("AIY_GE_SIM_MODE", "-1"))
_GE_POOLS = {}  # (device, N, Na) -> (solve slots, chain resources) of aiyagari_vfi_overlapped
_GE_STREAMS = {}  # device -> the driver's streams


def release_pools():
    """Free the cached workspaces of aiyagari_vfi_overlapped."""
    for slots, sims in _GE_POOLS.values():
        for x in slots + sims:
            x.ws.close()
    _GE_POOLS.clear()
