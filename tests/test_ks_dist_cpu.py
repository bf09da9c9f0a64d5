"""CPU: the sharded Krusell-Smith VFI driver (ks_dist.py) over gloo with 2 ranks.  The shard
backend here is the C restatement (oracle/ — test infrastructure only): it computes the whole
grid and writes only the rank's nodes, so what these tests pin is the driver — the shard
ranges, the Jacobi buffer handling, the value all-gather after every Howard sweep, the
all-reduce of the stop criterion and the final k_opt gather — against the unsharded C solve."""
import json
import math
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _pkg():
    sys.path.insert(0, str(ROOT))
    from tests.conftest import load_pkg
    return load_pkg()


class OracleShard:
    """Shard backend on the C restatement (tensors (4, K, k) on CPU)."""

    def __init__(self, p, kg, Kg, B, P, K0, K1, s0=0, s1=4):
        self.p, self.kg, self.Kg, self.B, self.P, self.K0, self.K1 = p, kg, Kg, B, P, K0, K1
        self.s0, self.s1 = s0, s1

    @staticmethod
    def _np(V):
        return np.asfortranarray(V.numpy().transpose(2, 1, 0))

    def improve(self, V, kopt):
        from oracle import corc
        import torch
        ko, _ = corc.ks_policy_improve(self.p, self.kg, self.Kg, self._np(V), self.B, self.P)
        kt = torch.from_numpy(np.ascontiguousarray(ko.transpose(2, 1, 0)))
        kopt[self.s0:self.s1, self.K0:self.K1, :] = kt[self.s0:self.s1, self.K0:self.K1, :]

    def howard(self, V, kopt, Vout):
        from oracle import corc
        import torch
        Vn = corc.ks_howard(self.p, self.kg, self.Kg, self._np(V), self._np(kopt), self.B,
                            self.P, 1)
        vt = torch.from_numpy(np.ascontiguousarray(Vn.transpose(2, 1, 0)))
        Vout[self.s0:self.s1, self.K0:self.K1, :] = vt[self.s0:self.s1, self.K0:self.K1, :]

    def slopes(self, V, dV):
        pass  # the restatement rebuilds the slopes inside every sweep

    def howard_fused(self, V, dV, kopt, Vout, dVout):
        self.howard(V, kopt, Vout)

    def ghost(self, K0, K1, s0, s1):
        g = OracleShard(self.p, self.kg, self.Kg, self.B, self.P, K0, K1, s0, s1)
        g.kp_idx = self.kp_idx
        return g

    def hints(self, kopt):
        pass

    def close(self):
        pass

    def reldiff(self, V, Vold):
        a = V[self.s0:self.s1, self.K0:self.K1, :].numpy()
        b = Vold[self.s0:self.s1, self.K0:self.K1, :].numpy()
        d = np.abs(a - b) / (np.abs(b) + 1e-10)
        return float(np.nanmax(d)) if not np.all(np.isnan(d)) else math.nan


# ALM whose forecast index moves by one to three K points: up below K* = 42.5 and down above it
# in one aggregate state, down everywhere in the other, so shards read their neighbours' columns
B_MIXED = np.array([0.6, 0.84, 0.1, 0.95])


def _setup(nK=4, B_alm=None):
    from oracle import corc
    from oracle import np_oracle as no
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=40, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975]) if B_alm is None else np.asarray(B_alm)
    cp = corc.ks_params(**{k: p[k] for k in ("beta", "alpha", "delta", "k_min", "k_max", "ug",
                                              "ub", "l_bar", "mu", "z_grid", "eps_grid")})
    return cp, kg, Kg, P, V0, B


def _worker(rank, world, port, outdir, nK, exchange="halo", depth=1, howard=3, B_alm=None,
            balanced=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from oracle import corc
    corc.num_threads(1)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kd = _pkg().ks_dist
    cp, kg, Kg, P, V0, B = _setup(nK, B_alm)
    kp = kd.forecast_index(Kg, B, _pkg().ks_params())  # host-only C ABI call
    bounds = kd.balanced_bounds(kp, len(Kg), world, depth) if balanced else None
    K0, K1, s0, s1 = kd.shard_slices(len(Kg), rank, world, bounds)
    V = torch.from_numpy(np.ascontiguousarray(V0.transpose(2, 1, 0)))
    ko = torch.ones_like(V)
    sh = OracleShard(cp, kg, Kg, B, P, K0, K1, s0, s1)
    sh.kp_idx = kp
    if depth > 1 or B_alm is not None:  # the test's geometry must need remote columns
        assert any(c for row in kd.halo_plan(sh.kp_idx, len(Kg), world, bounds) for c in row)
    it, rel = kd.ks_vfi_solve_dist(V, ko, sh, len(Kg), howard_steps=howard, tol=1e-6,
                                   max_vfi=6, rank=rank, world=world, exchange=exchange,
                                   poison=(exchange == "halo"), depth=depth, bounds=bounds)
    np.save(Path(outdir, f"V{rank}.npy"), V.numpy())
    np.save(Path(outdir, f"k{rank}.npy"), ko.numpy())
    Path(outdir, f"m{rank}.json").write_text(json.dumps(dict(it=it, rel=rel)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nK,exchange", [(2, 4, "halo"), (3, 5, "halo"), (3, 8, "halo"),
                                               (2, 4, "allgather"), (4, 2, "halo"),
                                               (3, 2, "allgather")])
def test_gloo_sharded_equals_unsharded(tmp_path, world, nK, exchange):
    """Halo runs poison every column a rank neither owns nor reads with NaN: equality with the
    unsharded solve then proves the halo plan covers every read."""
    import torch.multiprocessing as mp
    from oracle import corc
    port = 29600 + (os.getpid() % 1500) + 7 * world + 3 * nK + (exchange == "halo")
    mp.spawn(_worker, args=(world, port, str(tmp_path), nK, exchange), nprocs=world, join=True)
    cp, kg, Kg, P, V0, B = _setup(nK)
    R = corc.ks_vfi_solve(cp, kg, Kg, V0, np.ones_like(V0), B, P, howard=3, tol=1e-6, max_vfi=6)
    Vr = np.ascontiguousarray(R["value"].transpose(2, 1, 0))
    kr = np.ascontiguousarray(R["k_opt"].transpose(2, 1, 0))
    for rank in range(world):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        m = json.loads(Path(tmp_path, f"m{rank}.json").read_text())
        assert m["it"] == R["iters"]


@pytest.mark.parametrize("world,nK,depth,howard,balanced", [
    (2, 8, 1, 3, False), (3, 12, 1, 3, False), (2, 8, 2, 3, False), (3, 12, 3, 7, False),
    (4, 12, 4, 5, False), (5, 12, 2, 5, False), (2, 6, 6, 4, False), (8, 6, 3, 4, False),
    (4, 16, 4, 5, True), (3, 12, 2, 5, True)])
def test_gloo_ghost_sweeps_equal_unsharded(tmp_path, world, nK, depth, howard, balanced):
    """Communication-avoiding Howard (HowardSweeps depth > 1: one exchange per block of `depth`
    sweeps, ghost rectangles swept redundantly) — bit-identical to the unsharded solve, with
    every value column outside own ∪ R_depth and every k_opt column outside own ∪ R_{depth-1}
    NaN-poisoned.  Blocks that do not divide the sweep count (7 = 3 + 3 + 1) and depth larger
    than the sweep count are included; (8, 6) uses (K, Z) slices; depth 1 is the per-sweep halo on
    the same geometry; `balanced` cuts the K range at `balanced_bounds` instead of evenly."""
    import torch.multiprocessing as mp
    from oracle import corc
    port = 31200 + (os.getpid() % 1500) + 11 * world + 3 * nK + depth + 5 * balanced
    mp.spawn(_worker, args=(world, port, str(tmp_path), nK, "halo", depth, howard, B_MIXED,
                            balanced), nprocs=world, join=True)
    cp, kg, Kg, P, V0, B = _setup(nK, B_MIXED)
    R = corc.ks_vfi_solve(cp, kg, Kg, V0, np.ones_like(V0), B, P, howard=howard, tol=1e-6,
                          max_vfi=6)
    Vr = np.ascontiguousarray(R["value"].transpose(2, 1, 0))
    kr = np.ascontiguousarray(R["k_opt"].transpose(2, 1, 0))
    for rank in range(world):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        assert json.loads(Path(tmp_path, f"m{rank}.json").read_text())["it"] == R["iters"]


def test_balanced_bounds_scaling_grid():
    """balanced_bounds (exact DP over split points) at the scaling grid's forecast map: a
    partition of [0, 64) into 8 non-empty ranges whose largest ghost cost is no larger than the
    even split's — and no other contiguous split does better (checked against every split
    that moves one boundary by one)."""
    kd = _pkg().ks_dist
    from oracle import np_oracle as no
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=8, K_size=64)
    kp = kd.forecast_index(Kg, np.array([0.1, 0.97, 0.08, 0.975]), _pkg().ks_params())
    for depth in (2, 4):
        b = kd.balanced_bounds(kp, 64, 8, depth)
        assert b[0] == 0 and b[-1] == 64 and all(x < y for x, y in zip(b, b[1:]))
        cost = lambda bb: max(kd.ghost_cost(kp, 64, bb[r], bb[r + 1], depth) for r in range(8))
        even = [64 * r // 8 for r in range(9)]
        assert cost(b) <= cost(even)
        for r in range(1, 8):
            for d in (-1, 1):
                bb = list(b)
                bb[r] += d
                if bb[r - 1] < bb[r] < bb[r + 1]:
                    assert cost(b) <= cost(bb)
    assert kd.shard_slices(64, 3, 8, b) == (b[3], b[4], 0, 4)


def test_ghost_rects_cover_reads():
    """R_j holds R_{j-1} and every column R_{j-1}'s nodes read (the closure the schedule
    needs), at the scaling grid's forecast map over 8 ranks."""
    kd = _pkg().ks_dist
    from oracle import np_oracle as no
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=8, K_size=64)
    kp = kd.forecast_index(Kg, np.array([0.1, 0.97, 0.08, 0.975]), _pkg().ks_params())
    for rank in range(8):
        R = kd.ghost_rects(kp, 64, *kd.shard_slices(64, rank, 8), 6)
        for j in range(1, 7):
            prev, cur = set(kd.rect_columns(R[j - 1], 64)), set(kd.rect_columns(R[j], 64))
            reads = {sn * 64 + int(kp[c // 64, c % 64]) for c in prev for sn in range(4)}
            assert prev <= cur and reads <= cur


def test_shard_ranges_cover():
    kd = _pkg().ks_dist
    for nK in (1, 4, 7, 64):
        for world in (1, 2, 3, 8):
            if world > nK:
                continue
            rs = [kd.shard_range(nK, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == nK
            assert all(rs[i][1] == rs[i + 1][0] and rs[i][0] < rs[i][1] for i in range(world - 1))


@pytest.mark.parametrize("nK", [1, 2, 3, 4, 5, 64])
def test_kz_slices_partition_every_node(nK):
    """(K, Z) slices: up to 2·nK ranks, every (s, K) column owned by exactly one rank, every
    shard non-empty; the reference's K = 4 grid spreads over 8 ranks as one (K, z) each."""
    kd = _pkg().ks_dist
    for world in range(1, 2 * nK + 1):
        seen = []
        for r in range(world):
            K0, K1, s0, s1 = kd.shard_slices(nK, r, world)
            assert 0 <= K0 < K1 <= nK and (s0, s1) in ((0, 4), (0, 2), (2, 4))
            seen += kd.owned_columns(nK, r, world)
        assert sorted(seen) == list(range(4 * nK))
    with pytest.raises(ValueError):
        kd.shard_slices(nK, 0, 2 * nK + 1)
    if nK == 4:
        assert [kd.shard_slices(4, r, 8) for r in range(8)] == \
            [(K, K + 1, 0, 2) for K in range(4)] + [(K, K + 1, 2, 4) for K in range(4)]


def test_forecast_index_and_halo_plan():
    """ks_forecast_index (host-only) is the clamp + nearest-index rule of bellman_value
    (Krusell_Smith_VFI.m:335-343); halo_plan lists exactly the foreign columns a rank reads."""
    kd = _pkg().ks_dist
    prm = _pkg().ks_params()
    Kg = np.linspace(30.0, 50.0, 64)
    for B in ([0.1, 0.97, 0.08, 0.975], [0.0, 1.0, 0.0, 1.0], [0.5, 0.8, -0.3, 1.1]):
        B = np.array(B)
        kp = kd.forecast_index(Kg, B, prm)
        z1, z2 = prm[9], prm[10]
        for s in range(4):
            z = z2 if s + 1 <= 2 else z1            # flipped current_z (:332)
            b0, b1 = (B[0], B[1]) if z == z1 else (B[2], B[3])
            Kp = np.clip(np.exp(b0 + b1 * np.log(Kg)), Kg[0], Kg[-1])
            want = np.argmin(np.abs(Kg[None, :] - Kp[:, None]), axis=1)
            assert np.array_equal(kp[s], want)
        for nK, world in ((64, 2), (64, 3), (64, 8), (4, 8), (4, 6)):
            kpn = kd.forecast_index(np.linspace(30.0, 50.0, nK), B, prm) if nK != 64 else kp
            plan = kd.halo_plan(kpn, nK, world)
            for q in range(world):
                K0, K1, s0, s1 = kd.shard_slices(nK, q, world)
                mine = set(kd.owned_columns(nK, q, world))
                targets = np.unique(kpn[s0:s1, K0:K1]).tolist()
                need = {sn * nK + t for t in targets for sn in range(4)} - mine
                got = [c for p in range(world) for c in plan[q][p]]
                assert sorted(got) == sorted(need) and not plan[q][q]
                for p in range(world):
                    assert set(plan[q][p]) <= set(kd.owned_columns(nK, p, world))
    # identity ALM: every node forecasts its own K, so no halo at all
    kp = kd.forecast_index(Kg, np.array([0.0, 1.0, 0.0, 1.0]), prm)
    assert np.array_equal(kp, np.tile(np.arange(64), (4, 1)))
    assert all(not c for row in kd.halo_plan(kp, 64, 8) for c in row)


def test_calibration_matches_oracle_setup():
    """The package's KS calibration (used by the benches) equals the oracle's restatement."""
    from oracle import np_oracle as no
    cal = _pkg().calibration
    for k, K in ((100, 4), (1000, 64)):
        p, kg, Kg, P, V0, B = no.ks_setup(k_size=k, K_size=K)
        kg2, Kg2, P2, V02 = cal.krusell_smith(k_size=k, K_size=K)
        for a, b in ((kg, kg2), (Kg, Kg2), (P, P2), (V0, V02)):
            assert np.array_equal(a, b)


def _agree_worker(rank, world, port, outdir, failing):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kd = _pkg().ks_dist
    cleaned = []
    msg = "boom" if rank in failing else None
    try:
        kd._agree_or_raise(msg, "cpu", "probe", lambda: cleaned.append(1))
        res = "ok"
    except RuntimeError as e:
        res = str(e)
    dist.barrier()   # every rank is out of the collective: nobody was left inside it
    Path(outdir, f"a{rank}.json").write_text(json.dumps(dict(res=res, cleaned=len(cleaned))))
    dist.destroy_process_group()


@pytest.mark.parametrize("failing", [(), (1,), (0, 2)])
def test_direct_failures_are_agreed(tmp_path, failing):
    """DirectPeers raises setup failures and wait timeouts on EVERY rank together
    (ks_dist._agree_or_raise: one all-reduce), after its cleanup, so a failure on one rank never
    leaves the others inside a collective — gloo, 3 ranks."""
    import torch.multiprocessing as mp
    port = 32100 + (os.getpid() % 1000) + 7 * len(failing)
    mp.spawn(_agree_worker, args=(3, port, str(tmp_path), failing), nprocs=3, join=True)
    for rank in range(3):
        d = json.loads(Path(tmp_path, f"a{rank}.json").read_text())
        if failing:
            assert d["res"].startswith("probe: ") and d["cleaned"] == 1
            assert ("boom" in d["res"]) == (rank in failing)
        else:
            assert d["res"] == "ok" and d["cleaned"] == 0


def test_direct_peers_bound_to_their_shard():
    """a DirectPeers carries the neighbour mask and column tables of the shard (the
    forecast index of one ALM B) it was built for; handing it to a solve of another shard
    raises before any wait or launch."""
    kd = _pkg().ks_dist

    class _Shard:  # stand-ins: only identity matters to the check
        pass

    class _Peers:
        def __init__(self, shard):
            self.shard = shard

    a, b = _Shard(), _Shard()
    with pytest.raises(ValueError, match="another shard"):
        kd._solve_direct(None, None, b, 4, 3, 1e-6, 1, 0, 2, None, peers=_Peers(a))


def test_staged_plan_matches_the_forecast_reads():
    """ks_dist.staged_plan (the staged direct schedule's halo and interior/boundary split)
    against a brute-force walk over every node of every rank: the halo is exactly the peer-owned
    columns some own node's forecast reads, interior columns read only own columns, and every
    own column is in exactly one list — for K-range and (K, Z) slices, identity and shifted ALMs."""
    kd = _pkg().ks_dist
    rng = np.random.default_rng(7)
    for nK, world in ((4, 8), (6, 2), (12, 3), (64, 8), (16, 5)):
        for shift in (0, -1, 1, "rand"):
            if shift == "rand":
                kp = rng.integers(0, nK, size=(4, nK))
            else:
                kp = np.clip(np.arange(nK)[None, :] + shift, 0, nK - 1).repeat(4, axis=0)
            owner = [0] * (4 * nK)
            for q in range(world):
                for c in kd.owned_columns(nK, q, world):
                    owner[c] = q
            for rank in range(world):
                own = kd.owned_columns(nK, rank, world)
                remote, interior, boundary = kd.staged_plan(own, kp, owner, nK, rank)
                reads = {c: {sn * nK + int(kp[c // nK, c % nK]) for sn in range(4)} for c in own}
                assert remote == sorted({t for c in own for t in reads[c] if owner[t] != rank})
                assert sorted(interior + boundary) == sorted(own)
                assert not set(interior) & set(boundary)
                for c in interior:
                    assert all(owner[t] == rank for t in reads[c])
                for c in boundary:
                    assert any(owner[t] != rank for t in reads[c])
