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

    def __init__(self, p, kg, Kg, B, P, K0, K1):
        self.p, self.kg, self.Kg, self.B, self.P, self.K0, self.K1 = p, kg, Kg, B, P, K0, K1

    @staticmethod
    def _np(V):
        return np.asfortranarray(V.numpy().transpose(2, 1, 0))

    def improve(self, V, kopt):
        from oracle import corc
        import torch
        ko, _ = corc.ks_policy_improve(self.p, self.kg, self.Kg, self._np(V), self.B, self.P)
        kt = torch.from_numpy(np.ascontiguousarray(ko.transpose(2, 1, 0)))
        kopt[:, self.K0:self.K1, :] = kt[:, self.K0:self.K1, :]

    def howard(self, V, kopt, Vout):
        from oracle import corc
        import torch
        Vn = corc.ks_howard(self.p, self.kg, self.Kg, self._np(V), self._np(kopt), self.B,
                            self.P, 1)
        vt = torch.from_numpy(np.ascontiguousarray(Vn.transpose(2, 1, 0)))
        Vout[:, self.K0:self.K1, :] = vt[:, self.K0:self.K1, :]

    def reldiff(self, V, Vold):
        a, b = V[:, self.K0:self.K1, :].numpy(), Vold[:, self.K0:self.K1, :].numpy()
        d = np.abs(a - b) / (np.abs(b) + 1e-10)
        return float(np.nanmax(d)) if not np.all(np.isnan(d)) else math.nan


def _setup(nK=4):
    from oracle import corc
    from oracle import np_oracle as no
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=40, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])  # non-identity ALM: shards read remote columns
    cp = corc.ks_params(**{k: p[k] for k in ("beta", "alpha", "delta", "k_min", "k_max", "ug",
                                              "ub", "l_bar", "mu", "z_grid", "eps_grid")})
    return cp, kg, Kg, P, V0, B


def _worker(rank, world, port, outdir, nK):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from oracle import corc
    corc.num_threads(1)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kd = _pkg().ks_dist
    cp, kg, Kg, P, V0, B = _setup(nK)
    K0, K1 = kd.shard_range(len(Kg), rank, world)
    V = torch.from_numpy(np.ascontiguousarray(V0.transpose(2, 1, 0)))
    ko = torch.ones_like(V)
    it, rel = kd.ks_vfi_solve_dist(V, ko, OracleShard(cp, kg, Kg, B, P, K0, K1), len(Kg),
                                   howard_steps=3, tol=1e-6, max_vfi=6, rank=rank, world=world)
    np.save(Path(outdir, f"V{rank}.npy"), V.numpy())
    np.save(Path(outdir, f"k{rank}.npy"), ko.numpy())
    Path(outdir, f"m{rank}.json").write_text(json.dumps(dict(it=it, rel=rel)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nK", [(2, 4), (3, 5)])
def test_gloo_sharded_equals_unsharded(tmp_path, world, nK):
    import torch.multiprocessing as mp
    from oracle import corc
    port = 29600 + (os.getpid() % 1500) + 7 * world
    mp.spawn(_worker, args=(world, port, str(tmp_path), nK), nprocs=world, join=True)
    cp, kg, Kg, P, V0, B = _setup(nK)
    R = corc.ks_vfi_solve(cp, kg, Kg, V0, np.ones_like(V0), B, P, howard=3, tol=1e-6, max_vfi=6)
    Vr = np.ascontiguousarray(R["value"].transpose(2, 1, 0))
    kr = np.ascontiguousarray(R["k_opt"].transpose(2, 1, 0))
    for rank in range(world):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        m = json.loads(Path(tmp_path, f"m{rank}.json").read_text())
        assert m["it"] == R["iters"]


def test_shard_ranges_cover():
    kd = _pkg().ks_dist
    for nK in (1, 4, 7, 64):
        for world in (1, 2, 3, 8):
            if world > nK:
                continue
            rs = [kd.shard_range(nK, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == nK
            assert all(rs[i][1] == rs[i + 1][0] and rs[i][0] < rs[i][1] for i in range(world - 1))
