"""CPU: config 4's multisection GE driver (ge_batch.py) — the host logic and the collective.
The candidate evaluator is the C restatement (oracle/ — test infrastructure only), so these
tests exercise the tree construction, the path walk and the gloo all-gather, and pin the
multisection trace to the sequential bisection over the same evaluator, bit for bit."""
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


def _oracle_evaluator(Na=60):
    from oracle import corc
    from oracle import np_oracle as no
    gb = _pkg().ge_batch
    cal = no.calib_aiyagari(Na=Na)
    w0 = no.wage(0.04, 0.36, 0.08)
    v0 = corc.vfi_solve(np.zeros((7, Na)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0, 0.96,
                        5.0)["v_old"]

    def solve(v, r, w):
        return corc.vfi_solve(v, cal["a_grid"], cal["s"], cal["P"], r, w, 0.96, 5.0)

    def simulate(pk, z1, k1, u):
        return corc.sim_capital(pk, cal["a_grid"], cal["P"], z1 - 1, k1, u)
    return gb.vfi_evaluator(cal, solve, simulate, v0, T=2000), cal


def test_subtree_midpoints_are_the_sequential_ones():
    gb = _pkg().ge_batch
    lo, hi = -0.05, 1 / 0.96 - 1
    nodes = gb.subtree(lo, hi, 1, 4)
    assert len(nodes) == 15 and nodes[0].r == (lo + hi) / 2
    # every path of the sequential loop visits only subtree nodes, with identical values
    for target in np.linspace(lo, hi, 37):
        a, b = lo, hi
        keys = {(n.lo, n.hi): n.r for n in nodes}
        for _ in range(4):
            m = (a + b) / 2
            assert keys[(a, b)] == m
            a, b = (a, m) if m > target else (m, b)


@pytest.mark.parametrize("levels", [1, 3, 6])
def test_multisection_equals_bisection_synthetic(levels):
    """A synthetic excess demand (monotone, with an exact hit for the early stop)."""
    gb = _pkg().ge_batch
    root = 0.0123

    def ev(n):
        return (n.r - root + 100.0, 100.0, 1)
    A = gb.multisection(ev, -0.05, 0.04, max_steps=10, levels=levels)
    S = gb.bisection(ev, -0.05, 0.04, max_steps=10)
    assert A.r_history == S.r_history and A.k_supply == S.k_supply and A.r == S.r
    assert A.rounds == math.ceil(10 / levels)


def test_multisection_equals_bisection_oracle_single_rank():
    gb = _pkg().ge_batch
    ev, cal = _oracle_evaluator()
    lo, hi = -0.05, 1 / cal["beta"] - 1
    A = gb.multisection(ev, lo, hi, levels=6)
    S = gb.bisection(ev, lo, hi)
    assert A.r_history == S.r_history and A.k_supply == S.k_supply and A.iters == S.iters
    assert A.candidates == 63 + 15 and A.rounds == 2


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from oracle import corc
    corc.num_threads(1)  # two ranks share the container's cores
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gb = _pkg().ge_batch
    ev, cal = _oracle_evaluator()
    lo, hi = -0.05, 1 / cal["beta"] - 1
    A = gb.multisection(ev, lo, hi, levels=6, rank=rank, world=world,
                        allgather=gb.torch_allgather)
    Path(outdir, f"r{rank}.json").write_text(json.dumps(dict(r=A.r_history, ks=A.k_supply,
                                                               it=A.iters, final=A.r)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_equal_sequential(tmp_path, world):
    """The tensor all-gather (all_gather_into_tensor of [ceil(63/world), 4] float64 rows; 3
    ranks leave padding rows) reproduces the sequential trace on every rank."""
    import torch.multiprocessing as mp
    port = 29500 + (os.getpid() % 2000) + 7 * world
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    gb = _pkg().ge_batch
    ev, cal = _oracle_evaluator()
    S = gb.bisection(ev, -0.05, 1 / cal["beta"] - 1)
    for rank in range(world):
        R = json.loads(Path(tmp_path, f"r{rank}.json").read_text())
        assert R["r"] == S.r_history and R["ks"] == S.k_supply and R["it"] == S.iters
        assert R["final"] == S.r
