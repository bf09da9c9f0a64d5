"""GPU: the sharded Krusell-Smith VFI (ks_dist.py + ks_dev_* device tier) equals the
single-device solve (ks_vfi_solve) bit for bit — one rank, and two ranks sharing the card over
gloo (the RCCL path needs one GPU per rank; the exchange logic is the same)."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
B_ALM = np.array([0.1, 0.97, 0.08, 0.975])


def _pkg():
    sys.path.insert(0, str(ROOT))
    from tests.conftest import load_pkg
    return load_pkg()


# forecast index moving by one to three K points (tests/test_ks_dist_cpu.py B_MIXED): shards
# read their neighbours' columns and ghost rectangles grow with depth
B_MIXED = np.array([0.6, 0.84, 0.1, 0.95])


def _setup(nK, k_size=100):
    from oracle import np_oracle as no
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=k_size, K_size=nK)
    return kg, Kg, P, V0


def _run(rank, world, nK, steps=8, vfi=7, exchange="halo", depth=1, B_alm=B_ALM):
    import torch
    pkg = _pkg()
    kg, Kg, P, V0 = _setup(nK)
    prm = pkg.ks_params()
    K0, K1, s0, s1 = pkg.ks_dist.shard_slices(nK, rank, world)
    sh = pkg.ks_dist.HipShard(kg, Kg, B_alm, P, prm, K0, K1, s0, s1)
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device="cuda:0")
    ko = torch.ones_like(V)
    it, rel = pkg.ks_dist.ks_vfi_solve_dist(V, ko, sh, nK, howard_steps=steps, tol=1e-6,
                                            max_vfi=vfi, rank=rank, world=world,
                                            exchange=exchange, poison=(exchange == "halo"),
                                            depth=depth)
    torch.cuda.synchronize()
    sh.close()
    return V.cpu().numpy(), ko.cpu().numpy(), it, rel


def _reference(nK, steps=8, vfi=7, B_alm=B_ALM):
    pkg = _pkg()
    kg, Kg, P, V0 = _setup(nK)
    R = pkg.ks_vfi_solve(V0, np.ones_like(V0), kg, Kg, B_alm, P, pkg.ks_params(),
                         howard_steps=steps, tol=1e-6, max_vfi=vfi)
    return (np.ascontiguousarray(R["value"].transpose(2, 1, 0)),
            np.ascontiguousarray(R["k_opt"].transpose(2, 1, 0)), R["iters"], R["rel_diff"])


def test_one_rank_equals_single_device(pkg, gpu):
    V, ko, it, rel = _run(0, 1, 4)
    Vr, kr, itr, relr = _reference(4)
    assert it == itr and np.array_equal(V, Vr) and np.array_equal(ko, kr) and rel == relr


def _worker(rank, world, port, outdir, nK, exchange="halo", depth=1, B_alm=B_ALM):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if exchange == "timeout":
        _timeout_probe(rank, world, outdir, nK)
        dist.destroy_process_group()
        return
    if exchange == "bench":
        sys.path.insert(0, str(ROOT))
        import bench_ks
        leg = bench_ks.ks_direct_leg(_pkg(), world, rank, "cuda:0", nk=300, nK=nK, howard=7,
                                     reps=1, check_sweeps=5)
        Path(outdir, f"leg{rank}.json").write_text(json.dumps(leg))
        dist.destroy_process_group()
        return
    V, ko, it, rel = _run(rank, world, nK, exchange=exchange, depth=depth, B_alm=B_alm)
    np.save(Path(outdir, f"V{rank}.npy"), V)
    np.save(Path(outdir, f"k{rank}.npy"), ko)
    Path(outdir, f"m{rank}.json").write_text(json.dumps(dict(it=it, rel=rel)))
    dist.destroy_process_group()


@pytest.mark.parametrize("nK,exchange", [(4, "halo"), (6, "halo"), (6, "allgather")])
def test_two_ranks_gloo_equal_single_device(pkg, gpu, tmp_path, nK, exchange):
    """Halo runs NaN-poison every column a rank neither owns nor reads (ks_dist poison)."""
    import torch.multiprocessing as mp
    port = 29800 + (os.getpid() % 1000) + nK + 20 * (exchange == "halo")
    mp.spawn(_worker, args=(2, port, str(tmp_path), nK, exchange), nprocs=2, join=True)
    Vr, kr, itr, relr = _reference(nK)
    for rank in range(2):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        assert json.loads(Path(tmp_path, f"m{rank}.json").read_text())["it"] == itr


@pytest.mark.parametrize("world,nK,exchange", [(8, 4, "halo"), (6, 4, "allgather")])
def test_kz_slices_on_one_card(pkg, gpu, tmp_path, world, nK, exchange):
    """(K, Z) slices: the reference's K = 4 grid over 8 ranks (one (K, z) pair each) and over 6,
    HIP shards of the device tier (ks_dev_create_slice) sharing the card, gloo exchange."""
    import torch.multiprocessing as mp
    port = 29900 + (os.getpid() % 1000) + world + 10 * (exchange == "halo")
    mp.spawn(_worker, args=(world, port, str(tmp_path), nK, exchange), nprocs=world, join=True)
    Vr, kr, itr, relr = _reference(nK)
    for rank in range(world):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        assert json.loads(Path(tmp_path, f"m{rank}.json").read_text())["it"] == itr


@pytest.mark.parametrize("world,nK,depth", [(3, 12, 1), (3, 12, 3), (4, 12, 5), (6, 6, 4)])
def test_ghost_sweeps_on_one_card(pkg, gpu, tmp_path, world, nK, depth):
    """Communication-avoiding Howard sweeps (ks_dist.HowardSweeps, depth > 1): HIP ghost shards
    (ks_dev_share_hints / ks_dev_hints) sweep other ranks' columns redundantly between
    exchanges; every value column outside own ∪ R_depth and k_opt column outside
    own ∪ R_{depth-1} is NaN-poisoned; results equal the single-device solve bit for bit
    (8 sweeps per block schedule: 3 + 3 + 2, 5 + 3, 4 + 4; (6, 6) uses (K, Z) slices)."""
    import torch.multiprocessing as mp
    port = 30300 + (os.getpid() % 1000) + 13 * world + nK + depth
    mp.spawn(_worker, args=(world, port, str(tmp_path), nK, "halo", depth, B_MIXED),
             nprocs=world, join=True)
    Vr, kr, itr, relr = _reference(nK, B_alm=B_MIXED)
    for rank in range(world):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        assert json.loads(Path(tmp_path, f"m{rank}.json").read_text())["it"] == itr


def test_shared_hints_lifetime(pkg, gpu):
    """ks_dev_share_hints: the owner cannot be destroyed while a ghost shard shares its hint
    array (AIY_BAD_ARG), and can once the ghost is gone."""
    kd = pkg.ks_dist
    kg, Kg, P, V0 = _setup(6)
    sh = kd.HipShard(kg, Kg, B_MIXED, P, pkg.ks_params(), 2, 4, 0, 4)
    g = sh.ghost(0, 6, 0, 4)
    lib = pkg.lib()
    assert lib.ks_dev_destroy(sh._h) != 0          # refused: g still shares its hints
    assert b"share" in lib.aiy_last_error()
    g.close()
    assert lib.ks_dev_destroy(sh._h) == 0
    sh._h = None


@pytest.mark.parametrize("world,nK,B", [(2, 4, "alm"), (2, 6, "mixed"), (3, 12, "mixed"),
                                        (8, 4, "alm")])
def test_direct_ipc_ranks_on_one_card(pkg, gpu, tmp_path, world, nK, B):
    """The direct schedule under one process per rank (ks_dist.DirectPeers): each rank maps
    the others' parity buffers through IPC handles and reads its forecast columns there, the
    sweep hand-off runs through counters in a shared host page (aiy_flag_set /
    aiy_flags_wait, stream-ordered).  Ranks share the card (gloo for the host collectives);
    every non-own column of a rank's buffers is NaN, so a local read would show.  Equal to the
    single-device solve bit for bit — 2 and 3 K-range ranks, and the reference K = 4 grid on 8
    (K, Z) slices."""
    import torch.multiprocessing as mp
    Balm = B_ALM if B == "alm" else B_MIXED
    port = 31100 + (os.getpid() % 1000) + 7 * world + nK
    mp.spawn(_worker, args=(world, port, str(tmp_path), nK, "direct", 1, Balm), nprocs=world,
             join=True)
    Vr, kr, itr, relr = _reference(nK, B_alm=Balm)
    for rank in range(world):
        assert np.array_equal(np.load(Path(tmp_path, f"V{rank}.npy")), Vr)
        assert np.array_equal(np.load(Path(tmp_path, f"k{rank}.npy")), kr)
        assert json.loads(Path(tmp_path, f"m{rank}.json").read_text())["it"] == itr


def _timeout_probe(rank, world, outdir, nK):
    import torch
    pkg = _pkg()
    kg, Kg, P, V0 = _setup(nK)
    K0, K1, s0, s1 = pkg.ks_dist.shard_slices(nK, rank, world)
    sh = pkg.ks_dist.HipShard(kg, Kg, B_MIXED, P, pkg.ks_params(), K0, K1, s0, s1)
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device="cuda:0")
    dp = pkg.ks_dist.DirectPeers(sh, nK, rank, world, V, timeout_s=1.0)
    err = 0
    if rank == 0:            # waits for a sweep rank 1 never publishes
        dp.n = 3
        dp.wait()
        torch.cuda.synchronize()
        err = dp.error()
    dp.close()
    sh.close()
    Path(outdir, f"err{rank}.json").write_text(json.dumps(err))


def test_direct_ipc_wait_times_out(pkg, gpu, tmp_path):
    """A neighbour that never publishes: the waiting wave gives up after timeout_s, stores
    1 + the neighbour's rank in the rank's timeout word and releases the stream (no hang)."""
    import torch.multiprocessing as mp
    port = 31300 + (os.getpid() % 1000)
    mp.spawn(_worker, args=(2, port, str(tmp_path), 6, "timeout"), nprocs=2, join=True)
    assert json.loads(Path(tmp_path, "err0.json").read_text()) == 2
    assert json.loads(Path(tmp_path, "err1.json").read_text()) == 0


def test_bench_direct_leg_two_ranks(pkg, gpu, tmp_path):
    """bench_ks.ks_direct_leg (the N > 1 bench's `ks_direct` leg) on two ranks sharing the
    card: its built-in check (direct vs halo schedule, own columns bit for bit) holds."""
    import torch.multiprocessing as mp
    port = 31500 + (os.getpid() % 1000)
    mp.spawn(_worker, args=(2, port, str(tmp_path), 8, "bench"), nprocs=2, join=True)
    for rank in range(2):
        leg = json.loads(Path(tmp_path, f"leg{rank}.json").read_text())
        assert leg["bit_exact_vs_halo"] is True and leg["value"] > 0
