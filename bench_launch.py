"""`--gpus N` means N ranks (VERDICT r3 "do this" 2).

The driver launches `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
itself; a plain `python bench.py --gpus N` (no WORLD_SIZE in the environment) used to run one
process on GPU 0 and report n_gpus = 1.  `relaunch()` now starts N workers through
torch.distributed.run as a CHILD process (this parent never touches the GPU and never
exec()s), streams their output and exits with the child's status; `check_world()` makes every
worker refuse to run when WORLD_SIZE differs from --gpus.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(nproc: int, script: str, argv: list[str]) -> None:
    """If nproc > 1 and this process is not already a rank, run `script argv` as nproc ranks
    of torch.distributed.run (127.0.0.1 rendezvous) in a child process and exit with its
    return code.  Returns (does nothing) otherwise."""
    if nproc <= 1 or "WORLD_SIZE" in os.environ:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.call(cmd, env=env)
    sys.exit(rc)


def check_world(gpus: int) -> tuple[int, int, int]:
    """(world, rank, local_rank) from the environment; exits non-zero when world != gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        print(f"error: --gpus {gpus} but WORLD_SIZE = {world} (launch with --nproc-per-node "
              f"{gpus}, or without a launcher to let --gpus start the ranks)", file=sys.stderr,
              flush=True)
        sys.exit(2)
    return world, rank, local
