"""Probe (GPU box, one card): can two RCCL ranks share one GPU (torch "nccl" backend), and can a
point-to-point exchange be captured in a HIP graph?  Decides how the KS multi-rank RCCL path can
be tested on this pool's 1-GPU boxes.  Prints one line per check; never retries."""
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
    peer = 1 - rank
    x = torch.full((1024,), float(rank), device="cuda")
    y = torch.empty_like(x)
    t0 = time.time()
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, x, peer), dist.P2POp(dist.irecv, y, peer)])
    for r in reqs:
        r.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: eager p2p ok={bool((y == peer).all())} {time.time() - t0:.3f}s", flush=True)
    pg = dist.distributed_c10d._get_default_group()
    try:
        be = pg._get_backend(torch.device("cuda"))
        print(f"rank {rank}: comm_ptr={be._comm_ptr():#x}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: comm_ptr unavailable: {e}", flush=True)
    # graph capture of 10 exchanges
    try:
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        x2 = torch.full((1 << 16,), float(rank), device="cuda")
        y2 = torch.zeros_like(x2)
        torch.cuda.synchronize()
        dist.barrier()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                x2.add_(1.0)
                rq = dist.batch_isend_irecv([dist.P2POp(dist.isend, x2, peer),
                                             dist.P2POp(dist.irecv, y2, peer)])
                for r in rq:
                    r.wait()
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        want = float(peer) + 20.0
        print(f"rank {rank}: graph p2p ok={bool((y2 == want).all())} y={float(y2[0])} want={want}",
              flush=True)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        print(f"rank {rank}: graph replay 10x10 exchanges {(time.time() - t0) * 1e6 / 100:.1f} us each",
              flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: graph capture failed: {type(e).__name__}: {e}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    port = 29500 + os.getpid() % 1000
    mp.spawn(worker, args=(2, port), nprocs=2, join=True)
    print("probe done", flush=True)
    sys.exit(0)
