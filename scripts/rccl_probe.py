"""Does RCCL run two ranks on one GPU here?  Each rank all-reduces a vector over the "nccl" (RCCL) backend and
checks the sum.  usage: python scripts/rccl_probe.py  (spawns 2 ranks on cuda:0)"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    x = torch.full((1 << 20,), float(rank + 1), device="cuda:0")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    ok = bool((x == sum(range(1, world + 1))).all().item())
    print(f"rank {rank}: all_reduce ok={ok} backend={dist.get_backend()} nccl_version={torch.cuda.nccl.version()}",
          flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(2, port), nprocs=2, join=True)
    sys.exit(0)
