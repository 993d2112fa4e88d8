"""Rank start-up for the multi-process GPU rehearsals (gloo ranks sharing the one GPU of the test box).

VERDICT r4: the 8-rank rehearsal aborted with HSA_STATUS_ERROR_ILLEGAL_INSTRUCTION in the first PyTorch kernel of
one rank (a 4096-float fill), before any liblrl kernel of that rank had run, with 8 rank contexts plus the pytest
parent's on one device.  What the tests do about it ("multi-process rehearsals on one GPU"):
  * every rank names itself (rank, world, pid) on stderr first, so a record of a dead rank says which one it was;
  * the ranks bring their GPU context up one after another (context creation, the first PyTorch kernel and the
    liblrl code object load, finished with a device synchronise) under a token passed by gloo barriers, so no two
    processes load code objects onto the device at the same time;
  * ``spawn_env`` caps the hardware queues each rank opens, so the ranks together do not oversubscribe the device's
    queue slots (8 ranks x HIP's default 4 queues = 32 user queues plus the parent's).
"""
import os
import sys

import torch
import torch.distributed as dist


def spawn_env(world):
    """Environment overrides for the spawned ranks (applied around ``mp.spawn``; the children inherit them)."""
    if world <= 2:
        return {}
    return {"GPU_MAX_HW_QUEUES": "1"}


class rank_env:
    """Context manager: set ``spawn_env(world)`` in os.environ for the duration of an ``mp.spawn``."""

    def __init__(self, world):
        self.over = spawn_env(world)
        self.saved = {}

    def __enter__(self):
        for k, v in self.over.items():
            self.saved[k] = os.environ.get(k)
            os.environ[k] = v
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return False


def _first_liblrl_kernel():
    import ctypes as C
    from lrl import _abi
    a = torch.ones(32, 32, device="cuda:0")
    c = torch.empty(32, 32, device="cuda:0")
    p = lambda t: C.c_void_p(t.data_ptr())
    _abi.check(_abi.lib().lrl_gemm_f32(C.c_int32(0), C.c_int32(0), C.c_int32(32), C.c_int32(32), C.c_int32(32),
                                       p(a), C.c_int64(32), p(a), C.c_int64(32), p(c), C.c_int64(32), None, None,
                                       C.c_int64(0), None, None, C.c_int64(0),
                                       C.c_void_p(torch.cuda.current_stream().cuda_stream)))


def init_rank(rank, world, port, backend="gloo"):
    """Name the rank, join the process group, and bring the GPU context up in rank order."""
    print(f"[rank {rank}/{world}] pid {os.getpid()} GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', '-')}",
          file=sys.stderr, flush=True)
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group(backend, rank=rank, world_size=world)
    for r in range(world):
        if r == rank:
            torch.cuda.set_device(0)
            torch.ones(4096, device="cuda:0").neg_()  # first PyTorch kernels (code object load)
            _first_liblrl_kernel()  # liblrl code object
            torch.cuda.synchronize()
            print(f"[rank {rank}/{world}] pid {os.getpid()} GPU context up", file=sys.stderr, flush=True)
        if world > 1:
            dist.barrier()
