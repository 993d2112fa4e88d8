"""Data-parallel PPO on CPU with the gloo backend, world_size 2 (the N>1 path of bench.py runs the same
code over RCCL): gradient averaging, KL/LR agreement and the global advantage statistics keep every
rank's parameters identical although each rank holds different rollouts."""
import os
import socket
import zlib

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init_params(module):
    with torch.no_grad():
        for name, p in module.named_parameters():
            r = np.random.default_rng(zlib.crc32(name.encode()))
            fan_in = p.shape[-1] if p.dim() > 1 else 1
            if name == "std":
                p.fill_(1.0)
            else:
                p.copy_(torch.tensor(r.uniform(-1, 1, tuple(p.shape)) / np.sqrt(fan_in), dtype=torch.float))


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "rapid-locomotion-rl_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO, PPO_Args
    from oracle import oracle
    ac = ActorCritic(42, 18, 630, 12)
    _init_params(ac)
    alg = PPO(ac, device="cpu", fused=False)
    T, N = 8, 32
    alg.init_storage(N, T, [42], [18], [630], [12])
    st = alg.storage
    g = torch.Generator().manual_seed(7 + rank)  # different data per rank
    with torch.inference_mode():
        for t in range(T):
            obs, priv, hist = (torch.randn(N, 42, generator=g), torch.randn(N, 18, generator=g),
                               torch.randn(N, 630, generator=g))
            alg.act(obs, priv, hist)
            alg.process_env_step(torch.randn(N, generator=g), torch.zeros(N, dtype=torch.bool),
                                 {"env_bins": torch.zeros(N)})
        last = ac.evaluate(torch.randn(N, 42, generator=g), torch.randn(N, 18, generator=g))
    # GAE on the oracle with GLOBAL advantage statistics (what lrl_gae_partial + all-reduce does)
    ret, _ = oracle.gae(st.rewards.numpy(), st.dones.numpy(), st.values.numpy(), last.numpy(), PPO_Args.gamma,
                        PPO_Args.lam)
    adv = ret - st.values.numpy()
    stats = torch.tensor([adv.sum(), (adv.astype(np.float64) ** 2).sum(), adv.size], dtype=torch.float64)
    dist.all_reduce(stats)
    mean = stats[0] / stats[2]
    std = torch.sqrt((stats[1] - stats[2] * mean * mean) / (stats[2] - 1))
    st.returns.copy_(torch.tensor(ret))
    st.advantages.copy_(((torch.tensor(adv, dtype=torch.float64) - mean) / (std + 1e-8)).float())
    # grad averaging primitive
    p0 = next(ac.parameters())
    p0.grad = torch.full_like(p0, float(rank + 1))
    alg._allreduce_grads([p0])
    avg_ok = bool(torch.all(p0.grad == 1.5))
    p0.grad = None
    mv, ms, ma = alg.update()
    flat = torch.cat([p.detach().reshape(-1) for p in ac.parameters()])
    out[rank] = (avg_ok, flat.numpy().copy(), alg.learning_rate, [mv, ms, ma])
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_update_keeps_replicas_identical():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
    a, b = out[0], out[1]
    assert a[0] and b[0], "gradient all-reduce did not average"
    np.testing.assert_array_equal(a[1], b[1])  # identical replicas after 20 optimiser steps
    assert a[2] == b[2]                         # same adaptive learning rate on both ranks


def _curriculum_rows_worker(rank, world, port, out):
    import sys
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "rapid-locomotion-rl_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lrl.env import LeggedRobotEnv
    from lrl.curriculum import RewardThresholdCurriculum
    stub = types.SimpleNamespace(_dist=dist, device="cpu")
    counts = [3, 0, 5]  # a rank with no resampled envs still joins
    k = counts[rank]
    rows = np.stack([np.arange(k) + 10 * rank, np.full(k, 0.5 + rank), np.full(k, -1.0 - rank)], 1).astype(np.float64)
    got, off = LeggedRobotEnv._dist_gather_rows(stub, rows)
    total = LeggedRobotEnv._dist_count(stub, k)
    # every rank then runs the same curriculum update / draw over the gathered rows and keeps its slice
    cur = RewardThresholdCurriculum(seed=100, x_vel=(-1, 1, 5), y_vel=(-0.6, 0.6, 2), yaw_vel=(-1, 1, 5))
    cur.weights[:] = 1.0
    cmds, bins = cur.sample(batch_size=len(got))
    out[rank] = (got, off, total, cmds[off:off + k], bins[off:off + k])
    dist.destroy_process_group()


def test_curriculum_rows_gathered_in_rank_order():
    """LeggedRobotEnv._dist_gather_rows / _dist_count (the multi-rank command curriculum) over
    gloo with 3 ranks of 3 / 0 / 5 rows: every rank sees all rows in rank order and its own offset, so slicing
    one shared draw gives each rank the rows a single process would have drawn for its envs."""
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_curriculum_rows_worker, args=(world, _port(), out), nprocs=world, join=True)
    want = np.concatenate([np.stack([np.arange(k) + 10 * r, np.full(k, 0.5 + r), np.full(k, -1.0 - r)], 1)
                           for r, k in enumerate([3, 0, 5])])
    offs = [0, 3, 3]
    for r in range(world):
        got, off, total, cmds, bins = out[r]
        np.testing.assert_array_equal(got, want)
        assert off == offs[r] and total == 8
    allc = np.concatenate([out[r][3] for r in range(world)])
    from lrl.curriculum import RewardThresholdCurriculum
    cur = RewardThresholdCurriculum(seed=100, x_vel=(-1, 1, 5), y_vel=(-0.6, 0.6, 2), yaw_vel=(-1, 1, 5))
    cur.weights[:] = 1.0
    ref, _ = cur.sample(batch_size=8)
    np.testing.assert_array_equal(allc, ref)
