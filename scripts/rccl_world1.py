"""One native PPO update on cuda:0 inside a one-rank process group (tests/test_rccl_world1_gpu.py): with
LRL_FORCE_COLLECTIVES=1 the update issues every collective a multi-GPU run issues (the advantage statistics, the flat
policy gradient + KL slot per optimiser step, the adaptation gradient per substep) through the named backend, each
reducing over the one rank.  RCCL refuses two ranks on one GPU (scripts/rccl_probe.py), so this is how a one-GPU box
runs the `nccl` calls themselves on the update's own buffers and streams.
usage: MASTER_ADDR=127.0.0.1 MASTER_PORT=... python scripts/rccl_world1.py nccl|gloo|none out.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rapid-locomotion-rl_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    backend, out = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    elif backend == "gloo":
        dist.init_process_group("gloo", rank=0, world_size=1)
    calls = []
    orig = dist.all_reduce

    def counting(t, *a, **k):
        calls.append((t.numel(), t.is_cuda))
        return orig(t, *a, **k)
    dist.all_reduce = counting
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO
    from test_ppo_gpu import _random_storage, init_params
    ac = ActorCritic(42, 18, 630, 12)
    init_params(ac)
    alg = PPO(ac.cuda(), device="cuda:0", fused=True)
    N, T = 256, 24
    alg.init_storage(N, T, [42], [18], [630], [12])
    _random_storage(alg, N, T, seed=21)
    g = torch.Generator(device="cuda:0").manual_seed(22)
    with torch.no_grad():
        alg.storage.rewards.copy_(torch.randn(alg.storage.rewards.shape, device="cuda:0", generator=g))
        alg.storage.dones.zero_()
    alg.storage.step = T
    alg.compute_returns(torch.randn(N, 42, device="cuda:0", generator=g), torch.randn(N, 18, device="cuda:0", generator=g))
    torch.manual_seed(5)
    losses = alg.update()
    torch.cuda.synchronize()
    np.savez(out, flat=ac._flat.detach().cpu().numpy(), adv=alg.storage.advantages.detach().cpu().numpy(),
             losses=np.array([float(x) for x in losses]), sizes=np.array([c[0] for c in calls], np.int64),
             on_device=np.array([c[1] for c in calls], bool))
    if backend != "none":
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
