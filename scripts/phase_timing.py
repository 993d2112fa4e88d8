"""Rollout vs update split of a PPO iteration on the bench workload (development tool): GPU time between
events and the host's enqueue time of each phase.  A phase whose host time reaches its GPU time is
host(launch)-bound.  usage: python scripts/phase_timing.py [iterations]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402
from lrl.ppo import runner as R  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n = 4096
cfg = lcfg.make_cfg()
lcfg.config_mini_cheetah(cfg)
cfg.env.num_envs = n
R.RunnerArgs.save_interval = 0
R.RunnerArgs.log_freq = 10 ** 9
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234))
runner = R.Runner(env, device="cuda:0", seed=1234)
runner.learn(2, init_at_random_ep_len=True)
alg = runner.alg
obs_dict = env.get_observations()
obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
torch.cuda.synchronize()
res = []
for it in range(iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t0 = time.perf_counter()
    ev[0].record()
    with torch.inference_mode():
        for _ in range(runner.num_steps_per_env):
            actions = alg.act(obs, priv, hist)
            obs_dict, rewards, dones, infos = env.step(actions)
            obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
            alg.process_env_step(rewards, dones, infos)
        alg.compute_returns(obs, priv)
    ev[1].record()
    t1 = time.perf_counter()
    alg.update()
    ev[2].record()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    res.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t0) * 1e3))
for r in res:
    print(f"rollout gpu {r[0]:7.2f} ms (host {r[2]:6.2f})   update gpu {r[1]:7.2f} ms (host {r[3]:6.2f})   wall {r[4]:7.2f}")
