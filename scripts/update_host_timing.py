"""Is the update host-bound?  The bench's workload (4096 Mini Cheetah envs): per PPO update, the host time to issue
it (PPO.update with device-side losses, no sync) against the time until the GPU finishes it.
usage: python scripts/update_host_timing.py [iters]"""
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
cfg = lcfg.make_cfg()
lcfg.config_mini_cheetah(cfg)
cfg.env.num_envs = 4096
R.RunnerArgs.save_interval = 0
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234, legacy_fork=True))
runner = R.Runner(env, device="cuda:0", seed=1234)
runner.learn(2, init_at_random_ep_len=True)
alg = runner.alg
alg.async_losses = True
for it in range(iters):
    obs_dict = env.get_observations()
    obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
    with torch.inference_mode():
        for _ in range(24):
            a = alg.act(obs, priv, hist)
            obs_dict, rew, dones, infos = env.step(a)
            obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(obs, priv)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    alg.update()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"update {it}: host issue {1e3 * (t1 - t0):.2f} ms, GPU done after {1e3 * (t2 - t0):.2f} ms", flush=True)
