"""Where the Go1 rough-terrain iteration (bench.py `secondary`, BASELINE configs[2]) spends its time: wall time of
the rollout (24 env steps + acts + returns) and of the update, each bracketed by a device sync, and the GPU-busy
time of the rollout's env-step kernels (HIP events).  usage: python scripts/secondary_split.py [iters]"""
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

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = lcfg.make_cfg()
lcfg.config_go1(cfg)
cfg.env.num_envs = 4096
cfg.terrain.mesh_type = "trimesh"
cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
cfg.terrain.curriculum = True
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=4321, legacy_fork=False))
runner = R.Runner(env, device="cuda:0", seed=4321)
runner.learn(1, init_at_random_ep_len=True)
alg = runner.alg
print("obs", cfg.env.num_observations, "priv", cfg.env.num_privileged_obs, "fused", alg.fused)
obs_dict = env.get_observations()
obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
for it in range(iters):
    torch.cuda.synchronize()
    env.env.kernel_timing(True)
    t0 = time.perf_counter()
    t_act = t_step = t_proc = 0.0
    with torch.inference_mode():
        for _ in range(runner.num_steps_per_env):
            a0 = time.perf_counter()
            actions = alg.act(obs, priv, hist)
            a1 = time.perf_counter()
            obs_dict, rewards, dones, infos = env.step(actions)
            a2 = time.perf_counter()
            obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
            alg.process_env_step(rewards, dones, infos)
            a3 = time.perf_counter()
            t_act += a1 - a0
            t_step += a2 - a1
            t_proc += a3 - a2
        alg.compute_returns(obs, priv)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    k = env.env.kernel_timing(False)[1]
    alg.update()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"iter {it}: rollout {1e3 * (t1 - t0):.2f} ms (host: act {1e3 * t_act:.2f}, env.step {1e3 * t_step:.2f}, "
          f"process {1e3 * t_proc:.2f}; env kernels {k:.2f} ms GPU) update {1e3 * (t2 - t1):.2f} ms", flush=True)
env.env.close()
