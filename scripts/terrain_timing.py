"""Timing of the rough-terrain path (BASELINE configs[2]) against the flat one, on cuda:0:
env-step kernel time (HIP events) for Go1 on the plane vs the curriculum trimesh, and full PPO iterations
on the trimesh with fork semantics vs the upstream reset path (legacy_fork=False)."""
import json
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

N = 4096


def cfg_go1(rough):
    cfg = lcfg.make_cfg()
    lcfg.config_go1(cfg)
    cfg.env.num_envs = N
    if rough:
        cfg.terrain.mesh_type = "trimesh"
        cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
        cfg.terrain.curriculum = True
    return cfg


def env_kernel_ms(rough, steps=60):
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg_go1(rough), seed=7))
    env.reset()
    a = torch.randn(N, 12, device="cuda:0") * 0.3
    for _ in range(20):
        env.step(a)
    env.env.kernel_timing(True)
    for _ in range(steps):
        env.step(a)
    torch.cuda.synchronize()
    ms = env.env.kernel_timing(False)[0]
    env.env.close()
    return ms


def ppo_iter_ms(legacy_fork, iters=3):
    R.RunnerArgs.save_interval = 0
    R.RunnerArgs.log_freq = 10 ** 9
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg_go1(True), seed=7, legacy_fork=legacy_fork))
    runner = R.Runner(env, device="cuda:0", seed=7)
    runner.learn(1, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.learn(iters)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters * 1e3
    env.env.close()
    return dt


out = {"go1_plane_env_kernel_ms": env_kernel_ms(False), "go1_trimesh_env_kernel_ms": env_kernel_ms(True),
       "go1_trimesh_ppo_iter_ms_fork": ppo_iter_ms(True), "go1_trimesh_ppo_iter_ms_upstream": ppo_iter_ms(False)}
print(json.dumps({k: round(v, 4) for k, v in out.items()}), flush=True)
