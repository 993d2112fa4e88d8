"""Env step time with self-collision on (the presets' asset.self_collisions = 0) and off (= 1), Mini Cheetah and Go1,
4096 envs, random actions (development helper)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rapid-locomotion-rl_amd"))
import torch
from lrl import config as lcfg
from lrl.env import LeggedRobotEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for robot in ("mc", "go1"):
    for sc in (1, 0):
        cfg = lcfg.make_cfg()
        (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
        cfg.asset.self_collisions = sc
        env = LeggedRobotEnv("cuda:0", cfg=cfg, num_envs=n)
        env.reset()
        g = torch.Generator(device="cuda:0").manual_seed(0)
        acts = [torch.randn(n, 12, device="cuda:0", generator=g) * 0.5 for _ in range(8)]
        for i in range(30):
            env.step(acts[i % 8], _history=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 200
        e0.record()
        for i in range(K):
            env.step(acts[i % 8], _history=True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / K
        print(f"{robot} self_collisions={'on' if sc == 0 else 'off'}: env step {ms * 1e3:.1f} us "
              f"(z mean {env.root_states[:, 2].mean().item():.3f})", flush=True)
        env.close()
