"""Quick env-only timing (development helper)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rapid-locomotion-rl_amd"))
import torch
from lrl import config as lcfg
from lrl.env import LeggedRobotEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cfg = lcfg.make_cfg(); lcfg.config_mini_cheetah(cfg)
env = LeggedRobotEnv("cuda:0", cfg=cfg, num_envs=n)
env.reset()
a = torch.zeros(n, 12, device="cuda:0")
for _ in range(20): env.step(a, _history=True)
torch.cuda.synchronize(); t = time.time(); K = 200
for _ in range(K): env.step(a, _history=True)
torch.cuda.synchronize(); dt = (time.time() - t) / K
print(f"n={n} env step {dt*1e6:.1f} us  -> {n/dt/1e6:.2f} M env-steps/s; z mean {env.root_states[:,2].mean().item():.3f} resets {env._reset_u8.sum().item()}")
