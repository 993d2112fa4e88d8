"""Host-side cost of the upstream reset path (legacy_fork=False): cProfile of 100 env steps of 4096 Go1 envs
on the curriculum trimesh (or Mini Cheetah on its flat map: argv `mc`; fork semantics: argv `fork`) with random
actions (frequent terminations), wall time per step."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402

N = 4096
fork = "fork" in sys.argv[1:]
cfg = lcfg.make_cfg()
if "mc" in sys.argv[1:]:
    lcfg.config_mini_cheetah(cfg)
else:
    lcfg.config_go1(cfg)
    cfg.terrain.mesh_type = "trimesh"
    cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
    cfg.terrain.curriculum = True
cfg.env.num_envs = N
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=7, legacy_fork=fork))
env.reset()
a = torch.randn(N, 12, device="cuda:0") * 0.5
for _ in range(20):
    env.step(a)
torch.cuda.synchronize()
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    env.step(a)
torch.cuda.synchronize()
pr.disable()
print(f"{'fork' if fork else 'upstream'}: {(time.perf_counter() - t0) * 10:.3f} ms/step "
      f"resets/step {env.env._reset_u8.float().mean().item():.3f}")
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
