"""A/B timing of whole PPO iterations (the bench's workload: 4096 Mini Cheetah envs, flat, fork semantics) for the
library LRL_LIB names: warm-up, then each iteration timed alone between device syncs; prints one JSON line with the
median / min iteration and the env-kernel mean (scripts/ab_build.sh makes the builds).
usage: LRL_LIB=ab/A/.../liblrl.so python scripts/ab_iter.py [iters] [tag]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402
from lrl.ppo import runner as R  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 12
tag = sys.argv[2] if len(sys.argv) > 2 else os.environ.get("LRL_LIB", "default")
cfg = lcfg.make_cfg()
lcfg.config_mini_cheetah(cfg)
if "LRL_SOLVER_TYPE" in os.environ:  # 1 = TGS (the presets), 0 = PGS
    cfg.sim.physx.solver_type = int(os.environ["LRL_SOLVER_TYPE"])
cfg.env.num_envs = 4096
R.RunnerArgs.save_interval = 0
R.RunnerArgs.log_freq = 10 ** 9
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234))
g = torch.Generator(device="cuda:0").manual_seed(1)
cmd = torch.rand(4096, 3, device="cuda:0", generator=g)
env.env.commands[:, :3] = cmd * torch.tensor([1.2, 1.2, 2.0], device="cuda:0") - torch.tensor([0.6, 0.6, 1.0], device="cuda:0")
runner = R.Runner(env, device="cuda:0", seed=1234)
runner.learn(3, init_at_random_ep_len=True)
torch.cuda.synchronize()
env.env.kernel_timing(True)
ts = []
for _ in range(iters):
    t0 = time.perf_counter()
    runner.learn(1)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
# the bench's way as well: `iters` iterations in one learn() call, one sync at the end (host runs ahead across
# iterations), mean per iteration
t0 = time.perf_counter()
runner.learn(iters)
torch.cuda.synchronize()
batch_ms = (time.perf_counter() - t0) * 1e3 / iters
k = env.env.kernel_timing(False)[0]
print(json.dumps({"tag": tag, "median_ms": round(statistics.median(ts), 3), "min_ms": round(min(ts), 3),
                  "batch_mean_ms": round(batch_ms, 3), "env_kernel_ms": round(k, 4), "iters": iters}), flush=True)
