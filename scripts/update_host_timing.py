"""Host side of the native PPO update (development helper): the bench's workload (4096 Mini Cheetah envs), then
PPO.update() timed from an idle GPU — host enqueue time (until update() returns, no sync) against the wall time to
the final sync — and a cProfile of the host calls of one update.
usage: python scripts/update_host_timing.py [reps]"""
import cProfile
import io
import json
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
from lrl.ppo import runner as R  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
cfg = lcfg.make_cfg()
lcfg.config_mini_cheetah(cfg)
cfg.env.num_envs = 4096
R.RunnerArgs.save_interval = 0
R.RunnerArgs.log_freq = 10 ** 9
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234))
runner = R.Runner(env, device="cuda:0", seed=1234)
runner.learn(3, init_at_random_ep_len=True)
torch.cuda.synchronize()
alg = runner.alg
host, wall = [], []
for _ in range(reps):
    s = alg.storage
    s.step = s.num_transitions_per_env  # (the data of the last rollout is still there: update() only resets step)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    alg.update()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.append((t1 - t0) * 1e3)
    wall.append((t2 - t0) * 1e3)
s = alg.storage
s.step = s.num_transitions_per_env
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
alg.update()
pr.disable()
torch.cuda.synchronize()
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
print(json.dumps({"host_enqueue_ms": [round(x, 3) for x in host], "wall_ms": [round(x, 3) for x in wall]}))
print(buf.getvalue())
