"""Host time per section of LeggedRobotEnv.step over one PPO rollout (development tool): where the rollout's wall
time goes between the act launch, the pre-step command resampling, the env-kernel launch + the one device->host
copy (which waits for the GPU), reset_idx / observe of the reset envs and the extras.  Also the time spent outside
step (act + storage writes).  usage: python scripts/step_timing.py [mc|go1_rough] [rollouts]"""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402
from lrl.ppo import runner as R  # noqa: E402


class Timer:
    def __init__(self):
        self.acc = defaultdict(float)
        self.n = defaultdict(int)
        self.last = None

    def mark(self, name):
        t = time.perf_counter()
        if name == "entry":
            if self.last is not None:
                self.acc["outside_step"] += t - self.last
                self.n["outside_step"] += 1
        else:
            self.acc[name] += t - self.last
            self.n[name] += 1
        self.last = t


which = sys.argv[1] if len(sys.argv) > 1 else "go1_rough"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cfg = lcfg.make_cfg()
R.RunnerArgs.save_interval = 0
R.RunnerArgs.log_freq = 10 ** 9
if which == "go1_rough":
    lcfg.config_go1(cfg)
    cfg.env.num_envs = 4096
    cfg.terrain.mesh_type = "trimesh"
    cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
    cfg.terrain.curriculum = True
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=4321, legacy_fork=False))
else:
    lcfg.config_mini_cheetah(cfg)
    cfg.env.num_envs = 4096
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234))
runner = R.Runner(env, device="cuda:0", seed=1234)
runner.learn(2, init_at_random_ep_len=True)
torch.cuda.synchronize()
alg = runner.alg
obs_dict = env.get_observations()
obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
tm = Timer()
env.env._step_timer = tm
env.env.kernel_timing(True)
t0 = time.perf_counter()
with torch.inference_mode():
    for _ in range(reps):
        for _ in range(24):
            actions = alg.act(obs, priv, hist)
            od, rewards, dones, infos = env.step(actions)
            obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]
            alg.process_env_step(rewards, dones, infos)
        alg.storage.clear()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
env.env._step_timer = None
k_ms = env.env.kernel_timing(False)[0]
steps = 24 * reps
print(f"{which}: {steps} steps, {wall / steps * 1e3:.3f} ms per step (wall), env kernel {k_ms:.3f} ms")
for k, v in sorted(tm.acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:20s} {v / steps * 1e3:8.3f} ms per step")
