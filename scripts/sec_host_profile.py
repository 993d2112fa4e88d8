"""Host-side (Python) cost of bench.py's secondary line (configs[2]): cProfile over PPO iterations of the Go1
rough-terrain workload, the top functions by own time, plus the wall time per iteration with and without a device
sync per env step (when the host is the bound, the rollout's GPU idles between launches).
usage: python scripts/sec_host_profile.py [iters]"""
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
from lrl.ppo import runner as R  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = lcfg.make_cfg()
lcfg.config_go1(cfg)
cfg.env.num_envs = 4096
cfg.terrain.mesh_type = "trimesh"
cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
cfg.terrain.curriculum = True
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=4321, legacy_fork=False))
runner = R.Runner(env, device="cuda:0", seed=4321)
R.RunnerArgs.save_interval = 0
runner.learn(2, init_at_random_ep_len=True)
torch.cuda.synchronize()
# host time of the rollout alone: the env step + act calls, timed on the host without syncs
alg = runner.alg
obs_dict = env.get_observations()
obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
with torch.inference_mode():
    for tag in ("step", "act", "process"):
        pass
    t_step = t_act = t_proc = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(24):
        a = time.perf_counter()
        actions = alg.act(obs, priv, hist)
        b = time.perf_counter()
        obs_dict, rewards, dones, infos = env.step(actions)
        c = time.perf_counter()
        obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
        alg.process_env_step(rewards, dones, infos)
        d = time.perf_counter()
        t_act += b - a
        t_step += c - b
        t_proc += d - c
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    alg.storage.clear()
print(f"rollout of 24 steps: host issue {1e3 * t_issue:.2f} ms (act {1e3 * t_act:.2f}, env.step {1e3 * t_step:.2f}, "
      f"process_env_step {1e3 * t_proc:.2f}); wall incl. the GPU {1e3 * t_all:.2f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
runner.learn(iters)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
