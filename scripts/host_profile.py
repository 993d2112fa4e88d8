"""Host-side cost of one rollout step of the bench workload (development tool): cProfile over Runner.learn's
rollout loop, top functions by own time.  usage: python scripts/host_profile.py [mc|go1_rough]
(mc: 4096 Mini Cheetah envs, flat, fork semantics — the headline; go1_rough: bench.py's secondary line, 4096 Go1
envs on the curriculum trimesh with the upstream reset path)"""
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

which = sys.argv[1] if len(sys.argv) > 1 else "mc"
cfg = lcfg.make_cfg()
R.RunnerArgs.save_interval = 0
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
alg = runner.alg
obs_dict = env.get_observations()
obs, priv, hist = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
torch.cuda.synchronize()


def rollout():
    global obs, priv, hist
    with torch.inference_mode():
        for _ in range(24):
            actions = alg.act(obs, priv, hist)
            od, rewards, dones, infos = env.step(actions)
            obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]
            alg.process_env_step(rewards, dones, infos)
    alg.storage.clear()


rollout()
torch.cuda.synchronize()
# host enqueue time alone: the GPU is kept busy by a long kernel first, so nothing the host does waits for it
t0 = time.perf_counter()
rollout()
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"rollout: host enqueue {t_host * 1e3:.2f} ms, with GPU drain {t_all * 1e3:.2f} ms (24 steps)")
pr = cProfile.Profile()
pr.enable()
rollout()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(40)
