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
env_obs = env.get_observations()


def rollout():  # one rollout of the bench's loop (alg.act / env.step / process_env_step), nothing synchronised
    global env_obs
    with torch.inference_mode():
        for _ in range(runner.num_steps_per_env):
            a = alg.act(env_obs["obs"], env_obs["privileged_obs"], env_obs["obs_history"])
            env_obs, rew, done, infos = env.step(a)
            alg.process_env_step(rew, done, infos)
        alg.compute_returns(env_obs["obs"], env_obs["privileged_obs"])


# the update right after a rollout, once with a device sync between them and once without (the bench's order)
for mode in ("after_rollout_synced", "after_rollout_queued"):
    ts = []
    for _ in range(reps):
        rollout()
        if mode == "after_rollout_synced":
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        alg.update()
        e1.record()
        torch.cuda.synchronize()
        ts.append(round(e0.elapsed_time(e1), 3))
    print(json.dumps({mode + "_update_gpu_ms": ts}))
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
