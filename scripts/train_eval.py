"""Train from scratch, then play — an end-to-end check of the whole stack on one MI355X.

Mini Cheetah, 4096 envs, the upstream semantics the reference's published run had (legacy_fork=False: time-outs
and terminations reset inside step, commands resampled from the grid-adaptive curriculum every 10 s and at
resets); ``--iterations`` PPO iterations of the reference's Runner (24 steps x 4096 envs, 5 epochs x 4
minibatches, the adaptation module trained alongside); then the learned student policy (act_inference:
adaptation module on the history + actor) tracks constant forward commands (scripts/play.py).  Prints one JSON
line: wall time, iterations/s, the tracking rewards early vs late, the command area the curriculum reached, and
the measured forward velocity per command.

  python scripts/train_eval.py [--iterations 1500] [--out DIR]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402
from lrl.ppo import runner as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=1500)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = lcfg.make_cfg()
    lcfg.config_mini_cheetah(cfg)
    cfg.env.num_envs = a.envs
    R.RunnerArgs.save_interval = 0
    R.RunnerArgs.log_freq = 50
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=11, legacy_fork=False))
    runner = R.Runner(env, device="cuda:0", seed=11)
    t0 = time.time()
    chunk, hist = 50, []
    done = 0
    while done < a.iterations:
        k = min(chunk, a.iterations - done)
        runner.learn(k, init_at_random_ep_len=(done == 0))
        done += k
        ep = env.env.extras.get("train/episode", {})
        row = {"it": done, "t": round(time.time() - t0, 1)}
        for key in ("rew_total", "rew_tracking_lin_vel", "rew_tracking_ang_vel", "command_area"):
            v = ep.get(key)
            if v is not None:
                row[key] = round(float(v), 5)
        hist.append(row)
        print(json.dumps(row), flush=True)
    wall = time.time() - t0
    sd = runner.alg.actor_critic.state_dict()
    out = a.out or os.path.join(ROOT, "gpurun_out", "train_eval")
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "ac_weights_last.pt")
    torch.save({k: v.detach().cpu() for k, v in sd.items()}, path)
    env.env.close()
    import play
    evals = {}
    for vx in (0.0, 0.5, 1.0):
        vel, upright, _ = play.play("mc", path, num_envs=64, steps=500, vx=vx)
        evals[str(vx)] = {"measured_vx": round(float(vel[250:, :, 0].mean()), 4), "upright": upright}
    print(json.dumps({"iterations": a.iterations, "wall_s": round(wall, 1),
                      "iterations_per_s": round(a.iterations / wall, 3),
                      "env_steps_per_s": round(a.iterations * a.envs * 24 / wall, 1),
                      "first": hist[0], "last": hist[-1], "play": evals}), flush=True)


if __name__ == "__main__":
    main()
