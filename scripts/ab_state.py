"""Bit-identity check of a library change: runs the bench's workload (4096 Mini Cheetah envs, flat, fork semantics,
random-init policy; or 4096 Go1 envs on the curriculum trimesh with `rough`) for a few PPO iterations under the
library LRL_LIB names and saves the env state and the policy parameters; `compare` diffs two such files.
usage: LRL_LIB=... python scripts/ab_state.py run <out.npz> [iters] [mc|rough]
       python scripts/ab_state.py compare <a.npz> <b.npz>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))


def run(out, iters=2, workload="mc"):
    import torch
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    from lrl.ppo import runner as R
    n = 4096
    cfg = lcfg.make_cfg()
    legacy = True
    if workload == "rough":
        lcfg.config_go1(cfg)
        cfg.terrain.mesh_type = "trimesh"
        cfg.terrain.measure_heights = True
        cfg.terrain.curriculum = True
        cfg.env.num_observations = 42 + 187
        legacy = False
    else:
        lcfg.config_mini_cheetah(cfg)
    cfg.env.num_envs = n
    R.RunnerArgs.save_interval = 0
    R.RunnerArgs.log_freq = 10 ** 9
    torch.manual_seed(0)
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234, legacy_fork=legacy))
    runner = R.Runner(env, device="cuda:0", seed=1234)
    runner.learn(iters, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    e = env.env
    g = lambda t: t.detach().cpu().numpy().copy()
    np.savez(out, root=g(e.root_states), dof_pos=g(e.dof_pos), dof_vel=g(e.dof_vel), contact=g(e.contact_forces),
             torques=g(e.torques), obs=g(e.obs_buf), priv=g(e.privileged_obs_buf), rew=g(e.rew_buf),
             episode_sums=g(e._episode_sums), command_sums=g(e._command_sums),
             params=g(runner.alg.actor_critic._flat))
    print("saved", out)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        eq = np.array_equal(x.view(np.uint32), y.view(np.uint32)) if x.dtype == np.float32 else np.array_equal(x, y)
        diff = np.abs(x.astype(np.float64) - y.astype(np.float64))
        print(f"{k:10s} bit-identical={eq} max|diff|={diff.max():.3g} differing={int((diff > 0).sum())}/{x.size}")
        bad += not eq
    print("IDENTICAL" if not bad else f"{bad} arrays differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2, sys.argv[4] if len(sys.argv) > 4 else "mc")
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
