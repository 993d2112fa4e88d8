"""Bit-identity of single env steps between two libraries: the bench's Mini Cheetah env (4096 envs, fork semantics),
a few steps of fixed pseudo-random actions, every state row saved after each step.
usage: LRL_LIB=... python scripts/ab_step.py run <out.npz> [steps]; python scripts/ab_step.py compare <a> <b>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))


def run(out, steps=3):
    import torch
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    cfg = lcfg.make_cfg()
    lcfg.config_mini_cheetah(cfg)
    cfg.env.num_envs = 4096
    env = LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234, legacy_fork=True)
    g = lambda t: t.detach().cpu().numpy().copy()
    rng = np.random.default_rng(5)
    rec = {}
    torch.cuda.synchronize()
    for k in ["root_states", "dof_pos", "dof_vel", "_episode_sums", "_command_sums", "motor_strengths", "Kp_factors",
              "Kd_factors", "last_actions", "last_dof_vel", "feet_air_time", "commands", "episode_length_buf", "torques",
              "friction_coeffs", "payloads", "com_displacements", "contact_forces", "obs_buf", "rew_buf"]:
        rec[f"{k}_init"] = g(getattr(env, k))
    for s in range(steps):
        a = torch.as_tensor(rng.normal(size=(4096, 12)).astype(np.float32), device="cuda:0")
        env.step(a)
        torch.cuda.synchronize()
        for k, t in dict(root=env.root_states, dof_pos=env.dof_pos, dof_vel=env.dof_vel, contact=env.contact_forces,
                         obs=env.obs_buf, rew=env.rew_buf, es=env._episode_sums, cs=env._command_sums).items():
            rec[f"{k}_{s}"] = g(t)
    np.savez(out, **rec)
    print("saved", out)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
    else:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        from ab_state import compare
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
