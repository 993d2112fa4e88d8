"""Play a trained policy — the reference's scripts/play.py (load_env :16-92, play_mc :95-156) on this stack.

The ActorCritic comes from a state dict (``--weights file.pt``, loaded with ``weights_only=True``) or, by default,
from the reference run's trained ``ac_weights_last.pt`` as committed in tests/golden/checkpoint_last.npz (Mini
Cheetah, the robot that run used).  The env is the evaluation env of load_env (domain randomisation off, 3 x 5
terrain tiles, no border); the policy is act_inference = the adaptation module on the observation history +
the actor (``ActorCritic.act_student_fused``, the native GEMM chain).  A constant forward command is tracked for
``--steps`` policy steps after 20 zero-action steps, as play_mc does; the measured forward velocity is printed
(and plotted with ``--plot out.png``).  Rendering is out of scope.

  python scripts/play.py [--robot mc|go1] [--weights ac_weights.pt] [--envs 64] [--steps 1000] [--vx 1.0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402
from lrl.ppo.actor_critic import ActorCritic  # noqa: E402


def load_env(robot, num_envs, device):
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    dr = cfg.domain_rand
    for k in ("push_robots", "randomize_friction", "randomize_restitution", "randomize_motor_strength",
              "randomize_base_mass", "randomize_Kd_factor", "randomize_Kp_factor", "randomize_com_displacement"):
        setattr(dr, k, False)
    cfg.env.num_envs = num_envs
    if "LRL_SOLVER_TYPE" in os.environ:  # 1 = TGS (the presets' solver), 0 = PGS
        cfg.sim.physx.solver_type = int(os.environ["LRL_SOLVER_TYPE"])
    cfg.terrain.num_rows, cfg.terrain.num_cols, cfg.terrain.border_size = 3, 5, 0
    cfg.terrain.max_init_terrain_level = min(cfg.terrain.max_init_terrain_level, cfg.terrain.num_rows - 1)
    return HistoryWrapper(LeggedRobotEnv(device, cfg=cfg)), cfg


def load_policy(weights, cfg, device):
    ac = ActorCritic(cfg.env.num_observations, cfg.env.num_privileged_obs,
                     cfg.env.num_observations * cfg.env.num_observation_history, cfg.env.num_actions)
    if weights:
        sd = torch.load(weights, map_location="cpu", weights_only=True)
    else:
        g = np.load(os.path.join(ROOT, "tests", "golden", "checkpoint_last.npz"), allow_pickle=False)
        sd = {k: torch.from_numpy(g["sd/" + k]) for k in g["keys"]}
    ac.load_state_dict(sd, strict=True)
    ac = ac.to(device)
    return lambda ob: ac.act_student_fused(ob["obs"].contiguous(), ob["obs_history"])[0]


def play(robot="mc", weights=None, num_envs=64, steps=1000, vx=1.0, vy=0.0, wz=0.0, device="cuda:0"):
    env, cfg = load_env(robot, num_envs, device)
    policy = load_policy(weights, cfg, device)
    e = env.env

    def command():
        e.commands[:, 0], e.commands[:, 1], e.commands[:, 2] = vx, vy, wz

    command()
    obs = env.reset()
    actions = torch.zeros(num_envs, 12, device=device)
    with torch.no_grad():
        for _ in range(20):
            command()
            obs, rew, done, info = env.step(actions)
    vel = np.zeros((steps, num_envs, 3), np.float32)
    for i in range(steps):
        with torch.no_grad():
            actions = policy(obs)
        command()
        obs, rew, done, info = env.step(actions)
        vel[i, :, :2] = e.base_lin_vel[:, :2].cpu().numpy()
        vel[i, :, 2] = e.base_ang_vel[:, 2].cpu().numpy()
    upright = (e.projected_gravity[:, 2] < -0.8).float().mean().item()
    e.close()
    return vel, upright, e.dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="mc", choices=["mc", "go1"])
    ap.add_argument("--weights", default=None)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--vx", type=float, default=1.0)
    ap.add_argument("--plot", default=None)
    a = ap.parse_args()
    vel, upright, dt = play(a.robot, a.weights, a.envs, a.steps, a.vx)
    tail = vel[len(vel) // 2:]
    print(json.dumps({"robot": a.robot, "command_vx": a.vx, "steps": a.steps, "envs": a.envs,
                      "measured_vx_mean": round(float(tail[..., 0].mean()), 4),
                      "measured_vx_std_over_envs": round(float(tail[..., 0].mean(0).std()), 4),
                      "measured_vy_mean": round(float(tail[..., 1].mean()), 4),
                      "measured_wz_mean": round(float(tail[..., 2].mean()), 4), "upright_fraction": upright}))
    if a.plot:
        from matplotlib import pyplot as plt
        t = np.arange(len(vel)) * dt
        plt.figure(figsize=(12, 4))
        plt.plot(t, vel[:, 0, 0], "k-", label="Measured")
        plt.plot(t, np.full(len(vel), a.vx), "k--", label="Desired")
        plt.legend()
        plt.xlabel("Time (s)")
        plt.ylabel("Velocity (m/s)")
        plt.title("Forward Linear Velocity")
        plt.tight_layout()
        plt.savefig(a.plot)


if __name__ == "__main__":
    main()
