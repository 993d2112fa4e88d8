"""Drop-in for the reference's scripts/test.py (:14-46): a few Mini Cheetah envs, reset, zero-action
steps.  (The reference's config 0 runs Isaac Gym's CPU pipeline; here the env always runs through
liblrl on the GPU, and the CPU path is the oracle in oracle/.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))


def run_env(num_envs=16, steps=1000):
    import torch
    from mini_gym.envs.base.legged_robot_config import Cfg
    from mini_gym.envs.mini_cheetah.mini_cheetah_config import config_mini_cheetah
    from mini_gym.envs.mini_cheetah.velocity_tracking import VelocityTrackingEasyEnv
    config_mini_cheetah(Cfg)
    Cfg.env.num_envs = num_envs
    env = VelocityTrackingEasyEnv(sim_device="cuda:0", headless=True, cfg=Cfg)
    env.reset()
    for _ in range(steps):
        actions = 0.0 * torch.ones(env.num_envs, env.num_actions, device=env.device)
        obs, rew, done, info = env.step(actions)
    print("Done")
    return env


if __name__ == "__main__":
    run_env()
