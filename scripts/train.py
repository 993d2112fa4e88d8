"""Drop-in for the reference's scripts/train.py (scripts/train.py:1-54): same imports and calls,
resolved to the MI355X implementation.  Usage: python scripts/train.py [--iterations N]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))


def train_mc(headless=True, iterations=4000, robot="mc", run_dir=None):
    import torch  # noqa: F401

    from mini_gym.envs.base.legged_robot_config import Cfg
    from mini_gym.envs.go1.go1_config import config_go1
    from mini_gym.envs.mini_cheetah.mini_cheetah_config import config_mini_cheetah
    from mini_gym.envs.mini_cheetah.velocity_tracking import VelocityTrackingEasyEnv
    from mini_gym.envs.wrappers.history_wrapper import HistoryWrapper
    from mini_gym_learn.ppo import Runner
    from lrl.ppo.runner import Logger

    (config_mini_cheetah if robot == "mc" else config_go1)(Cfg)
    env = VelocityTrackingEasyEnv(sim_device="cuda:0", headless=headless, cfg=Cfg)
    env = HistoryWrapper(env)
    runner = Runner(env, device="cuda:0", logger=Logger(run_dir))
    runner.learn(num_learning_iterations=iterations, init_at_random_ep_len=True, eval_freq=100)
    return runner


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=4000)
    ap.add_argument("--robot", default="mc", choices=["mc", "go1"])
    ap.add_argument("--run-dir", default=None)
    a = ap.parse_args()
    train_mc(iterations=a.iterations, robot=a.robot, run_dir=a.run_dir)
