"""mini_gym/envs/base/legged_robot.py surface."""
from lrl.env import LeggedRobotEnv as LeggedRobot  # noqa: F401
