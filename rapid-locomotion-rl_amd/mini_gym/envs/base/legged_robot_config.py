"""``from mini_gym.envs.base.legged_robot_config import Cfg`` (legged_robot_config.py:6)."""
from lrl.config import Cfg  # noqa: F401
