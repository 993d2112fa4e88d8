"""mini_gym/envs/base/base_task.py surface: BaseTask's buffers (obs / privileged obs / reward / reset / episode
length / time-out) and step / reset / get_observations live on the native env class."""
from lrl.env import LeggedRobotEnv as BaseTask  # noqa: F401
