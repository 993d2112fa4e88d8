"""mini_gym/envs/mini_cheetah/velocity_tracking/velocity_tracking_easy_env.py surface."""
from lrl.env import VelocityTrackingEasyEnv  # noqa: F401
