"""mini_gym_learn/ppo/rollout_storage.py surface."""
from lrl.ppo.rollout_storage import RolloutStorage  # noqa: F401
