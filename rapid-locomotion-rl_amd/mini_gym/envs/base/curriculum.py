"""mini_gym/envs/base/curriculum.py surface."""
from lrl.curriculum import GridCurriculum as Curriculum, RewardThresholdCurriculum  # noqa: F401
