"""``mini_gym_learn.ppo`` surface: Runner, RunnerArgs, PPO, ActorCritic, RolloutStorage."""
from lrl.ppo.actor_critic import AC_Args, ActorCritic  # noqa: F401
from lrl.ppo.rollout_storage import RolloutStorage  # noqa: F401
from lrl.ppo.runner import Runner, RunnerArgs  # noqa: F401
