from lrl.ppo.actor_critic import AC_Args, ActorCritic, get_activation  # noqa: F401
