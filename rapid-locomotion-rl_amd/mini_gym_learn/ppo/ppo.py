from lrl.ppo.ppo import PPO, PPO_Args  # noqa: F401
