"""Minimal env interface (mini_gym_learn/env/vec_env.py:10-39): what Runner relies on."""
from abc import ABC, abstractmethod


class VecEnv(ABC):
    num_envs: int
    num_obs: int
    num_privileged_obs: int
    num_actions: int
    max_episode_length: int

    @abstractmethod
    def step(self, actions):
        ...

    @abstractmethod
    def reset(self):
        ...

    @abstractmethod
    def get_observations(self):
        ...

    @abstractmethod
    def get_privileged_observations(self):
        ...
