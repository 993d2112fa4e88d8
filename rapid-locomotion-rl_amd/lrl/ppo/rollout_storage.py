"""Rollout buffer (mini_gym_learn/ppo/rollout_storage.py:7-139) with the HIP GAE kernel.

Buffers keep the reference's [T, N, ...] shapes.  In the fused rollout path the policy kernel
writes obs / priv / history / actions / values / log-probs / mu / sigma straight into row
``self.step`` (``lrl_rollout_store``), so ``add_transitions`` only has the env outputs left to copy.
"""
import ctypes as C

import torch

from .. import _abi


class RolloutStorage:
    class Transition:
        def __init__(self):
            self.observations = None
            self.privileged_observations = None
            self.observation_histories = None
            self.critic_observations = None
            self.actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.env_bins = None

        def clear(self):
            self.__init__()

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, obs_history_shape,
                 actions_shape, device="cpu"):
        self.device = device
        self.obs_shape, self.privileged_obs_shape = obs_shape, privileged_obs_shape
        self.obs_history_shape, self.actions_shape = obs_history_shape, actions_shape
        T, N = num_transitions_per_env, num_envs
        z = lambda *s: torch.zeros(T, N, *s, device=device)
        self.observations = z(*obs_shape)
        self.privileged_observations = z(*privileged_obs_shape)
        # history rows at a 16-float pitch (zero padding): the adaptation module's first layer then reads
        # float4-aligned rows (lrl_ppo_batch.hist_ld); the [T, N, H] view keeps the reference's shape
        h = int(obs_history_shape[0]) if len(obs_history_shape) == 1 else None
        if h is not None and h % 16:
            hp = (h + 15) // 16 * 16
            self._hist_padded = torch.zeros(T, N, hp, device=device)
            self.observation_histories = self._hist_padded[..., :h]
        else:
            self.observation_histories = z(*obs_history_shape)
        self.rewards = z(1)
        self.actions = z(*actions_shape)
        self.dones = z(1).byte()
        self.actions_log_prob = z(1)
        self.values = z(1)
        self.returns = z(1)
        self.advantages = z(1)
        self.mu = z(*actions_shape)
        self.sigma = z(*actions_shape)
        self.env_bins = z(1)
        self.num_transitions_per_env, self.num_envs = T, N
        self.step = 0
        self._ws = None
        self.adv_stats = None

    def store_desc(self):
        """lrl_rollout_store pointing at the [T, N, ...] buffers (row selected at launch)."""
        s = _abi.LrlRolloutStore()
        s.obs, s.priv, s.hist = (self.observations.data_ptr(), self.privileged_observations.data_ptr(),
                                 self.observation_histories.data_ptr())
        s.actions, s.values, s.logp = self.actions.data_ptr(), self.values.data_ptr(), self.actions_log_prob.data_ptr()
        s.mu, s.sigma = self.mu.data_ptr(), self.sigma.data_ptr()
        s.hist_dim = self.obs_history_shape[0]
        s.hist_ld = self.observation_histories.stride(1)
        return s

    def add_transitions(self, transition, fused=False):
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        t = self.step
        if not fused:
            self.observations[t].copy_(transition.observations)
            self.privileged_observations[t].copy_(transition.privileged_observations)
            self.observation_histories[t].copy_(transition.observation_histories)
            self.actions[t].copy_(transition.actions)
            self.values[t].copy_(transition.values)
            self.actions_log_prob[t].copy_(transition.actions_log_prob.view(-1, 1))
            self.mu[t].copy_(transition.action_mean)
            self.sigma[t].copy_(transition.action_sigma)
        self.rewards[t].copy_(transition.rewards.view(-1, 1))
        self.dones[t].copy_(transition.dones.view(-1, 1))
        self.env_bins[t].copy_(transition.env_bins.view(-1, 1))
        self.step += 1

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam, reduce_stats=None):
        """GAE + advantage normalisation in two HIP launches (lrl_gae); ``reduce_stats`` lets a
        multi-GPU caller all-reduce (sum, sum of squares, count) before normalising."""
        T, N = self.num_transitions_per_env, self.num_envs
        if self._ws is None:
            self._ws = torch.empty(4096, device=self.device)
        lv = last_values.contiguous().float()
        p = lambda t: C.c_void_p(t.data_ptr())
        stream = _abi.stream_of(self.rewards.device)
        if reduce_stats is None:
            _abi.check(_abi.lib().lrl_gae(p(self.rewards), p(self.dones), p(self.values), p(lv), C.c_int32(T),
                                          C.c_int32(N), C.c_float(gamma), C.c_float(lam), p(self.returns),
                                          p(self.advantages), p(self._ws), stream))
        else:
            stats = torch.empty(3, dtype=torch.float64, device=self.device)
            _abi.check(_abi.lib().lrl_gae_partial(p(self.rewards), p(self.dones), p(self.values), p(lv),
                                                  C.c_int32(T), C.c_int32(N), C.c_float(gamma), C.c_float(lam),
                                                  p(self.returns), p(self.advantages), p(self._ws), p(stats), stream))
            stats = reduce_stats(stats)
            _abi.check(_abi.lib().lrl_adv_normalize(p(self.advantages), C.c_int64(T * N), p(stats), stream))

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        batch_size = self.num_envs * self.num_transitions_per_env
        mb = batch_size // num_mini_batches
        indices = torch.randperm(num_mini_batches * mb, requires_grad=False, device=self.device)
        flat = lambda t: t.flatten(0, 1)
        obs, priv, hist = flat(self.observations), flat(self.privileged_observations), flat(self.observation_histories)
        actions, values, returns = flat(self.actions), flat(self.values), flat(self.returns)
        logp, adv, mu, sigma, bins = (flat(self.actions_log_prob), flat(self.advantages), flat(self.mu),
                                      flat(self.sigma), flat(self.env_bins))
        for epoch in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mb:(i + 1) * mb]
                yield (obs[idx], obs[idx], priv[idx], hist[idx], actions[idx], values[idx], adv[idx], returns[idx],
                       logp[idx], mu[idx], sigma[idx], None, bins[idx])
