"""Teacher/student actor-critic (mini_gym_learn/ppo/actor_critic.py:23-173).

Parameters live in torch (nn.Module, so state dicts / checkpoints keep the reference's 35-key
layout, including the duplicate ``encoder.*`` registration of ``env_factor_encoder`` — Q13).  The
rollout forward of the teacher path (encoder -> actor / critic -> Normal sample -> log-prob -> storage
row) runs natively (``lrl_ppo_act``: fp32-MFMA GEMMs + one head kernel) on a flat parameter buffer
that the nn.Module's tensors are views of (``flatten_parameters``); the update uses the same buffer.
"""
import ctypes as C

import torch

import torch.nn as nn

from .. import _abi
from ..config import ArgsProto


class AC_Args(ArgsProto):
    """actor_critic.py:9-20"""
    init_noise_std = 1.0
    actor_hidden_dims = [512, 256, 128]
    critic_hidden_dims = [512, 256, 128]
    activation = "elu"
    adaptation_module_branch_hidden_dims = [[256, 32]]
    env_factor_encoder_branch_input_dims = [18]
    env_factor_encoder_branch_latent_dims = [18]
    env_factor_encoder_branch_hidden_dims = [[256, 128]]


def get_activation(name):
    return {"elu": nn.ELU(), "selu": nn.SELU(), "relu": nn.ReLU(), "crelu": nn.ReLU(), "lrelu": nn.LeakyReLU(),
            "tanh": nn.Tanh(), "sigmoid": nn.Sigmoid()}.get(name)


def _mlp(dims, act):
    layers = []
    for i in range(len(dims) - 1):
        layers.append(nn.Linear(dims[i], dims[i + 1]))
        if i < len(dims) - 2:
            layers.append(act)
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    is_recurrent = False

    def __init__(self, num_obs, num_privileged_obs, num_obs_history, num_actions, **kwargs):
        super().__init__()
        act = get_activation(AC_Args.activation)
        enc_in = AC_Args.env_factor_encoder_branch_input_dims[0]
        enc_lat = AC_Args.env_factor_encoder_branch_latent_dims[0]
        self.env_factor_encoder = _mlp([enc_in] + AC_Args.env_factor_encoder_branch_hidden_dims[0] + [enc_lat], act)
        self.add_module("encoder", self.env_factor_encoder)
        self.adaptation_module = _mlp([num_obs_history] + AC_Args.adaptation_module_branch_hidden_dims[0] + [enc_lat],
                                      act)
        latent = sum(AC_Args.env_factor_encoder_branch_latent_dims)
        self.actor_body = _mlp([latent + num_obs] + AC_Args.actor_hidden_dims + [num_actions], act)
        self.critic_body = _mlp([latent + num_obs] + AC_Args.critic_hidden_dims + [1], act)
        self.std = nn.Parameter(AC_Args.init_noise_std * torch.ones(num_actions))
        self.num_obs, self.num_privileged_obs, self.num_actions = num_obs, num_privileged_obs, num_actions
        self.distribution = None

    # ---- reference API (torch path; used by the update and for checkpoint-compatible inference) ----
    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def update_distribution(self, observations, privileged_observations):
        latent = self.env_factor_encoder(privileged_observations)
        mean = self.actor_body(torch.cat((observations, latent), dim=-1))
        self.distribution = torch.distributions.Normal(mean, mean * 0.0 + self.std, validate_args=False)

    def act(self, observations, privileged_observations, **kwargs):
        self.update_distribution(observations, privileged_observations)
        return self.distribution.sample()

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_expert(self, ob, policy_info={}):
        return self.act_teacher(ob["obs"], ob["privileged_obs"])

    def act_inference(self, ob, policy_info={}):
        if ob["privileged_obs"] is not None:
            policy_info["gt_latents"] = self.env_factor_encoder(ob["privileged_obs"]).detach().cpu().numpy()
        return self.act_student(ob["obs"], ob["obs_history"])

    def act_student(self, observations, observation_history, policy_info={}):
        latent = self.adaptation_module(observation_history)
        policy_info["latents"] = latent.detach().cpu().numpy()
        return self.actor_body(torch.cat((observations, latent), dim=-1))

    def act_teacher(self, observations, privileged_info, policy_info={}):
        latent = self.env_factor_encoder(privileged_info)
        policy_info["latents"] = latent.detach().cpu().numpy()
        return self.actor_body(torch.cat((observations, latent), dim=-1))

    def evaluate(self, critic_observations, privileged_observations, **kwargs):
        latent = self.env_factor_encoder(privileged_observations)
        return self.critic_body(torch.cat((critic_observations, latent), dim=-1))

    # ---- flat parameter buffer (lrl_ppo_net layout) ----
    def flatten_parameters(self):
        """Move every parameter into ONE flat fp32 buffer on its current device (the tensors become views,
        so state_dict / load_state_dict / the optimiser see the same storage).  Layout: the PPO step's
        parameters [actor/critic layer pairs adjacent, heads, encoder, std], one KL slot, then the
        adaptation module; returns the lrl_ppo_net descriptor (offsets in floats)."""
        net = getattr(self, "_net", None)
        if net is not None and self.std.data_ptr() == self._flat.data_ptr() + 4 * net.std_off:
            return net
        A = [m for m in self.actor_body if isinstance(m, nn.Linear)]
        Cb = [m for m in self.critic_body if isinstance(m, nn.Linear)]
        E = [m for m in self.env_factor_encoder if isinstance(m, nn.Linear)]
        D = [m for m in self.adaptation_module if isinstance(m, nn.Linear)]
        if len(A) != 4 or len(Cb) != 4 or len(E) != 3 or len(D) != 3:
            raise ValueError("lrl_ppo expects 4-layer actor/critic and 3-layer encoder/adaptation MLPs")
        if not isinstance(self.actor_body[1], nn.ELU):
            raise ValueError("lrl_ppo implements the ELU activation only")
        net = _abi.LrlPpoNet()
        order, off = [], 0

        def put(name, *tensors, align=64):
            nonlocal off
            off = (off + align - 1) // align * align
            start = off
            for t in tensors:
                order.append((t, off))
                off += t.numel()
            if name:
                setattr(net, name, start)
            return start

        net.main_begin = 0
        for i, nm in enumerate(("1", "2", "3")):
            put("w" + nm, A[i].weight, Cb[i].weight)
            put("b" + nm, A[i].bias, Cb[i].bias)
        put("w4a", A[3].weight); put("b4a", A[3].bias); put("w4c", Cb[3].weight); put("b4c", Cb[3].bias)
        put("e1w", E[0].weight); put("e1b", E[0].bias); put("e2w", E[1].weight); put("e2b", E[1].bias)
        put("e3w", E[2].weight); put("e3b", E[2].bias)
        put("std_off", self.std)
        net.main_end = off
        net.kl_slot = off
        off += 1
        off = (off + 63) // 64 * 64
        net.adapt_begin = off
        put("d1w", D[0].weight); put("d1b", D[0].bias); put("d2w", D[1].weight); put("d2b", D[1].bias)
        put("d3w", D[2].weight); put("d3b", D[2].bias)
        net.adapt_end = off
        net.total = (off + 63) // 64 * 64
        dev = self.std.device
        flat = torch.zeros(net.total, device=dev)
        with torch.no_grad():
            for t, o in order:
                flat[o:o + t.numel()].copy_(t.detach().reshape(-1))
            for t, o in order:
                t.data = flat[o:o + t.numel()].view_as(t)
        net.num_obs, net.num_priv = self.num_obs, self.num_privileged_obs
        net.num_hist, net.num_actions = D[0].in_features, self.num_actions
        net.enc_h0, net.enc_h1, net.latent = E[0].out_features, E[1].out_features, E[2].out_features
        net.ac_h0, net.ac_h1, net.ac_h2 = A[0].out_features, A[1].out_features, A[2].out_features
        net.ad_h0, net.ad_h1 = D[0].out_features, D[1].out_features
        if A[0].in_features != self.num_obs + net.latent or [m.out_features for m in Cb[:3]] != \
                [net.ac_h0, net.ac_h1, net.ac_h2]:
            raise ValueError("actor and critic must share hidden sizes and take [obs, latent]")
        self._flat, self._net = flat, net
        return net

    # ---- fused HIP rollout path ----
    def act_student_fused(self, obs, hist):
        """act_student (actor_critic.py:160-164) on the flat parameters (lrl_ppo_act_student: adaptation
        module + actor body as one fp32-MFMA GEMM chain).  ``hist`` may be a row-strided view (e.g. the
        rollout storage's padded history).  Returns (actions_mean [N, A], latent [N, L])."""
        n = obs.shape[0]
        dev = obs.device
        assert obs.is_contiguous() and obs.dtype == torch.float32 and hist.dtype == torch.float32
        assert hist.dim() == 2 and hist.stride(1) == 1 and hist.shape[0] == n
        net = self.flatten_parameters()
        ws = getattr(self, "_student_ws", None)
        if ws is None or ws[0] != n or ws[1].device != dev:
            nbytes = _abi.lib().lrl_ppo_act_student_workspace_bytes(C.byref(net), C.c_int32(n))
            if nbytes < 0:
                raise RuntimeError("lrl_ppo_act_student_workspace_bytes rejected the network")
            ws = self._student_ws = (n, torch.empty(nbytes, dtype=torch.uint8, device=dev))
        mean = torch.empty(n, self.num_actions, device=dev)
        latent = torch.empty(n, net.latent, device=dev)
        ptr = lambda t: C.c_void_p(t.data_ptr())
        stream = _abi.stream_of(dev)
        _abi.check(_abi.lib().lrl_ppo_act_student(C.byref(net), ptr(self._flat), ptr(obs), ptr(hist),
                                                  C.c_int32(hist.stride(0)), C.c_int32(n), ptr(mean), ptr(latent),
                                                  ptr(ws[1]), stream))
        return mean, latent

    def act_fused(self, obs, priv, hist=None, eps=None, seed=0, counter=0, store=None, store_row=0, row_offset=0):
        """PPO.act teacher path on the flat parameters (lrl_ppo_act: fp32-MFMA GEMM chain + one head
        kernel that samples, scores and writes the storage row).  Returns (actions, mu, values [N,1], logp [N]).
        The policy noise is keyed by (seed, counter, row_offset + row): row_offset is the global id of row 0 (the
        rank's env_offset), so a sharded rollout samples what one process holding every env would."""
        n = obs.shape[0]
        dev = obs.device
        assert obs.is_contiguous() and priv.is_contiguous() and obs.dtype == torch.float32
        net = self.flatten_parameters()
        ws = getattr(self, "_act_ws", None)
        if ws is None or ws[0] != n or ws[1].device != dev:
            nbytes = _abi.lib().lrl_ppo_act_workspace_bytes(C.byref(net), C.c_int32(n))
            if nbytes < 0:
                raise RuntimeError("lrl_ppo_act_workspace_bytes rejected the network")
            ws = self._act_ws = (n, torch.empty(nbytes, dtype=torch.uint8, device=dev))
        actions = torch.empty(n, self.num_actions, device=dev)
        mu = torch.empty(n, self.num_actions, device=dev)
        values = torch.empty(n, 1, device=dev)
        logp = torch.empty(n, device=dev)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
        st = C.byref(store) if store is not None else None
        stream = _abi.stream_of(dev)
        _abi.check(_abi.lib().lrl_ppo_act(C.byref(net), ptr(self._flat), ptr(obs), ptr(priv), ptr(hist), C.c_int32(n),
                                          ptr(eps), C.c_uint64(seed), C.c_uint64(counter), C.c_int64(row_offset),
                                          ptr(actions), ptr(mu),
                                          ptr(values), ptr(logp), st, C.c_int32(store_row), ptr(ws[1]), stream))
        return actions, mu, values, logp
