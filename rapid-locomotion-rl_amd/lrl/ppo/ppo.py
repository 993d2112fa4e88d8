"""PPO (mini_gym_learn/ppo/ppo.py:15-178) on the MI355X path.

Rollout: ``act`` is one fused HIP launch (encoder + actor + critic + Normal sample + log-prob +
storage write); GAE is the HIP kernel of RolloutStorage.compute_returns.  Update: the reference's
algorithm step for step — adaptive-KL learning rate, clipped surrogate, clipped value loss,
entropy bonus, grad-norm clip 1.0, Adam; then the adaptation-module regression with a second Adam
(Q14: it only ever sees adaptation-module gradients).

On the GPU (``fused``) the update runs natively (``lrl_ppo_*`` in liblrl.so, csrc/lrl_ppo.hip):
parameters, gradients and Adam moments are flat device buffers, each minibatch is four launch
sequences (PPO forward/backward, adaptive LR + clip + Adam, adaptation forward/backward, Adam) and
the learning rate stays on the device, so a single-GPU update synchronises with the host once, at
its end.  With ``torch.distributed`` initialised, the flat gradient (+ the KL mean riding in the same
buffer) is all-reduced once per optimiser step and the advantage statistics once per iteration, so
every rank takes identical steps.  ``fused=False`` keeps the torch-autograd restatement (CPU tests).
"""
import ctypes as C
import os

import torch

import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .. import _abi
from ..config import ArgsProto
from .actor_critic import ActorCritic
from .rollout_storage import RolloutStorage


# encoder-weight snapshots of the overlapped adaptation chain (see _update_native): how many minibatches the policy chain
# may run ahead of it (LRL_ENC_SNAPSHOTS; 2 = double buffering)
_SNAPSHOTS = max(2, int(os.environ.get("LRL_ENC_SNAPSHOTS", "4")))


class PPO_Args(ArgsProto):
    value_loss_coef = 1.0
    use_clipped_value_loss = True
    clip_param = 0.2
    entropy_coef = 0.01
    num_learning_epochs = 5
    num_mini_batches = 4
    learning_rate = 1.e-3
    adaptation_module_learning_rate = 1.e-3
    num_adaptation_module_substeps = 1
    schedule = "adaptive"
    gamma = 0.99
    lam = 0.95
    desired_kl = 0.01
    max_grad_norm = 1.


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _collective():
    """Whether the update's collectives run: a world of more than one rank, or an initialised one-rank world with
    LRL_FORCE_COLLECTIVES=1 (a test switch: one GPU then exercises the RCCL calls themselves, each reducing over one
    rank; tests/test_rccl_world1_gpu.py)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or os.environ.get("LRL_FORCE_COLLECTIVES") == "1"


def _all_reduce_(t):
    """Sum ``t`` over the ranks, in place.  RCCL reduces device memory directly; gloo (the CPU / one-GPU rehearsals)
    reduces host memory, so a device tensor is staged through a synchronous host copy rather than gloo's own
    CUDA-tensor path (its side stream and pinned staging buffers are one more ordering to reason about) — every call
    site (gradients, KL, advantage statistics) goes the same way."""
    if t.is_cuda and dist.get_backend() == "gloo":
        host = t.cpu()
        dist.all_reduce(host)
        t.copy_(host)
    else:
        dist.all_reduce(t)
    return t


class PPO:
    actor_critic: ActorCritic

    def __init__(self, actor_critic, device="cpu", fused=None, seed=0):
        self.device = device
        self.actor_critic = actor_critic.to(device)
        self.storage = None
        self.optimizer = torch.optim.Adam(self.actor_critic.parameters(), lr=PPO_Args.learning_rate)
        self.adaptation_module_optimizer = torch.optim.Adam(self.actor_critic.parameters(),
                                                            lr=PPO_Args.adaptation_module_learning_rate)
        self.transition = RolloutStorage.Transition()
        self._lr = float(PPO_Args.learning_rate)
        self.async_losses = False
        self._lr_dev = None  # the native update's ctrl tensor while its learning rate is newer than self._lr
        self.fused = (torch.device(device).type == "cuda") if fused is None else fused
        # policy noise: counter RNG keyed by (seed, act counter, global env id); row_offset = the global id of storage row
        # 0 (the rank's env_offset, set by the Runner), so the draws do not depend on how envs are sharded over ranks
        self.seed = seed
        self.row_offset = 0
        self._act_counter = 0
        self._store = None
        self.grad_allreduce = _collective()
        self._native = None  # flat grads / Adam moments / ctrl / workspace of the native update
        self.record_lr = False  # native path: keep the per-minibatch learning rates (self.lr_trace)
        self.overlap_adaptation = True  # native path: adaptation phases on a second stream (see _update_native)
        self.lr_trace = []
        if self.fused:
            self.actor_critic.flatten_parameters()

    def init_storage(self, num_envs, num_transitions_per_env, actor_obs_shape, privileged_obs_shape, obs_history_shape,
                     action_shape):
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, actor_obs_shape, privileged_obs_shape,
                                      obs_history_shape, action_shape, self.device)
        self._store = self.storage.store_desc() if self.fused else None

    def test_mode(self):
        self.actor_critic.eval()

    def train_mode(self):
        self.actor_critic.train()

    def act(self, obs, privileged_obs, obs_history, eps=None):
        if self.fused:
            self._act_counter += 1
            a, mu, v, lp = self.actor_critic.act_fused(
                obs.contiguous(), privileged_obs.contiguous(), obs_history.contiguous(), eps=eps, seed=self.seed,
                counter=self._act_counter, store=self._store, store_row=self.storage.step,
                row_offset=self.row_offset)
            t = self.transition
            t.actions, t.values, t.actions_log_prob, t.action_mean = a, v, lp, mu
            t.action_sigma = self.actor_critic.std.detach().expand_as(mu)
            t.observations = t.critic_observations = obs
            t.privileged_observations, t.observation_histories = privileged_obs, obs_history
            return a
        t = self.transition
        t.actions = self.actor_critic.act(obs, privileged_obs).detach()
        t.values = self.actor_critic.evaluate(obs, privileged_obs).detach()
        t.actions_log_prob = self.actor_critic.get_actions_log_prob(t.actions).detach()
        t.action_mean = self.actor_critic.action_mean.detach()
        t.action_sigma = self.actor_critic.action_std.detach()
        t.observations = t.critic_observations = obs
        t.privileged_observations, t.observation_histories = privileged_obs, obs_history
        return t.actions

    def process_env_step(self, rewards, dones, infos):
        t = self.transition
        if self.fused and self._store_step(rewards, dones, infos):  # one launch for the three storage rows
            t.clear()
            self.actor_critic.reset(dones)
            return
        t.rewards = rewards.clone()
        t.dones = dones
        t.env_bins = infos["env_bins"]
        if "time_outs" in infos:  # bootstrapping on time outs (ppo.py:81-83)
            t.rewards += PPO_Args.gamma * torch.squeeze(t.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(t, fused=self.fused)
        t.clear()
        self.actor_critic.reset(dones)

    def _store_step(self, rewards, dones, infos):
        """process_env_step's rewards (+ the time-out bootstrap), dones and env bins into storage row `step` in one
        launch (lrl_ppo_store_step); False (the torch form runs) for inputs outside its dtypes / layouts."""
        s, t = self.storage, self.transition
        bins, tout = infos["env_bins"], infos.get("time_outs")
        n = s.num_envs
        ok = lambda x, dt: (x.dtype == dt and x.is_cuda and x.is_contiguous() and x.numel() == n)
        if not (ok(rewards, torch.float32) and ok(dones, torch.bool) and ok(bins, torch.float32)):
            return False
        if tout is not None and not (ok(tout, torch.bool) and ok(t.values, torch.float32)):
            return False
        if s.step >= s.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        i = s.step
        p = lambda x: C.c_void_p(x.data_ptr()) if x is not None else None
        stream = _abi.stream_of(rewards.device)
        _abi.check(_abi.lib().lrl_ppo_store_step(p(rewards), p(dones), p(bins), p(t.values if tout is not None else None),
                                                 p(tout), C.c_float(PPO_Args.gamma), C.c_int32(n), p(s.rewards[i]),
                                                 p(s.dones[i]), p(s.env_bins[i]), stream))
        s.step += 1
        return True

    def compute_returns(self, last_critic_obs, last_critic_privileged_obs):
        if self.fused:
            _, _, last_values, _ = self.actor_critic.act_fused(last_critic_obs.contiguous(),
                                                               last_critic_privileged_obs.contiguous(),
                                                               seed=self.seed, counter=0, row_offset=self.row_offset)
        else:
            last_values = self.actor_critic.evaluate(last_critic_obs, last_critic_privileged_obs).detach()
        reduce = None
        if _collective():
            reduce = _all_reduce_
        self.storage.compute_returns(last_values, PPO_Args.gamma, PPO_Args.lam, reduce_stats=reduce)

    def _allreduce_grads(self, params):
        grads = [p.grad for p in params if p.grad is not None]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        _all_reduce_(flat)
        flat /= _world()
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    # ---- native update (csrc/lrl_ppo.hip) ----
    def _native_state(self, batch):
        ac = self.actor_critic
        net = ac.flatten_parameters()
        st = self._native
        if st is None or st["net_ptr"] != ac._flat.data_ptr():
            dev = ac._flat.device
            st = dict(net=net, net_ptr=ac._flat.data_ptr(), grads=torch.zeros(net.total, device=dev),
                      exp_avg=torch.zeros(net.total, device=dev), exp_avg_sq=torch.zeros(net.total, device=dev),
                      ctrl=torch.zeros(_abi.PPO_CTRL_BYTES // 8, dtype=torch.float64, device=dev),
                      steps=[0, 0], ws=None, ws_batch=0)
            hp = _abi.LrlPpoHparams()
            _abi.fill(hp, clip_param=PPO_Args.clip_param, entropy_coef=PPO_Args.entropy_coef,
                      value_loss_coef=PPO_Args.value_loss_coef, max_grad_norm=PPO_Args.max_grad_norm,
                      desired_kl=PPO_Args.desired_kl if PPO_Args.desired_kl is not None else 0.0,
                      use_clipped_value_loss=int(PPO_Args.use_clipped_value_loss),
                      adaptive_schedule=int(PPO_Args.desired_kl is not None and PPO_Args.schedule == "adaptive"),
                      beta1=0.9, beta2=0.999, eps=1e-8)
            st["hp"] = hp
            self._native = st
        if st["ws_batch"] != batch:
            nbytes = _abi.lib().lrl_ppo_workspace_bytes(C.byref(net), C.c_int32(batch))
            if nbytes < 0:
                raise RuntimeError("lrl_ppo_workspace_bytes rejected the network")
            st["ws"] = torch.empty(nbytes, dtype=torch.uint8, device=ac._flat.device)
            # the adaptation phases run on their own stream with their own workspace (see _update_native)
            st["ws_b"] = torch.empty(nbytes, dtype=torch.uint8, device=ac._flat.device)
            st["ws_batch"] = batch
        return st

    @property
    def learning_rate(self):
        """The adaptive learning rate (ppo.py:126-133).  The native update keeps it on the device between updates (no
        host sync at the end of an update); reading it here fetches it."""
        if self._lr_dev is not None:
            self._lr = float(self._lr_dev[0].item())
            self._lr_dev = None
            for g in self.optimizer.param_groups:
                g["lr"] = self._lr
        return self._lr

    @learning_rate.setter
    def learning_rate(self, v):
        self._lr = float(v)
        self._lr_dev = None

    def _update_native(self, sync=True):
        s = self.storage
        T, N = s.num_transitions_per_env, s.num_envs
        nmb = PPO_Args.num_mini_batches
        mb = (T * N) // nmb
        st = self._native_state(mb)
        net, hp = st["net"], st["hp"]
        world = _world()
        coll = _collective()
        L = _abi.lib()
        ptr = lambda t: C.c_void_p(t.data_ptr())
        stream = _abi.stream_of(st["grads"].device)
        indices = torch.randperm(nmb * mb, requires_grad=False, device=self.device)
        trace = []
        flat = lambda t: t.flatten(0, 1)
        bufs = dict(obs=flat(s.observations), priv=flat(s.privileged_observations),
                    hist=flat(s.observation_histories), actions=flat(s.actions), values=flat(s.values),
                    returns=flat(s.returns), logp=flat(s.actions_log_prob), adv=flat(s.advantages), mu=flat(s.mu),
                    sigma=flat(s.sigma))
        for k, v in bufs.items():
            assert v.dtype == torch.float32 and (v.is_contiguous() or (k == "hist" and v.stride(1) == 1)), k
        batch = _abi.LrlPpoBatch()
        for k, v in bufs.items():
            setattr(batch, k, v.data_ptr())
        batch.batch = mb
        batch.hist_ld = bufs["hist"].stride(0)
        ctrl = st["ctrl"]
        if self._lr_dev is not ctrl:  # the host value is newer (first update, or set since): upload it
            ctrl[0] = self._lr
        ctrl[1:4] = 0.0
        params, grads, m, v, ws = self.actor_critic._flat, st["grads"], st["exp_avg"], st["exp_avg_sq"], st["ws"]
        main = grads[net.main_begin:net.kl_slot + 1]
        adapt = grads[net.adapt_begin:net.adapt_end]
        scale = 1.0 / world
        # The adaptation-module regression of minibatch i (phases 3 / 4) reads the encoder weights phase 2 of i wrote
        # and touches only the adaptation module's parameters, gradients and Adam moments, which phases 1 / 2 never
        # read or write.  So it runs on a second stream, overlapping phases 1 / 2 of the next minibatches (the GEMM
        # tails and small launches of one chain leave the CUs the other fills).  Its encoder target reads a snapshot
        # of the encoder weights copied right after phase 2 of i (a ring of _SNAPSHOTS buffers), so phase 2 of i + 1 may
        # overwrite the live ones without waiting for it; the copy for i + 2 waits until phase 3 of i has read its
        # buffer.  Each chain keeps its own launch order, so the result is bit-identical to the sequential order of
        # ppo.py:94-178.
        cur = torch.cuda.current_stream(params.device)
        if self.overlap_adaptation:
            sb = st.get("stream_b")
            if sb is None:
                sb = st["stream_b"] = torch.cuda.Stream(params.device)
            stream_b, ws_b = C.c_void_p(sb.cuda_stream), st["ws_b"]
            if "enc_snap" not in st:
                st["enc_snap"] = [torch.zeros(net.total, device=params.device) for _ in range(_SNAPSHOTS)]
            e0, e1 = net.e1w, net.std_off  # the encoder's weights and biases: one contiguous range
        else:
            sb, stream_b, ws_b = cur, stream, ws
        # the adaptation chain's batch descriptor: the rows pointer of minibatch i must outlive the next C call
        batch_b = _abi.LrlPpoBatch()
        C.memmove(C.byref(batch_b), C.byref(batch), C.sizeof(batch))
        # per snapshot buffer: phase 3 of the minibatch that last read it has run.  The events live as long as the native
        # state (re-recorded each update): an event destroyed while a wait on it is still queued on the GPU is a hazard
        # this code does not take (round-4 audit of the round-3 core dump)
        if sb is not cur and "read_done_ev" not in st:
            st["read_done_ev"] = [torch.cuda.Event() for _ in range(_SNAPSHOTS)]
        read_done = [None] * _SNAPSHOTS
        k = 0
        for epoch in range(PPO_Args.num_learning_epochs):
            for i in range(nmb):
                rows = indices[i * mb:(i + 1) * mb]
                batch.rows = rows.data_ptr()
                _abi.check(L.lrl_ppo_forward_backward(C.byref(net), ptr(params), ptr(grads), C.byref(batch),
                                                      C.byref(hp), ptr(ws), ptr(ctrl), stream))
                if coll:
                    _all_reduce_(main)
                st["steps"][0] += 1
                _abi.check(L.lrl_ppo_optimizer_step(C.byref(net), ptr(params), ptr(grads), ptr(m), ptr(v),
                                                    C.c_int64(st["steps"][0]), C.c_float(scale), C.byref(hp),
                                                    ptr(ws), ptr(ctrl), stream))
                if self.record_lr:
                    trace.append(ctrl[0].clone())
                enc = None
                if sb is not cur:
                    snap = st["enc_snap"][k % _SNAPSHOTS]
                    if read_done[k % _SNAPSHOTS] is not None:
                        cur.wait_event(read_done[k % _SNAPSHOTS])
                    snap[e0:e1].copy_(params[e0:e1])
                    enc = ptr(snap)
                    sb.wait_stream(cur)
                batch_b.rows = rows.data_ptr()
                for _ in range(PPO_Args.num_adaptation_module_substeps):
                    _abi.check(L.lrl_ppo_adaptation_forward_backward(C.byref(net), ptr(params), enc, ptr(grads),
                                                                     C.byref(batch_b), ptr(ws_b), ptr(ctrl), stream_b))
                    if coll:
                        with torch.cuda.stream(sb):
                            _all_reduce_(adapt)
                    st["steps"][1] += 1
                    _abi.check(L.lrl_ppo_adaptation_step(C.byref(net), ptr(params), ptr(grads), ptr(m), ptr(v),
                                                         C.c_int64(st["steps"][1]),
                                                         C.c_double(PPO_Args.adaptation_module_learning_rate),
                                                         C.c_float(scale), C.byref(hp), ptr(ctrl), stream_b))
                if sb is not cur:
                    ev = st["read_done_ev"][k % _SNAPSHOTS]
                    ev.record(sb)
                    read_done[k % _SNAPSHOTS] = ev
                k += 1
        if sb is not cur:
            cur.wait_stream(sb)
            indices.record_stream(sb)
        num_updates = PPO_Args.num_learning_epochs * nmb
        if self.record_lr:
            self.lr_trace = torch.stack(trace).tolist()
        self._lr_dev = ctrl  # the learning rate stays on the device (read lazily by .learning_rate)
        self.storage.clear()
        # the divisors are a cached device tensor: a torch.tensor(list, device=...) here is a pageable host -> device
        # copy, which waits for the whole update to finish and so keeps the host from enqueuing the next rollout
        den_key = (num_updates, PPO_Args.num_adaptation_module_substeps)
        if st.get("loss_den_key") != den_key:
            st["loss_den"] = torch.tensor([num_updates, num_updates, num_updates * den_key[1]], dtype=ctrl.dtype,
                                          device=ctrl.device)
            st["loss_den_key"] = den_key
        losses = ctrl[1:4] / st["loss_den"]
        if not sync:  # the runner's path: device scalars, converted when its logger summarises
            return tuple(losses.unbind(0))
        vsum, ssum, asum = losses.tolist()
        return vsum, ssum, asum

    def update(self):
        """PPO.update (ppo.py:94-178): mean value / surrogate / adaptation losses.  With ``async_losses`` set (the Runner
        sets it) they come back as device scalars, so the host does not wait for the update before enqueuing the next
        rollout; host floats otherwise."""
        if self.fused:
            return self._update_native(sync=not self.async_losses)
        mean_value_loss = torch.zeros((), device=self.device)
        mean_surrogate_loss = torch.zeros((), device=self.device)
        mean_adaptation_module_loss = torch.zeros((), device=self.device)
        ac = self.actor_critic
        params = list(ac.parameters())
        gen = self.storage.mini_batch_generator(PPO_Args.num_mini_batches, PPO_Args.num_learning_epochs)
        for (obs_b, critic_obs_b, priv_b, hist_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
             old_sigma_b, masks_b, env_bins_b) in gen:
            ac.act(obs_b, priv_b, masks=masks_b)
            logp_b = ac.get_actions_log_prob(actions_b)
            value_b = ac.evaluate(critic_obs_b, priv_b, masks=masks_b)
            mu_b, sigma_b, entropy_b = ac.action_mean, ac.action_std, ac.entropy
            if PPO_Args.desired_kl is not None and PPO_Args.schedule == "adaptive":
                with torch.inference_mode():
                    kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1.e-5) + (
                        torch.square(old_sigma_b) + torch.square(old_mu_b - mu_b)) / (2.0 * torch.square(sigma_b))
                        - 0.5, axis=-1)
                    kl_mean = torch.mean(kl)
                    if _collective():
                        kl_mean = _all_reduce_(kl_mean.clone())
                        kl_mean /= _world()
                    kl_mean = kl_mean.item()
                    if kl_mean > PPO_Args.desired_kl * 2.0:
                        self.learning_rate = max(1e-5, self.learning_rate / 1.5)
                    elif kl_mean < PPO_Args.desired_kl / 2.0 and kl_mean > 0.0:
                        self.learning_rate = min(1e-2, self.learning_rate * 1.5)
                    for g in self.optimizer.param_groups:
                        g["lr"] = self.learning_rate
            ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
            surrogate = -torch.squeeze(adv_b) * ratio
            surrogate_clipped = -torch.squeeze(adv_b) * torch.clamp(ratio, 1.0 - PPO_Args.clip_param,
                                                                   1.0 + PPO_Args.clip_param)
            surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
            if PPO_Args.use_clipped_value_loss:
                value_clipped = target_values_b + (value_b - target_values_b).clamp(-PPO_Args.clip_param,
                                                                                    PPO_Args.clip_param)
                value_loss = torch.max((value_b - returns_b).pow(2), (value_clipped - returns_b).pow(2)).mean()
            else:
                value_loss = (returns_b - value_b).pow(2).mean()
            loss = surrogate_loss + PPO_Args.value_loss_coef * value_loss - PPO_Args.entropy_coef * entropy_b.mean()
            self.optimizer.zero_grad()
            loss.backward()
            if self.grad_allreduce:
                self._allreduce_grads(params)
            nn.utils.clip_grad_norm_(params, PPO_Args.max_grad_norm)
            self.optimizer.step()
            mean_value_loss += value_loss.detach()
            mean_surrogate_loss += surrogate_loss.detach()
            for _ in range(PPO_Args.num_adaptation_module_substeps):
                adaptation_pred = ac.adaptation_module(hist_b)
                with torch.no_grad():
                    adaptation_target = ac.env_factor_encoder(priv_b)
                adaptation_loss = F.mse_loss(adaptation_pred, adaptation_target)
                self.adaptation_module_optimizer.zero_grad()
                adaptation_loss.backward()
                if self.grad_allreduce:
                    self._allreduce_grads(params)
                self.adaptation_module_optimizer.step()
                mean_adaptation_module_loss += adaptation_loss.detach()
        num_updates = PPO_Args.num_learning_epochs * PPO_Args.num_mini_batches
        out = torch.stack([mean_value_loss / num_updates, mean_surrogate_loss / num_updates,
                           mean_adaptation_module_loss / (num_updates * PPO_Args.num_adaptation_module_substeps)])
        self.storage.clear()
        mv, ms, ma = out.tolist()
        return mv, ms, ma
