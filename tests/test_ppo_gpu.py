"""GPU parity of the PPO numeric core: GAE kernel vs the reference's golden vectors, fused rollout
policy kernel vs a plain torch fp32 forward of the same ActorCritic."""
import zlib

import numpy as np
import pytest
import torch

from helpers import golden
from lrl import _abi

pytestmark = pytest.mark.gpu


def init_params(module):
    """Same deterministic init as tests/golden/make_golden.py::init_params."""
    with torch.no_grad():
        for name, p in module.named_parameters():
            r = np.random.default_rng(zlib.crc32(name.encode()))
            fan_in = p.shape[-1] if p.dim() > 1 else 1
            scale = 1.0 / np.sqrt(fan_in) if p.dim() > 1 else 0.05
            if name == "std":
                p.copy_(torch.ones_like(p))
            else:
                p.copy_(torch.tensor(r.uniform(-1, 1, tuple(p.shape)) * scale, dtype=torch.float))


def test_gae_matches_reference():
    import ctypes as C
    g = golden("gae.npz")
    T, N = g["rewards"].shape[:2]
    d = lambda a, dt=torch.float32: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device="cuda:0")
    rew, val, done = d(g["rewards"]), d(g["values"]), d(g["dones"], torch.uint8)
    last = d(g["last_values"])
    ret, adv = torch.empty_like(rew), torch.empty_like(rew)
    ws = torch.empty(4096, device="cuda:0")
    p = lambda t: C.c_void_p(t.data_ptr())
    _abi.check(_abi.lib().lrl_gae(p(rew), p(done), p(val), p(last), C.c_int32(T), C.c_int32(N), C.c_float(0.99),
                                  C.c_float(0.95), p(ret), p(adv), p(ws),
                                  C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    np.testing.assert_allclose(ret.cpu().numpy(), g["returns"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(adv.cpu().numpy(), g["advantages"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,no", [(37, 42), (4096, 42), (300, 235)])
def test_fused_policy_act_matches_torch(n, no):
    """no = 235: the base config's perceptive policy (observe_vel + 17 x 11 height scan, X pitch 256)."""
    from lrl.ppo.actor_critic import ActorCritic
    ac = ActorCritic(no, 18, 15 * no, 12).cuda()
    init_params(ac)
    with torch.no_grad():
        ac.std.copy_(torch.linspace(0.5, 1.5, 12))
    g = torch.Generator(device="cuda:0").manual_seed(3)
    obs = torch.randn(n, no, device="cuda:0", generator=g)
    priv = torch.randn(n, 18, device="cuda:0", generator=g)
    eps = torch.randn(n, 12, device="cuda:0", generator=g)
    a, mu, v, lp = ac.act_fused(obs, priv, eps=eps)
    with torch.no_grad():
        ac.update_distribution(obs, priv)
        mu_ref = ac.action_mean
        a_ref = mu_ref + ac.action_std * eps
        lp_ref = ac.get_actions_log_prob(a_ref)
        v_ref = ac.evaluate(obs, priv)
    # fp32 MFMA (k-ordered fma chain) vs torch/hipBLASLt fp32 GEMMs: 1e-4 relative on O(1) outputs
    torch.testing.assert_close(mu, mu_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(a, a_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(v, v_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lp, lp_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n,no", [(4096, 42), (37, 42), (300, 235)])
def test_one_launch_act_matches_gemm_chain(n, no, monkeypatch):
    """The one-launch act (act_fused_kernel: fp32 MFMA, activations in LDS) against the GEMM-chain act
    (LRL_ACT_FUSED=0: x6 products + act_head_kernel) on the same inputs, noise drawn by the counter RNG: actions, means,
    values, log-probs to fp32 rounding; the storage row (obs / priv / history copies, sigma) exactly."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.rollout_storage import RolloutStorage
    ac = ActorCritic(no, 18, 15 * no, 12).cuda()
    init_params(ac)
    with torch.no_grad():
        ac.std.copy_(torch.linspace(0.5, 1.5, 12))
    g = torch.Generator(device="cuda:0").manual_seed(5)
    obs = torch.randn(n, no, device="cuda:0", generator=g)
    priv = torch.randn(n, 18, device="cuda:0", generator=g)
    hist = torch.randn(n, 15 * no, device="cuda:0", generator=g)
    outs = []
    for fused in ("1", "0"):  # (LRL_ACT_FUSED=1 selects the one-launch act)
        monkeypatch.setenv("LRL_ACT_FUSED", fused)
        st = RolloutStorage(n, 3, [no], [18], [15 * no], [12], "cuda:0")
        res = ac.act_fused(obs, priv, hist, seed=11, counter=3, store=st.store_desc(), store_row=1, row_offset=64)
        torch.cuda.synchronize()
        outs.append([r.clone() for r in res] + [st.observations[1].clone(), st.privileged_observations[1].clone(),
                                                st.observation_histories[1].clone(), st.actions[1].clone(),
                                                st.sigma[1].clone(), st.mu[1].clone(), st.values[1].clone(),
                                                st.actions_log_prob[1].clone()])
    (a, mu, v, lp, so, sp, sh, sa, ss, sm, sv, sl), (a0, mu0, v0, lp0, so0, sp0, sh0, sa0, ss0, sm0, sv0, sl0) = outs
    torch.testing.assert_close(mu, mu0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(a, a0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(v, v0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(lp, lp0, rtol=2e-5, atol=2e-4)
    assert torch.equal(a - mu, a0 - mu0) or torch.allclose(a - mu, a0 - mu0, rtol=0, atol=1e-6)  # the same noise
    for x, y in ((so, so0), (sp, sp0), (sh, sh0), (ss, ss0)):
        assert torch.equal(x, y)
    assert torch.equal(sa, a) and torch.equal(sm, mu) and torch.equal(sv.flatten(), v.flatten())
    assert torch.equal(sl.flatten(), lp.flatten())


@pytest.mark.parametrize("n,no", [(4096, 42), (37, 42), (300, 235)])
def test_act_fused_encoder_matches_encoder_chain(n, no, monkeypatch):
    """The GEMM-chain act's first launch (act_fused_kernel<., true>: the obs rows and the env-factor encoder's three
    layers in one workgroup per 16 rows, fp32 MFMA) against the prep kernel + three x6 / fp32 products it replaces
    (LRL_ACT_ENC_FUSED=0): actions, means, values, log-probs to fp32 rounding, the same noise, the storage row exactly."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.rollout_storage import RolloutStorage
    monkeypatch.setenv("LRL_ACT_FUSED", "0")
    ac = ActorCritic(no, 18, 15 * no, 12).cuda()
    init_params(ac)
    g = torch.Generator(device="cuda:0").manual_seed(13)
    obs = torch.randn(n, no, device="cuda:0", generator=g)
    priv = torch.randn(n, 18, device="cuda:0", generator=g)
    hist = torch.randn(n, 15 * no, device="cuda:0", generator=g)
    outs = []
    for enc in ("1", "0"):
        monkeypatch.setenv("LRL_ACT_ENC_FUSED", enc)
        st = RolloutStorage(n, 2, [no], [18], [15 * no], [12], "cuda:0")
        res = ac.act_fused(obs, priv, hist, seed=5, counter=4, store=st.store_desc(), store_row=0)
        torch.cuda.synchronize()
        outs.append([r.clone() for r in res] + [st.observations[0].clone(), st.privileged_observations[0].clone()])
    (a, mu, v, lp, so, sp), (a0, mu0, v0, lp0, so0, sp0) = outs
    torch.testing.assert_close(mu, mu0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(a, a0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(v, v0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(lp, lp0, rtol=2e-5, atol=2e-4)
    assert torch.allclose(a - mu, a0 - mu0, rtol=0, atol=1e-6)  # the same noise
    assert torch.equal(so, so0) and torch.equal(sp, sp0)


@pytest.mark.parametrize("n", [4096, 1000])
def test_act_with_weight_planes_is_bit_identical(n, monkeypatch):
    """The act's GEMM chain with its weight products on the pre-split-planes kernel (LRL_ACT_PLANES=1, gemm_x6p_kernel
    where the shapes fit) gives the same bits as without (gemm_x6_kernel): actions, means, values, log-probs."""
    from lrl.ppo.actor_critic import ActorCritic
    monkeypatch.setenv("LRL_ACT_FUSED", "0")
    ac = ActorCritic(42, 18, 630, 12).cuda()
    init_params(ac)
    g = torch.Generator(device="cuda:0").manual_seed(9)
    obs = torch.randn(n, 42, device="cuda:0", generator=g)
    priv = torch.randn(n, 18, device="cuda:0", generator=g)
    outs = []
    for planes in ("1", "0"):
        monkeypatch.setenv("LRL_ACT_PLANES", planes)
        res = ac.act_fused(obs, priv, seed=3, counter=2)
        torch.cuda.synchronize()
        outs.append([r.clone() for r in res])
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_fused_policy_sampling_statistics():
    """Counter-RNG Box-Muller sampling: actions - mu ~ N(0, std^2)."""
    from lrl.ppo.actor_critic import ActorCritic
    ac = ActorCritic(42, 18, 630, 12).cuda()
    init_params(ac)
    n = 8192
    obs = torch.zeros(n, 42, device="cuda:0")
    priv = torch.zeros(n, 18, device="cuda:0")
    a, mu, v, lp = ac.act_fused(obs, priv, seed=7, counter=1)
    z = (a - mu).cpu().numpy()
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1.0) < 0.02
    a2, _, _, _ = ac.act_fused(obs, priv, seed=7, counter=2)
    assert not torch.equal(a, a2)


def test_ppo_rollout_gae_update_match_reference():
    """PPO.act (fused kernel) -> process_env_step -> compute_returns (HIP GAE) -> update, against the
    reference's PPO run on the same weights / inputs / noise / permutation (tests/golden/ppo_update.npz)."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO
    g = golden("ppo_update.npz")
    T, N = g["eps"].shape[:2]
    ac = ActorCritic(42, 18, 630, 12)
    init_params(ac)
    alg = PPO(ac.cuda(), device="cuda:0")
    alg.init_storage(N, T, [42], [18], [630], [12])
    d = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda:0")
    with torch.inference_mode():
        for t in range(T):
            a = alg.act(d(g["obs_seq"][t]), d(g["priv_seq"][t]), d(g["hist_seq"][t]), eps=d(g["eps"][t]))
            np.testing.assert_allclose(a.cpu().numpy(), g["actions"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(alg.transition.values.cpu().numpy(), g["values"][t], rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(alg.transition.actions_log_prob.cpu().numpy(), g["logp"][t], rtol=1e-4,
                                       atol=2e-4)
            alg.process_env_step(d(g["rew"][t]), d(g["done"][t]).bool(), {"env_bins": torch.zeros(N, device="cuda:0")})
        alg.compute_returns(d(g["obs_seq"][T]), d(g["priv_seq"][T]))
    np.testing.assert_allclose(alg.storage.returns.cpu().numpy(), g["returns"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(alg.storage.advantages.cpu().numpy(), g["advantages"], rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(alg.storage.observation_histories.cpu().numpy(), g["hist_seq"][:T])
    assert alg.storage.observation_histories.stride(1) == 640  # padded pitch; the padding stays zero
    assert not alg.storage._hist_padded[..., 630:].any()
    alg.record_lr = True
    perm = torch.as_tensor(g["perm"], device="cuda:0")
    orig = torch.randperm
    torch.randperm = lambda n, **kw: perm
    try:
        mv, ms, ma = alg.update()
    finally:
        torch.randperm = orig
    lrs = alg.lr_trace  # learning rate used by each of the 20 PPO optimiser steps (device-side schedule)
    np.testing.assert_allclose(lrs, g["lrs"], rtol=1e-9)
    np.testing.assert_allclose([mv, ms, ma], [g["mean_value_loss"], g["mean_surrogate_loss"],
                                              g["mean_adaptation_loss"]], rtol=2e-3, atol=1e-5)
    params = dict(ac.named_parameters())
    names = [str(x) for x in g["param_names"]]
    sums = np.array([params[k].detach().double().sum().item() for k in names])
    np.testing.assert_allclose(sums, g["param_sums"], rtol=2e-3, atol=2e-3)
    heads = np.stack([np.pad(params[k].detach().cpu().numpy().ravel()[:16], (0, max(0, 16 - params[k].numel())))
                      for k in names])
    np.testing.assert_allclose(heads, g["param_head"], rtol=2e-3, atol=1e-4)


@pytest.mark.parametrize("N,T", [(512, 24), (4096, 24)])
def test_native_update_matches_torch_autograd(N, T):
    """The native update (csrc/lrl_ppo.hip: GEMMs + head kernels + device-side LR/clip/Adam) against the
    torch-autograd restatement (fused=False) on the same rollout storage and permutation, at the
    benchmark's minibatch size (4096 envs x 24 steps / 4 = 24,576 rows) and a smaller one."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO
    torch.manual_seed(0)
    algs = []
    for fused in (True, False):
        ac = ActorCritic(42, 18, 630, 12)
        init_params(ac)
        alg = PPO(ac.cuda(), device="cuda:0", fused=fused)
        alg.init_storage(N, T, [42], [18], [630], [12])
        algs.append(alg)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    st0 = algs[0].storage
    with torch.no_grad():
        for name in ("observations", "privileged_observations", "observation_histories", "actions", "mu"):
            getattr(st0, name).copy_(torch.randn(getattr(st0, name).shape, device="cuda:0", generator=g))
        st0.sigma.fill_(1.0)
        st0.values.copy_(torch.randn(st0.values.shape, device="cuda:0", generator=g))
        st0.returns.copy_(st0.values + 0.3 * torch.randn(st0.values.shape, device="cuda:0", generator=g))
        a = torch.randn(st0.advantages.shape, device="cuda:0", generator=g)
        st0.advantages.copy_((a - a.mean()) / a.std())
        # old log-probs near the current policy's so the ratio straddles the clip range
        st0.actions_log_prob.copy_(-11.0 + torch.randn(st0.values.shape, device="cuda:0", generator=g))
        for name in ("observations", "privileged_observations", "observation_histories", "actions", "mu", "sigma",
                     "values", "returns", "advantages", "actions_log_prob"):
            getattr(algs[1].storage, name).copy_(getattr(st0, name))
    perm = torch.randperm(N * T, device="cuda:0")
    orig = torch.randperm
    torch.randperm = lambda n, **kw: perm
    try:
        out = [alg.update() for alg in algs]
    finally:
        torch.randperm = orig
    assert algs[0].learning_rate == algs[1].learning_rate
    np.testing.assert_allclose(out[0], out[1], rtol=2e-3, atol=1e-5)
    p0 = dict(algs[0].actor_critic.named_parameters())
    for k, v in algs[1].actor_critic.named_parameters():
        d = (p0[k].detach() - v.detach()).abs().max().item()
        assert d <= 2e-3 * (v.detach().abs().max().item() + 1e-2), (k, d)


def test_overlapped_adaptation_phases_are_bit_identical():
    """The native update runs the adaptation-module regression (phases 3 / 4) of minibatch i on a second stream,
    overlapping phases 1 / 2 of minibatch i + 1 (ppo.py _update_native); each chain keeps its launch order, so every
    parameter, Adam moment, learning rate and loss equals the sequential single-stream update bit for bit — at the
    benchmark's minibatch (4096 envs x 24 steps / 4)."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO
    N, T = 4096, 24
    algs = []
    for overlap in (True, False):
        torch.manual_seed(0)
        ac = ActorCritic(42, 18, 630, 12)
        init_params(ac)
        alg = PPO(ac.cuda(), device="cuda:0", fused=True)
        alg.overlap_adaptation = overlap
        alg.init_storage(N, T, [42], [18], [630], [12])
        algs.append(alg)
    perm = torch.randperm(N * T, device="cuda:0")
    orig = torch.randperm
    torch.randperm = lambda n, **kw: perm
    try:
        outs = []
        for alg in algs:
            o = []
            for it in range(2):  # two iterations: the second starts from Adam state the first left
                _random_storage(alg, N, T, seed=1 + it)
                o.append(alg.update())
            outs.append(o)
    finally:
        torch.randperm = orig
    assert outs[0] == outs[1]
    assert algs[0].learning_rate == algs[1].learning_rate
    assert torch.equal(algs[0].actor_critic._flat, algs[1].actor_critic._flat)
    for k in ("exp_avg", "exp_avg_sq"):
        assert torch.equal(algs[0]._native[k], algs[1]._native[k]), k


def _random_storage(alg, N, T, seed=1):
    st = alg.storage
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    with torch.no_grad():
        for name in ("observations", "privileged_observations", "observation_histories", "actions", "mu"):
            getattr(st, name).copy_(torch.randn(getattr(st, name).shape, device="cuda:0", generator=g))
        st.sigma.fill_(1.0)
        st.values.copy_(torch.randn(st.values.shape, device="cuda:0", generator=g))
        st.returns.copy_(st.values + 0.3 * torch.randn(st.values.shape, device="cuda:0", generator=g))
        a = torch.randn(st.advantages.shape, device="cuda:0", generator=g)
        st.advantages.copy_((a - a.mean()) / a.std())
        st.actions_log_prob.copy_(-11.0 + torch.randn(st.values.shape, device="cuda:0", generator=g))


@pytest.mark.parametrize("padded_hist,no", [(True, 42), (False, 42), (True, 235)])
def test_native_minibatch_gradients_match_autograd(padded_hist, no):
    """One minibatch of lrl_ppo_forward_backward / lrl_ppo_adaptation_forward_backward against torch
    autograd of the reference's loss (ppo.py:98-147, 157-166): every parameter's gradient, the KL mean,
    the losses.  History rows either at the storage's padded pitch (640: the float4 / zero-k-padding
    path of the adaptation module's first layer) or packed (630)."""
    import ctypes as C
    import torch.nn.functional as F
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO, PPO_Args
    N, T = 256, 24
    nh = 15 * no
    ac = ActorCritic(no, 18, nh, 12)
    init_params(ac)
    alg = PPO(ac.cuda(), device="cuda:0", fused=True)
    alg.init_storage(N, T, [no], [18], [nh], [12])
    _random_storage(alg, N, T)
    mb = N * T // 4
    rows = torch.randperm(N * T, device="cuda:0")[:mb].contiguous()
    nst = alg._native_state(mb)
    net, hp, grads, ctrl, ws = nst["net"], nst["hp"], nst["grads"], nst["ctrl"], nst["ws"]
    s = alg.storage
    fl = lambda t: t.flatten(0, 1)
    batch = _abi.LrlPpoBatch()
    for k, t in dict(obs=s.observations, priv=s.privileged_observations, hist=s.observation_histories,
                     actions=s.actions, values=s.values, returns=s.returns, logp=s.actions_log_prob,
                     adv=s.advantages, mu=s.mu, sigma=s.sigma).items():
        setattr(batch, k, fl(t).data_ptr())
    batch.rows, batch.batch = rows.data_ptr(), mb
    hist_flat = fl(s.observation_histories)
    if not padded_hist:
        hist_flat = hist_flat.contiguous()
        batch.hist = hist_flat.data_ptr()
    assert hist_flat.stride(0) == ((nh + 15) // 16 * 16 if padded_hist else nh)
    batch.hist_ld = hist_flat.stride(0)
    p = lambda t: C.c_void_p(t.data_ptr())
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = _abi.lib()
    _abi.check(L.lrl_ppo_forward_backward(C.byref(net), p(ac._flat), p(grads), C.byref(batch), C.byref(hp), p(ws),
                                          p(ctrl), stream))
    _abi.check(L.lrl_ppo_adaptation_forward_backward(C.byref(net), p(ac._flat), None, p(grads), C.byref(batch),
                                                     p(ws), p(ctrl), stream))
    torch.cuda.synchronize()
    mbf = ctrl.view(torch.float32)[8:12].tolist()  # value, surrogate, adaptation, (kl in grads)
    kl_native = grads[net.kl_slot].item()
    # torch autograd on the same minibatch
    obs, priv, hist = fl(s.observations)[rows], fl(s.privileged_observations)[rows], fl(s.observation_histories)[rows]
    act, tv, ret = fl(s.actions)[rows], fl(s.values)[rows], fl(s.returns)[rows]
    oldlp, adv, omu, osig = fl(s.actions_log_prob)[rows], fl(s.advantages)[rows], fl(s.mu)[rows], fl(s.sigma)[rows]
    ac.zero_grad(set_to_none=True)
    ac.act(obs, priv)
    logp = ac.get_actions_log_prob(act)
    value = ac.evaluate(obs, priv)
    mu, sigma, ent = ac.action_mean, ac.action_std, ac.entropy
    with torch.no_grad():
        kl = torch.sum(torch.log(sigma / osig + 1.e-5) + (torch.square(osig) + torch.square(omu - mu)) /
                       (2.0 * torch.square(sigma)) - 0.5, axis=-1).mean().item()
    ratio = torch.exp(logp - torch.squeeze(oldlp))
    surr = torch.max(-torch.squeeze(adv) * ratio,
                     -torch.squeeze(adv) * torch.clamp(ratio, 1 - PPO_Args.clip_param, 1 + PPO_Args.clip_param)).mean()
    vc = tv + (value - tv).clamp(-PPO_Args.clip_param, PPO_Args.clip_param)
    vl = torch.max((value - ret).pow(2), (vc - ret).pow(2)).mean()
    loss = surr + vl - PPO_Args.entropy_coef * ent.mean()
    loss.backward()
    pred = ac.adaptation_module(hist)
    with torch.no_grad():
        target = ac.env_factor_encoder(priv)
    al = F.mse_loss(pred, target)
    al.backward()
    np.testing.assert_allclose(kl_native, kl, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(mbf[:3], [vl.item(), surr.item(), al.item()], rtol=1e-4, atol=1e-7)
    fg = grads.cpu()
    bad = []
    for name, prm in ac.named_parameters():
        off = (prm.data_ptr() - ac._flat.data_ptr()) // 4
        got = fg[off:off + prm.numel()].view_as(prm)
        ref = prm.grad.cpu()
        err = (got - ref).abs().max().item()
        if err > 1e-4 * (ref.abs().max().item() + 1e-6) + 1e-7:
            bad.append(f"{name}: err {err:.3g} ref max {ref.abs().max().item():.3g} got max {got.abs().max().item():.3g}")
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("with_timeouts", [False, True])
def test_fused_store_step_matches_torch_form(with_timeouts):
    """PPO.process_env_step on the native path (one lrl_ppo_store_step launch) writes exactly what the reference's
    torch form writes (ppo.py:76-88, rollout_storage.py:57-71): rewards plus the time-out bootstrap
    gamma * V * time_out, dones, env bins."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO
    N, T = 1000, 3
    g = torch.Generator(device="cuda:0").manual_seed(4)
    outs = []
    for fused in (True, False):
        alg = PPO(ActorCritic(42, 18, 630, 12).cuda(), device="cuda:0", fused=True)
        alg.init_storage(N, T, [42], [18], [630], [12])
        if not fused:
            alg._store_step = lambda *a: False
        g.manual_seed(4)
        for _ in range(T):
            alg.transition.values = torch.randn(N, 1, device="cuda:0", generator=g)
            rew = torch.randn(N, device="cuda:0", generator=g)
            dones = torch.rand(N, device="cuda:0", generator=g) < 0.3
            infos = {"env_bins": torch.randint(0, 5202, (N,), device="cuda:0", generator=g).float()}
            tout = torch.rand(N, device="cuda:0", generator=g) < 0.5
            if with_timeouts:
                infos["time_outs"] = tout
            alg.transition.observations = None
            alg.process_env_step(rew, dones, infos)
        s = alg.storage
        assert s.step == T
        outs.append([s.rewards.clone(), s.dones.clone(), s.env_bins.clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
