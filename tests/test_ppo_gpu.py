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


@pytest.mark.parametrize("n", [37, 4096])
def test_fused_policy_act_matches_torch(n):
    from lrl.ppo.actor_critic import ActorCritic
    ac = ActorCritic(42, 18, 630, 12).cuda()
    init_params(ac)
    with torch.no_grad():
        ac.std.copy_(torch.linspace(0.5, 1.5, 12))
    g = torch.Generator(device="cuda:0").manual_seed(3)
    obs = torch.randn(n, 42, device="cuda:0", generator=g)
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
    lrs = []
    orig_step = alg.optimizer.step

    def step_rec(*a, **k):
        lrs.append(alg.learning_rate)
        return orig_step(*a, **k)
    alg.optimizer.step = step_rec
    perm = torch.as_tensor(g["perm"], device="cuda:0")
    orig = torch.randperm
    torch.randperm = lambda n, **kw: perm
    try:
        mv, ms, ma = alg.update()
    finally:
        torch.randperm = orig
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
