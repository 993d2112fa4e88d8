"""Checkpoint compatibility: the reference run's trained ac_weights_last.pt
(35-key state dict incl. the duplicate encoder.* registration, actor_critic.py:46-110) loads strictly into
this ActorCritic and reproduces the reference's teacher / student / value outputs
(tests/golden/checkpoint_last.npz, made by tests/golden/make_golden.py from the reference itself)."""
import json
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN, golden


def _trained():
    from lrl.ppo.actor_critic import ActorCritic
    g = golden("checkpoint_last.npz")
    sd = {k: torch.from_numpy(g["sd/" + k]) for k in g["keys"]}
    ac = ActorCritic(42, 18, 630, 12)
    ac.load_state_dict(sd, strict=True)
    return ac, g


def test_state_dict_layout_matches_reference():
    from lrl.ppo.actor_critic import ActorCritic
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))
    ours = [[k, list(v.shape)] for k, v in ActorCritic(42, 18, 630, 12).state_dict().items()]
    assert ours == ref
    assert sum(p.numel() for p in ActorCritic(42, 18, 630, 12).parameters()) == 603037


def test_trained_checkpoint_outputs_match_reference():
    ac, g = _trained()
    obs, priv, hist = (torch.from_numpy(g[k]) for k in ("obs", "priv", "hist"))
    with torch.no_grad():
        ti, si = {}, {}
        np.testing.assert_allclose(ac.act_teacher(obs, priv, ti).numpy(), g["mean_teacher"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ac.act_student(obs, hist, si).numpy(), g["mean_student"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ac.evaluate(obs, priv).numpy(), g["value"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ti["latents"], g["latent_teacher"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(si["latents"], g["latent_student"], rtol=1e-5, atol=1e-5)
    # the flat-buffer layout the native kernels use survives load_state_dict (views, not copies)
    ac.flatten_parameters()
    sd = {k: torch.from_numpy(g["sd/" + k]) for k in g["keys"]}
    ac.load_state_dict(sd, strict=True)
    assert ac.std.data_ptr() == ac._flat.data_ptr() + 4 * ac._net.std_off
    with torch.no_grad():
        np.testing.assert_allclose(ac.act_teacher(obs, priv).numpy(), g["mean_teacher"], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_trained_checkpoint_fused_act_matches_reference():
    """Native rollout act (lrl_ppo_act) and native student act (lrl_ppo_act_student) on the trained
    weights: mean actions, values and latents against the reference's outputs."""
    ac, g = _trained()
    ac = ac.cuda()
    d = lambda k: torch.from_numpy(g[k]).cuda()
    eps = torch.zeros(64, 12, device="cuda:0")
    actions, mu, values, logp = ac.act_fused(d("obs"), d("priv"), eps=eps)
    np.testing.assert_allclose(mu.cpu().numpy(), g["mean_teacher"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(actions.cpu().numpy(), g["mean_teacher"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(values.cpu().numpy(), g["value"], rtol=1e-4, atol=1e-4)
    mean_s, lat_s = ac.act_student_fused(d("obs"), d("hist"))
    np.testing.assert_allclose(mean_s.cpu().numpy(), g["mean_student"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(lat_s.cpu().numpy(), g["latent_student"], rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_trained_policy_walks_in_this_physics():
    """Sim-to-sim evidence for the physics model (PhysX parity is unpinned): the reference run's
    policy, trained in Isaac Gym / PhysX, driven through act_inference on this simulator (scripts/play.py), tracks
    a 1 m/s forward command and stays upright.  Measured on MI355X: 0.92 m/s mean over 64 envs, all upright
    (profiles/r1_play_trained_policy_mc.png); the test bars are 0.75-1.1 m/s and >= 95 % upright."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import play
    vel, upright, dt = play.play("mc", None, num_envs=64, steps=300, vx=1.0)
    vx = vel[150:, :, 0].mean()
    assert 0.75 < vx < 1.1, vx
    assert upright >= 0.95, upright


def test_learn_saves_after_the_loop(tmp_path):
    """The reference saves after the iteration loop whatever save_interval is (mini_gym_learn/ppo/__init__.py:
    246-265): learn(3) with save_interval 400 leaves ac_weights_000002.pt, ac_weights_last.pt and both TorchScript
    exports (iteration 0 is also a save_interval iteration, as in the reference).  CPU env: the oracle's build."""
    from oracle.cpu_env import CpuVecEnv, cpu_compute_returns
    from lrl.ppo import runner as R
    env = CpuVecEnv(16, threads=1)
    runner = R.Runner(env, device="cpu", seed=3, logger=R.Logger(str(tmp_path)))
    runner.alg.storage.compute_returns = cpu_compute_returns(runner.alg.storage)
    runner.learn(3)
    ck = tmp_path / "checkpoints"
    names = sorted(p.name for p in ck.iterdir())
    assert names == ["ac_weights_000000.pt", "ac_weights_000002.pt", "ac_weights_last.pt",
                     "adaptation_module_latest.jit", "body_latest.jit"], names
    last = torch.load(ck / "ac_weights_last.pt", weights_only=True)
    for k, v in runner.alg.actor_critic.state_dict().items():
        assert torch.equal(last[k], v.cpu()), k
    assert runner.current_learning_iteration == 3


def test_runner_save_torchscript_export_reproduces_student(tmp_path):
    """Runner.save (mini_gym_learn/ppo/__init__.py:220-242): the state dict plus TorchScript exports of the
    adaptation module and the actor body, the pair the reference's deployment loads (play scripts: latent =
    adaptation_module(history), action = body(cat(obs, latent))).  Reloaded from disk, the exports of the trained
    checkpoint reproduce the reference's student means."""
    import types
    from lrl.ppo.runner import Logger, Runner
    ac, g = _trained()
    fake = types.SimpleNamespace(logger=Logger(str(tmp_path)), alg=types.SimpleNamespace(actor_critic=ac))
    Runner.save(fake, 7)
    ck = tmp_path / "checkpoints"
    assert (ck / "ac_weights_000007.pt").exists() and (ck / "ac_weights_last.pt").exists()
    sd = torch.load(ck / "ac_weights_last.pt", weights_only=True)
    assert list(sd) == list(ac.state_dict())
    adapt = torch.jit.load(str(ck / "adaptation_module_latest.jit"))
    body = torch.jit.load(str(ck / "body_latest.jit"))
    obs, hist = torch.from_numpy(g["obs"]), torch.from_numpy(g["hist"])
    with torch.no_grad():
        mean = body(torch.cat((obs, adapt(hist)), dim=-1))
    np.testing.assert_allclose(mean.numpy(), g["mean_student"], rtol=1e-5, atol=1e-5)
