"""The collective call sites of the native update under an RCCL world, on the CPU with
a mocked torch.distributed and a mocked liblrl: per optimiser step exactly one all-reduce of the flat policy gradient
(its KL slot included — the adaptive learning rate's all-reduced KL mean rides in it), one of the adaptation
module's gradient per adaptation substep, and one of the advantage statistics per iteration; nothing else.
(ppo.py:94-178 / rollout_storage.py:76-90 of the reference run on one device; this is the data-parallel form.)"""
import ctypes as C
import os
import sys
import types

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))


class _FakeLib:
    def lrl_ppo_workspace_bytes(self, *a):
        return 1024

    def __getattr__(self, name):
        return lambda *a: 0


def _fake_dist(world, calls):
    def all_reduce(t, *a, **k):
        calls.append(t)
        return None
    return types.SimpleNamespace(is_available=lambda: True, is_initialized=lambda: True,
                                 get_world_size=lambda: world, get_backend=lambda: "nccl", all_reduce=all_reduce,
                                 ReduceOp=types.SimpleNamespace(SUM=0, MAX=1))


@pytest.mark.parametrize("substeps", [1, 2])
def test_native_update_issues_one_flat_gradient_allreduce_per_optimizer_step(monkeypatch, substeps):
    from lrl import _abi
    from lrl.ppo import ppo as P
    from lrl.ppo.actor_critic import ActorCritic
    calls = []
    monkeypatch.setattr(P, "dist", _fake_dist(2, calls))
    monkeypatch.setattr(_abi, "lib", lambda: _FakeLib())
    monkeypatch.setattr(_abi, "stream_of", lambda dev: C.c_void_p(0))
    cur = object()
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: cur)
    monkeypatch.setattr(P.PPO_Args, "num_adaptation_module_substeps", substeps)
    ac = ActorCritic(42, 18, 630, 12)
    alg = P.PPO(ac, device="cpu", fused=True)
    assert alg.grad_allreduce
    alg.overlap_adaptation = False
    alg.init_storage(64, 24, [42], [18], [630], [12])
    alg.storage.step = 24
    alg.update()
    net = alg._native["net"]
    grads = alg._native["grads"]
    steps = P.PPO_Args.num_learning_epochs * P.PPO_Args.num_mini_batches
    main = [t for t in calls if t.numel() == net.kl_slot + 1 - net.main_begin]
    adapt = [t for t in calls if t.numel() == net.adapt_end - net.adapt_begin]
    assert len(calls) == steps * (1 + substeps), [t.numel() for t in calls]
    assert len(main) == steps and len(adapt) == steps * substeps
    for t in main:  # in place on the flat gradient buffer (no gather / scatter copies), the KL slot last
        assert t.data_ptr() == grads.data_ptr() + 4 * net.main_begin
    for t in adapt:
        assert t.data_ptr() == grads.data_ptr() + 4 * net.adapt_begin


def test_advantage_statistics_are_one_allreduce_per_iteration(monkeypatch):
    """compute_returns normalises the advantages with (sum, sum of squares, count) all-reduced once over the ranks."""
    from lrl import _abi
    from lrl.ppo import ppo as P
    from lrl.ppo.actor_critic import ActorCritic
    calls = []
    monkeypatch.setattr(P, "dist", _fake_dist(2, calls))
    monkeypatch.setattr(_abi, "lib", lambda: _FakeLib())
    monkeypatch.setattr(_abi, "stream_of", lambda dev: C.c_void_p(0))
    ac = ActorCritic(42, 18, 630, 12)
    alg = P.PPO(ac, device="cpu", fused=False)
    alg.init_storage(16, 24, [42], [18], [630], [12])
    s = alg.storage
    g = torch.Generator().manual_seed(0)
    s.values.copy_(torch.randn(s.values.shape, generator=g))
    s.rewards.copy_(torch.randn(s.rewards.shape, generator=g))
    s.step = 24
    alg.compute_returns(torch.zeros(16, 42), torch.zeros(16, 18))
    assert len(calls) == 1 and calls[0].numel() == 3, [t.shape for t in calls]
