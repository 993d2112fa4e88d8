"""CPU checks of the oracle's joint-limit rows: with the limits on, joints driven into their URDF
limits stop there; with them off (params.joint_limits = 0) the same drive carries them past.  The GPU parity of
the kernel's rows against these is tests/test_env_gpu.py::test_joint_limits_match_oracle."""
import numpy as np
import pytest

from helpers import make
from lrl import _abi
from oracle import oracle


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_oracle_joint_limits_hold(robot):
    n = 8
    out = {}
    for on in (1, 0):
        cfg, rob, M, P = make(robot, **{"env.num_envs": n})
        P.joint_limits = on
        P.self_collisions = 0  # (the alternating limit poses fold legs into the base box: the limits alone here)
        lo, hi = np.array(M.dof_lower[:], np.float32), np.array(M.dof_upper[:], np.float32)
        st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
        st["root"][:] = 0
        st["root"][:, 2] = 0.6  # airborne: only the drive and the limits act on the joints
        st["root"][:, 6] = 1
        st["dof_pos"][:] = np.where(np.arange(12) % 2 == 0, hi - 0.05, lo + 0.05)
        st["dof_vel"][:] = np.where(np.arange(12) % 2 == 0, 2.0, -2.0)
        scale = np.full(12, P.action_scale, np.float32)
        scale[0::3] *= P.hip_scale_reduction
        default = np.array(P.default_dof_pos[:], np.float32)
        beyond = np.where(np.arange(12) % 2 == 0, hi + 0.5, lo - 0.5)
        act = np.broadcast_to(np.clip((beyond - default) / scale, -P.clip_actions, P.clip_actions),
                              (n, 12)).astype(np.float32).copy()
        for s in range(10):
            oracle.env_step(M, P, st, act, _abi.STEP_PHYSICS, common_step_counter=s + 1)
        out[on] = np.maximum(st["dof_pos"] - hi, lo - st["dof_pos"]).max()
    assert out[1] < 1e-3, out  # held at the limit
    assert out[0] > 0.05, out  # the same drive crosses it without the rows


def test_oracle_narrow_joint_range_holds_when_the_nearer_limit_switches():
    """A joint range narrower than 2 (margin + 2 dt |qd|) puts both limits inside the detection window: the nearer
    limit (sigma) can switch between sub-steps while the row stays active.  The carried impulse is stored with its
    sigma and a switched row starts cold, so the joint is held inside the range instead of being pushed
    out by the previous limit's impulse."""
    n = 4
    cfg, rob, M, P = make("mc", **{"env.num_envs": n})
    P.self_collisions = 0
    default = np.array(P.default_dof_pos[:], np.float32)
    lo = np.array(M.dof_lower[:], np.float32)
    hi = np.array(M.dof_upper[:], np.float32)
    j = 1  # front-right thigh
    lo[j], hi[j] = default[j] - 0.004, default[j] + 0.004
    for k in range(12):
        M.dof_lower[k], M.dof_upper[k] = float(lo[k]), float(hi[k])
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    st["root"][:, 2] = 0.6
    st["dof_pos"][:] = default
    st["dof_vel"][:] = 0.0
    st["dof_vel"][:, j] = np.array([4.0, -4.0, 8.0, -8.0], np.float32)
    act = np.zeros((n, 12), np.float32)
    for s in range(5):
        oracle.env_step(M, P, st, act, _abi.STEP_PHYSICS, common_step_counter=s + 1)
        assert np.isfinite(st["dof_pos"]).all()
        over = np.maximum(st["dof_pos"][:, j] - hi[j], lo[j] - st["dof_pos"][:, j]).max()
        assert over < 0.01, (s, over)
