"""Pin the CPU oracle against golden vectors produced by running the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from helpers import POST_PHYSICS, golden, make
from oracle import oracle
from lrl import _abi
from lrl import params as lparams


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_derived_constants_match_reference(robot):
    g = golden(f"post_physics_{robot}.npz")
    cfg, rob, M, P = make(robot)
    keys, scales = lparams.reward_layout(cfg)
    assert keys == [str(k) for k in g["reward_names"]]
    np.testing.assert_allclose([scales[k] for k in keys], g["reward_scales"], rtol=0, atol=0)
    np.testing.assert_array_equal(lparams.noise_vec(cfg), g["noise_scale_vec"])
    lim = g["dof_pos_limits"]
    np.testing.assert_array_equal(np.array(P.soft_dof_pos_lower[:], np.float32), lim[:, 0])
    np.testing.assert_array_equal(np.array(P.soft_dof_pos_upper[:], np.float32), lim[:, 1])
    assert P.rand_interval == int(g["rand_interval"]) == 301
    assert P.max_episode_length == int(g["max_episode_length"]) == 1001
    assert float(np.float32(g["dt"])) == P.dt


def _state_from_golden(g, cfg, M, P):
    n = g["root_in"].shape[1]
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    st["friction"][:] = g["init_friction"]
    st["restitution"][:] = g["init_restitution"]
    st["payload"][:] = g["init_payload"]
    st["com"][:] = g["init_com"]
    st["motor_strength"][:] = g["init_motor_strengths"]
    st["episode_length"][:] = g["init_episode_length"]
    st["episode_sums"][:] = g["init_episode_sums"]
    st["command_sums"][:] = g["init_command_sums"]
    st["feet_air_time"][:] = g["init_feet_air_time"]
    st["last_contacts"][:] = g["init_last_contacts"]
    st["last_actions"][:] = g["init_last_actions"]
    st["last_dof_vel"][:] = g["init_last_dof_vel"]
    return st


@pytest.mark.parametrize("case", list(POST_PHYSICS))
def test_oracle_post_physics_matches_reference(case):
    """LeggedRobot.step with identity physics: torques, obs, priv-obs, rewards, sums, termination,
    teleport and DR redraw, 3 consecutive steps (stateful feet_air_time / last_*)."""
    robot, fixture, over = POST_PHYSICS[case]
    g = golden(fixture)
    cfg, rob, M, P = make(robot, **over)
    keys = lparams.reward_layout(cfg)[0]
    assert [k for k in keys if k != "termination"] == [str(k) for k in g["reward_names"]]
    assert keys + ["total"] == [str(k) for k in g["episode_sum_keys"]]
    st = _state_from_golden(g, cfg, M, P)
    flags = _abi.STEP_INJECT_UNIFORM
    for s in range(g["root_in"].shape[0]):
        st["root"][:] = g["root_in"][s]
        st["dof_pos"][:] = g["dof_pos_in"][s]
        st["dof_vel"][:] = g["dof_vel_in"][s]
        st["contact"][:] = g["contact_in"][s]
        st["commands"][:] = g["commands"][s]
        push_u = np.nan_to_num(g["push_u"][s]) if "push_u" in g.files else None
        oracle.env_step(M, P, st, g["actions"][s], flags, noise_u=g["noise_u"][s], dr_u=g["ms_u"][s], push_u=push_u)
        tight = dict(rtol=2e-6, atol=2e-6)
        np.testing.assert_array_equal(st["torques"], g["torques"][s])
        np.testing.assert_array_equal(st["joint_pos_target"], g["joint_pos_target"][s])
        np.testing.assert_allclose(st["base_lin_vel"], g["base_lin_vel"][s], **tight)
        np.testing.assert_allclose(st["base_ang_vel"], g["base_ang_vel"][s], **tight)
        np.testing.assert_allclose(st["projected_gravity"], g["projected_gravity"][s], **tight)
        np.testing.assert_array_equal(st["root"], g["root_out"][s])  # teleport
        np.testing.assert_array_equal(st["motor_strength"], g["motor_strengths"][s])
        np.testing.assert_array_equal(st["reset"], g["reset"][s])
        np.testing.assert_array_equal(st["episode_length"], g["episode_length"][s])
        np.testing.assert_array_equal(st["last_contacts"].astype(bool), g["last_contacts"][s])
        np.testing.assert_allclose(st["feet_air_time"], g["feet_air_time"][s], **tight)
        np.testing.assert_allclose(st["rew"], g["rew"][s], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(st["episode_sums"], g["episode_sums"][s], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(st["command_sums"], g["command_sums"][s], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(st["obs"], g["obs"][s], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(st["priv"], g["priv"][s], rtol=1e-6, atol=1e-6)


def test_oracle_gae_matches_reference():
    g = golden("gae.npz")
    ret, adv = oracle.gae(g["rewards"], g["dones"], g["values"], g["last_values"], 0.99, 0.95)
    np.testing.assert_allclose(ret, g["returns"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(adv, g["advantages"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case,robot,mode", [("mc_fork", "mc", 0), ("go1_fork", "go1", 1), ("go1_up", "go1", 2)])
def test_reset_device_part_matches_reference(case, robot, mode):
    """oracle.reset_idx_device against the reference's reset_idx (reset.npz): DR redraw, dof and root reset (the
    fork's Q4 for custom origins, the plane path, the upstream spawn draw over unequal init ranges), zeroing."""
    g = golden("reset.npz")
    f = lambda k: g[f"{case}/{k}"]
    over = {}
    if case == "go1_up":
        over = {"terrain.mesh_type": "trimesh", "terrain.x_init_range": -0.5, "terrain.y_init_range": 0.75,
                "terrain.x_init_offset": 0.25, "terrain.y_init_offset": -0.125}
    cfg, rob, M, P = make(robot, **over)
    n = f("in_root").shape[0]
    st = {"root": f("in_root").copy(), "dof_pos": f("in_dof_pos").copy(), "dof_vel": f("in_dof_vel").copy(),
          "env_origins": f("in_env_origins"), "last_actions": f("in_last_actions").copy(),
          "last_dof_vel": f("in_last_dof_vel").copy(), "feet_air_time": f("in_feet_air_time").copy(),
          "episode_length": f("in_episode_length").astype(np.int32), "reset": np.zeros(n, np.uint8),
          "motor_strength": f("in_motor_strengths").copy(), "kp": np.ones((n, 12), np.float32),
          "kd": np.ones((n, 12), np.float32)}
    t = cfg.terrain
    oracle.reset_idx_device(P, st, f("ids"), f("u"), mode, float(t.x_init_range),
                            float(t.y_init_range) - float(t.x_init_range), float(t.x_init_offset), float(t.y_init_offset))
    for k, ref in (("root", "root"), ("dof_pos", "dof_pos"), ("dof_vel", "dof_vel"),
                   ("motor_strength", "motor_strengths"), ("last_actions", "last_actions"),
                   ("last_dof_vel", "last_dof_vel"), ("feet_air_time", "feet_air_time"),
                   ("episode_length", "episode_length"), ("reset", "reset")):
        np.testing.assert_array_equal(st[k], f(ref), err_msg=k)
