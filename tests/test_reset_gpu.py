"""reset_idx parity against the REFERENCE (tests/golden/reset.npz, made by running legged_robot.py's reset_idx
with injected torch.rand draws): the device part through ``lrl_sim_reset_idx_ex`` (DR redraw, dof / root reset,
buffer zeroing) and the host bookkeeping of ``LeggedRobotEnv.reset_idx`` (uniform command curriculum, grid
curriculum resampling, episode logging, extras), for

* mc_fork  — Mini Cheetah preset on its flat trimesh: the fork's Q4, roots untouched;
* go1_fork — Go1 preset on the plane: roots to base_init_state + env origin;
* go1_up   — upstream semantics (legacy_fork=False) with custom origins: the U[x_init_range, y_init_range] spawn
             draw with unequal ranges (Q8), init offsets, _resample_commands and the yaw curriculum.

Integers, masks and every state value bit-exact; the episode means (a float32 reduction whose order differs
between torch on the CPU and the GPU) within 1e-6 relative.
"""
import numpy as np
import pytest
import torch

from helpers import golden

pytestmark = pytest.mark.gpu

CASES = {"mc_fork": ("mc", True), "go1_fork": ("go1", True), "go1_up": ("go1", False)}


def _env(case, n):
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    robot, fork = CASES[case]
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    cfg.env.num_envs = n
    if case == "go1_up":
        cfg.terrain.mesh_type = "trimesh"
        cfg.terrain.x_init_range, cfg.terrain.y_init_range = -0.5, 0.75
        cfg.terrain.x_init_offset, cfg.terrain.y_init_offset = 0.25, -0.125
        cfg.commands.yaw_command_curriculum = True
    return LeggedRobotEnv("cuda:0", cfg=cfg, legacy_fork=fork)


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda:0")


@pytest.mark.parametrize("case", list(CASES))
def test_reset_idx_matches_reference(case):
    g = golden("reset.npz")
    f = lambda k: g[f"{case}/{k}"]
    n = f("in_root").shape[0]
    env = _env(case, n)
    try:
        env.root_states.copy_(_t(f("in_root")))
        env.dof_pos.copy_(_t(f("in_dof_pos")))
        env.dof_vel.copy_(_t(f("in_dof_vel")))
        env.env_origins.copy_(_t(f("in_env_origins")))
        env.last_actions.copy_(_t(f("in_last_actions")))
        env.last_dof_vel.copy_(_t(f("in_last_dof_vel")))
        env.feet_air_time.copy_(_t(f("in_feet_air_time")))
        env.episode_length_buf.copy_(_t(f("in_episode_length"), torch.int32))
        env._time_out_u8.copy_(_t(f("in_time_out"), torch.uint8))
        env._reset_u8.zero_()
        env.commands.copy_(_t(f("in_commands")))
        env._episode_sums.copy_(_t(f("in_episode_sums")))
        env._command_sums.copy_(_t(f("in_command_sums")))
        env.motor_strengths.copy_(_t(f("in_motor_strengths")))
        env.env_command_bins[:] = f("in_env_command_bins")
        np.testing.assert_array_equal(env.curriculum.weights, f("in_weights"))  # same seed-100 curriculum
        env.common_step_counter = int(f("common_step_counter"))
        ids = torch.as_tensor(f("ids"), device="cuda:0")
        env.reset_uniforms = _t(f("u"))
        env.reset_idx(ids)
        torch.cuda.synchronize()
        npy = lambda t: t.detach().cpu().numpy()
        eq = np.testing.assert_array_equal
        eq(npy(env.root_states), f("root"))
        eq(npy(env.dof_pos), f("dof_pos"))
        eq(npy(env.dof_vel), f("dof_vel"))
        eq(npy(env.motor_strengths), f("motor_strengths"))
        eq(npy(env.last_actions), f("last_actions"))
        eq(npy(env.last_dof_vel), f("last_dof_vel"))
        eq(npy(env.feet_air_time), f("feet_air_time"))
        eq(npy(env.episode_length_buf), f("episode_length"))
        eq(npy(env._reset_u8), f("reset"))
        eq(npy(env.commands), f("commands"))
        eq(npy(env._episode_sums), f("episode_sums"))
        eq(npy(env._command_sums), f("command_sums"))
        eq(env.env_command_bins, f("env_command_bins"))
        eq(env.curriculum.weights, f("weights"))
        eq(npy(env.extras["env_bins"]), f("env_bins"))
        eq(npy(env.extras["time_outs"]).astype(np.uint8), f("time_outs"))
        ep = env.extras["train/episode"]
        assert sorted(ep) == list(f("ep_keys"))
        got = np.array([float(ep[k]) for k in f("ep_keys")])
        np.testing.assert_allclose(got, f("ep_values"), rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(np.array(env.cfg.command_ranges["lin_vel_x"], np.float64), f("lin_vel_x"))
        np.testing.assert_array_equal(np.array(env.cfg.command_ranges["ang_vel_yaw"], np.float64), f("ang_vel_yaw"))
    finally:
        env.close()


def test_caller_written_episode_length_resamples_the_right_envs():
    """with legacy_fork=False a caller that writes episode_length_buf between steps (upstream's
    init_at_random_ep_len) must get commands resampled for the envs due under the NEW lengths, the host bins
    included.  Checked against a host replay of the same curriculum calls."""
    import copy
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    cfg = lcfg.make_cfg()
    lcfg.config_go1(cfg)
    cfg.env.num_envs = 64
    env = LeggedRobotEnv("cuda:0", cfg=cfg, legacy_fork=False)  # plane: standing robots do not terminate
    try:
        interval = int(env.cfg.commands.resampling_time / env.dt)
        zero = torch.zeros(64, 12, device="cuda:0")
        env.reset()
        env.step(zero)
        torch.cuda.synchronize()
        # lengths such that exactly envs 5..12 reach the resampling interval in the next step
        eplen = torch.full((64,), 3, dtype=torch.int32, device="cuda:0")
        eplen[5:13] = interval - 1
        env.episode_length_buf.copy_(eplen)
        cur = copy.deepcopy(env.curriculum)
        bins0 = env.env_command_bins.copy()
        sums = env._command_sums[env._track_rows].cpu().numpy()
        cmd0 = env.commands.cpu().numpy()
        env.step(zero)
        torch.cuda.synchronize()
        assert not env._reset_u8.any(), "an env terminated: the replay below assumes no resets"
        due = np.arange(5, 13)
        timesteps = int(env.cfg.commands.resampling_time / env.dt)
        ep_len = min(env.cfg.env.max_episode_length, timesteps)
        lin, ang = sums[:, due] / np.float32(ep_len)
        thr_l = env.cfg.commands.forward_curriculum_threshold * env.reward_scales["tracking_lin_vel"]
        thr_a = env.cfg.commands.yaw_curriculum_threshold * env.reward_scales["tracking_ang_vel"]
        cur.update(bins0[due], lin, ang, thr_l, thr_a, local_range=0.5)
        cmds, bins = cur.sample(batch_size=len(due))
        want_bins = bins0.copy()
        want_bins[due] = bins
        np.testing.assert_array_equal(env.env_command_bins, want_bins)
        c = cmds.astype(np.float32)
        keep = (np.sqrt(c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]) > np.float32(0.2)).astype(np.float32)
        c[:, :2] *= keep[:, None]
        got = env.commands.cpu().numpy()
        np.testing.assert_array_equal(got[due, :3], c)
        others = np.setdiff1d(np.arange(64), due)
        np.testing.assert_array_equal(got[others], cmd0[others])
    finally:
        env.close()
