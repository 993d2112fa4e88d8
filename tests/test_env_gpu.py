"""GPU parity of the fused env step (liblrl.so on cuda:0).

* post-physics bookkeeping vs the REFERENCE (golden vectors from running legged_robot.py itself,
  identity physics, injected uniforms): torques, obs, priv-obs, rewards, sums, termination,
  teleport, DR redraw — 3 consecutive steps, Mini Cheetah and Go1.
* physics vs the CPU oracle (dense double-precision restatement of the same model): one env step
  (4 sub-steps) from many states, fp32 tolerance stated below.
* multi-step behaviour: a standing robot settles with foot forces carrying its weight.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from helpers import (MAX_EXCLUDED, POST_PHYSICS, ROBOT_FILES, SEP_EPS_1, VEL_EPS, golden, make, oracle_sensitivity,
                     perturb_state, physics_mismatch, record_errors)
from lrl import _abi
from lrl import config as lcfg
from lrl.robot import load_robot
from oracle import oracle

pytestmark = pytest.mark.gpu


def _cfg(robot, n, **over):
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    cfg.env.num_envs = n
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    return cfg


def _env(robot, n, **over):
    from lrl.env import LeggedRobotEnv
    return LeggedRobotEnv("cuda:0", cfg=_cfg(robot, n, **over))


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda:0")


def _step_raw(env, actions, flags, noise=None, dr=None):
    L = _abi.lib()
    if noise is not None:
        env._inj = (noise, dr)  # keep alive
        _abi.check(L.lrl_sim_inject_uniforms(env._sim, C.c_void_p(noise.data_ptr()), C.c_void_p(dr.data_ptr())))
    _abi.check(L.lrl_sim_step(env._sim, C.c_void_p(actions.data_ptr()), C.c_uint32(flags), env._stream()))
    torch.cuda.synchronize()


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("case", list(POST_PHYSICS))
def test_post_physics_matches_reference(case):
    robot, fixture, over = POST_PHYSICS[case]
    g = golden(fixture)
    n = g["root_in"].shape[1]
    env = _env(robot, n, **over)
    assert env.reward_names == [str(k) for k in g["reward_names"]]
    env.friction_coeffs[:] = _dev(g["init_friction"])
    env.restitutions[:] = _dev(g["init_restitution"])
    env.payloads[:] = _dev(g["init_payload"])
    env.com_displacements[:] = _dev(g["init_com"])
    env.motor_strengths[:] = _dev(g["init_motor_strengths"])
    env.Kp_factors[:] = 1.0
    env.Kd_factors[:] = 1.0
    env.episode_length_buf[:] = _dev(g["init_episode_length"], torch.int32)
    env._episode_sums[:] = _dev(g["init_episode_sums"])
    env._command_sums[:] = _dev(g["init_command_sums"])
    env.feet_air_time[:] = _dev(g["init_feet_air_time"])
    env._last_contacts_u8[:] = _dev(g["init_last_contacts"], torch.uint8)
    env.last_actions[:] = _dev(g["init_last_actions"])
    env.last_dof_vel[:] = _dev(g["init_last_dof_vel"])
    for s in range(g["root_in"].shape[0]):
        env.root_states[:] = _dev(g["root_in"][s])
        env.dof_pos[:] = _dev(g["dof_pos_in"][s])
        env.dof_vel[:] = _dev(g["dof_vel_in"][s])
        env.contact_forces[:] = _dev(g["contact_in"][s])
        env.commands[:] = _dev(g["commands"][s])
        act = _dev(g["actions"][s])
        noise = _dev(g["noise_u"][s])
        dr = _dev(np.nan_to_num(g["ms_u"][s]))
        if "push_u" in g.files:  # _push_robots draws (NaN rows: envs not pushed in this step)
            env._inj_push = _dev(np.nan_to_num(g["push_u"][s]))
            _abi.check(_abi.lib().lrl_sim_inject_push_uniforms(env._sim, C.c_void_p(env._inj_push.data_ptr())))
        _step_raw(env, act, _abi.STEP_INJECT_UNIFORM, noise, dr)
        np.testing.assert_array_equal(_np(env.torques), g["torques"][s])
        np.testing.assert_array_equal(_np(env.joint_pos_target), g["joint_pos_target"][s])
        np.testing.assert_array_equal(_np(env.root_states), g["root_out"][s])
        np.testing.assert_array_equal(_np(env.motor_strengths), g["motor_strengths"][s])
        np.testing.assert_array_equal(_np(env._reset_u8), g["reset"][s])
        np.testing.assert_array_equal(_np(env.episode_length_buf), g["episode_length"][s])
        np.testing.assert_array_equal(_np(env.last_contacts), g["last_contacts"][s])
        tol = dict(rtol=2e-6, atol=2e-6)
        np.testing.assert_allclose(_np(env.base_lin_vel), g["base_lin_vel"][s], **tol)
        np.testing.assert_allclose(_np(env.base_ang_vel), g["base_ang_vel"][s], **tol)
        np.testing.assert_allclose(_np(env.projected_gravity), g["projected_gravity"][s], **tol)
        np.testing.assert_allclose(_np(env.feet_air_time), g["feet_air_time"][s], **tol)
        np.testing.assert_allclose(_np(env.rew_buf), g["rew"][s], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(_np(env._episode_sums), g["episode_sums"][s], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(_np(env._command_sums), g["command_sums"][s], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(_np(env.obs_buf), g["obs"][s], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(_np(env.privileged_obs_buf), g["priv"][s], rtol=1e-6, atol=1e-6)
    env.close()


def _random_states(rng, n, P, robot):
    """A mix of standing, perturbed, airborne and fallen robots."""
    root = np.zeros((n, 13), np.float32)
    root[:, 0:2] = rng.uniform(10, 60, (n, 2))
    root[:, 2] = rng.uniform(0.24, 0.34, n)
    ang = rng.normal(size=(n, 3)) * 0.15
    th = np.linalg.norm(ang, axis=1, keepdims=True)
    q = np.concatenate([ang / np.maximum(th, 1e-9) * np.sin(th / 2), np.cos(th / 2)], 1)
    root[:, 3:7] = q
    root[:, 7:10] = rng.normal(size=(n, 3)) * 0.3
    root[:, 10:13] = rng.normal(size=(n, 3)) * 0.5
    k = n // 4
    root[:k, 2] = 0.6  # airborne
    root[k:2 * k, 2] = 0.08  # fallen / lying
    dof = np.array(P.default_dof_pos[:], np.float32)[None] + rng.normal(size=(n, 12)).astype(np.float32) * 0.2
    dofv = rng.normal(size=(n, 12)).astype(np.float32)
    return root, dof, dofv


def _limit_states(rng, n, P, M, root, dof, dofv):
    """Joints placed at or just past their URDF limits (lrl_model dof_lower / dof_upper), moving into them, with
    position targets beyond them: every env drives about half of its joints into a limit."""
    lo, hi = np.array(M.dof_lower[:], np.float32), np.array(M.dof_upper[:], np.float32)
    pick = rng.random((n, 12)) < 0.5
    upper = rng.random((n, 12)) < 0.5
    off = rng.uniform(-0.03, 0.08, (n, 12)).astype(np.float32)
    dof = np.where(pick, np.where(upper, hi - off, lo + off), dof).astype(np.float32)
    dofv = np.where(pick, np.where(upper, 1.0, -1.0) * rng.uniform(0.0, 6.0, (n, 12)), dofv).astype(np.float32)
    # action pushing the target past the limit: target = a * action_scale (x hip reduction) + default
    scale = np.full(12, P.action_scale, np.float32)
    scale[0::3] *= P.hip_scale_reduction
    default = np.array(P.default_dof_pos[:], np.float32)
    beyond = np.where(upper, hi + 0.4, lo - 0.4)
    act = np.where(pick, np.clip((beyond - default) / scale, -P.clip_actions, P.clip_actions), 0).astype(np.float32)
    return dof, dofv, act, pick


def _self_states(rng, n, M, root, dof):
    """Joint angles uniform inside the URDF limits, kept when no candidate pair overlaps by more than 5 mm (a deeper
    start is a violent Baumgarte push-out, chaotic over ten steps) and filled so that half of the envs start within
    the contact offset of a self-contact (legs folded into each other or into the base box); half of the robots
    airborne."""
    lo, hi = np.array(M.dof_lower[:], np.float32), np.array(M.dof_upper[:], np.float32)
    near, far = [], []
    while len(near) < n // 2 or len(far) < n - n // 2:
        q = rng.uniform(lo + 0.05, hi - 0.05, 12).astype(np.float32)
        m = oracle.self_pairs(M, q)[1].min()
        if m < -0.005:
            continue
        (near if m < 0.01 else far).append(q)
    dof = np.stack(near[: n // 2] + far[: n - n // 2])[rng.permutation(n)]
    root = root.copy()
    root[: n // 2, 2] = 0.8
    return root, dof


def _lying_states(rng, n, P):
    """Robots on their sides (roll +-90 deg with noise, any yaw), base just clear of the plane, legs spread: the legs of
    the lower side lie along the ground, so the ab/ad, thigh and calf colliders (support tables on the plane, not
    just the feet) are in contact."""
    root = np.zeros((n, 13), np.float32)
    root[:, 0:2] = rng.uniform(10, 60, (n, 2))
    root[:, 2] = rng.uniform(0.10, 0.14, n)
    roll = np.where(rng.random(n) < 0.5, 1.0, -1.0) * (np.pi / 2 + rng.normal(size=n) * 0.2)
    pitch, yaw = rng.normal(size=n) * 0.2, rng.uniform(-np.pi, np.pi, n)
    cr, sr, cp, sp, cy, sy = (np.cos(roll / 2), np.sin(roll / 2), np.cos(pitch / 2), np.sin(pitch / 2), np.cos(yaw / 2),
                              np.sin(yaw / 2))
    root[:, 3:7] = np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
                             cr * cp * cy + sr * sp * sy], 1)
    root[:, 7:10] = rng.normal(size=(n, 3)) * 0.1
    root[:, 10:13] = rng.normal(size=(n, 3)) * 0.2
    dof = np.array(P.default_dof_pos[:], np.float32)[None] + rng.normal(size=(n, 12)).astype(np.float32) * 0.3
    dofv = rng.normal(size=(n, 12)).astype(np.float32) * 0.5
    return root, dof, dofv


def _physics_vs_oracle(robot, n, steps, limits=False, selfc=False, self_on=True, extra=None, lying=False):
    """Kernel vs oracle physics over ``steps`` env steps, re-synchronised: before every step the oracle's state
    (root, joint positions / rates) is written into the sim, so each step is compared from identical inputs — the
    DR values, motor-strength redraws, pushes and injected draws are the same on both sides anyway.  Per step: every
    env within helpers.within_tolerance except the envs the oracle puts on a contact-model discontinuity (a sphere
    within SEP_EPS_1 of contact_offset, a restitution switch within VEL_EPS) or whose fp64 result itself moves under
    fp32-size input noise; those are counted and capped at MAX_EXCLUDED of the envs per step."""
    over = {} if self_on else {"asset.self_collisions": 1}
    over.update(extra or {})
    cfg, rob, M, P = make(robot, **{"env.num_envs": n}, **over)
    env = _env(robot, n, **over)
    assert P.self_collisions == int(self_on) and env._P.self_collisions == int(self_on)  # presets: asset.self_collisions 0
    assert env._P.solver_tgs == P.solver_tgs == int(cfg.sim.physx.solver_type == 1)  # presets: solver_type 1 (TGS)
    rng = np.random.default_rng(5 + steps + (100 if limits else 0) + (200 if selfc else 0) + (300 if lying else 0))
    root, dof, dofv = _random_states(rng, n, P, robot)
    if lying:
        root, dof, dofv = _lying_states(rng, n, P)
    act_lim = None
    if limits:
        dof, dofv, act_lim, picked = _limit_states(rng, n, P, M, root, dof, dofv)
    if selfc:
        root, dof = _self_states(rng, n, M, root, dof)
        # position targets at the start pose (+ small noise): legs held pressed into their self-contacts
        scale = np.full(12, P.action_scale, np.float32)
        scale[0::3] *= P.hip_scale_reduction
        hold = np.clip((dof - np.array(P.default_dof_pos[:], np.float32)) / scale, -P.clip_actions, P.clip_actions)
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    fr = rng.uniform(0.05, 4.5, n).astype(np.float32)
    rs = rng.uniform(0, 1, n).astype(np.float32)
    pl = rng.uniform(-1, 3, n).astype(np.float32)
    com = rng.uniform(-0.1, 0.1, (n, 3)).astype(np.float32)
    for k, v in dict(root=root, dof_pos=dof, dof_vel=dofv, friction=fr, restitution=rs, payload=pl, com=com).items():
        st[k][:] = v
    env.friction_coeffs[:] = _dev(fr)
    env.restitutions[:] = _dev(rs)
    env.payloads[:] = _dev(pl)
    env.com_displacements[:] = _dev(com)
    flags = _abi.STEP_PHYSICS | _abi.STEP_INJECT_UNIFORM
    rng_p = np.random.default_rng(77)
    B = M.num_bodies
    tmask = np.array([(P.termination_mask >> b) & 1 for b in range(B)], bool)
    worst = 0.0
    for s in range(steps):
        env.root_states[:] = _dev(st["root"])  # re-synchronise: this step starts from the oracle's state
        env.dof_pos[:] = _dev(st["dof_pos"])
        env.dof_vel[:] = _dev(st["dof_vel"])
        act = (rng.normal(size=(n, 12)) * 0.5).astype(np.float32)
        if selfc:
            act = (hold + rng.normal(size=(n, 12)) * 0.05).astype(np.float32)
        if act_lim is not None:
            act = np.where(picked, act_lim, act).astype(np.float32)
        noise = rng.random((n, P.num_obs)).astype(np.float32)
        dr = rng.random(n).astype(np.float32)
        pu = None
        if P.push_robots:  # _push_robots draws of the envs pushed in this step (both sides read the same rows)
            pu = rng.random((n, 2)).astype(np.float32)
            env._inj_push = _dev(pu)
            _abi.check(_abi.lib().lrl_sim_inject_push_uniforms(env._sim, C.c_void_p(env._inj_push.data_ptr())))
        _step_raw(env, _dev(act), flags, _dev(noise), _dev(dr))
        # the oracle's own conditioning: the same step from two fp32-rounding-size perturbations of the same start (one
        # draw misses envs whose spread is wide but lopsided: a lying Mini Cheetah under TGS with 63 of 64 perturbed
        # replays outside tolerance passed the single draw, scripts/tgs_probe.py)
        st_p = perturb_state(st, rng_p)
        st_q = perturb_state(st, rng_p)
        m = np.zeros((n, 2))
        oracle.env_step(M, P, st, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1, margins=m, push_u=pu)
        oracle.env_step(M, P, st_p, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1, push_u=pu)
        oracle.env_step(M, P, st_q, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1, push_u=pu)
        got = {k: _np(getattr(env, a)) for k, a in dict(root="root_states", dof_pos="dof_pos", dof_vel="dof_vel",
                                                          contact="contact_forces", obs="obs_buf").items()}
        assert np.isfinite(got["root"]).all() and np.isfinite(got["dof_vel"]).all()
        sens = oracle_sensitivity(st, st_p) | oracle_sensitivity(st, st_q)
        bad, excl = physics_mismatch(got, st, m, sens, sep_eps=SEP_EPS_1)
        record_errors(f"{robot} n={n} step {s + 1}/{steps} limits={limits} self={selfc} extra={sorted(over)}", got, st,
                      excl, st_p)
        worst = max(worst, excl.mean())
        print(f"{robot} n={n} step {s + 1}/{steps} limits={limits} self={selfc}: {excl.sum()} of {n} envs excluded "
              f"(discontinuity margin {((m[:, 0] < SEP_EPS_1) | (m[:, 1] < VEL_EPS)).sum()}, oracle-sensitive "
              f"{sens.sum()}), {bad.sum()} outside tolerance")
        for e in np.flatnonzero(bad)[:4]:  # per-field errors of the first bad envs (diagnostics)
            errs = {k: float(np.abs(got[k][e] - st[k][e]).max()) for k in ("root", "dof_pos", "dof_vel", "contact")}
            print("bad env", e, errs, "margins", m[e], "sens", sens[e])
        assert bad.sum() == 0, (s, np.flatnonzero(bad)[:16])
        assert excl.mean() <= MAX_EXCLUDED, (s, excl.mean())
        # termination (check_termination, legged_robot.py:190-202): the kernel's flag is exactly its own force test,
        # and equals the oracle's wherever the oracle's termination-body force is not within 5 % of the 1 N threshold
        own = (np.linalg.norm(got["contact"][:, tmask], axis=-1) > 1.0).any(axis=1)
        np.testing.assert_array_equal(_np(env._reset_u8).astype(bool), own)
        fmax = np.linalg.norm(st["contact"][:, tmask], axis=-1).max(axis=1)
        clear = ~excl & (np.abs(fmax - 1.0) > 0.05)
        np.testing.assert_array_equal(_np(env._reset_u8)[clear], st["reset"][clear])
    print(f"worst step: {100 * worst:.1f} % excluded")
    env.close()
    return got, st, M


@pytest.mark.parametrize("robot,n,steps", [("mc", 256, 1), ("go1", 256, 1), ("mc", 4096, 1), ("go1", 4096, 1),
                                           ("mc", 256, 24), ("go1", 256, 24), ("mc", 4096, 10), ("mc", 1001, 3),
                                           ("go1", 37, 3)])
def test_physics_matches_oracle(robot, n, steps):
    """The fused step kernel's physics against the fp64 oracle over 1, 10 or 24 steps (a PPO rollout's length),
    re-synchronised to the oracle's state before every step, at test grids, at the bench's 4096-env launch grid
    (1,024 four-env workgroups on the plane) and at ragged env counts (1,001 and 37: a last workgroup with padded
    env slots).  Every env of every step within the tolerances of helpers.within_tolerance except the envs
    the oracle reports on a contact-model discontinuity (at most MAX_EXCLUDED per step)."""
    _physics_vs_oracle(robot, n, steps)


@pytest.mark.parametrize("robot,steps", [("mc", 1), ("go1", 1), ("mc", 3), ("go1", 3)])
def test_lying_robots_match_oracle(robot, steps):
    """The leg colliders' support tables in contact: 1,024 robots lying on their sides, so the ab/ad /
    thigh / calf colliders of the lower legs touch the plane, not only the feet — kernel vs oracle as above, and the
    contact forces show those links carrying load in many envs."""
    got, st, M = _physics_vs_oracle(robot, 1024, steps, lying=True)
    names = load_robot(ROBOT_FILES[robot])["body_names"]
    links = [b for b, nm in enumerate(names) if nm.endswith("_hip") or nm.endswith("_thigh")]
    loaded = (np.linalg.norm(got["contact"][:, links], axis=-1) > 1e-3).any(axis=1)
    print(f"{robot}: {loaded.mean() * 100:.1f} % of envs with a loaded hip / thigh collider")
    assert loaded.mean() > 0.2


@pytest.mark.parametrize("robot,n,steps", [("mc", 256, 10), ("go1", 256, 3), ("mc", 37, 3)])
def test_pgs_solver_matches_oracle(robot, n, steps):
    """Cfg.sim.physx.solver_type 0 (PhysX's PGS; the presets select 1 = TGS, legged_robot_config.py:247): the
    iterations sweep the whole sub-step with the sub-step-start targets and positions integrate dt x the final
    velocities.  Kernel and oracle agree the same way as under TGS."""
    _physics_vs_oracle(robot, n, steps, extra={"sim.physx.solver_type": 0})


@pytest.mark.parametrize("robot,ctl,steps", [("go1", "V", 1), ("go1", "V", 3), ("mc", "T", 1), ("mc", "T", 3)])
def test_control_types_and_pushes_match_oracle(robot, ctl, steps):
    """Velocity ('V') and torque ('T') control (legged_robot.py:672-676) through the physics, with _push_robots
    (:757-766) every step (push_interval_s = dt): the pushed root velocities enter the next step's dynamics.  Kernel
    and oracle agree within the physics tolerances (every env outside the oracle's discontinuity margins)."""
    extra = {"control.control_type": ctl, "domain_rand.push_robots": True, "domain_rand.push_interval_s": 0.02,
             "domain_rand.max_push_vel_xy": 0.5}
    if ctl == "V":  # velocity-loop gains (the presets' position gains saturate every joint in 'V')
        extra.update({"control.stiffness": {"joint": 2.0}, "control.damping": {"joint": 0.002}})
    _physics_vs_oracle(robot, 128, steps, extra=extra)


@pytest.mark.parametrize("robot,steps", [("mc", 1), ("go1", 1), ("mc", 10), ("go1", 10)])
def test_joint_limits_match_oracle(robot, steps):
    """Joint position limits (the URDF limits PhysX enforces): joints started at or past a limit,
    moving into it, with position targets 0.4 rad beyond it.  Kernel and oracle agree within the physics
    tolerances, and the limit holds: no joint ends more than the Baumgarte-recovering overshoot past its limit.
    (Self-collision off: the limit poses fold legs into the base box, where the two constraints cannot both hold.)"""
    got, st, M = _physics_vs_oracle(robot, 256, steps, limits=True, self_on=False)
    lo, hi = np.array(M.dof_lower[:], np.float32), np.array(M.dof_upper[:], np.float32)
    over = np.maximum(got["dof_pos"] - hi, lo - got["dof_pos"]).max()
    assert over < (0.09 if steps == 1 else 0.03), over  # started up to 0.03 rad past; recovers at 0.2 / sub-step


@pytest.mark.parametrize("robot,steps", [("mc", 1), ("go1", 1), ("mc", 10), ("go1", 10)])
def test_self_collision_matches_oracle(robot, steps):
    """Self-collision (Cfg.asset.self_collisions = 0 in both presets): legs folded into each other
    and into the base box, position targets holding them there, for 1 and 10 re-synchronised steps.  Kernel and
    oracle agree within the physics tolerances, contact forces included (the base's self-contact force feeds the
    termination test)."""
    _physics_vs_oracle(robot, 256, steps, selfc=True)


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_self_contact_stats_leave_results_unchanged(robot):
    """lrl_sim_self_contact_stats: with the counters on, the detection counts every pair in contact (not only the
    capped slots) and the step's results stay bit-identical; the counters see the folded-leg poses' contacts."""
    n = 256
    cfg, rob, M, P = make(robot, **{"env.num_envs": n})
    rng = np.random.default_rng(12)
    root, dof, dofv = _random_states(rng, n, P, robot)
    root, dof = _self_states(rng, n, M, root, dof)
    act = _dev((rng.normal(size=(n, 12)) * 0.5).astype(np.float32))
    noise = _dev(rng.random((n, P.num_obs)).astype(np.float32))
    dr = _dev(rng.random(n).astype(np.float32))
    outs = []
    for stats in (False, True):
        env = _env(robot, n)
        env.root_states[:] = _dev(root)
        env.dof_pos[:] = _dev(dof)
        env.dof_vel[:] = _dev(dofv)
        if stats:
            env.self_contact_stats(True)
        _step_raw(env, act, _abi.STEP_PHYSICS | _abi.STEP_INJECT_UNIFORM, noise, dr)
        sc = env.self_contact_stats(False) if stats else None
        outs.append([_np(getattr(env, a)).copy() for a in ("root_states", "dof_pos", "dof_vel", "contact_forces")])
        env.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    print(robot, sc)
    assert sc["env_substeps_in_self_contact"] > 0.1 * n  # the folded poses touch
    assert sc["self_pairs_in_contact"] >= sc["env_substeps_in_self_contact"]
    assert sc["self_pairs_dropped"] >= sc["env_substeps_over_cap"]


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_standing_settles(robot):
    n = 128
    # physical sanity check, not a parity test: no COM/mass randomisation (a 10 cm COM shift can tip a
    # robot that only holds its default pose)
    env = _env(robot, n, **{"noise.add_noise": False, "domain_rand.randomize_com_displacement": False,
                            "domain_rand.randomize_base_mass": False})
    env.reset()
    zero = torch.zeros(n, 12, device="cuda:0")
    for _ in range(150):
        env.step(zero)
    torch.cuda.synchronize()
    z = _np(env.root_states[:, 2])
    mass = env.robot["base_mass"] + sum(sum(x) for x in env.robot["link_mass"]) + _np(env.payloads)
    fz = _np(env.contact_forces[:, env.feet_indices, 2]).sum(1)
    assert np.isfinite(z).all()
    assert (z > 0.2).all() and (z < 0.4).all(), z
    np.testing.assert_allclose(fz, mass * 9.81, rtol=0.05)
    assert _np(env._reset_u8).sum() == 0
    env.close()


def test_history_and_reset_semantics():
    from lrl.history import HistoryWrapper
    n = 64
    env = HistoryWrapper(_env("mc", n))
    d = env.reset()
    assert d["obs_history"].abs().sum().item() == 0.0  # reset zeroes the history (history_wrapper.py:36-41)
    obs_dict, rew, done, info = env.step(torch.zeros(n, 12, device="cuda:0"))
    h = obs_dict["obs_history"]
    assert torch.equal(h[:, -42:], obs_dict["obs"])
    assert h[:, :-42].abs().sum().item() == 0.0
    prev = h.clone()
    obs_dict, _, _, _ = env.step(torch.zeros(n, 12, device="cuda:0"))
    assert torch.equal(obs_dict["obs_history"][:, -84:-42], prev[:, -42:])
    assert "env_bins" in info and "time_outs" in info and info["privileged_obs"].shape == (n, 18)
    before = obs_dict["obs_history"].clone()
    d2 = env.get_observations()  # shifts the history (Q6)
    assert torch.equal(d2["obs_history"][:, :-42], before[:, 42:])
    env.env.close()


def test_upstream_resets_timeouts_and_command_resampling():
    """legacy_fork=False (SURVEY.md §8(f) rank 2, Q2/Q3 re-enabled): time-outs (legged_robot.py:196-198) and
    terminations reset envs inside step (:177 reset_idx -> _reset_dofs / _reset_root_states / buffer
    zeroing, :227-290); the reset envs observe their post-reset state (compute_observations after reset_idx,
    :179) incl. the newest history slot; episode logging and time_outs reach extras; commands are resampled
    from the curriculum every resampling_time (:578-581) and at resets (_resample_commands :595-626)."""
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    n = 64
    cfg = _cfg("mc", n, **{"env.episode_length_s": 0.1, "commands.resampling_time": 0.06, "noise.add_noise": False})
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, legacy_fork=False))
    inner = env.env
    M = int(inner.max_episode_length)
    interval = int(cfg.commands.resampling_time / inner.dt)
    assert M == 6 and interval == 3
    env.reset()
    q0 = inner.default_dof_pos.expand(n, 12)
    zero = torch.zeros(n, 12, device="cuda:0")
    seen_timeout = seen_resample = False
    for step in range(16):
        elen = inner.episode_length_buf.clone().long()
        cmd0 = inner.commands.clone()
        obs_dict, rew, done, info = env.step(zero)
        torch.cuda.synchronize()
        tout = inner.time_out_buf
        assert torch.equal(tout, elen + 1 > M)  # time-out exactly when the episode passes max_episode_length
        assert bool(done[tout].all())
        reset = done
        assert torch.equal(inner.episode_length_buf[reset].long(), torch.zeros_like(elen[reset]))
        assert torch.equal(inner.episode_length_buf[~reset].long(), elen[~reset] + 1)
        if reset.any():
            assert torch.equal(inner.dof_pos[reset], q0[reset])
            assert inner.dof_vel[reset].abs().max().item() == 0.0
            o = obs_dict["obs"][reset]
            assert o[:, 6:30].abs().max().item() == 0.0  # (q - q0) and qd terms of the post-reset state
            assert "train/episode" in info and "time_outs" in info
            seen_timeout |= bool(tout.any())
        # the newest history slot is the step's (post-reset) observation for every env
        assert torch.equal(obs_dict["obs_history"][:, -42:], obs_dict["obs"])
        changed = (inner.commands != cmd0).any(dim=1)
        due = (elen + 1) % interval == 0
        assert not bool((changed & ~(due | reset)).any())  # commands move only when due or reset
        seen_resample |= bool((changed & due & ~reset).any())
    assert seen_timeout and seen_resample
    inner.close()


def test_train_eval_split():
    """eval_cfg (base_task.py:43-50, legged_robot.py:204-290, 456-469): eval envs follow the train envs in one
    sim; resets log train envs into extras['train/episode'] and keep each eval env's first finished episode;
    reset_evaluation_envs reports the batch and resets the eval envs; Runner drives the eval envs with the
    student policy.  An eval cfg that changes per-step kernel parameters is refused."""
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    from lrl.ppo import runner as R
    n_tr, n_ev = 64, 32
    env = LeggedRobotEnv("cuda:0", cfg=_cfg("mc", n_tr), eval_cfg=_cfg("mc", n_ev))
    assert (env.num_train_envs, env.num_eval_envs, env.num_envs) == (n_tr, n_ev, n_tr + n_ev)
    env.reset()  # (the initial reset_idx of every env records the eval envs' zero sums, as in the reference)
    env.reset_evaluation_envs()  # a fresh evaluation batch: every eval env unset (-1)
    a = torch.zeros(n_tr + n_ev, 12, device="cuda:0")
    for _ in range(3):
        env.step(a)
    sums = {k: v.clone() for k, v in env.episode_sums.items()}
    ids = torch.tensor([1, 5, n_tr + 2, n_tr + 7], device="cuda:0")
    env.reset_idx(ids)
    torch.cuda.synchronize()
    assert "train/episode" in env.extras and "eval/episode" in env.extras
    k0 = next(iter(env.episode_sums_eval))
    ev = env.episode_sums_eval[k0]
    assert torch.equal(ev[ids[2:]], sums[k0][ids[2:]])  # eval envs: their finished episode kept
    assert bool((ev[:n_tr] == -1).all()) and bool((ev[n_tr:][ev[n_tr:] != -1].numel() == 2))
    np.testing.assert_allclose(env.extras["train/episode"]["rew_" + k0].item(), sums[k0][ids[:2]].mean().item(),
                               rtol=1e-6)
    assert bool((env.episode_sums[k0][ids] == 0).all())
    logged = {}
    env.extras["eval/episode"] = logged
    env.reset_evaluation_envs()
    # the batch means land in the current eval/episode dict; reset_idx of the eval envs then starts a fresh
    # one (legged_robot.py:216 then :270 — the reference's order, reproduced)
    assert set("rew_" + k for k in env.episode_sums_eval) <= set(logged)
    assert env.extras["eval/episode"] is not logged
    assert bool((env.episode_sums_eval[k0] == -1).all())
    assert bool((env.episode_length_buf[n_tr:] == 0).all())
    env.close()
    bad = _cfg("mc", n_ev)
    bad.control.stiffness = {k: 2 * v for k, v in bad.control.stiffness.items()}
    with pytest.raises(NotImplementedError):
        LeggedRobotEnv("cuda:0", cfg=_cfg("mc", n_tr), eval_cfg=bad)
    # Runner: train envs through PPO.act, eval envs through the student (act_student_fused)
    R.RunnerArgs.save_interval = 0
    henv = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=_cfg("mc", n_tr), eval_cfg=_cfg("mc", n_ev)))
    runner = R.Runner(henv, device="cuda:0", seed=3)
    runner.learn(1, eval_freq=1)
    assert runner.alg.storage.num_envs == n_tr
    assert "eval/episode" in henv.env.extras
    henv.env.close()


def test_extras_are_step_time_snapshots():
    """VelocityTrackingEasyEnv.step's numpy extras (velocity_tracking_easy_env.py:48-62): what a caller took from
    ``info`` — an array read, or the dict copied — holds the step it came from after later steps; ``info`` itself is
    one dict updated by every step (as the reference's ``self.extras.update``), so a read after the next step gives
    that step's values.  Values against the live tensors at the step they snapshot."""
    from lrl.env import LeggedRobotEnv
    cfg = lcfg.make_cfg()
    lcfg.config_mini_cheetah(cfg)
    n = 64
    env = LeggedRobotEnv("cuda:0", cfg=cfg, num_envs=n)
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(2)

    def live():
        torch.cuda.synchronize()
        f = env.feet_indices
        return {"joint_pos": _np(env.dof_pos), "joint_vel": _np(env.dof_vel), "joint_pos_target": _np(env.joint_pos_target),
                "body_linear_vel": _np(env.base_lin_vel), "body_angular_vel": _np(env.base_ang_vel),
                "body_linear_vel_cmd": _np(env.commands)[:, 0:2], "body_angular_vel_cmd": _np(env.commands)[:, 2:],
                "contact_states": _np(env.contact_forces[:, f, 2] > 1.0), "foot_positions": _np(env._foot_positions()),
                "body_pos": _np(env.root_states[:, 0:3]), "torques": _np(env.torques)}
    env.commands[:, :3] = torch.rand(n, 3, generator=g, device="cuda:0")
    _, _, _, info = env.step(torch.randn(n, 12, generator=g, device="cuda:0") * 0.5)
    want0 = live()
    held = dict(info)          # the dict copied at step t
    jp = info["joint_pos"]     # an array read at step t
    items = info.copy()
    env.commands[:, :3] = torch.rand(n, 3, generator=g, device="cuda:0")
    env.step(torch.randn(n, 12, generator=g, device="cuda:0") * 0.5)
    env.step(torch.randn(n, 12, generator=g, device="cuda:0") * 0.5)
    want2 = live()
    assert np.abs(want2["joint_pos"] - want0["joint_pos"]).max() > 1e-3  # the state moved
    for k, v in want0.items():
        tol = 1e-6 if k == "foot_positions" else 0.0  # (the same FK in another kernel: contraction may differ)
        assert held[k].shape == v.shape and items[k].shape == v.shape, k
        np.testing.assert_allclose(held[k], v, rtol=0, atol=tol, err_msg=k)
        np.testing.assert_allclose(items[k], v, rtol=0, atol=tol, err_msg=k)
        np.testing.assert_allclose(info[k], want2[k], rtol=0, atol=tol, err_msg=k)  # the live dict: latest step
    np.testing.assert_array_equal(jp, want0["joint_pos"])
    assert set(info.keys()) >= set(want0) | {"privileged_obs", "joint_vel_target"} and len(info) == len(info.keys())
    env.close()


@pytest.mark.parametrize("rough,resampling_time", [(False, 0.14), (True, 0.14), (False, 0.5), (False, 1e9)])
def test_device_reset_path_matches_host_path(rough, resampling_time):
    """The upstream step without a host round trip (LeggedRobotEnv._step_device: device id lists and counts, the
    command curriculum's update / sample on the device, lrl_sim_curriculum_resample_dev) against the host path
    (device_resets=False: one device->host copy per step, numpy / native-host curriculum) on the same seeds and actions:
    time-outs every 25 steps, resampling every 7, thresholds that pass (the weights change, the cdf cache is exercised),
    terrain curriculum on the rough tiles.  Every buffer, the curriculum (weights, MT19937 state, episode rewards), the
    env bins, terrain levels / origins and the logged episode means are bit-identical.  resampling_time = 0.5 (the
    episode length: ep_len = min(max_episode_length, interval) is the float max_episode_length) and 1e9 (the
    reference's eval setting: an interval past int32) resample at resets only."""
    from lrl.env import LeggedRobotEnv
    n = 256
    cfgs = []
    for _ in range(2):
        cfg = lcfg.make_cfg()
        lcfg.config_go1(cfg)
        cfg.env.num_envs = n
        cfg.env.episode_length_s = 0.5
        cfg.commands.resampling_time = resampling_time
        cfg.commands.forward_curriculum_threshold = 0.05
        cfg.commands.yaw_curriculum_threshold = 0.05
        if rough:
            cfg.terrain.mesh_type = "trimesh"
            cfg.terrain.curriculum = True
            cfg.terrain.num_rows, cfg.terrain.num_cols, cfg.terrain.border_size = 4, 4, 3.0
            cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
            cfg.terrain.max_init_terrain_level = 3
        cfgs.append(cfg)
    envs = [LeggedRobotEnv("cuda:0", cfg=cfgs[i], seed=7, legacy_fork=False, device_resets=bool(i)) for i in range(2)]
    host, dev = envs
    assert dev._dev_path and not host._dev_path
    for e in envs:
        e.reset()
    g = torch.Generator(device="cuda:0").manual_seed(4)
    keys = ["root_states", "dof_pos", "dof_vel", "commands", "_command_sums", "_episode_sums", "obs_buf",
            "privileged_obs_buf", "rew_buf", "episode_length_buf", "_reset_u8", "env_origins"]
    for s in range(80):
        act = torch.randn(n, 12, generator=g, device="cuda:0") * 0.6
        for e in envs:
            e.step(act)
        if s % 10 == 9 or s == 79:
            torch.cuda.synchronize()
            for k in keys:
                np.testing.assert_array_equal(_np(getattr(dev, k)), _np(getattr(host, k)), err_msg=f"{k} step {s}")
            if rough:
                np.testing.assert_array_equal(_np(dev.terrain_levels), _np(host.terrain_levels))
            np.testing.assert_array_equal(dev.env_command_bins, host.env_command_bins)
            np.testing.assert_array_equal(_np(dev.env_command_bins_t), _np(host.env_command_bins_t))
            cd, ch = dev.curriculum, host.curriculum
            np.testing.assert_array_equal(cd.weights, ch.weights)
            np.testing.assert_array_equal(cd.episode_reward_lin, ch.episode_reward_lin)
            np.testing.assert_array_equal(cd.episode_reward_ang, ch.episode_reward_ang)
            cd._sync_from_rng()
            ch._sync_from_rng()
            assert int(cd._mt_pos[0]) == int(ch._mt_pos[0])
            np.testing.assert_array_equal(cd._mt_key, ch._mt_key)
            ed, eh = dev.extras["train/episode"], host.extras["train/episode"]
            for k, v in eh.items():
                a = float(v) if not isinstance(v, torch.Tensor) else float(v.item())
                b = ed[k]
                b = float(b) if not isinstance(b, torch.Tensor) else float(b.item())
                assert a == b or (a != a and b != b), (k, a, b, s)
    assert host.curriculum.weights.sum() > 1.0 + (host.curriculum.weights > 0).sum() * 0  # weights grew
    assert int(_np(host._reset_u8).sum()) >= 0
    for e in envs:
        e.close()


def test_device_path_episode_log_is_not_overwritten():
    """on the device reset path each step publishes extras['train/episode'] / extras['env_bins'] in fresh
    buffers, so a dict a consumer keeps (the reference runner's logger.store_metrics(**infos['train/episode'])) still
    holds the values of its own step after later steps; before any reset is logged the key is absent, as in the
    reference, whose extras gain it at the first reset batch."""
    from lrl.env import LeggedRobotEnv
    n = 256
    cfg = lcfg.make_cfg()
    lcfg.config_go1(cfg)
    cfg.env.num_envs = n
    cfg.env.episode_length_s = 0.3
    cfg.commands.resampling_time = 0.14
    env = LeggedRobotEnv("cuda:0", cfg=cfg, seed=3, legacy_fork=False)
    assert env._dev_path
    g = torch.Generator(device="cuda:0").manual_seed(1)
    act = lambda: torch.randn(n, 12, generator=g, device="cuda:0") * 0.3
    # the robots placed at their initial state without reset() (which would log), so the first step resets nobody
    env.root_states[:] = env.base_init_state
    env.root_states[:, :3] += env.env_origins
    env.dof_pos[:] = env.default_dof_pos
    env.dof_vel[:] = 0.0
    _, _, done, _ = env.step(act() * 0.1)
    assert not bool(done.any())
    assert "train/episode" not in env.extras  # no reset logged yet (episodes are 15 steps long)
    kept = []
    for s in range(40):
        _, _, done, ex = env.step(act())
        if "train/episode" in ex:
            ep = ex["train/episode"]
            now = {k: (float(v.item()) if isinstance(v, torch.Tensor) else float(v)) for k, v in ep.items()}
            kept.append((s, ep, now, ex["env_bins"], ex["env_bins"].cpu().numpy().copy()))
    assert len(kept) >= 20 and kept[0][0] <= 16
    changed = 0
    for s, ep, now, bins, bins_now in kept:
        later = {k: (float(v.item()) if isinstance(v, torch.Tensor) else float(v)) for k, v in ep.items()}
        for k in now:
            assert later[k] == now[k] or (later[k] != later[k] and now[k] != now[k]), (s, k, now[k], later[k])
        np.testing.assert_array_equal(bins.cpu().numpy(), bins_now)
        changed += int(now != kept[-1][2])
    assert changed > 0  # the logged values did move over the run
    env.close()


def test_sim_create_refuses_shared_or_out_of_range_sum_rows():
    """lrl_sim_create checks the episode / command sum rows the kernel writes: every reward term and the termination
    term its own row below num_sum_keys (a shared or out-of-range row would be a lost update or a write past the
    rows' arena slice)."""
    cfg, rob, Mo, P = make("mc")
    L = _abi.lib()

    def create(P):
        sim = C.c_void_p()
        rc = L.lrl_sim_create(C.byref(Mo), C.byref(P), C.c_int32(16), C.c_int64(0), C.c_uint64(1), C.c_int32(0),
                              C.byref(sim))
        if rc == 0:
            L.lrl_sim_destroy(sim)
        return rc
    assert P.num_reward_terms >= 2
    assert create(P) == 0
    for field, t, v in [("reward_slot", 1, None), ("reward_slot", 0, P.num_sum_keys), ("reward_slot", 0, -1)]:
        saved = getattr(P, field)[t]
        getattr(P, field)[t] = P.reward_slot[0] if v is None else v
        assert create(P) != 0, (field, t, v)
        assert b"sum row" in L.lrl_last_error()
        getattr(P, field)[t] = saved
    assert create(P) == 0
