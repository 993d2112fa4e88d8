"""Shared test helpers: configs, fixture loading, oracle state set-up."""
import os

import numpy as np

from lrl import config as lcfg
from lrl import params as lparams
from lrl.robot import load_robot

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
ROBOT_FILES = {"mc": "mini_cheetah.urdf", "go1": "go1.urdf"}


def make(robot="mc", **over):
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    rob = load_robot(ROBOT_FILES[robot])
    if robot == "mc":
        cfg.terrain.x_offset = 0
    P = lparams.build_params(cfg, rob)
    M = lparams.build_model(rob)
    return cfg, rob, M, P


def make_rough(robot="go1", border_size=2.0, **over):
    """Rough-terrain variant of ``make``: trimesh ground, height scan (17 x 11 points -> 42 + 187 obs), terrain
    curriculum; the params carry terrain_mesh = 1 (contacts against lrl_sim_set_terrain's / the oracle's mesh)."""
    over = dict({"terrain.mesh_type": "trimesh", "terrain.measure_heights": True, "terrain.curriculum": True,
                 "terrain.border_size": border_size, "terrain.teleport_robots": False,
                 "env.num_observations": 42 + 187}, **over)
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    cfg.terrain.x_offset = 0
    rob = load_robot(ROBOT_FILES[robot])
    P = lparams.build_params(cfg, rob, terrain_mesh=1)
    M = lparams.build_model(rob)
    return cfg, rob, M, P


ALL_TERMS = {"rewards.scales.energy": -1e-3, "rewards.scales.energy_expenditure": -2e-3, "rewards.scales.dof_vel": -1e-4,
             "rewards.scales.survival": 0.3, "rewards.scales.dof_vel_limits": -0.5, "rewards.scales.torque_limits": -0.02,
             "rewards.scales.stumble": -0.4, "rewards.scales.stand_still": -0.2,
             "rewards.scales.feet_contact_forces": -0.01, "rewards.scales.orientation": -5.0,
             "rewards.scales.base_height": -30.0, "rewards.scales.termination": -2.0,
             "rewards.soft_dof_vel_limit": 0.05, "rewards.soft_torque_limit": 0.4, "rewards.max_contact_force": 20.0,
             "rewards.only_positive_rewards": False}
# (robot, fixture, cfg overrides): the presets' 12 terms for both robots, and Mini Cheetah with every _reward_* term
# of legged_robot.py:1506-1646 plus termination at a non-zero scale (make_golden.py ALL_TERMS, in that key order)
POST_PHYSICS = {"mc": ("mc", "post_physics_mc.npz", {}), "go1": ("go1", "post_physics_go1.npz", {}),
                "all_terms": ("mc", "post_physics_all_terms.npz", ALL_TERMS),
                # control_type 'V' + _push_robots every 5 steps (Go1), control_type 'T' (Mini Cheetah):
                # make_golden.py _control_tweak
                "ctl_v_push": ("go1", "post_physics_ctl_v_push.npz",
                               {"control.control_type": "V", "control.stiffness": {"joint": 2.0},
                                "control.damping": {"joint": 0.002}, "domain_rand.push_robots": True,
                                "domain_rand.push_interval_s": 0.1, "domain_rand.max_push_vel_xy": 0.5}),
                "ctl_t": ("mc", "post_physics_ctl_t.npz", {"control.control_type": "T"})}


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


# fp32 kernel vs the fp64 oracle after the 4 sub-steps of a step (abs tolerance, + relative part where given):
# base position / quaternion 2e-4, joint angles 2e-3 rad, velocities 5e-2 + 1 % (m/s, rad/s), contact forces
# 2 N + 2 %.  Every env must meet all of them, except envs the oracle reports as sitting on a discontinuity of the
# contact model (oracle.env_step margins: a sphere within SEP_EPS of contact_offset, a nearest-triangle or
# normal-rule switch within SEP_EPS, a restitution switch within VEL_EPS) — there fp32 and fp64 may legitimately
# take different branches.
SEP_EPS, VEL_EPS = 1e-4, 1e-3
# the margin of comparisons that start from identical state (one step, or re-synchronised steps): positions of the two
# runs differ by ~1e-7 m after the step's four sub-steps, so a branch within 1e-5 m is the most fp32 can flip
SEP_EPS_1 = 1e-5
# at most this fraction of the envs of one compared step may sit on such a discontinuity
MAX_EXCLUDED = 0.06


def within_tolerance(got, st, pose_tol=2e-4):
    """Per-env mask: every physics output of ``got`` within the tolerances above of ``st`` (``pose_tol``: base position
    / orientation, 2e-4 after one step; multi-step runs pass a larger one, their per-step fp32 differences add up)."""
    n = st["root"].shape[0]

    def ok(a, b, atol, rtol=0.0):
        err = np.abs(a - b) - rtol * np.abs(b)
        return np.all(err.reshape(n, -1) <= atol, axis=1)
    return (ok(got["root"][:, :3], st["root"][:, :3], pose_tol)
            & ok(got["root"][:, 3:7], st["root"][:, 3:7], pose_tol)
            & ok(got["dof_pos"], st["dof_pos"], 2e-3) & ok(got["dof_vel"], st["dof_vel"], 5e-2, 1e-2)
            & ok(got["root"][:, 7:], st["root"][:, 7:], 5e-2, 1e-2) & ok(got["contact"], st["contact"], 2.0, 0.02))


def physics_mismatch(got, st, margins, sensitive=None, pose_tol=2e-4, sep_eps=SEP_EPS):
    """(bad, excluded) env masks: ``bad`` = outside tolerance and not excluded.  Excluded: the oracle's
    discontinuity margins below ``sep_eps`` / VEL_EPS, or (``sensitive``) envs whose fp64 oracle result itself leaves
    the tolerance when its input state is perturbed at float32 rounding level (see ``oracle_sensitivity``)."""
    excluded = (margins[:, 0] < sep_eps) | (margins[:, 1] < VEL_EPS)
    if sensitive is not None:
        excluded = excluded | sensitive
    return ~within_tolerance(got, st, pose_tol) & ~excluded, excluded


def perturb_state(st, rng, rel=2e-7):
    """A copy of an oracle state with root / joint state moved by ~float32 rounding (relative ``rel``, at least
    ``rel`` absolute): the size of the difference an fp32 restatement carries into the same step."""
    out = {k: v.copy() for k, v in st.items()}
    for k in ("root", "dof_pos", "dof_vel"):
        a = out[k]
        a += (rng.choice([-1.0, 1.0], a.shape) * rel * np.maximum(np.abs(a), 1.0)).astype(np.float32)
    return out


def oracle_sensitivity(ref, alt, pose_tol=2e-4):
    """Envs whose oracle outputs from a perturbed start (``alt``) leave the tolerance of the unperturbed ones."""
    return ~within_tolerance(alt, ref, pose_tol)
