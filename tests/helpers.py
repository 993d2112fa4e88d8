"""Shared test helpers: configs, fixture loading, oracle state set-up."""
import json
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


# fp32 kernel vs the fp64 oracle after the 4 sub-steps of a step, per field (atol, rtol): |got - ref| <= atol + rtol |ref|
# for every element.  Set from the measured error distribution (round 4, profiles/r4b_parity_stats.jsonl, 128 compared
# steps / 89,344 env-steps of every physics test: scripts/parity_stats_summary.py): each bar sits 2-25x above the
# largest kernel-vs-oracle error over the compared envs and about 10x above its 99.9th percentile; 4-25x tighter than
# rounds 1-3 (base position / quaternion 2e-4, joint angles 2e-3 rad, velocities 5e-2 + 1 %, contact forces 2 N + 2 %).
TOL = {"pos": (5e-5, 0.0), "quat": (1e-5, 0.0), "dof_pos": (2e-4, 0.0), "dof_vel": (2e-2, 4e-3),
       "lin_vel": (2e-3, 4e-4), "ang_vel": (5e-3, 1e-3), "contact": (0.5, 5e-3)}
# Every env must meet all of them, except envs the oracle reports as sitting on a discontinuity of the contact model
# (oracle.env_step margins: a sphere within SEP_EPS of contact_offset, a nearest-triangle or normal-rule switch within
# SEP_EPS, a restitution switch within VEL_EPS) — there fp32 and fp64 may legitimately take different branches — or
# whose fp64 result itself leaves the bars under fp32-size input noise (oracle_sensitivity).
SEP_EPS, VEL_EPS = 1e-4, 1e-3
# the margin of comparisons that start from identical state (one step, or re-synchronised steps): positions of the two
# runs differ by ~1e-7 m after the step's four sub-steps, so a branch within 1e-5 m is the most fp32 can flip
SEP_EPS_1 = 1e-5
# at most this fraction of the envs of one compared step may sit on such a discontinuity
MAX_EXCLUDED = 0.06


def within_tolerance(got, st, tol=None):
    """Per-env mask: every physics output of ``got`` within the per-field bars ``tol`` (default TOL) of ``st``."""
    tol = TOL if tol is None else tol
    n = st["root"].shape[0]

    def ok(f, a, b):
        atol, rtol = tol[f]
        err = np.abs(a - b) - rtol * np.abs(b)
        return np.all(err.reshape(n, -1) <= atol, axis=1)
    return (ok("pos", got["root"][:, :3], st["root"][:, :3]) & ok("quat", got["root"][:, 3:7], st["root"][:, 3:7])
            & ok("dof_pos", got["dof_pos"], st["dof_pos"]) & ok("dof_vel", got["dof_vel"], st["dof_vel"])
            & ok("lin_vel", got["root"][:, 7:10], st["root"][:, 7:10])
            & ok("ang_vel", got["root"][:, 10:13], st["root"][:, 10:13])
            & ok("contact", got["contact"], st["contact"]))


def physics_mismatch(got, st, margins, sensitive=None, sep_eps=SEP_EPS):
    """(bad, excluded) env masks: ``bad`` = outside tolerance and not excluded.  Excluded: the oracle's
    discontinuity margins below ``sep_eps`` / VEL_EPS, or (``sensitive``) envs whose fp64 oracle result itself leaves
    the tolerance when its input state is perturbed at float32 rounding level (see ``oracle_sensitivity``)."""
    excluded = (margins[:, 0] < sep_eps) | (margins[:, 1] < VEL_EPS)
    if sensitive is not None:
        excluded = excluded | sensitive
    return ~within_tolerance(got, st) & ~excluded, excluded


def perturb_state(st, rng, rel=2e-7):
    """A copy of an oracle state with root / joint state moved by ~float32 rounding (relative ``rel``, at least
    ``rel`` absolute): the size of the difference an fp32 restatement carries into the same step."""
    out = {k: v.copy() for k, v in st.items()}
    for k in ("root", "dof_pos", "dof_vel"):
        a = out[k]
        a += (rng.choice([-1.0, 1.0], a.shape) * rel * np.maximum(np.abs(a), 1.0)).astype(np.float32)
    return out


def oracle_sensitivity(ref, alt):
    """Envs whose oracle outputs from a perturbed start (``alt``) leave the tolerance of the unperturbed ones."""
    return ~within_tolerance(alt, ref)


# per-field views of a physics state for the error statistics
_FIELDS = {"pos": ("root", slice(0, 3)), "quat": ("root", slice(3, 7)), "dof_pos": ("dof_pos", slice(None)),
           "dof_vel": ("dof_vel", slice(None)), "lin_vel": ("root", slice(7, 10)), "ang_vel": ("root", slice(10, 13)),
           "contact": ("contact", slice(None))}


def error_stats(got, st, keep):
    """Per field: max / p99 / p50 over the kept envs of each env's largest element error |got - st| (abs) and of
    |got - st| / (1 + |st|) (scaled)."""
    out = {"envs": int(keep.sum())}
    n = st["root"].shape[0]
    for f, (k, sl) in _FIELDS.items():
        a = np.asarray(got[k], np.float64)[..., sl] if k != "contact" else np.asarray(got[k], np.float64)
        b = np.asarray(st[k], np.float64)[..., sl] if k != "contact" else np.asarray(st[k], np.float64)
        d = np.abs(a - b).reshape(n, -1)
        r = (np.abs(a - b) / (1.0 + np.abs(b))).reshape(n, -1)
        ea, er = d.max(1)[keep], r.max(1)[keep]
        if len(ea) == 0:
            continue
        out[f] = {"abs_max": float(ea.max()), "abs_p99": float(np.percentile(ea, 99)),
                  "abs_p50": float(np.percentile(ea, 50)), "scaled_max": float(er.max()),
                  "scaled_p99": float(np.percentile(er, 99))}
    return out


def record_errors(tag, got, st, excluded, alt=None):
    """Error distribution of one compared step over the non-excluded envs — kernel vs oracle, and (``alt``: the oracle
    from an fp32-rounding-size perturbed start) the fp64 oracle's own spread — appended as one JSON line to
    $LRL_PARITY_STATS when set (profiles/r4*_parity_stats.jsonl), and returned."""
    keep = ~excluded
    rec = {"tag": tag, "n": int(len(keep)), "excluded": int(excluded.sum()), "kernel_vs_oracle": error_stats(got, st, keep)}
    if alt is not None:
        rec["oracle_spread"] = error_stats(alt, st, keep)
    path = os.environ.get("LRL_PARITY_STATS")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
        # per-env element errors (kernel vs oracle, oracle spread) for offline analysis of tolerance choices
        arrs = {"excluded": excluded}
        for f_, (k, sl) in _FIELDS.items():
            ref = np.asarray(st[k], np.float64)
            sel = (lambda a: a[..., sl]) if k != "contact" else (lambda a: a)
            n = ref.shape[0]
            arrs["ko_" + f_] = np.abs(sel(np.asarray(got[k], np.float64)) - sel(ref)).reshape(n, -1).astype(np.float32)
            arrs["ref_" + f_] = np.abs(sel(ref)).reshape(n, -1).astype(np.float32)
            if alt is not None:
                arrs["os_" + f_] = np.abs(sel(np.asarray(alt[k], np.float64)) - sel(ref)).reshape(n, -1).astype(np.float32)
        i = sum(1 for _ in open(path)) - 1
        np.savez_compressed(path.replace(".jsonl", f"_{i:03d}.npz"), tag=np.array(tag), **arrs)
    return rec
