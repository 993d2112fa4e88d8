"""CPU checks of the oracle's self-collision (Cfg.asset.self_collisions = 0 in both presets,
mini_cheetah_config.py:44, go1_config.py:44, passed to create_actor at legged_robot.py:1246-1247).

* the candidate list follows PhysX's articulation filter: every pair of collision spheres on different links except
  a link and its parent (the fixed Go1 feet merged into the calves), leg spheres below the hip against the base box;
* with self-collision on, legs driven into each other and into the base stop there (the Baumgarte-recovered overlap
  stays small); with it off, the same drive interpenetrates.
The GPU parity of the kernel against these rows is tests/test_env_gpu.py::test_self_collision_matches_oracle."""
import os

import numpy as np
import pytest

from helpers import make
from lrl import _abi
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dyn(M, s):
    b = M.sphere_body[s]
    return M.body_leg[b], min(M.body_link[b], 2)


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_candidate_pairs_follow_the_articulation_filter(robot):
    cfg, rob, M, P = make(robot)
    pairs, _ = oracle.self_pairs(M)
    got = {(int(a), int(b)) for a, b in pairs}
    assert len(got) == len(pairs)  # no duplicates
    want = set()
    legs = [s for s in range(M.num_spheres) if M.body_leg[M.sphere_body[s]] >= 0 and M.sphere_radius[s] > 0]
    for a in legs:
        la, ka = _dyn(M, a)
        if ka >= 1:
            want.add((a, -1))  # not the hip, whose parent is the base
        for b in legs:
            lb, kb = _dyn(M, b)
            if lb < la or (lb == la and (b <= a or abs(ka - kb) < 2)):
                continue
            want.add((a, b))
    assert got == want
    # canonical order: leg of a, then group (same leg, legs above, the box), then a, then b
    grp = [(_dyn(M, a)[0], 4 if b < 0 else _dyn(M, b)[0] - _dyn(M, a)[0], a, b) for a, b in pairs]
    assert grp == sorted(grp)


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_oracle_self_collision_separates_and_holds(robot):
    """Passive legs (PD gains 0) started interpenetrating each other or the base by 0.5-2 cm, at rest, in free fall:
    the self-contact rows push the links apart (Baumgarte) and keep them apart; without them nothing moves them."""
    n = 4096
    rng = np.random.default_rng(11)
    cfg, rob, M, P = make(robot, **{"env.num_envs": 1})
    lo, hi = np.array(M.dof_lower[:], np.float32), np.array(M.dof_upper[:], np.float32)
    q0 = rng.uniform(lo + 0.05, hi - 0.05, (n, 12)).astype(np.float32)
    worst0 = np.array([oracle.self_pairs(M, q)[1].min() for q in q0])
    q0 = q0[(worst0 < -0.005) & (worst0 > -0.02)][:24]
    n = len(q0)
    assert n >= 8
    act = np.zeros((n, 12), np.float32)
    pen = np.array([oracle.self_pairs(M, q)[1] for q in q0]) < 0  # the pairs interpenetrating at the start
    worst = {}
    for on in (1, 0):
        cfg, rob, M, P = make(robot, **{"env.num_envs": n})
        P.self_collisions = on
        for j in range(12):
            P.p_gains[j] = P.d_gains[j] = 0.0
        st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
        st["root"][:] = 0
        st["root"][:, 2] = 0.8  # airborne: only the self-contacts act on the legs
        st["root"][:, 6] = 1
        st["dof_pos"][:] = q0
        for s in range(5):
            oracle.env_step(M, P, st, act, _abi.STEP_PHYSICS, common_step_counter=s + 1)
        sep = np.array([oracle.self_pairs(M, q)[1] for q in st["dof_pos"]])
        worst[on] = sep[pen].min()
    assert worst[0] < -0.005, worst  # still interpenetrated without the rows
    assert worst[1] > -1e-3, worst  # pushed apart (Baumgarte) with them, within 0.1 s


def test_oracle_tgs_variant_matches_pgs_on_standing():
    """The PGS-vs-TGS study's solver switch (lrl_oracle.c lrlo_set_solver_tgs, scripts/tgs_vs_pgs.py): from the same
    standing state both solvers hold the robot (base height within 3 mm of each other after 0.5 s, foot forces carrying
    the weight), and the switch off restores the kernel's model exactly."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("tgs_vs_pgs", os.path.join(ROOT, "scripts", "tgs_vs_pgs.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cfg, P, M = mod.setup()
    res = []
    for tgs in (0, 1, 0):
        oracle.set_solver_tgs(tgs)
        st = mod.state(P, M)
        h, fz, vx, up = mod.run(P, M, st, 25)
        res.append((h, fz, st["dof_pos"].copy()))
    oracle.set_solver_tgs(0)
    (h0, f0, q0), (h1, f1, q1), (h2, f2, q2) = res
    assert np.abs(h0 - h1).max() < 3e-3 and abs(f1[-5:].mean() - 1.0) < 0.1 and abs(f0[-5:].mean() - 1.0) < 0.1
    assert np.abs(h0 - h1).max() > 0  # the variant is a different solver
    np.testing.assert_array_equal(h0, h2)
    np.testing.assert_array_equal(q0, q2)


def test_solver_switch_follows_the_config():
    """Cfg.sim.physx.solver_type drives lrl_env_params.solver_tgs (legged_robot_config.py:247: 1 = TGS, the presets'
    solver; the terrain mesh solves with PGS), and the oracle's TGS under that flag is the study's switch exactly."""
    import importlib.util
    from lrl import params as lparams
    from lrl.robot import load_robot
    from helpers import ROBOT_FILES
    cfg, rob, M, P = make("mc")
    assert cfg.sim.physx.solver_type == 1 and P.solver_tgs == 1
    assert lparams.build_params(cfg, load_robot(ROBOT_FILES["mc"]), solver_type=0).solver_tgs == 0
    assert lparams.build_params(cfg, load_robot(ROBOT_FILES["mc"]), terrain_mesh=1).solver_tgs == 0
    spec = importlib.util.spec_from_file_location("tgs_vs_pgs", os.path.join(ROOT, "scripts", "tgs_vs_pgs.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    _, P0, M0 = mod.setup()  # solver_type 0: the study's switch picks the solver
    assert P0.solver_tgs == 0
    res = []
    for flag, switch in ((1, 0), (0, 1), (0, 0)):
        P0.solver_tgs = flag
        oracle.set_solver_tgs(switch)
        st = mod.state(P0, M0, dz=0.15)
        h, _, _, _ = mod.run(P0, M0, st, 10)
        res.append((h, st["dof_pos"].copy(), st["dof_vel"].copy()))
    oracle.set_solver_tgs(0)
    for a, b in zip(res[0], res[1]):  # the flag and the switch: the same solver
        np.testing.assert_array_equal(a, b)
    assert not np.array_equal(res[0][2], res[2][2])  # and not PGS
