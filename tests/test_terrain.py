"""Rough-terrain generation (lrl/terrain.py) against the reference's Terrain class (mini_gym/utils/terrain.py,
run over the same terrain_utils restatement: tests/golden/terrain.npz) — bit-exact layout, tile types and
env origins — plus structural properties of the primitives (parity unpinned: isaacgym.terrain_utils is not
vendored)."""
import types

import numpy as np

from helpers import golden
from lrl import terrain as T


def _cfg(**kw):
    c = types.SimpleNamespace(mesh_type="trimesh", curriculum=True, selected=False, terrain_kwargs=None,
                              terrain_proportions=[0.1] * 10, num_rows=3, num_cols=10, terrain_length=8.0,
                              terrain_width=8.0, horizontal_scale=0.1, vertical_scale=0.005, border_size=2.0,
                              difficulty_scale=1.0, max_platform_height=0.2, terrain_smoothness=0.005,
                              terrain_noise_magnitude=0.1, slope_treshold=0.75)
    c.__dict__.update(kw)
    return c


def test_terrain_matches_reference_layout():
    g = golden("terrain.npz")
    for name, kw in (("curriculum", {}), ("random", dict(curriculum=False, num_rows=2, num_cols=3))):
        np.random.seed(int(g[name + "_seed"]))
        c = _cfg(**kw)
        t = T.Terrain(c, 64)
        np.testing.assert_array_equal(t.height_field_raw, g[name + "_hf"])
        np.testing.assert_array_equal(c.env_origins, g[name + "_origins"])
        if name == "curriculum":
            assert len(t.triangles) == int(g["curriculum_ntri"])
            np.testing.assert_allclose(t.vertices.astype(np.float64).sum(0), g["curriculum_vsum"], rtol=1e-9)


def test_primitives_structure():
    sub = lambda: T.SubTerrain(width=80, length=80, vertical_scale=0.005, horizontal_scale=0.1)
    t = T.pyramid_stairs_terrain(sub(), step_width=0.31, step_height=0.1, platform_size=3.0)
    hf = t.height_field_raw
    assert hf[0, 0] == 0 and hf[40, 40] == hf.max() and np.all(np.diff(hf[40, :40]) >= 0)
    assert set(np.unique(hf)) <= set(range(0, hf.max() + 1, 20))  # steps of 0.1 m = 20 units
    t = T.pyramid_sloped_terrain(sub(), slope=0.2, platform_size=3.0)
    assert t.height_field_raw[40, 40] == t.height_field_raw.max() and t.height_field_raw[0, 0] == 0
    np.random.seed(0)
    t = T.random_uniform_terrain(sub(), min_height=-0.05, max_height=0.05, step=0.005, downsampled_scale=0.2)
    assert np.abs(t.height_field_raw).max() <= 10
    np.random.seed(0)
    t = T.stepping_stones_terrain(sub(), stone_size=1.0, stone_distance=0.1, max_height=0.0, platform_size=4.0)
    assert t.height_field_raw.min() == int(-10 / 0.005) and t.height_field_raw[40, 40] == 0
    v, tri = T.convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    assert v.shape == (80 * 80, 3) and tri.shape == (2 * 79 * 79, 3) and tri.max() == 80 * 80 - 1


def _oracle_terrain(g, P):
    """The golden map as the oracle's terrain: trimesh vertices in the world frame + height samples (m)."""
    from oracle import oracle
    hf = g["hf"]
    v, _ = T.convert_heightfield_to_trimesh(hf, float(g["horizontal_scale"]), float(g["vertical_scale"]), 0.75)
    v = v.reshape(hf.shape[0], hf.shape[1], 3).copy()
    v[..., :2] -= np.float32(g["border_size"])
    oracle.set_terrain(v, hf.astype(np.float32) * np.float32(g["vertical_scale"]))


def test_oracle_height_scan_matches_reference():
    """_get_heights (legged_robot.py:1469-1503) of the oracle vs the reference on its own Terrain map, random
    base poses incl. yaw and poses off the map (index clipping): bit-exact."""
    from helpers import make_rough
    from oracle import oracle
    g = golden("heights.npz")
    cfg, rob, M, P = make_rough(border_size=float(g["border_size"]))
    assert P.num_height_points == 187 and P.num_obs == 229
    _oracle_terrain(g, P)
    got = np.array([[oracle.height_sample(P, r, k) for k in range(187)] for r in g["root"]], np.float32)
    np.testing.assert_array_equal(got, g["heights"])


def test_oracle_height_observations_match_reference():
    """The height entries of compute_observations (:386-389) with the height noise (:924-927): oracle env_step
    (identity physics) on the golden poses vs the reference."""
    from helpers import make_rough
    from oracle import oracle
    from lrl import _abi
    from lrl import params as lparams
    g = golden("heights.npz")
    cfg, rob, M, P = make_rough(border_size=float(g["border_size"]))
    np.testing.assert_array_equal(lparams.noise_vec(cfg), g["noise_vec"])
    _oracle_terrain(g, P)
    n = g["root"].shape[0]
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5,
                           num_height_points=P.num_height_points)
    st["root"][:] = g["root"]
    oracle.env_step(M, P, st, np.zeros((n, 12), np.float32), _abi.STEP_INJECT_UNIFORM, noise_u=g["noise_u"],
                    dr_u=np.full(n, np.nan, np.float32))
    np.testing.assert_array_equal(st["heights"], g["heights"])
    np.testing.assert_allclose(st["obs"][:, 42:], g["obs_heights"], rtol=0, atol=1e-6)


def test_terrain_curriculum_matches_reference():
    """_update_terrain_curriculum (legged_robot.py:793-818) of the env host code vs the reference, with the
    reference's randint_like draws injected: levels and origins bit-exact."""
    import torch
    from lrl.env import LeggedRobotEnv
    g = golden("terrain_curriculum.npz")
    n = len(g["levels_in"])
    draws = iter([torch.tensor(g["draws"])])
    env = types.SimpleNamespace(init_done=True, terrain_levels=torch.tensor(g["levels_in"]),
                                terrain_types=torch.tensor(g["types"]), env_origins=torch.tensor(g["env_origins_in"]),
                                root_states=torch.zeros(n, 13), commands=torch.zeros(n, 4),
                                _rand_levels=lambda like, high: next(draws)[:len(like)])
    env.root_states[:, :2] = torch.tensor(g["root_xy"])
    env.commands[:, :2] = torch.tensor(g["commands_xy"])
    cfg = types.SimpleNamespace(
        terrain=types.SimpleNamespace(curriculum=True, env_length=float(g["env_length"]),
                                      max_terrain_level=int(g["num_rows"]),
                                      terrain_origins=torch.tensor(g["origins_table"])),
        env=types.SimpleNamespace(episode_length_s=float(g["episode_length_s"])))
    LeggedRobotEnv._update_terrain_curriculum(env, torch.tensor(g["ids"]), cfg)
    np.testing.assert_array_equal(env.terrain_levels.numpy(), g["levels_out"])
    np.testing.assert_array_equal(env.env_origins.numpy(), g["env_origins_out"])


def test_oracle_terrain_contact_geometry():
    """The mesh contact model on a 0.2 m step (slope-corrected trimesh -> a vertical wall): floor, wall from the
    low side, step top, convex edge from outside, penetration."""
    from helpers import make_rough
    from oracle import oracle
    cfg, rob, M, P = make_rough(border_size=0.0)
    hf = np.zeros((20, 20), np.int16)
    hf[10:, :] = 40  # rows i >= 10 (x >= 1.0 m) are 0.2 m high
    v, _ = T.convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    oracle.set_terrain(v.reshape(20, 20, 3), hf.astype(np.float32) * np.float32(0.005))
    r = 0.02
    sep, n = oracle.terrain_query(P, [0.5, 1.0, 0.05], r)  # above the floor
    np.testing.assert_allclose([sep, *n], [0.03, 0, 0, 1], atol=1e-7)
    sep, n = oracle.terrain_query(P, [0.985, 1.0, 0.1], r)  # touching the wall (x = 1.0 after the move)
    np.testing.assert_allclose([sep, *n], [-0.005, -1, 0, 0], atol=1e-7)
    sep, n = oracle.terrain_query(P, [0.95, 1.0, 0.1], r)  # wall beyond r + contact_offset in xy: the floor
    np.testing.assert_allclose([sep, *n], [0.08, 0, 0, 1], atol=1e-7)
    sep, n = oracle.terrain_query(P, [1.5, 1.0, 0.23], r)  # on the step top
    np.testing.assert_allclose([sep, *n], [0.01, 0, 0, 1], atol=1e-7)
    sep, n = oracle.terrain_query(P, [0.98, 1.0, 0.22], r)  # past the convex edge: distance to the edge
    d = np.hypot(0.02, 0.02)
    np.testing.assert_allclose([sep, *n], [d - r, -0.02 / d, 0, 0.02 / d], atol=1e-7)
    sep, n = oracle.terrain_query(P, [1.004, 1.0, 0.1], r)  # inside the step, behind the wall plane
    np.testing.assert_allclose([sep, *n], [-0.004 - r, -1, 0, 0], atol=1e-7)
    sep, n = oracle.terrain_query(P, [0.5, 1.0, -0.01], r)  # below the floor
    np.testing.assert_allclose([sep, *n], [-0.01 - r, 0, 0, 1], atol=1e-7)
