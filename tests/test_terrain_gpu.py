"""GPU parity of the rough-terrain path on cuda:0 through liblrl.so.

* height scan (_get_heights, legged_robot.py:1469-1503) and the height observations (:386-389) vs the
  REFERENCE on its own Terrain map (tests/golden/heights.npz): the env regenerates the same map from the
  same seed; heights bit-exact.
* physics against the triangle mesh (own contact model, PhysX parity unpinned) vs the CPU oracle: one env
  step (4 sub-steps) from poses on stairs / slopes / obstacles.
* terrain curriculum through reset_idx (:793-818 then _reset_root_states :714-742).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from helpers import (MAX_EXCLUDED, SEP_EPS_1, VEL_EPS, golden, make_rough, oracle_sensitivity, perturb_state,
                     physics_mismatch, record_errors)
from lrl import _abi
from lrl import config as lcfg
from oracle import oracle

pytestmark = pytest.mark.gpu

GOLDEN_TERRAIN = {"terrain.num_rows": 3, "terrain.num_cols": 10, "terrain.terrain_proportions": [0.1] * 10,
                  "terrain.terrain_noise_magnitude": 0.1, "terrain.difficulty_scale": 1.0,
                  "terrain.max_platform_height": 0.2, "terrain.terrain_smoothness": 0.005}


def _rough_cfg(n, border_size=2.0, **over):
    over = dict({"terrain.mesh_type": "trimesh", "terrain.measure_heights": True, "terrain.curriculum": True,
                 "terrain.terrain_proportions": [0.1, 0.1, 0.35, 0.25, 0.2],  # legged_robot_config.py:57
                 "terrain.border_size": border_size, "terrain.teleport_robots": False,
                 "env.num_observations": 42 + 187}, **over)
    cfg = lcfg.make_cfg()
    lcfg.config_go1(cfg)
    cfg.env.num_envs = n
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    # initial levels must index the generated rows (the preset's max_init_terrain_level 5 assumes 10 rows)
    cfg.terrain.max_init_terrain_level = min(cfg.terrain.max_init_terrain_level, cfg.terrain.num_rows - 1)
    return cfg


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda:0")


def _np(t):
    return t.detach().cpu().numpy()


def _step_raw(env, actions, flags, noise, dr):
    L = _abi.lib()
    env._inj = (noise, dr)
    _abi.check(L.lrl_sim_inject_uniforms(env._sim, C.c_void_p(noise.data_ptr()), C.c_void_p(dr.data_ptr())))
    _abi.check(L.lrl_sim_step(env._sim, C.c_void_p(actions.data_ptr()), C.c_uint32(flags), env._stream()))
    torch.cuda.synchronize()


def _oracle_terrain(env):
    t, tc = env.terrain, env.cfg.terrain
    rows, cols = t.heightsamples.shape
    v = t.vertices.reshape(rows, cols, 3).copy()
    v[..., :2] -= np.float32(tc.border_size)
    oracle.set_terrain(v, t.heightsamples.astype(np.float32) * np.float32(tc.vertical_scale))


def test_height_scan_matches_reference():
    from lrl.env import LeggedRobotEnv
    g = golden("heights.npz")
    n = g["root"].shape[0]
    env = LeggedRobotEnv("cuda:0", cfg=_rough_cfg(n, float(g["border_size"]), **GOLDEN_TERRAIN), seed=3)
    np.testing.assert_array_equal(env.terrain.heightsamples, g["hf"])  # same map from the same seed
    env.root_states[:] = _dev(g["root"])
    act = torch.zeros(n, 12, device="cuda:0")
    _step_raw(env, act, _abi.STEP_INJECT_UNIFORM, _dev(g["noise_u"]), _dev(np.full(n, np.nan, np.float32)))
    np.testing.assert_array_equal(_np(env.measured_heights), g["heights"])
    np.testing.assert_allclose(_np(env.obs_buf)[:, 42:], g["obs_heights"], rtol=0, atol=1e-6)
    env.close()


def _poses_on_terrain(rng, env, n, P):
    """Bases 0.25-0.40 m above the local terrain top, random xy over the curriculum tiles (stairs, slopes,
    obstacles, stepping stones), tilted and moving; a quarter dropped low so links touch the ground."""
    t, tc = env.terrain, env.cfg.terrain
    hs = t.heightsamples.astype(np.float32) * np.float32(tc.vertical_scale)
    rows, cols = hs.shape
    root = np.zeros((n, 13), np.float32)
    root[:, 0] = rng.uniform(0.5, tc.num_rows * tc.terrain_length - 0.5, n)
    root[:, 1] = rng.uniform(0.5, tc.num_cols * tc.terrain_width - 0.5, n)
    ix = ((root[:, 0] + tc.border_size) / tc.horizontal_scale).astype(int)
    iy = ((root[:, 1] + tc.border_size) / tc.horizontal_scale).astype(int)
    top = np.array([hs[max(i - 3, 0):i + 4, max(j - 3, 0):j + 4].max() for i, j in zip(ix, iy)], np.float32)
    root[:, 2] = top + rng.uniform(0.25, 0.40, n)
    k = n // 4
    root[:k, 2] = top[:k] + 0.12
    ang = rng.normal(size=(n, 3)) * 0.15
    ang[:, 2] = rng.uniform(-np.pi, np.pi, n)
    th = np.linalg.norm(ang, axis=1, keepdims=True)
    root[:, 3:7] = np.concatenate([ang / np.maximum(th, 1e-9) * np.sin(th / 2), np.cos(th / 2)], 1)
    root[:, 7:10] = rng.normal(size=(n, 3)) * 0.3
    root[:, 10:13] = rng.normal(size=(n, 3)) * 0.5
    dof = np.array(P.default_dof_pos[:], np.float32)[None] + rng.normal(size=(n, 12)).astype(np.float32) * 0.2
    dofv = rng.normal(size=(n, 12)).astype(np.float32)
    return root, dof, dofv


@pytest.mark.parametrize("steps", [1, 10])
def test_rough_terrain_physics_matches_oracle(steps):
    """Mesh physics (stairs, slopes, obstacles, stepping stones) against the oracle on the same mesh, 1 and 10 steps
    re-synchronised to the oracle's state before each step; the height scan of the GPU's poses bit-exact."""
    from lrl.env import LeggedRobotEnv
    n = 256
    over = {"terrain.num_rows": 4, "terrain.num_cols": 5, "terrain.border_size": 3.0}
    env = LeggedRobotEnv("cuda:0", cfg=_rough_cfg(n, **over), seed=5)
    assert env._P.terrain_mesh == 1 and np.abs(env.terrain.heightsamples).max() > 0
    cfg, rob, M, P = make_rough(**{k: v for k, v in over.items()})
    P.terrain_mesh = 1
    _oracle_terrain(env)
    rng = np.random.default_rng(9)
    root, dof, dofv = _poses_on_terrain(rng, env, n, P)
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5,
                           num_height_points=P.num_height_points)
    fr = rng.uniform(0.05, 4.5, n).astype(np.float32)
    rs = rng.uniform(0, 1, n).astype(np.float32)
    for k, v in dict(root=root, dof_pos=dof, dof_vel=dofv, friction=fr, restitution=rs).items():
        st[k][:] = v
    env.friction_coeffs[:] = _dev(fr)
    env.restitutions[:] = _dev(rs)
    env.payloads[:] = 0.0
    env.com_displacements[:] = 0.0
    flags = _abi.STEP_PHYSICS | _abi.STEP_INJECT_UNIFORM
    rng_p = np.random.default_rng(78)
    touched = 0.0
    for s in range(steps):
        env.root_states[:] = _dev(st["root"])  # re-synchronise: every step starts from the oracle's state
        env.dof_pos[:] = _dev(st["dof_pos"])
        env.dof_vel[:] = _dev(st["dof_vel"])
        act = (rng.normal(size=(n, 12)) * 0.5).astype(np.float32)
        noise = rng.random((n, P.num_obs)).astype(np.float32)
        dr = np.full(n, np.nan, np.float32)
        _step_raw(env, _dev(act), flags, _dev(noise), _dev(dr))
        margins = np.zeros((n, 2))
        st_p, st_q = perturb_state(st, rng_p), perturb_state(st, rng_p)  # (two draws, as the plane tests)
        oracle.env_step(M, P, st, act, flags, noise_u=noise, dr_u=dr, margins=margins, common_step_counter=s + 1)
        oracle.env_step(M, P, st_p, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1)
        oracle.env_step(M, P, st_q, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1)
        sens = oracle_sensitivity(st, st_p) | oracle_sensitivity(st, st_q)
        got = {k: _np(getattr(env, a)) for k, a in dict(root="root_states", dof_pos="dof_pos", dof_vel="dof_vel",
                                                          contact="contact_forces", h="measured_heights").items()}
        # fp32 kernel vs double oracle after 4 sub-steps against the mesh, tolerances as for the plane
        # (helpers.physics_mismatch): every env, except those on a contact-model discontinuity — a contact at the
        # contact_offset boundary, and on the mesh a nearest-triangle flip with a different normal or a switch of the
        # normal rule (step edges / corners) within SEP_EPS_1 — which are counted and capped
        touched = max(touched, (np.abs(st["contact"]).sum((1, 2)) > 0).mean())
        bad, excl = physics_mismatch(got, st, margins, sens, sep_eps=SEP_EPS_1)
        record_errors(f"terrain n={n} step {s + 1}/{steps}", got, st, excl, st_p)
        print(f"terrain n={n} step {s + 1}/{steps}: {excl.sum()} envs excluded (discontinuity margin "
              f"{((margins[:, 0] < SEP_EPS_1) | (margins[:, 1] < VEL_EPS)).sum()}, oracle-sensitive {sens.sum()}), "
              f"{bad.sum()} outside tolerance")
        for e in np.flatnonzero(bad)[:4]:  # diagnostics of a failure
            print(e, "margins", margins[e], "root", got["root"][e] - st["root"][e],
                  "dq", got["dof_pos"][e] - st["dof_pos"][e])
        assert bad.sum() == 0, (s, np.flatnonzero(bad)[:16])
        assert excl.mean() <= MAX_EXCLUDED, (s, excl.mean())
        assert np.isfinite(got["root"]).all() and np.isfinite(got["dof_vel"]).all()
        # the height scan runs on the post-step base pose: compare the scan of the GPU's own final pose through the
        # oracle (fp32 vs fp64 poses differ)
        ref_h = np.stack([np.array([oracle.height_sample(P, r, k) for r in got["root"]], np.float32)
                          for k in range(P.num_height_points)], 1)
        np.testing.assert_array_equal(got["h"], ref_h)
    assert touched > 0.5, touched  # the poses do touch the terrain
    env.close()


def test_rough_terrain_standing_and_curriculum():
    """A few hundred steps of standing on the curriculum tiles stay finite and supported; reset_idx moves
    envs that walked far a level up and places them at the new tile's origin (+ the x/y init offset)."""
    from lrl.env import LeggedRobotEnv
    n = 128
    cfg = _rough_cfg(n, 3.0, **{"terrain.num_rows": 6, "terrain.num_cols": 4, "noise.add_noise": False,
                                "domain_rand.randomize_com_displacement": False,
                                "domain_rand.randomize_base_mass": False})
    # upstream semantics: reset_idx places the robots at base_init_state over their tile origin (the fork leaves
    # custom-origin roots where they are, SURVEY Q4, so its robots would start at the creation pose on the ground)
    env = LeggedRobotEnv("cuda:0", cfg=cfg, seed=1, legacy_fork=False)
    env.reset()
    zero = torch.zeros(n, 12, device="cuda:0")
    for _ in range(100):
        env.step(zero)
    torch.cuda.synchronize()
    root = _np(env.root_states)
    assert np.isfinite(root).all()
    h = _np(env.measured_heights)
    centre = 8 * 11 + 5  # scan point (0, 0): meshgrid(x 17, y 11) 'ij' order
    above = root[:, 2] - h[:, centre]
    # supported by the mesh (no tunnelling): the base stays above the ground under it; robots dropped from the tile
    # origin height (the tile's highest point, terrain.py:182-184) into pits may lie on their side
    assert np.mean(above > 0.02) > 0.97, np.sort(above)[:10]
    assert np.mean(above > 0.1) > 0.75, np.sort(above)[:10]
    lv0 = env.terrain_levels.clone()
    ids = torch.arange(0, n, 2, device="cuda:0")
    env.root_states[ids, 0] = env.env_origins[ids, 0] + 5.0  # walked more than env_length / 2
    env.reset_idx(ids)
    torch.cuda.synchronize()
    lv = env.terrain_levels
    up = (lv0[ids] + 1).clamp(max=cfg.terrain.num_rows)
    wrapped = up >= cfg.terrain.num_rows
    assert bool((lv[ids][~wrapped] == up[~wrapped]).all())
    assert bool(((lv[ids][wrapped] >= 0) & (lv[ids][wrapped] < cfg.terrain.num_rows)).all())
    org = cfg.terrain.terrain_origins[lv[ids], env.terrain_types[ids]]
    assert torch.equal(env.env_origins[ids], org)
    xo = float(cfg.terrain.x_init_range) + float(cfg.terrain.x_init_offset)
    np.testing.assert_allclose(_np(env.root_states[ids, 0]), _np(org[:, 0]) + xo, rtol=0, atol=1e-5)
    np.testing.assert_allclose(_np(env.root_states[ids, 2]), _np(org[:, 2]) + cfg.init_state.pos[2], atol=1e-5)
    assert "terrain_level" in env.extras["train/episode"]
    env.close()


def test_native_terrain_curriculum_matches_reference():
    """lrl_sim_terrain_curriculum (the one-launch _update_terrain_curriculum of a sim-backed env) on the
    reference's fixture (tests/golden/terrain_curriculum.npz, the reference's randint_like draws injected):
    levels and origins bit-exact, as the host torch form is in tests/test_terrain.py."""
    import types
    from lrl.env import LeggedRobotEnv
    g = golden("terrain_curriculum.npz")
    n = len(g["levels_in"])
    env = LeggedRobotEnv("cuda:0", cfg=_rough_cfg(n, 2.0, **GOLDEN_TERRAIN), seed=5)
    env.terrain_levels[:] = _dev(g["levels_in"], torch.long)
    env.terrain_types[:] = _dev(g["types"], torch.long)
    env.env_origins[:] = _dev(g["env_origins_in"])
    env.root_states[:, :2] = _dev(g["root_xy"])
    env.commands[:, :2] = _dev(g["commands_xy"])
    draws = _dev(g["draws"], torch.long)
    env._rand_levels = lambda like, high: draws[:len(like)]
    cfg = types.SimpleNamespace(
        terrain=types.SimpleNamespace(curriculum=True, env_length=float(g["env_length"]),
                                      max_terrain_level=int(g["num_rows"]), terrain_origins=_dev(g["origins_table"])),
        env=types.SimpleNamespace(episode_length_s=float(g["episode_length_s"])))
    env._update_terrain_curriculum(_dev(g["ids"], torch.long), cfg)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(env.terrain_levels), g["levels_out"])
    np.testing.assert_array_equal(_np(env.env_origins), g["env_origins_out"])
    env.close()


def test_native_terrain_curriculum_matches_torch_form_on_random_inputs():
    """The one-launch terrain curriculum against the host torch form (legged_robot.py:793-818 as written, on
    CUDA tensors) over random positions, commands, levels and draws: levels and origins identical."""
    import types
    from lrl.env import LeggedRobotEnv
    n, rows, cols = 512, 6, 4
    cfg = _rough_cfg(n, 2.0, **{"terrain.num_rows": rows, "terrain.num_cols": cols})
    env = LeggedRobotEnv("cuda:0", cfg=cfg, seed=6)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    t = cfg.terrain
    env.terrain_levels[:] = torch.randint(-1, rows + 1, (n,), generator=g, device="cuda:0")
    env.terrain_types[:] = torch.randint(0, cols, (n,), generator=g, device="cuda:0")
    env.root_states[:, :2] = env.env_origins[:, :2] + (torch.rand(n, 2, generator=g, device="cuda:0") - 0.5) * 12.0
    env.commands[:, :2] = (torch.rand(n, 2, generator=g, device="cuda:0") - 0.5) * 2.0
    ids = torch.randperm(n, generator=g, device="cuda:0")[:300].sort().values
    draws = torch.randint(0, t.max_terrain_level, (len(ids),), generator=g, device="cuda:0")
    stub = types.SimpleNamespace(init_done=True, terrain_levels=env.terrain_levels.clone(),
                                 terrain_types=env.terrain_types.clone(), env_origins=env.env_origins.clone(),
                                 root_states=env.root_states.clone(), commands=env.commands.clone(),
                                 _rand_levels=lambda like, high: draws[:len(like)])
    env._rand_levels = lambda like, high: draws[:len(like)]
    LeggedRobotEnv._update_terrain_curriculum(stub, ids, cfg)   # torch form (no sim)
    env._update_terrain_curriculum(ids, cfg)                      # native
    torch.cuda.synchronize()
    assert torch.equal(env.terrain_levels, stub.terrain_levels)
    assert torch.equal(env.env_origins, stub.env_origins)
    env.close()


def test_terrain_curriculum_wraps_through_step_resets():
    """Resets driven by step() (upstream path: time-outs, int32 reset ids from lrl_sim_step_code) on the curriculum
    mesh with every env on the top level and walked past half a tile: each level wraps to the generator's own draw
    (the real _rand_levels, int64 whatever the ids' dtype), so new levels fall in [0, max) and the origins follow."""
    from lrl.env import LeggedRobotEnv
    n, rows, cols = 256, 5, 4
    cfg = _rough_cfg(n, 3.0, **{"terrain.num_rows": rows, "terrain.num_cols": cols})
    env = LeggedRobotEnv("cuda:0", cfg=cfg, seed=4, legacy_fork=False)
    env.reset()
    zero = torch.zeros(n, 12, device="cuda:0")
    env.step(zero)
    t = cfg.terrain
    env.terrain_levels[:] = t.max_terrain_level - 1
    env.root_states[:, 0] = env.env_origins[:, 0] + t.env_length  # walked more than env_length / 2: move up
    env.episode_length_buf[:] = cfg.env.max_episode_length  # every env times out in the next step
    env._due_next = None
    env.step(zero)
    torch.cuda.synchronize()
    lv = env.terrain_levels
    assert lv.dtype == torch.int64
    assert bool(((lv >= 0) & (lv < t.max_terrain_level)).all()), _np(lv)[:32]
    assert len(torch.unique(lv)) > 1  # random levels, not one fused value
    org = t.terrain_origins[lv, env.terrain_types]
    assert torch.equal(env.env_origins, org)
    m = float(env.extras["train/episode"]["terrain_level"])
    assert 0.0 <= m < t.max_terrain_level, m
    env.close()


def test_perceptive_policy_trains_on_rough_terrain():
    """The base config's perceptive layout (observe_vel + 17 x 11 height scan = 235 observations, history
    15 x 235) end to end: upstream resets on the curriculum trimesh, one Runner.learn iteration through the
    native act / update (X pitch 256) — finite losses, heights in the observations."""
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    from lrl.ppo import runner as R
    n = 256
    cfg = _rough_cfg(n, 3.0, **{"terrain.num_rows": 4, "terrain.num_cols": 4, "env.observe_vel": True,
                                "env.num_observations": 48 + 187})
    R.RunnerArgs.save_interval = 0
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=2, legacy_fork=False))
    assert env.num_obs == 235 and env.num_obs_history == 15 * 235
    runner = R.Runner(env, device="cuda:0", seed=2)
    runner.learn(1, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    obs = _np(env.env.obs_buf)
    assert np.isfinite(obs).all() and np.abs(obs[:, 48:]).max() > 0  # the scan reaches the policy
    st = runner.alg.storage
    assert torch.isfinite(st.values).all() and torch.isfinite(st.actions).all()
    p = runner.alg.actor_critic._flat
    assert torch.isfinite(p).all()
    env.env.close()
