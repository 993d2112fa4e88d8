"""Every BASELINE config at its real size on the GPU, checked against the oracle / reference.

* configs[1] (and the Go1 env of configs[4]): 4096 envs, the bench's 256-workgroup launch grid.  Post-physics
  bookkeeping through ``lrl_sim_step`` with injected draws and identity physics (the mode the reference fixtures
  pin, tests/test_oracle_golden.py) on every env: torques, targets, teleport, DR redraw, termination, episode
  counters, contact flags bit-exact; obs / priv <= 1e-6, rewards and sums <= 1e-5 rel — 3 consecutive steps from
  random states (standing, airborne, fallen; teleport band; DR redraw steps).  Then the physics on: one step of all
  4096 envs from the same states against the oracle, observations included.
* configs[2]: 4096 Go1 envs on the default 10 x 20 curriculum trimesh (legged_robot_config.py:52-57, border 50 m):
  one step of mesh physics against the oracle, and the height scan of the GPU's final poses bit-exact.
* configs[3] / [4]: gloo ranks sharing this GPU at the per-rank shape — 2 and 8 ranks of 4096 Mini Cheetah envs
  (8 x 4096 = configs[3]'s 32,768), 2 ranks of 4096 Go1 envs with the adaptation update — run one full PPO iteration
  (env + act + GAE + update): the replicas end bit-identical (parameters, both Adam moments, learning-rate trace), and
  the all-reduced first gradient equals the mean of the single-rank gradients, each recomputed by a world-1 process
  on that rank's rollout.  And the rollout does not depend on the GPU count: 2 x 2048 envs = 1 x 4096, bit for bit.
* configs[0]: scripts/test.py's run_env(16, 1000) stays finite and most robots stay up (the preset's COM / payload
  randomisation can tip a robot that only holds its default pose).
"""
import ctypes as C
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import (MAX_EXCLUDED, SEP_EPS_1, VEL_EPS, make, make_rough, oracle_sensitivity, perturb_state,
                     record_errors, within_tolerance)
from lrl import _abi
from oracle import oracle
from ranks import rank_env

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_BENCH = 4096


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


def _bookkeeping_state(rng, n, P, M, robot):
    """Random inputs for every field the post-physics step reads: poses over the whole Mini Cheetah map (teleport
    band included), velocities, contact forces around the termination / foot / collision thresholds, episode
    lengths that hit the DR redraw interval, stateful reward buffers, DR values, commands."""
    import test_env_gpu as T
    root, dof, dofv = T._random_states(rng, n, P, robot)
    root[:, 0] = rng.uniform(0.0, 80.0, n)
    root[:, 1] = rng.uniform(0.0, 160.0, n)
    B = M.num_bodies
    contact = (rng.normal(size=(n, B, 3)) * rng.choice([0.3, 3.0, 30.0], (n, B, 1))).astype(np.float32)
    contact[rng.random((n, B)) < 0.4] = 0.0
    s = dict(root=root, dof_pos=dof, dof_vel=dofv, contact=contact,
             commands=np.concatenate([rng.uniform(-1, 1, (n, 3)), np.zeros((n, 1))], 1).astype(np.float32),
             friction=rng.uniform(0.05, 4.5, n).astype(np.float32),
             restitution=rng.uniform(0, 1, n).astype(np.float32),
             payload=rng.uniform(-1, 3, n).astype(np.float32),
             com=rng.uniform(-0.1, 0.1, (n, 3)).astype(np.float32),
             motor_strength=np.repeat(rng.uniform(0.9, 1.1, (n, 1)), 12, 1).astype(np.float32),
             episode_length=rng.choice([0, 299, 300, 301, 600, 601, 602, 1000], n).astype(np.int32),
             feet_air_time=rng.uniform(0, 1, (n, 4)).astype(np.float32),
             last_contacts=(rng.random((n, 4)) < 0.5).astype(np.uint8),
             last_actions=rng.normal(size=(n, 12)).astype(np.float32),
             last_dof_vel=rng.normal(size=(n, 12)).astype(np.float32))
    anywhere = rng.random(n) < 0.5
    s["episode_length"][anywhere] = rng.integers(0, 1001, int(anywhere.sum()))
    return s


ENV_ATTR = dict(root="root_states", dof_pos="dof_pos", dof_vel="dof_vel", contact="contact_forces",
                commands="commands", friction="friction_coeffs", restitution="restitutions", payload="payloads",
                com="com_displacements", motor_strength="motor_strengths", episode_length="episode_length_buf",
                feet_air_time="feet_air_time", last_contacts="_last_contacts_u8", last_actions="last_actions",
                last_dof_vel="last_dof_vel")


def _load(env, st, s):
    for k, v in s.items():
        st[k][:] = v
        t = getattr(env, ENV_ATTR[k])
        t[:] = _dev(v, t.dtype)
    env.Kp_factors[:] = 1.0
    env.Kd_factors[:] = 1.0
    env._episode_sums[:] = 0.0
    env._command_sums[:] = 0.0


def _env(robot, n, **over):
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    cfg.env.num_envs = n
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    return LeggedRobotEnv("cuda:0", cfg=cfg)


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_bench_grid_post_physics_matches_oracle(robot):
    """configs[1] (Mini Cheetah) / the Go1 env of configs[4] at 4096 envs: three identity-physics steps, every
    post-physics output of every env against the oracle (itself pinned by the reference's post_physics_*.npz)."""
    n = N_BENCH
    cfg, rob, M, P = make(robot, **{"env.num_envs": n})
    env = _env(robot, n)
    assert (n + 15) // 16 == 256  # the bench's launch grid: 16 envs per single-wave workgroup
    rng = np.random.default_rng(41)
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    _load(env, st, _bookkeeping_state(rng, n, P, M, robot))
    flags = _abi.STEP_INJECT_UNIFORM
    redraws = 0
    for s in range(3):
        act = (rng.normal(size=(n, 12)) * 2.0).astype(np.float32)
        noise = rng.random((n, P.num_obs)).astype(np.float32)
        dr = rng.random(n).astype(np.float32)
        redraws += int(((st["episode_length"] + 1) % P.rand_interval == 0).sum())
        _step_raw(env, _dev(act), flags, _dev(noise), _dev(dr))
        oracle.env_step(M, P, st, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1)
        for k, attr in dict(torques="torques", joint_pos_target="joint_pos_target", root="root_states",
                            motor_strength="motor_strengths", reset="_reset_u8", episode_length="episode_length_buf",
                            last_contacts="_last_contacts_u8").items():
            np.testing.assert_array_equal(_np(getattr(env, attr)), st[k], err_msg=f"step {s} {k}")
        tol = dict(rtol=2e-6, atol=2e-6)
        for k, attr in dict(base_lin_vel="base_lin_vel", base_ang_vel="base_ang_vel",
                            projected_gravity="projected_gravity", feet_air_time="feet_air_time").items():
            np.testing.assert_allclose(_np(getattr(env, attr)), st[k], **tol, err_msg=f"step {s} {k}")
        np.testing.assert_allclose(_np(env.rew_buf), st["rew"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(_np(env._episode_sums), st["episode_sums"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(_np(env._command_sums), st["command_sums"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(_np(env.obs_buf), st["obs"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(_np(env.privileged_obs_buf), st["priv"], rtol=1e-6, atol=1e-6)
    # the inputs exercise what they are meant to: terminations, teleports, DR redraws, foot contacts
    assert 0.05 < st["reset"].mean() < 0.95
    assert redraws > 100
    assert st["last_contacts"].any() and not st["last_contacts"].all()
    env.close()


def _obs_within(got, st, ok_env, P):
    """Observations after a physics step: per column, the physics tolerances of helpers.within_tolerance carried
    through compute_observations (projected gravity ~ the base orientation, (q - q0) x 1, qd x 0.05; commands,
    actions and the injected noise exact)."""
    err = np.abs(got - st)
    tol = np.full(got.shape[1], 1e-6, np.float32)
    tol[0:3] = 1e-3                                         # projected gravity (rotation by a 2e-4 quaternion)
    tol[6:18] = 2e-3 * P.obs_scale_dof_pos + 1e-6           # joint angles
    vel = 0.05 + 0.01 * np.abs(st[:, 18:30])                # joint rates 5e-2 + 1 %
    bad = (err[:, :18] > tol[:18]).any(1) | (err[:, 30:] > tol[30:]).any(1) | \
          (err[:, 18:30] > vel * P.obs_scale_dof_vel + 1e-6).any(1)
    return ~bad | ~ok_env


@pytest.mark.parametrize("robot", ["mc", "go1"])
def test_bench_grid_physics_step_matches_oracle(robot):
    """configs[1] / [4] env at 4096 envs with the physics on: one step of every env from random states against the
    oracle — root / joint state / contact forces and the observations built from them; termination exact wherever
    the oracle's termination force is not within 5 % of its threshold.  Envs on a contact-model discontinuity (a
    sphere within 1e-5 m of contact_offset, a restitution switch) or whose fp64 result moves under fp32-size input
    noise are counted, capped at 6 %, and excluded."""
    import test_env_gpu as T
    n = N_BENCH
    cfg, rob, M, P = make(robot, **{"env.num_envs": n})
    env = _env(robot, n)
    rng = np.random.default_rng(43)
    root, dof, dofv = T._random_states(rng, n, P, robot)
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    s = dict(root=root, dof_pos=dof, dof_vel=dofv, friction=rng.uniform(0.05, 4.5, n).astype(np.float32),
             restitution=rng.uniform(0, 1, n).astype(np.float32), payload=rng.uniform(-1, 3, n).astype(np.float32),
             com=rng.uniform(-0.1, 0.1, (n, 3)).astype(np.float32),
             commands=np.concatenate([rng.uniform(-1, 1, (n, 3)), np.zeros((n, 1))], 1).astype(np.float32))
    _load(env, st, s)
    act = (rng.normal(size=(n, 12)) * 0.5).astype(np.float32)
    noise = rng.random((n, P.num_obs)).astype(np.float32)
    dr = rng.random(n).astype(np.float32)
    flags = _abi.STEP_PHYSICS | _abi.STEP_INJECT_UNIFORM
    _step_raw(env, _dev(act), flags, _dev(noise), _dev(dr))
    rp = np.random.default_rng(79)  # (two perturbation draws, as the plane tests: one misses lopsided spreads)
    sp, sq = perturb_state(st, rp), perturb_state(st, rp)
    m = np.zeros((n, 2))
    oracle.env_step(M, P, st, act, flags, noise_u=noise, dr_u=dr, margins=m)
    oracle.env_step(M, P, sp, act, flags, noise_u=noise, dr_u=dr)
    oracle.env_step(M, P, sq, act, flags, noise_u=noise, dr_u=dr)
    got = {k: _np(getattr(env, a)) for k, a in dict(root="root_states", dof_pos="dof_pos", dof_vel="dof_vel",
                                                      contact="contact_forces", obs="obs_buf").items()}
    excl = (m[:, 0] < SEP_EPS_1) | (m[:, 1] < VEL_EPS) | oracle_sensitivity(st, sp) | oracle_sensitivity(st, sq)
    record_errors(f"configs {robot} n={n} physics step", got, st, excl, sp)
    ok = within_tolerance(got, st) | excl
    print(f"{robot} n={n}: {excl.sum()} envs excluded, {(~ok).sum()} outside tolerance")
    for e in np.flatnonzero(~ok)[:4]:
        print("bad env", e, {k: float(np.abs(got[k][e] - st[k][e]).max()) for k in ("root", "dof_pos", "dof_vel",
                                                                                   "contact")}, "margins", m[e])
    assert ok.all(), np.flatnonzero(~ok)[:16]
    assert excl.mean() <= MAX_EXCLUDED, excl.mean()
    obs_ok = _obs_within(got["obs"], st["obs"], ~excl, P)
    assert obs_ok.all(), np.flatnonzero(~obs_ok)[:16]
    np.testing.assert_array_equal(got["obs"][:, 30:42], st["obs"][:, 30:42])  # the actions, exactly
    B = M.num_bodies
    tmask = np.array([(P.termination_mask >> b) & 1 for b in range(B)], bool)
    fmax = np.linalg.norm(st["contact"][:, tmask], axis=-1).max(axis=1)
    clear = ~excl & (np.abs(fmax - 1.0) > 0.05)
    np.testing.assert_array_equal(_np(env._reset_u8)[clear], st["reset"][clear])
    env.close()


def test_configs2_full_curriculum_trimesh_step_matches_oracle():
    """configs[2]: 4096 Go1 envs on the default curriculum trimesh (10 rows x 20 columns of 8 m tiles, border 50 m,
    proportions legged_robot_config.py:57) — one env step of mesh physics against the oracle on the same mesh, and
    the height scan of the GPU's final poses bit-exact through the oracle's sampler."""
    import test_terrain_gpu as TT
    from lrl.env import LeggedRobotEnv
    n = N_BENCH
    cfg = TT._rough_cfg(n, 50.0)
    assert (cfg.terrain.num_rows, cfg.terrain.num_cols) == (10, 20)
    env = LeggedRobotEnv("cuda:0", cfg=cfg, seed=5)
    assert env._P.terrain_mesh == 1
    cfg2, rob, M, P = make_rough(border_size=50.0)
    P.terrain_mesh = 1
    TT._oracle_terrain(env)
    rng = np.random.default_rng(9)
    root, dof, dofv = TT._poses_on_terrain(rng, env, n, P)
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5,
                           num_height_points=P.num_height_points)
    fr = rng.uniform(0.05, 4.5, n).astype(np.float32)
    rs = rng.uniform(0, 1, n).astype(np.float32)
    for k, v in dict(root=root, dof_pos=dof, dof_vel=dofv, friction=fr, restitution=rs).items():
        st[k][:] = v
    env.root_states[:] = _dev(root)
    env.dof_pos[:] = _dev(dof)
    env.dof_vel[:] = _dev(dofv)
    env.friction_coeffs[:] = _dev(fr)
    env.restitutions[:] = _dev(rs)
    env.payloads[:] = 0.0
    env.com_displacements[:] = 0.0
    act = (rng.normal(size=(n, 12)) * 0.5).astype(np.float32)
    noise = rng.random((n, P.num_obs)).astype(np.float32)
    dr = np.full(n, np.nan, np.float32)
    flags = _abi.STEP_PHYSICS | _abi.STEP_INJECT_UNIFORM
    _step_raw(env, _dev(act), flags, _dev(noise), _dev(dr))
    m = np.zeros((n, 2))
    rp = np.random.default_rng(78)  # (two perturbation draws, as the plane tests: one misses lopsided spreads)
    sp, sq = perturb_state(st, rp), perturb_state(st, rp)
    oracle.env_step(M, P, st, act, flags, noise_u=noise, dr_u=dr, margins=m)
    oracle.env_step(M, P, sp, act, flags, noise_u=noise, dr_u=dr)
    oracle.env_step(M, P, sq, act, flags, noise_u=noise, dr_u=dr)
    got = {k: _np(getattr(env, a)) for k, a in dict(root="root_states", dof_pos="dof_pos", dof_vel="dof_vel",
                                                      contact="contact_forces", h="measured_heights").items()}
    assert (np.abs(st["contact"]).sum((1, 2)) > 0).mean() > 0.4  # the poses do touch the terrain
    excl = (m[:, 0] < SEP_EPS_1) | (m[:, 1] < VEL_EPS) | oracle_sensitivity(st, sp) | oracle_sensitivity(st, sq)
    record_errors(f"configs[2] n={n} trimesh step", got, st, excl, sp)
    ok = within_tolerance(got, st) | excl
    print(f"configs[2] n={n}: {excl.sum()} envs excluded, {(~ok).sum()} outside tolerance")
    for e in np.flatnonzero(~ok)[:4]:
        print("bad env", e, "margins", m[e], "root", got["root"][e] - st["root"][e])
    assert ok.all(), np.flatnonzero(~ok)[:16]
    assert excl.mean() <= MAX_EXCLUDED, excl.mean()
    lv = _np(env.terrain_levels)
    assert len(np.unique(lv)) > 1 and len(np.unique(_np(env.terrain_types))) > 1  # envs spread over the tiles
    ref_h = np.stack([np.array([oracle.height_sample(P, r, k) for r in got["root"]], np.float32)
                      for k in range(P.num_height_points)], 1)
    np.testing.assert_array_equal(got["h"], ref_h)
    env.close()


# ------------------------------------------------------------------------------------------ configs[3] / [4]
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _iteration(robot, rank, world, tmp, n=N_BENCH, rollout_only=False, legacy_fork=True):
    """One Runner.learn iteration of ``robot`` at ``n`` envs for global rank ``rank`` (env_offset rank x n), the
    bench's setup.  The rollout the update sees (storage + the CUDA generator state its randperm draws from) and
    the initial parameters are written to ``tmp`` for the single-rank recomputation.  ``rollout_only``: the update is
    skipped, and the rollout storage plus the env's final state come back instead."""
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    from lrl.ppo import runner as R
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    cfg.env.num_envs = n
    R.RunnerArgs.save_interval = 0
    env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234, env_offset=rank * n, legacy_fork=legacy_fork))
    torch.manual_seed(0)  # same initial weights on every rank (as DDP broadcasts them)
    runner = R.Runner(env, device="cuda:0", seed=1234)
    alg = runner.alg
    alg.record_lr = True
    init = alg.actor_critic._flat.detach().clone()
    orig_update = alg.update
    roll = {}

    def update():
        s = alg.storage
        snap = {k: getattr(s, k).detach().cpu().clone() for k in STORE_KEYS}
        if rollout_only:
            roll.update({k: v.numpy().copy() for k, v in snap.items()})
            s.clear()
            return 0.0, 0.0, 0.0
        snap["cuda_rng"] = torch.cuda.get_rng_state()
        snap["init"] = init.cpu()
        snap["lr"] = alg.learning_rate
        # the update's first draw is its minibatch permutation: replay it from the same generator state
        snap["perm"] = torch.randperm(s.values.shape[0] * s.values.shape[1], device="cuda:0").cpu()
        torch.cuda.set_rng_state(snap["cuda_rng"])
        torch.save(snap, os.path.join(tmp, f"rollout_{robot}_{rank}.pt"))
        return orig_update()
    alg.update = update
    cap = []
    orig = dist.all_reduce

    def probe(t, *a, **k):  # the update's first all-reduce: minibatch 0's flat policy gradient + KL slot
        if not cap and t.numel() > 1000:
            cap.append(t.detach().cpu().numpy().copy())
            r = orig(t, *a, **k)
            cap.append(t.detach().cpu().numpy().copy())
            return r
        return orig(t, *a, **k)
    dist.all_reduce = probe
    try:
        runner.learn(1, init_at_random_ep_len=True)
    finally:
        dist.all_reduce = orig
    torch.cuda.synchronize()
    if rollout_only:
        e = env.env
        roll.update(root=_np(e.root_states).copy(), dof_pos=_np(e.dof_pos).copy(), dof_vel=_np(e.dof_vel).copy(),
                    contact=_np(e.contact_forces).copy(), hist=_np(e.obs_history_buf).copy(),
                    origins=_np(e.env_origins).copy())
        env.env.close()
        return roll
    nat = alg._native
    out = dict(params=alg.actor_critic._flat.detach().cpu().numpy().copy(),
               m=nat["exp_avg"].cpu().numpy().copy(), v=nat["exp_avg_sq"].cpu().numpy().copy(),
               lr=list(alg.lr_trace), pre=cap[0], post=cap[1],
               rew=float(alg.storage.rewards.sum()))
    env.env.close()
    return out


STORE_KEYS = ["observations", "privileged_observations", "observation_histories", "actions", "values", "returns",
              "actions_log_prob", "advantages", "mu", "sigma", "rewards", "dones"]


def _rank_worker(rank, world, port, robot, tmp, out, n=N_BENCH, rollout_only=False, legacy_fork=True):
    sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from ranks import init_rank
    init_rank(rank, world, port)
    out[rank] = _iteration(robot, rank, world, tmp, n, rollout_only, legacy_fork)
    if world > 1:
        dist.destroy_process_group()


def _autograd_first_grad(paths):
    """torch autograd of the reference's loss over minibatch 0 of each saved rank rollout (test_dist_gpu's helper),
    from the rollouts' shared initial parameters."""
    from lrl.ppo.actor_critic import ActorCritic
    from test_dist_gpu import ROLL_KEYS, autograd_union_grad
    snaps = [torch.load(p, weights_only=True) for p in paths]
    ac = ActorCritic(42, 18, 630, 12).cuda()
    ac.flatten_parameters()
    with torch.no_grad():
        ac._flat.copy_(snaps[0]["init"].cuda())
    rolls = [{k: sn[k].cuda() for k in ROLL_KEYS} for sn in snaps]
    return autograd_union_grad(ac, rolls, [sn["perm"].numpy() for sn in snaps])


def _single_rank_first_grad(path):
    """World 1: the native update on a saved rollout (same initial parameters, same CUDA generator state for its
    randperm) up to minibatch 0's optimiser step; returns that step's flat policy gradient + KL slot."""
    from lrl.ppo.actor_critic import ActorCritic
    from lrl.ppo.ppo import PPO
    snap = torch.load(path, weights_only=True)
    ac = ActorCritic(42, 18, 630, 12).cuda()
    ac.flatten_parameters()
    with torch.no_grad():
        ac._flat.copy_(snap["init"].cuda())
    alg = PPO(ac, device="cuda:0", fused=True)
    assert not alg.grad_allreduce
    T, N = snap["rewards"].shape[:2]
    alg.init_storage(N, T, [42], [18], [630], [12])
    for k in STORE_KEYS:
        getattr(alg.storage, k).copy_(snap[k].cuda())
    alg.storage.step = T
    alg.learning_rate = snap["lr"]
    L = _abi.lib()
    orig = L.lrl_ppo_optimizer_step
    cap = []

    def probe(*args):
        if not cap:
            net = alg._native["net"]
            cap.append(alg._native["grads"][net.main_begin:net.kl_slot + 1].detach().cpu().numpy().copy())
        return orig(*args)
    L.lrl_ppo_optimizer_step = probe
    try:
        torch.cuda.set_rng_state(snap["cuda_rng"])
        alg.update()
    finally:
        L.lrl_ppo_optimizer_step = orig
    return cap[0]


@pytest.mark.multiproc
@pytest.mark.timeout(900)
@pytest.mark.parametrize("robot,world", [("mc", 2), ("go1", 2), ("mc", 8)])
def test_multi_rank_full_iteration_at_bench_shape(robot, world):
    """configs[3] (Mini Cheetah, 4096 envs per rank: world 8 is its 32,768-env shape) and configs[4] (Go1, 4096 envs
    per rank, teacher PPO + adaptation update) as gloo ranks sharing this GPU: one full PPO iteration per rank.  The
    replicas end bit-identical (parameters, both Adam moments, learning-rate trace) and the all-reduced first gradient
    is the mean of the ranks' gradients, each recomputed by a world-1 update on that rank's saved rollout."""
    mgr = mp.get_context("spawn").Manager()  # (a forked server would inherit this process's HIP state)
    out = mgr.dict()
    with tempfile.TemporaryDirectory() as tmp:
        with rank_env(world):
            mp.spawn(_rank_worker, args=(world, _port(), robot, tmp, out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
        a = res[0]
        assert np.isfinite(a["params"]).all()
        assert len({r["rew"] for r in res}) == world  # the ranks stepped different envs (env_offset)
        for b in res[1:]:
            np.testing.assert_array_equal(a["params"], b["params"])
            np.testing.assert_array_equal(a["m"], b["m"])
            np.testing.assert_array_equal(a["v"], b["v"])
            assert a["lr"] == b["lr"] and len(a["lr"]) == 20
            np.testing.assert_array_equal(a["post"], b["post"])
        single = [_single_rank_first_grad(os.path.join(tmp, f"rollout_{robot}_{r}.pt")) for r in range(world)]
        g_ref, kl_ref = _autograd_first_grad([os.path.join(tmp, f"rollout_{robot}_{r}.pt") for r in range(world)])
    for r in range(world):
        np.testing.assert_allclose(res[r]["pre"], single[r], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(a["post"] / world, sum(single) / world, rtol=1e-6, atol=1e-8)
    assert np.abs(single[0] - single[1]).max() > 1e-4
    # pinned to the reference's loss as well: the all-reduced gradient / world is torch autograd's
    # gradient of the mean minibatch-0 loss over every rank's rollout (one process holding all the envs)
    got = a["post"][:-1] / world
    err = np.abs(got - g_ref).max()
    assert err <= 1e-4 * np.abs(g_ref).max() + 1e-7, (err, np.abs(g_ref).max())
    np.testing.assert_allclose(a["post"][-1] / world, kl_ref, rtol=1e-4, atol=1e-7)


@pytest.mark.multiproc
@pytest.mark.timeout(600)
@pytest.mark.parametrize("legacy_fork,n", [(True, N_BENCH), (False, N_BENCH), (False, 512)])
def test_rollout_does_not_depend_on_the_gpu_count(legacy_fork, n):
    """every draw is keyed by the global env id (env: env_offset; policy noise: PPO.row_offset) and the
    env origins are the global layout's, so 2 ranks x 2048 Mini Cheetah envs roll out exactly what 1 x 4096 does: a
    24-step Runner rollout's storage (observations, histories, actions, values, log-probs, means, rewards, dones,
    returns) and the final env state are bit-identical per global env; the advantages, normalised with all-reduced
    statistics (another summation order), agree to fp32 rounding.  With the upstream resets (legacy_fork=False) the
    reset draws too; at 512 envs some step resets envs of one shard only."""
    mgr = mp.get_context("spawn").Manager()  # (a forked server would inherit this process's HIP state)
    one, two = mgr.dict(), mgr.dict()
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_rank_worker, args=(1, 0, "mc", tmp, one, n, True, legacy_fork), nprocs=1, join=True)
        mp.spawn(_rank_worker, args=(2, _port(), "mc", tmp, two, n // 2, True, legacy_fork), nprocs=2, join=True)
    ref = one[0]
    h = n // 2
    bad = []  # every differing key, located by (step, env, field), before the assertion
    for k in STORE_KEYS + ["root", "dof_pos", "dof_vel", "contact", "hist", "origins"]:
        whole = ref[k]
        ax = 1 if k in STORE_KEYS else 0  # storage is [T, N, ...]
        parts = np.concatenate([two[0][k], two[1][k]], axis=ax)
        if k == "advantages":
            ne = np.abs(parts - whole) > 2e-6 * max(1.0, np.abs(whole).max())
        else:
            ne = parts != whole
        if ne.any():
            idx = np.argwhere(ne.reshape(ne.shape[:2] + (-1,)) if ne.ndim > 2 else ne)
            cols = [np.unique(idx[:, c])[:16].tolist() for c in range(idx.shape[1])]
            bad.append(f"{k}: {int(ne.sum())} differ, max |d| {np.abs(parts.astype(np.float64) - whole.astype(np.float64))[ne].max():.3e}, indices {cols}")
    assert not bad, "\n".join(bad)
    assert np.abs(ref["actions"][:, :h] - ref["actions"][:, h:]).max() > 0.1  # the halves are different envs
    if not legacy_fork:  # upstream resets happened; at 512 envs some step resets envs of one shard only (ADVICE r4:
        # the reset draws are keyed by each env's own reset count, not by a per-process counter that only that shard's
        # resets advance)
        d = ref["dones"].reshape(ref["dones"].shape[0], -1).astype(bool)
        one_sided = (d[:, :h].any(1) != d[:, h:].any(1)).sum()
        assert d.any() and (n > 512 or one_sided > 0), (d.sum(), one_sided)


# ------------------------------------------------------------------------------------------ configs[0]
def test_configs0_scripts_test_run_env():
    """configs[0]: the reference's scripts/test.py loop (16 Mini Cheetah envs, reset, 1000 zero-action steps;
    scripts/test.py here) — the state stays finite and the robots stay up."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("lrl_scripts_test", os.path.join(ROOT, "scripts", "test.py"))
    script = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(script)
    env = script.run_env(16, 1000)
    root = _np(env.root_states)
    assert np.isfinite(root).all() and np.isfinite(_np(env.dof_vel)).all()
    # the preset randomises the base COM by up to 10 cm and the payload by -1..3 kg (mini_cheetah_config.py:87-105):
    # a robot holding its default pose under zero actions can tip over (MI355X: 14 of 16 upright; without that DR
    # every robot stands, test_env_gpu.py::test_standing_settles)
    up = _np(env.projected_gravity)[:, 2] < -0.8
    print("configs[0]: upright", up.mean(), "base z", root[:, 2].round(3))
    assert up.mean() >= 0.75, up.mean()
    assert int(_np(env.episode_length_buf).max()) == 1001  # the fork never resets
    env.close()
