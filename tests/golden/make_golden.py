"""Generate the golden fixtures under tests/golden/ by RUNNING the reference's own Python.

IN-CONTAINER ONLY: imports /root/reference (read-only) with the stub modules of
``_ref_stubs.py``; nothing here runs on the GPU box, and no reference source is copied.
Every random draw the reference makes (obs noise ``rand_like``, motor-strength redraw
``torch.rand``, minibatch ``randperm``, Normal samples) is injected/recorded so the fixtures do
not depend on torch-version RNG streams.

Fixtures written (all small .npz, inputs + expected outputs):
  post_physics_mc.npz / post_physics_go1.npz
      LeggedRobot.step (legged_robot.py:106-137) driven with an identity "physics" fake:
      per step the state the simulator would have produced is written into the sim tensors,
      then step() runs _compute_torques x4 (:653-688), post_physics_step (:139-188),
      teleport (:768-791), DR redraw (:544-560), check_termination (:190-202),
      compute_reward (:314-340, 12 terms), compute_observations (:342-417), clip (:133-136).
  post_physics_all_terms.npz
      the same for Mini Cheetah with all 21 _reward_* terms (:1506-1646) plus termination at non-zero
      scales and only_positive_rewards off.
  reset.npz           reset_idx (:227-290) on a subset of envs: Mini Cheetah fork (Q4), Go1 plane fork, Go1
                      upstream (custom-origin spawn draw, _resample_commands, yaw curriculum), with the
                      command curriculum, DR redraw, buffer zeroing and extras.
  curriculum.npz      RewardThresholdCurriculum set_to/sample/update/sample (curriculum.py).
  gae.npz             RolloutStorage.compute_returns (rollout_storage.py:76-90).
  ppo_update.npz      PPO.act/process_env_step/compute_returns/update (ppo.py:62-178) with
                      deterministic weights (see ``init_params``) and injected randomness.
  state_dict_keys.json  ActorCritic state-dict layout (actor_critic.py, 35 keys incl. encoder.*)
  terrain.npz         the reference's Terrain (terrain.py) over this repo's terrain_utils restatement.
  checkpoint_last.npz   the reference run's trained ac_weights_last.pt (loaded weights_only=True) and the
                      reference ActorCritic's teacher / student / value outputs on it for fixed inputs.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [generator ...]
"""
import json
import os
import sys
import types
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, REF)
import _ref_stubs  # noqa: E402

_ref_stubs.install()

from mini_gym.envs.base import legged_robot as lr_mod  # noqa: E402
from mini_gym.envs.base.legged_robot import LeggedRobot  # noqa: E402

F32_DT = float(np.float32(0.005))


# ----------------------------------------------------------------------------------------
def ns_from_class(cls):
    """Reference Cfg class tree (after the preset functions) -> SimpleNamespace tree."""
    out = types.SimpleNamespace()
    for k, v in vars(cls).items():
        if k.startswith("__"):
            continue
        if isinstance(v, type):
            v = ns_from_class(v)
        elif isinstance(v, (list, dict)):
            v = json.loads(json.dumps(v))
        setattr(out, k, v)
    return out


def fresh_cfg(robot):
    # re-import the config module so each robot starts from pristine class attributes
    for m in list(sys.modules):
        if m.startswith("mini_gym.envs.base.legged_robot_config") or m.startswith(
                "mini_gym.envs.mini_cheetah.mini_cheetah_config") or m.startswith("mini_gym.envs.go1"):
            del sys.modules[m]
    from mini_gym.envs.base.legged_robot_config import Cfg
    if robot == "mc":
        from mini_gym.envs.mini_cheetah.mini_cheetah_config import config_mini_cheetah
        config_mini_cheetah(Cfg)
    else:
        from mini_gym.envs.go1.go1_config import config_go1
        config_go1(Cfg)
    return ns_from_class(Cfg)


class FakeGym:
    """Identity 'simulator': the test writes the post-simulate state into the sim tensors."""

    def __init__(self, env):
        self.env = env

    def set_dof_actuation_force_tensor(self, sim, t):
        pass

    def simulate(self, sim):
        pass

    def fetch_results(self, sim, b):
        pass

    def refresh_dof_state_tensor(self, sim):
        pass

    def refresh_actor_root_state_tensor(self, sim):
        pass

    def refresh_net_contact_force_tensor(self, sim):
        pass

    def refresh_rigid_body_state_tensor(self, sim):
        pass

    def set_actor_root_state_tensor(self, sim, t):
        self.env.all_root_states[:] = t

    def set_actor_root_state_tensor_indexed(self, sim, t, ids, n):
        pass

    def set_dof_state_tensor_indexed(self, sim, t, ids, n):
        pass

    def find_actor_index(self, env, name, domain):
        return env


lr_mod.gymtorch.unwrap_tensor = lambda t: t
lr_mod.gymapi.DOMAIN_SIM = 0

# Isaac Gym asset order (depth first, children alphabetical): FL, FR, RL, RR
LEGS = ["FL", "FR", "RL", "RR"]
DOF_NAMES = [f"{l}_{j}_joint" for l in LEGS for j in ["hip", "thigh", "calf"]]
URDF_LIMITS = {
    # (lower, upper, effort, velocity) per joint kind, from the URDFs (mini_cheetah.urdf:104,133,162; go1.urdf)
    "mc": {"hip": (-1.6, 1.6, 18.0, 40.0), "thigh": (-2.6, 2.6, 18.0, 40.0), "calf": (-2.6, 2.6, 26.0, 26.0)},
    "go1": {"hip": (-0.802851455917, 0.802851455917, 33.5, 50.0), "thigh": (-1.0471975512, 4.18879020479, 33.5, 28.0),
            "calf": (-2.69653369433, -0.916297857297, 33.5, 28.0)},
}


def make_env(robot, n, seed, tweak=None):
    rng = np.random.default_rng(seed)
    cfg = fresh_cfg(robot)
    if tweak is not None:
        tweak(cfg)
    env = object.__new__(LeggedRobot)
    env.cfg = cfg
    env.eval_cfg = None
    env.sim_params = types.SimpleNamespace(dt=F32_DT)
    env._parse_cfg(cfg)
    env.gym = FakeGym(env)
    env.sim = None
    env.viewer = None
    env.headless = True
    env.debug_viz = False
    env.record_now = False
    env.record_eval_now = False
    env.device = "cpu"
    env.num_envs = env.num_train_envs = n
    env.num_eval_envs = 0
    env.num_obs = cfg.env.num_observations
    env.num_privileged_obs = cfg.env.num_privileged_obs
    env.num_actions = cfg.env.num_actions
    env.num_dof = env.num_dofs = 12
    env.dof_names = DOF_NAMES
    if robot == "mc":
        body_names = ["base"] + [f"{l}_{b}" for l in LEGS for b in ["hip", "thigh", "calf"]]
    else:
        body_names = ["base"] + [f"{l}_{b}" for l in LEGS for b in ["hip", "thigh", "calf", "foot"]]
    env.num_bodies = len(body_names)
    B = env.num_bodies
    idx = lambda names: torch.tensor([body_names.index(s) for s in names], dtype=torch.long)
    env.feet_indices = idx([s for s in body_names if cfg.asset.foot_name in s])
    pen = [s for nm in cfg.asset.penalize_contacts_on for s in body_names if nm in s]
    env.penalised_contact_indices = idx(pen)
    term = [s for nm in cfg.asset.terminate_after_contacts_on for s in body_names if nm in s]
    env.termination_contact_indices = idx(term)

    # limits & gains (legged_robot.py:501-516, 1012-1028)
    lim = URDF_LIMITS[robot]
    props = np.zeros(12, dtype=[("lower", np.float32), ("upper", np.float32), ("velocity", np.float32),
                                ("effort", np.float32)])
    for i, name in enumerate(DOF_NAMES):
        lo, hi, eff, vel = lim[name.split("_")[1]]
        props[i] = (lo, hi, vel, eff)
    env._process_dof_props(props, 0)  # the reference's own soft-limit arithmetic (:501-516)

    # sim tensors (identity gather indices: one actor per env)
    env.all_root_states = torch.zeros(n, 13)
    env.go1_indices = torch.arange(n)
    env.all_dof_state = torch.zeros(12 * n, 2)
    env.go1_dof_indices = torch.arange(12 * n)
    env.all_rigid_body_state = torch.zeros(B * n, 13)
    env.go1_rb_indices = torch.arange(B * n)
    env.all_contact_forces = torch.zeros(B * n, 3)
    env.custom_origins = cfg.terrain.mesh_type in ["heightfield", "trimesh"]
    if robot == "mc":
        cfg.terrain.x_offset = 0  # terrain.py:50 (set when a Terrain is built)

    # DR buffers (legged_robot.py:1032-1046, 519-542)
    env.friction_coeffs = torch.tensor(rng.uniform(0.05, 4.5, n), dtype=torch.float)
    env.restitutions = torch.tensor(rng.uniform(0, 1, n), dtype=torch.float)
    env.payloads = torch.tensor(rng.uniform(-1, 3, n), dtype=torch.float)
    env.com_displacements = torch.tensor(rng.uniform(-0.1, 0.1, (n, 3)), dtype=torch.float)
    ms = rng.uniform(0.9, 1.1, (n, 1)).repeat(12, axis=1)
    env.motor_strengths = torch.tensor(ms, dtype=torch.float)
    env.Kp_factors = torch.ones(n, 12)
    env.Kd_factors = torch.ones(n, 12)

    # buffers (base_task.py:56-63; legged_robot.py:935-1030)
    env.obs_buf = torch.zeros(n, env.num_obs)
    env.rew_buf = torch.zeros(n)
    env.reset_buf = torch.ones(n, dtype=torch.long)
    env.episode_length_buf = torch.zeros(n, dtype=torch.long)
    env.time_out_buf = torch.zeros(n, dtype=torch.bool)
    env.privileged_obs_buf = torch.zeros(n, env.num_privileged_obs)
    env.extras = {}
    env.common_step_counter = 0
    env.measured_heights = 0
    env.obs_scales = cfg.normalization.obs_scales
    env.noise_scale_vec = env._get_noise_scale_vec(cfg)
    env.gravity_vec = torch.tensor([0.0, 0.0, -1.0]).repeat((n, 1))
    env.forward_vec = torch.tensor([1.0, 0.0, 0.0]).repeat((n, 1))
    env.torques = torch.zeros(n, 12)
    env.p_gains = torch.zeros(12)
    env.d_gains = torch.zeros(12)
    env.default_dof_pos = torch.zeros(12)
    for i, name in enumerate(DOF_NAMES):
        env.default_dof_pos[i] = cfg.init_state.default_joint_angles[name]
        for k in cfg.control.stiffness:
            if k in name:
                env.p_gains[i] = cfg.control.stiffness[k]
                env.d_gains[i] = cfg.control.damping[k]
    env.default_dof_pos = env.default_dof_pos.unsqueeze(0)
    env.actions = torch.zeros(n, 12)
    env.last_actions = torch.zeros(n, 12)
    env.dof_state = env.all_dof_state[env.go1_dof_indices]
    env.dof_pos = env.dof_state.view(n, 12, 2)[..., 0]
    env.dof_vel = env.dof_state.view(n, 12, 2)[..., 1]
    env.last_dof_vel = torch.zeros(n, 12)
    env.root_states = env.all_root_states[env.go1_indices]
    env.base_quat = env.root_states[:, 3:7].clone()
    env.last_root_vel = torch.zeros(n, 6)
    env.commands = torch.zeros(n, cfg.commands.num_commands)
    env.commands_scale = torch.tensor([env.obs_scales.lin_vel, env.obs_scales.lin_vel, env.obs_scales.ang_vel])
    env.feet_air_time = torch.zeros(n, len(env.feet_indices))
    env.last_contacts = torch.zeros(n, len(env.feet_indices), dtype=torch.bool)
    env.base_lin_vel = torch.zeros(n, 3)
    env.base_ang_vel = torch.zeros(n, 3)
    env.projected_gravity = torch.zeros(n, 3)
    env.enable_viewer_sync = True
    env.init_done = True
    env._prepare_reward_function()
    return env, rng


def rand_quat(rng, n, tilt=0.6):
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(-tilt, tilt, n)
    q = np.concatenate([axis * np.sin(ang / 2)[:, None], np.cos(ang / 2)[:, None]], axis=1)
    return q.astype(np.float32)


class InjectRand:
    """Patch torch.rand_like / torch.rand during one env.step: return/record injected draws."""

    def __init__(self, noise_u, ms_rng):
        self.noise_u = noise_u
        self.ms_rng = ms_rng
        self.ms_draws = []
        self._rl, self._r = torch.rand_like, torch.rand

    def __enter__(self):
        def rand_like(t, **kw):
            assert tuple(t.shape) == tuple(self.noise_u.shape)
            return self.noise_u.clone()

        def rand(*shape, **kw):
            shape = shape[0] if len(shape) == 1 and isinstance(shape[0], (tuple, list)) else shape
            u = torch.tensor(self.ms_rng.random(tuple(shape)), dtype=torch.float)
            self.ms_draws.append(u.clone())
            return u

        torch.rand_like, torch.rand = rand_like, rand
        return self

    def __exit__(self, *a):
        torch.rand_like, torch.rand = self._rl, self._r


ALL_TERMS = dict(energy=-1e-3, energy_expenditure=-2e-3, dof_vel=-1e-4, survival=0.3, dof_vel_limits=-0.5,
                 torque_limits=-0.02, stumble=-0.4, stand_still=-0.2, feet_contact_forces=-0.01, orientation=-5.0,
                 base_height=-30.0, termination=-2.0)


def _all_terms_tweak(cfg):
    """Every reward function of legged_robot.py:1506-1646 at a non-zero scale (the presets activate 12), with
    limits low enough that the limit terms fire on the fixture's states."""
    for k, v in ALL_TERMS.items():
        setattr(cfg.rewards.scales, k, v)
    cfg.rewards.soft_dof_vel_limit = 0.05
    cfg.rewards.soft_torque_limit = 0.4
    cfg.rewards.max_contact_force = 20.0
    cfg.rewards.only_positive_rewards = False


def _control_tweak(ctl, push):
    """control_type 'V' / 'T' (legged_robot.py:672-676) and _push_robots every 5 policy steps (push_interval_s 0.1 at
    dt 0.02, max_push_vel_xy 0.5 as the presets' value; :757-766)"""
    def tweak(cfg):
        cfg.control.control_type = ctl
        if ctl == "V":  # gains of a velocity loop, so that few torques saturate at the 33.5 N m limit
            cfg.control.stiffness = {"joint": 2.0}
            cfg.control.damping = {"joint": 0.002}
        if push:
            cfg.domain_rand.push_robots = True
            cfg.domain_rand.push_interval_s = 0.1
            cfg.domain_rand.max_push_vel_xy = 0.5
    return tweak


def gen_post_physics(robot, n=16, steps=3, seed=7, tweak=None, name=None):
    env, rng = make_env(robot, n, seed, tweak)
    B = env.num_bodies
    rec = {k: [] for k in [
        "root_in", "dof_pos_in", "dof_vel_in", "contact_in", "actions", "commands", "noise_u", "ms_u", "push_u",
        "obs", "priv", "rew", "reset", "torques", "root_out", "motor_strengths", "episode_sums",
        "command_sums", "feet_air_time", "last_contacts", "episode_length", "base_lin_vel",
        "base_ang_vel", "projected_gravity", "joint_pos_target"]}
    init = dict(
        friction=env.friction_coeffs.numpy().copy(), restitution=env.restitutions.numpy().copy(),
        payload=env.payloads.numpy().copy(), com=env.com_displacements.numpy().copy(),
        motor_strengths=env.motor_strengths.numpy().copy(),
    )
    # episode lengths chosen so that some envs hit the DR interval (301) during the run
    ep0 = rng.integers(0, 1000, n)
    ep0[:4] = [300, 299, 601, 902 - 1]
    env.episode_length_buf[:] = torch.tensor(ep0)
    init["episode_length"] = ep0.copy()
    # pre-existing accumulators / stateful buffers
    for d in (env.episode_sums, env.command_sums):
        for k in d:
            d[k][:] = torch.tensor(rng.normal(size=n), dtype=torch.float)
    init["episode_sums"] = np.stack([env.episode_sums[k].numpy().copy() for k in env.episode_sums])
    init["command_sums"] = np.stack([env.command_sums[k].numpy().copy() for k in env.command_sums])
    env.feet_air_time[:] = torch.tensor(rng.uniform(0, 0.8, (n, 4)) * (rng.random((n, 4)) < 0.6), dtype=torch.float)
    env.last_contacts[:] = torch.tensor(rng.random((n, 4)) < 0.5)
    env.last_actions[:] = torch.tensor(rng.normal(size=(n, 12)) * 0.5, dtype=torch.float)
    env.last_dof_vel[:] = torch.tensor(rng.normal(size=(n, 12)), dtype=torch.float)
    init["feet_air_time"] = env.feet_air_time.numpy().copy()
    init["last_contacts"] = env.last_contacts.numpy().copy()
    init["last_actions"] = env.last_actions.numpy().copy()
    init["last_dof_vel"] = env.last_dof_vel.numpy().copy()
    env.common_step_counter = 5
    ms_rng = np.random.default_rng(seed + 1)
    for s in range(steps):
        # state "produced by physics" for this step
        root = np.zeros((n, 13), np.float32)
        if robot == "mc":
            root[:, 0] = rng.uniform(0, 80, n)
            root[:, 1] = rng.uniform(0, 160, n)
            root[:3, 0] = [1.0, 79.5, 40.0]
            root[:3, 1] = [80.0, 1.5, 159.0]
        else:
            root[:, :2] = rng.uniform(-5, 5, (n, 2))
        root[:, 2] = rng.uniform(0.2, 0.4, n)
        root[:, 3:7] = rand_quat(rng, n)
        root[:, 7:13] = rng.normal(size=(n, 6)) * 0.7
        dof_pos = (env.default_dof_pos.numpy() + rng.normal(size=(n, 12)) * 0.4).astype(np.float32)
        dof_pos[0, 2] = 2.5  # exceed soft limits
        dof_pos[1, 0] = -1.55
        dof_vel = (rng.normal(size=(n, 12)) * 3).astype(np.float32)
        contact = np.zeros((n, B, 3), np.float32)
        mask = rng.random((n, B)) < 0.35
        contact[mask] = rng.normal(size=(mask.sum(), 3)) * 2.0
        feet = env.feet_indices.numpy()
        fz = rng.uniform(-0.5, 40, (n, 4)) * (rng.random((n, 4)) < 0.6)
        contact[:, feet, 2] = fz
        contact[:, feet, 0] += rng.normal(size=(n, 4))
        contact[2] = 0.0  # an env with no contact at all
        contact[3, 0] = [0.3, 0.2, 0.9]  # |f| just above 1 N
        actions = (rng.normal(size=(n, 12)) * 1.5).astype(np.float32)
        actions[0, 0] = 150.0  # exercise action clipping
        commands = np.zeros((n, 4), np.float32)
        commands[:, :3] = rng.uniform(-1, 1, (n, 3))
        commands[4, :2] = [0.05, 0.05]  # ||cmd_xy|| < 0.1: no air-time reward
        noise_u = torch.tensor(rng.random((n, env.num_obs)), dtype=torch.float)

        env.all_root_states[:] = torch.tensor(root)
        env.all_dof_state.view(n, 12, 2)[..., 0] = torch.tensor(dof_pos)
        env.all_dof_state.view(n, 12, 2)[..., 1] = torch.tensor(dof_vel)
        env.dof_state[:] = env.all_dof_state
        env.all_contact_forces[:] = torch.tensor(contact.reshape(n * B, 3))
        env.commands[:] = torch.tensor(commands)
        with InjectRand(noise_u, ms_rng) as inj:
            obs, priv, rew, reset, extras = env.step(torch.tensor(actions))
        ms_u = np.full(n, np.nan, np.float32)
        push_u = np.full((n, 2), np.nan, np.float32)
        redraw = np.nonzero((env.episode_length_buf.numpy() % int(env.cfg.domain_rand.rand_interval)) == 0)[0]
        # torch.rand draws of this step in call order: _push_robots' (k, 2) (legged_robot.py:763-764), then the
        # motor-strength redraw's (k,) (:547)
        dr_draws = [d for d in inj.ms_draws if d.dim() == 1]
        for d in inj.ms_draws:
            if d.dim() == 2:
                pushed = np.nonzero((env.episode_length_buf.numpy() % int(env.cfg.domain_rand.push_interval)) == 0)[0]
                push_u[pushed] = d.numpy()
        if len(dr_draws):
            ms_u[redraw] = dr_draws[0].numpy()
        for k, v in dict(root_in=root, dof_pos_in=dof_pos, dof_vel_in=dof_vel, contact_in=contact,
                         actions=actions, commands=commands, noise_u=noise_u.numpy(), ms_u=ms_u, push_u=push_u,
                         obs=obs.numpy(), priv=priv.numpy(), rew=rew.numpy(),
                         reset=reset.numpy().astype(np.uint8), torques=env.torques.numpy(),
                         root_out=env.root_states.numpy(), motor_strengths=env.motor_strengths.numpy(),
                         episode_sums=np.stack([env.episode_sums[k].numpy() for k in env.episode_sums]),
                         command_sums=np.stack([env.command_sums[k].numpy() for k in env.command_sums]),
                         feet_air_time=env.feet_air_time.numpy(), last_contacts=env.last_contacts.numpy(),
                         episode_length=env.episode_length_buf.numpy(),
                         base_lin_vel=env.base_lin_vel.numpy(), base_ang_vel=env.base_ang_vel.numpy(),
                         projected_gravity=env.projected_gravity.numpy(),
                         # set by 'P' control only (:669); 'V' / 'T' never create it: our buffer stays zero
                         joint_pos_target=getattr(env, "joint_pos_target", torch.zeros(n, 12)).numpy()).items():
            rec[k].append(np.array(v, copy=True))
    out = {k: np.stack(v) for k, v in rec.items()}
    out.update({"init_" + k: v for k, v in init.items()})
    out["reward_names"] = np.array(env.reward_names)
    out["reward_scales"] = np.array([env.reward_scales[k] for k in env.reward_names])
    out["episode_sum_keys"] = np.array(list(env.episode_sums.keys()))
    out["command_sum_keys"] = np.array(list(env.command_sums.keys()))
    out["noise_scale_vec"] = env.noise_scale_vec.numpy()
    out["dof_pos_limits"] = env.dof_pos_limits.numpy()
    out["common_step_counter"] = np.array(env.common_step_counter)
    out["dt"] = np.array(env.dt)
    out["max_episode_length"] = np.array(env.max_episode_length)
    out["rand_interval"] = np.array(env.cfg.domain_rand.rand_interval)
    np.savez_compressed(os.path.join(HERE, name or f"post_physics_{robot}.npz"), **out)
    print("post_physics", robot, "reward terms:", list(env.reward_names))


# ----------------------------------------------------------------------------------------
def gen_curriculum():
    from mini_gym.envs.base.curriculum import RewardThresholdCurriculum
    c = RewardThresholdCurriculum(seed=100, x_vel=(-10.0, 10.0, 51), y_vel=(-0.6, 0.6, 2),
                                  yaw_vel=(-10.0, 10.0, 51))
    c.set_to(low=np.array([-0.6, -0.6, -1.0]), high=np.array([0.6, 0.6, 1.0]))
    w0 = c.weights.copy()
    cmds1, bins1 = c.sample(batch_size=64)
    rng = np.random.default_rng(3)
    upd_bins = bins1[:32]
    lin = rng.uniform(0, 1.0, 32) * 0.02
    ang = rng.uniform(0, 1.0, 32) * 0.01
    lin_thr = 0.8 * 1.0 * float(np.float32(0.005)) * 4
    ang_thr = 0.5 * 0.5 * float(np.float32(0.005)) * 4
    c.update(upd_bins, lin, ang, lin_thr, ang_thr, local_range=0.5)
    w1 = c.weights.copy()
    cmds2, bins2 = c.sample(batch_size=4096)
    np.savez_compressed(os.path.join(HERE, "curriculum.npz"), grid=c.grid, weights0=w0, cmds1=cmds1, bins1=bins1,
                        upd_bins=upd_bins, lin=lin, ang=ang, lin_thr=lin_thr, ang_thr=ang_thr, weights1=w1,
                        cmds2=cmds2, bins2=bins2)
    print("curriculum: nonzero bins", int((w0 > 0).sum()), "->", int((w1 > 0).sum()))


# ----------------------------------------------------------------------------------------
def gen_gae():
    from mini_gym_learn.ppo.rollout_storage import RolloutStorage
    T, N = 24, 64
    rng = np.random.default_rng(11)
    st = RolloutStorage(N, T, [42], [18], [630], [12], "cpu")
    rew = rng.normal(size=(T, N, 1)).astype(np.float32)
    val = rng.normal(size=(T, N, 1)).astype(np.float32)
    done = (rng.random((T, N, 1)) < 0.08).astype(np.uint8)
    last = rng.normal(size=(N, 1)).astype(np.float32)
    st.rewards[:] = torch.tensor(rew)
    st.values[:] = torch.tensor(val)
    st.dones[:] = torch.tensor(done)
    st.compute_returns(torch.tensor(last), 0.99, 0.95)
    np.savez_compressed(os.path.join(HERE, "gae.npz"), rewards=rew, values=val, dones=done, last_values=last,
                        returns=st.returns.numpy(), advantages=st.advantages.numpy())
    print("gae ok")


# ----------------------------------------------------------------------------------------
def init_params(module):
    """Deterministic, order-independent init shared with the repo's tests (crc32 of the name)."""
    with torch.no_grad():
        for name, p in module.named_parameters():
            r = np.random.default_rng(zlib.crc32(name.encode()))
            fan_in = p.shape[-1] if p.dim() > 1 else 1
            scale = 1.0 / np.sqrt(fan_in) if p.dim() > 1 else 0.05
            if name == "std":
                p.copy_(torch.ones_like(p))
            else:
                p.copy_(torch.tensor(r.uniform(-1, 1, tuple(p.shape)) * scale, dtype=torch.float))


def gen_ppo():
    import mini_gym_learn.ppo as P
    from mini_gym_learn.ppo.actor_critic import ActorCritic
    from mini_gym_learn.ppo.ppo import PPO

    torch.manual_seed(0)
    ac = ActorCritic(42, 18, 630, 12)
    init_params(ac)
    sd_keys = [(k, list(v.shape)) for k, v in ac.state_dict().items()]
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(sd_keys, f, indent=0)
    params0 = {k: v.detach().clone() for k, v in ac.named_parameters()}

    N, T = 16, 24
    alg = PPO(ac, device="cpu")
    alg.init_storage(N, T, [42], [18], [630], [12])
    rng = np.random.default_rng(21)
    # inputs quantised to multiples of 1/64 so the fixture compresses (values stay exact in fp32)
    q = lambda a: (np.round(a * 64) / 64).astype(np.float32)
    obs_seq = q(rng.normal(size=(T + 1, N, 42)))
    priv_seq = q(rng.normal(size=(T + 1, N, 18)))
    hist_seq = q(rng.normal(size=(T + 1, N, 630)))
    eps = q(rng.normal(size=(T, N, 12)))  # Normal.sample = mean + std * eps
    rew = rng.normal(size=(T, N)).astype(np.float32) * 0.1
    done = rng.random((T, N)) < 0.05
    perm = rng.permutation(T * N)
    actions_rec, values_rec, logp_rec, mu_rec = [], [], [], []
    orig_normal_sample = torch.distributions.Normal.sample
    for t in range(T):
        def fake_sample(self, sample_shape=torch.Size(), _t=t):
            return self.mean + self.stddev * torch.tensor(eps[_t])
        torch.distributions.Normal.sample = fake_sample
        with torch.inference_mode():
            a = alg.act(torch.tensor(obs_seq[t]), torch.tensor(priv_seq[t]), torch.tensor(hist_seq[t]))
            actions_rec.append(a.numpy().copy())
            values_rec.append(alg.transition.values.numpy().copy())
            logp_rec.append(alg.transition.actions_log_prob.numpy().copy())
            mu_rec.append(alg.transition.action_mean.numpy().copy())
            alg.process_env_step(torch.tensor(rew[t]), torch.tensor(done[t]),
                                 {"env_bins": torch.zeros(N)})
    torch.distributions.Normal.sample = orig_normal_sample
    with torch.inference_mode():
        alg.compute_returns(torch.tensor(obs_seq[T]), torch.tensor(priv_seq[T]))
    returns = alg.storage.returns.numpy().copy()
    adv = alg.storage.advantages.numpy().copy()

    # record per-minibatch lr / losses via wrappers
    lrs, kls = [], []
    orig_randperm = torch.randperm
    torch.randperm = lambda n, **kw: torch.tensor(perm)
    orig_step = alg.optimizer.step

    def step_rec(*a, **k):
        lrs.append(alg.learning_rate)
        return orig_step(*a, **k)
    alg.optimizer.step = step_rec
    mv, ms_, ma = alg.update()
    torch.randperm = orig_randperm
    params1 = {k: v.detach().numpy().copy() for k, v in ac.named_parameters()}
    out = dict(obs_seq=obs_seq, priv_seq=priv_seq, hist_seq=hist_seq, eps=eps, rew=rew, done=done.astype(np.uint8),
               perm=perm, actions=np.stack(actions_rec), values=np.stack(values_rec), logp=np.stack(logp_rec),
               mu=np.stack(mu_rec), returns=returns, advantages=adv, lrs=np.array(lrs),
               mean_value_loss=np.array(mv), mean_surrogate_loss=np.array(ms_), mean_adaptation_loss=np.array(ma))
    names = sorted(params1)
    out["param_names"] = np.array(names)
    out["param_sums"] = np.array([params1[k].astype(np.float64).sum() for k in names])
    out["param_abs_sums"] = np.array([np.abs(params1[k].astype(np.float64)).sum() for k in names])
    out["param_delta_norm"] = np.array([np.linalg.norm((params1[k] - params0[k].numpy()).astype(np.float64))
                                        for k in names])
    out["param_head"] = np.stack([np.pad(params1[k].ravel()[:16], (0, max(0, 16 - params1[k].size)))
                                  for k in names])
    np.savez_compressed(os.path.join(HERE, "ppo_update.npz"), **out)
    print("ppo: lr", lrs[:4], "losses", mv, ms_, ma)


# ----------------------------------------------------------------------------------------
CKPT = REF + "/runs/rapid-locomotion/example/train/201852.132488/checkpoints/ac_weights_last.pt"


def gen_checkpoint():
    """The reference's trained checkpoint (35-key ActorCritic state dict, loaded with weights_only=True)
    and the reference ActorCritic's outputs on it: act_teacher / act_student (adaptation module on the
    630-history) / evaluate / both latents (actor_critic.py:149-173) for fixed inputs."""
    from mini_gym_learn.ppo.actor_critic import ActorCritic
    sd = torch.load(CKPT, map_location="cpu", weights_only=True)
    ac = ActorCritic(42, 18, 630, 12)
    ac.load_state_dict(sd, strict=True)
    rng = np.random.default_rng(31)
    q = lambda a: (np.round(a * 64) / 64).astype(np.float32)
    n = 64
    obs, priv, hist = q(rng.normal(size=(n, 42))), q(rng.normal(size=(n, 18))), q(rng.normal(size=(n, 630)))
    with torch.no_grad():
        ti, si = {}, {}
        mean_t = ac.act_teacher(torch.tensor(obs), torch.tensor(priv), ti).numpy()
        mean_s = ac.act_student(torch.tensor(obs), torch.tensor(hist), si).numpy()
        value = ac.evaluate(torch.tensor(obs), torch.tensor(priv)).numpy()
    out = {"sd/" + k: v.numpy() for k, v in sd.items()}
    out.update(keys=np.array(list(sd.keys())), obs=obs, priv=priv, hist=hist, mean_teacher=mean_t,
               mean_student=mean_s, value=value, latent_teacher=ti["latents"], latent_student=si["latents"])
    np.savez_compressed(os.path.join(HERE, "checkpoint_last.npz"), **out)
    print("checkpoint:", len(sd), "tensors,", sum(v.numel() for v in sd.values()), "values")


# ----------------------------------------------------------------------------------------
def _terrain_cfg(**kw):
    c = types.SimpleNamespace(mesh_type="trimesh", curriculum=True, selected=False, terrain_kwargs=None,
                              terrain_proportions=[0.1] * 10, num_rows=3, num_cols=10, terrain_length=8.0,
                              terrain_width=8.0, horizontal_scale=0.1, vertical_scale=0.005, border_size=2.0,
                              difficulty_scale=1.0, max_platform_height=0.2, terrain_smoothness=0.005,
                              terrain_noise_magnitude=0.1, slope_treshold=0.75)
    c.__dict__.update(kw)
    return c


def gen_terrain():
    """The reference's Terrain (mini_gym/utils/terrain.py) over this repo's restatement of the un-vendored
    isaacgym.terrain_utils primitives (installed as the stub module): pins the tile layout, curriculum /
    random type selection, border and env origins; the primitives themselves stay parity-unpinned."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "rapid-locomotion-rl_amd"))
    from lrl import terrain as ours
    tu = sys.modules["isaacgym.terrain_utils"]
    for k in ("SubTerrain", "random_uniform_terrain", "pyramid_sloped_terrain", "pyramid_stairs_terrain",
              "discrete_obstacles_terrain", "stepping_stones_terrain", "convert_heightfield_to_trimesh"):
        setattr(tu, k, getattr(ours, k))
    from mini_gym.utils.terrain import Terrain
    out = {}
    for name, kw, seed in (("curriculum", {}, 3), ("random", dict(curriculum=False, num_rows=2, num_cols=3), 7)):
        np.random.seed(seed)
        c = _terrain_cfg(**kw)
        t = Terrain(c, 64)
        out[name + "_hf"] = t.height_field_raw
        out[name + "_origins"] = c.env_origins
        out[name + "_seed"] = np.array(seed)
        if name == "curriculum":
            out["curriculum_ntri"] = np.array(len(t.triangles))
            out["curriculum_vsum"] = np.array(t.vertices.astype(np.float64).sum(0))
    np.savez_compressed(os.path.join(HERE, "terrain.npz"), **out)
    print("terrain:", {k: v.shape for k, v in out.items()})


def _ref_terrain(seed=3):
    """A small curriculum terrain (3 levels x 10 types, 2 m border) built by the reference's Terrain class."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "rapid-locomotion-rl_amd"))
    from lrl import terrain as ours
    tu = sys.modules["isaacgym.terrain_utils"]
    for k in ("SubTerrain", "random_uniform_terrain", "pyramid_sloped_terrain", "pyramid_stairs_terrain",
              "discrete_obstacles_terrain", "stepping_stones_terrain", "convert_heightfield_to_trimesh"):
        setattr(tu, k, getattr(ours, k))
    from mini_gym.utils.terrain import Terrain
    np.random.seed(seed)
    c = _terrain_cfg()
    return Terrain(c, 64), c


def _rough_tweak(cfg):
    cfg.terrain.mesh_type = "trimesh"
    cfg.terrain.measure_heights = True
    cfg.terrain.curriculum = True
    cfg.env.num_height_points = len(cfg.terrain.measured_points_x) * len(cfg.terrain.measured_points_y)
    cfg.env.num_observations = 42 + cfg.env.num_height_points


def gen_heights(n=96, seed=11):
    """_get_heights (legged_robot.py:1469-1503, quat_apply_yaw math_utils.py:12-16) and the height entries
    of compute_observations (:386-389, noise :924-927) on the reference's Terrain, for random base poses
    (some outside the map, to hit the index clipping)."""
    t, tc = _ref_terrain()
    env, rng = make_env("go1", n, seed, _rough_tweak)
    env.terrain = t
    rows, cols = t.heightsamples.shape
    env.height_samples = torch.tensor(t.heightsamples).view(rows, cols)
    env.height_points = env._init_height_points(torch.arange(n), env.cfg)
    root = np.zeros((n, 13), np.float32)
    root[:, 0] = rng.uniform(-tc.border_size - 1.0, rows * tc.horizontal_scale - tc.border_size + 1.0, n)
    root[:, 1] = rng.uniform(-tc.border_size - 1.0, cols * tc.horizontal_scale - tc.border_size + 1.0, n)
    root[:, 2] = rng.uniform(0.1, 0.8, n)
    root[:, 3:7] = rand_quat(rng, n, tilt=3.0)
    env.root_states[:] = torch.tensor(root)
    env.base_quat[:] = env.root_states[:, 3:7]
    heights = env._get_heights(torch.arange(n), env.cfg)
    env.measured_heights = heights
    env.projected_gravity = torch.zeros(n, 3)
    noise_u = torch.tensor(rng.random((n, env.num_obs)), dtype=torch.float)
    with InjectRand(noise_u, rng):
        env.compute_observations()
    out = dict(hf=t.heightsamples, border_size=np.array(tc.border_size), horizontal_scale=np.array(tc.horizontal_scale),
               vertical_scale=np.array(tc.vertical_scale), root=root, heights=heights.numpy(),
               obs_heights=env.obs_buf[:, 42:].numpy(), noise_u=noise_u.numpy(),
               noise_vec=env.noise_scale_vec.numpy())
    np.savez_compressed(os.path.join(HERE, "heights.npz"), **out)
    print("heights:", {k: v.shape for k, v in out.items()})


def gen_terrain_curriculum(n=64, seed=13):
    """_update_terrain_curriculum (legged_robot.py:793-818) on the reference's terrain origins, with the
    randint_like draws of envs past the last level injected and recorded."""
    t, tc = _ref_terrain()
    env, rng = make_env("go1", n, seed, _rough_tweak)
    cfg = env.cfg
    cfg.terrain.num_rows, cfg.terrain.num_cols = tc.num_rows, tc.num_cols
    cfg.terrain.env_length = tc.env_length
    cfg.terrain.max_terrain_level = tc.num_rows
    cfg.terrain.terrain_origins = torch.from_numpy(tc.env_origins).to(torch.float)
    env.terrain_levels = torch.tensor(rng.integers(0, tc.num_rows, n), dtype=torch.long)
    env.terrain_levels[:6] = tc.num_rows - 1  # envs that will walk off the last level
    env.terrain_types = torch.tensor(rng.integers(0, tc.num_cols, n), dtype=torch.long)
    env.env_origins = cfg.terrain.terrain_origins[env.terrain_levels, env.terrain_types].clone()
    disp = rng.uniform(-6.0, 6.0, (n, 2)).astype(np.float32)
    disp[:6] = 5.0
    env.root_states[:, :2] = env.env_origins[:, :2] + torch.tensor(disp)
    env.commands[:, :2] = torch.tensor(rng.uniform(-0.6, 0.6, (n, 2)), dtype=torch.float)
    env.commands[8:12, :2] = 0.0
    levels_in, origins_in = env.terrain_levels.clone(), env.env_origins.clone()
    ids = torch.tensor(np.sort(rng.choice(n, 40, replace=False)), dtype=torch.long)
    ids[:6] = torch.arange(6)
    draws = []
    _ril = torch.randint_like

    def randint_like(x, high):
        d = torch.tensor(rng.integers(0, high, tuple(x.shape)), dtype=x.dtype)
        draws.append(d.clone())
        return d
    torch.randint_like = randint_like
    try:
        env._update_terrain_curriculum(ids, cfg)
    finally:
        torch.randint_like = _ril
    out = dict(origins_table=tc.env_origins.astype(np.float32), levels_in=levels_in.numpy(),
               types=env.terrain_types.numpy(), env_origins_in=origins_in.numpy(),
               root_xy=env.root_states[:, :2].numpy().copy(), commands_xy=env.commands[:, :2].numpy().copy(),
               ids=ids.numpy(), draws=draws[0].numpy(), levels_out=env.terrain_levels.numpy(),
               env_origins_out=env.env_origins.numpy(), env_length=np.array(tc.env_length),
               episode_length_s=np.array(cfg.env.episode_length_s), num_rows=np.array(tc.num_rows))
    np.savez_compressed(os.path.join(HERE, "terrain_curriculum.npz"), **out)
    print("terrain_curriculum:", {k: v.shape for k, v in out.items()})


class InjectResetRand:
    """Patch torch.rand during reset_idx: every draw (_randomize_dof_props' motor strength, torch_rand_float's xy
    offsets) comes from ``rng`` and is recorded in call order."""

    def __init__(self, rng):
        self.rng, self.draws, self._r = rng, [], torch.rand

    def __enter__(self):
        def rand(*shape, **kw):
            shape = shape[0] if len(shape) == 1 and isinstance(shape[0], (tuple, list)) else shape
            u = torch.tensor(self.rng.random(tuple(shape)), dtype=torch.float)
            self.draws.append(u.clone())
            return u
        torch.rand = rand
        return self

    def __exit__(self, *a):
        torch.rand = self._r


def _reset_case_tweak(case):
    def tweak(cfg):
        if case == "go1_up":  # custom origins + the upstream xy spawn draw with unequal ranges (Q8) and offsets
            cfg.terrain.mesh_type = "trimesh"
            cfg.terrain.x_init_range, cfg.terrain.y_init_range = -0.5, 0.75
            cfg.terrain.x_init_offset, cfg.terrain.y_init_offset = 0.25, -0.125
            cfg.commands.yaw_command_curriculum = True
    return tweak


def gen_reset(n=24, seed=17):
    """reset_idx (legged_robot.py:227-290) for a subset of envs, three cases:
      mc_fork  Mini Cheetah preset (trimesh, custom origins): the fork's Q4 — _reset_root_states (:724-741) writes
               the advanced-index copy root_states and pushes the unchanged all_root_states, so roots stay put;
      go1_fork Go1 preset (plane): roots to base_init_state + env origin (:736-737);
      go1_up   upstream semantics: custom origins with root_states aliasing all_root_states (the upstream view),
               _resample_commands (:595-626) inside reset_idx after the command curriculum (where the fork comments
               it out, :246), x/y init ranges -0.5 / 0.75 and init offsets, yaw command curriculum on.
    common_step_counter is a multiple of max_episode_length so _update_command_curriculum_uniform (:851-880) moves
    the command ranges.  torch.rand draws are injected and recorded."""
    out = {}
    for case, robot in (("mc_fork", "mc"), ("go1_fork", "go1"), ("go1_up", "go1")):
        env, rng = make_env(robot, n, seed, _reset_case_tweak(case))
        cfg = env.cfg
        env.custom_origins = cfg.terrain.mesh_type in ["heightfield", "trimesh"]
        env.init_done = True
        np.int = int  # Q12: the reference's _init_command_distribution uses the removed np.int alias
        env._init_command_distribution(torch.arange(n))
        env.terrain_levels = torch.zeros(n, dtype=torch.long)
        env.envs = list(range(n))  # FakeGym.find_actor_index returns the env handle = env index
        env.complete_video_frames, env.video_frames = None, []  # record_video bookkeeping (:743-748)
        i = cfg.init_state  # _init_buffers (legged_robot.py:1003-1005)
        env.base_init_state = torch.tensor(i.pos + i.rot + i.lin_vel + i.ang_vel, dtype=torch.float)
        upstream = case.endswith("_up")
        if upstream:
            env.root_states = env.all_root_states  # upstream: a view, so the custom-origin reset lands
            orig = env.update_command_curriculum

            def ucc(ids, c, episode_sums=None, _o=orig, _e=env):
                _o(ids, c)
                _e._resample_commands(ids)  # upstream position of the call the fork comments out (:246)
            env.update_command_curriculum = ucc
        B = env.num_bodies
        nz = np.flatnonzero(env.curriculum.weights > 0)
        env.env_command_bins[:] = rng.choice(nz, n)
        root = np.zeros((n, 13), np.float32)
        root[:, :3] = rng.uniform(-3, 3, (n, 3))
        root[:, 3:7] = rand_quat(rng, n)
        root[:, 7:13] = rng.normal(size=(n, 6))
        env.all_root_states[:] = torch.tensor(root)
        dof_pos = (rng.normal(size=(n, 12)) * 0.5).astype(np.float32)
        dof_vel = rng.normal(size=(n, 12)).astype(np.float32)
        env.all_dof_state.view(n, 12, 2)[..., 0] = torch.tensor(dof_pos)
        env.all_dof_state.view(n, 12, 2)[..., 1] = torch.tensor(dof_vel)
        env.dof_state[:] = env.all_dof_state
        env.env_origins = torch.tensor(rng.uniform(-20, 20, (n, 3)), dtype=torch.float)
        env.last_actions[:] = torch.tensor(rng.normal(size=(n, 12)), dtype=torch.float)
        env.last_dof_vel[:] = torch.tensor(rng.normal(size=(n, 12)), dtype=torch.float)
        env.feet_air_time[:] = torch.tensor(rng.uniform(0, 1, (n, 4)), dtype=torch.float)
        env.episode_length_buf[:] = torch.tensor(rng.integers(0, 1000, n))
        env.reset_buf = torch.zeros(n, dtype=torch.bool)
        env.time_out_buf[:] = torch.tensor(rng.random(n) < 0.4)
        env.commands[:] = torch.tensor(rng.uniform(-1, 1, (n, 4)), dtype=torch.float)
        for d in (env.episode_sums, env.command_sums):
            for k in d:
                d[k][:] = torch.tensor(rng.normal(size=n), dtype=torch.float)
        # tracking sums high enough that the uniform command curriculum widens the ranges (mean / 1001 > 0.8 * scale)
        env.episode_sums["tracking_lin_vel"][:] = torch.tensor(rng.uniform(15, 20, n), dtype=torch.float)
        env.episode_sums["tracking_ang_vel"][:] = torch.tensor(rng.uniform(7, 12, n), dtype=torch.float)
        # tracking command sums around the resampling thresholds, so some bins succeed and some do not
        ep_len = min(cfg.env.max_episode_length, int(cfg.commands.resampling_time / env.dt))
        env.command_sums["tracking_lin_vel"][:] = torch.tensor(rng.uniform(0.6, 1.0, n) * 0.02 * ep_len, dtype=torch.float)
        env.command_sums["tracking_ang_vel"][:] = torch.tensor(rng.uniform(0.3, 0.7, n) * 0.01 * ep_len, dtype=torch.float)
        env.motor_strengths[:] = torch.tensor(rng.uniform(0.9, 1.1, (n, 1)).repeat(12, 1), dtype=torch.float)
        env.common_step_counter = 2 * int(cfg.env.max_episode_length)
        env.extras = {}
        ranges0 = {k: list(map(float, v)) for k, v in cfg.command_ranges.items() if k in ("lin_vel_x", "ang_vel_yaw")}
        inp = dict(root=root, dof_pos=dof_pos, dof_vel=dof_vel, env_origins=env.env_origins.numpy().copy(),
                   last_actions=env.last_actions.numpy().copy(), last_dof_vel=env.last_dof_vel.numpy().copy(),
                   feet_air_time=env.feet_air_time.numpy().copy(), episode_length=env.episode_length_buf.numpy().copy(),
                   time_out=env.time_out_buf.numpy().astype(np.uint8), commands=env.commands.numpy().copy(),
                   episode_sums=np.stack([env.episode_sums[k].numpy().copy() for k in env.episode_sums]),
                   command_sums=np.stack([env.command_sums[k].numpy().copy() for k in env.command_sums]),
                   motor_strengths=env.motor_strengths.numpy().copy(), env_command_bins=env.env_command_bins.copy(),
                   weights=env.curriculum.weights.copy())
        ids = torch.tensor(np.sort(rng.choice(n, 14, replace=False)), dtype=torch.long)
        with InjectResetRand(np.random.default_rng(seed + 100)) as inj:
            env.reset_idx(ids)
        k = len(ids)
        u = np.full((k, 5), 0.5, np.float32)
        u[:, 0] = inj.draws[0].numpy()
        if env.custom_origins:  # torch_rand_float's (k, 2) draw (made in the fork too, into the discarded copy)
            u[:, 3:5] = inj.draws[1].numpy()
        assert len(inj.draws) == (2 if env.custom_origins else 1)
        ep = env.extras["train/episode"]
        res = dict(ids=ids.numpy(), u=u, root=env.all_root_states.numpy().copy(),
                   dof_pos=env.dof_pos.numpy().copy(), dof_vel=env.dof_vel.numpy().copy(),
                   all_dof=env.all_dof_state.view(n, 12, 2).numpy().copy(),
                   motor_strengths=env.motor_strengths.numpy().copy(), last_actions=env.last_actions.numpy().copy(),
                   last_dof_vel=env.last_dof_vel.numpy().copy(), feet_air_time=env.feet_air_time.numpy().copy(),
                   episode_length=env.episode_length_buf.numpy().copy(), reset=env.reset_buf.numpy().astype(np.uint8),
                   commands=env.commands.numpy().copy(),
                   episode_sums=np.stack([env.episode_sums[k_].numpy().copy() for k_ in env.episode_sums]),
                   command_sums=np.stack([env.command_sums[k_].numpy().copy() for k_ in env.command_sums]),
                   env_command_bins=env.env_command_bins.copy(), weights=env.curriculum.weights.copy(),
                   env_bins=env.extras["env_bins"].numpy().copy(), time_outs=env.extras["time_outs"].numpy().astype(np.uint8),
                   ep_keys=np.array(sorted(ep)), ep_values=np.array([float(ep[k_]) for k_ in sorted(ep)]),
                   lin_vel_x=np.array(cfg.command_ranges["lin_vel_x"], np.float64),
                   ang_vel_yaw=np.array(cfg.command_ranges["ang_vel_yaw"], np.float64),
                   lin_vel_x0=np.array(ranges0["lin_vel_x"]), ang_vel_yaw0=np.array(ranges0["ang_vel_yaw"]),
                   common_step_counter=np.array(env.common_step_counter))
        for key, v in inp.items():
            out[f"{case}/in_{key}"] = v
        for key, v in res.items():
            out[f"{case}/{key}"] = v
        print("reset", case, "ranges", ranges0, "->", cfg.command_ranges["lin_vel_x"], cfg.command_ranges["ang_vel_yaw"],
              "extras", sorted(ep))
    np.savez_compressed(os.path.join(HERE, "reset.npz"), **out)


def gen_high_level(n=32, T=40, seed=5):
    """HighLevelControlWrapper (scripts/high_level_play.py:30-363) driven over the scripted low-level env of
    fake_ll_env.py (the reference constructor's _load_env is replaced by it; its hard-coded cuda:0 tensors are
    made on the CPU): observations, rewards, resets, episode logging and the commands handed down, per step."""
    from fake_ll_env import FakeLowLevelEnv
    import importlib
    hlp = importlib.import_module("scripts.high_level_play")
    W = hlp.HighLevelControlWrapper
    fake = FakeLowLevelEnv(n, T, seed)
    policy = lambda ob: torch.zeros(n, 12)
    W._load_env = lambda self, num_envs, headless: (fake, policy)
    z, o = torch.zeros, torch.ones

    def cpu(fn):
        def g(*a, **k):
            k.pop("device", None)
            return fn(*a, **k)
        return g
    torch.zeros, torch.ones = cpu(z), cpu(o)
    try:
        env = W(num_envs=n)
        env.device = "cpu"
        rng = np.random.default_rng(seed + 1)
        acts = rng.uniform(-2.5, 2.5, (T, n, 3)).astype(np.float32)
        acts[:, 8:12, :2] = 0.1  # below the 0.2 command threshold
        rec = {k: [] for k in ("obs", "rew", "reset", "ep_total", "ep_distance", "ep_gs", "extra_total")}
        for t in range(T):
            obs, rew, reset, extras = env.step(torch.tensor(acts[t]))
            rec["obs"].append(obs["obs"].numpy().copy())
            rec["rew"].append(rew.numpy().copy())
            rec["reset"].append(reset.numpy().copy())
            rec["ep_total"].append(env.episode_sums["total"].numpy().copy())
            rec["ep_distance"].append(env.episode_sums["distance"].numpy().copy())
            rec["ep_gs"].append(env.episode_sums["terminal_distance_gs"].numpy().copy())
            ep = extras.get("train/episode", {})
            rec["extra_total"].append(np.float32(ep["rew_total"].item()) if "rew_total" in ep else np.float32(np.nan))
    finally:
        torch.zeros, torch.ones = z, o
    out = {k: np.stack(v) for k, v in rec.items()}
    out["actions"] = acts
    out["commands"] = np.stack([c.numpy() for c in fake.commands_log])
    np.savez_compressed(os.path.join(HERE, "high_level.npz"), **out)
    print("high_level:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    gens = dict(post_physics_mc=lambda: gen_post_physics("mc"), post_physics_go1=lambda: gen_post_physics("go1"),
                curriculum=gen_curriculum, gae=gen_gae, ppo=gen_ppo, checkpoint=gen_checkpoint, terrain=gen_terrain,
                heights=gen_heights, terrain_curriculum=gen_terrain_curriculum, high_level=gen_high_level,
                reset=gen_reset,
                post_physics_ctl_v_push=lambda: gen_post_physics("go1", tweak=_control_tweak("V", True), seed=21,
                                                                 name="post_physics_ctl_v_push.npz"),
                post_physics_ctl_t=lambda: gen_post_physics("mc", tweak=_control_tweak("T", False), seed=23,
                                                            name="post_physics_ctl_t.npz"),
                post_physics_all_terms=lambda: gen_post_physics("mc", tweak=_all_terms_tweak, seed=9,
                                                                name="post_physics_all_terms.npz"))
    for name in (sys.argv[1:] or list(gens)):
        gens[name]()
