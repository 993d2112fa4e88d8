"""Cfg tree + robot model table -> the ``lrl_model`` / ``lrl_env_params`` structs of include/lrl.h.

This is the host half of LeggedRobot's construction: ``_parse_cfg`` (legged_robot.py:1417-1429),
``_process_dof_props`` soft limits (:501-516), PD gains by joint-name substring and default joint
angles (:1012-1028), body index sets (:1201-1207, 1283-1300), ``_prepare_reward_function``
(:1074-1110: zero scales dropped, the rest multiplied by dt, declaration order kept),
``_get_noise_scale_vec`` (:882-932) and ``get_scale_shift`` for the privileged obs (math_utils.py:35-38).
"""
import math

import numpy as np

from . import _abi

F32 = lambda x: float(np.float32(x))


def get_scale_shift(rng):
    return 2.0 / (rng[1] - rng[0]), (rng[1] + rng[0]) / 2.0


def sim_dt(cfg):
    return F32(cfg.sim.dt)  # gymapi.SimParams.dt is a C float


CONTROL_TYPES = ("P", "V", "T")  # lrl_env_params.control_type 0 / 1 / 2 (legged_robot.py:667-676)


def policy_dt(cfg):
    return cfg.control.decimation * sim_dt(cfg)  # legged_robot.py:1418 (python double of a float32)


def derived(cfg):
    """Fields _parse_cfg writes back into the config (legged_robot.py:1417-1429)."""
    dt = policy_dt(cfg)
    cfg.command_ranges = vars(cfg.commands)
    if cfg.terrain.mesh_type not in ("heightfield", "trimesh"):
        cfg.terrain.curriculum = False
    cfg.env.max_episode_length = float(np.ceil(cfg.env.episode_length_s / dt))
    cfg.domain_rand.push_interval = float(np.ceil(cfg.domain_rand.push_interval_s / dt))
    cfg.domain_rand.rand_interval = float(np.ceil(cfg.domain_rand.rand_interval_s / dt))
    return dt


def reward_layout(cfg):
    """(names of reward_scales after zero removal in order, {name: scale*dt})."""
    dt = policy_dt(cfg)
    scales = {}
    for k, v in vars(cfg.rewards.scales).items():
        if v != 0:
            scales[k] = v * dt
    return list(scales), scales


def noise_vec(cfg):
    """legged_robot.py:882-932 (only the layouts the kernel implements)."""
    ns, lvl, s = cfg.noise.noise_scales, cfg.noise.noise_level, cfg.normalization.obs_scales
    parts = []
    if cfg.env.observe_vel:
        parts += [ns.lin_vel * lvl * s.lin_vel] * 3 + [ns.ang_vel * lvl * s.ang_vel] * 3
    parts += [ns.gravity * lvl] * 3
    if cfg.env.observe_command:
        parts += [0.0] * 3
    parts += [ns.dof_pos * lvl * s.dof_pos] * 12 + [ns.dof_vel * lvl * s.dof_vel] * 12 + [0.0] * 12
    if cfg.terrain.measure_heights:  # :924-927
        parts += [ns.height_measurements * lvl * s.height_measurements] * len(height_points(cfg))
    return np.array(parts, np.float32)


def height_points(cfg):
    """_init_height_points (legged_robot.py:1453-1467): meshgrid(x, y) ('ij'), flattened -> [(x, y)]."""
    t = cfg.terrain
    gx, gy = np.meshgrid(np.array(t.measured_points_x, np.float32), np.array(t.measured_points_y, np.float32),
                         indexing="ij")
    return np.stack([gx.ravel(), gy.ravel()], -1)


def build_model(robot):
    m = _abi.LrlModel()
    _abi.fill(m, num_bodies=robot["num_bodies"], body_leg=robot["body_leg"], body_link=robot["body_link"],
              joint_xyz=robot["joint_xyz"], joint_quat=robot["joint_quat"], joint_axis=robot["joint_axis"],
              foot_xyz=robot["foot_xyz"], base_mass=robot["base_mass"], base_com=robot["base_com"],
              base_inertia=robot["base_inertia"], link_mass=robot["link_mass"], link_com=robot["link_com"],
              link_inertia=robot["link_inertia"], num_spheres=robot["num_spheres"],
              sphere_body=robot["sphere_body"], sphere_pos=robot["sphere_pos"],
              sphere_radius=robot["sphere_radius"], dof_lower=robot["dof_lower"], dof_upper=robot["dof_upper"],
              dof_effort=robot["dof_effort"], dof_velocity=robot["dof_velocity"])
    if robot["num_bodies"] > _abi.MAX_BODIES or robot["num_spheres"] > _abi.MAX_SPHERES:
        raise ValueError("robot model exceeds liblrl limits")
    if robot.get("num_hulls", 0):  # mesh colliders' support tables (lrl/robot.py support_table; ABI 6)
        tab = np.ascontiguousarray(robot["hull_table"], np.float32)
        _abi.fill(m, sphere_hull=robot["sphere_hull"], num_hulls=robot["num_hulls"], hull_res=robot["hull_res"],
                  hull_k=robot["hull_k"])
        m.hull_table = tab.ctypes.data
        m._hull_table = tab  # (keeps the host table alive as long as the model)
    return m


def body_sets(cfg, robot):
    names = robot["body_names"]
    feet = [i for i, s in enumerate(names) if cfg.asset.foot_name in s]
    pen = [i for key in cfg.asset.penalize_contacts_on for i, s in enumerate(names) if key in s]
    term = [i for key in cfg.asset.terminate_after_contacts_on for i, s in enumerate(names) if key in s]
    return feet, pen, term


def build_params(cfg, robot, auto_reset=False, solver_iterations=None, baumgarte=0.2, terrain_mesh=0,
                 joint_limits=True, joint_limit_margin=0.02, self_collisions=None, solver_type=None):
    """terrain_mesh: 1 when the sim collides with a generated height field / trimesh (lrl_sim_set_terrain),
    0 for the plane z = 0 (mesh_type 'plane', or a trimesh whose heights are all zero).
    joint_limits: enforce the URDF joint position limits in the contact solve (Isaac Gym / PhysX always enforces
    them for limited revolute joints: the reference has no switch); joint_limit_margin: activation window, rad.
    self_collisions: None follows Cfg.asset.self_collisions (0 = enabled, Isaac Gym's filter semantics: both presets
    enable it, mini_cheetah_config.py:44, go1_config.py:44); True / False override.
    solver_type: None follows Cfg.sim.physx.solver_type (1 = TGS, legged_robot_config.py:247; 0 = PGS); the
    terrain-mesh build always solves with PGS."""
    dt = derived(cfg)
    P = _abi.LrlEnvParams()
    dof_names = robot["dof_names"]
    p_gains, d_gains, default = [], [], []
    for name in dof_names:
        default.append(cfg.init_state.default_joint_angles[name])
        kp = kd = 0.0
        for key in cfg.control.stiffness:
            if key in name:
                kp, kd = cfg.control.stiffness[key], cfg.control.damping[key]
        p_gains.append(kp)
        d_gains.append(kd)
    lo, hi = np.array(robot["dof_lower"]), np.array(robot["dof_upper"])
    mid, rng = (lo + hi) / 2, hi - lo
    soft = cfg.rewards.soft_dof_pos_limit
    # legged_robot.py:512-515 evaluates these in float32 tensor arithmetic
    lo32, hi32 = lo.astype(np.float32), hi.astype(np.float32)
    m32, r32 = (lo32 + hi32) / np.float32(2), hi32 - lo32
    soft_lo = (m32 - np.float32(0.5) * r32 * np.float32(soft)).astype(np.float32)
    soft_hi = (m32 + np.float32(0.5) * r32 * np.float32(soft)).astype(np.float32)
    del mid, rng
    feet, pen, term = body_sets(cfg, robot)
    if len(feet) != 4:
        raise ValueError(f"expected 4 feet matching {cfg.asset.foot_name!r}, got {feet}")
    keys, scales = reward_layout(cfg)
    terms, tscale, slots = [], [], []
    term_scale, term_slot = 0.0, -1
    for i, k in enumerate(keys):
        if k == "termination":
            term_scale, term_slot = scales[k], i
            continue
        if k not in _abi.REWARD_TERMS:
            raise AttributeError(f"'LeggedRobot' object has no attribute '_reward_{k}'")  # as :1093 would
        terms.append(_abi.REWARD_TERMS.index(k))
        tscale.append(F32(scales[k]))
        slots.append(i)
    nv = noise_vec(cfg)
    n_obs = cfg.env.num_observations
    if len(nv) != n_obs:
        raise ValueError(f"observation layout has {len(nv)} entries but num_observations={n_obs}")
    for flag in ("observe_only_ang_vel", "observe_only_lin_vel", "observe_yaw"):
        if getattr(cfg.env, flag):
            raise ValueError(f"Cfg.env.{flag} is not implemented by the fused kernel")
    mt = cfg.terrain.mesh_type
    if cfg.terrain.measure_heights and mt == "none":
        raise NameError("Can't measure height with terrain mesh type 'none'")  # :1484-1485
    hp = height_points(cfg) if cfg.terrain.measure_heights else np.zeros((0, 2), np.float32)
    if len(hp) > _abi.MAX_HEIGHT_POINTS:
        raise ValueError(f"{len(hp)} height points exceed liblrl's {_abi.MAX_HEIGHT_POINTS}")
    cfg.env.num_height_points = len(hp)
    ctl = cfg.control.control_type
    if ctl == "P_compliantfeet":  # legged_robot.py:677-681 indexes DOF 15 of the 12 (spring_idxs = [3, 7, 11, 15])
        raise IndexError("index 15 is out of bounds for dimension 0 with size 12")
    if ctl not in CONTROL_TYPES:
        raise NameError(f"Unknown controller type: {ctl}")  # :682-683
    dr0 = cfg.domain_rand
    push_max = float(dr0.max_push_vel_xy)
    nrm = cfg.normalization
    priv = [get_scale_shift(nrm.friction_range), get_scale_shift(nrm.restitution_range),
            get_scale_shift(nrm.added_mass_range), get_scale_shift(nrm.com_displacement_range),
            get_scale_shift(nrm.motor_strength_range)]
    flags = [cfg.env.priv_observe_friction, cfg.env.priv_observe_restitution, cfg.env.priv_observe_base_mass,
             cfg.env.priv_observe_com_displacement, cfg.env.priv_observe_motor_strength]
    priv_scale = [s if f else 0.0 for (s, _), f in zip(priv, flags)]
    priv_shift = [sh for _, sh in priv]
    dr = cfg.domain_rand
    physx = cfg.sim.physx
    s = cfg.normalization.obs_scales
    init = list(cfg.init_state.pos) + list(cfg.init_state.rot) + list(cfg.init_state.lin_vel) + \
        list(cfg.init_state.ang_vel)
    _abi.fill(
        P, sim_dt=sim_dt(cfg), decimation=cfg.control.decimation, dt=F32(dt), gravity=cfg.sim.gravity,
        contact_offset=physx.contact_offset, max_depenetration_velocity=physx.max_depenetration_velocity,
        bounce_threshold_velocity=physx.bounce_threshold_velocity, ground_friction=cfg.terrain.static_friction,
        ground_restitution=cfg.terrain.restitution,
        solver_iterations=solver_iterations or physx.num_position_iterations, baumgarte=baumgarte,
        control_type=CONTROL_TYPES.index(ctl), action_scale=cfg.control.action_scale, hip_scale_reduction=cfg.control.hip_scale_reduction,
        clip_actions=cfg.normalization.clip_actions, p_gains=p_gains, d_gains=d_gains, default_dof_pos=default,
        torque_limits=robot["dof_effort"], soft_dof_pos_lower=soft_lo.tolist(), soft_dof_pos_upper=soft_hi.tolist(),
        dof_vel_limits=robot["dof_velocity"], num_feet=4, feet=feet,
        termination_mask=sum(1 << b for b in set(term)), penalised_mask=sum(1 << b for b in set(pen)),
        num_reward_terms=len(terms), reward_term=terms, reward_scale=tscale, reward_slot=slots,
        num_sum_keys=len(keys), termination_scale=F32(term_scale), termination_slot=term_slot,
        only_positive_rewards=int(cfg.rewards.only_positive_rewards), tracking_sigma=cfg.rewards.tracking_sigma,
        tracking_sigma_yaw=cfg.rewards.tracking_sigma_yaw, base_height_target=cfg.rewards.base_height_target,
        soft_dof_vel_limit=cfg.rewards.soft_dof_vel_limit, soft_torque_limit=cfg.rewards.soft_torque_limit,
        max_contact_force=cfg.rewards.max_contact_force,
        use_terminal_body_height=int(cfg.rewards.use_terminal_body_height),
        terminal_body_height=cfg.rewards.terminal_body_height, num_obs=n_obs, observe_vel=int(cfg.env.observe_vel),
        observe_command=int(cfg.env.observe_command), obs_scale_lin_vel=s.lin_vel, obs_scale_ang_vel=s.ang_vel,
        obs_scale_dof_pos=s.dof_pos, obs_scale_dof_vel=s.dof_vel, commands_scale=[s.lin_vel, s.lin_vel, s.ang_vel],
        add_noise=int(cfg.noise.add_noise), noise_vec=nv.tolist(), clip_obs=nrm.clip_observations,
        priv_scale=priv_scale, priv_shift=priv_shift, rand_interval=int(cfg.domain_rand.rand_interval),
        randomize_motor_strength=int(dr.randomize_motor_strength), randomize_kp=int(dr.randomize_Kp_factor),
        randomize_kd=int(dr.randomize_Kd_factor), motor_strength_range=dr.motor_strength_range,
        kp_range=dr.Kp_factor_range, kd_range=dr.Kd_factor_range,
        teleport=int(cfg.terrain.teleport_robots and cfg.terrain.mesh_type in ("heightfield", "trimesh")),
        teleport_thresh=cfg.terrain.teleport_thresh,
        teleport_x_offset=float(getattr(cfg.terrain, "x_offset", 0)) * cfg.terrain.horizontal_scale,
        terrain_length=cfg.terrain.terrain_length, terrain_width=cfg.terrain.terrain_width,
        terrain_rows=cfg.terrain.num_rows, terrain_cols=cfg.terrain.num_cols, base_init_state=init,
        num_history=cfg.env.num_observation_history, auto_reset=int(auto_reset),
        max_episode_length=int(cfg.env.max_episode_length),
        terrain_mesh=int(terrain_mesh), border_size=cfg.terrain.border_size,
        horizontal_scale=cfg.terrain.horizontal_scale, vertical_scale=cfg.terrain.vertical_scale,
        measure_heights=int(cfg.terrain.measure_heights), num_height_points=len(hp),
        height_points=hp.tolist(), obs_scale_height=s.height_measurements, num_train_envs=2 ** 30,
        teleport_x_offset_eval=float(getattr(cfg.terrain, "x_offset", 0)) * cfg.terrain.horizontal_scale,
        dr_span=[float(r[1]) - float(r[0]) for r in (dr.motor_strength_range, dr.Kp_factor_range, dr.Kd_factor_range)],
        joint_limits=int(joint_limits), joint_limit_margin=joint_limit_margin,
        self_collisions=int(cfg.asset.self_collisions == 0 if self_collisions is None else self_collisions),
        # torch_rand_float(-max, max, (k, 2)) = (max - -max) * torch.rand + -max (legged_robot.py:763-764)
        push_robots=int(bool(dr0.push_robots)), push_interval=int(cfg.domain_rand.push_interval),
        push_lo=-push_max, push_span=push_max - (-push_max),
        solver_tgs=int((physx.solver_type if solver_type is None else solver_type) == 1 and not terrain_mesh),
    )
    return P
