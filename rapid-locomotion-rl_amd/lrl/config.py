"""Environment / training configuration tree with the reference's attribute paths.

Mirrors the surface of ``Cfg`` (mini_gym/envs/base/legged_robot_config.py:6-256) and the robot
presets ``config_mini_cheetah`` (mini_gym/envs/mini_cheetah/mini_cheetah_config.py:8-105) and
``config_go1`` (mini_gym/envs/go1/go1_config.py:8-107): the same section names, field names and
values, so that code written against ``Cfg.env.num_envs`` / ``vars(Cfg.rewards.scales)`` keeps
working.  The tree is built from plain dict specs into ``Section`` namespaces (no params_proto):
``vars(section)`` returns fields in declaration order, which fixes the reward-term order
(legged_robot.py:1079-1093).
"""
import copy
import types
import weakref

ROOT = None  # filled by lrl/__init__.py: directory holding resources/


_PATHS = {}  # id(Section) -> (weak ref, its dotted path in the tree: "terrain", "rewards.scales"), for _update's prefixes


def _update_fields(obj, names, own_paths, d=None, **kwargs):
    """params_proto's ``_update(deps)`` (scripts/play.py:30-44 restores a run's parameters with it): every key of
    ``d`` / ``kwargs`` that names a field of ``obj`` — plainly (``mesh_type``) or under the node's own prefix
    (``terrain.mesh_type``, ``Cfg.terrain.mesh_type``) — sets it; other keys are left for the other nodes."""
    items = dict(d or {}, **kwargs)
    for k, v in items.items():
        prefix, _, leaf = str(k).rpartition(".")
        if leaf not in names:
            continue
        if prefix and not any(prefix == p or prefix.endswith("." + p) for p in own_paths):
            continue
        setattr(obj, leaf, copy.deepcopy(v))


class ArgsProto:
    """Base of the algorithm argument classes (AC_Args, PPO_Args, RunnerArgs): ``Cls._update(dict)`` as params_proto's
    PrefixProto, keys plain or prefixed with the class name."""

    @classmethod
    def _update(cls, d=None, **kwargs):
        _update_fields(cls, {k for k in vars(cls) if not k.startswith("_")}, (cls.__name__,), d, **kwargs)


class Section(types.SimpleNamespace):
    """A config node; attribute access like the reference's PrefixProto classes."""

    def _update(self, d=None, **kwargs):
        ref, path = _PATHS.get(id(self), (None, None))
        path = path if ref is not None and ref() is self else None
        _update_fields(self, set(vars(self)), (path,) if path else (), d, **kwargs)

    def to_dict(self):
        out = {}
        for k, v in vars(self).items():
            out[k] = v.to_dict() if isinstance(v, Section) else copy.deepcopy(v)
        return out


def _build(spec, path=""):
    sec = Section()
    if path:
        _PATHS[id(sec)] = (weakref.ref(sec), path)
    for k, v in spec.items():
        setattr(sec, k, _build(v, f"{path}.{k}" if path else k)
                if isinstance(v, dict) and not k.endswith(("_angles", "stiffness", "damping")) else copy.deepcopy(v))
    return sec


# Base defaults (legged_robot_config.py:7-256), field order preserved.
_BASE = {
    "env": dict(num_envs=4096, num_observations=235, num_privileged_obs=18, privileged_future_horizon=1,
                num_actions=12, num_observation_history=15, env_spacing=3.0, send_timeouts=True,
                episode_length_s=20, observe_vel=True, observe_only_ang_vel=False, observe_only_lin_vel=False,
                observe_yaw=False, observe_command=True, record_video=True, priv_observe_friction=True,
                priv_observe_restitution=True, priv_observe_base_mass=True, priv_observe_com_displacement=True,
                priv_observe_motor_strength=True, priv_observe_Kp_factor=True, priv_observe_Kd_factor=True),
    "terrain": dict(mesh_type="trimesh", horizontal_scale=0.1, vertical_scale=0.005, border_size=0,
                    curriculum=True, static_friction=1.0, dynamic_friction=1.0, restitution=0.0,
                    terrain_noise_magnitude=0.1, terrain_smoothness=0.005, measure_heights=True,
                    measured_points_x=[round(-0.8 + 0.1 * i, 1) for i in range(17)],
                    measured_points_y=[round(-0.5 + 0.1 * i, 1) for i in range(11)],
                    selected=False, terrain_kwargs=None, min_init_terrain_level=0, max_init_terrain_level=5,
                    terrain_length=8.0, terrain_width=8.0, num_rows=10, num_cols=20,
                    terrain_proportions=[0.1, 0.1, 0.35, 0.25, 0.2], slope_treshold=0.75, difficulty_scale=1.0,
                    x_init_range=1.0, y_init_range=1.0, x_init_offset=0.0, y_init_offset=0.0,
                    teleport_robots=True, teleport_thresh=2.0, max_platform_height=0.2),
    "commands": dict(command_curriculum=False, max_reverse_curriculum=1.0, max_forward_curriculum=1.0,
                     forward_curriculum_threshold=0.8, yaw_command_curriculum=False, max_yaw_curriculum=1.0,
                     yaw_curriculum_threshold=0.5, num_commands=4, resampling_time=10.0, heading_command=True,
                     global_reference=False, num_lin_vel_bins=20, lin_vel_step=0.3, num_ang_vel_bins=20,
                     ang_vel_step=0.3, distribution_update_extension_distance=1, curriculum_seed=100,
                     lin_vel_x=[-1.0, 1.0], lin_vel_y=[-1.0, 1.0], ang_vel_yaw=[-1, 1],
                     body_height_cmd=[-0.05, 0.05], impulse_height_commands=False,
                     limit_vel_x=[-10.0, 10.0], limit_vel_y=[-0.6, 0.6], limit_vel_yaw=[-10.0, 10.0],
                     heading=[-3.14, 3.14]),
    "init_state": dict(pos=[0.0, 0.0, 1.0], rot=[0.0, 0.0, 0.0, 1.0], lin_vel=[0.0, 0.0, 0.0],
                       ang_vel=[0.0, 0.0, 0.0], default_joint_angles={"joint_a": 0.0, "joint_b": 0.0}),
    "control": dict(control_type="P", stiffness={"joint_a": 10.0, "joint_b": 15.0},
                    damping={"joint_a": 1.0, "joint_b": 1.5}, action_scale=0.5, hip_scale_reduction=1.0,
                    decimation=4),
    "asset": dict(file="", foot_name="None", penalize_contacts_on=[], terminate_after_contacts_on=[],
                  disable_gravity=False, collapse_fixed_joints=True, fix_base_link=False,
                  default_dof_drive_mode=3, self_collisions=0, replace_cylinder_with_capsule=True,
                  flip_visual_attachments=True, density=0.001, angular_damping=0.0, linear_damping=0.0,
                  max_angular_velocity=1000.0, max_linear_velocity=1000.0, armature=0.0, thickness=0.01),
    "domain_rand": dict(rand_interval_s=10, randomize_friction=True, friction_range=[0.5, 1.25],
                        randomize_restitution=False, restitution_range=[0, 1.0], randomize_base_mass=False,
                        added_mass_range=[-1.0, 1.0], randomize_com_displacement=False,
                        com_displacement_range=[-0.15, 0.15], randomize_motor_strength=False,
                        motor_strength_range=[0.9, 1.1], randomize_Kp_factor=False, Kp_factor_range=[0.8, 1.3],
                        randomize_Kd_factor=False, Kd_factor_range=[0.5, 1.5], push_robots=True,
                        push_interval_s=15, max_push_vel_xy=1.0),
    "rewards": dict(only_positive_rewards=True, tracking_sigma=0.25, tracking_sigma_lat=0.25,
                    tracking_sigma_long=0.25, tracking_sigma_yaw=0.25, soft_dof_pos_limit=1.0,
                    soft_dof_vel_limit=1.0, soft_torque_limit=1.0, base_height_target=1.0, max_contact_force=100.0,
                    use_terminal_body_height=False, terminal_body_height=0.20,
                    scales=dict(termination=-0.0, tracking_lin_vel=1.0, tracking_ang_vel=0.5, lin_vel_z=-2.0,
                                ang_vel_xy=-0.05, orientation=-0.0, torques=-0.00001, dof_vel=-0.0,
                                dof_acc=-2.5e-7, base_height=-0.0, feet_air_time=1.0, collision=-1.0,
                                feet_stumble=-0.0, action_rate=-0.01, stand_still=-0.0, tracking_lin_vel_lat=0.0,
                                tracking_lin_vel_long=0.0)),
    "normalization": dict(obs_scales=dict(lin_vel=2.0, ang_vel=0.25, dof_pos=1.0, dof_vel=0.05,
                                          height_measurements=5.0, body_height_cmd=2.0),
                          clip_observations=100.0, clip_actions=100.0, friction_range=[0.05, 4.5],
                          restitution_range=[0, 1.0], added_mass_range=[-1.0, 3.0],
                          com_displacement_range=[-0.1, 0.1], motor_strength_range=[0.9, 1.1],
                          Kp_factor_range=[0.8, 1.3], Kd_factor_range=[0.5, 1.5]),
    "noise": dict(add_noise=True, noise_level=1.0,
                  noise_scales=dict(dof_pos=0.01, dof_vel=1.5, lin_vel=0.1, ang_vel=0.2, gravity=0.05,
                                    height_measurements=0.1)),
    "viewer": dict(ref_env=0, pos=[-10, 0, 6], lookat=[0.0, 0, 3.0]),
    "sim": dict(dt=0.005, substeps=1, gravity=[0.0, 0.0, -9.81], up_axis=1, use_gpu_pipeline=True,
                physx=dict(num_threads=10, solver_type=1, num_position_iterations=4, num_velocity_iterations=0,
                           contact_offset=0.01, rest_offset=0.0, bounce_threshold_velocity=0.5,
                           max_depenetration_velocity=1.0, max_gpu_contact_pairs=2 ** 23,
                           default_buffer_size_multiplier=5, contact_collection=2)),
}


def make_cfg():
    """A fresh, independent base configuration tree."""
    return _build(_BASE)


Cfg = make_cfg()

_LEG_ORDER = ("FL", "RL", "FR", "RR")


def _angles(hip, thigh, calf):
    d = {}
    for part, vals in (("hip", hip), ("thigh", thigh), ("calf", calf)):
        for leg, v in zip(_LEG_ORDER, vals):
            d[f"{leg}_{part}_joint"] = v
    return d


def _apply(cfg, updates):
    for path, value in updates.items():
        node = cfg
        *parents, leaf = path.split(".")
        for p in parents:
            node = getattr(node, p)
        setattr(node, leaf, copy.deepcopy(value))


_COMMON_PRESET = {
    "control.control_type": "P", "control.stiffness": {"joint": 20.0}, "control.damping": {"joint": 0.5},
    "control.action_scale": 0.25, "control.hip_scale_reduction": 0.5, "control.decimation": 4,
    "asset.self_collisions": 0, "asset.flip_visual_attachments": False, "asset.fix_base_link": False,
    "rewards.soft_dof_pos_limit": 0.9, "rewards.scales.dof_pos_limits": -10.0,
    "rewards.scales.orientation": -5.0, "rewards.scales.base_height": -30.0,
    "terrain.measure_heights": False, "terrain.terrain_noise_magnitude": 0.0, "terrain.border_size": 50,
    "terrain.terrain_proportions": [0, 0, 0, 0, 0, 0, 0, 0, 1.0], "terrain.curriculum": False,
    "env.num_observations": 42, "env.observe_vel": False,
    "commands.heading_command": False, "commands.resampling_time": 10.0, "commands.command_curriculum": True,
    "commands.num_lin_vel_bins": 30, "commands.num_ang_vel_bins": 30, "commands.lin_vel_x": [-0.6, 0.6],
    "commands.lin_vel_y": [-0.6, 0.6], "commands.ang_vel_yaw": [-1, 1],
    "domain_rand.randomize_base_mass": True, "domain_rand.added_mass_range": [-1, 3],
    "domain_rand.push_robots": False, "domain_rand.max_push_vel_xy": 0.5, "domain_rand.randomize_friction": True,
    "domain_rand.friction_range": [0.05, 4.5], "domain_rand.randomize_restitution": True,
    "domain_rand.restitution_range": [0.0, 1.0], "domain_rand.restitution": 0.5,
    "domain_rand.randomize_com_displacement": True, "domain_rand.com_displacement_range": [-0.1, 0.1],
    "domain_rand.randomize_motor_strength": True, "domain_rand.motor_strength_range": [0.9, 1.1],
    "domain_rand.randomize_Kp_factor": False, "domain_rand.Kp_factor_range": [0.8, 1.3],
    "domain_rand.randomize_Kd_factor": False, "domain_rand.Kd_factor_range": [0.5, 1.5],
    "domain_rand.rand_interval_s": 6,
}


def config_mini_cheetah(cfg):
    """Mini Cheetah preset (mini_cheetah_config.py:8-105)."""
    upd = dict(_COMMON_PRESET)
    upd.update({
        "init_state.pos": [0.0, 0.0, 0.32],
        "init_state.default_joint_angles": _angles((0.1, 0.1, -0.1, -0.1), (-0.8,) * 4, (1.62,) * 4),
        "asset.file": "{MINI_GYM_ROOT_DIR}/resources/robots/mini_cheetah/urdf/mini_cheetah.urdf",
        "asset.foot_name": "calf", "asset.penalize_contacts_on": [],
        "asset.terminate_after_contacts_on": ["base", "thigh"],
        "rewards.base_height_target": 0.30, "rewards.scales.torques": -0.0002,
        "terrain.mesh_type": "trimesh", "terrain.teleport_robots": True, "env.num_envs": 4000,
    })
    _apply(cfg, upd)
    # keep the reference's declaration order: torques/orientation/base_height were already
    # declared in the base tree; dof_pos_limits is new and lands last (legged_robot.py:1079).
    return cfg


def config_go1(cfg):
    """Unitree Go1 preset (go1_config.py:8-107)."""
    upd = dict(_COMMON_PRESET)
    upd.update({
        "init_state.pos": [0.0, 0.0, 0.34],
        "init_state.default_joint_angles": _angles((0.1, 0.1, -0.1, -0.1), (0.8, 1.0, 0.8, 1.0), (-1.5,) * 4),
        "asset.file": "{MINI_GYM_ROOT_DIR}/resources/robots/go1/urdf/go1.urdf",
        "asset.foot_name": "foot", "asset.penalize_contacts_on": ["thigh", "calf"],
        "asset.terminate_after_contacts_on": ["base"],
        "rewards.base_height_target": 0.34, "rewards.scales.torques": -0.0001,
        "rewards.scales.action_rate": -0.01,
        "terrain.mesh_type": "plane", "terrain.teleport_robots": False, "env.num_envs": 4096,
    })
    _apply(cfg, upd)
    return cfg
