"""ctypes mirror of include/lrl.h (structs, enums) and the loader for liblrl.so.

The product path goes through liblrl.so only: if the library is missing or no GPU is visible the
env / PPO entry points raise instead of falling back to any CPU or eager implementation.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LRL_LIB overrides the library path (instrumented development builds); the default is the in-tree build
LIB_PATH = os.environ.get("LRL_LIB") or os.path.join(os.path.dirname(_HERE), "csrc", "liblrl.so")

MAX_BODIES, MAX_SPHERES, NUM_DOF, NUM_LEGS, MAX_OBS, MAX_REWARD_TERMS, NUM_PRIV = 20, 40, 12, 4, 256, 24, 18
MAX_HEIGHT_POINTS = 192
f32, i32, u32 = C.c_float, C.c_int32, C.c_uint32

REWARD_TERMS = ["lin_vel_z", "ang_vel_xy", "orientation", "base_height", "torques", "energy",
                "energy_expenditure", "dof_vel", "dof_acc", "action_rate", "collision", "survival",
                "dof_pos_limits", "dof_vel_limits", "torque_limits", "tracking_lin_vel", "tracking_ang_vel",
                "feet_air_time", "stumble", "stand_still", "feet_contact_forces"]

STEP_PHYSICS, STEP_HISTORY, STEP_INJECT_UNIFORM = 1, 2, 4

(T_ROOT_STATE, T_DOF_POS, T_DOF_VEL, T_CONTACT_FORCE, T_RIGID_BODY_STATE, T_TORQUES, T_ACTIONS, T_LAST_ACTIONS,
 T_LAST_DOF_VEL, T_LAST_ROOT_VEL, T_COMMANDS, T_OBS, T_PRIV_OBS, T_OBS_HISTORY, T_REWARD, T_RESET, T_TIME_OUT,
 T_EPISODE_LENGTH, T_EPISODE_SUMS, T_COMMAND_SUMS, T_FEET_AIR_TIME, T_LAST_CONTACTS, T_FRICTION, T_RESTITUTION,
 T_PAYLOAD, T_COM_DISPLACEMENT, T_MOTOR_STRENGTH, T_KP_FACTOR, T_KD_FACTOR, T_ENV_ORIGINS, T_BASE_LIN_VEL,
 T_BASE_ANG_VEL, T_PROJECTED_GRAVITY, T_JOINT_POS_TARGET, T_MEASURED_HEIGHTS, T_NUM) = range(36)


class LrlModel(C.Structure):
    _fields_ = [
        ("num_bodies", i32), ("body_leg", i32 * MAX_BODIES), ("body_link", i32 * MAX_BODIES),
        ("joint_xyz", f32 * 3 * 3 * NUM_LEGS), ("joint_quat", f32 * 4 * 3 * NUM_LEGS),
        ("joint_axis", f32 * 3 * 3 * NUM_LEGS), ("foot_xyz", f32 * 3 * NUM_LEGS),
        ("base_mass", f32), ("base_com", f32 * 3), ("base_inertia", f32 * 6),
        ("link_mass", f32 * 3 * NUM_LEGS), ("link_com", f32 * 3 * 3 * NUM_LEGS),
        ("link_inertia", f32 * 6 * 3 * NUM_LEGS),
        ("num_spheres", i32), ("sphere_body", i32 * MAX_SPHERES), ("sphere_pos", f32 * 3 * MAX_SPHERES),
        ("sphere_radius", f32 * MAX_SPHERES),
        ("dof_lower", f32 * NUM_DOF), ("dof_upper", f32 * NUM_DOF), ("dof_effort", f32 * NUM_DOF),
        ("dof_velocity", f32 * NUM_DOF),
        ("sphere_hull", i32 * MAX_SPHERES), ("num_hulls", i32), ("hull_res", i32), ("hull_k", i32),
        ("hull_table", C.c_void_p),
    ]


class LrlEnvParams(C.Structure):
    _fields_ = [
        ("sim_dt", f32), ("decimation", i32), ("dt", f32), ("gravity", f32 * 3),
        ("contact_offset", f32), ("max_depenetration_velocity", f32), ("bounce_threshold_velocity", f32),
        ("ground_friction", f32), ("ground_restitution", f32), ("solver_iterations", i32), ("baumgarte", f32),
        ("control_type", i32), ("action_scale", f32), ("hip_scale_reduction", f32), ("clip_actions", f32),
        ("p_gains", f32 * NUM_DOF), ("d_gains", f32 * NUM_DOF), ("default_dof_pos", f32 * NUM_DOF),
        ("torque_limits", f32 * NUM_DOF), ("soft_dof_pos_lower", f32 * NUM_DOF),
        ("soft_dof_pos_upper", f32 * NUM_DOF), ("dof_vel_limits", f32 * NUM_DOF),
        ("num_feet", i32), ("feet", i32 * NUM_LEGS), ("termination_mask", u32), ("penalised_mask", u32),
        ("num_reward_terms", i32), ("reward_term", i32 * MAX_REWARD_TERMS), ("reward_scale", f32 * MAX_REWARD_TERMS),
        ("reward_slot", i32 * MAX_REWARD_TERMS), ("num_sum_keys", i32), ("termination_scale", f32),
        ("termination_slot", i32), ("only_positive_rewards", i32),
        ("tracking_sigma", f32), ("tracking_sigma_yaw", f32), ("base_height_target", f32),
        ("soft_dof_vel_limit", f32), ("soft_torque_limit", f32), ("max_contact_force", f32),
        ("use_terminal_body_height", i32), ("terminal_body_height", f32),
        ("num_obs", i32), ("observe_vel", i32), ("observe_command", i32),
        ("obs_scale_lin_vel", f32), ("obs_scale_ang_vel", f32), ("obs_scale_dof_pos", f32),
        ("obs_scale_dof_vel", f32), ("commands_scale", f32 * 3), ("add_noise", i32), ("noise_vec", f32 * MAX_OBS),
        ("clip_obs", f32), ("priv_scale", f32 * 5), ("priv_shift", f32 * 5),
        ("rand_interval", i32), ("randomize_motor_strength", i32), ("randomize_kp", i32), ("randomize_kd", i32),
        ("motor_strength_range", f32 * 2), ("kp_range", f32 * 2), ("kd_range", f32 * 2),
        ("teleport", i32), ("teleport_thresh", f32), ("teleport_x_offset", f32), ("terrain_length", f32),
        ("terrain_width", f32), ("terrain_rows", i32), ("terrain_cols", i32),
        ("base_init_state", f32 * 13), ("num_history", i32), ("auto_reset", i32), ("max_episode_length", i32),
        ("terrain_mesh", i32), ("border_size", f32), ("horizontal_scale", f32), ("vertical_scale", f32),
        ("measure_heights", i32), ("num_height_points", i32), ("height_points", f32 * 2 * MAX_HEIGHT_POINTS),
        ("obs_scale_height", f32), ("num_train_envs", i32), ("teleport_x_offset_eval", f32), ("dr_span", f32 * 3),
        ("joint_limits", i32), ("joint_limit_margin", f32), ("self_collisions", i32),
        ("push_robots", i32), ("push_interval", i32), ("push_lo", f32), ("push_span", f32),
        ("solver_tgs", i32),
    ]


class LrlTensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("dtype", i32), ("ndim", i32), ("shape", C.c_int64 * 4),
                ("strides", C.c_int64 * 4)]


class LrlRolloutStore(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("priv", C.c_void_p), ("hist", C.c_void_p), ("actions", C.c_void_p),
                ("values", C.c_void_p), ("logp", C.c_void_p), ("mu", C.c_void_p), ("sigma", C.c_void_p),
                ("hist_dim", i32), ("hist_ld", i32)]


i64 = C.c_int64


class LrlPpoNet(C.Structure):
    _fields_ = [(k, i32) for k in ("num_obs", "num_priv", "num_hist", "num_actions", "enc_h0", "enc_h1", "latent",
                                    "ac_h0", "ac_h1", "ac_h2", "ad_h0", "ad_h1")] + \
               [(k, i64) for k in ("w1", "b1", "w2", "b2", "w3", "b3", "w4a", "b4a", "w4c", "b4c", "e1w", "e1b", "e2w",
                                    "e2b", "e3w", "e3b", "d1w", "d1b", "d2w", "d2b", "d3w", "d3b", "std_off",
                                    "main_begin", "main_end", "adapt_begin", "adapt_end", "kl_slot", "total")]


class LrlPpoBatch(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("obs", "priv", "hist", "actions", "values", "returns", "logp", "adv", "mu",
                                          "sigma", "rows")] + [("batch", i32), ("hist_ld", i32)]


class LrlPpoHparams(C.Structure):
    _fields_ = [("clip_param", f32), ("entropy_coef", f32), ("value_loss_coef", f32), ("max_grad_norm", f32),
                ("desired_kl", f32), ("use_clipped_value_loss", i32), ("adaptive_schedule", i32), ("beta1", f32),
                ("beta2", f32), ("eps", f32)]


class LrlDevCurriculum(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("weights", "cdf", "state", "mt_key", "ep_rew_lin", "ep_rew_ang", "env_bins",
                                          "env_bins_f", "command_area", "axes")] + \
               [("half", C.c_double * 3), ("nx", i32), ("ny", i32), ("nz", i32), ("words", C.c_void_p),
                ("draws", C.c_void_p), ("env_bins_f_prev", C.c_void_p), ("command_area_prev", C.c_void_p)]


PPO_CTRL_BYTES = 64  # sizeof(lrl_ppo_ctrl): double lr, double loss_sum[3], float mb[4], float x4


def fill(struct, **kw):
    """Assign python values (scalars / nested lists) into a ctypes struct."""
    for k, v in kw.items():
        cur = getattr(struct, k)
        if isinstance(cur, C.Array):
            _fill_array(cur, v)
        else:
            setattr(struct, k, v)
    return struct


def _fill_array(arr, v):
    for i, x in enumerate(v):
        if isinstance(arr[i], C.Array):
            _fill_array(arr[i], x)
        else:
            arr[i] = x


_lib = None

_CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
# the files and order of csrc/Makefile's SRC_HASH (SRCS then HDRS)
_HASHED = ["lrl_env.hip", "lrl_aux.hip", "lrl_gae.hip", "lrl_gemm.hip", "lrl_ppo.hip", "lrl_capi.cpp", "lrl_curriculum.cpp",
           "lrl_curriculum_dev.hip", "lrl_env_flat.hip", "lrl_kparams.h", "lrl_gemm.h", "../../include/lrl.h", "../../include/lrl_philox.h",
           "Makefile"]  # (the build flags too: a library built with other flags is stale)


def source_hash():
    """sha256 (first 16 hex digits) of the sources liblrl.so must have been built from."""
    import hashlib
    h = hashlib.sha256()
    for name in _HASHED:
        with open(os.path.join(_CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def lib():
    """liblrl.so, loaded once.  Raises (no fallback) if it was not built, or was built from other sources than the
    ones in this tree (a stale binary)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"liblrl.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        L.lrl_build_hash.restype = C.c_char_p
        built, want = L.lrl_build_hash().decode(), source_hash()
        # (an explicit LRL_LIB — an instrumented or A/B development build — is loaded as named)
        if built != want and not os.environ.get("LRL_LIB"):
            raise RuntimeError(f"{LIB_PATH} was built from other sources (hash {built}, tree {want}); "
                               "rebuild it: __graft_entry__.build()")
        L.lrl_last_error.restype = C.c_char_p
        for name in ["lrl_sim_create", "lrl_sim_destroy", "lrl_sim_tensor", "lrl_sim_step", "lrl_sim_reset_idx",
                     "lrl_sim_set_root_state_indexed", "lrl_sim_set_dof_state_indexed", "lrl_sim_inject_uniforms",
                     "lrl_sim_refresh_rigid_body_state", "lrl_sim_shift_history", "lrl_sim_randomize", "lrl_gae",
                     "lrl_ppo_act", "lrl_abi_version", "lrl_device_count", "lrl_gae_partial", "lrl_adv_normalize",
                     "lrl_sim_reset_idx_ex", "lrl_sim_observe_idx", "lrl_sim_set_step_counter", "lrl_ppo_forward_backward",
                     "lrl_ppo_optimizer_step", "lrl_ppo_adaptation_forward_backward", "lrl_ppo_adaptation_step",
                     "lrl_gemm_f32", "lrl_ppo_timing", "lrl_ppo_act_student", "lrl_sim_set_terrain",
                     "lrl_sim_terrain_curriculum", "lrl_sim_inject_reset_uniforms", "lrl_sim_inject_push_uniforms", "lrl_sim_timing",
                     "lrl_sim_self_contact_stats", "lrl_ppo_store_step", "lrl_curriculum_sample",
                     "lrl_curriculum_update_weights", "lrl_rows_mean_zero", "lrl_sim_step_code",
                     "lrl_sim_apply_commands", "lrl_sim_extras_snapshot", "lrl_sim_env_lists",
                     "lrl_sim_terrain_curriculum_dev", "lrl_sim_reset_idx_dev", "lrl_sim_observe_idx_dev",
                     "lrl_rows_mean_zero_dev", "lrl_sim_curriculum_resample_dev", "lrl_debug_gemm_paths",
                     "lrl_debug_sim_garbage", "lrl_debug_sim_arena"]:
            getattr(L, name).restype = C.c_int32
        L.lrl_np_sum_f64.restype = C.c_double
        L.lrl_np_sum_f64.argtypes = [C.c_void_p, C.c_int64]
        L.lrl_ppo_workspace_bytes.restype = C.c_int64
        L.lrl_ppo_act_workspace_bytes.restype = C.c_int64
        L.lrl_ppo_act_student_workspace_bytes.restype = C.c_int64
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().lrl_last_error()
        raise RuntimeError(f"liblrl error {rc}: {msg.decode() if msg else ''}")
    return rc


_dev_index_cache = {}


def stream_of(device):
    """The current HIP stream of `device` as a c_void_p (torch's raw-stream accessor: no Stream object built per call —
    a few microseconds less per launch on the host-bound upstream-reset path)."""
    idx = _dev_index_cache.get(device)
    if idx is None:
        import torch
        d = torch.device(device)
        idx = d.index if d.index is not None else torch.cuda.current_device()
        _dev_index_cache[device] = idx
    import torch
    return C.c_void_p(torch._C._cuda_getCurrentRawStream(idx))
