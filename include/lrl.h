/*
 * lrl.h — C ABI of liblrl.so, the MI355X-native hot path of rapid-locomotion-rl.
 *
 * What this library replaces (the reference's lower boundary): the Isaac Gym
 * Preview 3 gymapi/gymtorch calls that mini_gym/envs/base/legged_robot.py makes on every env step
 * and the torch elementwise work around them, plus the PPO numeric core of mini_gym_learn.
 *
 *   lrl_sim_create         ~ gym.create_sim + load_asset + create_env/create_actor loop + prepare_sim
 *                            (legged_robot.py:419-441, 1162-1319; base_task.py:17,70)
 *   lrl_sim_tensor         ~ gym.acquire_{actor_root_state,dof_state,net_contact_force,rigid_body_state}
 *                            _tensor + gymtorch.wrap_tensor (legged_robot.py:939-970)
 *   lrl_sim_step           ~ LeggedRobot.step (legged_robot.py:106-137): clip actions, 4 x
 *                            {_compute_torques :653-688, set_dof_actuation_force_tensor :118,
 *                            simulate/fetch_results :119-121, refresh_dof_state :122}, then
 *                            post_physics_step :139-188 (teleport :768-791, DR :544-560,
 *                            check_termination :190-202, compute_reward :314-340,
 *                            compute_observations :342-417), obs clip :133-136 and the
 *                            HistoryWrapper shift (history_wrapper.py:23) — one fused launch.
 *   lrl_sim_reset_idx      ~ LeggedRobot.reset_idx device part (:227-290: _reset_dofs :690-712,
 *                            _reset_root_states :714-755, buffer zeroing :255-259)
 *   lrl_sim_set_root_state_indexed / lrl_sim_set_dof_state_indexed
 *                          ~ gym.set_actor_root_state_tensor_indexed / set_dof_state_tensor_indexed
 *                            (legged_robot.py:303-312, 710-712, 739-741)
 *   lrl_sim_refresh_rigid_body_state ~ gym.refresh_rigid_body_state_tensor (:147)
 *   lrl_gae                ~ RolloutStorage.compute_returns (rollout_storage.py:76-90)
 *   lrl_ppo_act            ~ PPO.act teacher path (ppo.py:62-74 -> actor_critic.py:137-147,170-173)
 *                            fused with RolloutStorage.add_transitions (rollout_storage.py:57-71)
 *   lrl_ppo_*              ~ PPO.update (ppo.py:94-178): minibatch forward/backward of the PPO loss,
 *                            adaptive-KL LR + clip_grad_norm_ + Adam, the adaptation-module MSE step
 *   lrl_gemm_f32           ~ the torch.nn.Linear products those are built from (test entry point)
 *
 * Conventions: every function returns 0 on success or a negative LRL_E* code, with a message
 * available from lrl_last_error() (thread-local).  All data pointers passed to compute entry points
 * are DEVICE pointers (HBM); `stream` is a hipStream_t passed as void*.  A sim handle is bound to one
 * device and is not thread-safe.  No torch types cross this boundary.
 */
#ifndef LRL_H_
#define LRL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LRL_ABI_VERSION 6

#define LRL_OK 0
#define LRL_E_INVALID (-1)  /* bad argument / unsupported configuration */
#define LRL_E_HIP (-2)      /* HIP runtime error */
#define LRL_E_NOMEM (-3)
#define LRL_E_NOGPU (-4)

#define LRL_MAX_BODIES 20
#define LRL_MAX_SPHERES 40
#define LRL_NUM_DOF 12
#define LRL_NUM_LEGS 4
#define LRL_MAX_OBS 256       /* 42 + a 17 x 11 height scan (legged_robot_config.py:46-47) fits */
#define LRL_MAX_HEIGHT_POINTS 192
#define LRL_MAX_REWARD_TERMS 24
#define LRL_NUM_PRIV 18
#define LRL_SELF_SLOTS 8        /* self-contact rows per env and sub-step (solver slots) */
#define LRL_MAX_SELF_PAIRS 256  /* candidate self-collision sphere pairs of a model */
#define LRL_HULL_K 4            /* candidate vertices per support-table cell (lrl_model::hull_k) */

/* ------------------------------------------------------------------------------------------
 * Robot model: a floating base with 4 legs x 3 revolute joints (hip, thigh, calf) and an optional
 * fixed foot body per leg (Go1 `dont_collapse` feet).  Produced on the host from the URDF after
 * collapse_fixed_joints (legged_robot_config.py:128).  Body order = Isaac Gym asset order.
 * ------------------------------------------------------------------------------------------ */
typedef struct lrl_model {
  int32_t num_bodies;                 /* reported bodies B (13 Mini Cheetah, 17 Go1) */
  int32_t body_leg[LRL_MAX_BODIES];   /* -1 = base, else leg 0..3 */
  int32_t body_link[LRL_MAX_BODIES];  /* 0 hip, 1 thigh, 2 calf, 3 fixed foot (merged into calf) */
  /* per leg, per revolute joint j (0 hip, 1 thigh, 2 calf) */
  float joint_xyz[LRL_NUM_LEGS][3][3];   /* joint origin in parent-body frame */
  float joint_quat[LRL_NUM_LEGS][3][4];  /* fixed joint-origin rotation (xyzw) */
  float joint_axis[LRL_NUM_LEGS][3][3];  /* rotation axis in the child frame */
  float foot_xyz[LRL_NUM_LEGS][3];       /* fixed foot origin in calf frame (if present) */
  /* inertial data in the body frame: mass, COM, inertia about COM (xx yy zz xy xz yz) */
  float base_mass, base_com[3], base_inertia[6];
  float link_mass[LRL_NUM_LEGS][3], link_com[LRL_NUM_LEGS][3][3], link_inertia[LRL_NUM_LEGS][3][6];
  /* collision geometry as spheres (box corners radius 0): owning body index, center, radius */
  int32_t num_spheres;
  int32_t sphere_body[LRL_MAX_SPHERES];
  float sphere_pos[LRL_MAX_SPHERES][3];
  float sphere_radius[LRL_MAX_SPHERES];
  /* joint data in asset DOF order (FL hip, thigh, calf, FR ..., RL ..., RR ...) */
  float dof_lower[LRL_NUM_DOF], dof_upper[LRL_NUM_DOF], dof_effort[LRL_NUM_DOF], dof_velocity[LRL_NUM_DOF];
  /* ABI 6 — mesh colliders as support tables (PhysX collides a <mesh> as its convex hull).  With
   * num_hulls > 0, a leg sphere s with sphere_hull[s] = h >= 0 meets the ground plane at the support point of hull
   * table h in the direction of the plane's inward normal, in place of its sphere (whose centre / radius remain the
   * self-collision stand-in); num_hulls = 0 ignores sphere_hull.  hull_table (host memory, read during
   * lrl_sim_create only) is [num_hulls][6][hull_res][hull_res][hull_k][4]: per cube-map cell of the link-frame
   * direction d (face 2m + (d_m < 0) of the major axis m, first of x, y, z on ties; cell floor((d_(m+1) / |d_m| + 1)
   * hull_res / 2), floor((d_(m+2) / |d_m| + 1) hull_res / 2), clamped), hull_k candidate vertices (x, y, z, unused)
   * in the body frame the sphere centres use; the contact point is the candidate with the largest x . d (the first on a
   * tie); hull_k must be LRL_HULL_K.  On the terrain mesh (terrain_mesh = 1) the same support point (world -z) is the
   * triangle query's point, with radius 0. */
  int32_t sphere_hull[LRL_MAX_SPHERES];
  int32_t num_hulls, hull_res, hull_k;
  const float* hull_table;
} lrl_model;

/* Reward terms the fused kernel implements (legged_robot.py:1506-1646); the host passes the
 * active ones in the order of vars(Cfg.rewards.scales) after zero-scale removal. */
enum lrl_reward_term {
  LRL_R_LIN_VEL_Z = 0, LRL_R_ANG_VEL_XY, LRL_R_ORIENTATION, LRL_R_BASE_HEIGHT, LRL_R_TORQUES,
  LRL_R_ENERGY, LRL_R_ENERGY_EXPENDITURE, LRL_R_DOF_VEL, LRL_R_DOF_ACC, LRL_R_ACTION_RATE,
  LRL_R_COLLISION, LRL_R_SURVIVAL, LRL_R_DOF_POS_LIMITS, LRL_R_DOF_VEL_LIMITS, LRL_R_TORQUE_LIMITS,
  LRL_R_TRACKING_LIN_VEL, LRL_R_TRACKING_ANG_VEL, LRL_R_FEET_AIR_TIME, LRL_R_STUMBLE,
  LRL_R_STAND_STILL, LRL_R_FEET_CONTACT_FORCES, LRL_R_NUM_TERMS
};

/* Everything LeggedRobot derives from Cfg at construction time (_parse_cfg :1417-1429,
 * _init_buffers :935-1030, _prepare_reward_function :1074-1110, _get_noise_scale_vec :882-932). */
typedef struct lrl_env_params {
  /* timing */
  float sim_dt;      /* float32(Cfg.sim.dt) */
  int32_t decimation;
  float dt;          /* decimation * sim_dt, as float */
  float gravity[3];
  /* contact solver (own model; PhysX is closed: see DESIGN.md §physics) */
  float contact_offset, max_depenetration_velocity, bounce_threshold_velocity;
  float ground_friction, ground_restitution;
  int32_t solver_iterations;
  float baumgarte;
  /* control (legged_robot.py:653-688) */
  int32_t control_type; /* 0 = 'P', 1 = 'V', 2 = 'T' (legged_robot.py:668-675; 'P_compliantfeet' indexes DOF 15 of 12
                         * and raises in the reference, so the host refuses it) */
  float action_scale, hip_scale_reduction, clip_actions;
  float p_gains[LRL_NUM_DOF], d_gains[LRL_NUM_DOF], default_dof_pos[LRL_NUM_DOF];
  float torque_limits[LRL_NUM_DOF];
  float soft_dof_pos_lower[LRL_NUM_DOF], soft_dof_pos_upper[LRL_NUM_DOF], dof_vel_limits[LRL_NUM_DOF];
  /* bodies */
  int32_t num_feet, feet[LRL_NUM_LEGS];
  uint32_t termination_mask, penalised_mask; /* bit b = body b */
  /* rewards */
  int32_t num_reward_terms;
  int32_t reward_term[LRL_MAX_REWARD_TERMS];    /* enum lrl_reward_term */
  float reward_scale[LRL_MAX_REWARD_TERMS];     /* already x dt, as float */
  int32_t reward_slot[LRL_MAX_REWARD_TERMS];    /* row of episode_sums / command_sums */
  int32_t num_sum_keys;                         /* len(reward_scales) after zero removal */
  float termination_scale;                      /* 0 = no termination term */
  int32_t termination_slot;
  int32_t only_positive_rewards;
  float tracking_sigma, tracking_sigma_yaw, base_height_target, soft_dof_vel_limit, soft_torque_limit,
      max_contact_force;
  int32_t use_terminal_body_height;
  float terminal_body_height;
  /* observations (compute_observations :342-417) */
  int32_t num_obs, observe_vel, observe_command;
  float obs_scale_lin_vel, obs_scale_ang_vel, obs_scale_dof_pos, obs_scale_dof_vel;
  float commands_scale[3];
  int32_t add_noise;
  float noise_vec[LRL_MAX_OBS];
  float clip_obs;
  /* privileged obs: (x - shift) * scale for friction, restitution, payload, com, motor strength */
  float priv_scale[5], priv_shift[5];
  /* domain randomisation (legged_robot.py:519-560) */
  int32_t rand_interval;  /* steps */
  int32_t randomize_motor_strength, randomize_kp, randomize_kd;
  float motor_strength_range[2], kp_range[2], kd_range[2];
  /* teleport (legged_robot.py:768-791) */
  int32_t teleport;
  float teleport_thresh, teleport_x_offset, terrain_length, terrain_width;
  int32_t terrain_rows, terrain_cols;
  /* reset (legged_robot.py:690-755) */
  float base_init_state[13];
  int32_t num_history; /* HistoryWrapper length (15) */
  int32_t auto_reset;  /* 0 = fork semantics (no resets inside step, Q2); 1 = upstream */
  int32_t max_episode_length;
  /* terrain (legged_robot.py:419-441 create_sim, :1112-1160 ground / heightfield / trimesh,
   * :1453-1503 height scan).  terrain_mesh 0: ground plane z = 0 (plane, or a trimesh whose height
   * field is all zero); 1: contacts against the triangle mesh given to lrl_sim_set_terrain. */
  int32_t terrain_mesh;
  float border_size, horizontal_scale, vertical_scale;
  int32_t measure_heights;    /* _get_heights every step, obs += clip(z - 0.5 - h, -1, 1) * scale */
  int32_t num_height_points;  /* 17 x 11 = 187 */
  float height_points[LRL_MAX_HEIGHT_POINTS][2]; /* base-frame (x, y), meshgrid(x, y) order (:1453-1467) */
  float obs_scale_height;
  /* envs with index >= num_train_envs (the eval group, base_task.py:43-50) teleport with the eval tiles' x
   * offset (legged_robot.py:772 under _call_train_eval) */
  int32_t num_train_envs;
  float teleport_x_offset_eval;
  /* float32(hi - lo) of motor_strength_range / kp_range / kd_range with the difference taken in double, as
   * torch.rand(k) * (max - min) + min rounds the python-float difference once (legged_robot.py:544-560) */
  float dr_span[3];
  /* joint position limits (the URDF <limit lower upper> of every revolute joint, lrl_model::dof_lower / dof_upper),
   * enforced as unilateral joint-space rows of the contact solve, as PhysX articulations enforce URDF limits:
   * a joint whose distance d to its nearer limit is below joint_limit_margin + 2 sim_dt |qd| gets a row
   * (speculative target -d / sim_dt, Baumgarte for d < 0). 0 = off. */
  int32_t joint_limits;
  float joint_limit_margin; /* rad */
  /* self-collision (Cfg.asset.self_collisions == 0, the collision filter legged_robot.py:1246-1247 passes to create_actor: Isaac Gym
   * enables PhysX self-collision for 0): collision spheres of different, non-adjacent links of the articulation
   * (own model, DESIGN.md §4: sphere-sphere between legs and inside a leg, leg sphere against the base box the
   * base-corner spheres span), up to LRL_SELF_SLOTS contacts per env and sub-step in the canonical pair order,
   * friction / restitution of the robot's own material.  0 = off. */
  int32_t self_collisions;
  /* _push_robots (legged_robot.py:757-766, called from _post_physics_step_callback :588): envs whose episode length
   * (after this step's increment) is a multiple of push_interval get root linear velocity x / y =
   * push_span * u + push_lo (torch_rand_float(-max_push_vel_xy, max_push_vel_xy, (k, 2)), float32 order), after the
   * base-frame velocities of the step were taken (so it shows in root_states / last_root_vel, not in this step's obs).
   * 0 = off. */
  int32_t push_robots;
  int32_t push_interval;
  float push_lo, push_span;
  /* Cfg.sim.physx.solver_type (legged_robot_config.py:247; 1 = TGS): the contact / limit solve runs solver_iterations
   * sub-iterations of h = sim_dt / solver_iterations, each sweeping the rows once with targets from the separations
   * moved by the motion so far, and positions integrate the accumulated motion.  0 = PGS: the
   * iterations sweep the whole sub-step with the start targets.  Plane ground only (the terrain-mesh build solves
   * with PGS and the host passes 0 there). */
  int32_t solver_tgs;
} lrl_env_params;

/* ------------------------------------------------------------------------------------------
 * Sim object and its device tensors (acquire_*_tensor).
 * ------------------------------------------------------------------------------------------ */
typedef struct lrl_sim lrl_sim;

enum lrl_dtype { LRL_F32 = 0, LRL_I32 = 1, LRL_U8 = 2 };

typedef struct lrl_tensor {
  void* data;          /* device pointer */
  int32_t dtype;       /* enum lrl_dtype */
  int32_t ndim;
  int64_t shape[4];
  int64_t strides[4];  /* in elements */
} lrl_tensor;

enum lrl_tensor_id {
  LRL_T_ROOT_STATE = 0,  /* [N,13] pos, quat xyzw, lin vel (COM, world), ang vel (world) */
  LRL_T_DOF_POS,         /* [N,12] */
  LRL_T_DOF_VEL,         /* [N,12] */
  LRL_T_CONTACT_FORCE,   /* [N,B,3] net contact force per body, world frame, last sub-step */
  LRL_T_RIGID_BODY_STATE,/* [N,B,13] (valid after lrl_sim_refresh_rigid_body_state) */
  LRL_T_TORQUES,         /* [N,12] last sub-step torques */
  LRL_T_ACTIONS,         /* [N,12] clipped actions of the last step */
  LRL_T_LAST_ACTIONS, LRL_T_LAST_DOF_VEL, /* [N,12] */
  LRL_T_LAST_ROOT_VEL,   /* [N,6] */
  LRL_T_COMMANDS,        /* [N,4] */
  LRL_T_OBS,             /* [N,num_obs] */
  LRL_T_PRIV_OBS,        /* [N,18] */
  LRL_T_OBS_HISTORY,     /* [N,num_history*num_obs] */
  LRL_T_REWARD,          /* [N] */
  LRL_T_RESET,           /* [N] u8 */
  LRL_T_TIME_OUT,        /* [N] u8 */
  LRL_T_EPISODE_LENGTH,  /* [N] i32 */
  LRL_T_EPISODE_SUMS,    /* [num_terms+1(+1 if termination), N]  (dict order of episode_sums) */
  LRL_T_COMMAND_SUMS,    /* [num_terms(+1) + 5, N]                (dict order of command_sums) */
  LRL_T_FEET_AIR_TIME,   /* [N,4] */
  LRL_T_LAST_CONTACTS,   /* [N,4] u8 */
  LRL_T_FRICTION,        /* [N] */
  LRL_T_RESTITUTION,     /* [N] */
  LRL_T_PAYLOAD,         /* [N] */
  LRL_T_COM_DISPLACEMENT,/* [N,3] */
  LRL_T_MOTOR_STRENGTH,  /* [N,12] */
  LRL_T_KP_FACTOR, LRL_T_KD_FACTOR, /* [N,12] */
  LRL_T_ENV_ORIGINS,     /* [N,3] */
  LRL_T_BASE_LIN_VEL, LRL_T_BASE_ANG_VEL, LRL_T_PROJECTED_GRAVITY, /* [N,3] body frame */
  LRL_T_JOINT_POS_TARGET,/* [N,12] */
  LRL_T_MEASURED_HEIGHTS,/* [N,num_height_points] (_get_heights, written by lrl_sim_step when measure_heights) */
  LRL_T_NUM
};

/* step flags */
#define LRL_STEP_PHYSICS 1u        /* run the 4 physics sub-steps (off: identity physics, test hook) */
#define LRL_STEP_HISTORY 2u        /* shift obs into the history buffer (HistoryWrapper.step) */
#define LRL_STEP_INJECT_UNIFORM 4u /* read noise / DR uniforms from lrl_sim_inject_uniforms buffers */

int32_t lrl_abi_version(void);
/* First 16 hex digits of the sha256 of the csrc sources + headers the library was built from (csrc/Makefile
   SRC_HASH); lrl/_abi.py refuses to load a library whose hash differs from the sources beside it. */
const char* lrl_build_hash(void);
const char* lrl_last_error(void);
int32_t lrl_device_count(void);

int32_t lrl_sim_create(const lrl_model* model, const lrl_env_params* params, int32_t num_envs,
                       int64_t global_env_offset, uint64_t seed, int32_t device, lrl_sim** out);
int32_t lrl_sim_destroy(lrl_sim* sim);
int32_t lrl_sim_tensor(lrl_sim* sim, int32_t tensor_id, lrl_tensor* out);

/* Initialise the per-env domain randomisation draws (legged_robot.py:519-542, 544-560) */
int32_t lrl_sim_randomize(lrl_sim* sim, const float* friction_range, const float* restitution_range,
                          const float* payload_range, const float* com_range, uint32_t which, void* stream);

/* One policy step for all envs: the fused LeggedRobot.step hot path. `actions` [N,12] f32 device. */
int32_t lrl_sim_step(lrl_sim* sim, const float* actions, uint32_t flags, void* stream);

/* Launch timing of the fused env kernel (bench.py roofline): enable = 1 starts recording HIP events around each
 * env-kernel launch of lrl_sim_step on its stream (the history-shift launch before it is outside); the next call
 * returns the summed milliseconds and the launch count of the recorded launches (waiting for them) and
 * restarts (enable = 1) or stops (enable = 0) recording. */
int32_t lrl_sim_timing(lrl_sim* sim, int32_t enable, double* total_ms, int64_t* launches);

/* Self-contact slot statistics (no reference counterpart: PhysX solves every self-pair, this solver gives an env
   min(8, free spheres / 2) slots per sub-step).  enable = 1 zeroes the counters and starts counting
   (the detection then counts every pair in contact; the slots and results are unchanged); enable = 0 stops.  Either
   way `out` (may be null) receives the counters before the call: [0] env-sub-steps with a self-contact, [1] pairs in
   contact summed over them, [2] env-sub-steps with more pairs than slots, [3] pairs left without a slot. */
int32_t lrl_sim_self_contact_stats(lrl_sim* sim, int32_t enable, uint64_t* out);

/* Injected uniforms for parity tests: noise_u [N,num_obs], dr_u [N] (NaN = no redraw). */
int32_t lrl_sim_inject_uniforms(lrl_sim* sim, const float* noise_u, const float* dr_u);
/* Injected push uniforms for parity tests: u [N,2] f32 device, row e = env e's (x, y) draw of _push_robots when it is
 * pushed in the step (legged_robot.py:763-764); required with LRL_STEP_INJECT_UNIFORM when push_robots is on. */
int32_t lrl_sim_inject_push_uniforms(lrl_sim* sim, const float* u);

int32_t lrl_sim_reset_idx(lrl_sim* sim, const int32_t* env_ids, int32_t n, void* stream);
/* reset_idx (legged_robot.py:227-290) with the root-state policy made explicit.
 *   root_mode 0: the root is left untouched — the fork's custom-origin quirk (_reset_root_states
 *                :724-741 writes the advanced-index copy `root_states` and pushes the unchanged all_root_states);
 *   root_mode 1: base_init_state + env_origin (the plane path :736-737 / upstream);
 *   root_mode 2: custom origins, upstream semantics (:725-732): ((base_init_state + env_origin) + (xy_span * u
 *                + xy_lo)) + (x_off, y_off), one uniform u per env for x and one for y — torch_rand_float(
 *                x_init_range, y_init_range, (k, 2)) with xy_lo = x_init_range and xy_span = float32(y_init_range -
 *                x_init_range) rounded from the python-float difference — in that float32 order.
 * The uniforms (motor-strength / Kp / Kd redraws of _randomize_dof_props :544-560, then x, y) come from the
 * sim's counter RNG, or with flags & LRL_STEP_INJECT_UNIFORM from the lrl_sim_inject_reset_uniforms buffer.
 * env_ids must be distinct (as the reference's torch.arange / nonzero() id lists are): one thread resets each listed
 * env and bumps that env's reset counter (the key of its draws), so an id listed twice would race on both. */
int32_t lrl_sim_reset_idx_ex(lrl_sim* sim, const int32_t* env_ids, int32_t n, int32_t root_mode, float xy_lo,
                             float xy_span, float x_off, float y_off, uint32_t flags, void* stream);
/* Injected reset uniforms for parity tests: u [n, 5] f32 device, row t = (motor strength, Kp, Kd, x, y) of the
 * t-th env id of the next lrl_sim_reset_idx_ex call with LRL_STEP_INJECT_UNIFORM (torch.rand draw order). */
int32_t lrl_sim_inject_reset_uniforms(lrl_sim* sim, const float* u);
/* Upstream reset path (legged_robot.py:177 `reset_idx` inside post_physics_step, re-enabled with
 * legacy_fork=False): after lrl_sim_step + lrl_sim_reset_idx_ex of the envs the step reset, re-run
 * compute_observations (:342-417) for them from the post-reset state with the step's own noise draws, set
 * last_actions / last_dof_vel / last_root_vel as post_physics_step does after reset_idx (:182-184), and with
 * flags & LRL_STEP_HISTORY rewrite the newest history slot (the HistoryWrapper shift of that step). */
int32_t lrl_sim_observe_idx(lrl_sim* sim, const int32_t* env_ids, int32_t n, uint32_t flags, void* stream);
/* _update_terrain_curriculum (legged_robot.py:793-818) for the envs `env_ids` in one launch: distance = |root xy -
 * env origin xy|; move up when distance > half_env_length, down when distance < |command xy| * episode_length_s *
 * 0.5 and not up; a level >= max_level becomes rand_levels[t] (the caller's torch.randint_like draw, one per id),
 * others are clipped at 0; the env origin becomes terrain_origins[level][type].  levels / types: int64 [num_envs]
 * device arrays (the caller's terrain_levels / terrain_types), terrain_origins: f32 [rows][cols][3]; an index
 * outside rows / cols is an error of the caller (clamped on the device: the kernel never reads out of bounds). */
int32_t lrl_sim_terrain_curriculum(lrl_sim* sim, const int32_t* env_ids, int32_t n, int64_t* levels,
                                   const int64_t* types, const int64_t* rand_levels, const float* terrain_origins,
                                   int32_t rows, int32_t cols, float half_env_length, float episode_length_s,
                                   int32_t max_level, void* stream);
/* The upstream step's host-side bookkeeping input in one call (lrl/env.py step, legacy_fork=False): per env
 * code = reset | (((episode_length + 1) % interval == 0 or interval == 1) << 1) as a float, followed — when
 * row0 / row1 >= 0 — by the two command-sum rows (the tracking sums the next curriculum update reads), copied into
 * host_out (pinned host memory, [1 or 3][num_envs] f32) on `stream`; when reset_ids_out (a device int32 array of
 * num_envs) is given, the reset envs' ids in ascending order are written there too (their count is the number of
 * codes with bit 0 set).  Returns after the stream reached the copy. */
int32_t lrl_sim_step_code(lrl_sim* sim, int32_t interval, int32_t row0, int32_t row1, float* host_out,
                          int32_t* reset_ids_out, void* stream);
/* _resample_commands' device writes (legged_robot.py:595-626): commands[ids[i], 0:3] = cmds[i][0:3],
 * command_sums[:, ids] = 0; and, when bins_out is given, bins_out[0:nbins] = bins_in[0:nbins] (the float env-bins
 * tensor of the step's extras).  Device pointers; one launch on `stream`. */
int32_t lrl_sim_apply_commands(lrl_sim* sim, const int32_t* ids, int32_t n, const float* cmds, const float* bins_in,
                               float* bins_out, int32_t nbins, void* stream);
/* common_step_counter (legged_robot.py:153); lrl_sim_step increments it before the launch */
int32_t lrl_sim_set_step_counter(lrl_sim* sim, int64_t counter);
int32_t lrl_sim_set_root_state_indexed(lrl_sim* sim, const float* root /*[N,13] full tensor*/,
                                       const int32_t* env_ids, int32_t n, void* stream);
int32_t lrl_sim_set_dof_state_indexed(lrl_sim* sim, const float* dof_pos, const float* dof_vel,
                                      const int32_t* env_ids, int32_t n, void* stream);
int32_t lrl_sim_refresh_rigid_body_state(lrl_sim* sim, void* stream);
/* VelocityTrackingEasyEnv.step's numpy extras (velocity_tracking_easy_env.py:48-62) as a device snapshot of the
 * current state, enqueued on `stream`: out = device f32 [LRL_EXTRAS_ROWS][num_envs], rows at the LRL_EXTRAS_* offsets
 * (contact states as 1 / 0 for contact force z > 1 on each foot, foot positions as the rigid-body state's feet). */
#define LRL_EXTRAS_JOINT_POS 0
#define LRL_EXTRAS_JOINT_VEL 12
#define LRL_EXTRAS_JOINT_POS_TARGET 24
#define LRL_EXTRAS_BODY_LIN_VEL 36
#define LRL_EXTRAS_BODY_ANG_VEL 39
#define LRL_EXTRAS_COMMANDS 42
#define LRL_EXTRAS_CONTACT_STATES 46
#define LRL_EXTRAS_FOOT_POSITIONS 50
#define LRL_EXTRAS_BODY_POS 62
#define LRL_EXTRAS_TORQUES 65
#define LRL_EXTRAS_ROWS 77
int32_t lrl_sim_extras_snapshot(lrl_sim* sim, float* out, void* stream);

/* ---- the upstream step without a host round trip (lrl/env.py, legacy_fork=False, one process): id lists and their
 * counts stay on the device; `nmax` bounds a device count `dcount` (launch size).
 * lrl_sim_env_lists: mode 0 = the envs whose reset flag is set (reset_idx's ids after check_termination / time-outs),
 * mode 1 = the envs due for command resampling before this step's kernel ((episode_length + 1) % interval == 0, every
 * env when interval == 1: _post_physics_step_callback, legged_robot.py:578-581), ascending as np.flatnonzero. */
int32_t lrl_sim_env_lists(lrl_sim* sim, int32_t mode, int32_t interval, int32_t* ids_out, int32_t* count_out,
                          void* stream);
/* _update_terrain_curriculum (legged_robot.py:793-818) of the listed envs; the wrap-around level is a uniform draw of
 * the counter RNG (global env id, step counter).  lrl_sim_terrain_curriculum with rand_levels == NULL draws the same. */
int32_t lrl_sim_terrain_curriculum_dev(lrl_sim* sim, const int32_t* ids, int32_t nmax, const int32_t* dcount,
                                       int64_t* levels, const int64_t* types, const float* terrain_origins,
                                       int32_t rows, int32_t cols, float half_env_length, float episode_length_s,
                                       int32_t max_level, void* stream);
/* reset_idx's device part (as lrl_sim_reset_idx_ex, counter-RNG draws) and the observation refresh (as
 * lrl_sim_observe_idx) of the listed envs */
int32_t lrl_sim_reset_idx_dev(lrl_sim* sim, const int32_t* ids, int32_t nmax, const int32_t* dcount, int32_t root_mode,
                              float xy_lo, float xy_span, float x_off, float y_off, void* stream);
int32_t lrl_sim_observe_idx_dev(lrl_sim* sim, const int32_t* ids, int32_t nmax, const int32_t* dcount, uint32_t flags,
                                void* stream);
/* reset_idx's episode logging (torch.mean of each row over the ids, then zeroed) with a device count; an empty batch
 * writes `prev` into `means` (the reference's extras keep the last reset batch's values), or leaves `means` as they
 * were when prev is null.  With a fresh `means` buffer per step and the previous step's as `prev`, every step
 * publishes values no later step overwrites (ABI 4: `prev` added). */
int32_t lrl_rows_mean_zero_dev(float* table, int64_t ld, int32_t rows, const int32_t* ids, int32_t nmax,
                               const int32_t* dcount, float* means, const float* prev, int32_t zero, void* stream);
/* The grid-adaptive command curriculum on the device (RewardThresholdCurriculum, curriculum.py:16-124): its state in
 * caller-owned device buffers, bit-exact with the host forms (numpy RandomState MT19937, pairwise sums). */
typedef struct lrl_dev_curriculum {
  double* weights;                 /* [nbins] sampling weights */
  double* cdf;                     /* [nbins] normalised cdf cache */
  int32_t* state;                  /* [4]: cdf valid, MT position, error (1 NaN, 2 negative, 3 bad sum), spare */
  uint32_t* mt_key;                /* [624] MT19937 key (numpy RandomState.get_state()[1]) */
  double *ep_rew_lin, *ep_rew_ang; /* [nbins] episode_reward_lin / _ang */
  int64_t* env_bins;               /* [num_envs] env_command_bins */
  float* env_bins_f;               /* [num_envs] every env's bin as of the last reset batch (extras['env_bins']) */
  double* command_area;            /* [1] np.sum(weights) / nbins at the last resample with log_area */
  const double* axes;              /* [nx + ny + nz] the grid axes (np.linspace of each key range) */
  double half[3];                  /* bin_sizes / 2 */
  int32_t nx, ny, nz;
  uint32_t* words;                 /* scratch [8 * num_envs] */
  double* draws;                   /* scratch [4 * num_envs] */
  const float* env_bins_f_prev;    /* optional: with log_area and an empty batch, env_bins_f / command_area are */
  const double* command_area_prev; /* copied from these (fresh output buffers per step keep earlier steps' values) */
} lrl_dev_curriculum;
/* _resample_commands (legged_robot.py:595-626) of the listed envs: update(old bins, tracking sums / ep_len vs the
 * thresholds, local_range) when `update`, sample(count), then commands[ids, :3] (|xy| > 0.2 mask), command_sums[:, ids]
 * = 0 and the env bins — one workgroup, no host wait.  log_area: also command_area = np.sum(weights) / nbins after
 * the update (reset_idx's log, legged_robot.py:272). */
int32_t lrl_sim_curriculum_resample_dev(lrl_sim* sim, const lrl_dev_curriculum* cur, const int32_t* ids, int32_t nmax,
                                        const int32_t* dcount, int32_t ep_len, int32_t row_lin, int32_t row_ang,
                                        double lin_threshold, double ang_threshold, double local_range, int32_t update,
                                        int32_t log_area, void* stream);
/* Terrain mesh for params->terrain_mesh == 1 (gym.add_triangle_mesh / add_heightfield, legged_robot.py:
 * 1122-1160): `vertices` host [rows*cols][3] in the terrain frame (the Terrain class's trimesh vertices, or
 * the unmoved grid for a heightfield), placed at (-border_size, -border_size, 0) like tm_params.transform;
 * triangles follow the grid (cell (i, j): (v(i,j), v(i+1,j+1), v(i,j+1)) and (v(i,j), v(i+1,j), v(i+1,j+1))).
 * `height_samples` host int16 [rows*cols] (Terrain.heightsamples) feed the height scan. */
int32_t lrl_sim_set_terrain(lrl_sim* sim, const float* vertices, const int16_t* height_samples, int32_t rows,
                            int32_t cols);
/* HistoryWrapper.get_observations side effect (history_wrapper.py:26-30) */
int32_t lrl_sim_shift_history(lrl_sim* sim, void* stream);

/* ------------------------------------------------------------------------------------------
 * PPO numeric core.
 * ------------------------------------------------------------------------------------------ */

/* GAE + advantage normalisation (rollout_storage.py:76-90). rewards/values/returns/advantages
 * [T,N] f32, dones [T,N] u8, last_values [N].  Normalisation uses mean and unbiased std over T*N. */
int32_t lrl_gae(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                int32_t T, int32_t N, float gamma, float lam, float* returns, float* advantages,
                float* workspace /* >= 4096 floats */, void* stream);

/* Multi-GPU split of lrl_gae: returns + raw advantages and stats = (sum, sum of squares, count) as
 * fp64 (all-reduce them across ranks), then normalise with the (global) stats. */
int32_t lrl_gae_partial(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                        int32_t T, int32_t N, float gamma, float lam, float* returns, float* advantages,
                        float* workspace, double* stats /*[3] device*/, void* stream);
int32_t lrl_adv_normalize(float* advantages, int64_t total, const double* stats /*[3] device*/, void* stream);

/* PPO.process_env_step + RolloutStorage.add_transitions for the env outputs (ppo.py:76-88, rollout_storage.py:
 * 57-71) in one launch: dst_rew = rew (+ gamma * values * time_out when time_outs != NULL), dst_done = done (bool
 * bytes), dst_env_bins = env_bins (when given); all [n] device, the dst pointers = storage row t. */
int32_t lrl_ppo_store_step(const float* rew, const uint8_t* done, const float* env_bins, const float* values,
                           const uint8_t* time_outs, float gamma, int32_t n, float* dst_rew, uint8_t* dst_done,
                           float* dst_env_bins, void* stream);

/* ---------------- PPO update (ppo.py:94-178) ----------------
 * All ActorCritic parameters live in ONE flat fp32 buffer (the nn.Module's tensors are views of it);
 * gradients and the Adam moments (exp_avg / exp_avg_sq) are flat buffers of the same layout.  Actor and
 * critic layers are stored pairwise adjacent ([actor W; critic W]) so each pair runs as one grouped
 * GEMM.  Offsets are in floats, 16-B aligned. */
typedef struct lrl_ppo_net {
  int32_t num_obs, num_priv, num_hist, num_actions; /* 42, 18, 630, 12 */
  int32_t enc_h0, enc_h1, latent;                   /* env_factor_encoder 18 -> 256 -> 128 -> 18 */
  int32_t ac_h0, ac_h1, ac_h2;                      /* actor_body / critic_body hidden 512, 256, 128 */
  int32_t ad_h0, ad_h1;                             /* adaptation_module 630 -> 256 -> 32 -> 18 */
  int64_t w1, b1, w2, b2, w3, b3;                   /* [actor; critic] layer pairs */
  int64_t w4a, b4a, w4c, b4c;                       /* actor / critic heads */
  int64_t e1w, e1b, e2w, e2b, e3w, e3b;             /* env_factor_encoder */
  int64_t d1w, d1b, d2w, d2b, d3w, d3b;             /* adaptation_module */
  int64_t std_off;                                  /* std [num_actions] */
  int64_t main_begin, main_end;   /* parameters of the PPO optimiser step (encoder, actor, critic, std) */
  int64_t adapt_begin, adapt_end; /* parameters of the adaptation step */
  int64_t kl_slot;                /* grads[kl_slot] = minibatch KL mean (all-reduced with the grads) */
  int64_t total;                  /* buffer length */
} lrl_ppo_net;

/* One minibatch: the flattened rollout storage ([T*N, .]) and the minibatch's row indices (the int64
 * slice of torch.randperm that mini_batch_generator uses, rollout_storage.py:103-120). */
typedef struct lrl_ppo_batch {
  const float *obs, *priv, *hist, *actions, *values, *returns, *logp, *adv, *mu, *sigma;
  const int64_t* rows;
  int32_t batch;
  int32_t hist_ld; /* row pitch of hist in floats (0 = num_hist).  A pitch of num_hist rounded up to 16 with
                    * finite (zero) padding lets the adaptation module's first layer run on float4 rows. */
} lrl_ppo_batch;

typedef struct lrl_ppo_hparams { /* PPO_Args (ppo.py:15-34) + torch.optim.Adam defaults */
  float clip_param, entropy_coef, value_loss_coef, max_grad_norm, desired_kl;
  int32_t use_clipped_value_loss, adaptive_schedule;
  float beta1, beta2, eps;
} lrl_ppo_hparams;

/* Device-resident control block (caller allocates, zero-initialises and sets lr). */
typedef struct lrl_ppo_ctrl {
  double lr;            /* PPO optimiser learning rate (adaptive-KL schedule, ppo.py:113-124) */
  double loss_sum[3];   /* running sums of value, surrogate and adaptation losses (ppo.py:149-171) */
  float mb[4];          /* this minibatch: value loss, surrogate loss, adaptation loss, kl */
  float clip_scale, step_size, total_norm, pad;
} lrl_ppo_ctrl;

/* Rollout step of PPO.act (ppo.py:62-74): latent = enc(priv); mu = actor([obs, latent]);
 * a = mu + std * eps; value = critic([obs, latent]); logp = sum log N(a; mu, std) — the same fp32-MFMA
 * GEMM chain as the update's forward, then one head kernel.  eps [n, num_actions] is given (injected)
 * or drawn from the counter RNG (seed, counter, global env id = row_offset + row) when eps == NULL — with
 * row_offset the rank's env_offset, a sharded rollout draws what one process holding every env would.  If `store` != NULL the
 * transition (obs, priv, hist, actions, values, logp, mu, sigma) is written to row `store_row` of the
 * [T, n, ...] storage arrays (RolloutStorage.add_transitions, rollout_storage.py:57-71). */
typedef struct lrl_rollout_store {
  float *obs, *priv, *hist, *actions, *values, *logp, *mu, *sigma;
  int32_t hist_dim;
  int32_t hist_ld; /* row pitch of the history storage in floats (0 = hist_dim); padding is left untouched */
} lrl_rollout_store;

int64_t lrl_ppo_act_workspace_bytes(const lrl_ppo_net* net, int32_t n);
int32_t lrl_ppo_act(const lrl_ppo_net* net, const float* params, const float* obs, const float* priv,
                    const float* hist, int32_t n, const float* eps, uint64_t seed, uint64_t counter, int64_t row_offset,
                    float* actions,
                    float* mu, float* values, float* logp, const lrl_rollout_store* store, int32_t store_row,
                    void* workspace, void* stream);

/* Student act (actor_critic.py:160-164, the eval-env path of Runner.learn __init__.py:130-135 and the
 * deployed policy of play.py): latent = adaptation_module(hist) (630 -> 256 -> 32 -> 18, ELU), mean =
 * actor_body([obs, latent]) — deterministic, no sampling.  hist rows at pitch hist_ld (0 = num_hist; a
 * 16-float pitch with finite padding takes the float4 path).  latent [n, latent] may be NULL. */
int64_t lrl_ppo_act_student_workspace_bytes(const lrl_ppo_net* net, int32_t n);
int32_t lrl_ppo_act_student(const lrl_ppo_net* net, const float* params, const float* obs, const float* hist,
                            int32_t hist_ld, int32_t n, float* mean, float* latent, void* workspace, void* stream);

/* Workspace bytes for minibatches of `batch` rows. */
int64_t lrl_ppo_workspace_bytes(const lrl_ppo_net* net, int32_t batch);
/* Forward + backward of the PPO loss (ppo.py:98-147): writes grads[main_begin:main_end) and
 * grads[kl_slot]; ctrl->mb[0..1] = value / surrogate loss. */
int32_t lrl_ppo_forward_backward(const lrl_ppo_net* net, const float* params, float* grads,
                                 const lrl_ppo_batch* batch, const lrl_ppo_hparams* hp, void* workspace,
                                 lrl_ppo_ctrl* ctrl, void* stream);
/* Adaptive LR from the KL (x grad_scale), clip_grad_norm_(max_grad_norm) over grads x grad_scale
 * (grad_scale = 1/world after a SUM all-reduce), Adam step `step` (1-based) over the main region. */
int32_t lrl_ppo_optimizer_step(const lrl_ppo_net* net, float* params, const float* grads, float* exp_avg,
                               float* exp_avg_sq, int64_t step, float grad_scale, const lrl_ppo_hparams* hp,
                               void* workspace, lrl_ppo_ctrl* ctrl, void* stream);
/* Adaptation-module regression (ppo.py:157-171): forward/backward -> grads[adapt_begin:adapt_end),
 * ctrl->mb[2] = MSE.  The encoder target reads the encoder weights at enc_params + net->e1w .. (a snapshot
 * of the flat parameters' encoder range taken after the optimiser step; NULL = params), the adaptation module
 * its own weights in params. */
int32_t lrl_ppo_adaptation_forward_backward(const lrl_ppo_net* net, const float* params, const float* enc_params,
                                            float* grads, const lrl_ppo_batch* batch, void* workspace,
                                            lrl_ppo_ctrl* ctrl, void* stream);
/* Adam step of the adaptation optimiser (fixed lr) over the adaptation region. */
int32_t lrl_ppo_adaptation_step(const lrl_ppo_net* net, float* params, const float* grads, float* exp_avg,
                                float* exp_avg_sq, int64_t step, double lr, float grad_scale,
                                const lrl_ppo_hparams* hp, lrl_ppo_ctrl* ctrl, void* stream);

/* Timing hook for bench.py's roofline: while enabled, HIP events bracket every launch of the update's
 * largest product (actor/critic layer-2 weight gradient, 2 x 256 x 512 over the minibatch rows) on its
 * stream.  Each call returns the summed event time and launch count recorded since the previous call
 * (either pointer may be NULL), clears them, and sets the enable flag for what follows. */
int32_t lrl_ppo_timing(int32_t enable, double* total_ms, int64_t* launches);

/* Development switch of the update's GEMM kernels (tests compare them in one process): bit 0 set = no pre-split-B
 * kernel for the weight products, bit 1 set = no LDS-DMA weight-gradient kernel, bit 2 set = no LDS-DMA
 * forward / backward-data kernel (the fp32-staged x6 kernel takes those products instead); bit 3 set (bit 2 clear) =
 * the LDS-DMA kernel for every forward / backward-data product it fits (it is off by default).  Returns the previous
 * mask. */
int32_t lrl_debug_gemm_paths(int32_t disable_mask);

/* Determinism probe: with mode != 0 every lrl_sim_step of `s` launches, right before its env kernel, a pass that
 * fills every CU's LDS (mode bit 0) and / or every SIMD's VGPR and AGPR files (bit 1) with `pattern`, so an env result
 * that depends on state the launch never wrote moves with the pattern.  mode 0 turns it off. */
int32_t lrl_debug_sim_garbage(lrl_sim* s, uint32_t mode, uint32_t pattern);
/* The sim's state arena (device pointer, bytes) and its step counter, for replay-based determinism checks (a test
 * copies the arena, runs lrl_sim_step, restores the copy and the counter — lrl_sim_set_step_counter — and runs it
 * again).  Any out-pointer may be NULL. */
int32_t lrl_debug_sim_arena(lrl_sim* s, void** arena, int64_t* bytes, int64_t* step_counter);

/* Test entry point of the GEMM the update is built from: C = op(A) op(B) with
 * layout 0 (NT: C[m][n] = sum_k A[m][k] B[n][k]), 2 (NN: sum_k A[m][k] B[k][n]),
 * 3 (TN: sum_k A[k][m] B[k][n], split over k, partials reduced in place);
 * epi 0 store, 1 +bias[n], 2 elu(+bias[n]), 3 *elu'(aux[m][n]).  rows (optional) gathers A's rows
 * (NT/NN) or B's rows (TN).  layout | 0x100 (NT / NN): B is first split into hi / mid / lo bf16 planes in the
 * workspace (3 * N * round16(K) / 2 floats) and the product runs on the pre-split-B kernel the update uses for its
 * weight products, or fails if the shape is not one it takes. */
int32_t lrl_gemm_f32(int32_t layout, int32_t epi, int32_t M, int32_t N, int32_t K, const float* A, int64_t lda,
                     const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, const float* aux,
                     int64_t ld_aux, const int64_t* rows, float* workspace, int64_t workspace_floats, void* stream);

/* reset_idx's episode logging (legged_robot.py:261-276) for `rows` rows of a [rows][ld] f32 device table at once:
 * means[r] = mean over the n env ids of table[r][ids] (fixed-order reduction), then, when `zero`, those entries are
 * set to 0 (the reset envs' episode sums).  One launch on `stream`; means is a device array of `rows` floats (NaN for
 * n == 0, as torch.mean of an empty selection).  Returns 0, or non-zero on a bad argument / launch failure. */
int32_t lrl_rows_mean_zero(float* table, int64_t ld, int32_t rows, const int32_t* ids, int32_t n, float* means,
                           int32_t zero, void* stream);

/* ---- host-side grid-adaptive command curriculum (CPU functions, no device work) ----
 * Native form of RewardThresholdCurriculum.sample / .update (mini_gym/envs/base/curriculum.py:56-68, 105-115), which
 * the reference runs in numpy on every resampling (legged_robot.py:595-626; lrl/curriculum.py restates it): bit-exact
 * with numpy.random.RandomState.  mt_key / mt_pos: the generator's MT19937 state (624 words + position, numpy's
 * RandomState.get_state()[1:3]), advanced in place.
 * sample: bins[j] = choice(nbins, p = weights / weights.sum()) for j < n, then cmds[j][d] = uniform(grid[d][bin] +
 * half[d], grid[d][bin] - half[d]) in C order; grid is [3][nbins] f64.  Errors as numpy's choice (p not
 * non-negative / NaN / not summing to 1). */
int32_t lrl_curriculum_sample(uint32_t* mt_key, int32_t* mt_pos, const double* weights, int32_t nbins,
                              const double* grid, const double* half, int32_t n, double* cmds, int64_t* bins);
/* update's weight adds for the successful bins `centres`: weights[centres] = clip(weights[centres] + 0.2, 0, 1), then
 * every bin within +-local_range of each centre on all three axes (axes: the nx, ny, nz axis values, concatenated;
 * bin = (ix * ny + iy) * nz + iz) gets one clipped add per centre, in centre order. */
int32_t lrl_curriculum_update_weights(double* weights, const double* axes, int32_t nx, int32_t ny, int32_t nz,
                                      const int64_t* centres, int32_t n, double local_range);
/* numpy's np.sum of a contiguous f64 array (pairwise summation), the normaliser of the sample's p */
double lrl_np_sum_f64(const double* a, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* LRL_H_ */
