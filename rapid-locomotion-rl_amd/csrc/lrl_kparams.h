// Device-side parameter block of one sim: lrl_env_params + the model tables pre-digested for the
// quadruped kernel (per-leg joint frames, contact spheres grouped by leg and body).  Uploaded once
// by lrl_sim_create; every kernel reads it through a __restrict__ const pointer, so the compiler
// turns the (wave-uniform) accesses into scalar loads.
#pragma once
#include <stdint.h>

#include "../../include/lrl.h"

// Lanes per env-step workgroup (4 lanes per env).  A workgroup is one wave; with 4096 envs, 64 lanes give 256
// waves (one per CU: three of each CU's four SIMDs idle), 32 lanes give 512 and 16 give 1024 (one per SIMD).
// The kernel is bound by each env's dependent chain, and a wave's instruction stream costs the same whatever
// its active-lane count, so fewer envs per wave spreads the same chains over more SIMDs.
#ifndef LRL_ENV_LANES
#define LRL_ENV_LANES 64
#endif
// envs per workgroup: the terrain-mesh kernel keeps one quad per env (16 envs per wave); the plane kernel runs 4 envs
// per wave, 16 lanes (4 mirrored quads) per env (lrl_env.hip, lrl_env_flat.hip)
#define LRL_ENV_WG_ENVS_MESH (LRL_ENV_LANES / 4)
#define LRL_ENV_WG_ENVS_FLAT (LRL_ENV_LANES / 16)
// LDS fields per leg block / per contact-sphere row of the env kernel (lrl_env.hip): the plane build carries the TGS
// solver's extra fields (the leg's accumulated joint-space motion dz, a contact's restitution target), the terrain-mesh
// build has no room for them (its 16-env workgroup fills the CU's LDS) and solves with PGS
#define LRL_LEGF_MESH 51
#define LRL_LEGF_FLAT 54
#define LRL_NSF_MESH 67
#define LRL_NSF_FLAT 68

struct KLeg {
  float xyz[3][3];   // joint origin in the parent frame
  float rfix[3][9];  // fixed joint-origin rotation (row-major)
  float axis[3][3];  // joint axis (child frame)
  float mass[3], com[3][3], inertia[3][6];  // calf includes the fixed foot
};

struct KParams {
  lrl_env_params p;
  KLeg leg[LRL_NUM_LEGS];
  float base_mass, base_inertia[6];
  // joint position limits in dof order (3 l + j), +-1e30 for a joint without limits (lrl_model::dof_lower / upper)
  float dof_lo[LRL_NUM_DOF], dof_hi[LRL_NUM_DOF];
  int32_t num_bodies, num_spheres;
  // spheres sorted by body (model order: base, then leg 0..3)
  float sph_pos[LRL_MAX_SPHERES][3];
  float sph_rad[LRL_MAX_SPHERES];
  int32_t sph_link[LRL_MAX_SPHERES];  // 0..2 dynamic link inside the leg, -1 base
  int32_t sph_leg[LRL_MAX_SPHERES];   // 0..3, -1 base
  // mesh colliders (lrl_model::sphere_hull, ABI 6): support table of sphere s (-1: the sphere itself), the tables in
  // device memory [hull][6][hull_res][hull_res][hull_k] float4 (lrl_env.hip hull_support; both builds)
  int32_t sph_hull[LRL_MAX_SPHERES];
  const float* hull_tab;
  int32_t hull_res, hull_k;
  int32_t base_sph_end;               // spheres [0, base_sph_end) are on the base
  int32_t leg_sph_begin[LRL_NUM_LEGS], leg_sph_end[LRL_NUM_LEGS];
  int32_t body_sph_begin[LRL_MAX_BODIES], body_sph_end[LRL_MAX_BODIES];
  int32_t body_foot[LRL_MAX_BODIES];  // foot slot 0..3 or -1
  // self-collision candidates (p.self_collisions; lrl_capi.cpp::self_pairs): the canonical pair order is lane (leg
  // La) major, then per lane the groups g = 0 pairs inside leg La, g = 1..3 against leg La + g, g = 4 against the base
  // box; a pair packs sphere a | sphere b << 8 (255 = the base box) | body of a << 16 | body of b << 24
  int32_t self_npairs;
  int32_t self_nhip[LRL_NUM_LEGS];  // the leg's leading link-0 spheres with a radius (the same-leg group's sphere a)
  int32_t self_kmax;                // most spheres on one leg (<= 8)
  int32_t self_grp[LRL_NUM_LEGS][5][2];  // [lane][group] -> [begin, end) in self_pair
  uint32_t self_pair[LRL_MAX_SELF_PAIRS];
  float box_c[3], box_h[3];  // base box (the span of the base's spheres): centre and half extents, base frame
  int32_t num_history;
  int32_t n_es, n_cs;                 // rows of episode_sums / command_sums
  // terrain mesh (p.terrain_mesh == 1, lrl_sim_set_terrain): vertex grid [rows][cols] as (x, y, z, 0) in the
  // world frame, the max vertex z over the 4x4 vertices a contact query at cell (i, j) reads, and the height
  // samples in metres for the height scan
  const float* terr_vtx;
  const float* terr_hmax;
  const float* terr_h;
  const float* terr_wmax;  // max vertex z over the window around a base cell (terrain_window_max)
  int32_t terr_rows, terr_cols;
  float terr_inv_hs;
  // lrl_sim_self_contact_stats: null (off), or 4 device counters [env-sub-steps with a self-contact, pairs in contact,
  // env-sub-steps with more pairs than slots, pairs without a slot]
  uint32_t* self_stats;
};

// SoA device buffers of a sim (each [.][N] with N = padded env count unless noted).
struct KState {
  int32_t n;       // real env count
  int32_t stride;  // padded N (multiple of 64)
  int64_t env_offset;
  uint64_t seed;
  float *root, *dof_pos, *dof_vel, *contact, *rb_state, *torques, *actions, *last_actions, *last_dof_vel,
      *last_root_vel, *commands, *obs, *priv, *hist, *rew;
  uint8_t *reset, *time_out, *last_contacts;
  int32_t* episode_length;
  int32_t* reset_count;  // per-env reset_idx count: the reset draws' counter (independent of the sharding)
  float *episode_sums, *command_sums, *feet_air_time, *friction, *restitution, *payload, *com, *motor_strength,
      *kp, *kd, *env_origins, *base_lin_vel, *base_ang_vel, *projected_gravity, *joint_pos_target;
  float* heights;  // measured_heights [num_height_points][N]
  const float *inj_noise, *inj_dr;
  const float* inj_push;   // [n][2] injected _push_robots uniforms
  const float* inj_reset;  // [n_ids][5] (motor strength, Kp, Kd, x, y) uniforms of an injected reset_idx
};
