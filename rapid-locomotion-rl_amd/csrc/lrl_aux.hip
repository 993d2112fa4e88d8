// lrl_aux.hip — the non-step env kernels: reset_idx (device part), indexed state setters,
// rigid-body-state refresh (forward kinematics), HistoryWrapper shift, DR initialisation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <stdint.h>

#include "../../include/lrl_philox.h"
#include "lrl_kparams.h"

namespace lrl {

// The reset / curriculum kernels follow torch's float32 op order exactly: plain operators under this pragma (the
// build uses -ffp-contract=fast-honor-pragmas, so it really keeps multiply-adds unfused).  Not __fmul_rn / __fadd_rn:
// HIP defines them as plain operators in its own header, where contraction is on, so a product inlined from them
// still fuses with the sum around it.
#pragma clang fp contract(off)

// reset_idx (legged_robot.py:227-290) device part: _randomize_dof_props (:544-560), _reset_dofs
// (:690-712), _reset_root_states (:714-755), buffer zeroing (:255-259).  root_mode (lrl.h): 0 = leave the root
// (fork quirk Q4 for custom origins), 1 = base_init_state + env_origin, 2 = custom origins with the upstream
// xy draw xy_span * u + xy_lo and the (x_off, y_off) init offsets.  Uniform draws: (motor strength, Kp, Kd, x, y)
// from Philox keyed by (global env, reset counter), or row t of S.inj_reset (the reference's torch.rand draws,
// one row per env id in id order).  Float32 arithmetic in the reference's operation order, uncontracted.
// (dn: the id count on the device, the host's n is then the launch bound — the upstream step's asynchronous path.)
// The draws' counter is the env's own reset count (S.reset_count, bumped here), so a global env draws the same values
// whatever the sharding: it depends on that env's history only, not on which other envs share its process.
__global__ void reset_kernel(const KParams* __restrict__ K, KState S, const int32_t* __restrict__ ids, int32_t n,
                             const int32_t* __restrict__ dn, int32_t root_mode, float xy_lo, float xy_span, float x_off,
                             float y_off, int32_t inject) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (dn ? min(*dn, n) : n)) return;
  const lrl_env_params& P = K->p;
  const int N = S.stride;
  int e = ids[t];
  if (e < 0 || e >= S.n) return;
  const uint32_t counter = (uint32_t)S.reset_count[e];
  S.reset_count[e] = (int32_t)(counter + 1u);
  float u[5];
  if (inject) {
    for (int k = 0; k < 5; ++k) u[k] = S.inj_reset[(size_t)t * 5 + k];
  } else {
    uint64_t genv = (uint64_t)(S.env_offset + e);
    const uint32_t key = (uint32_t)LRL_RNG_RESET << 16;
    lrl_u32x4 r = lrl_philox((uint32_t)genv, counter, key, 0, S.seed);
    lrl_u32x4 r2 = lrl_philox((uint32_t)genv, counter, key, 1, S.seed);
    for (int k = 0; k < 4; ++k) u[k] = lrl_u01(r.v[k]);
    u[4] = lrl_u01(r2.v[0]);
  }
  // torch.rand(k) * (max - min) + min: two float32 roundings, the span rounded once from the python floats
  auto draw = [](float uu, float span, float lo) { return uu * span + lo; };
  if (P.randomize_motor_strength) {
    float v = draw(u[0], P.dr_span[0], P.motor_strength_range[0]);
    for (int j = 0; j < 12; ++j) S.motor_strength[j * N + e] = v;
  }
  if (P.randomize_kp) {
    float v = draw(u[1], P.dr_span[1], P.kp_range[0]);
    for (int j = 0; j < 12; ++j) S.kp[j * N + e] = v;
  }
  if (P.randomize_kd) {
    float v = draw(u[2], P.dr_span[2], P.kd_range[0]);
    for (int j = 0; j < 12; ++j) S.kd[j * N + e] = v;
  }
  for (int j = 0; j < 12; ++j) {
    S.dof_pos[j * N + e] = P.default_dof_pos[j];
    S.dof_vel[j * N + e] = 0.f;
    S.last_actions[j * N + e] = 0.f;
    S.last_dof_vel[j * N + e] = 0.f;
  }
  if (root_mode != 0) {
    // torch_rand_float(lo, hi, (k, 2)) = (hi - lo) * rand + lo, xy_span = float32(hi - lo) from the host
    for (int c = 0; c < 13; ++c) {
      float v = P.base_init_state[c];
      if (c < 3) v = v + S.env_origins[c * N + e];
      if (root_mode == 2 && c < 2) {
        v = v + (xy_span * u[3 + c] + xy_lo);
        v = v + (c == 0 ? x_off : y_off);
      }
      S.root[c * N + e] = v;
    }
  }
  for (int f = 0; f < 4; ++f) S.feet_air_time[f * N + e] = 0.f;
  S.episode_length[e] = 0;
  S.reset[e] = 1;
}

// _update_terrain_curriculum (legged_robot.py:793-818), one thread per reset env.  Float32 ops in torch's order
// without contraction (torch.norm of a 2-vector: x0*x0 + x1*x1, then sqrt; the command term (|c| * T) * 0.5).
// rnd: injected wrap-around draws (one per id, the tests' reference draws); null: a uniform level in [0, max_level) from
// the counter RNG keyed by (global env, step counter) — torch.randint_like's role (the reference's draws come from the
// global torch generator, not reproducible across process layouts either)
__global__ void terrain_curriculum_kernel(KState S, const int32_t* __restrict__ ids, int32_t n,
                                          const int32_t* __restrict__ dn, int64_t* levels,
                                          const int64_t* __restrict__ types, const int64_t* __restrict__ rnd,
                                          const float* __restrict__ torig, int32_t rows, int32_t cols, float half,
                                          float ep_len_s, int32_t max_level, int64_t step_counter) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (dn ? min(*dn, n) : n)) return;
  const int e = ids[t];
  if (e < 0 || e >= S.n) return;
  const int N = S.stride;
  const float dx = S.root[e] - S.env_origins[e], dy = S.root[N + e] - S.env_origins[N + e];
  const float dist = sqrtf(dx * dx + dy * dy);
  const float c0 = S.commands[e], c1 = S.commands[N + e];
  const float cn = sqrtf(c0 * c0 + c1 * c1);
  const bool up = dist > half;
  const bool down = dist < (cn * ep_len_s) * 0.5f && !up;
  int64_t lv = levels[e] + (up ? 1 : 0) - (down ? 1 : 0);
  if (lv >= max_level) {
    if (rnd) {
      lv = rnd[t];
    } else {
      const lrl_u32x4 r = lrl_philox((uint32_t)(S.env_offset + e), (uint32_t)step_counter,
                                     (LRL_RNG_TERRAIN << 16) ^ (uint32_t)(step_counter >> 32), 0, S.seed);
      lv = (int64_t)(((uint64_t)r.v[0] * (uint64_t)max_level) >> 32);
    }
  } else if (lv < 0) {
    lv = 0;
  }
  levels[e] = lv;
  const int64_t li = lv < 0 ? 0 : (lv >= rows ? rows - 1 : lv);
  const int64_t ty = types[e] < 0 ? 0 : (types[e] >= cols ? cols - 1 : types[e]);
  const float* o = torig + (li * cols + ty) * 3;
  for (int c = 0; c < 3; ++c) S.env_origins[c * N + e] = o[c];
}

// gym.set_actor_root_state_tensor_indexed: rows `ids` of an AoS [n,13] source
__global__ void set_root_kernel(KState S, const float* __restrict__ src, const int32_t* __restrict__ ids, int32_t n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int e = ids[t];
  if (e < 0 || e >= S.n) return;
  for (int c = 0; c < 13; ++c) S.root[c * S.stride + e] = src[(size_t)e * 13 + c];
}

__global__ void set_dof_kernel(KState S, const float* __restrict__ pos, const float* __restrict__ vel,
                               const int32_t* __restrict__ ids, int32_t n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int e = ids[t];
  if (e < 0 || e >= S.n) return;
  for (int j = 0; j < 12; ++j) {
    S.dof_pos[j * S.stride + e] = pos[(size_t)e * 12 + j];
    S.dof_vel[j * S.stride + e] = vel[(size_t)e * 12 + j];
  }
}

// forward kinematics -> rigid body state [B][13][N]: pos, quat (xyzw), lin vel (origin), ang vel; world
__device__ inline void mat_to_quat(const float* m, float* q) {
  float t = m[0] + m[4] + m[8];
  if (t > 0.f) {
    float s = sqrtf(t + 1.f) * 2.f;
    q[3] = 0.25f * s; q[0] = (m[7] - m[5]) / s; q[1] = (m[2] - m[6]) / s; q[2] = (m[3] - m[1]) / s;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    float s = sqrtf(1.f + m[0] - m[4] - m[8]) * 2.f;
    q[3] = (m[7] - m[5]) / s; q[0] = 0.25f * s; q[1] = (m[1] + m[3]) / s; q[2] = (m[2] + m[6]) / s;
  } else if (m[4] > m[8]) {
    float s = sqrtf(1.f + m[4] - m[0] - m[8]) * 2.f;
    q[3] = (m[2] - m[6]) / s; q[0] = (m[1] + m[3]) / s; q[1] = 0.25f * s; q[2] = (m[5] + m[7]) / s;
  } else {
    float s = sqrtf(1.f + m[8] - m[0] - m[4]) * 2.f;
    q[3] = (m[3] - m[1]) / s; q[0] = (m[2] + m[6]) / s; q[1] = (m[5] + m[7]) / s; q[2] = 0.25f * s;
  }
}
__device__ inline void mm3(const float* A, const float* B, float* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
__device__ inline void mv3(const float* A, const float* v, float* o) {
  for (int i = 0; i < 3; ++i) o[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
}
__device__ inline void cr3(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
}

// Base pose of env e: rotation R (row-major, from the xyzw quaternion), origin p, origin velocity vo (COM velocity
// - w x (R c)) and angular velocity W
__device__ inline void base_pose(const KState& S, int e, float* R, float* p, float* vo, float* W) {
  const int N = S.stride;
  float q[4], V[3];
  for (int k = 0; k < 4; ++k) q[k] = S.root[(3 + k) * N + e];
  for (int k = 0; k < 3; ++k) { p[k] = S.root[k * N + e]; V[k] = S.root[(7 + k) * N + e]; W[k] = S.root[(10 + k) * N + e]; }
  float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
  float c[3] = {S.com[e], S.com[N + e], S.com[2 * N + e]}, Rc[3], wc[3];
  mv3(R, c, Rc);
  cr3(W, Rc, wc);
  for (int k = 0; k < 3; ++k) vo[k] = V[k] - wc[k];
}

// Forward kinematics of body (leg, link) of env e (leg < 0: the base; link 3: the foot frame at foot_xyz[leg]):
// rotation Rb, origin ob, origin velocity vb, angular velocity wb
__device__ inline void body_fk(const KParams* __restrict__ K, const KState& S, int e, int leg, int link,
                               const float* __restrict__ foot_xyz, const float* R, const float* p, const float* vo,
                               const float* W, float* Rb, float* ob, float* vb, float* wb) {
  const int N = S.stride;
  for (int k = 0; k < 9; ++k) Rb[k] = R[k];
  for (int k = 0; k < 3; ++k) { ob[k] = p[k]; vb[k] = vo[k]; wb[k] = W[k]; }
  if (leg < 0) return;
  const KLeg& L = K->leg[leg];
  int nj = link > 2 ? 3 : link + 1;
  for (int j = 0; j < nj; ++j) {
    float off[3], tmp[9], Rj[9], ax[3], axw[3];
    mv3(Rb, L.xyz[j], off);
    for (int k = 0; k < 3; ++k) ob[k] += off[k];
    // velocity of the new origin: v += w x off
    float wo[3];
    cr3(wb, off, wo);
    for (int k = 0; k < 3; ++k) vb[k] += wo[k];
    mm3(Rb, L.rfix[j], tmp);
    float th = S.dof_pos[(3 * leg + j) * N + e], sn, cs;
    sincosf(th, &sn, &cs);
    float t1 = 1.f - cs;
    for (int k = 0; k < 3; ++k) ax[k] = L.axis[j][k];
    float Ra[9] = {t1 * ax[0] * ax[0] + cs, t1 * ax[0] * ax[1] - sn * ax[2], t1 * ax[0] * ax[2] + sn * ax[1],
                   t1 * ax[0] * ax[1] + sn * ax[2], t1 * ax[1] * ax[1] + cs, t1 * ax[1] * ax[2] - sn * ax[0],
                   t1 * ax[0] * ax[2] - sn * ax[1], t1 * ax[1] * ax[2] + sn * ax[0], t1 * ax[2] * ax[2] + cs};
    mm3(tmp, Ra, Rj);
    for (int k = 0; k < 9; ++k) Rb[k] = Rj[k];
    mv3(Rb, ax, axw);
    float qd = S.dof_vel[(3 * leg + j) * N + e];
    for (int k = 0; k < 3; ++k) wb[k] += qd * axw[k];
  }
  if (link == 3) {
    float off[3], wo[3];
    mv3(Rb, &foot_xyz[3 * leg], off);
    cr3(wb, off, wo);
    for (int k = 0; k < 3; ++k) { ob[k] += off[k]; vb[k] += wo[k]; }
  }
}

__global__ void rigid_body_kernel(const KParams* __restrict__ K, KState S, const int32_t* __restrict__ body_leg,
                                  const int32_t* __restrict__ body_link, const float* __restrict__ foot_xyz) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const int N = S.stride;
  float R[9], p[3], vo[3], W[3];
  base_pose(S, e, R, p, vo, W);
  for (int b = 0; b < K->num_bodies; ++b) {
    float Rb[9], ob[3], vb[3], wb[3];
    body_fk(K, S, e, body_leg[b], body_link[b], foot_xyz, R, p, vo, W, Rb, ob, vb, wb);
    float qb[4];
    mat_to_quat(Rb, qb);
    float* out = S.rb_state + (size_t)b * 13 * N;
    for (int k = 0; k < 3; ++k) out[k * N + e] = ob[k];
    for (int k = 0; k < 4; ++k) out[(3 + k) * N + e] = qb[k];
    for (int k = 0; k < 3; ++k) { out[(7 + k) * N + e] = vb[k]; out[(10 + k) * N + e] = wb[k]; }
  }
}

// VelocityTrackingEasyEnv.step's per-step numpy extras (velocity_tracking_easy_env.py:48-62) as one device snapshot,
// rows of n floats (lrl.h LRL_EXTRAS_*): dof_pos, dof_vel, joint_pos_target (12 each), base_lin_vel, base_ang_vel (3),
// commands (4), contact states of the feet (contact force z > 1: 1 / 0), foot positions (4 x 3, the rigid-body state's
// feet), root position (3), torques (12).  Coalesced: thread e reads row r of every SoA field at word e.
// four threads per env (wave-uniform quarter q = threadIdx.x / 64, 64 consecutive envs per wave: every store row is
// coalesced): the plain rows split over the quarters, foot q's forward kinematics on quarter q
__global__ __launch_bounds__(256) void extras_snapshot_kernel(const KParams* __restrict__ K, KState S,
                                                              const int32_t* __restrict__ body_leg,
                                                              const int32_t* __restrict__ body_link,
                                                              const float* __restrict__ foot_xyz, float* __restrict__ out) {
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  if (e >= S.n) return;
  const int N = S.stride, n = S.n;
  const lrl_env_params& P = K->p;
  // rows: dof_pos 0-11, dof_vel 12-23, joint_pos_target 24-35, base lin / ang vel 36-41, commands 42-45,
  // foot contacts 46-49, foot positions 50-61, base position 62-64, torques 65-76
  auto put = [&](int r, float v) { out[(int64_t)r * n + e] = v; };
  for (int k = q; k < 12; k += 4) {
    put(k, S.dof_pos[k * N + e]);
    put(12 + k, S.dof_vel[k * N + e]);
    put(24 + k, S.joint_pos_target[k * N + e]);
    put(65 + k, S.torques[k * N + e]);
  }
  if (q < 3) {
    put(36 + q, S.base_lin_vel[q * N + e]);
    put(39 + q, S.base_ang_vel[q * N + e]);
  }
  put(42 + q, S.commands[q * N + e]);
  put(46 + q, q < P.num_feet && S.contact[(P.feet[q] * 3 + 2) * N + e] > 1.f ? 1.f : 0.f);
  float R[9], p[3], vo[3], W[3];
  base_pose(S, e, R, p, vo, W);
  if (q < 3) put(62 + q, p[q]);
  float Rb[9], ob[3] = {0.f, 0.f, 0.f}, vb[3], wb[3];
  if (q < P.num_feet) body_fk(K, S, e, body_leg[P.feet[q]], body_link[P.feet[q]], foot_xyz, R, p, vo, W, Rb, ob, vb, wb);
  for (int k = 0; k < 3; ++k) put(50 + 3 * q + k, ob[k]);
}

// HistoryWrapper.get_observations shift: hist = cat(hist[:, NO:], obs)  (history_wrapper.py:26-30)
// HistoryWrapper history shift outside the step (get_observations, Q6): one workgroup per env row, the row
// staged through LDS so every load and store is coalesced
// append 0: the first H - NO floats only (hist[:, :H-NO] = hist[:, NO:]) — the shift half of the HistoryWrapper.step
// update, launched by lrl_sim_step before the env kernel, which then writes the newest slot from its obs tile (a
// bandwidth-shaped launch of 4096 workgroups instead of a latency-bound pass in the env kernel's single waves)
__global__ void shift_history_kernel(KState S, int NO, int H, int append) {
  extern __shared__ float row[];
  const int e = blockIdx.x;
  if (e >= S.n) return;
  float* h = S.hist + (size_t)e * H;
  const float* o = S.obs + (size_t)e * NO;
  const int W = append ? H : H - NO;
  for (int k = threadIdx.x; k < W; k += blockDim.x) row[k] = k < H - NO ? h[k + NO] : o[k - (H - NO)];
  __syncthreads();
  for (int k = threadIdx.x; k < W; k += blockDim.x) h[k] = row[k];
}

// _randomize_rigid_body_props (legged_robot.py:519-542) for all envs
__global__ void randomize_kernel(KState S, float f0, float f1, float r0, float r1, float p0, float p1, float c0,
                                 float c1, uint32_t which) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.stride) return;
  const int N = S.stride;
  uint64_t genv = (uint64_t)(S.env_offset + e);
  lrl_u32x4 a = lrl_philox((uint32_t)genv, 0u, (LRL_RNG_INIT << 16), 0, S.seed);
  lrl_u32x4 b = lrl_philox((uint32_t)genv, 0u, (LRL_RNG_INIT << 16), 1, S.seed);
  if (which & 1u) S.payload[e] = lrl_u01(a.v[0]) * (p1 - p0) + p0;
  if (which & 2u)
    for (int k = 0; k < 3; ++k) S.com[k * N + e] = lrl_u01(k == 0 ? a.v[1] : k == 1 ? a.v[2] : a.v[3]) * (c1 - c0) + c0;
  if (which & 4u) S.friction[e] = lrl_u01(b.v[0]) * (f1 - f0) + f0;
  if (which & 8u) S.restitution[e] = lrl_u01(b.v[1]) * (r1 - r0) + r0;
}

// reset_idx's episode logging (legged_robot.py:261-276: torch.mean(episode_sums[key][env_ids]), then the sums of
// those envs zeroed) for every row of a [rows][ld] table in one launch: workgroup r sums row r over the ids in a
// fixed order (strided per-thread partials, then an LDS tree), writes the mean, and after a barrier zeroes the
// entries it read.
// (dn: the id count on the device, n its bound; an empty batch then leaves the previous means in place, as the
// reference's extras keep the last reset batch's episode dict)
__global__ void rows_mean_zero_kernel(float* __restrict__ tab, int64_t ld, const int32_t* __restrict__ ids, int32_t n,
                                      const int32_t* __restrict__ dn, float* __restrict__ means,
                                      const float* __restrict__ prev, int32_t zero) {
  __shared__ float red[256];
  if (dn) {
    n = min(*dn, n);
    if (n == 0) {
      if (prev && threadIdx.x == 0) means[blockIdx.x] = prev[blockIdx.x];
      return;
    }
  }
  float* row = tab + (int64_t)blockIdx.x * ld;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += row[ids[i]];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) means[blockIdx.x] = n > 0 ? red[0] / (float)n : NAN;
  if (zero)
    for (int i = threadIdx.x; i < n; i += 256) row[ids[i]] = 0.f;
}

// The upstream step's per-env code for the host (lrl/env.py step): bit 0 = reset now, bit 1 = due for command
// resampling in the next step ((episode_length + 1) % interval == 0, episode length after this step's resets; every
// env when interval == 1), as a float, then the two tracking command-sum rows the next curriculum update reads:
// out = [code | sums[r0] | sums[r1]] (n floats each; the rows only when r0 >= 0).
__global__ void step_code_kernel(KState S, int32_t interval, int32_t r0, int32_t r1, float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  uint32_t code = S.reset[e];
  if (interval == 1 || (S.episode_length[e] + 1) % interval == 0) code |= 2u;
  out[e] = (float)code;
  if (r0 >= 0) {
    out[S.n + e] = S.command_sums[(int64_t)r0 * S.stride + e];
    out[2 * S.n + e] = S.command_sums[(int64_t)r1 * S.stride + e];
  }
}

// The step's reset env ids in ascending order (np.flatnonzero of the reset flags), compacted on the device by one
// 1024-thread workgroup: thread t counts the flags of its contiguous run, a block-wide exclusive scan gives its write
// offset (deterministic: the order is the env order).
// MODE 0: the reset flags; MODE 1: the envs due for command resampling before this step's kernel ((episode_length + 1)
// % interval == 0, every env when interval == 1: _post_physics_step_callback's set).  count_out (optional): the count.
template <int MODE>
__global__ __launch_bounds__(1024) void compact_kernel(KState S, int32_t interval, int32_t* __restrict__ ids_out,
                                                       int32_t* __restrict__ count_out) {
  __shared__ int cnt[1024];
  const int t = threadIdx.x, n = S.n;
  const int per = (n + 1023) / 1024, b = t * per, e = min(n, b + per);
  auto flag = [&](int i) {
    return MODE == 0 ? S.reset[i] != 0 : (interval == 1 || (S.episode_length[i] + 1) % interval == 0);
  };
  int c = 0;
  for (int i = b; i < e; ++i) c += flag(i);
  cnt[t] = c;
  __syncthreads();
  for (int w = 1; w < 1024; w <<= 1) {  // inclusive Hillis-Steele scan
    const int v = t >= w ? cnt[t - w] : 0;
    __syncthreads();
    cnt[t] += v;
    __syncthreads();
  }
  int o = cnt[t] - c;
  for (int i = b; i < e; ++i)
    if (flag(i)) ids_out[o++] = i;
  if (count_out && t == 1023) count_out[0] = cnt[1023];
}

// _resample_commands' device writes (legged_robot.py:595-626 as lrl/env.py restates it): commands[ids, :3] = cmds,
// command_sums[:, ids] = 0 (every row); then, when given, bins_out[:nb] = bins_in[:nb] (the env-bins tensor).
__global__ void apply_commands_kernel(KState S, int32_t ncs, const int32_t* __restrict__ ids, int32_t n,
                                      const float* __restrict__ cmds, const float* __restrict__ bins_in,
                                      float* __restrict__ bins_out, int32_t nb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int e = ids[i];
    for (int k = 0; k < 3; ++k) S.commands[(int64_t)k * S.stride + e] = cmds[i * 3 + k];
    for (int r = 0; r < ncs; ++r) S.command_sums[(int64_t)r * S.stride + e] = 0.f;
  }
  if (bins_out && i < nb) bins_out[i] = bins_in[i];
}

// Determinism probe (lrl_debug_sim_garbage): state a launch never wrote — LDS outside what the env kernel stores first,
// VGPR / AGPR lanes it reads before defining them — holds whatever the previous wave on that CU / SIMD left, which in a
// multi-process run is another process's data.  These kernels leave a known pattern there right before the env
// kernel, so an env result that moves with the pattern names such a read.  Vector moves and LDS stores only.
__global__ __launch_bounds__(64) void garbage_lds_kernel(uint32_t pat) {
  extern __shared__ uint32_t g_lds[];
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += 64) g_lds[i] = pat ^ (uint32_t)(i & 3);
}
#define LRL_GV(n) asm volatile("v_mov_b32 v" #n ", %0" ::"s"(pat) : "v" #n);
#define LRL_GA(n) asm volatile("v_accvgpr_write_b32 a" #n ", %0" ::"v"(pv) : "a" #n);
#define LRL_G10(M, d) M(d##0) M(d##1) M(d##2) M(d##3) M(d##4) M(d##5) M(d##6) M(d##7) M(d##8) M(d##9)
#define LRL_G250(M)                                                                                                   \
  M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) LRL_G10(M, 1) LRL_G10(M, 2) LRL_G10(M, 3) LRL_G10(M, 4)            \
  LRL_G10(M, 5) LRL_G10(M, 6) LRL_G10(M, 7) LRL_G10(M, 8) LRL_G10(M, 9) LRL_G10(M, 10) LRL_G10(M, 11) LRL_G10(M, 12) \
  LRL_G10(M, 13) LRL_G10(M, 14) LRL_G10(M, 15) LRL_G10(M, 16) LRL_G10(M, 17) LRL_G10(M, 18) LRL_G10(M, 19)           \
  LRL_G10(M, 20) LRL_G10(M, 21) LRL_G10(M, 22) LRL_G10(M, 23) LRL_G10(M, 24)
__global__ __launch_bounds__(64) void garbage_vgpr_kernel(uint32_t pat) {
  const uint32_t pv = pat ^ threadIdx.x;  // (lane-varying in the AGPRs)
  LRL_G250(LRL_GA)
  LRL_GA(250) LRL_GA(251) LRL_GA(252) LRL_GA(253) LRL_GA(254) LRL_GA(255)
  LRL_G250(LRL_GV)
  LRL_GV(250) LRL_GV(251) LRL_GV(252) LRL_GV(253) LRL_GV(254) LRL_GV(255)
}
#undef LRL_GV
#undef LRL_GA
#undef LRL_G10
#undef LRL_G250

}  // namespace lrl

extern "C" {
hipError_t lrl_launch_step_code(const KState* S, int32_t interval, int32_t r0, int32_t r1, float* out, int32_t* ids_out,
                                hipStream_t st) {
  if (out)
    hipLaunchKernelGGL(lrl::step_code_kernel, dim3((S->n + 255) / 256), dim3(256), 0, st, *S, interval, r0, r1, out);
  if (ids_out)
    hipLaunchKernelGGL(lrl::compact_kernel<0>, dim3(1), dim3(1024), 0, st, *S, interval, ids_out, (int32_t*)nullptr);
  return hipGetLastError();
}
hipError_t lrl_launch_env_lists(const KState* S, int32_t mode, int32_t interval, int32_t* ids_out, int32_t* count_out,
                                hipStream_t st) {
  if (mode == 0)
    hipLaunchKernelGGL(lrl::compact_kernel<0>, dim3(1), dim3(1024), 0, st, *S, interval, ids_out, count_out);
  else
    hipLaunchKernelGGL(lrl::compact_kernel<1>, dim3(1), dim3(1024), 0, st, *S, interval, ids_out, count_out);
  return hipGetLastError();
}
hipError_t lrl_launch_apply_commands(const KState* S, int32_t ncs, const int32_t* ids, int32_t n, const float* cmds,
                                     const float* bins_in, float* bins_out, int32_t nb, hipStream_t st) {
  const int m = std::max(n, bins_out ? nb : 0);
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(lrl::apply_commands_kernel, dim3((m + 255) / 256), dim3(256), 0, st, *S, ncs, ids, n, cmds,
                     bins_in, bins_out, nb);
  return hipGetLastError();
}
int32_t lrl_rows_mean_zero(float* table, int64_t ld, int32_t rows, const int32_t* ids, int32_t n, float* means,
                           int32_t zero, void* stream) {
  if (!table || !means || rows < 0 || n < 0 || (n > 0 && !ids)) return 1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(lrl::rows_mean_zero_kernel, dim3(rows), dim3(256), 0, static_cast<hipStream_t>(stream), table,
                     ld, ids, n, (const int32_t*)nullptr, means, (const float*)nullptr, zero);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int32_t lrl_rows_mean_zero_dev(float* table, int64_t ld, int32_t rows, const int32_t* ids, int32_t nmax,
                               const int32_t* dcount, float* means, const float* prev, int32_t zero, void* stream) {
  if (!table || !means || rows < 0 || nmax < 0 || !dcount || (nmax > 0 && !ids)) return 1;
  if (rows == 0) return 0;
  if (nmax == 0)
    return !prev || hipMemcpyAsync(means, prev, rows * sizeof(float), hipMemcpyDeviceToDevice,
                                   static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : 2;
  hipLaunchKernelGGL(lrl::rows_mean_zero_kernel, dim3(rows), dim3(256), 0, static_cast<hipStream_t>(stream), table,
                     ld, ids, nmax, dcount, means, prev, zero);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
hipError_t lrl_launch_reset(const KParams* K, const KState* S, const int32_t* ids, int32_t n, const int32_t* dn,
                            int32_t root_mode, float xy_lo, float xy_span, float x_off, float y_off, int32_t inject,
                            hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lrl::reset_kernel, dim3((n + 255) / 256), dim3(256), 0, st, K, *S, ids, n, dn, root_mode, xy_lo,
                     xy_span, x_off, y_off, inject);
  return hipGetLastError();
}
hipError_t lrl_launch_terrain_curriculum(const KState* S, const int32_t* ids, int32_t n, const int32_t* dn,
                                         int64_t* levels, const int64_t* types, const int64_t* rnd, const float* torig,
                                         int32_t rows, int32_t cols, float half, float ep_len_s, int32_t max_level,
                                         int64_t step_counter, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lrl::terrain_curriculum_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *S, ids, n, dn, levels,
                     types, rnd, torig, rows, cols, half, ep_len_s, max_level, step_counter);
  return hipGetLastError();
}
hipError_t lrl_launch_set_root(const KState* S, const float* src, const int32_t* ids, int32_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lrl::set_root_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *S, src, ids, n);
  return hipGetLastError();
}
hipError_t lrl_launch_set_dof(const KState* S, const float* pos, const float* vel, const int32_t* ids, int32_t n,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lrl::set_dof_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *S, pos, vel, ids, n);
  return hipGetLastError();
}
hipError_t lrl_launch_rigid_body(const KParams* K, const KState* S, const int32_t* body_leg, const int32_t* body_link,
                                 const float* foot_xyz, hipStream_t st) {
  hipLaunchKernelGGL(lrl::rigid_body_kernel, dim3((S->n + 255) / 256), dim3(256), 0, st, K, *S, body_leg, body_link,
                     foot_xyz);
  return hipGetLastError();
}
hipError_t lrl_launch_extras_snapshot(const KParams* K, const KState* S, const int32_t* body_leg, const int32_t* body_link,
                                      const float* foot_xyz, float* out, hipStream_t st) {
  static_assert(LRL_NUM_LEGS == 4, "one quarter-thread per foot");
  hipLaunchKernelGGL(lrl::extras_snapshot_kernel, dim3((S->n + 63) / 64), dim3(256), 0, st, K, *S, body_leg,
                     body_link, foot_xyz, out);
  return hipGetLastError();
}
hipError_t lrl_launch_garbage(uint32_t mode, uint32_t pat, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)lrl::garbage_lds_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  // one 160 KiB workgroup per CU at a time (8 rounds over 256 CUs); 512-register waves, one per SIMD at a time
  if (mode & 1u) hipLaunchKernelGGL(lrl::garbage_lds_kernel, dim3(2048), dim3(64), 160 * 1024, st, pat);
  if (mode & 2u) hipLaunchKernelGGL(lrl::garbage_vgpr_kernel, dim3(8192), dim3(64), 0, st, pat);
  return hipGetLastError();
}
hipError_t lrl_launch_shift_history(const KState* S, int NO, int H, int append, hipStream_t st) {
  hipLaunchKernelGGL(lrl::shift_history_kernel, dim3(S->n), dim3(128), H * sizeof(float), st, *S, NO, H, append);
  return hipGetLastError();
}
hipError_t lrl_launch_randomize(const KState* S, const float* fr, const float* rr, const float* pr, const float* cr,
                                uint32_t which, hipStream_t st) {
  hipLaunchKernelGGL(lrl::randomize_kernel, dim3((S->stride + 255) / 256), dim3(256), 0, st, *S, fr[0], fr[1], rr[0],
                     rr[1], pr[0], pr[1], cr[0], cr[1], which);
  return hipGetLastError();
}
}
