// lrl_capi.cpp — the extern "C" boundary of liblrl.so (include/lrl.h): sim object lifetime, the
// SoA HBM arena, tensor descriptors (acquire_*_tensor) and the launch entry points.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "lrl_kparams.h"

static thread_local char g_err[512];
static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
extern "C" int lrl_set_error(int code, const char* msg) { return fail(code, "%s", msg); }

#define HIPCHECK(x)                                                                     \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(LRL_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

extern "C" {
hipError_t lrl_launch_env_step(const KParams*, const KState*, int, const float*, uint32_t, int64_t, int, hipStream_t);
hipError_t lrl_launch_observe(const KParams*, const KState*, const int32_t*, int32_t, const int32_t*, uint32_t, int64_t,
                              hipStream_t);
hipError_t lrl_env_kernel_setup(int lds_bytes);
hipError_t lrl_launch_reset(const KParams*, const KState*, const int32_t*, int32_t, const int32_t*, int32_t, float, float,
                            float, float, int32_t, hipStream_t);
hipError_t lrl_launch_env_lists(const KState*, int32_t, int32_t, int32_t*, int32_t*, hipStream_t);
hipError_t lrl_launch_curriculum_dev(const lrl_dev_curriculum*, const KState*, int32_t, const int32_t*, int32_t,
                                     const int32_t*, int32_t, int32_t, int32_t, double, double, double, int32_t,
                                     int32_t, hipStream_t);
hipError_t lrl_launch_set_root(const KState*, const float*, const int32_t*, int32_t, hipStream_t);
hipError_t lrl_launch_step_code(const KState*, int32_t, int32_t, int32_t, float*, int32_t*, hipStream_t);
hipError_t lrl_launch_apply_commands(const KState*, int32_t, const int32_t*, int32_t, const float*, const float*, float*,
                                     int32_t, hipStream_t);
hipError_t lrl_launch_terrain_curriculum(const KState*, const int32_t*, int32_t, const int32_t*, int64_t*, const int64_t*,
                                         const int64_t*, const float*, int32_t, int32_t, float, float, int32_t, int64_t,
                                         hipStream_t);
hipError_t lrl_launch_set_dof(const KState*, const float*, const float*, const int32_t*, int32_t, hipStream_t);
hipError_t lrl_launch_rigid_body(const KParams*, const KState*, const int32_t*, const int32_t*, const float*,
                                 hipStream_t);
hipError_t lrl_launch_extras_snapshot(const KParams*, const KState*, const int32_t*, const int32_t*, const float*, float*,
                                      hipStream_t);
hipError_t lrl_launch_shift_history(const KState*, int, int, int, hipStream_t);
hipError_t lrl_launch_garbage(uint32_t mode, uint32_t pat, hipStream_t st);
hipError_t lrl_launch_randomize(const KState*, const float*, const float*, const float*, const float*, uint32_t,
                                hipStream_t);
}

struct lrl_sim {
  int device = 0;
  KParams hk;
  KParams* dk = nullptr;
  KState S;
  void* arena = nullptr;
  size_t arena_bytes = 0;
  int lds_bytes = 0;
  int64_t step_counter = 0;
  lrl_tensor t[LRL_T_NUM];
  int32_t* d_body_leg = nullptr;
  int32_t* d_body_link = nullptr;
  float* d_foot_xyz = nullptr;
  void* terr = nullptr;  // terrain mesh buffers (lrl_sim_set_terrain)
  float* d_hull = nullptr;  // mesh colliders' support tables (KParams::hull_tab)
  uint32_t* self_stats = nullptr;  // lrl_sim_self_contact_stats counters
  float* d_code = nullptr;         // lrl_sim_step_code scratch [3][n]
  // lrl_sim_timing: HIP events around each env-kernel launch of lrl_sim_step (not the history-shift launch before it)
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t ev_used = 0;
  uint32_t garbage_mode = 0, garbage_pat = 0;  // lrl_debug_sim_garbage
};

static void quat_to_rowmajor(const float* q, float* R) {
  float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}

// Self-collision candidates (the oracle enumerates the same list, oracle/lrl_oracle.c::self_pairs).
// PhysX collides every pair of shapes on different links of an articulation except a link and its parent; with the
// fixed feet merged into the calves, a leg sphere's dynamic link is min(body_link, 2).  Candidates: leg spheres with a
// radius (the base's radius-0 corner spheres span the base box instead), in the canonical order lane La major, then
// g = 0: inside leg La, links two apart (hip - calf); g = 1..3: against leg La + g; g = 4: a leg sphere below the hip
// (whose parent is the base) against the base box.  Inside a group: sphere a, then sphere b, in model order.
static int self_pairs(const lrl_model* m, KParams* k) {
  auto leg_of = [&](int s) { return m->body_leg[m->sphere_body[s]]; };
  auto link_of = [&](int s) { int l = m->body_link[m->sphere_body[s]]; return l > 2 ? 2 : l; };
  auto on_leg = [&](int s, int L) { return leg_of(s) == L && m->sphere_radius[s] > 0.f; };
  float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
  int nbase = 0;
  for (int s = 0; s < m->num_spheres; ++s)
    if (leg_of(s) < 0) {
      ++nbase;
      for (int c = 0; c < 3; ++c) {
        lo[c] = fminf(lo[c], m->sphere_pos[s][c] - m->sphere_radius[s]);
        hi[c] = fmaxf(hi[c], m->sphere_pos[s][c] + m->sphere_radius[s]);
      }
    }
  for (int c = 0; c < 3; ++c) {
    k->box_c[c] = nbase ? 0.5f * (lo[c] + hi[c]) : 0.f;
    k->box_h[c] = nbase ? 0.5f * (hi[c] - lo[c]) : -1.f;  // no base shapes: no box group
  }
  int n = 0;
  auto add = [&](int a, int b) {
    if (n >= LRL_MAX_SELF_PAIRS) return false;
    const int bb = b < 0 ? 0 : m->sphere_body[b];
    k->self_pair[n++] = (uint32_t)a | (uint32_t)(b < 0 ? 255 : b) << 8 | (uint32_t)m->sphere_body[a] << 16 | (uint32_t)bb << 24;
    return true;
  };
  for (int La = 0; La < 4; ++La)
    for (int g = 0; g < 5; ++g) {
      k->self_grp[La][g][0] = n;
      const int Lb = g == 0 ? La : La + g;
      for (int a = 0; a < m->num_spheres; ++a) {
        if (!on_leg(a, La)) continue;
        if (g == 4) {
          if (nbase && link_of(a) >= 1 && !add(a, -1)) return fail(LRL_E_INVALID, "too many self-collision pairs");
          continue;
        }
        if (Lb > 3) continue;
        for (int b = g == 0 ? a + 1 : 0; b < m->num_spheres; ++b) {
          if (!on_leg(b, Lb)) continue;
          if (g == 0 && abs(link_of(a) - link_of(b)) < 2) continue;
          if (!add(a, b)) return fail(LRL_E_INVALID, "too many self-collision pairs");
        }
      }
      k->self_grp[La][g][1] = n;
    }
  k->self_npairs = n;
  k->self_kmax = 0;
  for (int L = 0; L < 4; ++L) {
    int cnt = 0, nh = 0, lead = 1;
    for (int s = 0; s < m->num_spheres; ++s) {
      if (leg_of(s) != L) continue;
      ++cnt;
      if (lead && link_of(s) == 0 && m->sphere_radius[s] > 0.f) ++nh;
      else lead = 0;
    }
    k->self_nhip[L] = nh;
    if (cnt > k->self_kmax) k->self_kmax = cnt;
  }
  if (k->self_kmax > 8) return fail(LRL_E_INVALID, "more than 8 collision spheres on a leg");
  return 0;
}

static int digest(const lrl_model* m, const lrl_env_params* p, KParams* k) {
  memset(k, 0, sizeof(*k));
  k->p = *p;
  if (m->num_bodies < 5 || m->num_bodies > LRL_MAX_BODIES) return fail(LRL_E_INVALID, "num_bodies %d", m->num_bodies);
  if (m->num_spheres < 0 || m->num_spheres > LRL_MAX_SPHERES) return fail(LRL_E_INVALID, "num_spheres %d", m->num_spheres);
  if (p->num_obs <= 0 || p->num_obs > LRL_MAX_OBS) return fail(LRL_E_INVALID, "num_obs %d", p->num_obs);
  if (p->decimation < 1 || p->sim_dt <= 0.f) return fail(LRL_E_INVALID, "bad timing");
  if (p->control_type < 0 || p->control_type > 2) return fail(LRL_E_INVALID, "bad control_type %d", p->control_type);
  if (p->push_robots && p->push_interval < 1) return fail(LRL_E_INVALID, "push_robots with push_interval < 1");
  if (p->num_reward_terms < 0 || p->num_reward_terms > LRL_MAX_REWARD_TERMS) return fail(LRL_E_INVALID, "reward terms");
  for (int t = 0; t < p->num_reward_terms; ++t)
    if (p->reward_term[t] < 0 || p->reward_term[t] >= LRL_R_NUM_TERMS) return fail(LRL_E_INVALID, "reward term id");
  {  // the sum rows: each term (and the termination term) its own row below num_sum_keys (the kernel writes rows
     // reward_slot[t] / termination_slot of episode_sums and command_sums, sized num_sum_keys + 1 / + 5)
    uint64_t used = 0;
    const bool term = p->termination_scale != 0.f;
    if (p->num_sum_keys < 0 || p->num_sum_keys > 64) return fail(LRL_E_INVALID, "num_sum_keys %d", p->num_sum_keys);
    for (int t = 0; t < p->num_reward_terms + (term ? 1 : 0); ++t) {
      const int r = t < p->num_reward_terms ? p->reward_slot[t] : p->termination_slot;
      if (r < 0 || r >= p->num_sum_keys || ((used >> r) & 1ull)) return fail(LRL_E_INVALID, "sum row %d of term %d", r, t);
      used |= 1ull << r;
    }
  }
  if (p->measure_heights && (p->num_height_points <= 0 || p->num_height_points > LRL_MAX_HEIGHT_POINTS))
    return fail(LRL_E_INVALID, "num_height_points %d", p->num_height_points);
  if (p->terrain_mesh && p->horizontal_scale <= 0.f) return fail(LRL_E_INVALID, "horizontal_scale");
  int obs_expected = 3 + (p->observe_command ? 3 : 0) + 36 + (p->observe_vel ? 6 : 0) +
                     (p->measure_heights ? p->num_height_points : 0);
  if (obs_expected != p->num_obs) return fail(LRL_E_INVALID, "obs layout %d != num_obs %d", obs_expected, p->num_obs);
  for (int l = 0; l < 4; ++l)
    for (int j = 0; j < 3; ++j) {
      KLeg& L = k->leg[l];
      for (int c = 0; c < 3; ++c) {
        L.xyz[j][c] = m->joint_xyz[l][j][c];
        L.axis[j][c] = m->joint_axis[l][j][c];
        L.com[j][c] = m->link_com[l][j][c];
      }
      quat_to_rowmajor(m->joint_quat[l][j], L.rfix[j]);
      L.mass[j] = m->link_mass[l][j];
      for (int c = 0; c < 6; ++c) L.inertia[j][c] = m->link_inertia[l][j][c];
    }
  k->base_mass = m->base_mass;
  for (int c = 0; c < 6; ++c) k->base_inertia[c] = m->base_inertia[c];
  if (p->joint_limits && !(p->joint_limit_margin >= 0.f)) return fail(LRL_E_INVALID, "joint_limit_margin");
  for (int j = 0; j < LRL_NUM_DOF; ++j) {
    const bool lim = m->dof_lower[j] < m->dof_upper[j];  // (a URDF joint without <limit> has lower = upper = 0)
    k->dof_lo[j] = lim ? m->dof_lower[j] : -1e30f;
    k->dof_hi[j] = lim ? m->dof_upper[j] : 1e30f;
  }
  k->num_bodies = m->num_bodies;
  k->num_spheres = m->num_spheres;
  // spheres must be grouped: base first, then legs in order, bodies contiguous
  int prev_key = -1;
  for (int b = 0; b < LRL_MAX_BODIES; ++b) { k->body_sph_begin[b] = 0; k->body_sph_end[b] = 0; k->body_foot[b] = -1; }
  for (int l = 0; l < 4; ++l) { k->leg_sph_begin[l] = k->leg_sph_end[l] = 0; }
  k->base_sph_end = 0;
  for (int s = 0; s < m->num_spheres; ++s) {
    int b = m->sphere_body[s];
    if (b < 0 || b >= m->num_bodies) return fail(LRL_E_INVALID, "sphere body");
    int leg = m->body_leg[b], link = m->body_link[b];
    int key = (leg + 1) * 64 + b;
    if (key < prev_key) return fail(LRL_E_INVALID, "spheres not grouped by leg/body");
    if (key != prev_key) k->body_sph_begin[b] = s;
    k->body_sph_end[b] = s + 1;
    prev_key = key;
    for (int c = 0; c < 3; ++c) k->sph_pos[s][c] = m->sphere_pos[s][c];
    k->sph_rad[s] = m->sphere_radius[s];
    k->sph_link[s] = leg < 0 ? -1 : (link > 2 ? 2 : link);
    k->sph_leg[s] = leg;
    if (leg < 0) k->base_sph_end = s + 1;
    // support tables of the mesh colliders (legs only: the base's spheres are detected before the leg frames exist)
    const int h = m->num_hulls > 0 ? m->sphere_hull[s] : -1;
    if (h < -1 || h >= m->num_hulls) return fail(LRL_E_INVALID, "sphere_hull[%d] = %d of %d tables", s, h, m->num_hulls);
    if (h >= 0 && leg < 0) return fail(LRL_E_INVALID, "sphere %d: support tables are for leg links only", s);
    k->sph_hull[s] = h;
  }
  if (m->num_hulls < 0 || m->num_hulls > LRL_MAX_SPHERES) return fail(LRL_E_INVALID, "num_hulls %d", m->num_hulls);
  if (m->num_hulls > 0 && (!m->hull_table || m->hull_res < 1 || m->hull_res > 64 || m->hull_k != LRL_HULL_K))
    return fail(LRL_E_INVALID, "hull tables: table %p, hull_res %d, hull_k %d", (const void*)m->hull_table, m->hull_res,
                m->hull_k);
  k->hull_res = m->num_hulls > 0 ? m->hull_res : 0;
  k->hull_k = m->num_hulls > 0 ? m->hull_k : 0;
  for (int l = 0; l < 4; ++l) {
    int b0 = -1, e0 = -1;
    for (int s = 0; s < m->num_spheres; ++s)
      if (m->body_leg[m->sphere_body[s]] == l) {
        if (b0 < 0) b0 = s;
        e0 = s + 1;
      }
    if (b0 < 0) b0 = e0 = k->base_sph_end;
    k->leg_sph_begin[l] = b0;
    k->leg_sph_end[l] = e0;
  }
  for (int f = 0; f < p->num_feet; ++f) {
    int b = p->feet[f];
    if (b < 0 || b >= m->num_bodies) return fail(LRL_E_INVALID, "foot index");
    k->body_foot[b] = f;
  }
  int rc = self_pairs(m, k);
  if (rc) return rc;
  k->num_history = p->num_history;
  k->n_es = p->num_sum_keys + 1;
  k->n_cs = p->num_sum_keys + 5;
  return 0;
}

static void set_t(lrl_tensor* t, void* data, int dtype, int ndim, const int64_t* shape, const int64_t* strides) {
  t->data = data;
  t->dtype = dtype;
  t->ndim = ndim;
  for (int i = 0; i < 4; ++i) { t->shape[i] = i < ndim ? shape[i] : 1; t->strides[i] = i < ndim ? strides[i] : 0; }
}

extern "C" {

int32_t lrl_abi_version(void) { return LRL_ABI_VERSION; }
const char* lrl_last_error(void) { return g_err; }
int32_t lrl_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int32_t lrl_sim_create(const lrl_model* model, const lrl_env_params* params, int32_t num_envs,
                       int64_t global_env_offset, uint64_t seed, int32_t device, lrl_sim** out) {
  if (!model || !params || !out || num_envs <= 0) return fail(LRL_E_INVALID, "bad arguments");
  int ndev = lrl_device_count();
  if (ndev <= 0) return fail(LRL_E_NOGPU, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(LRL_E_INVALID, "device %d of %d", device, ndev);
  lrl_sim* s = new lrl_sim();
  s->device = device;
  int rc = digest(model, params, &s->hk);
  if (rc) { delete s; return rc; }
  HIPCHECK(hipSetDevice(device));
  const int n = num_envs, N = (n + 63) / 64 * 64;
  const int B = model->num_bodies, NO = params->num_obs, H = params->num_history * NO;
  const int nes = s->hk.n_es, ncs = s->hk.n_cs;
  KState& S = s->S;
  memset(&S, 0, sizeof(S));
  S.n = n;
  S.stride = N;
  S.env_offset = global_env_offset;
  S.seed = seed;
  // arena layout (floats unless noted), every field 256-B aligned
  struct F { void** p; size_t bytes; };
  std::vector<F> fields;
  auto addf = [&](float** p, size_t cnt) { fields.push_back({(void**)p, cnt * 4}); };
  addf(&S.root, 13ull * N); addf(&S.dof_pos, 12ull * N); addf(&S.dof_vel, 12ull * N);
  addf(&S.contact, 3ull * B * N); addf(&S.rb_state, 13ull * B * N); addf(&S.torques, 12ull * N);
  addf(&S.actions, 12ull * N); addf(&S.last_actions, 12ull * N); addf(&S.last_dof_vel, 12ull * N);
  addf(&S.last_root_vel, 6ull * N); addf(&S.commands, 4ull * N); addf(&S.obs, (size_t)N * NO);
  addf(&S.priv, (size_t)N * LRL_NUM_PRIV); addf(&S.hist, (size_t)N * H); addf(&S.rew, N);
  fields.push_back({(void**)&S.reset, (size_t)N}); fields.push_back({(void**)&S.time_out, (size_t)N});
  fields.push_back({(void**)&S.last_contacts, 4ull * N}); fields.push_back({(void**)&S.episode_length, 4ull * N});
  fields.push_back({(void**)&S.reset_count, 4ull * N});
  addf(&S.episode_sums, (size_t)nes * N); addf(&S.command_sums, (size_t)ncs * N); addf(&S.feet_air_time, 4ull * N);
  addf(&S.friction, N); addf(&S.restitution, N); addf(&S.payload, N); addf(&S.com, 3ull * N);
  addf(&S.motor_strength, 12ull * N); addf(&S.kp, 12ull * N); addf(&S.kd, 12ull * N); addf(&S.env_origins, 3ull * N);
  addf(&S.base_lin_vel, 3ull * N); addf(&S.base_ang_vel, 3ull * N); addf(&S.projected_gravity, 3ull * N);
  addf(&S.joint_pos_target, 12ull * N);
  const int NP = params->measure_heights ? params->num_height_points : 0;
  addf(&S.heights, (size_t)(NP > 0 ? NP : 1) * N);
  size_t total = 0;
  for (auto& f : fields) total += (f.bytes + 255) / 256 * 256;
  void* arena = nullptr;
  if (hipMalloc(&arena, total) != hipSuccess) { delete s; return fail(LRL_E_NOMEM, "hipMalloc %zu bytes", total); }
  s->arena = arena;
  s->arena_bytes = total;
  size_t off = 0;
  for (auto& f : fields) { *f.p = (char*)arena + off; off += (f.bytes + 255) / 256 * 256; }
  HIPCHECK(hipMemset(arena, 0, total));
  // initial values: identity quaternion, unit DR factors, default friction 1
  std::vector<float> ones(N, 1.f);
  HIPCHECK(hipMemcpy(S.root + 6ull * N, ones.data(), N * 4, hipMemcpyHostToDevice));
  for (int j = 0; j < 12; ++j) {
    HIPCHECK(hipMemcpy(S.motor_strength + (size_t)j * N, ones.data(), N * 4, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(S.kp + (size_t)j * N, ones.data(), N * 4, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(S.kd + (size_t)j * N, ones.data(), N * 4, hipMemcpyHostToDevice));
  }
  HIPCHECK(hipMemcpy(S.friction, ones.data(), N * 4, hipMemcpyHostToDevice));
  if (model->num_hulls > 0) {  // the mesh colliders' support tables, read by the plane env kernel's detection
    const size_t hb = (size_t)model->num_hulls * 6 * model->hull_res * model->hull_res * model->hull_k * 16;
    HIPCHECK(hipMalloc(&s->d_hull, hb));
    HIPCHECK(hipMemcpy(s->d_hull, model->hull_table, hb, hipMemcpyHostToDevice));
    s->hk.hull_tab = s->d_hull;
  }
  HIPCHECK(hipMalloc(&s->dk, sizeof(KParams)));
  HIPCHECK(hipMemcpy(s->dk, &s->hk, sizeof(KParams), hipMemcpyHostToDevice));
  HIPCHECK(hipMalloc(&s->d_body_leg, sizeof(int32_t) * LRL_MAX_BODIES));
  HIPCHECK(hipMalloc(&s->d_body_link, sizeof(int32_t) * LRL_MAX_BODIES));
  HIPCHECK(hipMalloc(&s->d_foot_xyz, sizeof(float) * 12));
  HIPCHECK(hipMemcpy(s->d_body_leg, model->body_leg, sizeof(int32_t) * LRL_MAX_BODIES, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(s->d_body_link, model->body_link, sizeof(int32_t) * LRL_MAX_BODIES, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(s->d_foot_xyz, model->foot_xyz, sizeof(float) * 12, hipMemcpyHostToDevice));
  // env step kernel LDS: wg_envs envs per workgroup: leg blocks + contact rows, or the obs tiles
  const int wg_envs = params->terrain_mesh ? LRL_ENV_WG_ENVS_MESH : LRL_ENV_WG_ENVS_FLAT;
  const int legf = params->terrain_mesh ? LRL_LEGF_MESH : LRL_LEGF_FLAT, nsf = params->terrain_mesh ? LRL_NSF_MESH : LRL_NSF_FLAT;
  int lds_contacts = (4 * legf + model->num_spheres * nsf) * wg_envs * 4;  // LEGF, NSF of lrl_env.hip
  // terrain query vertex block, float4 [16][lanes]; the joint-limit rows (12 x 19 fields per env) alias it after the
  // queries, and have their own region on the plane
  lds_contacts += params->terrain_mesh ? 16 * LRL_ENV_LANES * 16 : LRL_NUM_DOF * 19 * wg_envs * 4;
  lds_contacts += (4 * (int)(sizeof(KLeg) / 4) + 5 * model->num_spheres) * 4;  // staged model tables (Lds::ktab)
  lds_contacts += (40 + s->hk.self_npairs + 1) * 4;  // + the self-collision groups and pairs
  if (params->terrain_mesh) lds_contacts += LRL_ENV_LANES * 20;  // + the terrain query work list (Lds::wl)
  int lds_tiles = (NO + LRL_NUM_PRIV + LRL_MAX_REWARD_TERMS) * wg_envs * 4;  // obs / priv tiles + reward rows
  s->lds_bytes = lds_contacts > lds_tiles ? lds_contacts : lds_tiles;
  if (s->lds_bytes > 160 * 1024) return fail(LRL_E_INVALID, "LDS budget exceeded (%d B)", s->lds_bytes);
  HIPCHECK(lrl_env_kernel_setup(s->lds_bytes));
  // tensor descriptors: [n, k] views over SoA [k][N] -> strides (1, N)
  const int64_t sN = N;
  auto soa2 = [&](int id, void* d, int k, int dt) {
    int64_t sh[2] = {n, k}, st[2] = {1, sN};
    set_t(&s->t[id], d, dt, 2, sh, st);
  };
  auto soa1 = [&](int id, void* d, int dt) {
    int64_t sh[1] = {n}, st[1] = {1};
    set_t(&s->t[id], d, dt, 1, sh, st);
  };
  soa2(LRL_T_ROOT_STATE, S.root, 13, LRL_F32);
  soa2(LRL_T_DOF_POS, S.dof_pos, 12, LRL_F32);
  soa2(LRL_T_DOF_VEL, S.dof_vel, 12, LRL_F32);
  { int64_t sh[3] = {n, B, 3}, st[3] = {1, 3 * sN, sN}; set_t(&s->t[LRL_T_CONTACT_FORCE], S.contact, LRL_F32, 3, sh, st); }
  { int64_t sh[3] = {n, B, 13}, st[3] = {1, 13 * sN, sN}; set_t(&s->t[LRL_T_RIGID_BODY_STATE], S.rb_state, LRL_F32, 3, sh, st); }
  soa2(LRL_T_TORQUES, S.torques, 12, LRL_F32);
  soa2(LRL_T_ACTIONS, S.actions, 12, LRL_F32);
  soa2(LRL_T_LAST_ACTIONS, S.last_actions, 12, LRL_F32);
  soa2(LRL_T_LAST_DOF_VEL, S.last_dof_vel, 12, LRL_F32);
  soa2(LRL_T_LAST_ROOT_VEL, S.last_root_vel, 6, LRL_F32);
  soa2(LRL_T_COMMANDS, S.commands, 4, LRL_F32);
  { int64_t sh[2] = {n, NO}, st[2] = {NO, 1}; set_t(&s->t[LRL_T_OBS], S.obs, LRL_F32, 2, sh, st); }
  { int64_t sh[2] = {n, LRL_NUM_PRIV}, st[2] = {LRL_NUM_PRIV, 1}; set_t(&s->t[LRL_T_PRIV_OBS], S.priv, LRL_F32, 2, sh, st); }
  { int64_t sh[2] = {n, H}, st[2] = {H, 1}; set_t(&s->t[LRL_T_OBS_HISTORY], S.hist, LRL_F32, 2, sh, st); }
  soa1(LRL_T_REWARD, S.rew, LRL_F32);
  soa1(LRL_T_RESET, S.reset, LRL_U8);
  soa1(LRL_T_TIME_OUT, S.time_out, LRL_U8);
  soa1(LRL_T_EPISODE_LENGTH, S.episode_length, LRL_I32);
  { int64_t sh[2] = {nes, n}, st[2] = {sN, 1}; set_t(&s->t[LRL_T_EPISODE_SUMS], S.episode_sums, LRL_F32, 2, sh, st); }
  { int64_t sh[2] = {ncs, n}, st[2] = {sN, 1}; set_t(&s->t[LRL_T_COMMAND_SUMS], S.command_sums, LRL_F32, 2, sh, st); }
  soa2(LRL_T_FEET_AIR_TIME, S.feet_air_time, 4, LRL_F32);
  soa2(LRL_T_LAST_CONTACTS, S.last_contacts, 4, LRL_U8);
  soa1(LRL_T_FRICTION, S.friction, LRL_F32);
  soa1(LRL_T_RESTITUTION, S.restitution, LRL_F32);
  soa1(LRL_T_PAYLOAD, S.payload, LRL_F32);
  soa2(LRL_T_COM_DISPLACEMENT, S.com, 3, LRL_F32);
  soa2(LRL_T_MOTOR_STRENGTH, S.motor_strength, 12, LRL_F32);
  soa2(LRL_T_KP_FACTOR, S.kp, 12, LRL_F32);
  soa2(LRL_T_KD_FACTOR, S.kd, 12, LRL_F32);
  soa2(LRL_T_ENV_ORIGINS, S.env_origins, 3, LRL_F32);
  soa2(LRL_T_BASE_LIN_VEL, S.base_lin_vel, 3, LRL_F32);
  soa2(LRL_T_BASE_ANG_VEL, S.base_ang_vel, 3, LRL_F32);
  soa2(LRL_T_PROJECTED_GRAVITY, S.projected_gravity, 3, LRL_F32);
  soa2(LRL_T_JOINT_POS_TARGET, S.joint_pos_target, 12, LRL_F32);
  soa2(LRL_T_MEASURED_HEIGHTS, S.heights, NP, LRL_F32);
  *out = s;
  return 0;
}

int32_t lrl_sim_set_terrain(lrl_sim* s, const float* vertices, const int16_t* height_samples, int32_t rows,
                            int32_t cols) {
  if (!s || !vertices || !height_samples || rows < 2 || cols < 2) return fail(LRL_E_INVALID, "bad terrain arguments");
  if (!s->hk.p.terrain_mesh) return fail(LRL_E_INVALID, "params.terrain_mesh is 0 (plane ground)");
  const size_t nv = (size_t)rows * cols;
  const float bs = s->hk.p.border_size, vs = s->hk.p.vertical_scale;
  // vertex grid in the world frame (tm_params.transform.p = (-border, -border, 0), legged_robot.py:1152-1154)
  std::vector<float> vtx(4 * nv), h(nv), hmax(nv, 0.f), rowmax(nv);
  for (size_t v = 0; v < nv; ++v) {
    vtx[4 * v] = vertices[3 * v] - bs;
    vtx[4 * v + 1] = vertices[3 * v + 1] - bs;
    vtx[4 * v + 2] = vertices[3 * v + 2];
    vtx[4 * v + 3] = 0.f;
    h[v] = (float)height_samples[v] * vs;  // torch: int16 tensor * python float -> float32
  }
  // reach of the model: largest distance of a sphere surface from the base origin (chain of joint offsets)
  const KParams& k = s->hk;
  float reach = 0.f;
  for (int q = 0; q < k.num_spheres; ++q) {
    float d = sqrtf(k.sph_pos[q][0] * k.sph_pos[q][0] + k.sph_pos[q][1] * k.sph_pos[q][1] +
                    k.sph_pos[q][2] * k.sph_pos[q][2]) + k.sph_rad[q];
    const int l = k.sph_leg[q];
    if (l >= 0)
      for (int j = 0; j < 3; ++j)
        d += sqrtf(k.leg[l].xyz[j][0] * k.leg[l].xyz[j][0] + k.leg[l].xyz[j][1] * k.leg[l].xyz[j][1] +
                   k.leg[l].xyz[j][2] * k.leg[l].xyz[j][2]);
    reach = fmaxf(reach, d);
  }
  const int W = (int)ceilf(reach / s->hk.p.horizontal_scale) + 2;
  // a query at cell (i, j) reads vertices [i-1, i+2] x [j-1, j+2]: separable max filter of the vertex z
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) {
      float m = -3.0e38f;
      for (int jj = j - 1; jj <= j + 2; ++jj)
        if (jj >= 0 && jj < cols) m = fmaxf(m, vtx[4 * ((size_t)i * cols + jj) + 2]);
      rowmax[(size_t)i * cols + j] = m;
    }
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) {
      float m = -3.0e38f;
      for (int ii = i - 1; ii <= i + 2; ++ii)
        if (ii >= 0 && ii < rows) m = fmaxf(m, rowmax[(size_t)ii * cols + j]);
      hmax[(size_t)i * cols + j] = m;
    }
  // window max around a base cell: [i-W, i+W] x [j-W, j+W] (terrain_window_max), two sliding passes
  std::vector<float> wmax(nv);
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) {
      float m = -3.0e38f;
      for (int jj = (j - W > 0 ? j - W : 0); jj <= (j + W < cols - 1 ? j + W : cols - 1); ++jj)
        m = fmaxf(m, vtx[4 * ((size_t)i * cols + jj) + 2]);
      rowmax[(size_t)i * cols + j] = m;
    }
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) {
      float m = -3.0e38f;
      for (int ii = (i - W > 0 ? i - W : 0); ii <= (i + W < rows - 1 ? i + W : rows - 1); ++ii)
        m = fmaxf(m, rowmax[(size_t)ii * cols + j]);
      wmax[(size_t)i * cols + j] = m;
    }
  HIPCHECK(hipSetDevice(s->device));
  (void)hipFree(s->terr);
  s->terr = nullptr;
  const size_t bytes = nv * 4 * sizeof(float) + 3 * nv * sizeof(float);
  if (hipMalloc(&s->terr, bytes) != hipSuccess) return fail(LRL_E_NOMEM, "hipMalloc %zu bytes (terrain)", bytes);
  float* dv = (float*)s->terr;
  float* dmax = dv + 4 * nv;
  float* dh = dmax + nv;
  float* dw = dh + nv;
  HIPCHECK(hipMemcpy(dv, vtx.data(), nv * 16, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(dmax, hmax.data(), nv * 4, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(dh, h.data(), nv * 4, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(dw, wmax.data(), nv * 4, hipMemcpyHostToDevice));
  s->hk.terr_wmax = dw;
  s->hk.terr_vtx = dv;
  s->hk.terr_hmax = dmax;
  s->hk.terr_h = dh;
  s->hk.terr_rows = rows;
  s->hk.terr_cols = cols;
  s->hk.terr_inv_hs = 1.f / s->hk.p.horizontal_scale;
  HIPCHECK(hipMemcpy(s->dk, &s->hk, sizeof(KParams), hipMemcpyHostToDevice));
  return 0;
}

int32_t lrl_sim_destroy(lrl_sim* s) {
  if (!s) return 0;
  (void)hipSetDevice(s->device);
  (void)hipFree(s->arena);
  (void)hipFree(s->dk);
  (void)hipFree(s->d_body_leg);
  (void)hipFree(s->d_body_link);
  (void)hipFree(s->d_foot_xyz);
  (void)hipFree(s->terr);
  (void)hipFree(s->d_hull);
  (void)hipFree(s->self_stats);
  (void)hipFree(s->d_code);
  for (auto& pr : s->ev) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  delete s;
  return 0;
}

int32_t lrl_sim_tensor(lrl_sim* s, int32_t id, lrl_tensor* out) {
  if (!s || !out || id < 0 || id >= LRL_T_NUM) return fail(LRL_E_INVALID, "bad tensor id %d", id);
  *out = s->t[id];
  return 0;
}

int32_t lrl_sim_inject_uniforms(lrl_sim* s, const float* noise_u, const float* dr_u) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  s->S.inj_noise = noise_u;
  s->S.inj_dr = dr_u;
  return 0;
}

int32_t lrl_sim_inject_push_uniforms(lrl_sim* s, const float* u) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  s->S.inj_push = u;
  return 0;
}

int32_t lrl_sim_step(lrl_sim* s, const float* actions, uint32_t flags, void* stream) {
  if (!s || !actions) return fail(LRL_E_INVALID, "null argument");
  if ((flags & LRL_STEP_INJECT_UNIFORM) && (!s->S.inj_noise || !s->S.inj_dr))
    return fail(LRL_E_INVALID, "injected uniforms not set");
  if ((flags & LRL_STEP_INJECT_UNIFORM) && s->hk.p.push_robots && !s->S.inj_push)
    return fail(LRL_E_INVALID, "push_robots on but injected push uniforms not set");
  if (s->hk.p.terrain_mesh && !s->hk.terr_vtx) return fail(LRL_E_INVALID, "terrain_mesh set but no lrl_sim_set_terrain");
  s->step_counter += 1;  // common_step_counter (legged_robot.py:153)
  if (flags & LRL_STEP_HISTORY)  // HistoryWrapper.step's shift; the env kernel appends the step's obs row
    HIPCHECK(lrl_launch_shift_history(&s->S, s->hk.p.num_obs, s->hk.p.num_history * s->hk.p.num_obs, 0,
                                      (hipStream_t)stream));
  if (s->garbage_mode) HIPCHECK(lrl_launch_garbage(s->garbage_mode, s->garbage_pat, (hipStream_t)stream));
  std::pair<hipEvent_t, hipEvent_t>* tp = nullptr;
  if (s->timing) {
    if (s->ev_used == s->ev.size()) {
      hipEvent_t a = nullptr, b = nullptr;
      HIPCHECK(hipEventCreate(&a));
      HIPCHECK(hipEventCreate(&b));
      s->ev.emplace_back(a, b);
    }
    tp = &s->ev[s->ev_used++];
    HIPCHECK(hipEventRecord(tp->first, (hipStream_t)stream));
  }
  HIPCHECK(lrl_launch_env_step(s->dk, &s->S, s->lds_bytes, actions, flags, s->step_counter, s->hk.p.terrain_mesh,
                               (hipStream_t)stream));
  if (tp) HIPCHECK(hipEventRecord(tp->second, (hipStream_t)stream));
  return 0;
}

int32_t lrl_debug_sim_garbage(lrl_sim* s, uint32_t mode, uint32_t pattern) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  if (mode > 3u) return fail(LRL_E_INVALID, "garbage mode %u", mode);
  s->garbage_mode = mode;
  s->garbage_pat = pattern;
  return 0;
}

int32_t lrl_debug_sim_arena(lrl_sim* s, void** arena, int64_t* bytes, int64_t* step_counter) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  if (arena) *arena = s->arena;
  if (bytes) *bytes = (int64_t)s->arena_bytes;
  if (step_counter) *step_counter = s->step_counter;
  return 0;
}

int32_t lrl_sim_timing(lrl_sim* s, int32_t enable, double* total_ms, int64_t* launches) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  if (total_ms) {
    double t = 0.0;
    for (size_t i = 0; i < s->ev_used; ++i) {
      float ms = 0.f;
      HIPCHECK(hipEventSynchronize(s->ev[i].second));
      HIPCHECK(hipEventElapsedTime(&ms, s->ev[i].first, s->ev[i].second));
      t += ms;
    }
    *total_ms = t;
  }
  if (launches) *launches = (int64_t)s->ev_used;
  s->ev_used = 0;
  s->timing = enable != 0;
  return 0;
}

int32_t lrl_sim_self_contact_stats(lrl_sim* s, int32_t enable, uint64_t* out) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  HIPCHECK(hipSetDevice(s->device));
  HIPCHECK(hipDeviceSynchronize());  // no env kernel in flight reads the parameter block below
  if (out) {
    uint32_t c[4] = {0, 0, 0, 0};
    if (s->self_stats) HIPCHECK(hipMemcpy(c, s->self_stats, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out[i] = c[i];
  }
  if (enable) {
    if (!s->self_stats && hipMalloc(&s->self_stats, 4 * sizeof(uint32_t)) != hipSuccess)
      return fail(LRL_E_NOMEM, "hipMalloc (self-contact counters)");
    HIPCHECK(hipMemset(s->self_stats, 0, 4 * sizeof(uint32_t)));
  }
  s->hk.self_stats = enable ? s->self_stats : nullptr;
  HIPCHECK(hipMemcpy(s->dk, &s->hk, sizeof(KParams), hipMemcpyHostToDevice));
  return 0;
}

int32_t lrl_sim_set_step_counter(lrl_sim* s, int64_t c) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  s->step_counter = c;
  return 0;
}

int32_t lrl_sim_reset_idx(lrl_sim* s, const int32_t* ids, int32_t n, void* stream) {
  return lrl_sim_reset_idx_ex(s, ids, n, 1, 0.f, 0.f, 0.f, 0.f, 0u, stream);
}

int32_t lrl_sim_inject_reset_uniforms(lrl_sim* s, const float* u) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  s->S.inj_reset = u;
  return 0;
}

int32_t lrl_sim_reset_idx_ex(lrl_sim* s, const int32_t* ids, int32_t n, int32_t root_mode, float xy_lo, float xy_span,
                             float x_off, float y_off, uint32_t flags, void* stream) {
  if (!s || (n > 0 && !ids)) return fail(LRL_E_INVALID, "null argument");
  if (n < 0) return fail(LRL_E_INVALID, "negative env count");
  if (root_mode < 0 || root_mode > 2) return fail(LRL_E_INVALID, "root_mode %d", root_mode);
  const bool inject = (flags & LRL_STEP_INJECT_UNIFORM) != 0;
  if (inject && n > 0 && !s->S.inj_reset) return fail(LRL_E_INVALID, "injected reset uniforms not set");
  HIPCHECK(lrl_launch_reset(s->dk, &s->S, ids, n, nullptr, root_mode, xy_lo, xy_span, x_off, y_off, inject ? 1 : 0,
                            (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_reset_idx_dev(lrl_sim* s, const int32_t* ids, int32_t nmax, const int32_t* dcount, int32_t root_mode,
                              float xy_lo, float xy_span, float x_off, float y_off, void* stream) {
  if (!s || !dcount || nmax < 0 || (nmax > 0 && !ids)) return fail(LRL_E_INVALID, "null argument");
  if (root_mode < 0 || root_mode > 2) return fail(LRL_E_INVALID, "root_mode %d", root_mode);
  HIPCHECK(lrl_launch_reset(s->dk, &s->S, ids, nmax, dcount, root_mode, xy_lo, xy_span, x_off, y_off, 0,
                            (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_curriculum_resample_dev(lrl_sim* s, const lrl_dev_curriculum* c, const int32_t* ids, int32_t nmax,
                                        const int32_t* dcount, int32_t ep_len, int32_t row_lin, int32_t row_ang,
                                        double lin_thr, double ang_thr, double local_range, int32_t update,
                                        int32_t log_area, void* stream) {
  if (!s || !c || !dcount || nmax < 0 || (nmax > 0 && !ids) || ep_len <= 0 || nmax > s->S.n)
    return fail(LRL_E_INVALID, "lrl_sim_curriculum_resample_dev: bad argument");
  if (!c->weights || !c->cdf || !c->state || !c->mt_key || !c->ep_rew_lin || !c->ep_rew_ang || !c->env_bins ||
      !c->env_bins_f || !c->command_area || !c->axes || !c->words || !c->draws || c->nx <= 0 || c->ny <= 0 || c->nz <= 0)
    return fail(LRL_E_INVALID, "lrl_sim_curriculum_resample_dev: incomplete curriculum");
  if (row_lin < 0 || row_ang < 0 || row_lin >= s->hk.n_cs || row_ang >= s->hk.n_cs)
    return fail(LRL_E_INVALID, "lrl_sim_curriculum_resample_dev: command-sum rows out of range");
  if (nmax == 0) return 0;
  HIPCHECK(lrl_launch_curriculum_dev(c, &s->S, s->hk.n_cs, ids, nmax, dcount, ep_len, row_lin, row_ang, lin_thr, ang_thr,
                                     local_range, update, log_area, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_env_lists(lrl_sim* s, int32_t mode, int32_t interval, int32_t* ids_out, int32_t* count_out,
                          void* stream) {
  if (!s || !ids_out || !count_out || (mode != 0 && mode != 1) || interval < 1) return fail(LRL_E_INVALID, "bad argument");
  HIPCHECK(lrl_launch_env_lists(&s->S, mode, interval, ids_out, count_out, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_terrain_curriculum(lrl_sim* s, const int32_t* ids, int32_t n, int64_t* levels, const int64_t* types,
                                   const int64_t* rand_levels, const float* terrain_origins, int32_t rows,
                                   int32_t cols, float half_env_length, float episode_length_s, int32_t max_level,
                                   void* stream) {
  if (!s || (n > 0 && (!ids || !levels || !types || !terrain_origins)))  // (rand_levels null: counter-RNG draws)
    return fail(LRL_E_INVALID, "null argument");
  if (n < 0 || rows <= 0 || cols <= 0) return fail(LRL_E_INVALID, "bad sizes");
  HIPCHECK(lrl_launch_terrain_curriculum(&s->S, ids, n, nullptr, levels, types, rand_levels, terrain_origins, rows, cols,
                                         half_env_length, episode_length_s, max_level, s->step_counter,
                                         (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_terrain_curriculum_dev(lrl_sim* s, const int32_t* ids, int32_t nmax, const int32_t* dcount,
                                       int64_t* levels, const int64_t* types, const float* terrain_origins,
                                       int32_t rows, int32_t cols, float half_env_length, float episode_length_s,
                                       int32_t max_level, void* stream) {
  if (!s || !dcount || nmax < 0 || (nmax > 0 && (!ids || !levels || !types || !terrain_origins)))
    return fail(LRL_E_INVALID, "null argument");
  if (rows <= 0 || cols <= 0) return fail(LRL_E_INVALID, "bad sizes");
  HIPCHECK(lrl_launch_terrain_curriculum(&s->S, ids, nmax, dcount, levels, types, nullptr, terrain_origins, rows, cols,
                                         half_env_length, episode_length_s, max_level, s->step_counter,
                                         (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_step_code(lrl_sim* s, int32_t interval, int32_t row0, int32_t row1, float* host_out,
                          int32_t* reset_ids_out, void* stream) {
  if (!s || !host_out || interval < 1) return fail(LRL_E_INVALID, "bad argument");
  if ((row0 >= 0) != (row1 >= 0) || row0 >= s->hk.n_cs || row1 >= s->hk.n_cs)
    return fail(LRL_E_INVALID, "command-sum rows out of range");
  const int n = s->S.n;
  if (!s->d_code) HIPCHECK(hipMalloc(&s->d_code, 3ull * n * sizeof(float)));
  hipStream_t st = (hipStream_t)stream;
  HIPCHECK(lrl_launch_step_code(&s->S, interval, row0, row1, s->d_code, reset_ids_out, st));
  HIPCHECK(hipMemcpyAsync(host_out, s->d_code, (row0 >= 0 ? 3ull : 1ull) * n * sizeof(float), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  return 0;
}

int32_t lrl_sim_apply_commands(lrl_sim* s, const int32_t* ids, int32_t n, const float* cmds, const float* bins_in,
                               float* bins_out, int32_t nbins, void* stream) {
  if (!s || n < 0 || (n > 0 && (!ids || !cmds)) || (bins_out && (!bins_in || nbins < 0 || nbins > s->S.n)))
    return fail(LRL_E_INVALID, "bad argument");
  HIPCHECK(lrl_launch_apply_commands(&s->S, s->hk.n_cs, ids, n, cmds, bins_in, bins_out, nbins, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_observe_idx(lrl_sim* s, const int32_t* ids, int32_t n, uint32_t flags, void* stream) {
  if (!s || (n > 0 && !ids)) return fail(LRL_E_INVALID, "null argument");
  HIPCHECK(lrl_launch_observe(s->dk, &s->S, ids, n, nullptr, flags, s->step_counter, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_observe_idx_dev(lrl_sim* s, const int32_t* ids, int32_t nmax, const int32_t* dcount, uint32_t flags,
                                void* stream) {
  if (!s || !dcount || nmax < 0 || (nmax > 0 && !ids)) return fail(LRL_E_INVALID, "null argument");
  HIPCHECK(lrl_launch_observe(s->dk, &s->S, ids, nmax, dcount, flags, s->step_counter, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_set_root_state_indexed(lrl_sim* s, const float* root, const int32_t* ids, int32_t n, void* stream) {
  if (!s || !root || (n > 0 && !ids)) return fail(LRL_E_INVALID, "null argument");
  HIPCHECK(lrl_launch_set_root(&s->S, root, ids, n, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_set_dof_state_indexed(lrl_sim* s, const float* pos, const float* vel, const int32_t* ids, int32_t n,
                                      void* stream) {
  if (!s || !pos || !vel || (n > 0 && !ids)) return fail(LRL_E_INVALID, "null argument");
  HIPCHECK(lrl_launch_set_dof(&s->S, pos, vel, ids, n, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_extras_snapshot(lrl_sim* s, float* out, void* stream) {
  if (!s || !out) return fail(LRL_E_INVALID, "lrl_sim_extras_snapshot: null argument");
  HIPCHECK(lrl_launch_extras_snapshot(s->dk, &s->S, s->d_body_leg, s->d_body_link, s->d_foot_xyz, out,
                                      (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_refresh_rigid_body_state(lrl_sim* s, void* stream) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  HIPCHECK(lrl_launch_rigid_body(s->dk, &s->S, s->d_body_leg, s->d_body_link, s->d_foot_xyz, (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_shift_history(lrl_sim* s, void* stream) {
  if (!s) return fail(LRL_E_INVALID, "null sim");
  HIPCHECK(lrl_launch_shift_history(&s->S, s->hk.p.num_obs, s->hk.p.num_history * s->hk.p.num_obs, 1,
                                    (hipStream_t)stream));
  return 0;
}

int32_t lrl_sim_randomize(lrl_sim* s, const float* fr, const float* rr, const float* pr, const float* cr,
                          uint32_t which, void* stream) {
  if (!s || !fr || !rr || !pr || !cr) return fail(LRL_E_INVALID, "null argument");
  HIPCHECK(lrl_launch_randomize(&s->S, fr, rr, pr, cr, which, (hipStream_t)stream));
  return 0;
}

}  // extern "C"
