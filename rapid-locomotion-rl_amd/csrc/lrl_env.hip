// lrl_env.hip — fused LeggedRobot.step for gfx950 (CDNA4).
//
// A quad of lanes per env (layout below: 16 envs per single-wave workgroup on the terrain mesh, 4 envs with four
// mirrored quads each on the plane, lrl_env_flat.hip).  A launch performs the whole policy step
// (legged_robot.py:106-137): action clip, `decimation` x {PD torques (:653-688) + one physics
// sub-step}, post_physics_step (:139-188) with teleport (:768-791), DR redraw (:544-560, :591-593),
// termination (:190-202), rewards (:314-340, :1506-1646), observations + noise (:342-417), the
// obs/priv clip (:133-136) and the HistoryWrapper shift (history_wrapper.py:23).
//
// State lives in HBM as struct-of-arrays [field][N] (coalesced: lane i touches word i of each
// field).  Physics (own model; PhysX is closed and unavailable — DESIGN.md §physics):
//   * joint-space dynamics of the 18-DOF floating quadruped in the BASE frame: per-leg composite
//     inertias and 3x3 leg blocks D_l, K_l = D_l^-1 B_l^T, the 6x6 base Schur complement
//     S = A - sum B_l K_l (Cholesky in registers), RNEA bias with gravity as base acceleration;
//   * contacts of collision spheres with the ground plane: speculative/Baumgarte velocity targets,
//     restitution above the bounce threshold, Coulomb cone, projected Gauss-Seidel on 3x3 Delassus
//     blocks computed through the Schur complement;  per-sphere solver rows are staged in LDS as
//     [sphere][field][lane] tiles (bank-conflict free, each lane owns one column);
//   * semi-implicit Euler, quaternion exponential map for the base.
// Post-physics arithmetic runs with FP contraction OFF so it follows torch's op order (the
// reference's elementwise kernels do not fuse multiply-adds).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/lrl_philox.h"
#include "lrl_kparams.h"

#define BLOCK LRL_ENV_LANES  // lanes per workgroup (one wave; see lrl_kparams.h)
// Quad layout: 4 lanes per env (lane & 3 = the leg it owns), 16 envs per single-wave workgroup (the mesh build).  The leg
// work (kinematics, composite inertias, leg blocks, RNEA, contact detection and Delassus rows of the leg's
// spheres, warm-start impulses) runs leg-parallel; the base quantities are summed over the 4 lanes with
// cross-lane shuffles; the Gauss-Seidel sweep and the integration run redundantly in the 4 lanes (so
// every lane holds the full env state); post-physics runs in lane 0 of each env.
#define QL 4
// Plane build (lrl_env_flat.hip includes this file with LRL_ENV_FLAT_TU): 4 envs per wave, 16 lanes per env = 4
// mirrored quads.  Every quad of an env runs the quad code above on the same data (identical values, identical
// stores), and the per-sphere work — ground detection and Delassus row setup — is split over the 4 quads (a lane
// takes every 4th of the spheres its leg owns), so those loops run a quarter of the spheres per lane; the wave's
// loops over max-over-envs contact counts run over 4 envs instead of 16; 1,024 single-wave workgroups fill every
// SIMD of the chip (the 16-env form leaves 3 of each CU's 4 SIMDs idle).  The terrain-mesh build keeps 16 envs per
// wave: its rows do not fit 4 workgroups' LDS per CU.
#ifdef LRL_ENV_FLAT_TU
#define ENVS LRL_ENV_WG_ENVS_FLAT
#define LRL_ENV_NS flat
#else
#define ENVS (BLOCK / QL)
#define LRL_ENV_NS mesh
#endif
#define MIRROR (BLOCK / (QL * ENVS))  // quads per env
static_assert(MIRROR == 1 || MIRROR == 4, "an env has one quad or four mirrored quads");
#define NSF (MIRROR > 1 ? LRL_NSF_FLAT : LRL_NSF_MESH)  // LDS fields per contact sphere (map above contact_setup)
#define LIMF 19  // LDS fields per joint-limit row (map above limit_setup)

namespace lrl {
inline namespace LRL_ENV_NS {

// XCD-aware env blocks: the hardware deals workgroup ids round-robin over the 8 XCDs, so block b is renumbered to
// the env block it covers with consecutive env blocks on one XCD.  A wave's SoA field access is 16 envs x 4 B = half
// a 128-B line; with the plain mapping the two halves of each line were read (and written) through two different
// XCD L2s, each fetching the whole line.
__device__ __forceinline__ int env_block() {
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Phase timers (build with -DLRL_ENV_PROFILE; read with lrl_debug_env_profile): per-wave shader-clock
// cycles of the step kernel's phases, summed over waves.
#ifdef LRL_ENV_PROFILE
__device__ unsigned long long g_env_prof[24];
#define LRL_PROF_DECL unsigned long long prof_t = clock64();
#define LRL_PROF(i)                                   \
  {                                                   \
    const unsigned long long t_ = clock64();          \
    prof[i] += t_ - prof_t;                           \
    prof_t = t_;                                      \
  }
#else
#define LRL_PROF_DECL
#define LRL_PROF(i)
#endif
// Terrain-contact debug records (build with -DLRL_ENV_DEBUG; buffer set with lrl_debug_env_buffer): per env and
// sphere 8 floats — candidate flag, separation found, world centre (x, y, z), window max, radius, 1 — of the last
// sub-step of the launch (scripts/terrain_debug.py runs one sub-step per launch).
#ifdef LRL_ENV_DEBUG
__device__ float* g_env_dbg;
#endif

struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
struct M3 {
  float m[9];
};
__device__ __forceinline__ V3 mul(const M3& R, V3 v) {
  return v3(R.m[0] * v.x + R.m[1] * v.y + R.m[2] * v.z, R.m[3] * v.x + R.m[4] * v.y + R.m[5] * v.z,
            R.m[6] * v.x + R.m[7] * v.y + R.m[8] * v.z);
}
__device__ __forceinline__ V3 mulT(const M3& R, V3 v) {
  return v3(R.m[0] * v.x + R.m[3] * v.y + R.m[6] * v.z, R.m[1] * v.x + R.m[4] * v.y + R.m[7] * v.z,
            R.m[2] * v.x + R.m[5] * v.y + R.m[8] * v.z);
}
__device__ __forceinline__ M3 mul(const M3& A, const M3& B) {
  M3 C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
  return C;
}
__device__ __forceinline__ M3 quat_mat(float x, float y, float z, float w) {
  M3 R;
  R.m[0] = 1.f - 2.f * (y * y + z * z); R.m[1] = 2.f * (x * y - z * w); R.m[2] = 2.f * (x * z + y * w);
  R.m[3] = 2.f * (x * y + z * w); R.m[4] = 1.f - 2.f * (x * x + z * z); R.m[5] = 2.f * (y * z - x * w);
  R.m[6] = 2.f * (x * z - y * w); R.m[7] = 2.f * (y * z + x * w); R.m[8] = 1.f - 2.f * (x * x + y * y);
  return R;
}
__device__ __forceinline__ M3 axis_rot(V3 a, float th) {
  float s, c;
  sincosf(th, &s, &c);
  float t = 1.f - c;
  M3 R;
  R.m[0] = t * a.x * a.x + c; R.m[1] = t * a.x * a.y - s * a.z; R.m[2] = t * a.x * a.z + s * a.y;
  R.m[3] = t * a.x * a.y + s * a.z; R.m[4] = t * a.y * a.y + c; R.m[5] = t * a.y * a.z - s * a.x;
  R.m[6] = t * a.x * a.z - s * a.y; R.m[7] = t * a.y * a.z + s * a.x; R.m[8] = t * a.z * a.z + c;
  return R;
}

// spatial inertia about the base origin, base coordinates: mass, h = m*c, I_O (xx yy zz xy xz yz)
struct SI {
  float m;
  V3 h;
  float i[6];
};
struct SV {
  V3 a, l;  // angular; linear
};
__device__ __forceinline__ SV operator+(SV p, SV q) { return SV{p.a + q.a, p.l + q.l}; }
__device__ __forceinline__ SV scale(SV p, float s) { return SV{s * p.a, s * p.l}; }
__device__ __forceinline__ float sdot(SV p, SV q) { return dot(p.a, q.a) + dot(p.l, q.l); }
__device__ __forceinline__ V3 symmul(const float* I, V3 v) {
  return v3(I[0] * v.x + I[3] * v.y + I[4] * v.z, I[3] * v.x + I[1] * v.y + I[5] * v.z,
            I[4] * v.x + I[5] * v.y + I[2] * v.z);
}
__device__ __forceinline__ SV simul(const SI& I, SV v) {  // f = (I_O w + h x v, m v - h x w)
  return SV{symmul(I.i, v.a) + cross(I.h, v.l), I.m * v.l - cross(I.h, v.a)};
}
__device__ __forceinline__ SI siadd(const SI& p, const SI& q) {
  SI r;
  r.m = p.m + q.m;
  r.h = p.h + q.h;
#pragma unroll
  for (int k = 0; k < 6; ++k) r.i[k] = p.i[k] + q.i[k];
  return r;
}
__device__ __forceinline__ SI make_si(float m, V3 c, const M3& R, const float* Ib) {
  // Ic = R Ib R^T (Ib symmetric about COM in body frame), then shift to the base origin
  float Ibm[9] = {Ib[0], Ib[3], Ib[4], Ib[3], Ib[1], Ib[5], Ib[4], Ib[5], Ib[2]};
  float T[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) T[3 * r + k] = R.m[3 * r] * Ibm[k] + R.m[3 * r + 1] * Ibm[3 + k] + R.m[3 * r + 2] * Ibm[6 + k];
  float Ic[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k) Ic[3 * r + k] = T[3 * r] * R.m[3 * k] + T[3 * r + 1] * R.m[3 * k + 1] + T[3 * r + 2] * R.m[3 * k + 2];
  SI s;
  s.m = m;
  s.h = m * c;
  float cc = dot(c, c);
  s.i[0] = Ic[0] + m * (cc - c.x * c.x);
  s.i[1] = Ic[4] + m * (cc - c.y * c.y);
  s.i[2] = Ic[8] + m * (cc - c.z * c.z);
  s.i[3] = Ic[1] - m * c.x * c.y;
  s.i[4] = Ic[2] - m * c.x * c.z;
  s.i[5] = Ic[5] - m * c.y * c.z;
  return s;
}
__device__ __forceinline__ SV crm(SV v, SV m) { return SV{cross(v.a, m.a), cross(v.a, m.l) + cross(v.l, m.a)}; }
__device__ __forceinline__ SV crf(SV v, SV f) { return SV{cross(v.a, f.a) + cross(v.l, f.l), cross(v.a, f.l)}; }
__device__ __forceinline__ float sv_get(const SV& s, int r) {
  return r == 0 ? s.a.x : r == 1 ? s.a.y : r == 2 ? s.a.z : r == 3 ? s.l.x : r == 4 ? s.l.y : s.l.z;
}

// Per-leg solver blocks live in LDS as [leg][field][lane] columns (each lane owns one column, so
// the accesses are bank-conflict free).  Field map inside a leg (LEGF floats):
//   0..8  joint axes a_j (base frame)   9..17 joint origins o_j   18..35 K = D^-1 B^T (3x6)
//   36..41 D^-1 (00 11 22 01 02 12)   42..44 per-joint bias / solve scratch
//   45..47 leg joint rates at the start of the contact solve   48..50 Y = sum of D^-1 p_l over the
//   impulses applied to this leg (lazy propagation: qd_l = qd0_l + Y_l - K_l (v_b - v_b0))
//   51..53 (plane build, TGS) dz = sum over the sub-iterations of h (q0_l + Y_l) = the leg's joint motion + K_l dx_b
#define LEGF (MIRROR > 1 ? LRL_LEGF_FLAT : LRL_LEGF_MESH)
#define LF_DZ 51
#define LI(r, c) ((r) * ((r) + 1) / 2 + (c))

#define KLEGF ((int)(sizeof(KLeg) / sizeof(float)))  // floats of one leg's model table
struct Lds {
  float* base;     // leg blocks, then contact rows: [field][env slot] columns shared by the env's 4 lanes
  int sph_off;     // field offset of the contact rows
  int es;          // env slot of this lane inside the workgroup
  float* ktab;     // the model tables a lane reads at a lane-dependent index, staged once per launch:
                   // K->leg[4], then per sphere (x, y, z, radius), then per sphere its link (int)
  int nsph;
  int lim_off;     // field offset of the joint-limit rows (LIM_* map below contact_pgs_q)
  float* wl;       // terrain query work list (after the staged tables): [BLOCK] candidate masks, [BLOCK] offsets,
                   // [BLOCK] masks of the candidates found in contact
  __device__ __forceinline__ float* wlist() const { return wl; }
  __device__ __forceinline__ const KLeg& kleg(int l) const { return reinterpret_cast<const KLeg*>(ktab)[l]; }
  __device__ __forceinline__ float4 sph4(int s) const {
    return reinterpret_cast<const float4*>(ktab + 4 * KLEGF)[s];
  }
  // per sphere: its link (low byte, sign-extended: -1 on the base) | (its support table + 1) << 8 (lrl_model::sphere_hull)
  __device__ __forceinline__ int slink_raw(int s) const {
    return reinterpret_cast<const int*>(ktab + 4 * KLEGF + 4 * nsph)[s];
  }
  __device__ __forceinline__ int slink(int s) const { return (slink_raw(s) << 24) >> 24; }
  // the terrain query's radius of sphere s: its own, or 0 for a support-table collider (its query point is the
  // support point)
  __device__ __forceinline__ float qrad(int s) const { return (slink_raw(s) >> 8) ? 0.f : sph4(s).w; }
  // self-collision groups [lane][g][begin, end) (KParams::self_grp) and pairs (KParams::self_pair), after the links
  __device__ __forceinline__ const int* sgrp() const { return reinterpret_cast<const int*>(ktab + 4 * KLEGF + 5 * nsph); }
  __device__ __forceinline__ uint32_t spair(int p) const {
    return reinterpret_cast<const uint32_t*>(ktab + 4 * KLEGF + 5 * nsph + 40)[p];
  }
  // field f of a row = row pointer + f * ENVS (a constant f folds into the ds_read / ds_write immediate offset)
  __device__ __forceinline__ float& leg(int l, int f) const { return lp(l)[f * ENVS]; }
  __device__ __forceinline__ float& sph(int s, int f) const { return sp(s)[f * ENVS]; }
  __device__ __forceinline__ V3 a(int l, int j) const { return v3(leg(l, 3 * j), leg(l, 3 * j + 1), leg(l, 3 * j + 2)); }
  __device__ __forceinline__ V3 o(int l, int j) const {
    return v3(leg(l, 9 + 3 * j), leg(l, 9 + 3 * j + 1), leg(l, 9 + 3 * j + 2));
  }
  // column pointers: field f of the row is p[f * ENVS] (constant offsets fold into the ds_read / ds_write
  // immediate instead of one address computation per field)
  __device__ __forceinline__ float* sp(int s) const { return base + (sph_off + s * NSF) * ENVS + es; }
  __device__ __forceinline__ float* lp(int l) const { return base + l * LEGF * ENVS + es; }
  __device__ __forceinline__ float* lm(int r) const { return base + (lim_off + r * LIMF) * ENVS + es; }
  __device__ __forceinline__ float Kx(int l, int j, int r) const { return leg(l, 18 + 6 * j + r); }
  __device__ __forceinline__ float Di(int l, int k) const { return leg(l, 36 + k); }
};

// reciprocal on the hardware v_rcp_f32 (1 ulp) instead of the IEEE division sequence (≈ 10 instructions): the
// physics sub-step's divisions are all of this form; the fp64 oracle bounds the result, not bit identity
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ void chol6(float* L) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float s = L[LI(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[LI(j, k)] * L[LI(j, k)];
    float d = sqrtf(fmaxf(s, 1e-12f));
    L[LI(j, j)] = d;
    float inv = frcp(d);
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      float t = L[LI(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[LI(i, k)] * L[LI(j, k)];
      L[LI(i, j)] = t * inv;
    }
  }
}
// S^-1 = L^-T L^-1 from the Cholesky factor, packed lower (in place).  One inversion per sub-step
// keeps every later solve a dense 6x6 multiply: short dependency chains, no divisions.
__device__ __forceinline__ void chol_to_inverse6(float* L) {
  float Li[21];
#pragma unroll
  for (int j = 0; j < 6; ++j) Li[LI(j, j)] = frcp(L[LI(j, j)]);
#pragma unroll
  for (int i = 1; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = j; k < i; ++k) s += L[LI(i, k)] * Li[LI(k, j)];
      Li[LI(i, j)] = -s * Li[LI(i, i)];
    }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = i; k < 6; ++k) s += Li[LI(k, i)] * Li[LI(k, j)];
      L[LI(i, j)] = s;
    }
}
__device__ __forceinline__ void sym6mul(const float* S, const float* x, float* y) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 6; ++j) s += S[i >= j ? LI(i, j) : LI(j, i)] * x[j];
    y[i] = s;
  }
}
__device__ __forceinline__ V3 sym3mul(float d0, float d1, float d2, float d3, float d4, float d5, V3 v) {
  return v3(d0 * v.x + d3 * v.y + d4 * v.z, d3 * v.x + d1 * v.y + d5 * v.z, d4 * v.x + d5 * v.y + d2 * v.z);
}
__device__ __forceinline__ V3 di_mul(const Lds& M, int l, V3 v) {
  return sym3mul(M.Di(l, 0), M.Di(l, 1), M.Di(l, 2), M.Di(l, 3), M.Di(l, 4), M.Di(l, 5), v);
}
__device__ __forceinline__ void sym3inv(const float* D, float* Di) {
  float a = D[0], b = D[3], c = D[4], d = D[1], e = D[5], f = D[2];
  float c00 = d * f - e * e, c01 = c * e - b * f, c02 = b * e - c * d;
  float det = a * c00 + b * c01 + c * c02;
  float id = frcp(det);
  Di[0] = c00 * id;
  Di[3] = c01 * id;
  Di[4] = c02 * id;
  Di[1] = (a * f - c * c) * id;
  Di[5] = (b * c - a * e) * id;
  Di[2] = (a * d - b * b) * id;
}

// c_j = a_j x (x - o_j) for the joints carrying the point (j <= link)
__device__ __forceinline__ void leg_dirs(const Lds& M, int lsel, int link, V3 x, V3* c) {
#pragma unroll
  for (int j = 0; j < 3; ++j) c[j] = (j <= link) ? cross(M.a(lsel, j), x - M.o(lsel, j)) : v3(0.f, 0.f, 0.f);
}

// current joint rates of leg L under lazy propagation: qd_L = q0_L + Y_L - K_L v_b  (q0 = qd0 + K v_b0)
__device__ __forceinline__ V3 leg_qd(const Lds& M, int L, const float* vb) {
  float q[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float k = 0.f;
#pragma unroll
    for (int r = 0; r < 6; ++r) k += M.Kx(L, j, r) * vb[r];
    q[j] = M.leg(L, 45 + j) + M.leg(L, 48 + j) - k;
  }
  return v3(q[0], q[1], q[2]);
}

// ------------------------------------------------------------------------------------------------
// Terrain mesh contact (own model; PhysX's trimesh / heightfield collision is closed): the sphere centre p
// is tested against the 18 triangles of the 3x3 grid cells around it (vertex moves of the slope-corrected
// trimesh are at most one cell, so every triangle within a cell of p is among them); the triangle whose
// closest point q is nearest wins (ties: first in cell order).  The separation is the signed distance to the
// terrain surface minus r: |p - q| with the sign of the height-field test — p is inside the terrain when it is
// below the plane of the triangle under it (the triangle whose xy projection holds p's xy; all triangles face
// up) — so a centre above every vertex is never inside, whatever the slope of the nearest triangle.  The normal
// is the winning face normal inside its face region and otherwise the direction from p towards the outside
// ((p - q) / |p - q| above the surface, (q - p) / |p - q| below).  With no triangle under p (degenerate cells)
// the sign falls back to the winning triangle's plane.  Triangles whose xy bounding box, grown by
// r + contact_offset, does not hold p's xy are skipped (part of the model: the oracle applies the same rule);
// a conservative max-height map skips the test, exactly, for spheres clear of the terrain.
// ------------------------------------------------------------------------------------------------
struct THit {
  float sep;
  V3 n;  // world frame
};
__device__ __forceinline__ V3 terr_v(const float* __restrict__ vtx, int idx) {
  const float4 v = reinterpret_cast<const float4*>(vtx)[idx];
  return v3(v.x, v.y, v.z);
}
// closest point of triangle (a, b, c) to p (Voronoi regions, Ericson 5.1.5); face = p projects inside.  The region
// ratios use the hardware reciprocal (1 ulp) instead of the IEEE division sequence (≈ 10 instructions each): a few
// 1e-9 m at these distances, far inside the oracle's 1e-5 m nearest-triangle margin
__device__ __forceinline__ V3 closest_on_tri(V3 p, V3 a, V3 b, V3 c, bool& face) {
  face = false;
  const V3 ab = b - a, ac = c - a, ap = p - a;
  const float d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) return a;
  const V3 bp = p - b;
  const float d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.f && d4 <= d3) return b;
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) return a + (d1 * __builtin_amdgcn_rcpf(d1 - d3)) * ab;
  const V3 cp = p - c;
  const float d5 = dot(ab, cp), d6 = dot(ac, cp);
  if (d6 >= 0.f && d5 <= d6) return c;
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) return a + (d2 * __builtin_amdgcn_rcpf(d2 - d6)) * ac;
  const float va = d3 * d6 - d5 * d4;
  if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f)
    return b + ((d4 - d3) * __builtin_amdgcn_rcpf((d4 - d3) + (d5 - d6))) * (c - b);
  face = true;
  const float dn = __builtin_amdgcn_rcpf(va + vb + vc);
  return a + (vb * dn) * ab + (vc * dn) * ac;
}
// tv: this wave's LDS scratch for the 4 x 4 vertex block, [vertex][lane] float4 (conflict-free b128 accesses)
__device__ THit terrain_query(const KParams* __restrict__ K, V3 p, float r, float margin, float4* tv, int lane,
                              unsigned long long* prof) {
#ifdef LRL_ENV_PROFILE
  const unsigned long long tq_a = clock64();
#endif
  THit h;
  h.sep = 1e30f;
  h.n = v3(0.f, 0.f, 1.f);
  const int R = K->terr_rows, Cn = K->terr_cols;
  const float bs = K->p.border_size, ih = K->terr_inv_hs;
  const int ci = min(max((int)floorf((p.x + bs) * ih), 0), R - 2);
  const int cj = min(max((int)floorf((p.y + bs) * ih), 0), Cn - 2);
  const float g = r + margin;
  // the max-height word and the 4 x 4 vertices of the 3 x 3 cells in one memory round trip (rows / columns
  // clamped for the load; cells off the grid are never marked), staged in LDS for the triangle walk
  const float4* __restrict__ vtx = reinterpret_cast<const float4*>(K->terr_vtx);
  const float hmax = K->terr_hmax[ci * Cn + cj];
  // the block's 16 gathers are issued with the max-height word, not after its test: one memory round trip per query
  // instead of two (a query that ends at the test has fetched its block for nothing — L2-resident terrain)
  float4 V[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int vi = min(max(ci - 1 + a, 0), R - 1);
#pragma unroll
    for (int b = 0; b < 4; ++b) V[a][b] = vtx[vi * Cn + min(max(cj - 1 + b, 0), Cn - 1)];
  }
  if (p.z - r - margin > hmax) {
#ifdef LRL_ENV_PROFILE
    prof[21] += 1;  // queries that end at the max-height test
#endif
    return h;
  }
  // local frame at vertex (ci, cj): differences of nearby fp32 coordinates are exact (Sterbenz), so the walk
  // resolves distances to ~1e-8 m instead of the ~2e-6 m ulp of world coordinates 20-40 m from the origin
  // (nearest-triangle ties between coplanar neighbours then go the way the exact geometry does)
  {
    const float4 O = V[1][1];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) V[a][b] = make_float4(V[a][b].x - O.x, V[a][b].y - O.y, V[a][b].z - O.z, 0.f);
    p = p - v3(O.x, O.y, O.z);
  }
  // triangles (bit 2 * (3 di + dj) + t) whose xy bounding box grown by g holds p's xy: a triangle under / over p
  // always qualifies, so penetrating spheres keep the triangle they are in
  uint32_t tris = 0;
#pragma unroll
  for (int di = 0; di < 3; ++di)
#pragma unroll
    for (int dj = 0; dj < 3; ++dj) {
      const int i = ci - 1 + di, j = cj - 1 + dj;
      const bool cell = i >= 0 && i <= R - 2 && j >= 0 && j <= Cn - 2;
      const float4 A = V[di][dj], B = V[di][dj + 1], Cc = V[di + 1][dj], D = V[di + 1][dj + 1];
      // t = 0: (v(i,j), v(i+1,j+1), v(i,j+1)) = (A, D, B);  t = 1: (v(i,j), v(i+1,j), v(i+1,j+1)) = (A, Cc, D)
      // ... and that p is not more than g above everywhere (its distance exceeds g, so it decides no contact),
      // except a triangle whose plain bounding box holds p's xy (it may be the one under p, which sets the side)
      auto mark = [&](float4 a, float4 b, float4 c) {
        const float x0 = fminf(fminf(a.x, b.x), c.x), x1 = fmaxf(fmaxf(a.x, b.x), c.x);
        const float y0 = fminf(fminf(a.y, b.y), c.y), y1 = fmaxf(fmaxf(a.y, b.y), c.y);
        const bool in = p.x >= x0 && p.x <= x1 && p.y >= y0 && p.y <= y1;
        const bool high = p.z - g > fmaxf(fmaxf(a.z, b.z), c.z);
        return cell && p.x >= x0 - g && p.x <= x1 + g && p.y >= y0 - g && p.y <= y1 + g && (in || !high);
      };
      const bool t0 = mark(A, D, B), t1 = mark(A, Cc, D);
      const int k = 2 * (3 * di + dj);
      tris |= (t0 ? 1u << k : 0u) | (t1 ? 2u << k : 0u);
    }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) tv[(4 * a + b) * BLOCK + lane] = V[a][b];
#ifdef LRL_ENV_PROFILE
  const unsigned long long tq_b = clock64();
  prof[16] += tq_b - tq_a;  // vertex block gathers + staging
  prof[19] += __popc(tris);  // marked triangles (summed over lanes)
#endif
  float best = 3.0e38f;
  int bk = -1;     // the nearest triangle so far (its closest point / normal are formed once, after the walk)
  int under = -1;  // height-field side of p from the triangle under it: 1 above / on, 0 below, -1 none found
  // each lane walks its own marked triangles in order (the wave runs max-over-lanes triangles, not 18)
  // (the next marked triangle's vertices are read while this one is tested: the LDS round trip overlaps the arithmetic;
  // an exhausted lane re-reads its last triangle, unused)
  auto tri_load = [&](int k, float4& fa, float4& fb, float4& fc) {
    const int c = k >> 1, di = c / 3, dj = c - 3 * di;
    const int ia = 4 * di + dj;  // v(i,j) in the block
    const int ib = (k & 1) ? ia + 4 : ia + 5, ic = (k & 1) ? ia + 5 : ia + 1;
    fa = tv[ia * BLOCK + lane];
    fb = tv[ib * BLOCK + lane];
    fc = tv[ic * BLOCK + lane];
  };
  int kn = tris ? __builtin_ctz(tris) : 0;
  float4 na, nb, nc;
  tri_load(kn, na, nb, nc);
  while (__any((int)(tris != 0u))) {
#ifdef LRL_ENV_PROFILE
    prof[18] += 1;  // walk iterations (per wave: the busiest lane's count)
#endif
    if (tris) {
      const int k = kn;
      const float4 fa = na, fb = nb, fc = nc;
      tris &= tris - 1u;
      kn = tris ? __builtin_ctz(tris) : k;
      tri_load(kn, na, nb, nc);
      const V3 va = v3(fa.x, fa.y, fa.z), b = v3(fb.x, fb.y, fb.z), cv = v3(fc.x, fc.y, fc.z);
      const V3 nf = cross(b - va, cv - va);
      const float a2 = dot(nf, nf);
      // under p: p's xy inside the triangle's xy projection (counter-clockwise when nf.z > 0)
      if (nf.z > 0.f) {
        const float wa = (b.x - p.x) * (cv.y - p.y) - (b.y - p.y) * (cv.x - p.x);
        const float wb = (cv.x - p.x) * (va.y - p.y) - (cv.y - p.y) * (va.x - p.x);
        const float wc = (va.x - p.x) * (b.y - p.y) - (va.y - p.y) * (b.x - p.x);
        if (wa >= 0.f && wb >= 0.f && wc >= 0.f) under = dot(nf, p - va) >= 0.f ? 1 : 0;
      }
      if (a2 >= 1e-12f) {  // (zero area: collapsed by the slope correction)
        bool face;
        const V3 q = closest_on_tri(p, va, b, cv, face);
        const V3 dq = p - q;
        const float d2 = dot(dq, dq);
        bk = d2 < best ? k : bk;
        best = fminf(d2, best);
      }
    }
  }
  // the winner's closest point, face region and unit normal: the same evaluation once more
  V3 bc = v3(0.f, 0.f, 0.f), bn = v3(0.f, 0.f, 1.f), ba = v3(0.f, 0.f, 0.f);
  bool bface = true;
  if (bk >= 0) {
    const int c = bk >> 1, di = c / 3, dj = c - 3 * di;
    const int ia = 4 * di + dj;
    const int ib = (bk & 1) ? ia + 4 : ia + 5, ic = (bk & 1) ? ia + 5 : ia + 1;
    const float4 fa = tv[ia * BLOCK + lane], fb = tv[ib * BLOCK + lane], fc = tv[ic * BLOCK + lane];
    const V3 va = v3(fa.x, fa.y, fa.z), b = v3(fb.x, fb.y, fb.z), cv = v3(fc.x, fc.y, fc.z);
    const V3 nf = cross(b - va, cv - va);
    bc = closest_on_tri(p, va, b, cv, bface);
    bn = rsqrtf(dot(nf, nf)) * nf;
    ba = va;
  }
#ifdef LRL_ENV_PROFILE
  prof[17] += clock64() - tq_b;  // the triangle walk
#endif
  const float dist = sqrtf(best), sd = dot(bn, p - ba);
  const bool above = under >= 0 ? under == 1 : sd >= 0.f;
  h.sep = (above ? dist : -dist) - r;
  if (bface || dist <= 1e-6f) {
    h.n = (bface && (sd >= 0.f) != above) ? -1.f * bn : bn;
  } else {
    h.n = ((above ? 1.f : -1.f) / dist) * (p - bc);
  }
  return h;
}
// max terrain height over the vertex window around the base's cell (lrl_sim_set_terrain: +-(ceil(reach / h) + 2)
// rows / columns, reach = the model's largest xy distance of a sphere surface from the base origin), so every
// vertex a query of one of the env's spheres can read is inside it; a sphere above it cannot touch the terrain
__device__ __forceinline__ float terrain_window_max(const KParams* __restrict__ K, const float* pos) {
  const float bs = K->p.border_size, ih = K->terr_inv_hs;
  const int ci = min(max((int)floorf((pos[0] + bs) * ih), 0), K->terr_rows - 2);
  const int cj = min(max((int)floorf((pos[1] + bs) * ih), 0), K->terr_cols - 2);
  return K->terr_wmax[ci * K->terr_cols + cj];
}
// tangents of a contact normal: t1 = x (or y when n is close to x) made orthogonal to n, t2 = n x t1
__device__ __forceinline__ void contact_frame(V3 n, V3& t1, V3& t2) {
  const V3 t = fabsf(n.x) < 0.9f ? v3(1.f - n.x * n.x, -n.x * n.y, -n.x * n.z) : v3(-n.y * n.x, 1.f - n.y * n.y, -n.y * n.z);
  t1 = rsqrtf(dot(t, t)) * t;
  t2 = cross(n, t1);
}

// Contact-row field map (NSF floats per sphere, LDS [field][env slot]):
//   0..2 contact point x (base frame)   3 1/W_nn   4 W_t1n   5 W_t2n   6..8 (W_tt)^-1 (11, 12, 22)
//   9 velocity target   10..12 impulse (n, t1, t2)
//   13..30 g_d (d = n, t1, t2): base-velocity row of the contact velocity along world direction d,
//          g_d = [x x n_d, n_d] - K_L^T h_d   (the same row maps an impulse to the base: r = sum_d lambda_d g_d)
//   31..39 h_d = C_L^T n_d (joint-rate row; C_L = joint directions of the carrying joints)
//   40..57 z_d = S^-1 g_d (base-velocity change per unit impulse)   58..66 e_d = D_L^-1 h_d (change of Y_L)
//   (plane build, TGS) field 9 holds the sub-step-start separation instead of the velocity target, 67 the restitution
//   target (-1e30 without one); each sub-iteration forms the target from sep_0 + J_n dx (below)
// so one Gauss-Seidel update is u_d = g_d . v_b + h_d . (q0_L + Y_L), the cone projection, and
// v_b += sum_d dlambda_d z_d,  Y_L += sum_d dlambda_d e_d  — short independent dot products.
#define SF_G 13
#define SF_H 31
#define SF_Z 40
#define SF_E 58
#define SF_BR 67

// apply a world-frame impulse change dl = (n, t1, t2) of sphere s (leg lsel) to v_b and Y_lsel (every read
// before the first store, so the rows arrive in one LDS round trip)
__device__ __forceinline__ void apply_impulse(const Lds& M, int s, int lsel, float dn, float dt1, float dt2,
                                              float* vb) {
  const int L = lsel < 0 ? 0 : lsel;
  float z[18], ev[9], y[3];
#pragma unroll
  for (int k = 0; k < 18; ++k) z[k] = M.sph(s, SF_Z + k);
#pragma unroll
  for (int k = 0; k < 9; ++k) ev[k] = M.sph(s, SF_E + k);
#pragma unroll
  for (int j = 0; j < 3; ++j) y[j] = M.leg(L, 48 + j);
#pragma unroll
  for (int r = 0; r < 6; ++r) vb[r] += dn * z[r] + dt1 * z[6 + r] + dt2 * z[12 + r];
  if (lsel >= 0) {
#pragma unroll
    for (int j = 0; j < 3; ++j) M.leg(lsel, 48 + j) = y[j] + (dn * ev[j] + dt1 * ev[3 + j] + dt2 * ev[6 + j]);
  }
}

// A mesh collider's contact point (lrl_model::sphere_hull; lrl/robot.py support_table): the hull's support point in
// the link-frame direction d, from the cube-map cell of d (major axis m, the first of x, y, z on ties; face 2 m +
// (d_m < 0); u, v = the other two components over |d_m|, each cell index floor((u + 1) N / 2) clamped to [0, N)) and
// the cell's LRL_HULL_K candidates, the one furthest along d (the first on a tie).  One aligned 64-B block per cell;
// the tables (≈ 0.6 MB for the Mini Cheetah) stay in L2.  The division is IEEE (not frcp), so the cell is the fp64
// oracle's except within rounding of a cell edge (lrl_oracle.c hull_support).
__device__ __forceinline__ V3 hull_support(const KParams* __restrict__ K, int h, V3 d) {
  const int N = K->hull_res;
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  const int m = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
  const float dm = m == 0 ? d.x : m == 1 ? d.y : d.z;
  const float du = m == 0 ? d.y : m == 1 ? d.z : d.x;
  const float dv = m == 0 ? d.z : m == 1 ? d.x : d.y;
  const float adm = fabsf(dm), hn = 0.5f * (float)N;
  const int iu = min(max((int)floorf((du / adm + 1.f) * hn), 0), N - 1);
  const int iv = min(max((int)floorf((dv / adm + 1.f) * hn), 0), N - 1);
  const int cell = ((2 * m + (dm < 0.f ? 1 : 0)) * N + iu) * N + iv;
  const float4* c = reinterpret_cast<const float4*>(K->hull_tab) + ((size_t)h * 6 * N * N + cell) * LRL_HULL_K;
  float4 v[LRL_HULL_K];
#pragma unroll
  for (int k = 0; k < LRL_HULL_K; ++k) v[k] = c[k];
  V3 best = v3(v[0].x, v[0].y, v[0].z);
  float bd = dot(best, d);
#pragma unroll
  for (int k = 1; k < LRL_HULL_K; ++k) {
    const V3 p = v3(v[k].x, v[k].y, v[k].z);
    const float pd = dot(p, d);
    if (pd > bd) {
      bd = pd;
      best = p;
    }
  }
  return best;
}

// One contact sphere's solver rows: g_d, h_d, z_d, e_d and the 3x3 Delassus block W_de = g_d . z_e + h_d . e_e
// Terrain contacts (TERR): detection leaves the world normal n in fields 3..5 (free until the Delassus values
// land there); contact_setup builds the frame (n, t1, t2) from it and parks n in fields 0..2 (the contact point
// is dead after the rows are built) for the contact-force pass.  Flat ground: n = z, t1 = x, t2 = y.
template <bool TERR>
__device__ __forceinline__ void contact_setup(const Lds& M, const float* Si, const M3& R, int s, int lsel, int link) {
  // every LDS read up front (the point, the leg's joint axes / origins, K and D^-1; base spheres read leg 0's
  // and discard them by selection), every store at the end: one round trip instead of one per dependent read
  const int L = lsel < 0 ? 0 : lsel;
  const bool onleg = lsel >= 0;
  // (the detection / activation leaves the contact point in fields 6..8 — the sphere centre, or a collider's support
  // point — and the centre in 0..2 for the self-collision pairs)
  const V3 x = v3(M.sph(s, 6), M.sph(s, 7), M.sph(s, 8));
  V3 nw = v3(0.f, 0.f, 1.f);
  if constexpr (TERR) nw = v3(M.sph(s, 3), M.sph(s, 4), M.sph(s, 5));
  V3 ax[3], og[3];
  float kx[3][6], di[6];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    ax[j] = M.a(L, j);
    og[j] = M.o(L, j);
#pragma unroll
    for (int r = 0; r < 6; ++r) kx[j][r] = M.Kx(L, j, r);
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) di[k] = M.Di(L, k);
  V3 c[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) c[j] = (onleg && j <= link) ? cross(ax[j], x - og[j]) : v3(0.f, 0.f, 0.f);
  float g[3][6], z[3][6];
  V3 h[3], ev[3];
  V3 fr[3];  // contact frame in base coordinates
  if constexpr (TERR) {
    V3 t1, t2;
    contact_frame(nw, t1, t2);
    fr[0] = mulT(R, nw);
    fr[1] = mulT(R, t1);
    fr[2] = mulT(R, t2);
  } else {
    fr[0] = v3(R.m[6], R.m[7], R.m[8]);
    fr[1] = v3(R.m[0], R.m[1], R.m[2]);
    fr[2] = v3(R.m[3], R.m[4], R.m[5]);
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const V3 nd = fr[d];
    const V3 xn = cross(x, nd);
    g[d][0] = xn.x; g[d][1] = xn.y; g[d][2] = xn.z; g[d][3] = nd.x; g[d][4] = nd.y; g[d][5] = nd.z;
    h[d] = v3(dot(c[0], nd), dot(c[1], nd), dot(c[2], nd));
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const float gk = g[d][r] - (kx[0][r] * h[d].x + kx[1][r] * h[d].y + kx[2][r] * h[d].z);
      g[d][r] = onleg ? gk : g[d][r];
    }
    const V3 e = sym3mul(di[0], di[1], di[2], di[3], di[4], di[5], h[d]);
    ev[d] = onleg ? e : v3(0.f, 0.f, 0.f);
    sym6mul(Si, g[d], z[d]);
  }
  float W[3][3];
#pragma unroll
  for (int e = 0; e < 3; ++e)
#pragma unroll
    for (int d = 0; d <= e; ++d) {
      float w = 0.f;
#pragma unroll
      for (int r = 0; r < 6; ++r) w += g[d][r] * z[e][r];
      w += dot(h[d], ev[e]);
      W[d][e] = w;
      W[e][d] = w;
    }
  const float id = frcp(W[1][1] * W[2][2] - W[1][2] * W[2][1]);
#pragma unroll
  for (int d = 0; d < 3; ++d) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      M.sph(s, SF_G + 6 * d + r) = g[d][r];
      M.sph(s, SF_Z + 6 * d + r) = z[d][r];
    }
    M.sph(s, SF_H + 3 * d) = h[d].x; M.sph(s, SF_H + 3 * d + 1) = h[d].y; M.sph(s, SF_H + 3 * d + 2) = h[d].z;
    M.sph(s, SF_E + 3 * d) = ev[d].x; M.sph(s, SF_E + 3 * d + 1) = ev[d].y; M.sph(s, SF_E + 3 * d + 2) = ev[d].z;
  }
  M.sph(s, 3) = frcp(W[0][0]);
  M.sph(s, 4) = W[1][0];
  M.sph(s, 5) = W[2][0];
  M.sph(s, 6) = W[2][2] * id;  // (W_tt)^-1: 11, 12, 22
  M.sph(s, 7) = -W[1][2] * id;
  M.sph(s, 8) = W[1][1] * id;
  if constexpr (TERR) {
    M.sph(s, 0) = nw.x;
    M.sph(s, 1) = nw.y;
    M.sph(s, 2) = nw.z;
  }
}

struct Body {  // per-lane env state during the step: the base in every lane of the quad, the joints of the lane's leg
  float pos[3], quat[4], V[3], W[3];
  float q[3], qd[3];  // joints 3 ql .. 3 ql + 2 (the whole 12 are gathered over the quad for the post-physics)
  float lo[3], hi[3];  // their position limits (KParams::dof_lo / dof_hi)
  float llam[3];       // their limit-row impulses x sigma after the last sub-step (warm start; on the terrain mesh the
                       // rows' LDS is the next sub-step's query scratch)
};


// ------------------------------------------------------------------------------------------------
// One physics sub-step.  Contact impulses of the sub-step stay in the LDS rows (fields 10..12).
// ------------------------------------------------------------------------------------------------
// sum of a value over the 4 lanes of an env (xor-shuffles inside the quad)
// quad exchanges through DPP quad_perm (a VALU operand modifier, no LDS crossbar round trip):
// xor 1 = [1,0,3,2] (0xB1), xor 2 = [2,3,0,1] (0x4E), broadcast of quad lane l = [l,l,l,l] (l * 0x55)
template <int CTRL>
__device__ __forceinline__ int qperm(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float qperm(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// sum over the quad: every lane gets (v0 + v1) + (v2 + v3) with the operands of each add swapped at most, so
// the four lanes hold bitwise the same value
__device__ __forceinline__ float quad_sum(float v) {
  v += qperm<0xB1>(v);
  v += qperm<0x4E>(v);
  return v;
}
// value of quad lane l
__device__ __forceinline__ float quad_bcast(float v, int l) {
  switch (l) {
    case 0: return qperm<0x00>(v);
    case 1: return qperm<0x55>(v);
    case 2: return qperm<0xAA>(v);
    default: return qperm<0xFF>(v);
  }
}
__device__ __forceinline__ uint64_t quad_or(uint64_t v) {
  int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
  lo |= qperm<0xB1>(lo);
  hi |= qperm<0xB1>(hi);
  lo |= qperm<0x4E>(lo);
  hi |= qperm<0x4E>(hi);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
// OR over the env's lanes: the quad, then (MIRROR 4) the env's 4 quads = one DPP row of 16 lanes: row_mirror pairs
// quad q with quad 3 - q, row_half_mirror quad 0 with 1 and 2 with 3 (after the quad OR every lane of a quad holds
// the same value, so the lane pairing inside the quads does not matter)
__device__ __forceinline__ uint64_t env_or(uint64_t v) {
  v = quad_or(v);
  if constexpr (MIRROR > 1) {
    int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    lo |= qperm<0x140>(lo);
    hi |= qperm<0x140>(hi);
    lo |= qperm<0x141>(lo);
    hi |= qperm<0x141>(hi);
    v = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
  }
  return v;
}
// sum over the env's lanes (used where at most one lane holds a non-zero term, or small integers: exact in any order)
__device__ __forceinline__ float env_sum(float v) {
  v = quad_sum(v);
  if constexpr (MIRROR > 1) {
    v += qperm<0x140>(v);
    v += qperm<0x141>(v);
  }
  return v;
}
// mirrored quad qi of this lane (0 with one quad per env)
__device__ __forceinline__ int mirror_quad() { return MIRROR > 1 ? (int)((threadIdx.x >> 2) & (MIRROR - 1)) : 0; }
// the spheres / limit rows of `own` that mirrored quad qi detects and builds rows for: every MIRROR-th in bit order
__device__ __forceinline__ uint64_t own_split(uint64_t own, int qi) {
  if constexpr (MIRROR == 1) return own;
  uint64_t r = 0;
  int k = 0;
  for (uint64_t m = own; m; m &= m - 1ull, ++k)
    if ((k & (MIRROR - 1)) == qi) r |= m & (~m + 1ull);
  return r;
}
// The Gauss-Seidel update with the base velocity spread over the env's quad: lane q holds v_b[q] (vo0) and, for
// q < 2, v_b[q + 4] (vo1, 0 in lanes 2 and 3), and owns component q < 3 of the leg accumulators Y_L.  Each lane
// forms its part of the three contact-velocity rows, one quad sum gives every lane the same u, the cone
// projection runs in all four lanes, and each lane updates only what it owns — a quarter of the row reads and
// fused multiply-adds of the redundant form, and no lane reads what another lane writes (no barrier).
template <bool B>
struct BoolC {
  static constexpr bool value = B;
};
// TGS (plane build, solver_type 1): the sub-iteration's motion so far, dx = (dx_b spread over the quad as v_b is, dz of
// the legs in LDS), and what turns a separation into a target (h = dt / iterations)
struct Tgs {
  float dxo0, dxo1, ih, baum, maxdep;
};
// target of a row whose separation moved from sep0 by the quad's share ds of J_n dx: -sep/h, or Baumgarte below contact
__device__ __forceinline__ float tgs_target(const Tgs& T, float sep0, float ds) {
  const float sp = sep0 + quad_sum(ds);
  return sp >= 0.f ? -sp * T.ih : fminf(-T.baum * sp * T.ih, T.maxdep);
}
template <bool TGS>
__device__ __forceinline__ void contact_pgs_q(const Lds& M, int s, int lsel, float mu, int q, float& vo0, float& vo1,
                                              const Tgs& T) {
  const int L = lsel < 0 ? 0 : lsel;
  const bool hj = q < 3;
  const int qh = hj ? q : 2;  // lane 3 reads lane 2's fields and zeroes them by selection (no divergent branches)
  // every read of the update is issued before any compute or store: one LDS round trip per update instead of
  // one per row (a conditional read becomes an exec-masked branch with its own lgkmcnt(0) wait); the per-lane
  // columns are addressed from three row pointers so the field offsets are instruction immediates
  float* const rs = M.sp(s);
  const float* const rq = rs + q * ENVS;
  const float* const rh = rs + qh * ENVS;
  float* const lg = M.lp(L) + qh * ENVS;
  float g0[3], g1[3], hv[3], z0[3], z1[3], ev[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    g0[d] = rq[(SF_G + 6 * d) * ENVS];
    g1[d] = rq[(SF_G + 6 * d + 4) * ENVS];
    hv[d] = rh[(SF_H + 3 * d) * ENVS];
    z0[d] = rq[(SF_Z + 6 * d) * ENVS];
    z1[d] = rq[(SF_Z + 6 * d + 4) * ENVS];
    ev[d] = rh[(SF_E + 3 * d) * ENVS];
  }
  const float y45 = lg[45 * ENVS], y48 = lg[48 * ENVS];
  const float iWnn = rs[3 * ENVS], Wt1n = rs[4 * ENVS], Wt2n = rs[5 * ENVS];
  const float i11 = rs[6 * ENVS], i12 = rs[7 * ENVS], i22 = rs[8 * ENVS], b9 = rs[9 * ENVS];
  const float ln0 = rs[10 * ENVS], lt10 = rs[11 * ENVS], lt20 = rs[12 * ENVS];
  const float yq = hj ? y45 + y48 : 0.f;
  float b;
  if constexpr (TGS) {  // field 9 = sep0, the restitution target a floor under the sub-iteration's target
    const float dz = lg[LF_DZ * ENVS];
    b = fmaxf(tgs_target(T, b9, g0[0] * T.dxo0 + g1[0] * T.dxo1 + (hj ? hv[0] * dz : 0.f)), rs[SF_BR * ENVS]);
  } else {
    b = b9;
  }
  float u[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float a = g0[d] * vo0 + g1[d] * vo1;
    a += (hj ? hv[d] : 0.f) * yq;
    u[d] = quad_sum(a);
  }
  const float ln = fmaxf(ln0 - (u[0] - b) * iWnn, 0.f);
  const float dn = ln - ln0;
  const float ut1 = u[1] + Wt1n * dn, ut2 = u[2] + Wt2n * dn;
  float lt1 = lt10 - (i11 * ut1 + i12 * ut2), lt2 = lt20 - (i12 * ut1 + i22 * ut2);
  const float lim = mu * ln, nt2 = lt1 * lt1 + lt2 * lt2;
  const float sc = nt2 > lim * lim ? (nt2 > 0.f ? lim * rsqrtf(nt2) : 0.f) : 1.f;
  lt1 *= sc;
  lt2 *= sc;
  rs[10 * ENVS] = ln;
  rs[11 * ENVS] = lt1;
  rs[12 * ENVS] = lt2;
  const float dt1 = lt1 - lt10, dt2 = lt2 - lt20;
  vo0 += dn * z0[0] + dt1 * z0[1] + dt2 * z0[2];
  const float d1 = dn * z1[0] + dt1 * z1[1] + dt2 * z1[2];
  vo1 = q < 2 ? vo1 + d1 : 0.f;
  if (hj) lg[48 * ENVS] = y48 + (dn * ev[0] + dt1 * ev[1] + dt2 * ev[2]);
}

// ------------------------------------------------------------------------------------------------
// Joint position limits (the URDF limits PhysX articulations enforce; own formulation): joint j of
// leg L near its nearer limit gets a unilateral joint-space row with the generalised force sigma e_j (sigma = +1
// at the lower limit, -1 at the upper), so its separation rate is u = sigma qd_j = g . v_b + sigma (q0_L + Y_L)_j
// with g = -sigma K_L[j] (no base part: the limit pushes joint against joint), z = S^-1 g, e = sigma D_L^-1[:, j],
// W = g . z + (D_L^-1)_jj.  Rows live after the contact spheres in the solver's index space (bit nsph + 3 L + j),
// are owned by leg L's lane and are visited after the spheres, in joint order.  Row field map (LIMF floats,
// LDS [field][env slot], after the contact rows; on the terrain mesh they alias the query's vertex blocks, which
// are dead by the time the rows are written):
//   0..5 g   6..11 z   12..14 e   15 1/W   16 velocity target   17 impulse   18 sigma
// ------------------------------------------------------------------------------------------------
#define LIM_G 0
#define LIM_Z 6
#define LIM_E 12
#define LIM_IW 15
#define LIM_B 16
#define LIM_LAM 17
#define LIM_SG 18

// rows of joint r = 3 L + j (lane L): every LDS read up front, every store at the end
__device__ __forceinline__ void limit_setup(const Lds& M, const float* Si, int r, int L) {
  float* const row = M.lm(r);
  const int j = r - 3 * L;
  const float sg = row[LIM_SG * ENVS];
  float kx[3][6], di[6];
#pragma unroll
  for (int jj = 0; jj < 3; ++jj)
#pragma unroll
    for (int c = 0; c < 6; ++c) kx[jj][c] = M.Kx(L, jj, c);
#pragma unroll
  for (int k = 0; k < 6; ++k) di[k] = M.Di(L, k);
  float g[6], z[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) g[c] = -sg * (j == 0 ? kx[0][c] : j == 1 ? kx[1][c] : kx[2][c]);
  sym6mul(Si, g, z);
  // column j of D^-1 (packed 00 11 22 01 02 12)
  const float c0 = j == 0 ? di[0] : j == 1 ? di[3] : di[4];
  const float c1 = j == 0 ? di[3] : j == 1 ? di[1] : di[5];
  const float c2 = j == 0 ? di[4] : j == 1 ? di[5] : di[2];
  float w = 0.f;
#pragma unroll
  for (int c = 0; c < 6; ++c) w += g[c] * z[c];
  w += j == 0 ? di[0] : j == 1 ? di[1] : di[2];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    row[(LIM_G + c) * ENVS] = g[c];
    row[(LIM_Z + c) * ENVS] = z[c];
  }
  row[LIM_E * ENVS] = sg * c0;
  row[(LIM_E + 1) * ENVS] = sg * c1;
  row[(LIM_E + 2) * ENVS] = sg * c2;
  row[LIM_IW * ENVS] = frcp(w);
}

// warm start of a limit row in its owner lane with the carried impulse: v_b += lam z (summed over the quad by the
// caller), Y_L += lam e.  The carried value is lam x the sigma it was solved with (lam >= 0): a row whose nearer limit
// switched since the previous sub-step (sigma flipped) starts cold instead of pushing the wrong way.
__device__ __forceinline__ void limit_apply(const Lds& M, int r, int L, float lam_sg, float* dvb) {
  float* const row = M.lm(r);
  const float lam = fmaxf(lam_sg * row[LIM_SG * ENVS], 0.f);
  float z[6], ev[3], y[3];
#pragma unroll
  for (int c = 0; c < 6; ++c) z[c] = row[(LIM_Z + c) * ENVS];
#pragma unroll
  for (int k = 0; k < 3; ++k) ev[k] = row[(LIM_E + k) * ENVS];
#pragma unroll
  for (int k = 0; k < 3; ++k) y[k] = M.leg(L, 48 + k);
  row[LIM_LAM * ENVS] = lam;
#pragma unroll
  for (int c = 0; c < 6; ++c) dvb[c] += lam * z[c];
#pragma unroll
  for (int k = 0; k < 3; ++k) M.leg(L, 48 + k) = y[k] + lam * ev[k];
}

// Gauss-Seidel update of limit row r (leg L, joint j) with the base velocity spread over the quad as in
// contact_pgs_q: lane q owns v_b[q], v_b[q + 4] (q < 2) and component q of Y_L; lane j adds sigma (q0 + Y)_j
// (TGS: LIM_B holds the sub-step-start separation; the row's J dx = g . dx_b + sigma dz_j)
template <bool TGS>
__device__ __forceinline__ void limit_pgs_q(const Lds& M, int r, int q, float& vo0, float& vo1, const Tgs& T) {
  const int L = (r * 11) >> 5;  // r / 3 for r < 12
  const int j = r - 3 * L;
  const bool hj = q < 3;
  const int qh = hj ? q : 2;
  float* const row = M.lm(r);
  const float* const rq = row + q * ENVS;
  float* const lg = M.lp(L) + qh * ENVS;
  // (lanes 2, 3 read g / z entries 6, 7 of the next field group for the v_b[q + 4] terms and zero them with vo1 = 0)
  const float g0 = rq[LIM_G * ENVS], g1 = rq[(LIM_G + 4) * ENVS];
  const float z0 = rq[LIM_Z * ENVS], z1 = rq[(LIM_Z + 4) * ENVS];
  const float ev = row[(LIM_E + qh) * ENVS];
  const float y45 = lg[45 * ENVS], y48 = lg[48 * ENVS];
  const float iw = row[LIM_IW * ENVS], b9 = row[LIM_B * ENVS], l0 = row[LIM_LAM * ENVS], sg = row[LIM_SG * ENVS];
  float b;
  if constexpr (TGS)
    b = tgs_target(T, b9, g0 * T.dxo0 + g1 * T.dxo1 + (q == j ? sg * lg[LF_DZ * ENVS] : 0.f));
  else
    b = b9;
  float a = g0 * vo0 + g1 * vo1;
  a += q == j ? sg * (y45 + y48) : 0.f;
  const float u = quad_sum(a);
  const float ln = fmaxf(l0 - (u - b) * iw, 0.f);
  const float dn = ln - l0;
  row[LIM_LAM * ENVS] = ln;
  vo0 += dn * z0;
  vo1 = q < 2 ? vo1 + dn * z1 : 0.f;
  if (hj) lg[48 * ENVS] = y48 + dn * ev;
}

// lane of the quad that owns sphere s: its leg, or round-robin for the base spheres
__device__ __forceinline__ int sph_owner(const KParams* __restrict__ K, int s) {
  const int l = K->sph_leg[s];
  return l >= 0 ? l : (s & 3);
}
// leg of sphere s from the (wave-uniform) leg sphere ranges: a few compares against scalar registers instead
// of a per-lane global load of K->sph_leg[s] on the solver's dependency chain
struct SphLegs {
  int b[4], e[4];
};
__device__ __forceinline__ SphLegs sph_legs(const KParams* __restrict__ K) {
  SphLegs r;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    r.b[l] = __builtin_amdgcn_readfirstlane(K->leg_sph_begin[l]);
    r.e[l] = __builtin_amdgcn_readfirstlane(K->leg_sph_end[l]);
  }
  return r;
}
// L.b[l] / L.e[l] for a lane-varying l as masked ORs: a select chain over l is turned into a lookup table in a private
// (scratch) array by the compiler
__device__ __forceinline__ int sel4(const int* v, int l) {
  return (v[0] & -(int)(l == 0)) | (v[1] & -(int)(l == 1)) | (v[2] & -(int)(l == 2)) | (v[3] & -(int)(l == 3));
}
__device__ __forceinline__ int sph_leg_of(const SphLegs& L, int s) {
  int l = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) l = (s >= L.b[k] && s < L.e[k]) ? k : l;
  return l;
}

// ------------------------------------------------------------------------------------------------
// Self-collision (PhysX collides the links of an articulation with each other when Cfg.asset.self_collisions is
// 0, except a link and its parent; own formulation).  Candidate pairs (KParams::self_pair, canonical
// order: lane / leg La major, then its groups) are sphere-sphere between the legs and inside a leg, and leg sphere
// against the base box.  The contact normal n points from body B to body A (an impulse lambda n pushes A, -lambda n
// pushes B) and both bodies share the contact point x, so the base motion cancels from the relative velocity:
//   u_d = hA_d . qd_A + hB_d . qd_B,  hA_d = C_A^T n_d,  hB_d = -C_B^T n_d  (C = joint directions at x)
//       = g_d . v_b + hA_d . (q0_A + Y_A) + hB_d . (q0_B + Y_B)  with  g_d = -K_A^T hA_d - K_B^T hB_d,
// an impulse moves v_b by lambda S^-1 g_d and Y_A / Y_B by lambda D^-1 hA_d / D^-1 hB_d (a same-leg pair folds hB
// into hA; the base box has no hB).  The first LRL_SELF_SLOTS active pairs of an env in the canonical order get
// the solver rows after the joint limits (bits nsph + 12 + slot), built cold every sub-step (no warm start: a
// pair's slot can change between sub-steps).  A row lives in the LDS rows of two contact spheres the env has NOT in
// ground contact in the sub-step (fields 3..66 of each, 128 floats; fields 0..2 keep the sphere centres the detection
// reads): slot k takes the env's free spheres 2k and 2k + 1 in index order, so an env gets min(LRL_SELF_SLOTS, free / 2)
// slots (the oracle applies the same cap).  Field map:
//   0..2 n (base frame)  3..5 x (base frame)  6 leg A  7 leg B (-1: base box)  8 link A  9 link B  10 velocity target
//   11..13 impulse (n, t1, t2)  14 1/W_nn  15 W_t1n  16 W_t2n  17..19 (W_tt)^-1 (11, 12, 22)  20..37 g_d
//   38..46 hA_d  47..55 hB_d  56..73 z_d = S^-1 g_d  74..82 D_A^-1 hA_d  83..91 D_B^-1 hB_d
//   92..100 (n, t1, t2) in the world frame (contact forces)  101 body A  102 body B
// ------------------------------------------------------------------------------------------------
#define SR_N 0
#define SR_X 3
#define SR_LA 6
#define SR_LB 7
#define SR_KA 8
#define SR_KB 9
#define SR_B 10
#define SR_LAM 11
#define SR_IW 14
#define SR_G 20
#define SR_HA 38
#define SR_HB 47
#define SR_Z 56
#define SR_EA 74
#define SR_EB 83
#define SR_F 92
#define SR_BA 101
#define SR_BB 102

// the n-th set bit of m (n < popcount(m))
__device__ __forceinline__ int nth_bit(uint64_t m, int n) {
  for (int i = 0; i < n; ++i) m &= m - 1ull;
  return __builtin_ctzll(m);
}
// self-contact row k of this env in the rows of its free spheres 2k, 2k + 1 (constant field indices fold the choice)
struct SRow {
  float* a;
  float* b;
  __device__ __forceinline__ float& operator[](int f) const { return f < 64 ? a[f * ENVS] : b[(f - 64) * ENVS]; }
};
__device__ __forceinline__ SRow self_row(const Lds& M, uint64_t freem, int k) {
  const int h1 = nth_bit(freem, 2 * k);
  const int h2 = __builtin_ctzll(freem & ~((2ull << h1) - 1ull));  // the next free sphere
  return SRow{M.sp(h1) + 3 * ENVS, M.sp(h2) + 3 * ENVS};
}
// spheres of the env free of ground contact (the quad-ORed active mask's sphere bits)
__device__ __forceinline__ uint64_t free_spheres(const Lds& M, uint64_t act) {
  const uint64_t all = M.nsph >= 64 ? ~0ull : (1ull << M.nsph) - 1ull;
  return ~act & all;
}

// separation of a sphere (centre ca, radius ra) against a sphere (cb, rb) or, box, the base box: n from B to A, x = the
// contact point (contraction off: the register gate and the LDS pass evaluate it bitwise alike)
__device__ __forceinline__ float self_geom_c(const KParams* __restrict__ K, V3 ca, float ra, V3 cb, float rb, bool box,
                                             V3& n, V3& x) {
#pragma clang fp contract(off)
  if (!box) {
    const V3 d = ca - cb;
    const float dd = dot(d, d), dist = sqrtf(dd);
    n = dd > 1e-18f ? frcp(dist) * d : v3(0.f, 0.f, 1.f);
    x = 0.5f * ((ca - ra * n) + (cb + rb * n));
    return dist - ra - rb;
  }
  const V3 bc = v3(K->box_c[0], K->box_c[1], K->box_c[2]), bh = v3(K->box_h[0], K->box_h[1], K->box_h[2]);
  const V3 c = ca - bc;
  const V3 q = v3(fminf(fmaxf(c.x, -bh.x), bh.x), fminf(fmaxf(c.y, -bh.y), bh.y), fminf(fmaxf(c.z, -bh.z), bh.z));
  const V3 d = c - q;
  const float dd = dot(d, d);
  if (dd > 0.f) {  // centre outside the box: nearest surface point
    const float dist = sqrtf(dd);
    n = frcp(dist) * d;
    x = q + bc;
    return dist - ra;
  }
  // centre inside: the nearest face (first of x, y, z on ties)
  const float dx = bh.x - fabsf(c.x), dy = bh.y - fabsf(c.y), dz = bh.z - fabsf(c.z);
  const int k = (dx <= dy && dx <= dz) ? 0 : (dy <= dz ? 1 : 2);
  const float sx = c.x < 0.f ? -1.f : 1.f, sy = c.y < 0.f ? -1.f : 1.f, sz = c.z < 0.f ? -1.f : 1.f;
  n = k == 0 ? v3(sx, 0.f, 0.f) : k == 1 ? v3(0.f, sy, 0.f) : v3(0.f, 0.f, sz);
  x = v3(k == 0 ? sx * bh.x : c.x, k == 1 ? sy * bh.y : c.y, k == 2 ? sz * bh.z : c.z) + bc;
  return -(k == 0 ? dx : k == 1 ? dy : dz) - ra;
}
// the same for candidate pair pk, centres from the contact rows' fields 0..2 (the leg pass writes every centre there)
__device__ __forceinline__ float self_geom(const KParams* __restrict__ K, const Lds& M, uint32_t pk, V3& n, V3& x) {
  const int a = pk & 255u, b = (pk >> 8) & 255u;
  const V3 ca = v3(M.sph(a, 0), M.sph(a, 1), M.sph(a, 2));
  const bool box = b == 255;
  const int bb = box ? a : b;
  const V3 cb = v3(M.sph(bb, 0), M.sph(bb, 1), M.sph(bb, 2));
  return self_geom_c(K, ca, M.sph4(a).w, cb, M.sph4(bb).w, box, n, x);
}

__device__ __forceinline__ bool aabb_overlap(V3 alo, V3 ahi, V3 blo, V3 bhi) {
  return alo.x <= bhi.x && blo.x <= ahi.x && alo.y <= bhi.y && blo.y <= ahi.y && alo.z <= bhi.z && blo.z <= ahi.z;
}

__device__ __forceinline__ int quad_bcast_i(int v, int l) { return __float_as_int(quad_bcast(__int_as_float(v), l)); }

// Per-lane gate (no barrier; it runs every sub-step, so it is kept to a few instructions per sphere — the kernel
// issues about one VALU instruction per 6 cycles): this leg's same-leg and box candidates within the offset and its
// bounding box for the leg-leg groups, from its own sphere centres in LDS (written by this lane in the leg pass), every
// read up front over a clamped index (a leg has at most 8 spheres, lrl_capi.cpp).  Squared distances against the
// offset widened by 1e-5 m: conservative, the LDS pass decides every pair the gate lets through exactly.
struct SelfGate {
  V3 lo, hi;     // this leg's sphere surfaces grown by contact_offset / 2
  int hits;      // same-leg + box candidates (and 1 for a leg with more than two link-0 spheres: the LDS pass decides)
};
__device__ __forceinline__ SelfGate self_gate(const KParams* __restrict__ K, const Lds& M, const SphLegs& SL, int ql,
                                              float co) {
  const int b = sel4(SL.b, ql);
  const int e = sel4(SL.e, ql);
  const int kmax = __builtin_amdgcn_readfirstlane(K->self_kmax);  // (wave-uniform loop bound)
  const int nhip = K->self_nhip[ql];
  if constexpr (MIRROR > 1) {
    // mirrored quads: quad q takes the leg's spheres k = q, q + 4 (one uniform pass of the loop body per 4 spheres, the
    // sphere index varying by lane); the box is min / max-reduced and the hits summed over the env's quads with DPP
    // row rotations by 4 and 8 lanes (lane ql meets lane ql of every quad) — exact in any order, as the loop's form
    const int qi = mirror_quad();
    const float cw = co + 1e-5f, hc = 0.5f * co;
    const float bcx = K->box_c[0], bcy = K->box_c[1], bcz = K->box_c[2];
    const float bhx = K->box_h[0], bhy = K->box_h[1], bhz = K->box_h[2];
    const bool box = bhx >= 0.f;
    const int s0 = min(b, e - 1), s1 = min(b + 1, e - 1);
    const float h0x = M.sph(s0, 0), h0y = M.sph(s0, 1), h0z = M.sph(s0, 2);
    const float h1x = M.sph(s1, 0), h1y = M.sph(s1, 1), h1z = M.sph(s1, 2);
    const float h0r = nhip >= 1 ? M.sph4(s0).w + cw : -1e30f, h1r = nhip >= 2 ? M.sph4(s1).w + cw : -1e30f;
    SelfGate G;
    G.lo = v3(1e30f, 1e30f, 1e30f);
    G.hi = v3(-1e30f, -1e30f, -1e30f);
    int hits = (nhip > 2 && qi == 0) ? 1 : 0;
#pragma unroll
    for (int j = 0; j < 8 / MIRROR; ++j)
      if (MIRROR * j < kmax) {
        const int k = MIRROR * j + qi;
        const int s = min(b + k, e - 1);
        const float cx = M.sph(s, 0), cy = M.sph(s, 1), cz = M.sph(s, 2), r = M.sph4(s).w;
        const int lk = M.slink(s);
        const bool use = k < kmax && b + k < e;
        const float rg = r + hc;
        const float xl = use ? cx - rg : 1e30f, yl = use ? cy - rg : 1e30f, zl = use ? cz - rg : 1e30f;
        const float xh = use ? cx + rg : -1e30f, yh = use ? cy + rg : -1e30f, zh = use ? cz + rg : -1e30f;
        G.lo = v3(fminf(G.lo.x, xl), fminf(G.lo.y, yl), fminf(G.lo.z, zl));
        G.hi = v3(fmaxf(G.hi.x, xh), fmaxf(G.hi.y, yh), fmaxf(G.hi.z, zh));
        const float qx = fmaxf(fabsf(cx - bcx) - bhx, 0.f), qy = fmaxf(fabsf(cy - bcy) - bhy, 0.f),
                    qz = fmaxf(fabsf(cz - bcz) - bhz, 0.f);
        const float rb = r + cw;
        const bool hb = box && lk >= 1 && qx * qx + qy * qy + qz * qz < rb * rb;
        const float ax = cx - h0x, ay = cy - h0y, az = cz - h0z, rh = h0r + r;
        const float bx = cx - h1x, by = cy - h1y, bz = cz - h1z, ri = h1r + r;
        const bool hh = lk == 2 && ((rh > 0.f && ax * ax + ay * ay + az * az < rh * rh) ||
                                    (ri > 0.f && bx * bx + by * by + bz * bz < ri * ri));
        hits += (use && (hb || hh)) ? 1 : 0;
      }
    auto rmin = [](float v) {
      v = fminf(v, qperm<0x124>(v));
      return fminf(v, qperm<0x128>(v));
    };
    auto rmax = [](float v) {
      v = fmaxf(v, qperm<0x124>(v));
      return fmaxf(v, qperm<0x128>(v));
    };
    G.lo = v3(rmin(G.lo.x), rmin(G.lo.y), rmin(G.lo.z));
    G.hi = v3(rmax(G.hi.x), rmax(G.hi.y), rmax(G.hi.z));
    hits += qperm<0x124>(hits);
    hits += qperm<0x128>(hits);
    G.hits = hits;
    return G;
  }
  float cx[8], cy[8], cz[8], r[8];
  int lk[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < kmax) {
      const int s = min(b + k, e - 1);
      cx[k] = M.sph(s, 0);
      cy[k] = M.sph(s, 1);
      cz[k] = M.sph(s, 2);
      r[k] = M.sph4(s).w;
      lk[k] = M.slink(s);
    }
  const float cw = co + 1e-5f, hc = 0.5f * co;
  const float bcx = K->box_c[0], bcy = K->box_c[1], bcz = K->box_c[2];
  const float bhx = K->box_h[0], bhy = K->box_h[1], bhz = K->box_h[2];
  const bool box = bhx >= 0.f;
  // the leg's hip spheres (its first one or two spheres when it has them)
  const float h0x = cx[0], h0y = cy[0], h0z = cz[0], h0r = nhip >= 1 ? r[0] + cw : -1e30f;
  const float h1x = cx[1], h1y = cy[1], h1z = cz[1], h1r = nhip >= 2 ? r[1] + cw : -1e30f;
  SelfGate G;
  G.lo = v3(1e30f, 1e30f, 1e30f);
  G.hi = v3(-1e30f, -1e30f, -1e30f);
  int hits = nhip > 2 ? 1 : 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < kmax) {
      const bool use = b + k < e;
      const float rg = r[k] + hc;
      const float xl = use ? cx[k] - rg : 1e30f, yl = use ? cy[k] - rg : 1e30f, zl = use ? cz[k] - rg : 1e30f;
      const float xh = use ? cx[k] + rg : -1e30f, yh = use ? cy[k] + rg : -1e30f, zh = use ? cz[k] + rg : -1e30f;
      G.lo = v3(fminf(G.lo.x, xl), fminf(G.lo.y, yl), fminf(G.lo.z, zl));
      G.hi = v3(fmaxf(G.hi.x, xh), fmaxf(G.hi.y, yh), fmaxf(G.hi.z, zh));
      // base box: squared distance of the centre from the box (0 inside) against (r + offset)^2
      const float qx = fmaxf(fabsf(cx[k] - bcx) - bhx, 0.f), qy = fmaxf(fabsf(cy[k] - bcy) - bhy, 0.f),
                  qz = fmaxf(fabsf(cz[k] - bcz) - bhz, 0.f);
      const float rb = r[k] + cw;
      const bool hb = box && lk[k] >= 1 && qx * qx + qy * qy + qz * qz < rb * rb;
      // the hip spheres against the calf's
      const float ax = cx[k] - h0x, ay = cy[k] - h0y, az = cz[k] - h0z, rh = h0r + r[k];
      const float bx = cx[k] - h1x, by = cy[k] - h1y, bz = cz[k] - h1z, ri = h1r + r[k];
      const bool hh = lk[k] == 2 && ((rh > 0.f && ax * ax + ay * ay + az * az < rh * rh) ||
                                     (ri > 0.f && bx * bx + by * by + bz * bz < ri * ri));
      hits += (use && (hb || hh)) ? 1 : 0;
    }
  G.hits = hits;
  return G;
}

// Rows of the quad's self-contacts, entered only by waves the gate flags (a hit, a leg-leg bounding-box overlap, or a
// leg with more than two link-0 spheres): the canonical count over this lane's live groups from the LDS centres, the
// quad prefix of the counts, then the first LRL_SELF_SLOTS hits get rows — geometry, legs / links / bodies and the
// velocity target (restitution from the sub-step-start joint rates, LDS leg fields 45..47).
__device__ void self_detect(const KParams* __restrict__ K, const Lds& M, const SphLegs& SL, int ql, unsigned live,
                            float dt, float rest, uint64_t& active, uint64_t& sown) {
  const lrl_env_params& P = K->p;
  const float co = P.contact_offset, idt = frcp(dt);
  const int* G = M.sgrp() + 10 * ql;
  const uint64_t freem = free_spheres(M, quad_or(active));
  const int cap = min(LRL_SELF_SLOTS, __builtin_popcountll(freem) >> 1);  // the env's slots
  // the count stops at cap: a lane's count only places the lanes after it, and a prefix that reaches cap leaves
  // them no slot either way, so the capped counts assign exactly the slots the full counts would
  // (lrl_sim_self_contact_stats on: the full count, so the pairs the cap drops are counted; the slots are the same)
  uint32_t* const stats = K->self_stats;
  const int lim = stats ? 0x7fffffff : cap;
  int cnt = 0;
#pragma unroll
  for (int g = 0; g < 5; ++g)
    if ((live >> g) & 1u)
      for (int p = G[2 * g]; p < G[2 * g + 1] && cnt < lim; ++p) {
        V3 n, x;
        cnt += self_geom(K, M, M.spair(p), n, x) < co ? 1 : 0;
      }
  const int c0 = quad_bcast_i(cnt, 0), c1 = quad_bcast_i(cnt, 1), c2 = quad_bcast_i(cnt, 2);
  if (stats) {
    const int total = c0 + c1 + c2 + quad_bcast_i(cnt, 3);
    if (ql == 0 && mirror_quad() == 0 && total > 0) {  // per env and sub-step: pairs in contact, pairs without a slot
      atomicAdd(stats + 0, 1u);
      atomicAdd(stats + 1, (uint32_t)total);
      if (total > cap) {
        atomicAdd(stats + 2, 1u);
        atomicAdd(stats + 3, (uint32_t)(total - cap));
      }
    }
  }
  int slot = ql == 0 ? 0 : ql == 1 ? c0 : ql == 2 ? c0 + c1 : c0 + c1 + c2;
  const int end = min(slot + cnt, cap);
  if (slot >= end) return;
#pragma unroll
  for (int g = 0; g < 5; ++g)
    if ((live >> g) & 1u)
      for (int p = G[2 * g]; p < G[2 * g + 1] && slot < end; ++p) {
        const uint32_t pk = M.spair(p);
        V3 n, x;
        const float sep = self_geom(K, M, pk, n, x);
        if (!(sep < co)) continue;
        const int a = pk & 255u, b = (pk >> 8) & 255u;
        const int la = ql, lb = b == 255 ? -1 : sph_leg_of(SL, b);
        const int ka = M.slink(a), kb = b == 255 ? 0 : M.slink(b);
        // relative normal velocity at the sub-step start: sum_j (a_j x (x - o_j)) . n qd_j over A's carrying joints,
        // minus the same over B's
        float u0 = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (j <= ka) u0 += dot(cross(M.a(la, j), x - M.o(la, j)), n) * M.leg(la, 45 + j);
          if (lb >= 0 && j <= kb) u0 -= dot(cross(M.a(lb, j), x - M.o(lb, j)), n) * M.leg(lb, 45 + j);
        }
        float tgt = sep >= 0.f ? -sep * idt : fminf(-P.baumgarte * sep * idt, P.max_depenetration_velocity);
        if (u0 < -P.bounce_threshold_velocity && rest > 0.f) tgt = fmaxf(tgt, -rest * u0);
        const SRow row = self_row(M, freem, slot);
        row[SR_N + 0] = n.x; row[SR_N + 1] = n.y; row[SR_N + 2] = n.z;
        row[SR_X + 0] = x.x; row[SR_X + 1] = x.y; row[SR_X + 2] = x.z;
        row[SR_LA] = (float)la;
        row[SR_LB] = (float)lb;
        row[SR_KA] = (float)ka;
        row[SR_KB] = (float)kb;
        row[SR_B] = tgt;
        row[SR_BA] = (float)((pk >> 16) & 255u);
        row[SR_BB] = (float)(pk >> 24);
        const uint64_t bit = 1ull << (M.nsph + LRL_NUM_DOF + slot);
        active |= bit;
        sown |= bit;
        ++slot;
      }
}

// solver rows of self-contact slot k in its owner lane (every global / LDS read up front)
__device__ void self_setup(const Lds& M, const float* Si, const M3& R, uint64_t freem, int k) {
  const SRow row = self_row(M, freem, k);
  const V3 n = v3(row[SR_N], row[SR_N + 1], row[SR_N + 2]);
  const V3 x = v3(row[SR_X], row[SR_X + 1], row[SR_X + 2]);
  const int la = (int)row[SR_LA], lb = (int)row[SR_LB], ka = (int)row[SR_KA], kb = (int)row[SR_KB];
  const int lbr = lb < 0 ? la : lb;
  V3 ca[3], cbv[3];
  float kxa[3][6], kxb[3][6], dia[6], dib[6];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    ca[j] = j <= ka ? cross(M.a(la, j), x - M.o(la, j)) : v3(0.f, 0.f, 0.f);
    cbv[j] = (lb >= 0 && j <= kb) ? cross(M.a(lbr, j), x - M.o(lbr, j)) : v3(0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      kxa[j][r] = M.Kx(la, j, r);
      kxb[j][r] = M.Kx(lbr, j, r);
    }
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    dia[c] = M.Di(la, c);
    dib[c] = M.Di(lbr, c);
  }
  const bool same = lb == la;
  V3 fr[3];
  fr[0] = n;
  contact_frame(n, fr[1], fr[2]);
  V3 ha[3], hb[3], ea[3], eb[3];
  float g[3][6], z[3][6];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    V3 h1 = v3(dot(ca[0], fr[d]), dot(ca[1], fr[d]), dot(ca[2], fr[d]));
    V3 h2 = v3(-dot(cbv[0], fr[d]), -dot(cbv[1], fr[d]), -dot(cbv[2], fr[d]));
    if (same) {
      h1 = h1 + h2;
      h2 = v3(0.f, 0.f, 0.f);
    }
    ha[d] = h1;
    hb[d] = h2;
#pragma unroll
    for (int r = 0; r < 6; ++r)
      g[d][r] = -(kxa[0][r] * h1.x + kxa[1][r] * h1.y + kxa[2][r] * h1.z) -
                (kxb[0][r] * h2.x + kxb[1][r] * h2.y + kxb[2][r] * h2.z);
    ea[d] = sym3mul(dia[0], dia[1], dia[2], dia[3], dia[4], dia[5], h1);
    eb[d] = sym3mul(dib[0], dib[1], dib[2], dib[3], dib[4], dib[5], h2);
    sym6mul(Si, g[d], z[d]);
  }
  float W[3][3];
#pragma unroll
  for (int e = 0; e < 3; ++e)
#pragma unroll
    for (int d = 0; d <= e; ++d) {
      float w = 0.f;
#pragma unroll
      for (int r = 0; r < 6; ++r) w += g[d][r] * z[e][r];
      w += dot(ha[d], ea[e]) + dot(hb[d], eb[e]);
      W[d][e] = w;
      W[e][d] = w;
    }
  // a relative Jacobian of zero (contact point on the joint axes) leaves an inert row
  const float det = W[1][1] * W[2][2] - W[1][2] * W[2][1];
  const float id = det > 1e-12f ? frcp(det) : 0.f;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      row[SR_G + 6 * d + r] = g[d][r];
      row[SR_Z + 6 * d + r] = z[d][r];
    }
    row[SR_HA + 3 * d] = ha[d].x; row[SR_HA + 3 * d + 1] = ha[d].y; row[SR_HA + 3 * d + 2] = ha[d].z;
    row[SR_HB + 3 * d] = hb[d].x; row[SR_HB + 3 * d + 1] = hb[d].y; row[SR_HB + 3 * d + 2] = hb[d].z;
    row[SR_EA + 3 * d] = ea[d].x; row[SR_EA + 3 * d + 1] = ea[d].y; row[SR_EA + 3 * d + 2] = ea[d].z;
    row[SR_EB + 3 * d] = eb[d].x; row[SR_EB + 3 * d + 1] = eb[d].y; row[SR_EB + 3 * d + 2] = eb[d].z;
    const V3 fw = mul(R, fr[d]);
    row[SR_F + 3 * d] = fw.x; row[SR_F + 3 * d + 1] = fw.y; row[SR_F + 3 * d + 2] = fw.z;
    row[SR_LAM + d] = 0.f;
  }
  row[SR_IW] = W[0][0] > 1e-12f ? frcp(W[0][0]) : 0.f;
  row[SR_IW + 1] = W[1][0];
  row[SR_IW + 2] = W[2][0];
  row[SR_IW + 3] = W[2][2] * id;
  row[SR_IW + 4] = -W[1][2] * id;
  row[SR_IW + 5] = W[1][1] * id;
}

// Gauss-Seidel update of self-contact slot k with the base velocity spread over the quad as in contact_pgs_q: lane q
// owns v_b[q], v_b[q + 4] (q < 2) and component q of Y_A and Y_B
__device__ __forceinline__ void self_pgs_q(const Lds& M, uint64_t freem, int k, float mu, int q,
                                           float& vo0, float& vo1) {
  const SRow row = self_row(M, freem, k);
  const bool hj = q < 3;
  const int qh = hj ? q : 2;
  const int la = (int)row[SR_LA], lb = (int)row[SR_LB];
  const int lbr = lb < 0 ? la : lb;
  float g0[3], g1[3], ha[3], hb[3], z0[3], z1[3], ea[3], eb[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {  // (lanes 2, 3 read g / z entries 6, 7 of the next field group for the v_b[q + 4]
    g0[d] = row[SR_G + 6 * d + q];  //  terms; vo1 = 0 there)
    g1[d] = row[SR_G + 6 * d + q + 4];
    z0[d] = row[SR_Z + 6 * d + q];
    z1[d] = row[SR_Z + 6 * d + q + 4];
    ha[d] = row[SR_HA + 3 * d + qh];
    hb[d] = row[SR_HB + 3 * d + qh];
    ea[d] = row[SR_EA + 3 * d + qh];
    eb[d] = row[SR_EB + 3 * d + qh];
  }
  const float iWnn = row[SR_IW], Wt1n = row[SR_IW + 1], Wt2n = row[SR_IW + 2];
  const float i11 = row[SR_IW + 3], i12 = row[SR_IW + 4], i22 = row[SR_IW + 5], b = row[SR_B];
  const float ln0 = row[SR_LAM], lt10 = row[SR_LAM + 1], lt20 = row[SR_LAM + 2];
  float* const lga = M.lp(la) + qh * ENVS;
  float* const lgb = M.lp(lbr) + qh * ENVS;
  const float ya45 = lga[45 * ENVS], ya48 = lga[48 * ENVS], yb45 = lgb[45 * ENVS], yb48 = lgb[48 * ENVS];
  float u[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float a = g0[d] * vo0 + g1[d] * vo1;
    a += hj ? ha[d] * (ya45 + ya48) + hb[d] * (yb45 + yb48) : 0.f;
    u[d] = quad_sum(a);
  }
  const float ln = fmaxf(ln0 - (u[0] - b) * iWnn, 0.f);
  const float dn = ln - ln0;
  const float ut1 = u[1] + Wt1n * dn, ut2 = u[2] + Wt2n * dn;
  float lt1 = lt10 - (i11 * ut1 + i12 * ut2), lt2 = lt20 - (i12 * ut1 + i22 * ut2);
  const float lim = mu * ln, nt2 = lt1 * lt1 + lt2 * lt2;
  const float sc = nt2 > lim * lim ? (nt2 > 0.f ? lim * rsqrtf(nt2) : 0.f) : 1.f;
  lt1 *= sc;
  lt2 *= sc;
  row[SR_LAM] = ln;  // (the four lanes store the same values)
  row[SR_LAM + 1] = lt1;
  row[SR_LAM + 2] = lt2;
  const float dt1 = lt1 - lt10, dt2 = lt2 - lt20;
  vo0 += dn * z0[0] + dt1 * z0[1] + dt2 * z0[2];
  const float d1 = dn * z1[0] + dt1 * z1[1] + dt2 * z1[2];
  vo1 = q < 2 ? vo1 + d1 : 0.f;
  if (hj) lga[48 * ENVS] = ya48 + (dn * ea[0] + dt1 * ea[1] + dt2 * ea[2]);
  if (hj && lb >= 0 && lb != la) lgb[48 * ENVS] = yb48 + (dn * eb[0] + dt1 * eb[1] + dt2 * eb[2]);
}

template <bool TERR>
__device__ void substep(const KParams* __restrict__ K, Body& st, const float* tau3, float mb, const float* Ib, V3 cb,
                        float mu, float rest, const Lds& M, uint64_t& active, int ql, uint64_t own, uint64_t odet,
                        float mu_s, float rest_s, unsigned long long* prof) {
  LRL_PROF_DECL
  const uint64_t prev_active = active;  // spheres in contact during the previous sub-step (warm start)
  const SphLegs SL = sph_legs(K);
  const lrl_env_params& P = K->p;
  const float dt = P.sim_dt, idt = frcp(dt);
  // TGS (legged_robot_config.py:247 solver_type 1; host: plane only) — the oracle's restatement, lrl_oracle.c
  // physics_substep: N sub-iterations of h = dt / N, targets from the separations moved by the motion so far, positions
  // from the accumulated motion
  const bool tgs = MIRROR > 1 && P.solver_tgs != 0 && P.solver_iterations > 0;
  const M3 R = quat_mat(st.quat[0], st.quat[1], st.quat[2], st.quat[3]);
  const V3 wb = mulT(R, v3(st.W[0], st.W[1], st.W[2]));
  const V3 vb = mulT(R, v3(st.V[0], st.V[1], st.V[2])) - cross(wb, cb);
  float nu[9];  // base twist (6), then this lane's leg joint rates (3)
  nu[0] = wb.x; nu[1] = wb.y; nu[2] = wb.z; nu[3] = vb.x; nu[4] = vb.y; nu[5] = vb.z;
#pragma unroll
  for (int j = 0; j < 3; ++j) nu[6 + j] = st.qd[j];
  const V3 gb = mulT(R, v3(P.gravity[0], P.gravity[1], P.gravity[2]));
  const SV v0 = SV{wb, vb};
  const SV a0 = SV{v3(0.f, 0.f, 0.f), v3(-gb.x, -gb.y, -gb.z)};
  const V3 Rz = v3(R.m[6], R.m[7], R.m[8]);  // world z in base coordinates
  const float pz = st.pos[2];

  SI A;
  {
    M3 E;
#pragma unroll
    for (int k = 0; k < 9; ++k) E.m[k] = (k % 4 == 0) ? 1.f : 0.f;
    A = make_si(mb, cb, E, Ib);
  }
  SV Cb = simul(A, a0) + crf(v0, simul(A, v0));
  float Sch[21];
#pragma unroll
  for (int k = 0; k < 21; ++k) Sch[k] = 0.f;
  active = 0;

  // contact detection helper: separation, restitution/speculative target (needs nu at sub-step start)
  // contact activation: velocity target (restitution / speculative / Baumgarte) along the normal nb (base frame)
  auto activate = [&](int s, V3 x, int lsel, int link, float sep, V3 nb) {
    active |= (1ull << s);
    M.sph(s, 6) = x.x;  // the contact point (contact_setup; the query's world point there is dead now)
    M.sph(s, 7) = x.y;
    M.sph(s, 8) = x.z;
    V3 u = cross(wb, x) + vb;
    if (lsel >= 0) {  // (a sphere recorded by this lane: its leg is the lane's own)
      V3 c[3];
      leg_dirs(M, lsel, link, x, c);
#pragma unroll
      for (int j = 0; j < 3; ++j) u = u + st.qd[j] * c[j];
    }
    const float u0 = dot(nb, u);
    float tgt = sep >= 0.f ? -sep * idt : fminf(-P.baumgarte * sep * idt, P.max_depenetration_velocity);
    if (u0 < -P.bounce_threshold_velocity && rest > 0.f) tgt = fmaxf(tgt, -rest * u0);
    M.sph(s, 9) = tgt;
  };
  // TERR: spheres are only recorded here (centre, world query point in the rows' free fields 6..8); those not
  // clear of the terrain window around the base (one load) are queried after the leg pass, each lane walking its
  // own list, so a wave pays max-over-lanes queries instead of every sphere of the model
  uint64_t cand = 0;
  float hwin = 0.f;

  if constexpr (TERR) hwin = terrain_window_max(K, st.pos);
  // aa / oo: the carrying leg's joint axes / origins in registers (the leg pass has them; no LDS read-back)
  // x: the sphere centre; xc, rad: the contact geometry — the centre and radius, or a support-table collider's support
  // point with radius 0 (hull_support)
  auto detect = [&](int s, V3 x, V3 xc, float rad, int lsel, int link, const V3* aa, const V3* oo) {
    if constexpr (TERR) {
      const V3 pw = v3(st.pos[0], st.pos[1], pz) + mul(R, xc);  // (the query point: centre, or support point)
      M.sph(s, 0) = x.x;
      M.sph(s, 1) = x.y;
      M.sph(s, 2) = x.z;
      M.sph(s, SF_G) = xc.x;  // the contact point in the base frame, for the activation (free until contact_setup)
      M.sph(s, SF_G + 1) = xc.y;
      M.sph(s, SF_G + 2) = xc.z;
      M.sph(s, 6) = pw.x;
      M.sph(s, 7) = pw.y;
      M.sph(s, 8) = pw.z;
      if (pw.z - rad - P.contact_offset <= hwin) cand |= 1ull << s;
#ifdef LRL_ENV_DEBUG
      {
        const int e_ = env_block() * ENVS + (int)(threadIdx.x >> 2);
        float* d = g_env_dbg + ((size_t)e_ * 64 + s) * 8;
        d[0] = (float)((cand >> s) & 1ull); d[1] = 1e30f; d[2] = pw.x; d[3] = pw.y; d[4] = pw.z; d[5] = hwin;
        d[6] = rad; d[7] = 1.f;
      }
#endif
      return;
    }
    const float sep = pz + dot(Rz, xc) - rad;
    M.sph(s, 0) = x.x;  // (every centre: the self-collision pairs read them)
    M.sph(s, 1) = x.y;
    M.sph(s, 2) = x.z;
    if (sep < P.contact_offset) {
      active |= (1ull << s);
      M.sph(s, 6) = xc.x;  // the contact point (contact_setup)
      M.sph(s, 7) = xc.y;
      M.sph(s, 8) = xc.z;
      V3 u = cross(wb, xc) + vb;
      if (lsel >= 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (j <= link) u = u + st.qd[j] * cross(aa[j], xc - oo[j]);
      }
      const float u0 = dot(Rz, u);
      const bool bounce = u0 < -P.bounce_threshold_velocity && rest > 0.f;
      if constexpr (MIRROR > 1) {
        if (tgs) {  // separation and restitution target; the sub-iterations form the targets
          M.sph(s, 9) = sep;
          M.sph(s, SF_BR) = bounce ? -rest * u0 : -1e30f;
          return;
        }
      }
      float tgt = sep >= 0.f ? -sep * idt : fminf(-P.baumgarte * sep * idt, P.max_depenetration_velocity);
      if (bounce) tgt = fmaxf(tgt, -rest * u0);
      M.sph(s, 9) = tgt;
    }
  };
  for (int s = ql; s < K->base_sph_end; s += QL)
    if (MIRROR == 1 || ((odet >> s) & 1ull)) {
      const float4 sp = M.sph4(s);
      detect(s, v3(sp.x, sp.y, sp.z), v3(sp.x, sp.y, sp.z), sp.w, -1, 0, nullptr, nullptr);
    }

  // ---- this lane's leg ----
  SI Aleg;     // composite inertia of the leg about the base origin
  SV Cleg;     // its RNEA force on the base
  {
    const int l = ql;
    const KLeg& kl = M.kleg(l);  // (LDS copy: a per-lane global read here was one memory round trip per joint)
    M3 Rp;
#pragma unroll
    for (int k = 0; k < 9; ++k) Rp.m[k] = (k % 4 == 0) ? 1.f : 0.f;
    V3 op = v3(0.f, 0.f, 0.f);
    SI Ij[3];
    SV S[3];
    V3 aa[3], oo[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      M3 Rf;
#pragma unroll
      for (int k = 0; k < 9; ++k) Rf.m[k] = kl.rfix[j][k];
      const V3 ax = v3(kl.axis[j][0], kl.axis[j][1], kl.axis[j][2]);
      const M3 Rj = mul(mul(Rp, Rf), axis_rot(ax, st.q[j]));
      const V3 o = op + mul(Rp, v3(kl.xyz[j][0], kl.xyz[j][1], kl.xyz[j][2]));
      const V3 a = mul(Rj, ax);
      M.leg(l, 3 * j) = a.x; M.leg(l, 3 * j + 1) = a.y; M.leg(l, 3 * j + 2) = a.z;
      M.leg(l, 9 + 3 * j) = o.x; M.leg(l, 9 + 3 * j + 1) = o.y; M.leg(l, 9 + 3 * j + 2) = o.z;
      S[j] = SV{a, cross(o, a)};
      aa[j] = a;
      oo[j] = o;
      const V3 c = o + mul(Rj, v3(kl.com[j][0], kl.com[j][1], kl.com[j][2]));
      Ij[j] = make_si(kl.mass[j], c, Rj, kl.inertia[j]);
      // contact detection for this link's spheres (needs only a_j', o_j' for j' <= j, already in LDS)
      const int sb = sel4(SL.b, l);
      const int se = sel4(SL.e, l);
      // mirrored quads: each lane walks only the leg's spheres its quad detects, the highest first, so the quads' spheres
      // of one link are handled in the same round (the wave runs max-over-lanes rounds per link, not one per sphere of
      // the link: with support-table lookups every round is a memory round trip); one quad per env: every sphere
      const uint64_t legm = (se >= 64 ? ~0ull : (1ull << se) - 1ull) & ~((1ull << sb) - 1ull);
      uint64_t walk = MIRROR > 1 ? (odet & legm) : legm;
      while (walk) {
        const int s = 63 - __builtin_clzll(walk);
        walk &= ~(1ull << s);
        const int raw = M.slink_raw(s);
        if ((raw & 0xff) == j) {
          const float4 sp = M.sph4(s);
          const V3 x = o + mul(Rj, v3(sp.x, sp.y, sp.z));
          V3 xc = x;
          float rad = sp.w;
          const int h = (raw >> 8) - 1;
          if (h >= 0) {  // a support-table collider: its support point towards the ground (world -z, in the link frame;
                         // on the terrain mesh the triangle query then takes that point with radius 0)
            xc = o + mul(Rj, hull_support(K, h, -1.f * mulT(Rj, Rz)));
            rad = 0.f;
          }
          detect(s, x, xc, rad, l, j, aa, oo);
        }
      }
      Rp = Rj;
      op = o;
    }
    const SI Ic2 = Ij[2], Ic1 = siadd(Ij[1], Ic2), Ic0 = siadd(Ij[0], Ic1);
    Aleg = Ic0;
    const SV F0 = simul(Ic0, S[0]), F1 = simul(Ic1, S[1]), F2 = simul(Ic2, S[2]);
    float D[6] = {sdot(S[0], F0), sdot(S[1], F1), sdot(S[2], F2), sdot(S[0], F1), sdot(S[0], F2), sdot(S[1], F2)};
    float Di[6];
    sym3inv(D, Di);
#pragma unroll
    for (int k = 0; k < 6; ++k) M.leg(l, 36 + k) = Di[k];
    float Kl[3][6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      float b0 = sv_get(F0, r), b1 = sv_get(F1, r), b2 = sv_get(F2, r);
      Kl[0][r] = Di[0] * b0 + Di[3] * b1 + Di[4] * b2;
      Kl[1][r] = Di[3] * b0 + Di[1] * b1 + Di[5] * b2;
      Kl[2][r] = Di[4] * b0 + Di[5] * b1 + Di[2] * b2;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 6; ++r) M.leg(l, 18 + 6 * j + r) = Kl[j][r];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c <= r; ++c)
        Sch[LI(r, c)] -= sv_get(F0, r) * Kl[0][c] + sv_get(F1, r) * Kl[1][c] + sv_get(F2, r) * Kl[2][c];
    // RNEA (qdd = 0): velocity-product and gravity forces
    SV vj = v0, aj = a0, f[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const SV sq = scale(S[j], st.qd[j]);
      vj = vj + sq;
      aj = aj + crm(vj, sq);
      f[j] = simul(Ij[j], aj) + crf(vj, simul(Ij[j], vj));
    }
    const SV Fc2 = f[2], Fc1 = f[1] + Fc2, Fc0 = f[0] + Fc1;
    M.leg(l, 42) = sdot(S[0], Fc0);
    M.leg(l, 43) = sdot(S[1], Fc1);
    M.leg(l, 44) = sdot(S[2], Fc2);
    // the sub-step-start joint rates, for the self-contact restitution test of the other lanes (overwritten by q0
    // when the contact solve starts)
    M.leg(l, 45) = st.qd[0];
    M.leg(l, 46) = st.qd[1];
    M.leg(l, 47) = st.qd[2];
    Cleg = Fc0;
  }
  if constexpr (TERR) {  // terrain queries of the recorded spheres (the leg frames are in LDS now)
#ifdef LRL_ENV_PROFILE
    const unsigned long long tq0 = clock64();
#endif
    // The workgroup's candidate (env slot, sphere) pairs are dealt over all its lanes, so the wave runs
    // ceil(total / BLOCK) queries instead of the most any one lane recorded (4.6 per lane and step on average
    // under random actions, a few times that for the busiest lane): each lane publishes its candidate mask and
    // the exclusive prefix of the counts; item j goes to lane j % BLOCK, which finds the owner lane (the last
    // one whose prefix is <= j) and the owner's sphere, queries it, and leaves the separation in the row's field
    // 9 (and the world normal in 3..5 when in contact) of the owner's env slot.  The owners then activate their
    // own contacts (the activation reads the owner's leg rates).  Same queries, same results.
    {
      const int lane = threadIdx.x;
      // the query's own max-height test (terrain_query: a sphere more than r + offset above its cell's max height is
      // clear) applied to the owner's first CF candidates before they enter the work list, so the wave deals fewer
      // queries; every load of the test issued at once (one memory round trip).  Same test, same cells: the dropped
      // spheres are the ones whose query would have ended there (their row fields are never read: not in contact)
      {
        constexpr int CF = 8;
        const float bs = K->p.border_size, ih = K->terr_inv_hs;
        const int R = K->terr_rows, Cn = K->terr_cols;
        int cs[CF];
        float cz[CF], hm[CF];
        uint64_t m = cand;
#pragma unroll
        for (int k = 0; k < CF; ++k) {
          cs[k] = m ? __builtin_ctzll(m) : -1;
          m &= m - 1ull;
        }
#pragma unroll
        for (int k = 0; k < CF; ++k) {
          const int sk = cs[k] < 0 ? 0 : cs[k];
          const float px = M.sph(sk, 6), py = M.sph(sk, 7);
          cz[k] = M.sph(sk, 8) - M.qrad(sk) - P.contact_offset;
          const int ci = min(max((int)floorf((px + bs) * ih), 0), R - 2);
          const int cj = min(max((int)floorf((py + bs) * ih), 0), Cn - 2);
          hm[k] = cs[k] < 0 ? 3.0e38f : K->terr_hmax[ci * Cn + cj];
        }
#pragma unroll
        for (int k = 0; k < CF; ++k)
          if (cs[k] >= 0 && cz[k] > hm[k]) cand &= ~(1ull << cs[k]);
      }
      const int cnt = __popcll(cand);
      int inc = cnt;
#pragma unroll
      for (int d = 1; d < BLOCK; d <<= 1) {
        const int v = __shfl_up(inc, d, BLOCK);
        if (lane >= d) inc += v;
      }
      const int total = __shfl(inc, BLOCK - 1, BLOCK);
      uint64_t* wl_mask = reinterpret_cast<uint64_t*>(M.wlist());
      int* wl_off = reinterpret_cast<int*>(wl_mask + BLOCK);
      uint64_t* wl_hit = reinterpret_cast<uint64_t*>(wl_off + BLOCK);  // candidates found in contact, per owner lane
      wl_mask[lane] = cand;
      wl_off[lane] = inc - cnt;
      wl_hit[lane] = 0ull;
      __syncthreads();
#ifdef LRL_ENV_PROFILE
      prof[22] += clock64() - tq0;  // scan + work-list publication
#endif
      float4* tv = reinterpret_cast<float4*>(M.base + (M.sph_off + K->num_spheres * NSF) * ENVS);
      // item j -> (owner lane L, sphere s): the last lane whose prefix is <= j, then the owner's (j - prefix)-th set bit.
      // Located one round ahead: round r + 1's chain of dependent LDS reads runs under round r's query
      auto locate = [&](int j, int& L, int& s) {
        L = 0;
#pragma unroll
        for (int step = BLOCK / 2; step; step >>= 1)
          if (wl_off[L + step] <= j) L += step;
        uint64_t mk = wl_mask[L];
        for (int q = j - wl_off[L]; q > 0; --q) mk &= mk - 1ull;
        s = __builtin_ctzll(mk);
      };
      int Ln = 0, sn = 0;
      if (lane < total) locate(lane, Ln, sn);
      for (int j = lane; j - lane < total; j += BLOCK) {
        if (j < total) {
          const int L = Ln, s = sn;
          if (j + BLOCK < total) locate(j + BLOCK, Ln, sn);
          float* row = M.base + (M.sph_off + s * NSF) * ENVS + (L >> 2);
          const THit th = terrain_query(K, v3(row[6 * ENVS], row[7 * ENVS], row[8 * ENVS]), M.qrad(s),
                                        P.contact_offset, tv, lane, prof);
#ifdef LRL_ENV_PROFILE
          prof[20] += 1;  // query rounds of this lane (lane 0: the wave's rounds)
#endif
#ifdef LRL_ENV_DEBUG
          g_env_dbg[((size_t)(env_block() * ENVS + (L >> 2)) * 64 + s) * 8 + 1] = th.sep;
#endif
          row[9 * ENVS] = th.sep;
          if (th.sep < P.contact_offset) {
            row[3 * ENVS] = th.n.x;
            row[4 * ENVS] = th.n.y;
            row[5 * ENVS] = th.n.z;
            atomicOr(reinterpret_cast<unsigned long long*>(wl_hit + L), 1ull << s);
          }
        }
      }
      __syncthreads();
#ifdef LRL_ENV_PROFILE
      const unsigned long long ta0 = clock64();
#endif
      // the owners activate only their candidates found in contact (the wave walks max-over-lanes contacts, not
      // max-over-lanes candidates)
      for (uint64_t m = wl_hit[lane]; m;) {
        const int s = __builtin_ctzll(m);
        m &= m - 1ull;
        // (contact point: the centre, or a support-table collider's support point, as the detection left it)
        activate(s, v3(M.sph(s, SF_G), M.sph(s, SF_G + 1), M.sph(s, SF_G + 2)), sph_leg_of(SL, s), M.slink(s), M.sph(s, 9),
                 mulT(R, v3(M.sph(s, 3), M.sph(s, 4), M.sph(s, 5))));
      }
#ifdef LRL_ENV_PROFILE
      prof[23] += clock64() - ta0;  // activation of the contacts
#endif
#ifdef LRL_ENV_PROFILE
      prof[15] += cnt;
#endif
    }
#ifdef LRL_ENV_PROFILE
    prof[14] += clock64() - tq0;  // terrain queries (part of kin+dyn+detect)
#endif
  }
  // joint limits of this lane's leg (after the terrain queries: on the mesh the rows alias their vertex blocks)
  if (P.joint_limits) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float sh = st.hi[j] - st.q[j], sl = st.q[j] - st.lo[j];
      const bool up = sh < sl;
      const float sep = up ? sh : sl;
      if (sep < P.joint_limit_margin + 2.f * dt * fabsf(st.qd[j])) {
        active |= 1ull << (M.nsph + 3 * ql + j);
        float* const row = M.lm(3 * ql + j);
        row[LIM_SG * ENVS] = up ? -1.f : 1.f;
        row[LIM_B * ENVS] =
            tgs ? sep : (sep >= 0.f ? -sep * idt : fminf(-P.baumgarte * sep * idt, P.max_depenetration_velocity));
      }
    }
  }
  // ---- quad reductions: legs -> base ----
#pragma unroll
  for (int k = 0; k < 21; ++k) Sch[k] = quad_sum(Sch[k]);
  A.m += quad_sum(Aleg.m);
  A.h = A.h + v3(quad_sum(Aleg.h.x), quad_sum(Aleg.h.y), quad_sum(Aleg.h.z));
#pragma unroll
  for (int k = 0; k < 6; ++k) A.i[k] += quad_sum(Aleg.i[k]);
  Cb = Cb + SV{v3(quad_sum(Cleg.a.x), quad_sum(Cleg.a.y), quad_sum(Cleg.a.z)),
               v3(quad_sum(Cleg.l.x), quad_sum(Cleg.l.y), quad_sum(Cleg.l.z))};
  active = env_or(active);
  if constexpr (MIRROR > 1) __syncthreads();  // sphere centres / targets of the other quads' detections
  LRL_PROF(0)  // kinematics, composite inertias, leg blocks, RNEA, contact detection
  // base block A (6x6) + Schur complement, Cholesky in registers
  Sch[LI(0, 0)] += A.i[0]; Sch[LI(1, 1)] += A.i[1]; Sch[LI(2, 2)] += A.i[2];
  Sch[LI(1, 0)] += A.i[3]; Sch[LI(2, 0)] += A.i[4]; Sch[LI(2, 1)] += A.i[5];
  Sch[LI(3, 1)] += A.h.z;  Sch[LI(3, 2)] -= A.h.y;
  Sch[LI(4, 0)] -= A.h.z;  Sch[LI(4, 2)] += A.h.x;
  Sch[LI(5, 0)] += A.h.y;  Sch[LI(5, 1)] -= A.h.x;
  Sch[LI(3, 3)] += A.m; Sch[LI(4, 4)] += A.m; Sch[LI(5, 5)] += A.m;
  chol6(Sch);
  chol_to_inverse6(Sch);  // Sch now holds S^-1
  // free acceleration: M acc = [0; tau] - C  (leg terms in the owner lane, summed over the quad)
  {
    float pb[6];
    {
      const int l = ql;
      const V3 rl = v3(tau3[0] - M.leg(l, 42), tau3[1] - M.leg(l, 43), tau3[2] - M.leg(l, 44));
#pragma unroll
      for (int r = 0; r < 6; ++r) pb[r] = -(M.Kx(l, 0, r) * rl.x + M.Kx(l, 1, r) * rl.y + M.Kx(l, 2, r) * rl.z);
      const V3 y = di_mul(M, l, rl);
      M.leg(l, 42) = y.x;  // reuse as y_l
      M.leg(l, 43) = y.y;
      M.leg(l, 44) = y.z;
    }
    {
      const float cbv[6] = {Cb.a.x, Cb.a.y, Cb.a.z, Cb.l.x, Cb.l.y, Cb.l.z};
#pragma unroll
      for (int r = 0; r < 6; ++r) pb[r] = quad_sum(pb[r]) - cbv[r];
    }
    float xb[6];
    sym6mul(Sch, pb, xb);
#pragma unroll
    for (int r = 0; r < 6; ++r) nu[r] += dt * xb[r];
    // this lane's leg (its own K and y_l rows: no other lane's data, no barrier)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float kx = 0.f;
#pragma unroll
      for (int r = 0; r < 6; ++r) kx += M.Kx(ql, j, r) * xb[r];
      nu[6 + j] += dt * (M.leg(ql, 42 + j) - kx);
    }
  }
  // self-collision detection here, after the Schur / free-acceleration arithmetic (the leg pass's LDS stores have
  // drained by now, so the gate's reads do not wait on them) and before the contact solve overwrites the sub-step-start
  // joint rates in leg fields 45..47
  uint64_t sown = 0;  // self-contact slots this lane detected (their rows are built here)
  if (P.self_collisions) {
#ifdef LRL_ENV_PROFILE
    const unsigned long long ts0 = clock64();
#endif
    // live groups of this lane: same leg and box always (the gate counted their hits), the legs above when the
    // bounding boxes (grown by contact_offset / 2) overlap — a culled pair is separated by more than the offset
    const SelfGate sg = self_gate(K, M, SL, ql, P.contact_offset);
    unsigned live = 1u | (K->box_h[0] >= 0.f ? 16u : 0u);
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      const V3 lo = v3(quad_bcast(sg.lo.x, l), quad_bcast(sg.lo.y, l), quad_bcast(sg.lo.z, l));
      const V3 hi = v3(quad_bcast(sg.hi.x, l), quad_bcast(sg.hi.y, l), quad_bcast(sg.hi.z, l));
      if (l > ql && aabb_overlap(sg.lo, sg.hi, lo, hi)) live |= 1u << (l - ql);
    }
    if (__any((int)(sg.hits > 0 || (live & 14u)))) {  // rare: the LDS pass over the live groups
      __syncthreads();  // sphere centres, joint frames and rates of the whole quad
      self_detect(K, M, SL, ql, live, dt, rest_s, active, sown);
      active = quad_or(active);
#ifdef LRL_ENV_PROFILE
      if constexpr (!TERR) prof[15] += 1;  // waves entering the LDS pass (per lane: summed over the wave's lanes)
#endif
    }
#ifdef LRL_ENV_PROFILE
    if constexpr (!TERR) prof[14] += clock64() - ts0;  // self-collision detection (part of schur+free acc)
#endif
  }
  LRL_PROF(1)  // Schur complement factor / inverse, free acceleration
  // contact solve.  Start state: v_b0 = free base velocity, qd0 = free joint rates (LDS), Y = 0.
  float vb0[6], vbc[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) vb0[r] = vbc[r] = nu[r];
  {  // owner lane: q0 = qd0 + K v_b0 and Y = 0 of its leg
    const int l = ql;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float k = 0.f;
#pragma unroll
      for (int r = 0; r < 6; ++r) k += M.Kx(l, j, r) * vb0[r];
      M.leg(l, 45 + j) = nu[6 + j] + k;
      M.leg(l, 48 + j) = 0.f;
      if constexpr (MIRROR > 1) M.leg(l, LF_DZ + j) = 0.f;
    }
  }
  // Delassus rows of the active spheres, each in the lane that owns the sphere (only spheres active in some
  // env of the wave are visited)
  // (each lane walks its own active spheres: the 4 legs' rows are built at the same time)
  for (uint64_t m = active & odet; __any((int)(m != 0ull));) {
    if (m) {
      const int s = __builtin_ctzll(m);
      m &= m - 1ull;
      if (s >= M.nsph)
        limit_setup(M, Sch, s - M.nsph, ql);
      else
        contact_setup<TERR>(M, Sch, R, s, sph_leg_of(SL, s), M.slink(s));
    }
  }
  // self-contact rows (owner lanes; rare: only waves with a detected pair enter)
  if (__any((int)(sown != 0ull)))
    for (uint64_t m = sown >> (M.nsph + LRL_NUM_DOF); m; m &= m - 1ull)
      self_setup(M, Sch, R, free_spheres(M, active), __builtin_ctzll(m));
  // (mirrored quads: the warm start below reads the z / e rows another quad's lanes just built — one LDS fence, as at the
  // leg pass's end, so no compiler reordering can move those reads above the builds)
  if constexpr (MIRROR > 1) __syncthreads();
  // warm start: spheres in contact in the previous sub-step keep their impulse (world frame); the owner
  // lanes apply them in parallel and the base-velocity changes are summed over the quad
  {
    float dvb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint64_t m = active & own & ~prev_active; m; m &= m - 1ull) {
      const int s = __builtin_ctzll(m);
      if (s >= M.nsph) {
        M.lm(s - M.nsph)[LIM_LAM * ENVS] = 0.f;
      } else {
        M.sph(s, 10) = 0.f;
        M.sph(s, 11) = 0.f;
        M.sph(s, 12) = 0.f;
      }
    }
    for (uint64_t m = active & own & prev_active; __any((int)(m != 0ull));) {
      if (m) {
        const int s = __builtin_ctzll(m);
        m &= m - 1ull;
        if (s >= M.nsph) {
          const int j = s - M.nsph - 3 * ql;
          limit_apply(M, s - M.nsph, ql, j == 0 ? st.llam[0] : j == 1 ? st.llam[1] : st.llam[2], dvb);
        } else {
          apply_impulse(M, s, sph_leg_of(SL, s), M.sph(s, 10), M.sph(s, 11), M.sph(s, 12), dvb);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) vbc[r] += quad_sum(dvb[r]);
  }
  __syncthreads();  // contact rows and leg accumulators of every owner lane are read by the whole quad
  LRL_PROF(2)  // Delassus rows + warm start
  float dxb[6];  // (TGS) the base's accumulated motion over the sub-step's sub-iterations
  // projected Gauss-Seidel, sphere order = model order (base, legs 0..3)
  // (each env walks its own active spheres in model order; the wave runs max-over-envs sphere updates,
  // not the union of the 16 envs' contact sets)
  {
    float vo0 = vbc[0], vo1 = vbc[4];
#pragma unroll
    for (int r = 1; r < 4; ++r) vo0 = ql == r ? vbc[r] : vo0;
    vo1 = ql == 1 ? vbc[5] : (ql == 0 ? vo1 : 0.f);
    const uint64_t sact = active >> (M.nsph + LRL_NUM_DOF);  // self-contact slots of the env
    const uint64_t cact = active & ~(sact << (M.nsph + LRL_NUM_DOF));
    const float h = dt / (float)(P.solver_iterations > 0 ? P.solver_iterations : 1);
    Tgs T{0.f, 0.f, frcp(h), P.baumgarte, P.max_depenetration_velocity};
    auto sweeps = [&](auto tgs_c) {
      constexpr bool TG = decltype(tgs_c)::value;
      for (int it = 0; it < P.solver_iterations; ++it) {
        for (uint64_t m = cact; __any((int)(m != 0ull));) {
          if (m) {
            const int s = __builtin_ctzll(m);
            m &= m - 1ull;
            if (s >= M.nsph)
              limit_pgs_q<TG>(M, s - M.nsph, ql, vo0, vo1, T);
            else
              contact_pgs_q<TG>(M, s, sph_leg_of(SL, s), mu, ql, vo0, vo1, T);
          }
        }
        if (__any((int)(sact != 0ull)))  // self-contact slots after the contacts and limits
          for (uint64_t m = sact; __any((int)(m != 0ull));) {
            if (m) {
              const int k = __builtin_ctzll(m);
              m &= m - 1ull;
              self_pgs_q(M, free_spheres(M, active), k, mu_s, ql, vo0, vo1);
            }
          }
        if constexpr (TG) {  // dx += h nu: lane q advances its share of dx_b and component q of every leg's dz
          T.dxo0 += h * vo0;
          T.dxo1 += h * vo1;
          if (ql < 3) {
#pragma unroll
            for (int l = 0; l < 4; ++l) {
              float* const lg = M.lp(l) + ql * ENVS;
              lg[LF_DZ * ENVS] += h * (lg[45 * ENVS] + lg[48 * ENVS]);
            }
          }
        }
      }
    };
    if constexpr (MIRROR > 1) {
      if (tgs)
        sweeps(BoolC<true>{});
      else
        sweeps(BoolC<false>{});
    } else {
      sweeps(BoolC<false>{});
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      vbc[r] = quad_bcast(vo0, r);
      dxb[r] = quad_bcast(T.dxo0, r);
    }
    vbc[4] = quad_bcast(vo1, 0);
    vbc[5] = quad_bcast(vo1, 1);
    dxb[4] = quad_bcast(T.dxo1, 0);
    dxb[5] = quad_bcast(T.dxo1, 1);
  }
  __syncthreads();  // the leg accumulators each lane owned are read by the whole quad below
  if (P.joint_limits) {  // this leg's limit impulses, carried to the next sub-step in registers
#pragma unroll
    for (int j = 0; j < 3; ++j) st.llam[j] = M.lm(3 * ql + j)[LIM_LAM * ENVS] * M.lm(3 * ql + j)[LIM_SG * ENVS];
  }
  LRL_PROF(3)  // PGS iterations
  // materialise the lazily propagated joint rates of this lane's leg
#pragma unroll
  for (int r = 0; r < 6; ++r) nu[r] = vbc[r];
  {
    const V3 q = leg_qd(M, ql, vbc);
    nu[6] = q.x;
    nu[7] = q.y;
    nu[8] = q.z;
  }
  // semi-implicit integration (TGS: positions move by the accumulated motion dx — joints dz - K dx_b — and the
  // rotation by exp(dx_w); velocities end at the last sweep's either way)
  const V3 w = v3(nu[0], nu[1], nu[2]);
  float dq[4];
  if (tgs) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float k = 0.f;
#pragma unroll
      for (int r = 0; r < 6; ++r) k += M.Kx(ql, j, r) * dxb[r];
      st.qd[j] = nu[6 + j];
      st.q[j] += M.leg(ql, LF_DZ + j) - k;
    }
    const V3 dp = mul(R, v3(dxb[3], dxb[4], dxb[5]));
    st.pos[0] += dp.x;
    st.pos[1] += dp.y;
    st.pos[2] += dp.z;
    const float th = sqrtf(dxb[0] * dxb[0] + dxb[1] * dxb[1] + dxb[2] * dxb[2]);
    if (th > 1e-12f) {
      float sn, cs;
      sincosf(0.5f * th, &sn, &cs);
      const float k = sn * frcp(th);
      dq[0] = dxb[0] * k; dq[1] = dxb[1] * k; dq[2] = dxb[2] * k; dq[3] = cs;
    } else {
      dq[0] = 0.5f * dxb[0]; dq[1] = 0.5f * dxb[1]; dq[2] = 0.5f * dxb[2]; dq[3] = 1.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      st.qd[j] = nu[6 + j];
      st.q[j] += dt * st.qd[j];
    }
    const V3 vw = mul(R, v3(nu[3], nu[4], nu[5]));
    st.pos[0] += dt * vw.x;
    st.pos[1] += dt * vw.y;
    st.pos[2] += dt * vw.z;
    const float wn = sqrtf(dot(w, w)), th = wn * dt;
    if (th > 1e-12f) {
      float sn, cs;
      sincosf(0.5f * th, &sn, &cs);
      const float k = sn * frcp(wn);
      dq[0] = w.x * k; dq[1] = w.y * k; dq[2] = w.z * k; dq[3] = cs;
    } else {
      dq[0] = 0.5f * dt * w.x; dq[1] = 0.5f * dt * w.y; dq[2] = 0.5f * dt * w.z; dq[3] = 1.f;
    }
  }
  const float x1 = st.quat[0], y1 = st.quat[1], z1 = st.quat[2], w1 = st.quat[3];
  float nq[4] = {w1 * dq[0] + x1 * dq[3] + y1 * dq[2] - z1 * dq[1], w1 * dq[1] - x1 * dq[2] + y1 * dq[3] + z1 * dq[0],
                 w1 * dq[2] + x1 * dq[1] - y1 * dq[0] + z1 * dq[3], w1 * dq[3] - x1 * dq[0] - y1 * dq[1] - z1 * dq[2]};
  const float inv = rsqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) st.quat[k] = nq[k] * inv;
  const M3 R2 = quat_mat(st.quat[0], st.quat[1], st.quat[2], st.quat[3]);
  const V3 V = mul(R2, v3(nu[3], nu[4], nu[5]) + cross(w, cb)), Wv = mul(R2, w);
  st.V[0] = V.x; st.V[1] = V.y; st.V[2] = V.z;
  st.W[0] = Wv.x; st.W[1] = Wv.y; st.W[2] = Wv.z;
  LRL_PROF(4)  // integration
}

// ------------------------------------------------------------------------------------------------
// post-physics helpers: torch op order, no contraction
// ------------------------------------------------------------------------------------------------
#pragma clang fp contract(off)
__device__ __forceinline__ float act_scaled(const lrl_env_params& P, const float* act, int j) {
  float as = act[j] * P.action_scale;
  if (j % 3 == 0) as = as * P.hip_scale_reduction;  // hip columns 0,3,6,9 (legged_robot.py:666)
  return as;
}
__device__ __forceinline__ float pos_target(const lrl_env_params& P, const float* act, int j) {
  return act_scaled(P, act, j) + P.default_dof_pos[j];
}
__device__ __forceinline__ V3 quat_rotate_inverse(const float* q, V3 v) {
  float w = q[3];
  float s = 2.0f * (w * w) - 1.0f;
  V3 a = v3(v.x * s, v.y * s, v.z * s);
  V3 c = v3(q[1] * v.z - q[2] * v.y, q[2] * v.x - q[0] * v.z, q[0] * v.y - q[1] * v.x);
  V3 b = v3(c.x * w * 2.0f, c.y * w * 2.0f, c.z * w * 2.0f);
  float d = q[0] * v.x + q[1] * v.y + q[2] * v.z;
  V3 e = v3(q[0] * d * 2.0f, q[1] * d * 2.0f, q[2] * d * 2.0f);
  return v3(a.x - b.x + e.x, a.y - b.y + e.y, a.z - b.z + e.z);
}
__device__ __forceinline__ float sq(float x) { return x * x; }
__device__ __forceinline__ float nrm3(float x, float y, float z) { return sqrtf(x * x + y * y + z * z); }

// _get_heights for scan point k (legged_robot.py:1469-1503, quat_apply_yaw math_utils.py:12-16), in torch's
// float32 op order: yaw-only quaternion normalised, rotated point + root position, + border, / horizontal
// scale, truncation, clip to the sample grid, min of three samples (already in metres)
__device__ __forceinline__ float height_sample(const KParams* __restrict__ K, const float* pos, const float* quat, int k) {
  const lrl_env_params& P = K->p;
  if (!P.terrain_mesh) return 0.f;  // plane: zeros (:1482-1483)
  const float qz = quat[2], qw = quat[3];
  const float nrm = fmaxf(sqrtf(qz * qz + qw * qw), 1e-9f);
  const float z = qz / nrm, w = qw / nrm;
  const float px = P.height_points[k][0], py = P.height_points[k][1];
  const float t0 = (0.f * 0.f - z * py) * 2.f, t1 = (z * px - 0.f * 0.f) * 2.f;
  const float rx = (px + w * t0) + (0.f * 0.f - z * t1);
  const float ry = (py + w * t1) + (z * t0 - 0.f * 0.f);
  float x = rx + pos[0], y = ry + pos[1];
  x = (x + P.border_size) / P.horizontal_scale;
  y = (y + P.border_size) / P.horizontal_scale;
  const int R = K->terr_rows, Cn = K->terr_cols;
  const int ix = min(max((int)x, 0), R - 2), iy = min(max((int)y, 0), Cn - 2);
  const float* __restrict__ H = K->terr_h;
  return fminf(fminf(H[ix * Cn + iy], H[(ix + 1) * Cn + iy]), H[ix * Cn + iy + 1]);
}

// ------------------------------------------------------------------------------------------------
// the fused step kernel
// ------------------------------------------------------------------------------------------------
// compute_observations (legged_robot.py:342-417) in two parts: the row's values — obs_base_values writes its base
// entries ([lin vel, ang vel,] gravity, [commands]), the step kernel's quads write the dof positions / velocities and the
// actions after them (each lane its leg's joints) — then obs_noise_clip adds U[-1,1] x noise_vec from the counter RNG
// keyed by (env, step counter, 4-entry chunk) and clips, for chunks c0, c0 + cstep, ... (the step kernel spreads the
// chunks over an env's lanes; a re-evaluation after a reset draws the same noise)
__device__ __forceinline__ void obs_base_values(const lrl_env_params& P, V3 blv, V3 bav, V3 pg, const float* cmd,
                                                float* ob) {
  int o = 0;
  if (P.observe_vel) {
    ob[o++] = blv.x * P.obs_scale_lin_vel; ob[o++] = blv.y * P.obs_scale_lin_vel; ob[o++] = blv.z * P.obs_scale_lin_vel;
    ob[o++] = bav.x * P.obs_scale_ang_vel; ob[o++] = bav.y * P.obs_scale_ang_vel; ob[o++] = bav.z * P.obs_scale_ang_vel;
  }
  ob[o++] = pg.x; ob[o++] = pg.y; ob[o++] = pg.z;
  if (P.observe_command) {
#pragma unroll
    for (int k = 0; k < 3; ++k) ob[o++] = cmd[k] * P.commands_scale[k];
  }
}
__device__ __forceinline__ void obs_noise_clip(const lrl_env_params& P, const KState& S, int e, uint64_t genv,
                                               int64_t step_counter, bool inject, float* ob, int c0, int cstep) {
  const int NO = P.num_obs;
  for (int i0 = 4 * c0; i0 < NO; i0 += 4 * cstep) {
    if (P.add_noise) {
      lrl_u32x4 r = lrl_philox((uint32_t)genv, (uint32_t)step_counter,
                               (LRL_RNG_OBS_NOISE << 16) ^ (uint32_t)(step_counter >> 32), (uint32_t)(i0 >> 2), S.seed);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int i = i0 + k;
        if (i < NO) {
          // (padded env slots e >= n read no injected row: the injected buffers hold n rows)
          float u = inject ? (e < S.n ? S.inj_noise[(size_t)e * NO + i] : 0.5f) : lrl_u01(r.v[k]);
          ob[i] += (2.f * u - 1.f) * P.noise_vec[i];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k < NO) ob[i0 + k] = fminf(fmaxf(ob[i0 + k], -P.clip_obs), P.clip_obs);
  }
}
__device__ __forceinline__ void priv_row(const lrl_env_params& P, const KState& S, int e, float payload, V3 cb,
                                         const float* ms, float* pr) {
  pr[0] = (S.friction[e] - P.priv_shift[0]) * P.priv_scale[0];
  pr[1] = (S.restitution[e] - P.priv_shift[1]) * P.priv_scale[1];
  pr[2] = (payload - P.priv_shift[2]) * P.priv_scale[2];
  pr[3] = (cb.x - P.priv_shift[3]) * P.priv_scale[3];
  pr[4] = (cb.y - P.priv_shift[3]) * P.priv_scale[3];
  pr[5] = (cb.z - P.priv_shift[3]) * P.priv_scale[3];
#pragma unroll
  for (int j = 0; j < 12; ++j) pr[6 + j] = (ms[j] - P.priv_shift[4]) * P.priv_scale[4];
#pragma unroll
  for (int i = 0; i < LRL_NUM_PRIV; ++i) pr[i] = fminf(fmaxf(pr[i], -P.clip_obs), P.clip_obs);
}

template <bool TERR>
__global__ __launch_bounds__(BLOCK) void env_step_kernel(const KParams* __restrict__ K, KState S,
                                                        const float* __restrict__ actions_in, uint32_t flags,
                                                        int64_t step_counter) {
#ifdef LRL_ENV_PROFILE
  const unsigned long long kt0 = clock64();
#endif
  extern __shared__ float lds[];
  const lrl_env_params& P = K->p;
  const int lane = threadIdx.x;
#ifdef LRL_ENV_SLOT_REV  // (determinism probe build: env slots in reverse lane order)
  const int es = ENVS - 1 - lane / (QL * MIRROR), ql = lane & 3;
#else
  const int es = lane / (QL * MIRROR), ql = lane & 3;  // env slot, owned leg
#endif
  const int blk = env_block();
  const int e = blk * ENVS + es;
  const int N = S.stride;
  const bool valid = e < S.n;
  const uint64_t genv = (uint64_t)(S.env_offset + e);

  Body st;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    st.pos[k] = S.root[k * N + e];
    st.V[k] = S.root[(7 + k) * N + e];
    st.W[k] = S.root[(10 + k) * N + e];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) st.quat[k] = S.root[(3 + k) * N + e];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    st.q[j] = S.dof_pos[(3 * ql + j) * N + e];
    st.qd[j] = S.dof_vel[(3 * ql + j) * N + e];
    st.lo[j] = K->dof_lo[3 * ql + j];
    st.hi[j] = K->dof_hi[3 * ql + j];
    st.llam[j] = 0.f;
  }
  float act[12];
  {
    const float c = P.clip_actions;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      float a = valid ? actions_in[(size_t)e * 12 + j] : 0.f;
      act[j] = fminf(fmaxf(a, -c), c);
    }
  }
  // per-env inputs read before the LDS staging barrier below, so their memory latency overlaps the table copy
  const int ctl = P.control_type;
  const float payload = S.payload[e];
  const V3 cb = v3(S.com[e], S.com[N + e], S.com[2 * N + e]);
  const float fr_e = S.friction[e], rs_e = S.restitution[e];
  float kpf3[3], kdf3[3], ms3[3], lqd3[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int jj = 3 * ql + j;
    kpf3[j] = S.kp[jj * N + e];
    kdf3[j] = S.kd[jj * N + e];
    ms3[j] = S.motor_strength[jj * N + e];
    lqd3[j] = ctl == 1 ? S.last_dof_vel[jj * N + e] : 0.f;
  }
  // leg blocks first, then the contact rows, (terrain: the query's vertex block), then the model tables
  const int nsph = K->num_spheres;
  static_assert(LRL_NUM_DOF * LIMF * ENVS <= 64 * BLOCK, "joint-limit rows must fit the terrain vertex blocks");
  float* const ktab = lds + (4 * LEGF + nsph * NSF) * ENVS + (TERR ? 64 * BLOCK : LRL_NUM_DOF * LIMF * ENVS);
  const Lds M{lds, 4 * LEGF, es, ktab, nsph, 4 * LEGF + nsph * NSF,
              ktab + ((4 * KLEGF + 5 * nsph + 40 + K->self_npairs + 1) & ~1)};
  {
    const float* src = reinterpret_cast<const float*>(K->leg);
    for (int i = lane; i < 4 * KLEGF; i += BLOCK) M.ktab[i] = src[i];
    float4* s4 = reinterpret_cast<float4*>(M.ktab + 4 * KLEGF);
    int* sl = reinterpret_cast<int*>(M.ktab + 4 * KLEGF + 4 * nsph);
    for (int s = lane; s < nsph; s += BLOCK) {
      s4[s] = make_float4(K->sph_pos[s][0], K->sph_pos[s][1], K->sph_pos[s][2], K->sph_rad[s]);
      sl[s] = (K->sph_link[s] & 0xff) | ((K->sph_hull[s] + 1) << 8);  // (base: link byte 0xff = -1, no table)
    }
    if (P.self_collisions) {
      int* sg = sl + nsph;
      const int* kg = &K->self_grp[0][0][0];
      for (int i = lane; i < 40; i += BLOCK) sg[i] = kg[i];
      uint32_t* sp = reinterpret_cast<uint32_t*>(sg + 40);
      for (int i = lane; i < K->self_npairs; i += BLOCK) sp[i] = K->self_pair[i];
    }
    __syncthreads();
  }
  const float mb = K->base_mass + payload;
  float Ib[6];
  {
    float sc = mb / K->base_mass;  // recomputeInertia: inertia scales with the new mass
#pragma unroll
    for (int k = 0; k < 6; ++k) Ib[k] = K->base_inertia[k] * sc;
  }
  const float mu = 0.5f * (fr_e + P.ground_friction);
  const float rest = 0.5f * (rs_e + P.ground_restitution);
  // self-contacts: both shapes carry the env's robot material, so PhysX's average combine is that material
  const float mu_s = fr_e, rest_s = rs_e;
  const bool physics = flags & LRL_STEP_PHYSICS;
  uint64_t active = 0;
  uint64_t own = 0;  // spheres whose detection / Delassus rows / warm start this lane owns
  for (int s = 0; s < K->num_spheres; ++s)
    if (sph_owner(K, s) == ql) own |= 1ull << s;
  own |= 7ull << (nsph + 3 * ql);  // this leg's joint-limit rows
  const uint64_t odet = own_split(own, mirror_quad());  // of those, the ones this quad detects / builds rows for
  unsigned long long prof[24] = {};
  LRL_PROF_DECL
#ifdef LRL_ENV_PROFILE
  prof_t = kt0;
#endif
  LRL_PROF(5)  // kernel start: state loads, setup
  // _compute_torques (legged_robot.py:653-688) for this lane's leg: the gain / strength factors and the
  // position targets do not change over the sub-steps, so they are read once
  // 'P': kp3 / kd3 = gains x Kp / Kd factors, tg3 = position target; 'V': kp3 / kd3 = the bare gains, tg3 = the
  // scaled action (a velocity target), lqd3 = last_dof_vel (constant over the sub-steps: post_physics_step sets it);
  // 'T': tg3 = the scaled action (a torque)
  float kp3[3], kd3[3], tg3[3], lim3[3], tau3[3], act3[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int jj = 3 * ql + j;
    act3[j] = act[jj];  // (the clipped actions of this lane's joints: its share of the state write-back)
    const bool pos = ctl == 0;
    kp3[j] = pos ? P.p_gains[jj] * kpf3[j] : P.p_gains[jj];
    kd3[j] = pos ? P.d_gains[jj] * kdf3[j] : P.d_gains[jj];
    tg3[j] = pos ? pos_target(P, act, jj) : act_scaled(P, act, jj);
    lim3[j] = P.torque_limits[jj];
  }
  for (int sub = 0; sub < P.decimation; ++sub) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float t;
      if (ctl == 0) {
        t = kp3[j] * (tg3[j] - st.q[j]) - kd3[j] * st.qd[j];  // :669-671
      } else if (ctl == 1) {
        const float a = kp3[j] * (tg3[j] - st.qd[j]);  // :673-674, torch order: (d * (qd - lqd)) / sim_dt
        const float b = kd3[j] * (st.qd[j] - lqd3[j]);
        t = a - b / P.sim_dt;
      } else {
        t = tg3[j];  // :676
      }
      t = t * ms3[j];
      tau3[j] = fminf(fmaxf(t, -lim3[j]), lim3[j]);
    }
    LRL_PROF(8)  // PD torques
    if (physics) substep<TERR>(K, st, tau3, mb, Ib, cb, mu, rest, M, active, ql, own, odet, mu_s, rest_s, prof);
#ifdef LRL_ENV_PROFILE
    prof_t = clock64();
#endif
  }
#ifdef LRL_ENV_PROFILE
  prof_t = clock64();
#endif

  // the post-physics inputs, read before the contact pass so their latency hides under it
  float cmd[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) cmd[k] = S.commands[k * N + e];
  // the joint-indexed reward inputs of this lane's leg (the joint terms are summed over the quad, below)
  float la3[3], lqdp3[3], slo3[3], shi3[3], dvl3[3], ddp3[3], fat[4];
  uint8_t lc[4];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int jj = 3 * ql + j;
    la3[j] = S.last_actions[jj * N + e];
    lqdp3[j] = S.last_dof_vel[jj * N + e];
    slo3[j] = P.soft_dof_pos_lower[jj];
    shi3[j] = P.soft_dof_pos_upper[jj];
    dvl3[j] = P.dof_vel_limits[jj];
    ddp3[j] = P.default_dof_pos[jj];
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    fat[f] = S.feet_air_time[f * N + e];
    lc[f] = S.last_contacts[f * N + e];
  }
  // ---- contact forces per body (last sub-step) and the contact-derived signals ----
  int rst = 0;
  float collision = 0.f;
  float ff[4][3];
#pragma unroll
  for (int f = 0; f < 4; ++f) ff[f][0] = ff[f][1] = ff[f][2] = 0.f;
  const float inv_dt = 1.f / P.sim_dt;
  // bodies spread over the env's lanes, then OR / sums over them (each foot is one lane's body, so its force sums
  // exactly with zeros)
  for (int b = lane & (QL * MIRROR - 1); b < K->num_bodies; b += QL * MIRROR) {
    float fx = 0.f, fy = 0.f, fz = 0.f;
    if (physics) {
      for (int s = K->body_sph_begin[b]; s < K->body_sph_end[b]; ++s)
        if ((active >> s) & 1ull) {
          if constexpr (TERR) {  // impulse (n, t1, t2) in the sphere's contact frame -> world
            const V3 nw = v3(M.sph(s, 0), M.sph(s, 1), M.sph(s, 2));
            V3 t1, t2;
            contact_frame(nw, t1, t2);
            const float ln = M.sph(s, 10), l1 = M.sph(s, 11), l2 = M.sph(s, 12);
            fx += ln * nw.x + l1 * t1.x + l2 * t2.x;
            fy += ln * nw.y + l1 * t1.y + l2 * t2.y;
            fz += ln * nw.z + l1 * t1.z + l2 * t2.z;
          } else {
            fx += M.sph(s, 11);
            fy += M.sph(s, 12);
            fz += M.sph(s, 10);
          }
        }
      if (active >> (nsph + LRL_NUM_DOF)) {  // self-contacts: +impulse on body A, -impulse on body B (world frame)
        for (int k = 0; k < LRL_SELF_SLOTS; ++k)
          if ((active >> (nsph + LRL_NUM_DOF + k)) & 1ull) {
            const SRow row = self_row(M, free_spheres(M, active), k);
            const int ba = (int)row[SR_BA], bb = (int)row[SR_BB];
            if (ba != b && bb != b) continue;
            const float sg = ba == b ? 1.f : -1.f;
            const float l0 = row[SR_LAM], l1 = row[SR_LAM + 1], l2 = row[SR_LAM + 2];
            fx += sg * (l0 * row[SR_F] + l1 * row[SR_F + 3] + l2 * row[SR_F + 6]);
            fy += sg * (l0 * row[SR_F + 1] + l1 * row[SR_F + 4] + l2 * row[SR_F + 7]);
            fz += sg * (l0 * row[SR_F + 2] + l1 * row[SR_F + 5] + l2 * row[SR_F + 8]);
          }
      }
      fx *= inv_dt;
      fy *= inv_dt;
      fz *= inv_dt;
      S.contact[(3 * b) * N + e] = fx;
      S.contact[(3 * b + 1) * N + e] = fy;
      S.contact[(3 * b + 2) * N + e] = fz;
    } else {
      fx = S.contact[(3 * b) * N + e];
      fy = S.contact[(3 * b + 1) * N + e];
      fz = S.contact[(3 * b + 2) * N + e];
    }
    float n = nrm3(fx, fy, fz);
    if ((P.termination_mask >> b) & 1u) rst |= n > 1.0f;
    if ((P.penalised_mask >> b) & 1u) collision += n > 0.1f ? 1.f : 0.f;
    int fs = K->body_foot[b];
#pragma unroll
    for (int f = 0; f < 4; ++f)
      if (fs == f) { ff[f][0] = fx; ff[f][1] = fy; ff[f][2] = fz; }
  }
  rst = env_or((uint64_t)rst) != 0ull;
  collision = env_sum(collision);
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int c = 0; c < 3; ++c) ff[f][c] = env_sum(ff[f][c]);
  __syncthreads();  // LDS contact rows are dead from here on; the obs tile reuses them
  LRL_PROF(10)  // contact forces per body
  const int NO = P.num_obs;
  float* otile = lds;                    // [ENVS][NO]
  float* ptile = lds + ENVS * NO;        // [ENVS][18]
  // _teleport_robots (legged_robot.py:768-791), in every lane of the env (the height scan below needs it)
  if (P.teleport) {
    float th = P.teleport_thresh;
    float xo = (float)(int)(e < P.num_train_envs ? P.teleport_x_offset : P.teleport_x_offset_eval);
    if (st.pos[0] < th + xo) st.pos[0] += P.terrain_length * (float)(P.terrain_rows - 1);
    if (st.pos[0] > P.terrain_length * (float)P.terrain_rows - th + xo) st.pos[0] -= P.terrain_length * (float)(P.terrain_rows - 1);
    if (st.pos[1] < th) st.pos[1] += P.terrain_width * (float)(P.terrain_cols - 1);
    if (st.pos[1] > P.terrain_width * (float)P.terrain_cols - th) st.pos[1] -= P.terrain_width * (float)(P.terrain_cols - 1);
  }
  // _get_heights (legged_robot.py:1469-1503) after the teleport (:575-585): the scan points spread over the
  // env's 4 lanes, written to measured_heights and to the height entries of the obs row (:386-389)
  float hsum = 0.f;
  if (P.measure_heights) {
    const int NP = P.num_height_points, NB = NO - NP;
    float* orow = otile + es * NO + NB;
    for (int k = ql; k < NP; k += QL) {
      const float hk = height_sample(K, st.pos, st.quat, k);
      if (valid) S.heights[k * N + e] = hk;
      hsum += st.pos[2] - hk;
      orow[k] = fminf(fmaxf(st.pos[2] - 0.5f - hk, -1.f), 1.f) * P.obs_scale_height;
    }
    hsum = quad_sum(hsum);
  }
  // ---- post_physics_step ----
  // (every lane of the env: the base-frame velocities and the push feed the spread state write-back below)
  const int32_t eplen = S.episode_length[e] + 1;
  const float* quat = st.quat;
  const V3 blv = quat_rotate_inverse(quat, v3(st.V[0], st.V[1], st.V[2]));
  const V3 bav = quat_rotate_inverse(quat, v3(st.W[0], st.W[1], st.W[2]));
  const V3 pg = quat_rotate_inverse(quat, v3(0.f, 0.f, -1.f));
  const bool inject = flags & LRL_STEP_INJECT_UNIFORM;
  // _push_robots (legged_robot.py:757-766): after the base-frame velocities above, before the rewards; the pushed
  // root velocity is what root_states, the next step's physics and last_root_vel see
  if (P.push_robots && eplen % P.push_interval == 0) {
    float u0, u1;
    if (inject) {
      u0 = valid ? S.inj_push[(size_t)e * 2] : 0.5f;
      u1 = valid ? S.inj_push[(size_t)e * 2 + 1] : 0.5f;
    } else {
      lrl_u32x4 r = lrl_philox((uint32_t)genv, (uint32_t)step_counter, (LRL_RNG_PUSH << 16) ^ (uint32_t)(step_counter >> 32),
                               0, S.seed);
      u0 = lrl_u01(r.v[0]);
      u1 = lrl_u01(r.v[1]);
    }
    st.V[0] = P.push_span * u0 + P.push_lo;  // (upper - lower) * torch.rand + lower
    st.V[1] = P.push_span * u1 + P.push_lo;
  }
  // termination (legged_robot.py:190-202): the contact test above, the body height, and (upstream) the time-out
  if (P.use_terminal_body_height && st.pos[2] < P.terminal_body_height) rst = 1;
  // time-outs (legged_robot.py:196-198, commented out in the fork — Q2): upstream semantics only
  const int tout = (P.auto_reset && eplen > P.max_episode_length) ? 1 : 0;
  rst |= tout;
  // ---- the reward terms' values (:1506-1646), in every lane of the env ----
  // The terms over the 12 joints are summed from each lane's own leg (its 3 joints, in joint order) and then over the
  // quad ((leg 0 + leg 1) + (leg 2 + leg 3)): a quarter of the sequential form's work, and no 12-wide copies of the joint
  // state in every lane; the other terms are a few operations each, the same in every lane.  The lead lane then adds the
  // active terms in the configured order (below).
  float jt[10];  // torques, energy, energy expenditure, dof_vel, dof_acc, action_rate, dof_pos / dof_vel / torque limits,
                 // stand_still (before its command gate)
  {
#pragma unroll
    for (int k = 0; k < 10; ++k) jt[k] = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float tq = tau3[j], q = st.q[j], qd = st.qd[j];
      jt[0] += sq(tq);
      jt[1] += tq * qd;
      jt[2] += fmaxf(tq * qd, 0.f);
      jt[3] += sq(qd);
      jt[4] += sq((lqdp3[j] - qd) / P.dt);
      jt[5] += sq(la3[j] - act3[j]);
      float o = -fminf(q - slo3[j], 0.f);
      o += fmaxf(q - shi3[j], 0.f);
      jt[6] += o;
      jt[7] += fminf(fmaxf(fabsf(qd) - dvl3[j] * P.soft_dof_vel_limit, 0.f), 1.f);
      jt[8] += fmaxf(fabsf(tq) - lim3[j] * P.soft_torque_limit, 0.f);
      jt[9] += fabsf(q - ddp3[j]);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) jt[k] = quad_sum(jt[k]);
  }
  bool has_air = false;  // _reward_feet_air_time updates feet_air_time / last_contacts only when it is a term
  for (int t = 0; t < P.num_reward_terms; ++t) has_air |= P.reward_term[t] == LRL_R_FEET_AIR_TIME;
  float air = 0.f;
  if (has_air) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      int c = ff[f][2] > 1.0f;
      int filt = c || lc[f];
      lc[f] = (uint8_t)c;
      float first = (fat[f] > 0.f && filt) ? 1.f : 0.f;
      fat[f] = fat[f] + P.dt;
      air += (fat[f] - 0.5f) * first;
      if (filt) fat[f] = 0.f;
    }
  }
  const float cnorm = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]);
  // the observation row's values (compute_observations :342-417) into the LDS tile, spread over the env's quads: quad 0
  // the dof positions, 1 the dof velocities, 2 the actions (each lane its leg's 3 joints), quad 3's lead lane the base
  // entries; the same expressions, so the same values as one lane writing the row
  {
    float* ob = otile + es * NO;
    const int o = (P.observe_vel ? 6 : 0) + 3 + (P.observe_command ? 3 : 0);
    const int qi = mirror_quad();  // (one quad per env on the terrain mesh: it writes all four groups)
    if (MIRROR == 1 || qi == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) ob[o + 3 * ql + j] = (st.q[j] - ddp3[j]) * P.obs_scale_dof_pos;
    }
    if (MIRROR == 1 || qi == 1) {
#pragma unroll
      for (int j = 0; j < 3; ++j) ob[o + 12 + 3 * ql + j] = st.qd[j] * P.obs_scale_dof_vel;
    }
    if (MIRROR == 1 || qi == 2) {
#pragma unroll
      for (int j = 0; j < 3; ++j) ob[o + 24 + 3 * ql + j] = act3[j];
    }
    if ((MIRROR == 1 || qi == 3) && ql == 0) obs_base_values(P, blv, bav, pg, cmd, ob);
  }
  // post-physics rewards, observations and the per-env state write-back: lane 0 of each env (of its first quad)
  if (ql == 0 && mirror_quad() == 0) {
  float ms_e[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) ms_e[j] = S.motor_strength[j * N + e];
  if (P.rand_interval > 0 && eplen % P.rand_interval == 0) {
    int k = 0;
    lrl_u32x4 r = lrl_philox((uint32_t)genv, (uint32_t)step_counter, (LRL_RNG_DR << 16) ^ (uint32_t)(step_counter >> 32), 0,
                             S.seed);
    // the draw's words as scalars, selected by the runtime word index k (indexing r.v[k] directly would put the
    // array in scratch)
    const uint32_t w0 = r.v[0], w1 = r.v[1], w2 = r.v[2];
    auto word = [&](int i) { return i == 0 ? w0 : (i == 1 ? w1 : w2); };
    if (P.randomize_motor_strength) {
      float u = inject ? (valid ? S.inj_dr[e] : 0.5f) : lrl_u01(word(k));
      k++;
      // torch.rand * (max - min) + min: two float32 roundings, the span rounded from the python-float difference
      float v = u * P.dr_span[0] + P.motor_strength_range[0];
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        ms_e[j] = v;
        S.motor_strength[j * N + e] = v;
      }
    }
    if (P.randomize_kp) {
      float u = lrl_u01(word(k++));
      float v = u * P.dr_span[1] + P.kp_range[0];
#pragma unroll
      for (int j = 0; j < 12; ++j) S.kp[j * N + e] = v;
    }
    if (P.randomize_kd) {
      float u = lrl_u01(word(k++));
      float v = u * P.dr_span[2] + P.kd_range[0];
#pragma unroll
      for (int j = 0; j < 12; ++j) S.kd[j * N + e] = v;
    }
  }

  LRL_PROF(11)  // post-physics loads, teleport, DR redraw
  // rewards
  // per-term rewards go to an LDS row first (the contact rows are dead): no global traffic inside the term
  // loop, so the episode / command sum updates below can keep all their loads in flight at once
  float* rt = lds + ENVS * (NO + LRL_NUM_PRIV) + es * LRL_MAX_REWARD_TERMS;
  float rew = 0.f;
  for (int t = 0; t < P.num_reward_terms; ++t) {
    float r = 0.f;
    switch (P.reward_term[t]) {
      case LRL_R_LIN_VEL_Z: r = sq(blv.z); break;
      case LRL_R_ANG_VEL_XY: r = sq(bav.x) + sq(bav.y); break;
      case LRL_R_ORIENTATION: r = sq(pg.x) + sq(pg.y); break;
      case LRL_R_BASE_HEIGHT:  // mean(z - measured_heights) (:1518-1521); measured_heights = 0 without a scan
        r = sq((P.measure_heights ? hsum / (float)P.num_height_points : st.pos[2]) - P.base_height_target);
        break;
      case LRL_R_TORQUES: r = jt[0]; break;
      case LRL_R_ENERGY: r = jt[1]; break;
      case LRL_R_ENERGY_EXPENDITURE: r = jt[2]; break;
      case LRL_R_DOF_VEL: r = jt[3]; break;
      case LRL_R_DOF_ACC: r = jt[4]; break;
      case LRL_R_ACTION_RATE: r = jt[5]; break;
      case LRL_R_COLLISION: r = collision; break;
      case LRL_R_SURVIVAL: r = rst ? 0.f : 1.f; break;
      case LRL_R_DOF_POS_LIMITS: r = jt[6]; break;
      case LRL_R_DOF_VEL_LIMITS: r = jt[7]; break;
      case LRL_R_TORQUE_LIMITS: r = jt[8]; break;
      case LRL_R_TRACKING_LIN_VEL: {
        float err = sq(cmd[0] - blv.x) + sq(cmd[1] - blv.y);
        r = expf(-err / P.tracking_sigma);
      } break;
      case LRL_R_TRACKING_ANG_VEL: r = expf(-sq(cmd[2] - bav.z) / P.tracking_sigma_yaw); break;
      case LRL_R_FEET_AIR_TIME: r = air * (cnorm > 0.1f ? 1.f : 0.f); break;  // (feet state updated above)
      case LRL_R_STUMBLE:
#pragma unroll
        for (int f = 0; f < 4; ++f)
          if (sqrtf(ff[f][0] * ff[f][0] + ff[f][1] * ff[f][1]) > 5.f * fabsf(ff[f][2])) r = 1.f;
        break;
      case LRL_R_STAND_STILL: r = jt[9] * (cnorm < 0.1f ? 1.f : 0.f); break;
      case LRL_R_FEET_CONTACT_FORCES:
#pragma unroll
        for (int f = 0; f < 4; ++f) r += fmaxf(nrm3(ff[f][0], ff[f][1], ff[f][2]) - P.max_contact_force, 0.f);
        break;
      default: break;
    }
    r = r * P.reward_scale[t];
    rew += r;
    rt[t] = r;
  }
  {  // episode_sums / command_sums rows of the terms (distinct rows), 8 terms' loads in flight per batch
    const int nt = P.num_reward_terms;
    for (int t0 = 0; t0 < nt; t0 += 8) {
      // the batch's slots (scalar) and reward values (LDS) read up front and unconditionally (clamped index), so
      // the scalar and LDS reads share one wait instead of one lgkmcnt(0) per term
      int sl[8];
      float rv[8], ev[8], cv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = min(t0 + u, nt - 1);
        sl[u] = P.reward_slot[t];
        rv[u] = rt[t];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        ev[u] = S.episode_sums[sl[u] * N + e];
        cv[u] = S.command_sums[sl[u] * N + e];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (t0 + u < nt) {
          S.episode_sums[sl[u] * N + e] = ev[u] + rv[u];
          S.command_sums[sl[u] * N + e] = cv[u] + rv[u];
        }
      }
    }
  }
  if (P.only_positive_rewards) rew = fmaxf(rew, 0.f);
  {
    const int KS = P.num_sum_keys;
    const bool term = P.termination_scale != 0.f;
    const int ts = term ? P.termination_slot : KS;
    const float e_tot = S.episode_sums[KS * N + e];
    const float e_term = S.episode_sums[ts * N + e], c_term = S.command_sums[ts * N + e];
    float cx[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) cx[k] = S.command_sums[(KS + k) * N + e];
    S.episode_sums[KS * N + e] = e_tot + rew;
    if (term) {
      const float r = ((rst && !tout) ? 1.f : 0.f) * P.termination_scale;  // _reward_termination: reset & ~time_out
      rew += r;
      S.episode_sums[ts * N + e] = e_term + r;
      S.command_sums[ts * N + e] = c_term + r;
    }
    S.command_sums[(KS + 0) * N + e] = cx[0] + blv.x;
    S.command_sums[(KS + 1) * N + e] = cx[1] + bav.z;
    S.command_sums[(KS + 2) * N + e] = cx[2] + sq(blv.x - cmd[0]);
    S.command_sums[(KS + 3) * N + e] = cx[3] + sq(bav.z - cmd[2]);
    S.command_sums[(KS + 4) * N + e] = cx[4] + 1.f;
  }

  // observations / privileged observations -> LDS tiles [env slot][.]
  LRL_PROF(12)  // rewards, termination, episode / command sums
  priv_row(P, S, e, payload, cb, ms_e, ptile + es * LRL_NUM_PRIV);  // (the obs row's values: spread above)

  LRL_PROF(13)  // obs / priv rows
  // ---- write back the SoA state ----
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    S.feet_air_time[f * N + e] = fat[f];
    S.last_contacts[f * N + e] = lc[f];
  }
  S.episode_length[e] = eplen;
  S.reset[e] = (uint8_t)rst;
  S.time_out[e] = (uint8_t)tout;
  S.rew[e] = rew;
  }  // ql == 0
  // the joint-indexed state rows, from the lanes that hold them: lane ql writes its leg's 3 joints (the values the
  // quad broadcast gave the lead lane, bit for bit); with mirrored quads, quad qi takes field group qi
  {
    const int qi = mirror_quad();
    auto put3 = [&](float* f, const float* v) {
#pragma unroll
      for (int j = 0; j < 3; ++j) f[(3 * ql + j) * N + e] = v[j];
    };
    if (MIRROR == 1 || qi == 0) {
      put3(S.dof_pos, st.q);
      put3(S.dof_vel, st.qd);
    }
    if (MIRROR == 1 || qi == 1) {
      put3(S.torques, tau3);
      if (P.control_type == 0) put3(S.joint_pos_target, tg3);  // set by 'P' only (:669); tg3 = pos_target there
    }
    if (MIRROR == 1 || qi == 2) {
      put3(S.actions, act3);
      put3(S.last_actions, act3);
    }
    if (MIRROR == 1 || qi == 3) put3(S.last_dof_vel, st.qd);
  }
  // the base rows, spread over the env's lanes (lane k of the env writes field k; every lane holds the values)
  {
    constexpr int EL = QL * MIRROR;
    const int sl = lane & (EL - 1);
    auto sel3 = [](int k, float a, float b, float c) { return k == 0 ? a : (k == 1 ? b : c); };
    for (int k = sl; k < 13; k += EL) {  // root_states: pos, quat (xyzw), lin vel, ang vel
      const float v = k < 3 ? sel3(k, st.pos[0], st.pos[1], st.pos[2])
                    : k < 7 ? (k == 3 ? st.quat[0] : k == 4 ? st.quat[1] : k == 5 ? st.quat[2] : st.quat[3])
                    : k < 10 ? sel3(k - 7, st.V[0], st.V[1], st.V[2]) : sel3(k - 10, st.W[0], st.W[1], st.W[2]);
      S.root[k * N + e] = v;
    }
    for (int k = sl; k < 6; k += EL)
      S.last_root_vel[k * N + e] = k < 3 ? sel3(k, st.V[0], st.V[1], st.V[2]) : sel3(k - 3, st.W[0], st.W[1], st.W[2]);
    for (int k = sl; k < 9; k += EL) {
      const int c = k % 3;
      const float v = k < 3 ? sel3(c, blv.x, blv.y, blv.z) : k < 6 ? sel3(c, bav.x, bav.y, bav.z) : sel3(c, pg.x, pg.y, pg.z);
      float* f = k < 3 ? S.base_lin_vel : k < 6 ? S.base_ang_vel : S.projected_gravity;
      f[c * N + e] = v;
    }
  }
  // observation noise + clip, the row's 4-entry chunks spread over the env's lanes
  __syncthreads();
  obs_noise_clip(P, S, e, genv, step_counter, (flags & LRL_STEP_INJECT_UNIFORM) != 0, otile + es * NO,
                 lane & (QL * MIRROR - 1), QL * MIRROR);

  LRL_PROF(6)  // contact forces + post_physics_step + SoA write-back
  // ---- AoS tiles (obs, priv) and the history shift: coalesced over the wave's contiguous rows ----
  __syncthreads();
  const size_t row0 = (size_t)blk * ENVS;
  {
    float* og = S.obs + row0 * NO;
    for (int i = lane; i < ENVS * NO; i += BLOCK) og[i] = otile[i];
    float* pgp = S.priv + row0 * LRL_NUM_PRIV;
    for (int i = lane; i < ENVS * LRL_NUM_PRIV; i += BLOCK) pgp[i] = ptile[i];
  }
  if (flags & LRL_STEP_HISTORY) {
    // HistoryWrapper.step (history_wrapper.py:17-21): lrl_sim_step launched the shift of the older slots before this
    // kernel (shift_history_kernel, append 0); the newest slot is this step's obs row, from the tile
    const int H = K->num_history * NO;
    float* hg = S.hist + row0 * H + (H - NO);
    for (int i = lane; i < ENVS * NO; i += BLOCK) {
      const int r = i / NO, c = i - r * NO;
      hg[(size_t)r * H + c] = otile[i];
    }
  }
  LRL_PROF(7)  // obs / priv tiles + history shift
#ifdef LRL_ENV_PROFILE
  prof[9] = clock64() - kt0;  // the wave's whole lifetime (the phases above should sum to it)
  if (lane == 0)
    for (int i = 0; i < 24; ++i) atomicAdd(&g_env_prof[i], prof[i]);
#endif
}

}  // namespace LRL_ENV_NS
}  // namespace lrl

#ifdef LRL_ENV_FLAT_TU
// the plane build's entry points (lrl_env_flat.hip); lrl_launch_env_step & co. below dispatch to them
extern "C" int lrl_debug_env_profile_flat(unsigned long long* out, int reset) {
#ifdef LRL_ENV_PROFILE
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lrl::g_env_prof), sizeof(unsigned long long) * 24) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[24] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lrl::g_env_prof), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 24;
#else
  (void)out;
  (void)reset;
  return 0;
#endif
}

extern "C" hipError_t lrl_env_kernel_setup_flat(int lds_bytes) {
  return hipFuncSetAttribute((const void*)lrl::env_step_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             lds_bytes);
}

extern "C" hipError_t lrl_launch_env_step_flat(const KParams* K, const KState* S, int lds_bytes, const float* actions,
                                               uint32_t flags, int64_t step_counter, hipStream_t stream) {
  hipLaunchKernelGGL(lrl::env_step_kernel<false>, dim3(S->stride / ENVS), dim3(BLOCK), lds_bytes, stream, K, *S,
                     actions, flags, step_counter);
  return hipGetLastError();
}
#else
extern "C" int lrl_debug_env_profile_flat(unsigned long long* out, int reset);
extern "C" hipError_t lrl_env_kernel_setup_flat(int lds_bytes);
extern "C" hipError_t lrl_launch_env_step_flat(const KParams* K, const KState* S, int lds_bytes, const float* actions,
                                               uint32_t flags, int64_t step_counter, hipStream_t stream);

// the sum of the two builds' timers (a simulation runs one of them)
extern "C" int lrl_debug_env_profile(unsigned long long* out, int reset) {
#ifdef LRL_ENV_PROFILE
  unsigned long long f[24];
  if (lrl_debug_env_profile_flat(f, reset) != 24) return -2;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lrl::g_env_prof), sizeof(unsigned long long) * 24) != hipSuccess) return -2;
  for (int i = 0; i < 24; ++i) out[i] += f[i];
  if (reset) {
    unsigned long long z[24] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lrl::g_env_prof), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 24;
#else
  (void)out;
  (void)reset;
  return 0;
#endif
}

extern "C" int lrl_debug_env_buffer(float* buf) {
#ifdef LRL_ENV_DEBUG
  return hipMemcpyToSymbol(HIP_SYMBOL(lrl::g_env_dbg), &buf, sizeof(buf)) == hipSuccess ? 1 : -2;
#else
  (void)buf;
  return 0;
#endif
}

extern "C" hipError_t lrl_env_kernel_setup(int lds_bytes) {
  hipError_t e = lrl_env_kernel_setup_flat(lds_bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)lrl::env_step_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             lds_bytes);
}

namespace lrl {
inline namespace LRL_ENV_NS {
// compute_observations for envs just reset inside a step (upstream semantics, legged_robot.py:177-184):
// obs / priv rows from the post-reset state with the step's noise draws, the newest history slot, and the
// last_* buffers post_physics_step sets after the reset (last_actions = actions, last_dof_vel = dof_vel,
// last_root_vel = root velocity).  One thread per listed env.
// 16 lanes per env (OBS_LANES): lane c forms, noises, clips and stores only its 4-wide chunks of the observation row
// (chunk i0 / 4 on lane (i0 / 4) % 16: one Philox draw each instead of the whole row's draws on one thread), reading
// the state entries those need; lane 0 writes the base-frame velocities, the privileged row and the last_* buffers.
// Every element's value, draw and operation order are the step kernel's (obs_base_values + its quads' joint entries /
// obs_noise_clip), so the rows are bit-identical.
constexpr int OBS_LANES = 16;
// observation entry i of env e (the step kernel's layout: [lin vel, ang vel,] gravity, [commands,] dof pos, dof vel,
// actions, then the height rows against base height z)
__device__ __forceinline__ float obs_entry(const lrl_env_params& P, const KState& S, int e, int i, V3 blv, V3 bav,
                                           V3 pg) {
  const int N = S.stride;
  int o = 0;
  if (P.observe_vel) {
    if (i < 3) return (i == 0 ? blv.x : i == 1 ? blv.y : blv.z) * P.obs_scale_lin_vel;
    if (i < 6) return (i == 3 ? bav.x : i == 4 ? bav.y : bav.z) * P.obs_scale_ang_vel;
    o = 6;
  }
  if (i < o + 3) return i == o ? pg.x : i == o + 1 ? pg.y : pg.z;
  o += 3;
  if (P.observe_command) {
    if (i < o + 3) return S.commands[(i - o) * N + e] * P.commands_scale[i - o];
    o += 3;
  }
  if (i < o + 12) return (S.dof_pos[(i - o) * N + e] - P.default_dof_pos[i - o]) * P.obs_scale_dof_pos;
  if (i < o + 24) return S.dof_vel[(i - o - 12) * N + e] * P.obs_scale_dof_vel;
  if (i < o + 36) return S.actions[(i - o - 24) * N + e];
  const int k = i - (P.num_obs - P.num_height_points);  // height row k (measure_heights)
  return fminf(fmaxf(S.root[2 * N + e] - 0.5f - S.heights[k * N + e], -1.f), 1.f) * P.obs_scale_height;
}
__global__ __launch_bounds__(256) void observe_kernel(const KParams* __restrict__ K, KState S,
                                                      const int32_t* __restrict__ ids, int32_t n,
                                                      const int32_t* __restrict__ dn, uint32_t flags,
                                                      int64_t step_counter) {
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gt / OBS_LANES, c = gt % OBS_LANES;
  if (t >= (dn ? min(*dn, n) : n)) return;  // (dn: device count, n its bound)
  const int e = ids[t];
  if (e < 0 || e >= S.n) return;
  const lrl_env_params& P = K->p;
  const int N = S.stride, NO = P.num_obs;
  const uint64_t genv = (uint64_t)(S.env_offset + e);
  const bool inject = (flags & LRL_STEP_INJECT_UNIFORM) != 0;
  float quat[4], V[3], W[3];
#pragma unroll
  for (int k = 0; k < 4; ++k) quat[k] = S.root[(3 + k) * N + e];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    V[k] = S.root[(7 + k) * N + e];
    W[k] = S.root[(10 + k) * N + e];
  }
  const V3 blv = quat_rotate_inverse(quat, v3(V[0], V[1], V[2]));
  const V3 bav = quat_rotate_inverse(quat, v3(W[0], W[1], W[2]));
  const V3 pg = quat_rotate_inverse(quat, v3(0.f, 0.f, -1.f));
  float* row = S.obs + (size_t)e * NO;
  float* h = (flags & LRL_STEP_HISTORY) ? S.hist + (size_t)e * (K->num_history * NO) + (K->num_history - 1) * NO
                                        : nullptr;
  for (int i0 = 4 * c; i0 < NO; i0 += 4 * OBS_LANES) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i0 + k < NO ? obs_entry(P, S, e, i0 + k, blv, bav, pg) : 0.f;
    if (P.add_noise) {  // (obs_noise_clip's chunk i0 / 4)
      lrl_u32x4 r = lrl_philox((uint32_t)genv, (uint32_t)step_counter,
                               (LRL_RNG_OBS_NOISE << 16) ^ (uint32_t)(step_counter >> 32), (uint32_t)(i0 >> 2), S.seed);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = i0 + k;
        if (i < NO) {
          float u = inject ? (e < S.n ? S.inj_noise[(size_t)e * NO + i] : 0.5f) : lrl_u01(r.v[k]);
          v[k] += (2.f * u - 1.f) * P.noise_vec[i];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k < NO) {
        const float x = fminf(fmaxf(v[k], -P.clip_obs), P.clip_obs);
        row[i0 + k] = x;
        if (h) h[i0 + k] = x;
      }
  }
  if (c != 0) return;
  float ms[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) ms[j] = S.motor_strength[j * N + e];
  S.base_lin_vel[e] = blv.x; S.base_lin_vel[N + e] = blv.y; S.base_lin_vel[2 * N + e] = blv.z;
  S.base_ang_vel[e] = bav.x; S.base_ang_vel[N + e] = bav.y; S.base_ang_vel[2 * N + e] = bav.z;
  S.projected_gravity[e] = pg.x; S.projected_gravity[N + e] = pg.y; S.projected_gravity[2 * N + e] = pg.z;
  priv_row(P, S, e, S.payload[e], v3(S.com[e], S.com[N + e], S.com[2 * N + e]), ms, S.priv + (size_t)e * LRL_NUM_PRIV);
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    S.last_actions[j * N + e] = S.actions[j * N + e];
    S.last_dof_vel[j * N + e] = S.dof_vel[j * N + e];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    S.last_root_vel[k * N + e] = V[k];
    S.last_root_vel[(3 + k) * N + e] = W[k];
  }
}
}  // namespace LRL_ENV_NS
}  // namespace lrl

extern "C" hipError_t lrl_launch_env_step(const KParams* K, const KState* S, int lds_bytes, const float* actions,
                                          uint32_t flags, int64_t step_counter, int terrain_mesh, hipStream_t stream) {
  if (!terrain_mesh) return lrl_launch_env_step_flat(K, S, lds_bytes, actions, flags, step_counter, stream);
  hipLaunchKernelGGL(lrl::env_step_kernel<true>, dim3(S->stride / ENVS), dim3(BLOCK), lds_bytes, stream, K, *S,
                     actions, flags, step_counter);
  return hipGetLastError();
}

extern "C" hipError_t lrl_launch_observe(const KParams* K, const KState* S, const int32_t* ids, int32_t n,
                                         const int32_t* dn, uint32_t flags, int64_t step_counter, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lrl::observe_kernel, dim3((int)(((int64_t)n * lrl::OBS_LANES + 255) / 256)), dim3(256), 0, stream,
                     K, *S, ids, n, dn, flags, step_counter);
  return hipGetLastError();
}
#endif  // LRL_ENV_FLAT_TU
