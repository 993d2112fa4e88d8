// lrl_curriculum_dev.hip — the grid-adaptive command curriculum's per-resample work on the device, so the upstream
// env step (legacy_fork=False) never waits for the host: RewardThresholdCurriculum.update then .sample
// (mini_gym/envs/base/curriculum.py:56-68, 105-115) for the resampled envs, and _resample_commands' writes
// (legged_robot.py:595-626: commands[ids, :3], the |cmd_xy| > 0.2 mask, command_sums[:, ids] = 0, the env bins) — one
// workgroup, bit-exact with the host forms (lrl/curriculum.py numpy, csrc/lrl_curriculum.cpp):
//   * MT19937 exactly as numpy's RandomState, its 624-word key + position kept on the device (the host mirror is
//     refreshed on access: lrl/env.py);
//   * the update's clipped +0.2 adds (the listed bins once from their old values, then each centre's +-local_range
//     neighbourhood once per centre: a bin's adds are all the same clipped add, so only their count matters);
//   * RandomState.choice(p = w / w.sum()): numpy's pairwise sum, p = w / S, cdf = sequential cumsum, cdf /= cdf[-1]
//     (cached while the weights are unchanged), random_sample doubles, searchsorted(side='right');
//   * RandomState.uniform(low = c + half, high = c - half) per (env, axis) in C order: low + (high - low) * u.
// Every double operation is a separate IEEE operation (no contraction), as numpy evaluates them.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/lrl.h"
#include "lrl_kparams.h"

namespace lrl {

constexpr int CD_THREADS = 1024;
constexpr int MT_N = 624, MT_M = 397;

__device__ inline double clip01(double x) { return fmin(fmax(x, 0.0), 1.0); }

// numpy's pairwise summation (the add.reduce inner loop) of a contiguous float64 array of n elements: leaves of <= 128
// elements (8 interleaved partial sums, or a plain loop below 8), a node's sum = left + right with the split at
// n2 = n / 2 - (n / 2) % 8.  cd_walk visits the tree on one thread: mode 0 lists the leaves left to right (offsets,
// lengths; returns their count), mode 1 combines the leaf sums `val` (in that order) as the recursion does.
// (its stack lives in LDS: as a private array it was scratch memory, a global round trip per step of the walk)
struct CdStack {
  double res[32];
  int off[32], len[32], st[32];
};
__device__ double cd_walk(int n, int mode, int* leaf_off, int* leaf_len, const double* val, int* nleaves, CdStack& K) {
  double* res = K.res;
  int *off = K.off, *len = K.len, *st = K.st;
  int sp = 0, li = 0;
  off[0] = 0; len[0] = n; st[0] = 0;
  double ret = 0.0;
  while (sp >= 0) {
    const int o = off[sp], m = len[sp];
    if (m <= 128) {
      if (mode == 0) {
        leaf_off[li] = o;
        leaf_len[li] = m;
      } else {
        ret = val[li];
      }
      ++li;
      --sp;
      while (sp >= 0) {
        if (st[sp] == 1) {  // left subtree done: keep its sum, walk the right one
          res[sp] = ret;
          st[sp] = 2;
          int n2 = len[sp] / 2;
          n2 -= n2 % 8;
          ++sp;
          off[sp] = off[sp - 1] + n2;
          len[sp] = len[sp - 1] - n2;
          st[sp] = 0;
          break;
        }
        ret = res[sp] + ret;  // right subtree done: left + right
        --sp;
      }
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    st[sp] = 1;
    ++sp;
    off[sp] = o;
    len[sp] = n2;
    st[sp] = 0;
  }
  if (nleaves) *nleaves = li;
  return ret;
}

__device__ double cd_leaf(const double* a, int m) {
  if (m < 8) {
    double r = 0.0;
    for (int i = 0; i < m; ++i) r += a[i];
    return r;
  }
  double q[8];
  for (int j = 0; j < 8; ++j) q[j] = a[j];
  int i = 8;
  for (; i < m - (m % 8); i += 8)
    for (int j = 0; j < 8; ++j) q[j] += a[i + j];
  double r = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  for (; i < m; ++i) r += a[i];
  return r;
}

// The same pairwise sum, level by level: wave 0 lays the recursion out top-down (each level's nodes in LDS, a node of
// more than 128 elements splitting at n2 = n / 2 - (n / 2) % 8 into two children on the next level, placed by a ballot
// prefix count), every thread sums the leaves, wave 0 adds each internal node's left + right bottom-up.  The same
// leaves, the same adds in the same tree as cd_walk, without its serial chain of dependent LDS stack operations.
// Returns false (nothing written) when the tree exceeds CD_LV levels or CD_LN nodes on a level.
constexpr int CD_LV = 10, CD_LN = 128;
struct CdLevels {
  int off[CD_LV][CD_LN], len[CD_LV][CD_LN], child[CD_LV][CD_LN];
  double val[CD_LV][CD_LN];
  int cnt[CD_LV + 1];
  int ok, depth;
};
__device__ bool cd_pairwise_levels(const double* a, int n, CdLevels& T, double* out) {
  const int t = threadIdx.x, lane = t & 63;
  if (t == 0) {
    T.off[0][0] = 0;
    T.len[0][0] = n;
    T.cnt[0] = 1;
    T.ok = 1;
    T.depth = 0;
  }
  __syncthreads();
  if (t < 64) {
    for (int L = 0; L < CD_LV; ++L) {
      const int c = T.cnt[L];
      int base = 0;
      for (int i0 = 0; i0 < c; i0 += 64) {
        const int i = i0 + lane;
        const bool in = i < c;
        const int m = in ? T.len[L][i] : 0;
        const bool internal = in && m > 128;
        const uint64_t mask = __ballot(internal);
        const int rank = base + __popcll(mask & ((1ull << lane) - 1ull));
        if (in) T.child[L][i] = internal ? 2 * rank : -1;
        if (internal) {
          if (L + 1 >= CD_LV || 2 * rank + 1 >= CD_LN) {
            T.ok = 0;
          } else {
            int n2 = m / 2;
            n2 -= n2 % 8;
            const int o = T.off[L][i];
            T.off[L + 1][2 * rank] = o;
            T.len[L + 1][2 * rank] = n2;
            T.off[L + 1][2 * rank + 1] = o + n2;
            T.len[L + 1][2 * rank + 1] = m - n2;
          }
        }
        base += __popcll(mask);
      }
      if (lane == 0) {
        T.cnt[L + 1] = 2 * base;
        if (base == 0) T.depth = L + 1;
      }
      __builtin_amdgcn_wave_barrier();
      if (base == 0 || !T.ok) break;
    }
  }
  __syncthreads();
  if (!T.ok || T.depth == 0) return false;
  const int D = T.depth;
  for (int L = 0; L < D; ++L)
    for (int i = t; i < T.cnt[L]; i += blockDim.x)
      if (T.child[L][i] < 0) T.val[L][i] = cd_leaf(a + T.off[L][i], T.len[L][i]);
  __syncthreads();
  if (t < 64) {
    for (int L = D - 2; L >= 0; --L) {
      for (int i = lane; i < T.cnt[L]; i += 64) {
        const int ch = T.child[L][i];
        if (ch >= 0) T.val[L][i] = T.val[L + 1][ch] + T.val[L + 1][ch + 1];
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) *out = T.val[0][0];
  }
  __syncthreads();
  return true;
}

__device__ inline uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// one MT19937 twist of the key in LDS, by the workgroup: the sequential recurrence's dependencies split it into four
// phases (old words read before any write in each)
__device__ void mt_twist(uint32_t* k) {
  constexpr uint32_t A = 0x9908b0dfu, UP = 0x80000000u, LO = 0x7fffffffu;
  const int t = threadIdx.x;
  auto mix = [&](uint32_t hi, uint32_t lo, uint32_t src) {
    const uint32_t y = (hi & UP) | (lo & LO);
    return src ^ (y >> 1) ^ (-(y & 1u) & A);
  };
  // [0, 227): k[i + 397] old
  uint32_t v = 0;
  if (t < MT_N - MT_M) v = mix(k[t], k[t + 1], k[t + MT_M]);
  __syncthreads();
  if (t < MT_N - MT_M) k[t] = v;
  __syncthreads();
  // [227, 454): k[i - 227] new (phase one)
  if (t < 227) v = mix(k[227 + t], k[228 + t], k[t]);
  __syncthreads();
  if (t < 227) k[227 + t] = v;
  __syncthreads();
  // [454, 623): k[i - 227] new (phase two)
  if (t < 623 - 454) v = mix(k[454 + t], k[455 + t], k[227 + t]);
  __syncthreads();
  if (t < 623 - 454) k[454 + t] = v;
  __syncthreads();
  if (t == 0) k[623] = mix(k[623], k[0], k[MT_M - 1]);
  __syncthreads();
}

struct CurDevArgs {
  lrl_dev_curriculum c;
  KState S;
  int32_t n_cs;
  const int32_t* ids;
  int32_t nmax;
  const int32_t* dcount;
  float ep_len;
  int32_t row_lin, row_ang;
  float lin_thr, ang_thr;
  double local_range;
  int32_t update;
  int32_t log_area;  // reset_idx's resample: command_area = np.sum(weights) / nbins after the update (legged_robot.py:272)
};

constexpr int CD_MAX_LEAVES = 256;  // pairwise-sum leaves (>= nbins / 64)

__global__ __launch_bounds__(CD_THREADS) void curriculum_dev_kernel(CurDevArgs a) {
  extern __shared__ __attribute__((aligned(16))) double cd_lds[];
  const lrl_dev_curriculum& c = a.c;
  const int nb = c.nx * c.ny * c.nz;
  double* cdf = cd_lds;                                           // [nb] weights, then p, then the cdf
  int* counts = reinterpret_cast<int*>(cdf + nb);                 // [nb]
  int* last = counts + nb;                                        // [nb]
  uint32_t* key = reinterpret_cast<uint32_t*>(last + nb);         // [624]
  __shared__ int changed, posv, bad, nleaves;
  __shared__ int leaf_off[CD_MAX_LEAVES], leaf_len[CD_MAX_LEAVES];
  __shared__ double leaf_val[CD_MAX_LEAVES];
  __shared__ double Ssum;
  __shared__ CdStack cstack;
  __shared__ CdLevels clev;
  const int t = threadIdx.x;
  const int n = min(*a.dcount, a.nmax);
  if (n <= 0) {  // (resample_commands returns before touching the generator)
    if (a.log_area && c.env_bins_f_prev) {  // the step's fresh log buffers keep the last reset batch's values
      const int N0 = a.S.n;
      for (int e = t; e < N0; e += CD_THREADS) c.env_bins_f[e] = c.env_bins_f_prev[e];
      if (t == 0 && c.command_area_prev) c.command_area[0] = c.command_area_prev[0];
    }
    return;
  }
  const KState& S = a.S;
  const int N = S.stride;
  if (t == 0) changed = 0;
  auto rewards = [&](int i, int& e, int& b, float& lin, float& ang) {
    e = a.ids[i];
    b = (int)c.env_bins[e];
    lin = S.command_sums[(int64_t)a.row_lin * N + e] / a.ep_len;
    ang = S.command_sums[(int64_t)a.row_ang * N + e] / a.ep_len;
  };
  // ---- update (curriculum.py:105-115) ----
  if (a.update) {
    for (int b = t; b < nb; b += CD_THREADS) {
      counts[b] = 0;
      last[b] = -1;
    }
    __syncthreads();
    for (int i = t; i < n; i += CD_THREADS) atomicMax(&last[(int)c.env_bins[a.ids[i]]], i);
    __syncthreads();
    // episode_reward_*[bins] = rewards (the last duplicate wins, as a numpy fancy assignment); each centre's new value
    // from its old weight, parked in the draw scratch until every centre has read
    for (int i = t; i < n; i += CD_THREADS) {
      int e, b;
      float lin, ang;
      rewards(i, e, b, lin, ang);
      if (last[b] == i) {
        c.ep_rew_lin[b] = (double)lin;
        c.ep_rew_ang[b] = (double)ang;
      }
      const bool ok = lin > a.lin_thr && ang > a.ang_thr;
      c.draws[i] = ok ? clip01(c.weights[b] + 0.2) : -1.0;
    }
    __syncthreads();
    for (int i = t; i < n; i += CD_THREADS) {
      const double v = c.draws[i];
      if (v >= 0.0) {
        c.weights[(int)c.env_bins[a.ids[i]]] = v;  // (duplicates write the same value)
        changed = 1;
      }
    }
    // neighbourhood counts: per axis the grid values within +-local_range of the centre's (contiguous: monotone axes)
    const double* ax[3] = {c.axes, c.axes + c.nx, c.axes + c.nx + c.ny};
    const int len[3] = {c.nx, c.ny, c.nz};
    for (int i = t; i < n; i += CD_THREADS) {
      if (!(c.draws[i] >= 0.0)) continue;
      const int b = (int)c.env_bins[a.ids[i]];
      const int idx[3] = {b / (c.nz * c.ny), (b / c.nz) % c.ny, b % c.nz};
      int lo[3], hi[3];
      for (int d = 0; d < 3; ++d) {
        const double ce = ax[d][idx[d]], l = ce - a.local_range, h = ce + a.local_range;
        lo[d] = len[d];
        hi[d] = -1;
        for (int q = 0; q < len[d]; ++q)
          if (ax[d][q] >= l && ax[d][q] <= h) {
            lo[d] = min(lo[d], q);
            hi[d] = max(hi[d], q);
          }
      }
      for (int x = lo[0]; x <= hi[0]; ++x)
        for (int y = lo[1]; y <= hi[1]; ++y)
          for (int z = lo[2]; z <= hi[2]; ++z) atomicAdd(&counts[(x * c.ny + y) * c.nz + z], 1);
    }
    __syncthreads();
    for (int b = t; b < nb; b += CD_THREADS) {
      int k = counts[b];
      if (k == 0) continue;
      double w = c.weights[b];
      for (; k > 0 && w < 1.0; --k) w = clip01(w + 0.2);
      c.weights[b] = w;
    }
  }
  __syncthreads();
  // ---- np.sum(weights) (pairwise: leaves in parallel, the tree on one thread), for the cdf and the logged area ----
  const bool need_cdf = changed || c.state[0] == 0;
  if (need_cdf || a.log_area) {
    for (int b = t; b < nb; b += CD_THREADS) cdf[b] = c.weights[b];
    if (t == 0) bad = 0;
    __syncthreads();
    if (cd_pairwise_levels(cdf, nb, clev, &Ssum)) {
      if (t == 0) Ssum = 0.0 + Ssum;
    } else {  // (a tree past the level tables: the serial walk)
      if (t == 0) cd_walk(nb, 0, leaf_off, leaf_len, nullptr, &nleaves, cstack);
      __syncthreads();
      for (int l = t; l < nleaves; l += CD_THREADS) leaf_val[l] = cd_leaf(cdf + leaf_off[l], leaf_len[l]);
      __syncthreads();
      if (t == 0) Ssum = 0.0 + cd_walk(nb, 1, nullptr, nullptr, leaf_val, nullptr, cstack);
    }
    if (t == 0 && a.log_area) c.command_area[0] = Ssum / (double)nb;
    __syncthreads();
  }
  // ---- the sampling cdf (cached while the weights are unchanged), staged in LDS ----
  if (need_cdf) {
    const double Sv = Ssum;
    for (int b = t; b < nb; b += CD_THREADS) {
      const double p = cdf[b] / Sv;
      cdf[b] = p;
      if (p != p) atomicOr(&bad, 1);
      if (p < 0.0) atomicOr(&bad, 2);
    }
    __syncthreads();
    if (bad || !(fabs(Sv) < INFINITY) || Sv == 0.0) {  // RandomState.choice's checks: no draw is made
      if (t == 0) {
        c.state[2] = (bad & 1) ? 1 : (bad & 2) ? 2 : 3;  // NaN / negative / do not sum to 1
        c.state[0] = 0;
      }
      return;
    }
    if (t == 0) {  // cumsum: a sequential chain of adds, as add.accumulate (the next 16 loads in flight under the chain)
      double acc = cdf[0];
      int b = 1;
      double nx[16];
      if (b + 16 <= nb) {
#pragma unroll
        for (int j = 0; j < 16; ++j) nx[j] = cdf[b + j];
      }
      for (; b + 16 <= nb; b += 16) {
        double v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = nx[j];
        if (b + 32 <= nb) {
#pragma unroll
          for (int j = 0; j < 16; ++j) nx[j] = cdf[b + 16 + j];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          acc = acc + v[j];
          v[j] = acc;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) cdf[b + j] = v[j];
      }
      for (; b < nb; ++b) {
        acc = acc + cdf[b];
        cdf[b] = acc;
      }
    }
    __syncthreads();
    const double lastv = cdf[nb - 1];
    __syncthreads();
    for (int b = t; b < nb; b += CD_THREADS) {
      cdf[b] = cdf[b] / lastv;
      c.cdf[b] = cdf[b];
    }
    if (t == 0) c.state[0] = 1;
  } else {
    for (int b = t; b < nb; b += CD_THREADS) cdf[b] = c.cdf[b];
  }
  __syncthreads();
  // ---- the draws: n choice doubles, then 3 n uniform doubles (2 words each) ----
  for (int i = t; i < MT_N; i += CD_THREADS) key[i] = c.mt_key[i];
  if (t == 0) posv = c.state[1];
  __syncthreads();
  const int W = 8 * n;
  int produced = 0;
  while (produced < W) {
    if (posv >= MT_N) {
      mt_twist(key);
      if (t == 0) posv = 0;
      __syncthreads();
    }
    const int p0 = posv, take = min(MT_N - p0, W - produced);
    for (int j = t; j < take; j += CD_THREADS) c.words[produced + j] = mt_temper(key[p0 + j]);
    produced += take;
    __syncthreads();
    if (t == 0) posv = p0 + take;
    __syncthreads();
  }
  for (int i = t; i < MT_N; i += CD_THREADS) c.mt_key[i] = key[i];
  if (t == 0) c.state[1] = posv;
  for (int m = t; m < 4 * n; m += CD_THREADS) {
    const int32_t hi = (int32_t)(c.words[2 * m] >> 5), lo = (int32_t)(c.words[2 * m + 1] >> 6);
    c.draws[m] = (hi * 67108864.0 + lo) / 9007199254740992.0;
  }
  __syncthreads();
  // ---- choice (searchsorted right), the cell's uniform draws, _resample_commands' writes ----
  const double* ax[3] = {c.axes, c.axes + c.nx, c.axes + c.nx + c.ny};
  for (int j = t; j < n; j += CD_THREADS) {
    const double u = c.draws[j];
    int lo = 0, hi = nb;  // the first index whose cdf exceeds u
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] <= u) lo = mid + 1;
      else hi = mid;
    }
    const int b = lo;
    const int idx[3] = {b / (c.nz * c.ny), (b / c.nz) % c.ny, b % c.nz};
    float cf[3];
    for (int d = 0; d < 3; ++d) {
      const double g = ax[d][idx[d]];
      const double l = g + c.half[d], h = g - c.half[d];
      const double range = h - l;
      cf[d] = (float)(l + range * c.draws[n + 3 * j + d]);
    }
    const float nrm = __fsqrt_rn(cf[0] * cf[0] + cf[1] * cf[1]);
    const float keep = nrm > 0.2f ? 1.f : 0.f;
    cf[0] *= keep;
    cf[1] *= keep;
    const int e = a.ids[j];
    c.env_bins[e] = b;
    for (int d = 0; d < 3; ++d) S.commands[(int64_t)d * N + e] = cf[d];
    for (int r = 0; r < a.n_cs; ++r) S.command_sums[(int64_t)r * N + e] = 0.f;
  }
  if (a.log_area) {  // reset_idx: extras['env_bins'] = torch.Tensor(env_command_bins), every env's bin at this reset
    __syncthreads();
    for (int e = t; e < S.n; e += CD_THREADS) c.env_bins_f[e] = (float)c.env_bins[e];
  }
}

}  // namespace lrl

extern "C" hipError_t lrl_launch_curriculum_dev(const lrl_dev_curriculum* c, const KState* S, int32_t n_cs,
                                                const int32_t* ids, int32_t nmax, const int32_t* dcount, int32_t ep_len,
                                                int32_t row_lin, int32_t row_ang, double lin_thr, double ang_thr,
                                                double local_range, int32_t update, int32_t log_area, hipStream_t st) {
  lrl::CurDevArgs a{};
  a.c = *c;
  a.S = *S;
  a.n_cs = n_cs;
  a.ids = ids;
  a.nmax = nmax;
  a.dcount = dcount;
  a.ep_len = (float)ep_len;
  a.row_lin = row_lin;
  a.row_ang = row_ang;
  a.lin_thr = (float)lin_thr;  // numpy 2 compares the float32 rewards with the Python threshold cast to float32
  a.ang_thr = (float)ang_thr;
  a.local_range = local_range;
  a.update = update;
  a.log_area = log_area;
  const int nb = c->nx * c->ny * c->nz;
  const size_t lds = (size_t)nb * 8 + (size_t)(2 * nb + lrl::MT_N) * 4;
  if (nb / 64 + 2 > lrl::CD_MAX_LEAVES) return hipErrorInvalidValue;
  constexpr size_t kMaxDyn = 124 * 1024;  // (+ the kernel's ~31 KB of static LDS, inside the CU's 160 KB)
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(lrl::curriculum_dev_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxDyn) != hipSuccess)
      return hipErrorInvalidValue;
    attr = true;
  }
  if (lds > kMaxDyn) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lrl::curriculum_dev_kernel, dim3(1), dim3(lrl::CD_THREADS), lds, st, a);
  return hipGetLastError();
}
