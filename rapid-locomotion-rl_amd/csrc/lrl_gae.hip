// lrl_gae.hip — RolloutStorage.compute_returns (rollout_storage.py:76-90) for gfx950.
//
// Lane per env: the reversed T loop of the GAE recurrence runs in registers (rewards/values/dones
// are read once, coalesced across lanes since storage is [T][N]); returns and raw advantages are
// written once.  The advantage normalisation (mean, unbiased std over T*N, +1e-8) needs a global
// reduction: each block writes one fp64 partial (sum, sum of squares) and a second tiny launch
// folds the partials and rescales in place.  HBM bytes per env-step: 4 (r) + 1 (done) + 4 (v) read,
// 4 (ret) + 4 (adv) write, then 4 + 4 read and 4 write for the normalisation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lrl.h"

extern "C" int lrl_set_error(int code, const char* msg);

namespace lrl {

constexpr int GAE_BLOCK = 256;

__global__ __launch_bounds__(GAE_BLOCK) void gae_kernel(const float* __restrict__ rew, const uint8_t* __restrict__ done,
                                                        const float* __restrict__ val,
                                                        const float* __restrict__ last_val, int T, int N, float gamma,
                                                        float lam, float* __restrict__ ret, float* __restrict__ adv,
                                                        double* __restrict__ part) {
  const int e = blockIdx.x * GAE_BLOCK + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (e < N) {
    float a = 0.f;
    float next_v = last_val[e];
    const float gl = gamma * lam;
    for (int t = T - 1; t >= 0; --t) {
      const size_t i = (size_t)t * N + e;
      const float v = val[i];
      const float nt = 1.0f - (float)done[i];
      const float delta = rew[i] + nt * gamma * next_v - v;
      a = delta + nt * gl * a;
      const float r = a + v;
      ret[i] = r;
      const float ad = r - v;  // advantages = returns - values (:89)
      adv[i] = ad;
      s1 += ad;
      s2 += (double)ad * ad;
      next_v = v;
    }
  }
  // block reduction (wave shuffle then LDS)
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_down(s1, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  __shared__ double red[2][GAE_BLOCK / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int k = 0; k < GAE_BLOCK / 64; ++k) {
      a += red[0][k];
      b += red[1][k];
    }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// fold the per-block partials into stats = (sum, sum of squares, count), fp64
__global__ void gae_fold_kernel(const double* __restrict__ part, int nparts, int64_t total, double* __restrict__ stats) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double a = 0, b = 0;
    for (int k = 0; k < nparts; ++k) {
      a += part[2 * k];
      b += part[2 * k + 1];
    }
    stats[0] = a;
    stats[1] = b;
    stats[2] = (double)total;
  }
}

// adv = (adv - mean) / (std_unbiased + 1e-8)   (rollout_storage.py:90)
__global__ __launch_bounds__(GAE_BLOCK) void adv_normalize_kernel(float* __restrict__ adv, int64_t total,
                                                                  const double* __restrict__ stats) {
  const double cnt = stats[2];
  const double mean = stats[0] / cnt;
  const double var = (stats[1] - cnt * mean * mean) / (cnt - 1.0);
  const float m = (float)mean, den = (float)sqrt(var > 0 ? var : 0.0) + 1e-8f;
  for (int64_t i = (int64_t)blockIdx.x * GAE_BLOCK + threadIdx.x; i < total; i += (int64_t)gridDim.x * GAE_BLOCK)
    adv[i] = (adv[i] - m) / den;
}

}  // namespace lrl

static int gae_partial(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                       int32_t T, int32_t N, float gamma, float lam, float* returns, float* advantages, float* workspace,
                       double* stats, hipStream_t st) {
  if (T <= 0 || N <= 0 || !rewards || !dones || !values || !last_values || !returns || !advantages || !workspace ||
      !stats)
    return lrl_set_error(LRL_E_INVALID, "lrl_gae: null argument or empty shape");
  const int blocks = (N + lrl::GAE_BLOCK - 1) / lrl::GAE_BLOCK;
  if (blocks > 1000) return lrl_set_error(LRL_E_INVALID, "lrl_gae: N > 256000 (workspace holds 1000 partials)");
  double* part = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(lrl::gae_kernel, dim3(blocks), dim3(lrl::GAE_BLOCK), 0, st, rewards, dones, values, last_values,
                     T, N, gamma, lam, returns, advantages, part);
  hipLaunchKernelGGL(lrl::gae_fold_kernel, dim3(1), dim3(64), 0, st, part, blocks, (int64_t)T * N, stats);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, hipGetErrorString(e));
}

static int adv_normalize(float* adv, int64_t total, const double* stats, hipStream_t st) {
  if (!adv || !stats || total < 2) return lrl_set_error(LRL_E_INVALID, "lrl_adv_normalize: bad arguments");
  int nb = (int)((total + lrl::GAE_BLOCK - 1) / lrl::GAE_BLOCK);
  if (nb > 1024) nb = 1024;
  hipLaunchKernelGGL(lrl::adv_normalize_kernel, dim3(nb), dim3(lrl::GAE_BLOCK), 0, st, adv, total, stats);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, hipGetErrorString(e));
}

extern "C" int32_t lrl_gae(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                           int32_t T, int32_t N, float gamma, float lam, float* returns, float* advantages,
                           float* workspace, void* stream) {
  if (!workspace) return lrl_set_error(LRL_E_INVALID, "lrl_gae: null workspace");
  double* stats = reinterpret_cast<double*>(workspace + 4000);
  int rc = gae_partial(rewards, dones, values, last_values, T, N, gamma, lam, returns, advantages, workspace, stats,
                       (hipStream_t)stream);
  if (rc) return rc;
  return adv_normalize(advantages, (int64_t)T * N, stats, (hipStream_t)stream);
}

extern "C" int32_t lrl_gae_partial(const float* rewards, const uint8_t* dones, const float* values,
                                   const float* last_values, int32_t T, int32_t N, float gamma, float lam,
                                   float* returns, float* advantages, float* workspace, double* stats, void* stream) {
  return gae_partial(rewards, dones, values, last_values, T, N, gamma, lam, returns, advantages, workspace, stats,
                     (hipStream_t)stream);
}

extern "C" int32_t lrl_adv_normalize(float* advantages, int64_t total, const double* stats, void* stream) {
  return adv_normalize(advantages, total, stats, (hipStream_t)stream);
}

// PPO.process_env_step + RolloutStorage.add_transitions (ppo.py:76-88, rollout_storage.py:57-71) of the env outputs
// in one launch: rewards (+ gamma * V * time_out, the time-out bootstrap, when time_outs is given), dones (bool
// bytes) and env_bins into storage row t.  The bootstrap is rounded as torch computes it: v * time_out, then
// gamma * that, then the add (no fused multiply-add).
namespace lrl {
__global__ void store_step_kernel(const float* __restrict__ rew, const uint8_t* __restrict__ done,
                                  const float* __restrict__ bins, const float* __restrict__ values,
                                  const uint8_t* __restrict__ time_outs, float gamma, int32_t n,
                                  float* __restrict__ dst_rew, uint8_t* __restrict__ dst_done,
                                  float* __restrict__ dst_bins) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r = rew[i];
  if (time_outs) {
    const float vt = values[i] * (time_outs[i] ? 1.f : 0.f);
    const float b = gamma * vt;
    r = r + b;
  }
  dst_rew[i] = r;
  dst_done[i] = done[i] ? 1 : 0;
  if (bins) dst_bins[i] = bins[i];
}
}  // namespace lrl

extern "C" int32_t lrl_ppo_store_step(const float* rew, const uint8_t* done, const float* env_bins,
                                      const float* values, const uint8_t* time_outs, float gamma, int32_t n,
                                      float* dst_rew, uint8_t* dst_done, float* dst_env_bins, void* stream) {
  if (!rew || !done || !dst_rew || !dst_done || n < 0 || (env_bins && !dst_env_bins) || (time_outs && !values))
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_store_step: bad argument");
  if (n == 0) return 0;
  hipLaunchKernelGGL(lrl::store_step_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, rew, done,
                     env_bins, values, time_outs, gamma, n, dst_rew, dst_done, dst_env_bins);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, hipGetErrorString(e));
}
