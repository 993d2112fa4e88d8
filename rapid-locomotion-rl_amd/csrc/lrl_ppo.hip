// lrl_ppo.hip — PPO.update (mini_gym_learn/ppo/ppo.py:94-178) for gfx950.
//
// Per minibatch (B rows gathered through the randperm slice, never copied):
//   phase 1  lrl_ppo_forward_backward      encoder / actor / critic forward (grouped fp32-MFMA GEMMs,
//            bias+ELU fused), one "head" kernel for the distribution, losses (clipped surrogate,
//            clipped value loss, entropy), KL and the loss gradient, then the backward pass
//            (backward-data GEMMs with ELU' fused, split-k weight-gradient GEMMs) and one segmented
//            reduction that lands every gradient in the flat grad buffer;
//   phase 2  lrl_ppo_optimizer_step        adaptive-KL learning rate, clip_grad_norm_, Adam — all on the
//            device (the learning rate lives in lrl_ppo_ctrl), so a single-GPU update never syncs the host;
//   phase 3  lrl_ppo_adaptation_forward_backward   target = encoder(priv) with the updated weights,
//            adaptation_module(history) forward, MSE and backward;
//   phase 4  lrl_ppo_adaptation_step       Adam on the adaptation module (Q14: the second optimiser only
//            ever sees adaptation-module gradients).
// Between phases 1/2 and 3/4 a multi-GPU caller all-reduces grads[main_begin:kl_slot+1) /
// grads[adapt_begin:adapt_end) (one flat RCCL all-reduce each) and passes grad_scale = 1/world.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/lrl.h"
#include "../../include/lrl_philox.h"
#include "lrl_gemm.h"

extern "C" int lrl_set_error(int code, const char* msg);

namespace lrl {

constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;  // math.log(math.sqrt(2 * math.pi))
constexpr int HEAD_ROWS = 32;                             // rows per head workgroup (LDS ~45 KB: 3 per CU)
constexpr int HEAD_THREADS = 256;
constexpr int HEAD_W = 128;                               // actor / critic last hidden width (ac_h2)
constexpr int MAX_ACT = 16;
constexpr int HEAD_NA = 12;  // the PPO head kernel is specialised for the quadrupeds' 12 actions
constexpr int MAX_LAT = 32;

__device__ __forceinline__ float delu(float h) { return h > 0.f ? 1.f : h + 1.f; }  // elu'(y) from h = elu(y)

// ---------------------------------------------------------------------------------------------------
// gather obs rows into the actor/critic input X = [obs | latent | 0-pad] ([B][64])
// thread = (group of PREP_R rows, column): the group's row indices, then its values, are loaded before any store, so
// a thread has PREP_R gathers in flight and the grid is resident in one round (one thread per element left most of
// a minibatch's workgroups waiting behind two dependent load latencies)
constexpr int PREP_R = 4;
__global__ void ppo_prep_kernel(const float* __restrict__ obs, const int64_t* __restrict__ rows, int B, int no,
                                int xs, float* __restrict__ X) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t ng = ((int64_t)B + PREP_R - 1) / PREP_R;
  if (i >= ng * xs) return;
  const int g = (int)(i / xs), c = (int)(i - (int64_t)g * xs);
  int64_t src[PREP_R];
  float v[PREP_R];
#pragma unroll
  for (int u = 0; u < PREP_R; ++u) {
    const int b = g * PREP_R + u;
    src[u] = b < B ? (rows ? rows[b] : (int64_t)b) : -1;
  }
#pragma unroll
  for (int u = 0; u < PREP_R; ++u) v[u] = (c < no && src[u] >= 0) ? obs[src[u] * no + c] : 0.f;
#pragma unroll
  for (int u = 0; u < PREP_R; ++u) {
    const int b = g * PREP_R + u;
    if (b < B) X[(int64_t)b * xs + c] = v[u];
  }
}

inline unsigned prep_blocks(int64_t rows, int xs) {
  return (unsigned)((((rows + PREP_R - 1) / PREP_R) * xs + 255) / 256);
}

// ---------------------------------------------------------------------------------------------------
// PPO head: mu = H3a W4a^T + b4a, v = H3c W4c^T + b4c, Normal(mu, std) log-prob / entropy, clipped
// surrogate, clipped value loss, KL(old || new) (ppo.py:98-147, actor_critic.py:126-135); gradient of
// loss = surrogate + c_v value - c_e entropy w.r.t. mu, v and std; dH3 = (dmu W4a | dv W4c) * elu'(H3);
// per-workgroup partials: dW4a, db4a, dW4c, db4c, dstd, sum kl, sum surrogate, sum value loss.
struct HeadArgs {
  const float* h3;      // [B][2*HW]: actor | critic
  float* dh3;           // [B][2*HW]
  const float *w4a, *b4a, *w4c, *b4c, *stdv;
  const float *actions, *old_mu, *old_sigma, *tv, *ret, *adv, *old_logp;
  const int64_t* rows;
  int B, na;
  float clip, ent_coef, vcoef;
  int clipped_value;
  float* part;          // [gridDim.x][part_len]
  int part_len;
};

// partial layout
__host__ __device__ constexpr int hp_w4a(int) { return 0; }
__host__ __device__ constexpr int hp_b4a(int na) { return na * HEAD_W; }
__host__ __device__ constexpr int hp_w4c(int na) { return na * HEAD_W + na; }
__host__ __device__ constexpr int hp_b4c(int na) { return na * HEAD_W + na + HEAD_W; }
__host__ __device__ constexpr int hp_std(int na) { return na * HEAD_W + na + HEAD_W + 1; }
__host__ __device__ constexpr int hp_kl(int na) { return na * HEAD_W + na + HEAD_W + 1 + na; }
__host__ __device__ constexpr int hp_len(int na) { return hp_kl(na) + 3; }  // kl, surrogate, value

__global__ __launch_bounds__(HEAD_THREADS) void ppo_head_kernel(HeadArgs a) {
  // phases: (0) stage H3 / head weights and the minibatch rows' indices, then issue the gathered per-(row, action)
  // and per-row loads (old actions / mu / sigma, advantage, old log-prob, target value, return) so their latency
  // hides under (1) mu, v; (2) per (row, action): log-prob and KL terms  (3) per row: ratio, clipped surrogate,
  // clipped value loss, their gradients  (4) per (row, action): d loss / d mu, d loss / d std  (5) per column: dH3
  // and the head weight-gradient partials.  Two global round trips in all (rows, then the gathered rows).
  // pitch 4 (mod 32) floats: the row-per-lane float4 reads of (1) hit distinct banks in every 8-lane group
  constexpr int HP = 2 * HEAD_W + 4;
  constexpr int NA = HEAD_NA;
  static_assert(NA % 4 == 0 && HEAD_W % 16 == 0, "float4 rows");
  constexpr int NG = (HEAD_ROWS * NA + HEAD_THREADS - 1) / HEAD_THREADS;  // gathered (row, action) items per thread
  __shared__ __attribute__((aligned(16))) float H[HEAD_ROWS][HP];
  __shared__ __attribute__((aligned(16))) float W4[NA + 1][HEAD_W];
  __shared__ float MU[HEAD_ROWS][NA + 1];   // mu_j, then d = a_j - mu_j
  __shared__ float VP[HEAD_ROWS][8];
  __shared__ __attribute__((aligned(16))) float LP[HEAD_ROWS][NA];  // log-prob term, then d loss / d mu
  __shared__ float KT[HEAD_ROWS][NA];       // KL term, then d loss / d std
  __shared__ float DR[HEAD_ROWS][2];        // d loss / d logp, d loss / d v
  __shared__ float SC[HEAD_ROWS][3];        // kl, surrogate, value loss per row
  __shared__ float SD[3][NA];               // std, log std, 1/std^2
  __shared__ float GA[3][HEAD_ROWS][NA];    // gathered old actions, old mu, old sigma
  __shared__ float GR[4][HEAD_ROWS];        // gathered advantage, old log-prob, target value, return
  __shared__ int64_t RW[HEAD_ROWS];
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * HEAD_ROWS;
  const int nrows = min(HEAD_ROWS, a.B - r0);
  if (t < HEAD_ROWS) RW[t] = t < nrows ? a.rows[r0 + t] : a.rows[r0];
  if (t < NA) {
    const float sd = a.stdv[t];
    SD[0][t] = sd;
    SD[1][t] = logf(sd);
    SD[2][t] = 1.f / (sd * sd);
  }
  {
    constexpr int NV = HEAD_ROWS * 2 * HEAD_W / 4 / HEAD_THREADS;
    float4 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = t + u * HEAD_THREADS, r = i / (HEAD_W / 2), c = 4 * (i % (HEAD_W / 2));
      v[u] = r < nrows ? *reinterpret_cast<const float4*>(a.h3 + (int64_t)(r0 + r) * (2 * HEAD_W) + c)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = t + u * HEAD_THREADS, r = i / (HEAD_W / 2), c = 4 * (i % (HEAD_W / 2));
      *reinterpret_cast<float4*>(&H[r][c]) = v[u];
    }
  }
  for (int i = t; i < (NA + 1) * HEAD_W; i += HEAD_THREADS) {
    const int j = i / HEAD_W, k = i - j * HEAD_W;
    W4[j][k] = j < NA ? a.w4a[j * HEAD_W + k] : a.w4c[k];
  }
  __syncthreads();
  // (0b) the gathered loads, all issued before (1) uses none of them
  float ga[3][NG], gr = 0.f;
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    const int i = t + u * HEAD_THREADS;
    const int r = i / NA, j = i - r * NA;
    const bool ok = i < HEAD_ROWS * NA;
    const int64_t o = RW[ok ? r : 0] * NA + j;
    ga[0][u] = ok ? a.actions[o] : 0.f;
    ga[1][u] = ok ? a.old_mu[o] : 0.f;
    ga[2][u] = ok ? a.old_sigma[o] : 1.f;
  }
  if (t < 4 * HEAD_ROWS) {
    const int q = t / HEAD_ROWS, r = t - q * HEAD_ROWS;
    const float* src = q == 0 ? a.adv : q == 1 ? a.old_logp : q == 2 ? a.tv : a.ret;
    gr = src[RW[r]];
  }
  // (1) thread (r, q): actions q, q+8 and an eighth of the value dot (float4 LDS reads, the same sequential fmaf
  // order over k as one element at a time)
  {
    const int r = t & (HEAD_ROWS - 1), q = t / HEAD_ROWS;
    const float4* hr = reinterpret_cast<const float4*>(&H[r][0]);
    auto dot4 = [](float s, float4 h, float4 w) {
      s = fmaf(h.x, w.x, s);
      s = fmaf(h.y, w.y, s);
      s = fmaf(h.z, w.z, s);
      return fmaf(h.w, w.w, s);
    };
    for (int j = q; j < NA; j += 8) {
      const float4* wr = reinterpret_cast<const float4*>(&W4[j][0]);
      float s = 0.f;
#pragma unroll 8
      for (int k4 = 0; k4 < HEAD_W / 4; ++k4) s = dot4(s, hr[k4], wr[k4]);
      MU[r][j] = s + a.b4a[j];
    }
    const float4* wv = reinterpret_cast<const float4*>(&W4[NA][q * (HEAD_W / 8)]);
    const float4* hv = hr + (HEAD_W + q * (HEAD_W / 8)) / 4;
    float s = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < HEAD_W / 32; ++k4) s = dot4(s, hv[k4], wv[k4]);
    VP[r][q] = s;
  }
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    const int i = t + u * HEAD_THREADS;
    if (i < HEAD_ROWS * NA) {
      const int r = i / NA, j = i - r * NA;
      GA[0][r][j] = ga[0][u];
      GA[1][r][j] = ga[1][u];
      GA[2][r][j] = ga[2][u];
    }
  }
  if (t < 4 * HEAD_ROWS) GR[t / HEAD_ROWS][t & (HEAD_ROWS - 1)] = gr;
  __syncthreads();
  // (2) per (row, action): Normal log-prob term and KL(old || new) term (ppo.py:111-114)
  for (int i = t; i < HEAD_ROWS * NA; i += HEAD_THREADS) {
    const int r = i / NA, j = i - r * NA;
    float lp = 0.f, kt = 0.f, d = 0.f;
    if (r < nrows) {
      const float s = SD[0][j], mu = MU[r][j];
      d = GA[0][r][j] - mu;
      lp = -(d * d) / (2.f * (s * s)) - SD[1][j] - LOG_SQRT_2PI;
      const float so = GA[2][r][j], dm = GA[1][r][j] - mu;
      kt = logf(s / so + 1.e-5f) + (so * so + dm * dm) / (2.f * (s * s)) - 0.5f;
    }
    MU[r][j] = d;
    LP[r][j] = lp;
    KT[r][j] = kt;
  }
  __syncthreads();
  const float invB = 1.f / (float)a.B;
  // (3) per row
  if (t < HEAD_ROWS) {
    const int r = t;
    float kl = 0.f, surr_loss = 0.f, vloss = 0.f, dv = 0.f, dlogp = 0.f;
    if (r < nrows) {
      const float v = (((VP[r][0] + VP[r][1]) + (VP[r][2] + VP[r][3])) + ((VP[r][4] + VP[r][5]) + (VP[r][6] + VP[r][7]))) +
                      a.b4c[0];
      float logp = 0.f;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        logp += LP[r][j];
        kl += KT[r][j];
      }
      const float adv = GR[0][r];
      const float ratio = expf(logp - GR[1][r]);
      const float surr = -adv * ratio;
      const float rc = fminf(fmaxf(ratio, 1.f - a.clip), 1.f + a.clip);
      const float surr_c = -adv * rc;
      surr_loss = fmaxf(surr, surr_c);
      // torch.max backward: the larger side takes the gradient, ties split it in half
      const float ga = surr > surr_c ? invB : (surr == surr_c ? 0.5f * invB : 0.f);
      const float gb = surr_c > surr ? invB : (surr == surr_c ? 0.5f * invB : 0.f);
      const bool in_rng = ratio >= 1.f - a.clip && ratio <= 1.f + a.clip;
      const float dratio = -adv * ga + (in_rng ? -adv * gb : 0.f);
      dlogp = dratio * ratio;
      // value loss (ppo.py:133-143)
      const float tv = GR[2][r], ret = GR[3][r];
      const float gv = a.vcoef * invB;
      if (a.clipped_value) {
        const float dvt = v - tv;
        const float vc = tv + fminf(fmaxf(dvt, -a.clip), a.clip);
        const float l1 = (v - ret) * (v - ret), l2 = (vc - ret) * (vc - ret);
        vloss = fmaxf(l1, l2);
        const float g1 = l1 > l2 ? gv : (l1 == l2 ? 0.5f * gv : 0.f);
        const float g2 = l2 > l1 ? gv : (l1 == l2 ? 0.5f * gv : 0.f);
        const bool vin = dvt >= -a.clip && dvt <= a.clip;
        dv = g1 * 2.f * (v - ret) + (vin ? g2 * 2.f * (vc - ret) : 0.f);
      } else {
        vloss = (ret - v) * (ret - v);
        dv = gv * 2.f * (v - ret);
      }
    }
    DR[r][0] = dlogp;
    DR[r][1] = dv;
    SC[r][0] = kl;
    SC[r][1] = surr_loss;
    SC[r][2] = vloss;
  }
  __syncthreads();
  // (4) per (row, action): d/d mu = dlogp (a - mu)/var; d/d std = dlogp ((a-mu)^2/var - 1)/std - c_e/(B std)
  for (int i = t; i < HEAD_ROWS * NA; i += HEAD_THREADS) {
    const int r = i / NA, j = i - r * NA;
    float dm = 0.f, ds = 0.f;
    if (r < nrows) {
      const float d = MU[r][j], dl = DR[r][0], s = SD[0][j], ivar = SD[2][j];
      dm = dl * (d * ivar);
      ds = dl * (d * d * ivar - 1.f) / s - a.ent_coef * invB / s;
    }
    LP[r][j] = dm;
    KT[r][j] = ds;
  }
  __syncthreads();
  // (5) backward into H3 and the head weight-gradient partials: thread = column of [actor | critic]
  float* P = a.part + (int64_t)blockIdx.x * a.part_len;
  {
    const int k = t;  // 0..255
    if (k < HEAD_W) {
      float wk[NA], accw[NA];
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        wk[j] = W4[j][k];
        accw[j] = 0.f;
      }
#pragma unroll 2
      for (int r = 0; r < nrows; ++r) {
        const float h = H[r][k];
        float dmr[NA];  // (row r's d loss / d mu: NA / 4 broadcast float4 reads)
#pragma unroll
        for (int j4 = 0; j4 < NA / 4; ++j4) {
          const float4 v = reinterpret_cast<const float4*>(&LP[r][0])[j4];
          dmr[4 * j4] = v.x; dmr[4 * j4 + 1] = v.y; dmr[4 * j4 + 2] = v.z; dmr[4 * j4 + 3] = v.w;
        }
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          const float dm = dmr[j];
          s = fmaf(dm, wk[j], s);
          accw[j] = fmaf(dm, h, accw[j]);
        }
        a.dh3[(int64_t)(r0 + r) * (2 * HEAD_W) + k] = s * delu(h);
      }
#pragma unroll
      for (int j = 0; j < NA; ++j) P[hp_w4a(NA) + j * HEAD_W + k] = accw[j];
    } else {
      const int kk = k - HEAD_W;
      const float wk = W4[NA][kk];
      float accc = 0.f;
      for (int r = 0; r < nrows; ++r) {
        const float h = H[r][k];
        const float d = DR[r][1];
        accc = fmaf(d, h, accc);
        a.dh3[(int64_t)(r0 + r) * (2 * HEAD_W) + k] = (d * wk) * delu(h);
      }
      P[hp_w4c(NA) + kk] = accc;
    }
  }
  if (t < NA) {
    float sb = 0.f, ss = 0.f;
    for (int r = 0; r < nrows; ++r) {
      sb += LP[r][t];
      ss += KT[r][t];
    }
    P[hp_b4a(NA) + t] = sb;
    P[hp_std(NA) + t] = ss;
  } else if (t == 16) {
    float sb = 0.f;
    for (int r = 0; r < nrows; ++r) sb += DR[r][1];
    P[hp_b4c(NA)] = sb;
  } else if (t >= 32 && t < 35) {
    const int c = t - 32;
    float s = 0.f;
    for (int r = 0; r < nrows; ++r) s += SC[r][c];
    P[hp_kl(NA) + c] = s;
  }
}

// ---------------------------------------------------------------------------------------------------
// Rollout head of PPO.act (ppo.py:62-74, actor_critic.py:126-135,170-173): mu = H3a W4a^T + b,
// value = H3c W4c^T + b, a = mu + std * eps (eps injected or Box-Muller on the counter RNG), log-prob,
// and the transition row of RolloutStorage.add_transitions (rollout_storage.py:57-71).
struct ActHeadArgs {
  const float* h3;  // [n][2*HW]
  const float *w4a, *b4a, *w4c, *b4c, *stdv;
  const float *obs, *priv, *hist, *eps;
  int n, na, no, np;
  uint64_t seed, counter;
  int64_t row_offset;  // global id of row 0 (the rank's env_offset): the noise key, so draws do not depend on sharding
  float *actions, *mu, *values, *logp;
  lrl_rollout_store store;
  int store_row, do_store;
  float* xa_out;  // ENC_ONLY: the [obs | latent | 0] rows, pitch xs
};

// rows [0, nrows) of src (pitch sld) -> dst (pitch dld), `cols` floats each, by the block's HEAD_THREADS
// threads with 8 loads in flight per thread (float2 when both sides allow)
__device__ __forceinline__ void copy_rows(const float* __restrict__ src, int64_t sld, float* __restrict__ dst,
                                          int64_t dld, int nrows, int cols, int t) {
  if (((((uintptr_t)src | (uintptr_t)dst) & 7) == 0) && (((sld | dld | cols) & 1) == 0)) {
    const int c2 = cols / 2, n = nrows * c2;
    for (int i0 = t; i0 < n; i0 += 8 * HEAD_THREADS) {
      float2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * HEAD_THREADS, r = i / c2, c = i - r * c2;
        if (i < n) v[u] = reinterpret_cast<const float2*>(src + r * sld)[c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * HEAD_THREADS, r = i / c2, c = i - r * c2;
        if (i < n) reinterpret_cast<float2*>(dst + r * dld)[c] = v[u];
      }
    }
  } else {
    const int n = nrows * cols;
    for (int i0 = t; i0 < n; i0 += 8 * HEAD_THREADS) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * HEAD_THREADS, r = i / cols, c = i - r * cols;
        if (i < n) v[u] = src[r * sld + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * HEAD_THREADS, r = i / cols, c = i - r * cols;
        if (i < n) dst[r * dld + c] = v[u];
      }
    }
  }
}

// rollout head: ACT_ROWS rows per workgroup (4096 envs -> 256 workgroups, one per CU: the kernel holds one workgroup
// per CU (its register footprint), so 512 eight-row workgroups ran in two rounds — 18.3 against 13.7 us; 32 rows 20.7 us)
constexpr int ACT_ROWS = 16, ACT_Q = HEAD_THREADS / ACT_ROWS;  // 16 thread groups per row
__global__ __launch_bounds__(HEAD_THREADS) void act_head_kernel(ActHeadArgs a) {
  constexpr int HP = 2 * HEAD_W + 1;
  __shared__ float H[ACT_ROWS][HP];
  __shared__ float W4[MAX_ACT + 1][HEAD_W];
  __shared__ float MU[ACT_ROWS][MAX_ACT + 1];
  __shared__ float VP[ACT_ROWS][ACT_Q];
  const int t = threadIdx.x, na = a.na;
  const int r0 = blockIdx.x * ACT_ROWS;
  const int nrows = min(ACT_ROWS, a.n - r0);
  {
    constexpr int NV = ACT_ROWS * 2 * HEAD_W / 4 / HEAD_THREADS;
    float4 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = t + u * HEAD_THREADS, r = i / (HEAD_W / 2), c = 4 * (i % (HEAD_W / 2));
      v[u] = r < nrows ? *reinterpret_cast<const float4*>(a.h3 + (int64_t)(r0 + r) * (2 * HEAD_W) + c)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = t + u * HEAD_THREADS, r = i / (HEAD_W / 2), c = 4 * (i % (HEAD_W / 2));
      *reinterpret_cast<float4*>(&H[r][c]) = v[u];
    }
  }
  for (int i = t; i < (na + 1) * HEAD_W; i += HEAD_THREADS) {
    const int j = i / HEAD_W, k = i - j * HEAD_W;
    W4[j][k] = j < na ? a.w4a[j * HEAD_W + k] : a.w4c[k];
  }
  __syncthreads();
  {
    const int r = t & (ACT_ROWS - 1), q = t / ACT_ROWS;
    for (int j = q; j < na; j += ACT_Q) {
      float s = 0.f;
      for (int k = 0; k < HEAD_W; ++k) s = fmaf(H[r][k], W4[j][k], s);
      MU[r][j] = s + a.b4a[j];
    }
    float s = 0.f;
    for (int k = q * (HEAD_W / ACT_Q); k < (q + 1) * (HEAD_W / ACT_Q); ++k) s = fmaf(H[r][HEAD_W + k], W4[na][k], s);
    VP[r][q] = s;
  }
  __syncthreads();
  const int64_t so = (int64_t)a.store_row * a.n;
  // one thread per (row, action): sample + write; the per-row log-prob sum is formed after a barrier
  for (int i = t; i < nrows * na; i += HEAD_THREADS) {
    const int r = i / na, j = i - r * na, g = r0 + r;
    float e;
    if (a.eps) {
      e = a.eps[(int64_t)g * na + j];
    } else {  // Box-Muller on the counter RNG (stream POLICY): pairs of actions share one Philox draw
      lrl_u32x4 u = lrl_philox((uint32_t)(a.row_offset + g), (uint32_t)a.counter, (LRL_RNG_POLICY << 16) ^ (uint32_t)(a.counter >> 32),
                               (uint32_t)(j >> 1), a.seed);
      const float u1 = fmaxf(lrl_u01(u.v[0]), 1e-7f), u2 = lrl_u01(u.v[1]);
      const float rad = sqrtf(-2.f * logf(u1)), th = 6.283185307179586f * u2;
      e = (j & 1) ? rad * sinf(th) : rad * cosf(th);
    }
    const float m = MU[r][j], sd = a.stdv[j];
    const float act = m + sd * e;
    const float d = act - m;
    MU[r][j] = -(d * d) / (2.f * (sd * sd)) - logf(sd) - LOG_SQRT_2PI;  // log-prob term (mu no longer needed)
    a.actions[(int64_t)g * na + j] = act;
    if (a.mu) a.mu[(int64_t)g * na + j] = m;
    if (a.do_store) {
      const int64_t o = (so + g) * na + j;
      a.store.actions[o] = act;
      a.store.mu[o] = m;
      a.store.sigma[o] = sd;
    }
  }
  __syncthreads();
  if (t < nrows) {
    const int g = r0 + t;
    float lp = 0.f;
    for (int j = 0; j < na; ++j) lp += MU[t][j];
    float vs[ACT_Q];
#pragma unroll
    for (int q = 0; q < ACT_Q; ++q) vs[q] = VP[t][q];
#pragma unroll
    for (int w = ACT_Q / 2; w >= 1; w /= 2)  // pairwise tree, fixed order
#pragma unroll
      for (int q = 0; q < w; ++q) vs[q] = vs[2 * q] + vs[2 * q + 1];
    const float v = vs[0] + a.b4c[0];
    if (a.values) a.values[g] = v;
    if (a.logp) a.logp[g] = lp;
    if (a.do_store) {
      a.store.values[so + g] = v;
      a.store.logp[so + g] = lp;
    }
  }
  if (a.do_store) {  // obs / priv / history rows of this tile into storage row `store_row`
    const int64_t b = so + r0;
    copy_rows(a.obs + (int64_t)r0 * a.no, a.no, a.store.obs + b * a.no, a.no, nrows, a.no, t);
    copy_rows(a.priv + (int64_t)r0 * a.np, a.np, a.store.priv + b * a.np, a.np, nrows, a.np, t);
    if (a.hist && a.store.hist) {
      const int hd = a.store.hist_dim, ld = a.store.hist_ld > hd ? a.store.hist_ld : hd;
      copy_rows(a.hist + (int64_t)r0 * hd, hd, a.store.hist + b * ld, ld, nrows, hd, t);
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Fused rollout act (PPO.act, ppo.py:62-74 -> actor_critic.py:137-147,170-173, + RolloutStorage.add_transitions,
// rollout_storage.py:57-71): one workgroup carries FA_R = 16 env rows through the whole chain — encoder, actor / critic
// bodies, heads, sampling, log-prob and the storage row — with every activation in LDS, so a rollout step's act is one
// launch (the unfused chain is eight, each on its ~6-10 us load -> MFMA -> store floor at 4,096 rows).  The products
// run on the fp32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation): a wave owns a run of 16-column
// output tiles; per 16-k chunk lane (i, q) = (lane & 15, lane >> 4) reads A[i][k0 + 4q .. +3] from LDS (one b128) and,
// per tile, the 4 weights W[n][k0 + 4q .. +3] of its output column n straight from L2 (the next chunk's loads are in
// flight while this chunk's MFMAs run); step s of the chunk multiplies k = k0 + 4q + s.  16 rows per workgroup puts
// 4,096 envs on 256 workgroups, one per CU (115 KB of LDS).
constexpr int FA_R = 16, FA_THREADS = 256;
constexpr int FA_D = 2;       // weight chunks (32 k each) in flight per wave: the L2 round trip over the MFMA work
constexpr int FA_XP = 260;    // X / he1 / h3 pitch (widths <= 256) + 4: conflict-free b128 row reads
constexpr int FA_BIGP = 1028; // h1 pitch (2 x ac_h0 <= 1024)
constexpr int FA_MIDP = 516;  // h2 pitch (2 x ac_h1 <= 512); priv / he2 use narrower pitches in the same region
constexpr int FA_HW_FLOATS = (HEAD_NA + 1) * HEAD_W;  // the heads' weights, staged at the start
constexpr int FA_LDS_FLOATS = FA_R * (FA_XP + FA_BIGP + FA_MIDP) + FA_HW_FLOATS;
constexpr int FA_ENC_MIDP = 260;  // ENC_ONLY: priv [16][36] / he2 [16][enc_h1 + 4 <= 260]
constexpr int FA_ENC_LDS_FLOATS = FA_R * (FA_XP + FA_XP + FA_ENC_MIDP);  // ENC_ONLY: X, he1, priv / he2 (49.9 KB)

// Phase timers of the fused act (build with -DLRL_ACT_PROFILE, read with lrl_debug_act_profile): shader-clock cycles
// per phase summed over workgroups (thread 0's view): stage, enc1..3, ac1..3, heads, sampling, storage copies
#ifdef LRL_ACT_PROFILE
__device__ unsigned long long g_act_prof[12];
#define FA_PROF_DECL unsigned long long fa_t = clock64();
#define FA_PROF(i)                                                  \
  if (threadIdx.x == 0) {                                           \
    const unsigned long long t_ = clock64();                        \
    atomicAdd(&g_act_prof[i], t_ - fa_t);                           \
    fa_t = t_;                                                      \
  }
#else
#define FA_PROF_DECL
#define FA_PROF(i)
#endif

typedef float fa_f32x4 __attribute__((ext_vector_type(4)));

struct FaLayer {
  const float* A;   // LDS input rows
  int pa, ga, K;    // pitch, column offset of group g's input (g * ga), k extent (multiple of 16, zero-padded)
  const float* W;   // weights of group 0: [Nw rows][ldw], group g at W + g * gw
  int ldw, Kw, Nw;  // row pitch, valid k (< Kw), valid rows (< Nw)
  int64_t gw;
  const float* b;   // bias of group 0 (group g at b + g * Nw)
  float* C;         // LDS output: group g's column n at C[row * pc + coff + g * Ng + n]
  int pc, coff, Ng, groups;
  int elu, vec;     // ELU after the bias; vec: 16-B aligned weight rows with Kw % 4 == 0 (float4 loads)
};

// NB column tiles of one group from t0; VEC: 16-B aligned weight rows (float4 loads), else dword loads.  The loads are
// branch-free (addresses clamped into the weights, out-of-range elements zeroed by selection) so the compiler keeps the
// FA_D chunks in flight with counted vmcnt waits instead of draining at every guarded load
template <int NB, bool VEC>
__device__ __forceinline__ void fa_tiles(const FaLayer& L, int t0) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
  const int tpg = L.Ng >> 4, g = t0 / tpg;  // a run never crosses a group (fa_layer)
  const float* A = L.A + i * L.pa + g * L.ga + 8 * q;
  const float* W = L.W + g * L.gw;
  const float* rowp[NB];
  bool rok[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = (t0 + j - g * tpg) * 16 + i;
    rok[j] = n < L.Nw;
    rowp[j] = W + (int64_t)(rok[j] ? n : L.Nw - 1) * L.ldw;
  }
  fa_f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = fa_f32x4{0.f, 0.f, 0.f, 0.f};
  // per 32-k chunk lane (i, q) holds the 8 weights W[n][k0 + 8q .. +7] of each tile (a whole 128-B line per row and
  // chunk over the 4 lane groups) and A[i][k0 + 8q .. +7]; step s multiplies k = k0 + 8q + s
  auto load_b = [&](float4 (&bv)[NB][2], int k0) {
    const int k = k0 + 8 * q;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if constexpr (VEC) {  // (Kw % 4 == 0: a float4 is wholly inside or wholly outside the row)
        const int k1 = min(k, L.Kw - 4), k2 = min(k + 4, L.Kw - 4);
        float4 v0 = *reinterpret_cast<const float4*>(rowp[j] + k1);
        float4 v1 = *reinterpret_cast<const float4*>(rowp[j] + k2);
        const bool o0 = rok[j] && k < L.Kw, o1 = rok[j] && k + 4 < L.Kw;
        bv[j][0] = o0 ? v0 : make_float4(0.f, 0.f, 0.f, 0.f);
        bv[j][1] = o1 ? v1 : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float x = rowp[j][min(k + u, L.Kw - 1)];
          v[u] = (rok[j] && k + u < L.Kw) ? x : 0.f;
        }
        bv[j][0] = make_float4(v[0], v[1], v[2], v[3]);
        bv[j][1] = make_float4(v[4], v[5], v[6], v[7]);
      }
    }
  };
  // FA_D chunks of weights in flight (a ring of register sets, indexed at compile time by unrolling FA_D chunks)
  const int nck = L.K >> 5;
  float4 ring[FA_D][NB][2];
#pragma unroll
  for (int d = 0; d < FA_D; ++d) load_b(ring[d], 32 * min(d, nck - 1));
  for (int c0 = 0; c0 < nck; c0 += FA_D) {
#pragma unroll
    for (int d = 0; d < FA_D; ++d) {
      const int c = c0 + d;
      if (c < nck) {
        const float4 a0 = *reinterpret_cast<const float4*>(A + 32 * c);
        const float4 a1 = *reinterpret_cast<const float4*>(A + 32 * c + 4);
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const float4& bq = ring[d][j][u >> 2];
            const float b = (u & 3) == 0 ? bq.x : (u & 3) == 1 ? bq.y : (u & 3) == 2 ? bq.z : bq.w;
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b, acc[j], 0, 0, 0);
          }
        }
        load_b(ring[d], 32 * min(c + FA_D, nck - 1));  // (past the end: a harmless re-read of the last chunk)
      }
    }
  }
  // C/D: column i of the tile, rows 4q .. 4q + 3 in the four registers
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = (t0 + j - g * tpg) * 16 + i;
    if (n < L.Nw) {
      const float bias = L.b[g * L.Nw + n];
      float* c = L.C + (4 * q) * L.pc + L.coff + g * L.Ng + n;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[j][r] + bias;
        if (L.elu) v = v > 0.f ? v : expm1f(v);
        c[r * L.pc] = v;
      }
    }
  }
}

// one layer: the T = groups * Ng / 16 column tiles split into equal runs over the 4 waves (T < 4: one tile per wave).
// NBC > 0: the run length known at compile time (the presets' widths), else dispatched on it
template <int NBC, bool VEC>
__device__ __forceinline__ void fa_layer(const FaLayer& L) {
  const int w = threadIdx.x >> 6, T = L.groups * (L.Ng >> 4);
  const int tpw = T >= 4 ? T / 4 : 1;
  if (w * tpw >= T) return;
  const int t0 = w * tpw;
  if constexpr (NBC == 16) {
    fa_tiles<8, VEC>(L, t0);
    fa_tiles<8, VEC>(L, t0 + 8);
  } else if constexpr (NBC > 0) {
    fa_tiles<NBC, VEC>(L, t0);
  } else {
    switch (tpw) {
      case 1: fa_tiles<1, VEC>(L, t0); break;
      case 2: fa_tiles<2, VEC>(L, t0); break;
      case 4: fa_tiles<4, VEC>(L, t0); break;
      case 8: fa_tiles<8, VEC>(L, t0); break;
      case 16: fa_tiles<8, VEC>(L, t0); fa_tiles<8, VEC>(L, t0 + 8); break;
      default:
        for (int t = t0; t < t0 + tpw; ++t) fa_tiles<1, VEC>(L, t);
    }
  }
}

struct FusedActArgs {
  const float* w;
  lrl_ppo_net net;
  const float *obs, *priv, *hist, *eps;
  int n, xs;
  uint32_t vec;  // bit l: float4 weight loads allowed for layer l (FA_L_*)
  uint64_t seed, counter;
  int64_t row_offset;
  float *actions, *mu, *values, *logp;
  lrl_rollout_store store;
  int store_row, do_store;
  float* xa_out;  // ENC_ONLY: the [obs | latent | 0] rows, pitch xs
};

// PRESET: the presets' network (18 -> 256 -> 128 -> 18 encoder, 2 x (64 -> 512 -> 256 -> 128) bodies, aligned weights):
// every layer's run length and load width fixed at compile time; otherwise dispatched per layer.
// ENC_ONLY: the rollout act's first four launches in one (ppo_prep_kernel's obs rows and the env-factor encoder's
// three products): the X rows [obs | latent | 0] go to a.xa_out for the actor / critic chain, in FA_ENC_LDS_FLOATS
template <bool PRESET, bool ENC_ONLY = false>
__global__ __launch_bounds__(FA_THREADS) void act_fused_kernel(FusedActArgs a) {
  extern __shared__ __attribute__((aligned(16))) float fa_lds[];
  float* X = fa_lds;                     // [16][FA_XP]: obs | latent | 0
  float* BIG = X + FA_R * FA_XP;         // he1 [16][FA_XP], h1 [16][FA_BIGP], h3 [16][FA_XP]
  float* MID = BIG + FA_R * (ENC_ONLY ? FA_XP : FA_BIGP);  // priv [16][36], he2 [16][enc_h1 + 4], h2 [16][FA_MIDP]
  float* HW = MID + FA_R * FA_MIDP;      // [NA + 1][HEAD_W]: w4a rows, then w4c
  FA_PROF_DECL
  const lrl_ppo_net& nt = a.net;
  const int t = threadIdx.x, r0 = blockIdx.x * FA_R, nrows = min(FA_R, a.n - r0);
  const int no = nt.num_obs, np = nt.num_priv, PP = 36, EP2 = nt.enc_h1 + 4;
  // stage obs (zero padding and rows past n) and priv (k padded to 32)
  for (int e = t; e < FA_R * a.xs; e += FA_THREADS) {
    const int r = e / a.xs, c = e - r * a.xs;
    X[r * FA_XP + c] = (r < nrows && c < no) ? a.obs[(int64_t)(r0 + r) * no + c] : 0.f;
  }
  for (int e = t; e < FA_R * 32; e += FA_THREADS) {
    const int r = e >> 5, c = e & 31;
    MID[r * PP + c] = (r < nrows && c < np) ? a.priv[(int64_t)(r0 + r) * np + c] : 0.f;
  }
  if constexpr (!ENC_ONLY)
    for (int e = t; e < FA_HW_FLOATS; e += FA_THREADS)
      HW[e] = e < HEAD_NA * HEAD_W ? a.w[nt.w4a + e] : a.w[nt.w4c + (e - HEAD_NA * HEAD_W)];
  __syncthreads();
  FA_PROF(0)
  const float* w = a.w;
  FaLayer L;
  // env_factor_encoder: priv -> enc_h0 (ELU) -> enc_h1 (ELU) -> latent, the latent into X[:, no:]
  L = FaLayer{MID, PP, 0, 32, w + nt.e1w, np, np, nt.enc_h0, 0, w + nt.e1b, BIG, FA_XP, 0, nt.enc_h0, 1, 1, 0};
  fa_layer<PRESET ? 4 : 0, false>(L);
  __syncthreads();
  FA_PROF(1)
  L = FaLayer{BIG, FA_XP, 0, nt.enc_h0, w + nt.e2w, nt.enc_h0, nt.enc_h0, nt.enc_h1, 0, w + nt.e2b, MID, EP2, 0,
              nt.enc_h1, 1, 1, (int)(a.vec >> 1) & 1};
  if (PRESET || (a.vec & 2u)) fa_layer<PRESET ? 2 : 0, true>(L);
  else fa_layer<0, false>(L);
  __syncthreads();
  FA_PROF(2)
  L = FaLayer{MID, EP2, 0, nt.enc_h1, w + nt.e3w, nt.enc_h1, nt.enc_h1, nt.latent, 0, w + nt.e3b, X, FA_XP, no,
              (nt.latent + 15) / 16 * 16, 1, 0, (int)(a.vec >> 2) & 1};
  if (PRESET || (a.vec & 4u)) fa_layer<PRESET ? 1 : 0, true>(L);
  else fa_layer<0, false>(L);
  __syncthreads();
  FA_PROF(3)
  if constexpr (ENC_ONLY) {  // (xs % 32 == 0: whole float4s of the row)
    const int q4 = a.xs >> 2;
    for (int e = t; e < nrows * q4; e += FA_THREADS) {
      const int r = e / q4, c = 4 * (e - r * q4);
      *reinterpret_cast<float4*>(a.xa_out + (int64_t)(r0 + r) * a.xs + c) = *reinterpret_cast<const float4*>(X + r * FA_XP + c);
    }
    return;
  }
  // actor / critic bodies, both at once: [obs | latent] -> 2 x ac_h0 -> 2 x ac_h1 -> 2 x ac_h2 (ELU)
  const int nx = no + nt.latent;
  L = FaLayer{X, FA_XP, 0, a.xs, w + nt.w1, nx, nx, 2 * nt.ac_h0, 0, w + nt.b1, BIG, FA_BIGP, 0, 2 * nt.ac_h0, 1, 1,
              (int)(a.vec >> 3) & 1};
  if (PRESET || (a.vec & 8u)) fa_layer<PRESET ? 16 : 0, true>(L);
  else fa_layer<0, false>(L);
  __syncthreads();
  FA_PROF(4)
  L = FaLayer{BIG, FA_BIGP, nt.ac_h0, nt.ac_h0, w + nt.w2, nt.ac_h0, nt.ac_h0, nt.ac_h1, (int64_t)nt.ac_h1 * nt.ac_h0,
              w + nt.b2, MID, FA_MIDP, 0, nt.ac_h1, 2, 1, (int)(a.vec >> 4) & 1};
  if (PRESET || (a.vec & 16u)) fa_layer<PRESET ? 8 : 0, true>(L);
  else fa_layer<0, false>(L);
  __syncthreads();
  FA_PROF(5)
  L = FaLayer{MID, FA_MIDP, nt.ac_h1, nt.ac_h1, w + nt.w3, nt.ac_h1, nt.ac_h1, nt.ac_h2, (int64_t)nt.ac_h2 * nt.ac_h1,
              w + nt.b3, BIG, FA_XP, 0, nt.ac_h2, 2, 1, (int)(a.vec >> 5) & 1};
  if (PRESET || (a.vec & 32u)) fa_layer<PRESET ? 4 : 0, true>(L);
  else fa_layer<0, false>(L);
  __syncthreads();
  FA_PROF(6)
  // heads: thread (r, j) j < na: mu; (r, na): value — sequential fmaf over k, as act_head_kernel's mu
  constexpr int NA = HEAD_NA;
  float* MU = X;  // the obs tile is dead: [16][NA + 1] mu, then log-prob terms; value in column NA
  if (t < FA_R * (NA + 1)) {
    const int r = t / (NA + 1), j = t - r * (NA + 1);
    const float* h = BIG + r * FA_XP + (j < NA ? 0 : HEAD_W);
    const float* wr = HW + j * HEAD_W;  // (row NA: w4c)
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < HEAD_W; ++k) s = fmaf(h[k], wr[k], s);
    s += j < NA ? w[nt.b4a + j] : w[nt.b4c];
    MU[r * 16 + j] = s;
  }
  __syncthreads();
  FA_PROF(7)
  const int64_t so = (int64_t)a.store_row * a.n;
  if (t < FA_R * NA) {
    const int r = t / NA, j = t - r * NA, g = r0 + r;
    if (r < nrows) {
      float e;
      if (a.eps) {
        e = a.eps[(int64_t)g * NA + j];
      } else {  // Box-Muller on the counter RNG (stream POLICY), keyed by the global env id (as act_head_kernel)
        lrl_u32x4 u = lrl_philox((uint32_t)(a.row_offset + g), (uint32_t)a.counter,
                                 (LRL_RNG_POLICY << 16) ^ (uint32_t)(a.counter >> 32), (uint32_t)(j >> 1), a.seed);
        const float u1 = fmaxf(lrl_u01(u.v[0]), 1e-7f), u2 = lrl_u01(u.v[1]);
        const float rad = sqrtf(-2.f * logf(u1)), th = 6.283185307179586f * u2;
        e = (j & 1) ? rad * sinf(th) : rad * cosf(th);
      }
      const float m = MU[r * 16 + j], sd = w[nt.std_off + j];
      const float act = m + sd * e;
      const float d = act - m;
      MU[r * 16 + j] = -(d * d) / (2.f * (sd * sd)) - logf(sd) - LOG_SQRT_2PI;
      a.actions[(int64_t)g * NA + j] = act;
      if (a.mu) a.mu[(int64_t)g * NA + j] = m;
      if (a.do_store) {
        const int64_t o = (so + g) * NA + j;
        a.store.actions[o] = act;
        a.store.mu[o] = m;
        a.store.sigma[o] = sd;
      }
    }
  }
  __syncthreads();
  if (t < nrows) {
    const int g = r0 + t;
    float lp = 0.f;
    for (int j = 0; j < NA; ++j) lp += MU[t * 16 + j];
    const float v = MU[t * 16 + NA];
    if (a.values) a.values[g] = v;
    if (a.logp) a.logp[g] = lp;
    if (a.do_store) {
      a.store.values[so + g] = v;
      a.store.logp[so + g] = lp;
    }
  }
  FA_PROF(8)
  if (a.do_store) {  // obs / priv / history rows of this tile into storage row `store_row`
    const int64_t b = so + r0;
    copy_rows(a.obs + (int64_t)r0 * no, no, a.store.obs + b * no, no, nrows, no, t);
    copy_rows(a.priv + (int64_t)r0 * np, np, a.store.priv + b * np, np, nrows, np, t);
    if (a.hist && a.store.hist) {
      const int hd = a.store.hist_dim, ld = a.store.hist_ld > hd ? a.store.hist_ld : hd;
      copy_rows(a.hist + (int64_t)r0 * hd, hd, a.store.hist + b * ld, ld, nrows, hd, t);
    }
  }
  FA_PROF(9)
}

// ---------------------------------------------------------------------------------------------------
// Adaptation head: pred = HD2 W_D3^T + b, MSE against the encoder target (F.mse_loss, mean over B*L),
// dHD2 = dpred W_D3 * elu'(HD2); partials dW_D3 [L][H], db_D3 [L], sum of squared errors.
struct AdaptHeadArgs {
  const float* hd2;  // [B][ldh]
  int ldh;
  const float* tgt;  // [B][ldt]
  int ldt;
  float* dhd2;       // [B][ldh]
  const float *w, *b;
  int B, H, L;       // hidden (32), latent (18)
  float* part;
  int part_len;      // L*H + L + 1
};

// CH / CL: the hidden / latent widths as compile-time constants (the presets' 32 / 18: the dot-product loops unroll
// and their LDS reads issue ahead of the FMA chain, same FMA order), 0 = read from the arguments
template <int CH, int CL>
__global__ __launch_bounds__(HEAD_THREADS) void adapt_head_kernel(AdaptHeadArgs a) {
  // every global load (HD2 tile, weights, the encoder targets) issued up front; the prediction dots spread over
  // (row, output) pairs; per-row squared errors summed in output order (as a sequential loop would)
  const int H = CH ? CH : a.H, L = CL ? CL : a.L;
  __shared__ float HS[HEAD_ROWS][MAX_LAT + 1];
  __shared__ float DP[HEAD_ROWS][MAX_LAT + 1];
  __shared__ float WS[MAX_LAT][MAX_LAT + 1];
  __shared__ float TG[HEAD_ROWS][MAX_LAT + 1];  // targets, then squared errors
  __shared__ float ERR[HEAD_ROWS];
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * HEAD_ROWS;
  const int nrows = min(HEAD_ROWS, a.B - r0);
  for (int i = t; i < HEAD_ROWS * H; i += HEAD_THREADS) {
    const int r = i / H, c = i - r * H;
    HS[r][c] = r < nrows ? a.hd2[(int64_t)(r0 + r) * a.ldh + c] : 0.f;
  }
  for (int i = t; i < L * H; i += HEAD_THREADS) WS[i / H][i % H] = a.w[i];
  for (int i = t; i < HEAD_ROWS * L; i += HEAD_THREADS) {
    const int r = i / L, j = i - r * L;
    TG[r][j] = r < nrows ? a.tgt[(int64_t)(r0 + r) * a.ldt + j] : 0.f;
  }
  __syncthreads();
  const float scale = 2.f / ((float)a.B * (float)L);
  for (int i = t; i < HEAD_ROWS * L; i += HEAD_THREADS) {
    const int r = i / L, j = i - r * L;
    float d = 0.f;
    if (r < nrows) {
      float s = 0.f;
      for (int k = 0; k < H; ++k) s = fmaf(HS[r][k], WS[j][k], s);
      const float pred = s + a.b[j];
      d = pred - TG[r][j];
    }
    TG[r][j] = d * d;
    DP[r][j] = scale * d;
  }
  __syncthreads();
  if (t < HEAD_ROWS) {
    float e = 0.f;
    for (int j = 0; j < L; ++j) e += TG[t][j];
    ERR[t] = e;
  }
  __syncthreads();
  float* P = a.part + (int64_t)blockIdx.x * a.part_len;
  // dHD2 (thread = (row, k) pairs)
  for (int i = t; i < nrows * H; i += HEAD_THREADS) {
    const int r = i / H, k = i - r * H;
    float s = 0.f;
    for (int j = 0; j < L; ++j) s = fmaf(DP[r][j], WS[j][k], s);
    a.dhd2[(int64_t)(r0 + r) * a.ldh + k] = s * delu(HS[r][k]);
  }
  // dW_D3 partial (thread = (j, k)); the specialised form runs over every row of the tile (rows past nrows hold
  // DP = 0 and ERR = 0, so they add exact zeros) so that the row loops unroll
  const int nr = CH ? HEAD_ROWS : nrows;
  for (int i = t; i < L * H; i += HEAD_THREADS) {
    const int j = i / H, k = i - j * H;
    float s = 0.f;
    for (int r = 0; r < nr; ++r) s = fmaf(DP[r][j], HS[r][k], s);
    P[i] = s;
  }
  if (t < L) {
    float s = 0.f;
    for (int r = 0; r < nr; ++r) s += DP[r][t];
    P[L * H + t] = s;
  } else if (t == 64) {
    float s = 0.f;
    for (int r = 0; r < nr; ++r) s += ERR[r];
    P[L * H + L] = s;
  }
}

// ---------------------------------------------------------------------------------------------------
// Segmented reduction of partial slices: dst[i] = scale * sum_p src[p * stride + i] (fixed order).
struct Seg {
  const float* src;
  float* dst;
  int64_t len, stride;
  int parts;
  float scale;
  int lpg;      // log2 of the part groups a workgroup splits the parts into (set by launch_seg)
  int blk0, nblk;  // this segment's workgroups in the packed 1-D grid (set by launch_seg)
};
constexpr int MAX_SEGS = 24;
struct SegList {
  Seg s[MAX_SEGS];
  int n;
};

// dst[i] = scale * sum_q src[q * stride + i].  A 256-thread workgroup covers E = 256 / PG consecutive
// elements with PG part groups: thread (g, e) sums parts g, g + PG, ... (8 loads in flight, coalesced over e),
// then group 0 adds the PG partial sums in group order — a fixed order, so the result is deterministic.
// Few-element / many-part segments (per-workgroup head partials, thin weight gradients) use large PG.
__global__ __launch_bounds__(256) void seg_reduce_kernel(SegList L) {
  int si = 0;
  while (si + 1 < L.n && (int)blockIdx.x >= L.s[si + 1].blk0) ++si;
  const Seg& sg = L.s[si];
  const int lpg = sg.lpg, pg = 1 << lpg, E = 256 >> lpg;
  const int e = threadIdx.x & (E - 1), g = threadIdx.x >> (8 - lpg);
  __shared__ float red[256];
  for (int64_t base = (int64_t)(blockIdx.x - sg.blk0) * E; base < sg.len; base += (int64_t)sg.nblk * E) {
    const int64_t i = base + e;
    float acc = 0.f;
    if (i < sg.len) {
      const float* p = sg.src + i;
      int q = g;
      for (; q + 7 * pg < sg.parts; q += 8 * pg) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(q + u * pg) * sg.stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
      }
      for (; q < sg.parts; q += pg) acc += p[(int64_t)q * sg.stride];
    }
    if (pg == 1) {
      if (i < sg.len) sg.dst[i] = acc * sg.scale;
      continue;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (g == 0 && i < sg.len) {
      float t = 0.f;
      for (int k = 0; k < pg; ++k) t += red[k * E + e];
      sg.dst[i] = t * sg.scale;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------
// clip_grad_norm_ (torch.nn.utils.clip_grad_norm_): sum of squares partials, fp64
constexpr int NORM_BLOCKS = 256;
__global__ void sumsq_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = g[i];
    s += x * x;
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// adaptive learning rate (ppo.py:110-124), clip coefficient, Adam step size, loss bookkeeping
__global__ void ppo_finalize_kernel(const double* __restrict__ part, int nparts, const float* __restrict__ kl_slot,
                                    float grad_scale, float max_norm, float desired_kl, int adaptive, double bc1,
                                    float inv_B, lrl_ppo_ctrl* ctrl) {
  __shared__ double red[64];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  double tot = 0.0;
  for (int i = 0; i < 64; ++i) tot += red[i];
  const float total_norm = (float)sqrt(tot) * grad_scale;
  float clip = max_norm / (total_norm + 1e-6f);
  clip = fminf(clip, 1.f);
  double lr = ctrl->lr;
  const float kl = kl_slot[0] * grad_scale;
  if (adaptive) {
    const double k = (double)kl;
    if (k > (double)desired_kl * 2.0) lr = fmax(1e-5, lr / 1.5);
    else if (k < (double)desired_kl / 2.0 && k > 0.0) lr = fmin(1e-2, lr * 1.5);
  }
  ctrl->lr = lr;
  ctrl->mb[3] = kl;
  ctrl->clip_scale = clip;
  ctrl->total_norm = total_norm;
  ctrl->step_size = (float)(lr / bc1);
  ctrl->loss_sum[0] += (double)ctrl->mb[0];
  ctrl->loss_sum[1] += (double)ctrl->mb[1];
}

// torch.optim.Adam (foreach, no weight decay / amsgrad):
//   m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2; p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float grad_scale, const lrl_ppo_ctrl* __restrict__ ctrl,
                            float step_size_host, float one_minus_b1, float b2, float one_minus_b2, float bc2_sqrt,
                            float eps, lrl_ppo_ctrl* acc_ctrl) {
  const float clip = ctrl ? ctrl->clip_scale : 1.f;
  const float step = ctrl ? ctrl->step_size : step_size_host;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * grad_scale;
    gi = gi * clip;
    float mi = m[i];
    mi = mi + one_minus_b1 * (gi - mi);
    float vi = v[i] * b2;
    vi = vi + one_minus_b2 * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (-step) * (mi / denom);
  }
  if (acc_ctrl && blockIdx.x == 0 && threadIdx.x == 0) acc_ctrl->loss_sum[2] += (double)acc_ctrl->mb[2];
}

// ---------------------------------------------------------------------------------------------------
// W[r][0:h) -> Wp[r][0:hp) with zero columns [h, hp): the adaptation module's first layer over history rows
// stored at the padded pitch hp (the k-padding contributes exact zeros)
__global__ void pad_cols_kernel(const float* __restrict__ W, int rows, int h, int hp, float* __restrict__ Wp) {
  const int64_t n = (int64_t)rows * hp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / hp), c = (int)(i - (int64_t)r * hp);
    Wp[i] = c < h ? W[(int64_t)r * h + c] : 0.f;
  }
}

// host side: workspace plan
struct Plan {
  int B;
  float *xa, *he1, *he2, *h1, *h2, *h3, *dh3, *dh2, *dh1, *dlat, *dhe2, *dhe1;
  float *tgt, *hd1, *hd2, *dhd2, *dhd1;
  float* wd1p;     // adaptation layer-1 weights at the padded history pitch (zero columns past num_hist)
  float* part;     // partial area (reused by phases 1 and 3)
  int64_t part_floats;
  uint16_t* wpl;   // pre-split weight planes (x6p products): the caller's jobs, built once per call
  int64_t bytes;
};

// The weight products of the update that run on the x6p kernel (pre-split B, csrc/lrl_gemm.hip): their planes are
// split from the current parameters at the start of each forward_backward / adaptation call (one launch).
enum MainPlane { PL_W1, PL_W2, PL_W3, PL_E2, PL_W2T, PL_W3T, PL_E2T, PL_MAIN };
enum AdaptPlane { PL_D1, PL_AE2, PL_D2T, PL_ADAPT };
static int hist_pad(int h);
static int xs_of(const lrl_ppo_net& n);
// main: forward W1 (k padded to X's pitch), W2, W3, the encoder's W2; backward-data W2^T, W3^T, encoder W2^T
static void main_plane_jobs(const lrl_ppo_net& n, const float* w, uint16_t* base, PlaneJob (&j)[PL_MAIN]) {
  const int h0 = n.ac_h0, h1 = n.ac_h1, h2 = n.ac_h2, nx = n.num_obs + n.latent;
  auto set = [&](PlaneJob& q, int64_t off, int rows, int cols, int64_t ldw, int trans, int groups, int64_t gsrc) {
    q.W = w ? w + off : nullptr; q.rows = rows; q.cols = cols; q.ldw = ldw; q.trans = trans; q.groups = groups;
    q.gsrc = gsrc;
  };
  set(j[PL_W1], n.w1, 2 * h0, nx, nx, 0, 1, 0);
  set(j[PL_W2], n.w2, h1, h0, h0, 0, 2, (int64_t)h1 * h0);
  set(j[PL_W3], n.w3, h2, h1, h1, 0, 2, (int64_t)h2 * h1);
  set(j[PL_E2], n.e2w, n.enc_h1, n.enc_h0, n.enc_h0, 0, 1, 0);
  set(j[PL_W2T], n.w2, h1, h0, h0, 1, 2, (int64_t)h1 * h0);
  set(j[PL_W3T], n.w3, h2, h1, h1, 1, 2, (int64_t)h2 * h1);
  set(j[PL_E2T], n.e2w, n.enc_h1, n.enc_h0, n.enc_h0, 1, 1, 0);
  int64_t off = 0;
  for (auto& q : j) {
    q.dst = base ? base + off : nullptr;
    off += (plane_elems(q) + 127) / 128 * 128;
  }
}
// adaptation: forward Wd1 (k padded to the history pitch), the encoder-target W2 (from `we`), backward-data Wd2^T
static void adapt_plane_jobs(const lrl_ppo_net& n, const float* w, const float* we, uint16_t* base,
                             PlaneJob (&j)[PL_ADAPT]) {
  auto set = [&](PlaneJob& q, const float* src, int rows, int cols, int64_t ldw, int trans) {
    q.W = src; q.rows = rows; q.cols = cols; q.ldw = ldw; q.trans = trans; q.groups = 1; q.gsrc = 0;
  };
  set(j[PL_D1], w ? w + n.d1w : nullptr, n.ad_h0, n.num_hist, n.num_hist, 0);
  set(j[PL_AE2], we ? we + n.e2w : nullptr, n.enc_h1, n.enc_h0, n.enc_h0, 0);
  set(j[PL_D2T], w ? w + n.d2w : nullptr, n.ad_h1, n.ad_h0, n.ad_h0, 1);
  int64_t off = 0;
  for (auto& q : j) {
    q.dst = base ? base + off : nullptr;
    off += (plane_elems(q) + 127) / 128 * 128;
  }
}
static int64_t plane_area_elems(const lrl_ppo_net& n) {
  PlaneJob a[PL_MAIN], b[PL_ADAPT];
  main_plane_jobs(n, nullptr, nullptr, a);
  adapt_plane_jobs(n, nullptr, nullptr, nullptr, b);
  int64_t m = 0, d = 0;
  for (auto& q : a) m += (plane_elems(q) + 127) / 128 * 128;
  for (auto& q : b) d += (plane_elems(q) + 127) / 128 * 128;
  return std::max(m, d);
}

// X = [obs | latent] row pitch: 64 for the blind policies (42 + 18), else rounded up to 16 floats (a height-scan
// policy: 235 + 18 -> 256).  Columns nx..XS-1 are zero.
static int xs_of(const lrl_ppo_net& n) {
  const int nx = n.num_obs + n.latent;
  return nx <= 64 ? 64 : (nx + 15) / 16 * 16;
}
constexpr int LATS = 32;    // latent-wide buffers pitch
constexpr int HD2S = 32;    // adaptation hidden-2 pitch

static int hist_pad(int h) { return (h + 15) / 16 * 16; }

static int64_t tn_part_floats(int M, int N, int K, int groups) {
  const int s = gemm_pick_splits(M, N, K, groups);
  return (int64_t)s * groups * ((int64_t)M * N + M);
}

static Plan make_plan(const lrl_ppo_net& n, int B, char* base) {
  Plan p;
  p.B = B;
  int64_t off = 0;
  auto take = [&](int64_t floats) {
    float* r = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((floats * 4 + 255) / 256) * 256;
    return r;
  };
  const int64_t Bl = B;
  p.xa = take(Bl * xs_of(n));
  p.he1 = take(Bl * n.enc_h0);
  p.he2 = take(Bl * n.enc_h1);
  p.h1 = take(Bl * 2 * n.ac_h0);
  p.h2 = take(Bl * 2 * n.ac_h1);
  p.h3 = take(Bl * 2 * n.ac_h2);
  p.dh3 = take(Bl * 2 * n.ac_h2);
  p.dh2 = take(Bl * 2 * n.ac_h1);
  p.dh1 = take(Bl * 2 * n.ac_h0);
  p.dlat = take(Bl * LATS);
  p.dhe2 = take(Bl * n.enc_h1);
  p.dhe1 = take(Bl * n.enc_h0);
  p.tgt = take(Bl * LATS);
  p.hd1 = take(Bl * n.ad_h0);
  p.hd2 = take(Bl * HD2S);
  p.dhd2 = take(Bl * HD2S);
  p.dhd1 = take(Bl * n.ad_h0);
  p.wd1p = take((int64_t)n.ad_h0 * hist_pad(n.num_hist));
  const int hb = (B + HEAD_ROWS - 1) / HEAD_ROWS;
  int64_t ph1 = tn_part_floats(n.ac_h2, n.ac_h1, B, 2) + tn_part_floats(n.ac_h1, n.ac_h0, B, 2) +
                tn_part_floats(2 * n.ac_h0, n.num_obs + n.latent, B, 1) + tn_part_floats(n.latent, n.enc_h1, B, 1) +
                tn_part_floats(n.enc_h1, n.enc_h0, B, 1) + tn_part_floats(n.enc_h0, n.num_priv, B, 1) +
                (int64_t)hb * hp_len(n.num_actions) + 64 * 8;
  int64_t ph3 = tn_part_floats(n.ad_h1, n.ad_h0, B, 1) + tn_part_floats(n.ad_h0, n.num_hist, B, 1) +
                (int64_t)hb * (n.latent * n.ad_h1 + n.latent + 1) + 64 * 4;
  p.part_floats = std::max(ph1, ph3);
  p.part = take(p.part_floats);
  p.wpl = reinterpret_cast<uint16_t*>(take((plane_area_elems(n) + 1) / 2));
  p.bytes = off;
  return p;
}

static int check_net(const lrl_ppo_net* n) {
  if (!n) return lrl_set_error(LRL_E_INVALID, "lrl_ppo: null net");
  if (n->ac_h2 != HEAD_W) return lrl_set_error(LRL_E_INVALID, "lrl_ppo: last actor/critic hidden width must be 128");
  if (n->num_actions != HEAD_NA) return lrl_set_error(LRL_E_INVALID, "lrl_ppo: num_actions must be 12");
  if (n->latent > MAX_LAT || n->ad_h1 > MAX_LAT) return lrl_set_error(LRL_E_INVALID, "lrl_ppo: latent/adaptation widths > 32");
  return 0;
}

static void launch_seg(const SegList& L, hipStream_t st);

// Optional timing of the update's largest product (the actor/critic layer-2 weight gradient, 2 x 256x512
// over the minibatch rows): HIP events around that launch on its stream, read back by lrl_ppo_timing_read.
struct GemmTimer {
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t used = 0;
};
static GemmTimer g_timer;
static hipEvent_t timer_event() {
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
static void timer_begin(hipStream_t st) {
  if (!g_timer.on) return;
  if (g_timer.used == g_timer.ev.size()) g_timer.ev.emplace_back(timer_event(), timer_event());
  auto& pr = g_timer.ev[g_timer.used];
  if (pr.first) (void)hipEventRecord(pr.first, st);
}
static void timer_end(hipStream_t st) {
  if (!g_timer.on) return;
  auto& pr = g_timer.ev[g_timer.used++];
  if (pr.second) (void)hipEventRecord(pr.second, st);
}

// one GEMM helper per layout
struct G {
  hipStream_t st;
  float* part_end;  // end of the partial area: a product that would not fit is refused before launch
  int rc = 0;
  const PlaneJob* pl = nullptr;  // pre-split B of the next nt / nn product (consumed by it)
  G& with(const PlaneJob& j) {
    pl = &j;
    return *this;
  }
  void take_planes(GemmP& p) {
    if (pl) gemm_use_planes(p, *pl);
    pl = nullptr;
  }
  void nt(const float* A, int64_t lda, const int64_t* rows, const float* W, int64_t ldw, float* C, int64_t ldc,
          const float* bias, int M, int N, int K, bool elu, int groups = 1, int64_t ga = 0, int64_t gw = 0,
          int64_t gc = 0, int64_t gbias = 0) {
    if (rc) return;
    GemmP p{};
    p.A = A; p.lda = lda; p.a_rows = rows; p.B = W; p.ldb = ldw; p.C = C; p.ldc = ldc; p.bias = bias;
    p.M = M; p.N = N; p.K = K; p.splits = 1;
    p.ga = ga; p.gb = gw; p.gc = gc; p.gbias = gbias;
    take_planes(p);
    rc = gemm_launch(p, GEMM_NT, elu ? EPI_BIAS_ELU : EPI_BIAS, groups, st);
  }
  // dX = dY W (* elu'(aux) if aux)
  void nn(const float* dY, int64_t ldy, const float* W, int64_t ldw, float* dX, int64_t ldx, const float* aux,
          int64_t ldaux, int M, int N, int K, int groups = 1, int64_t gy = 0, int64_t gw = 0, int64_t gx = 0,
          int64_t gaux = 0) {
    if (rc) return;
    GemmP p{};
    p.A = dY; p.lda = ldy; p.B = W; p.ldb = ldw; p.C = dX; p.ldc = ldx; p.aux = aux; p.ld_aux = ldaux;
    p.M = M; p.N = N; p.K = K; p.splits = 1;
    p.ga = gy; p.gb = gw; p.gc = gx; p.gaux = gaux;
    take_planes(p);
    rc = gemm_launch(p, GEMM_NN, aux ? EPI_DELU : EPI_STORE, groups, st);
  }
  // partial dW[o][i] = sum_b dY[b][o] X[rows(b)][i]; returns the segments (weights then biases)
  void tn(const float* dY, int64_t ldy, const float* X, int64_t ldx, const int64_t* rows, int M, int N, int K,
          int groups, int64_t gy, int64_t gx, float*& part, float* dw, float* db, SegList& L) {
    if (rc) return;
    const int splits = gemm_pick_splits(M, N, K, groups);
    if (part + (int64_t)splits * groups * ((int64_t)M * N + M) > part_end) { rc = LRL_E_INVALID; return; }
    GemmP p{};
    p.A = dY; p.lda = ldy; p.B = X; p.ldb = ldx; p.b_rows = rows;
    p.M = M; p.N = N; p.K = K; p.splits = splits; p.kps = (K + splits - 1) / splits;
    p.ga = gy; p.gb = gx; p.gc = (int64_t)M * N; p.ldc = N;
    p.part_stride = (int64_t)groups * M * N;
    p.C = part;
    p.bias_part = part + (int64_t)splits * groups * M * N;
    rc = gemm_launch(p, GEMM_TN, EPI_PARTIAL, groups, st);
    if (rc) return;
    if (L.n + 2 > MAX_SEGS) { rc = LRL_E_INVALID; return; }
    L.s[L.n++] = Seg{part, dw, (int64_t)groups * M * N, (int64_t)groups * M * N, splits, 1.f};
    L.s[L.n++] = Seg{p.bias_part, db, (int64_t)groups * M, (int64_t)groups * M, splits, 1.f};
    part = p.bias_part + (int64_t)splits * groups * M;
    part = reinterpret_cast<float*>(((reinterpret_cast<uintptr_t>(part) + 255) / 256) * 256);
  }
};

// The env-factor encoder's backward chain (five small products at the minibatch's rows, latency-bound) runs on a
// second stream of the library's own, beside the actor / critic weight gradients of the same minibatch (they share no
// buffer: the chain reads dlat / he1 / he2 / priv and the weights, writes dhe1 / dhe2 and its own partial slices).
// One stream and two events per device, created on first use.  LRL_PPO_FORK=0 keeps everything on the caller's stream.
struct Fork {
  hipStream_t st = nullptr;
  hipEvent_t go = nullptr, done = nullptr;
};
// The fork lives on the device of the caller's stream (hipStreamGetDevice; the null stream means the current device),
// and each device's fork is created once under a mutex, so concurrent first calls do not race.  Host threads sharing a
// device share its fork: the stream is in order, so a later `done` record still covers an earlier caller's chain (at
// worst a caller waits for more work than its own).
static Fork* fork_for_device(hipStream_t caller) {
  static const bool on = [] {
    const char* e = getenv("LRL_PPO_FORK");
    return !(e && e[0] == '0');
  }();
  if (!on) return nullptr;
  static Fork forks[64];
  static std::mutex mu;
  int dev = 0;
  if (caller) {
    hipDevice_t d = 0;
    if (hipStreamGetDevice(caller, &d) != hipSuccess) return nullptr;
    dev = (int)d;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    return nullptr;
  }
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  Fork& f = forks[dev];
  if (!f.st) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    const bool sw = cur != dev;  // stream and events are created on the caller's device
    if (sw && hipSetDevice(dev) != hipSuccess) return nullptr;
    Fork nf;
    const bool ok = hipStreamCreateWithFlags(&nf.st, hipStreamNonBlocking) == hipSuccess &&
                    hipEventCreateWithFlags(&nf.go, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&nf.done, hipEventDisableTiming) == hipSuccess;
    if (sw) (void)hipSetDevice(cur);
    if (!ok) return nullptr;
    f = nf;
  }
  return &f;
}

static void launch_seg(const SegList& L0, hipStream_t st) {
  SegList L = L0;
  int total = 0;
  for (int i = 0; i < L.n; ++i) {
    Seg& s = L.s[i];
    // split the parts over more groups while the segment's grid is small and each group keeps >= 4 parts
    int lpg = 0;
    while (lpg < 6 && (4 << (lpg + 1)) <= s.parts && (s.len << lpg) < 2048 * 256) ++lpg;
    s.lpg = lpg;
    s.nblk = (int)std::min<int64_t>((s.len + (256 >> lpg) - 1) / (256 >> lpg), 2048);
    s.blk0 = total;
    total += s.nblk;
  }
  if (total > 0) hipLaunchKernelGGL(seg_reduce_kernel, dim3(total), dim3(256), 0, st, L);
}

}  // namespace lrl

using namespace lrl;

// rollout forward workspace: X [n][64], HE1, HE2, H1 [n][2 h0], H2, H3
struct ActPlan {
  float *xa, *he1, *he2, *h1, *h2, *h3;
  uint16_t* wpl;  // forward weight planes (LRL_ACT_PLANES=1: the x6p kernel for the act's weight products)
  int64_t bytes;
};
// the forward jobs of main_plane_jobs (PL_W1 .. PL_E2) are the act's weight products
constexpr int PL_FWD = PL_E2 + 1;
static bool act_planes_on() {
  const char* e = getenv("LRL_ACT_PLANES");  // (read per call: A/B timing in one process)
  return e && e[0] == '1' && gemm_x6p_enabled();
}
static ActPlan make_act_plan(const lrl_ppo_net& n, int rows, char* base) {
  ActPlan p;
  int64_t off = 0;
  auto take = [&](int64_t floats) {
    float* r = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((floats * 4 + 255) / 256) * 256;
    return r;
  };
  const int64_t R = rows;
  p.xa = take(R * xs_of(n));
  p.he1 = take(R * n.enc_h0);
  p.he2 = take(R * n.enc_h1);
  p.h1 = take(R * 2 * n.ac_h0);
  p.h2 = take(R * 2 * n.ac_h1);
  p.h3 = take(R * 2 * n.ac_h2);
  {
    PlaneJob j[PL_MAIN];
    main_plane_jobs(n, nullptr, nullptr, j);
    int64_t e = 0;
    for (int i = 0; i < PL_FWD; ++i) e += (plane_elems(j[i]) + 127) / 128 * 128;
    p.wpl = reinterpret_cast<uint16_t*>(take((e + 1) / 2));
  }
  p.bytes = off;
  return p;
}

// The fused act's envelope (LDS pitches, tile runs that never cross a group); LRL_ACT_FUSED=1 selects it over the GEMM chain
// (A/B timing and the tests that compare the two)
// the encoder part of act_fused_kernel in the rollout act's chain (LRL_ACT_ENC_FUSED=0: the prep kernel + three
// GEMM launches instead; read per call so a test can switch it inside one process)
static bool act_enc_fused(const lrl_ppo_net& n) {
  const char* e = getenv("LRL_ACT_ENC_FUSED");
  if (e && e[0] == '0') return false;
  auto run_ok = [](int Ng) {
    if (Ng % 16) return false;
    const int T = Ng / 16, tpw = T >= 4 ? T / 4 : 1;
    if (T >= 4 && T % 4) return false;
    return T % std::min(tpw, 8) == 0;
  };
  return xs_of(n) % 32 == 0 && xs_of(n) <= 256 && n.num_priv <= 32 && n.enc_h0 <= 256 && n.enc_h0 % 32 == 0 &&
         n.enc_h1 % 32 == 0 && n.enc_h1 + 4 <= FA_ENC_MIDP && n.latent <= 32 && run_ok(n.enc_h0) && run_ok(n.enc_h1) &&
         run_ok((n.latent + 15) / 16 * 16);
}

static bool fused_act_fits(const lrl_ppo_net& n) {
  const char* e = getenv("LRL_ACT_FUSED");  // (read per call: a test switches it inside one process)
  if (!(e && e[0] == '1')) return false;  // off by default until it measures faster than the chain
  auto run_ok = [](int groups, int Ng) {  // fa_layer: equal runs per wave inside one group
    if (Ng % 16) return false;
    const int T = groups * (Ng / 16), tpg = Ng / 16;
    const int tpw = T >= 4 ? T / 4 : 1;
    if (T >= 4 && T % 4) return false;
    return tpg % std::min(tpw, 8) == 0;
  };
  return xs_of(n) % 32 == 0 && n.enc_h0 % 32 == 0 && n.enc_h1 % 32 == 0 && n.ac_h0 % 32 == 0 && n.ac_h1 % 32 == 0 &&
         n.num_priv <= 32 && n.enc_h0 <= 256 && n.enc_h1 + 4 <= FA_MIDP && n.latent <= 32 && xs_of(n) <= 256 &&
         2 * n.ac_h0 <= 1024 && 2 * n.ac_h1 <= 512 && 2 * n.ac_h2 <= 256 && n.enc_h0 % 16 == 0 && n.enc_h1 % 16 == 0 &&
         n.ac_h0 % 16 == 0 && n.ac_h1 % 16 == 0 && run_ok(1, n.enc_h0) && run_ok(1, n.enc_h1) &&
         run_ok(1, (n.latent + 15) / 16 * 16) && run_ok(1, 2 * n.ac_h0) && run_ok(2, n.ac_h1) && run_ok(2, n.ac_h2);
}

extern "C" int64_t lrl_ppo_act_workspace_bytes(const lrl_ppo_net* net, int32_t n) {
  if (check_net(net) || n <= 0) return -1;
  return make_act_plan(*net, n, nullptr).bytes;
}

extern "C" int lrl_debug_act_profile(unsigned long long* out, int reset) {
#ifdef LRL_ACT_PROFILE
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_act_prof), sizeof(unsigned long long) * 12) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[12] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_act_prof), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 12;
#else
  (void)out;
  (void)reset;
  return 0;
#endif
}

extern "C" int32_t lrl_ppo_act(const lrl_ppo_net* net, const float* params, const float* obs, const float* priv,
                               const float* hist, int32_t n, const float* eps, uint64_t seed, uint64_t counter,
                               int64_t row_offset, float* actions, float* mu, float* values, float* logp, const lrl_rollout_store* store,
                               int32_t store_row, void* workspace, void* stream) {
  if (int rc = check_net(net)) return rc;
  if (!params || !obs || !priv || !actions || !workspace || n <= 0)
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_act: null argument or n <= 0");
  if (store && (!store->obs || !store->priv || !store->actions || !store->values || !store->logp || !store->mu ||
                !store->sigma || store->hist_dim < 0 || (store->hist_ld != 0 && store->hist_ld < store->hist_dim)))
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_act: incomplete rollout store");
  const lrl_ppo_net& nt = *net;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (fused_act_fits(nt)) {  // one launch: act_fused_kernel
    static const bool ok = [] {
      auto set = [](const void* f) {
        return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, FA_LDS_FLOATS * sizeof(float)) ==
               hipSuccess;
      };
      return set(reinterpret_cast<const void*>(act_fused_kernel<true>)) &&
             set(reinterpret_cast<const void*>(act_fused_kernel<false>));
    }();
    if (!ok) return lrl_set_error(LRL_E_HIP, "lrl_ppo_act: fused kernel LDS attribute");
    FusedActArgs fa{};
    fa.w = params; fa.net = nt; fa.obs = obs; fa.priv = priv; fa.hist = hist; fa.eps = eps;
    fa.n = n; fa.xs = xs_of(nt);
    auto al = [&](int64_t off, int ld) { return ((reinterpret_cast<uintptr_t>(params + off) & 15) == 0 && ld % 4 == 0); };
    const int nx = nt.num_obs + nt.latent;
    fa.vec = (al(nt.e2w, nt.enc_h0) ? 2u : 0u) | (al(nt.e3w, nt.enc_h1) ? 4u : 0u) | (al(nt.w1, nx) ? 8u : 0u) |
             (al(nt.w2, nt.ac_h0) ? 16u : 0u) | (al(nt.w3, nt.ac_h1) ? 32u : 0u);
    fa.seed = seed; fa.counter = counter; fa.row_offset = row_offset;
    fa.actions = actions; fa.mu = mu; fa.values = values; fa.logp = logp;
    if (store) fa.store = *store;
    fa.store_row = store_row; fa.do_store = store ? 1 : 0;
    const bool preset = nt.enc_h0 == 256 && nt.enc_h1 == 128 && nt.latent <= 32 && nt.ac_h0 == 512 && nt.ac_h1 == 256 &&
                        nt.ac_h2 == 128 && fa.vec == 62u;
    if (preset)
      hipLaunchKernelGGL(act_fused_kernel<true>, dim3((n + FA_R - 1) / FA_R), dim3(FA_THREADS),
                         FA_LDS_FLOATS * sizeof(float), st, fa);
    else
      hipLaunchKernelGGL(act_fused_kernel<false>, dim3((n + FA_R - 1) / FA_R), dim3(FA_THREADS),
                         FA_LDS_FLOATS * sizeof(float), st, fa);
    return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_act: launch failed");
  }
  ActPlan P = make_act_plan(nt, n, static_cast<char*>(workspace));
  G g{st, nullptr};
  const float* w = params;
  const int nx = nt.num_obs + nt.latent, XS = xs_of(nt);
  PlaneJob pj[PL_MAIN];
  main_plane_jobs(nt, w, P.wpl, pj);
  if (act_planes_on()) {
    if (int rc = x6_planes_launch(pj, PL_FWD, st)) return lrl_set_error(rc, "lrl_ppo_act: planes launch failed");
  } else {
    for (auto& q : pj) q.dst = nullptr;
  }
  if (act_enc_fused(nt)) {  // X = [obs | encoder(priv) | 0] in one launch (act_fused_kernel<., true>)
    FusedActArgs fa{};
    fa.w = params; fa.net = nt; fa.obs = obs; fa.priv = priv; fa.n = n; fa.xs = XS; fa.xa_out = P.xa;
    auto al = [&](int64_t off, int ld) { return ((reinterpret_cast<uintptr_t>(params + off) & 15) == 0 && ld % 4 == 0); };
    fa.vec = (al(nt.e2w, nt.enc_h0) ? 2u : 0u) | (al(nt.e3w, nt.enc_h1) ? 4u : 0u);
    const bool preset = nt.enc_h0 == 256 && nt.enc_h1 == 128 && nt.latent <= 32 && fa.vec == 6u;
    if (preset)
      hipLaunchKernelGGL((act_fused_kernel<true, true>), dim3((n + FA_R - 1) / FA_R), dim3(FA_THREADS),
                         FA_ENC_LDS_FLOATS * sizeof(float), st, fa);
    else
      hipLaunchKernelGGL((act_fused_kernel<false, true>), dim3((n + FA_R - 1) / FA_R), dim3(FA_THREADS),
                         FA_ENC_LDS_FLOATS * sizeof(float), st, fa);
  } else {
    hipLaunchKernelGGL(ppo_prep_kernel, dim3(prep_blocks(n, XS)), dim3(256), 0, st, obs,
                       (const int64_t*)nullptr, n, nt.num_obs, XS, P.xa);
    g.nt(priv, nt.num_priv, nullptr, w + nt.e1w, nt.num_priv, P.he1, nt.enc_h0, w + nt.e1b, n, nt.enc_h0, nt.num_priv,
         true);
    g.with(pj[PL_E2]).nt(P.he1, nt.enc_h0, nullptr, w + nt.e2w, nt.enc_h0, P.he2, nt.enc_h1, w + nt.e2b, n, nt.enc_h1,
                         nt.enc_h0, true);
    g.nt(P.he2, nt.enc_h1, nullptr, w + nt.e3w, nt.enc_h1, P.xa + nt.num_obs, XS, w + nt.e3b, n, nt.latent, nt.enc_h1,
         false);
  }
  g.with(pj[PL_W1]).nt(P.xa, XS, nullptr, w + nt.w1, nx, P.h1, 2 * nt.ac_h0, w + nt.b1, n, 2 * nt.ac_h0, XS, true);
  g.with(pj[PL_W2]).nt(P.h1, 2 * nt.ac_h0, nullptr, w + nt.w2, nt.ac_h0, P.h2, 2 * nt.ac_h1, w + nt.b2, n, nt.ac_h1,
                       nt.ac_h0, true, 2, nt.ac_h0, (int64_t)nt.ac_h1 * nt.ac_h0, nt.ac_h1, nt.ac_h1);
  g.with(pj[PL_W3]).nt(P.h2, 2 * nt.ac_h1, nullptr, w + nt.w3, nt.ac_h1, P.h3, 2 * nt.ac_h2, w + nt.b3, n, nt.ac_h2,
                       nt.ac_h1, true, 2, nt.ac_h1, (int64_t)nt.ac_h2 * nt.ac_h1, nt.ac_h2, nt.ac_h2);
  if (g.rc) return lrl_set_error(g.rc, "lrl_ppo_act: GEMM launch failed");
  ActHeadArgs ah{};
  ah.h3 = P.h3; ah.w4a = w + nt.w4a; ah.b4a = w + nt.b4a; ah.w4c = w + nt.w4c; ah.b4c = w + nt.b4c;
  ah.stdv = w + nt.std_off; ah.obs = obs; ah.priv = priv; ah.hist = hist; ah.eps = eps;
  ah.n = n; ah.na = nt.num_actions; ah.no = nt.num_obs; ah.np = nt.num_priv; ah.seed = seed; ah.counter = counter;
  ah.row_offset = row_offset;
  ah.actions = actions; ah.mu = mu; ah.values = values; ah.logp = logp;
  if (store) ah.store = *store;
  ah.store_row = store_row; ah.do_store = store ? 1 : 0;
  hipLaunchKernelGGL(act_head_kernel, dim3((n + ACT_ROWS - 1) / ACT_ROWS), dim3(HEAD_THREADS), 0, st, ah);
  return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_act: launch failed");
}

// ---- student act (actor_critic.py:160-164): latent = adaptation_module(hist), mean = actor_body([obs, latent]) ----
struct StudentPlan {
  float *xa, *hd1, *hd2, *h1, *h2, *h3, *wd1p;
  int64_t bytes;
};
static StudentPlan make_student_plan(const lrl_ppo_net& n, int rows, char* base) {
  StudentPlan p;
  int64_t off = 0;
  auto take = [&](int64_t floats) {
    float* r = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += ((floats * 4 + 255) / 256) * 256;
    return r;
  };
  const int64_t R = rows;
  p.xa = take(R * xs_of(n));
  p.hd1 = take(R * n.ad_h0);
  p.hd2 = take(R * HD2S);
  p.h1 = take(R * n.ac_h0);
  p.h2 = take(R * n.ac_h1);
  p.h3 = take(R * n.ac_h2);
  p.wd1p = take((int64_t)n.ad_h0 * hist_pad(n.num_hist));
  p.bytes = off;
  return p;
}

extern "C" int64_t lrl_ppo_act_student_workspace_bytes(const lrl_ppo_net* net, int32_t n) {
  if (check_net(net) || n <= 0) return -1;
  return make_student_plan(*net, n, nullptr).bytes;
}

extern "C" int32_t lrl_ppo_act_student(const lrl_ppo_net* net, const float* params, const float* obs,
                                       const float* hist, int32_t hist_ld, int32_t n, float* mean, float* latent,
                                       void* workspace, void* stream) {
  if (int rc = check_net(net)) return rc;
  if (!params || !obs || !hist || !mean || !workspace || n <= 0)
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_act_student: null argument or n <= 0");
  const lrl_ppo_net& nt = *net;
  const int hld = hist_ld ? hist_ld : nt.num_hist, hpad = hist_pad(nt.num_hist);
  if (hld < nt.num_hist) return lrl_set_error(LRL_E_INVALID, "lrl_ppo_act_student: hist_ld < num_hist");
  StudentPlan P = make_student_plan(nt, n, static_cast<char*>(workspace));
  hipStream_t st = static_cast<hipStream_t>(stream);
  G g{st, nullptr};
  const float* w = params;
  const int nx = nt.num_obs + nt.latent, XS = xs_of(nt);
  hipLaunchKernelGGL(ppo_prep_kernel, dim3(prep_blocks(n, XS)), dim3(256), 0, st, obs,
                     (const int64_t*)nullptr, n, nt.num_obs, XS, P.xa);
  if (hld >= hpad && hld % 4 == 0 && ((uintptr_t)hist & 15) == 0 && hpad != nt.num_hist) {
    const int64_t cnt = (int64_t)nt.ad_h0 * hpad;
    hipLaunchKernelGGL(pad_cols_kernel, dim3((unsigned)std::min<int64_t>((cnt + 255) / 256, 1024)), dim3(256), 0, st,
                       w + nt.d1w, nt.ad_h0, nt.num_hist, hpad, P.wd1p);
    g.nt(hist, hld, nullptr, P.wd1p, hpad, P.hd1, nt.ad_h0, w + nt.d1b, n, nt.ad_h0, hpad, true);
  } else {
    g.nt(hist, hld, nullptr, w + nt.d1w, nt.num_hist, P.hd1, nt.ad_h0, w + nt.d1b, n, nt.ad_h0, nt.num_hist, true);
  }
  g.nt(P.hd1, nt.ad_h0, nullptr, w + nt.d2w, nt.ad_h0, P.hd2, HD2S, w + nt.d2b, n, nt.ad_h1, nt.ad_h0, true);
  g.nt(P.hd2, HD2S, nullptr, w + nt.d3w, nt.ad_h1, P.xa + nt.num_obs, XS, w + nt.d3b, n, nt.latent, nt.ad_h1, false);
  // actor half of the grouped actor/critic layers (rows [0, h) of each grouped weight / bias)
  g.nt(P.xa, XS, nullptr, w + nt.w1, nx, P.h1, nt.ac_h0, w + nt.b1, n, nt.ac_h0, XS, true);  // k-padding: see phase 1
  g.nt(P.h1, nt.ac_h0, nullptr, w + nt.w2, nt.ac_h0, P.h2, nt.ac_h1, w + nt.b2, n, nt.ac_h1, nt.ac_h0, true);
  g.nt(P.h2, nt.ac_h1, nullptr, w + nt.w3, nt.ac_h1, P.h3, nt.ac_h2, w + nt.b3, n, nt.ac_h2, nt.ac_h1, true);
  g.nt(P.h3, nt.ac_h2, nullptr, w + nt.w4a, nt.ac_h2, mean, nt.num_actions, w + nt.b4a, n, nt.num_actions, nt.ac_h2,
       false);
  if (g.rc) return lrl_set_error(g.rc, "lrl_ppo_act_student: GEMM launch failed");
  if (latent &&
      hipMemcpy2DAsync(latent, (size_t)nt.latent * 4, P.xa + nt.num_obs, (size_t)XS * 4, (size_t)nt.latent * 4, n,
                       hipMemcpyDeviceToDevice, st) != hipSuccess)
    return lrl_set_error(LRL_E_HIP, "lrl_ppo_act_student: latent copy failed");
  return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_act_student: launch failed");
}

extern "C" int64_t lrl_ppo_workspace_bytes(const lrl_ppo_net* net, int32_t batch) {
  if (check_net(net) || batch <= 0) return -1;
  return make_plan(*net, batch, nullptr).bytes;
}

extern "C" int32_t lrl_ppo_forward_backward(const lrl_ppo_net* net, const float* params, float* grads,
                                            const lrl_ppo_batch* bt, const lrl_ppo_hparams* hp, void* workspace,
                                            lrl_ppo_ctrl* ctrl, void* stream) {
  if (int rc = check_net(net)) return rc;
  if (!bt || !hp || !params || !grads || !workspace || !ctrl || bt->batch <= 0)
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_forward_backward: null argument");
  const lrl_ppo_net& n = *net;
  const int B = bt->batch;
  Plan P = make_plan(n, B, static_cast<char*>(workspace));
  hipStream_t st = static_cast<hipStream_t>(stream);
  G g{st, P.part + P.part_floats};
  const float* w = params;
  const int nx = n.num_obs + n.latent, XS = xs_of(n);
  // ---- forward ----
  PlaneJob pj[PL_MAIN];
  main_plane_jobs(n, w, P.wpl, pj);
  if (gemm_x6p_enabled()) {
    if (int rc = x6_planes_launch(pj, PL_MAIN, st)) return lrl_set_error(rc, "lrl_ppo_forward_backward: planes launch failed");
  } else {
    for (auto& q : pj) q.dst = nullptr;
  }
  auto PJ = [&](int i) -> const PlaneJob& { return pj[i]; };
  hipLaunchKernelGGL(ppo_prep_kernel, dim3(prep_blocks(B, XS)), dim3(256), 0, st, bt->obs,
                     bt->rows, B, n.num_obs, XS, P.xa);
  g.nt(bt->priv, n.num_priv, bt->rows, w + n.e1w, n.num_priv, P.he1, n.enc_h0, w + n.e1b, B, n.enc_h0, n.num_priv, true);
  g.with(PJ(PL_E2)).nt(P.he1, n.enc_h0, nullptr, w + n.e2w, n.enc_h0, P.he2, n.enc_h1, w + n.e2b, B, n.enc_h1, n.enc_h0, true);
  g.nt(P.he2, n.enc_h1, nullptr, w + n.e3w, n.enc_h1, P.xa + n.num_obs, XS, w + n.e3b, B, n.latent, n.enc_h1, false);
  // k runs over all XS columns of X: columns nx..XS-1 are zero, so the extra products (with the next
  // row's first weights, or the first biases after the last row — finite values; zero planes on the x6p path) add
  // exactly 0, and the product takes the unguarded float4 path
  g.with(PJ(PL_W1)).nt(P.xa, XS, nullptr, w + n.w1, nx, P.h1, 2 * n.ac_h0, w + n.b1, B, 2 * n.ac_h0, XS, true);
  g.with(PJ(PL_W2)).nt(P.h1, 2 * n.ac_h0, nullptr, w + n.w2, n.ac_h0, P.h2, 2 * n.ac_h1, w + n.b2, B, n.ac_h1, n.ac_h0,
                       true, 2, n.ac_h0, (int64_t)n.ac_h1 * n.ac_h0, n.ac_h1, n.ac_h1);
  g.with(PJ(PL_W3)).nt(P.h2, 2 * n.ac_h1, nullptr, w + n.w3, n.ac_h1, P.h3, 2 * n.ac_h2, w + n.b3, B, n.ac_h2, n.ac_h1,
                       true, 2, n.ac_h1, (int64_t)n.ac_h2 * n.ac_h1, n.ac_h2, n.ac_h2);
  if (g.rc) return lrl_set_error(g.rc, "lrl_ppo_forward_backward: forward GEMM launch failed");
  // ---- head ----
  SegList L{};
  float* part = P.part;
  const int hb = (B + HEAD_ROWS - 1) / HEAD_ROWS;
  const int na = n.num_actions;
  HeadArgs ha{};
  ha.h3 = P.h3; ha.dh3 = P.dh3;
  ha.w4a = w + n.w4a; ha.b4a = w + n.b4a; ha.w4c = w + n.w4c; ha.b4c = w + n.b4c; ha.stdv = w + n.std_off;
  ha.actions = bt->actions; ha.old_mu = bt->mu; ha.old_sigma = bt->sigma; ha.tv = bt->values; ha.ret = bt->returns;
  ha.adv = bt->adv; ha.old_logp = bt->logp; ha.rows = bt->rows;
  ha.B = B; ha.na = na; ha.clip = hp->clip_param; ha.ent_coef = hp->entropy_coef; ha.vcoef = hp->value_loss_coef;
  ha.clipped_value = hp->use_clipped_value_loss;
  ha.part = part; ha.part_len = hp_len(na);
  hipLaunchKernelGGL(ppo_head_kernel, dim3(hb), dim3(HEAD_THREADS), 0, st, ha);
  {
    const int64_t pl = hp_len(na);
    const float invB = 1.f / (float)B;
    L.s[L.n++] = Seg{part + hp_w4a(na), grads + n.w4a, (int64_t)na * HEAD_W, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + hp_b4a(na), grads + n.b4a, na, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + hp_w4c(na), grads + n.w4c, HEAD_W, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + hp_b4c(na), grads + n.b4c, 1, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + hp_std(na), grads + n.std_off, na, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + hp_kl(na), grads + n.kl_slot, 1, pl, hb, invB};
    L.s[L.n++] = Seg{part + hp_kl(na) + 1, &ctrl->mb[1], 1, pl, hb, invB};
    L.s[L.n++] = Seg{part + hp_kl(na) + 2, &ctrl->mb[0], 1, pl, hb, invB};
    part += ((hb * pl + 63) / 64) * 64;
  }
  // ---- backward ----
  // the data-gradient chain first (dH2, dH1, the latent gradient), then the encoder's chain forks to the library's
  // second stream while the actor / critic weight gradients run here; the split-k reduction joins both
  const int h0 = n.ac_h0, h1 = n.ac_h1, h2 = n.ac_h2;
  g.with(PJ(PL_W3T)).nn(P.dh3, 2 * h2, w + n.w3, h1, P.dh2, 2 * h1, P.h2, 2 * h1, B, h1, h2, 2, h2, (int64_t)h2 * h1, h1, h1);
  g.with(PJ(PL_W2T)).nn(P.dh2, 2 * h1, w + n.w2, h0, P.dh1, 2 * h0, P.h1, 2 * h0, B, h0, h1, 2, h1, (int64_t)h1 * h0, h0, h0);
  // d latent = dH1 [W1a; W1c][:, num_obs:]  (sum over actor and critic halves: one reduction of length 2*h0)
  g.nn(P.dh1, 2 * h0, w + n.w1 + n.num_obs, nx, P.dlat, LATS, nullptr, 0, B, n.latent, 2 * h0);
  Fork* fk = fork_for_device(st);
  G ge{fk ? fk->st : st, g.part_end};
  if (fk) {
    if (hipEventRecord(fk->go, st) != hipSuccess || hipStreamWaitEvent(fk->st, fk->go, 0) != hipSuccess)
      return lrl_set_error(LRL_E_HIP, "lrl_ppo_forward_backward: stream fork failed");
  }
  ge.tn(P.dlat, LATS, P.he2, n.enc_h1, nullptr, n.latent, n.enc_h1, B, 1, 0, 0, part, grads + n.e3w, grads + n.e3b, L);
  ge.nn(P.dlat, LATS, w + n.e3w, n.enc_h1, P.dhe2, n.enc_h1, P.he2, n.enc_h1, B, n.enc_h1, n.latent);
  ge.tn(P.dhe2, n.enc_h1, P.he1, n.enc_h0, nullptr, n.enc_h1, n.enc_h0, B, 1, 0, 0, part, grads + n.e2w, grads + n.e2b, L);
  ge.with(PJ(PL_E2T)).nn(P.dhe2, n.enc_h1, w + n.e2w, n.enc_h0, P.dhe1, n.enc_h0, P.he1, n.enc_h0, B, n.enc_h0, n.enc_h1);
  ge.tn(P.dhe1, n.enc_h0, bt->priv, n.num_priv, bt->rows, n.enc_h0, n.num_priv, B, 1, 0, 0, part, grads + n.e1w,
        grads + n.e1b, L);
  if (fk && hipEventRecord(fk->done, fk->st) != hipSuccess)
    return lrl_set_error(LRL_E_HIP, "lrl_ppo_forward_backward: stream fork failed");
  g.tn(P.dh3, 2 * h2, P.h2, 2 * h1, nullptr, h2, h1, B, 2, h2, h1, part, grads + n.w3, grads + n.b3, L);
  timer_begin(st);
  g.tn(P.dh2, 2 * h1, P.h1, 2 * h0, nullptr, h1, h0, B, 2, h1, h0, part, grads + n.w2, grads + n.b2, L);
  timer_end(st);
  g.tn(P.dh1, 2 * h0, P.xa, XS, nullptr, 2 * h0, nx, B, 1, 0, 0, part, grads + n.w1, grads + n.b1, L);
  if (fk && hipStreamWaitEvent(st, fk->done, 0) != hipSuccess)
    return lrl_set_error(LRL_E_HIP, "lrl_ppo_forward_backward: stream join failed");
  if (g.rc || ge.rc) return lrl_set_error(g.rc ? g.rc : ge.rc, "lrl_ppo_forward_backward: backward GEMM launch failed");
  launch_seg(L, st);
  return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_forward_backward: launch failed");
}

extern "C" int32_t lrl_ppo_optimizer_step(const lrl_ppo_net* net, float* params, const float* grads, float* exp_avg,
                                          float* exp_avg_sq, int64_t step, float grad_scale,
                                          const lrl_ppo_hparams* hp, void* workspace, lrl_ppo_ctrl* ctrl,
                                          void* stream) {
  if (int rc = check_net(net)) return rc;
  if (!params || !grads || !exp_avg || !exp_avg_sq || !hp || !workspace || !ctrl || step < 1)
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_optimizer_step: bad argument");
  const lrl_ppo_net& n = *net;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // norm partials: the first 2 KB of the workspace (phase-1 scratch, dead once its reduction ran)
  double* norm_part = static_cast<double*>(workspace);
  const int64_t len = n.main_end - n.main_begin;
  hipLaunchKernelGGL(sumsq_kernel, dim3(NORM_BLOCKS), dim3(256), 0, st, grads + n.main_begin, len, norm_part);
  const double bc1 = 1.0 - pow((double)hp->beta1, (double)step);
  const double bc2 = 1.0 - pow((double)hp->beta2, (double)step);
  hipLaunchKernelGGL(ppo_finalize_kernel, dim3(1), dim3(64), 0, st, norm_part, NORM_BLOCKS,
                     grads + n.kl_slot, grad_scale, hp->max_grad_norm, hp->desired_kl, hp->adaptive_schedule, bc1,
                     0.f, ctrl);
  const int blocks = (int)std::min<int64_t>((len + 255) / 256, 2048);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, params + n.main_begin, grads + n.main_begin,
                     exp_avg + n.main_begin, exp_avg_sq + n.main_begin, len, grad_scale, ctrl, 0.f,
                     (float)(1.0 - (double)hp->beta1), hp->beta2, (float)(1.0 - (double)hp->beta2), (float)sqrt(bc2),
                     hp->eps, (lrl_ppo_ctrl*)nullptr);
  return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_optimizer_step: launch failed");
}

extern "C" int32_t lrl_ppo_adaptation_forward_backward(const lrl_ppo_net* net, const float* params,
                                                       const float* enc_params, float* grads, const lrl_ppo_batch* bt,
                                                       void* workspace, lrl_ppo_ctrl* ctrl, void* stream) {
  if (int rc = check_net(net)) return rc;
  if (!bt || !params || !grads || !workspace || !ctrl || bt->batch <= 0)
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_adaptation_forward_backward: null argument");
  const lrl_ppo_net& n = *net;
  const int B = bt->batch;
  Plan P = make_plan(n, B, static_cast<char*>(workspace));
  hipStream_t st = static_cast<hipStream_t>(stream);
  G g{st, P.part + P.part_floats};
  const float* w = params;
  // target = env_factor_encoder(priv) with the just-updated weights (torch.no_grad, ppo.py:159-160), read from
  // enc_params (a snapshot of them taken right after the optimiser step, so the next step may proceed) or params
  const float* we = enc_params ? enc_params : params;
  PlaneJob pj[PL_ADAPT];
  adapt_plane_jobs(n, w, we, P.wpl, pj);
  if (gemm_x6p_enabled()) {
    if (int rc = x6_planes_launch(pj, PL_ADAPT, st)) return lrl_set_error(rc, "lrl_ppo_adaptation: planes launch failed");
  } else {
    for (auto& q : pj) q.dst = nullptr;
  }
  g.nt(bt->priv, n.num_priv, bt->rows, we + n.e1w, n.num_priv, P.he1, n.enc_h0, we + n.e1b, B, n.enc_h0, n.num_priv, true);
  g.with(pj[PL_AE2]).nt(P.he1, n.enc_h0, nullptr, we + n.e2w, n.enc_h0, P.he2, n.enc_h1, we + n.e2b, B, n.enc_h1, n.enc_h0, true);
  g.nt(P.he2, n.enc_h1, nullptr, we + n.e3w, n.enc_h1, P.tgt, LATS, we + n.e3b, B, n.latent, n.enc_h1, false);
  // prediction = adaptation_module(obs_history)
  const int hld = bt->hist_ld ? bt->hist_ld : n.num_hist, hpad = hist_pad(n.num_hist);
  if (hld < n.num_hist) return lrl_set_error(LRL_E_INVALID, "lrl_ppo_adaptation: hist_ld < num_hist");
  if (hld >= hpad && hld % 4 == 0 && ((uintptr_t)bt->hist & 15) == 0 && hpad != n.num_hist) {
    // history rows carry finite padding up to hpad: run k = hpad against zero-padded weights (float4 rows)
    const int64_t cnt = (int64_t)n.ad_h0 * hpad;
    hipLaunchKernelGGL(pad_cols_kernel, dim3((unsigned)std::min<int64_t>((cnt + 255) / 256, 1024)), dim3(256), 0, st,
                       w + n.d1w, n.ad_h0, n.num_hist, hpad, P.wd1p);
    g.with(pj[PL_D1]).nt(bt->hist, hld, bt->rows, P.wd1p, hpad, P.hd1, n.ad_h0, w + n.d1b, B, n.ad_h0, hpad, true);
  } else {
    g.nt(bt->hist, hld, bt->rows, w + n.d1w, n.num_hist, P.hd1, n.ad_h0, w + n.d1b, B, n.ad_h0, n.num_hist, true);
  }
  g.nt(P.hd1, n.ad_h0, nullptr, w + n.d2w, n.ad_h0, P.hd2, HD2S, w + n.d2b, B, n.ad_h1, n.ad_h0, true);
  if (g.rc) return lrl_set_error(g.rc, "lrl_ppo_adaptation: forward GEMM launch failed");
  SegList L{};
  float* part = P.part;
  const int hb = (B + HEAD_ROWS - 1) / HEAD_ROWS;
  AdaptHeadArgs aa{};
  aa.hd2 = P.hd2; aa.ldh = HD2S; aa.tgt = P.tgt; aa.ldt = LATS; aa.dhd2 = P.dhd2; aa.w = w + n.d3w; aa.b = w + n.d3b;
  aa.B = B; aa.H = n.ad_h1; aa.L = n.latent; aa.part = part; aa.part_len = n.latent * n.ad_h1 + n.latent + 1;
  if (aa.H == 32 && aa.L == 18)
    hipLaunchKernelGGL((adapt_head_kernel<32, 18>), dim3(hb), dim3(HEAD_THREADS), 0, st, aa);
  else
    hipLaunchKernelGGL((adapt_head_kernel<0, 0>), dim3(hb), dim3(HEAD_THREADS), 0, st, aa);
  {
    const int64_t pl = aa.part_len;
    L.s[L.n++] = Seg{part, grads + n.d3w, (int64_t)n.latent * n.ad_h1, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + n.latent * n.ad_h1, grads + n.d3b, n.latent, pl, hb, 1.f};
    L.s[L.n++] = Seg{part + n.latent * n.ad_h1 + n.latent, &ctrl->mb[2], 1, pl, hb,
                     1.f / ((float)B * (float)n.latent)};
    part += ((hb * pl + 63) / 64) * 64;
  }
  g.tn(P.dhd2, HD2S, P.hd1, n.ad_h0, nullptr, n.ad_h1, n.ad_h0, B, 1, 0, 0, part, grads + n.d2w, grads + n.d2b, L);
  g.with(pj[PL_D2T]).nn(P.dhd2, HD2S, w + n.d2w, n.ad_h0, P.dhd1, n.ad_h0, P.hd1, n.ad_h0, B, n.ad_h0, n.ad_h1);
  g.tn(P.dhd1, n.ad_h0, bt->hist, hld, bt->rows, n.ad_h0, n.num_hist, B, 1, 0, 0, part, grads + n.d1w,
       grads + n.d1b, L);
  if (g.rc) return lrl_set_error(g.rc, "lrl_ppo_adaptation: backward GEMM launch failed");
  launch_seg(L, st);
  return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_adaptation: launch failed");
}

extern "C" int32_t lrl_ppo_adaptation_step(const lrl_ppo_net* net, float* params, const float* grads, float* exp_avg,
                                           float* exp_avg_sq, int64_t step, double lr, float grad_scale,
                                           const lrl_ppo_hparams* hp, lrl_ppo_ctrl* ctrl, void* stream) {
  if (int rc = check_net(net)) return rc;
  if (!params || !grads || !exp_avg || !exp_avg_sq || !hp || step < 1)
    return lrl_set_error(LRL_E_INVALID, "lrl_ppo_adaptation_step: bad argument");
  const lrl_ppo_net& n = *net;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const double bc1 = 1.0 - pow((double)hp->beta1, (double)step);
  const double bc2 = 1.0 - pow((double)hp->beta2, (double)step);
  const int64_t len = n.adapt_end - n.adapt_begin;
  const int blocks = (int)std::min<int64_t>((len + 255) / 256, 2048);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, params + n.adapt_begin, grads + n.adapt_begin,
                     exp_avg + n.adapt_begin, exp_avg_sq + n.adapt_begin, len, grad_scale,
                     (const lrl_ppo_ctrl*)nullptr, (float)(lr / bc1), (float)(1.0 - (double)hp->beta1), hp->beta2,
                     (float)(1.0 - (double)hp->beta2), (float)sqrt(bc2), hp->eps, ctrl);
  return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_ppo_adaptation_step: launch failed");
}

// ---- GEMM test entry point ----
extern "C" int32_t lrl_gemm_f32(int32_t layout, int32_t epi, int32_t M, int32_t N, int32_t K, const float* A,
                                int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias,
                                const float* aux, int64_t ld_aux, const int64_t* rows, float* workspace,
                                int64_t workspace_floats, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  GemmP p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.C = C; p.ldc = ldc; p.bias = bias; p.aux = aux; p.ld_aux = ld_aux;
  p.M = M; p.N = N; p.K = K; p.splits = 1;
  if (layout == GEMM_TN) {
    // split-k into the workspace, then reduce into C (C must be [M][N] contiguous: ldc == N)
    if (ldc != N) return lrl_set_error(LRL_E_INVALID, "lrl_gemm_f32: TN needs ldc == N");
    int splits = gemm_pick_splits(M, N, K, 1);
    if (const char* e = getenv("LRL_GEMM_SPLITS")) {  // development knob (scripts/tn_sweep.py)
      const int s = atoi(e);
      if (s > 0) splits = s;
    }
    if ((int64_t)splits * ((int64_t)M * N + M) > workspace_floats)
      return lrl_set_error(LRL_E_INVALID, "lrl_gemm_f32: workspace too small");
    p.b_rows = rows; p.splits = splits; p.kps = (K + splits - 1) / splits;
    p.C = workspace; p.gc = (int64_t)M * N; p.part_stride = (int64_t)M * N;
    p.bias_part = workspace + (int64_t)splits * M * N;
    int rc = gemm_launch(p, GEMM_TN, EPI_PARTIAL, 1, st);
    if (rc) return lrl_set_error(rc, "lrl_gemm_f32: launch failed");
    SegList L{};
    L.s[L.n++] = Seg{workspace, C, (int64_t)M * N, (int64_t)M * N, splits, 1.f};
    if (bias) L.s[L.n++] = Seg{p.bias_part, const_cast<float*>(bias), M, M, splits, 1.f};  // bias = db output
    launch_seg(L, st);
    return hipGetLastError() == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, "lrl_gemm_f32: launch failed");
  }
  p.a_rows = rows;
  if (layout & 0x100) {
    // pre-split B: planes of op(B) built in the workspace, then the x6p kernel (and nothing else) runs the product
    layout &= 0xff;
    if (layout != GEMM_NT && layout != GEMM_NN) return lrl_set_error(LRL_E_INVALID, "lrl_gemm_f32: planes need NT / NN");
    PlaneJob j{};
    j.W = B; j.ldw = ldb; j.gsrc = 0; j.groups = 1; j.trans = layout == GEMM_NN ? 1 : 0;
    j.rows = layout == GEMM_NN ? K : N; j.cols = layout == GEMM_NN ? N : K;
    j.dst = reinterpret_cast<uint16_t*>(workspace);
    if (!workspace || plane_elems(j) > 2 * workspace_floats)
      return lrl_set_error(LRL_E_INVALID, "lrl_gemm_f32: workspace too small for the planes");
    if (int rc = x6_planes_launch(&j, 1, st)) return lrl_set_error(rc, "lrl_gemm_f32: planes launch failed");
    gemm_use_planes(p, j);
    int rc = gemm_launch(p, layout, epi, 1, st);
    if (rc) return lrl_set_error(rc, "lrl_gemm_f32: launch failure");
    return gemm_last_path() == 1 ? 0 : lrl_set_error(LRL_E_INVALID, "lrl_gemm_f32: shape not eligible for the x6p kernel");
  }
  int rc = gemm_launch(p, layout, epi, 1, st);
  return rc ? lrl_set_error(rc, "lrl_gemm_f32: bad layout/epilogue or launch failure") : 0;
}

// ---- timing hook of the dominant update product (bench.py roofline) ----
extern "C" int32_t lrl_ppo_timing(int32_t enable, double* total_ms, int64_t* launches) {
  if (total_ms) {
    double t = 0.0;
    for (size_t i = 0; i < g_timer.used; ++i) {
      float ms = 0.f;
      if (hipEventSynchronize(g_timer.ev[i].second) != hipSuccess ||
          hipEventElapsedTime(&ms, g_timer.ev[i].first, g_timer.ev[i].second) != hipSuccess)
        return lrl_set_error(LRL_E_HIP, "lrl_ppo_timing: event query failed");
      t += ms;
    }
    *total_ms = t;
  }
  if (launches) *launches = (int64_t)g_timer.used;
  g_timer.used = 0;
  g_timer.on = enable != 0;
  return 0;
}
