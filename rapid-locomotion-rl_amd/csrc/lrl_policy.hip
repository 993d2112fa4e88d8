// lrl_policy.hip — fused rollout step of PPO.act (ppo.py:62-74) for gfx950.
//
// One 256-thread workgroup (4 waves) owns 32 env rows and runs the whole teacher path of
// ActorCritic (actor_critic.py:137-147,170-173) on fp32 MFMA (v_mfma_f32_32x32x2_f32: exact fp32,
// k-ordered FMA chain):
//   latent = enc(priv)              18 -> 256 -> 128 -> 18   (ELU, ELU)
//   x      = [obs, latent]          42 + 18 = 60
//   mu     = actor(x)               60 -> 512 -> 256 -> 128 -> 12
//   value  = critic(x)              60 -> 512 -> 256 -> 128 -> 1
//   a = mu + std * eps,  logp = sum_j log N(a_j; mu_j, std_j)      (torch.distributions.Normal)
// and, when asked, writes the transition into row `store_row` of the rollout storage
// (RolloutStorage.add_transitions, rollout_storage.py:57-71).
//
// Activations stay in LDS ([row][feature], row stride padded to out+1 -> conflict-free column
// reads for the A operand); weights stream from L2 (the whole 2.4 MB teacher stack is L2/MALL
// resident): lane (j, h) of a wave reads W[j0 + j][k0 + h] for the B operand.  Each wave owns a set
// of 32-column output tiles; the C/D fragment (col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5))
// is written back to LDS with bias + ELU fused.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/lrl.h"
#include "../../include/lrl_philox.h"

extern "C" int lrl_set_error(int code, const char* msg);

namespace lrl {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int PROWS = 32;     // env rows per workgroup
constexpr int PTHREADS = 256; // 4 waves
constexpr int MAXW = 512;     // widest layer

__device__ __forceinline__ float elu(float x) { return x > 0.f ? x : expm1f(x); }

// Y[32][out] = act(X[32][in] W^T + b); X row stride xs, Y row stride ys (both in LDS)
__device__ void mlp_layer(const float* __restrict__ W, const float* __restrict__ b, int in, int out, bool act,
                          const float* X, int xs, float* Y, int ys) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int li = lane & 31, h = lane >> 5;
  const int ntiles = (out + 31) / 32;
  for (int t0 = wave; t0 < ntiles; t0 += 4 * 4) {
    // up to 4 tiles per wave per pass: t0, t0+4, t0+8, t0+12
    f32x16 acc[4];
    int tiles[4];
    int nt = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      tiles[u] = t0 + 4 * u;
      acc[u] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (tiles[u] < ntiles) nt = u + 1;
    }
    for (int k0 = 0; k0 < in; k0 += 2) {
      const int k = k0 + h;
      const float a = k < in ? X[li * xs + k] : 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < nt) {
          const int j = tiles[u] * 32 + li;
          const float bw = (k < in && j < out) ? W[(size_t)j * in + k] : 0.f;
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw, acc[u], 0, 0, 0);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < nt) {
        const int j = tiles[u] * 32 + li;
        if (j < out) {
          const float bj = b[j];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = acc[u][r] + bj;
            Y[row * ys + j] = act ? elu(v) : v;
          }
        }
      }
  }
  __syncthreads();
}

__device__ void mlp_chain(const lrl_mlp_desc& d, const float* X, int xs, float* bufA, float* bufB, float* out,
                          int outs) {
  // hidden layers ping-pong between bufA / bufB (stride MAXW+1); the last layer writes `out`
  const float* cur = X;
  int cs = xs;
  for (int l = 0; l < d.num_layers; ++l) {
    const bool last = l == d.num_layers - 1;
    float* dst = last ? out : ((l & 1) ? bufB : bufA);
    const int ds = last ? outs : MAXW + 1;
    mlp_layer(d.weight[l], d.bias[l], d.dims[l], d.dims[l + 1], !last, cur, cs, dst, ds);
    cur = dst;
    cs = ds;
  }
}

__global__ __launch_bounds__(PTHREADS) void policy_act_kernel(lrl_mlp_desc enc, lrl_mlp_desc actor, lrl_mlp_desc critic,
                                                              const float* __restrict__ stdv, const float* __restrict__ obs,
                                                              const float* __restrict__ priv, const float* __restrict__ hist,
                                                              int n, int no, int np, const float* __restrict__ eps,
                                                              uint64_t seed, uint64_t counter, float* __restrict__ actions,
                                                              float* __restrict__ mu_out, float* __restrict__ values,
                                                              float* __restrict__ logp, lrl_rollout_store store,
                                                              int store_row, int do_store) {
  extern __shared__ float sm[];
  float* bufA = sm;                                  // [32][MAXW+1]
  float* bufB = bufA + PROWS * (MAXW + 1);           // [32][MAXW+1]
  const int xs = 64;                                 // x row stride (obs + latent <= 64)
  float* X = bufB + PROWS * (MAXW + 1);              // [32][64]
  float* P = X + PROWS * xs;                         // [32][32] priv input
  float* MU = P + PROWS * 32;                        // [32][16]
  float* V = MU + PROWS * 16;                        // [32][2]
  const int row0 = blockIdx.x * PROWS;
  const int nl = enc.dims[enc.num_layers];           // latent width
  for (int i = threadIdx.x; i < PROWS * 32; i += PTHREADS) {
    int r = i >> 5, c = i & 31, g = row0 + r;
    P[r * 32 + c] = (g < n && c < np) ? priv[(size_t)g * np + c] : 0.f;
  }
  for (int i = threadIdx.x; i < PROWS * xs; i += PTHREADS) {
    int r = i / xs, c = i - r * xs, g = row0 + r;
    if (c < no) X[r * xs + c] = g < n ? obs[(size_t)g * no + c] : 0.f;
  }
  __syncthreads();
  // latent = enc(priv) -> X[:, no:no+nl]
  mlp_chain(enc, P, 32, bufA, bufB, X + no, xs);
  mlp_chain(actor, X, xs, bufA, bufB, MU, 16);
  mlp_chain(critic, X, xs, bufA, bufB, V, 2);
  // sampling + log-prob (one thread per (row, action))
  const int na = actor.dims[actor.num_layers];
  if (threadIdx.x < PROWS) {
    const int r = threadIdx.x, g = row0 + r;
    if (g < n) {
      float lp = 0.f;
      const float LOG_SQRT_2PI = 0.91893853320467274178f;
      for (int j = 0; j < na; ++j) {
        float e;
        if (eps) {
          e = eps[(size_t)g * na + j];
        } else {  // Box-Muller on the counter RNG (stream POLICY)
          lrl_u32x4 u = lrl_philox((uint32_t)g, (uint32_t)counter, (LRL_RNG_POLICY << 16) ^ (uint32_t)(counter >> 32),
                                   (uint32_t)(j >> 1), seed);
          float u1 = fmaxf(lrl_u01(u.v[0]), 1e-7f), u2 = lrl_u01(u.v[1]);
          float rad = sqrtf(-2.f * logf(u1)), th = 6.283185307179586f * u2;
          e = (j & 1) ? rad * sinf(th) : rad * cosf(th);
        }
        const float m = MU[r * 16 + j], s = stdv[j];
        const float a = m + s * e;
        const float d = a - m;
        lp += -(d * d) / (2.f * (s * s)) - logf(s) - LOG_SQRT_2PI;
        actions[(size_t)g * na + j] = a;
        if (mu_out) mu_out[(size_t)g * na + j] = m;
        if (do_store) {
          const size_t o = ((size_t)store_row * n + g) * na + j;
          store.actions[o] = a;
          store.mu[o] = m;
          store.sigma[o] = s;
        }
      }
      if (values) values[g] = V[r * 2];
      if (logp) logp[g] = lp;
      if (do_store) {
        store.values[(size_t)store_row * n + g] = V[r * 2];
        store.logp[(size_t)store_row * n + g] = lp;
      }
    }
  }
  if (do_store) {  // obs / priv / history rows of this tile (coalesced copies)
    const size_t b = (size_t)store_row * n;
    for (int i = threadIdx.x; i < PROWS * no; i += PTHREADS) {
      size_t g = row0 + i / no;
      if (g < (size_t)n) store.obs[(b + row0) * no + i] = obs[(size_t)row0 * no + i];
    }
    for (int i = threadIdx.x; i < PROWS * np; i += PTHREADS) {
      size_t g = row0 + i / np;
      if (g < (size_t)n) store.priv[(b + row0) * np + i] = priv[(size_t)row0 * np + i];
    }
    if (hist && store.hist) {  // the tile's history rows are one contiguous span in both buffers
      const int hd = store.hist_dim;
      const int rows = min(PROWS, n - row0);
      const float* src = hist + (size_t)row0 * hd;
      float* dst = store.hist + (b + row0) * hd;
      const int cnt = rows * hd;
      if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0 && (cnt & 3) == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (int i = threadIdx.x; i < cnt / 4; i += PTHREADS) d4[i] = s4[i];
      } else if ((((uintptr_t)src | (uintptr_t)dst) & 7) == 0 && (cnt & 1) == 0) {
        const float2* s2 = reinterpret_cast<const float2*>(src);
        float2* d2 = reinterpret_cast<float2*>(dst);
        for (int i = threadIdx.x; i < cnt / 2; i += PTHREADS) d2[i] = s2[i];
      } else {
        for (int i = threadIdx.x; i < cnt; i += PTHREADS) dst[i] = src[i];
      }
    }
  }
}

}  // namespace lrl

static int policy_lds_bytes() {
  return (2 * lrl::PROWS * (lrl::MAXW + 1) + lrl::PROWS * (64 + 32 + 16 + 2)) * 4;
}

extern "C" int32_t lrl_policy_act(const lrl_mlp_desc* encoder, const lrl_mlp_desc* actor, const lrl_mlp_desc* critic,
                                  const float* std_, const float* obs, const float* priv, const float* hist, int32_t n,
                                  int32_t num_obs, int32_t num_priv, const float* eps, uint64_t seed, uint64_t counter,
                                  float* actions, float* mu, float* values, float* logp, const lrl_rollout_store* store,
                                  int32_t store_row, void* stream) {
  if (!encoder || !actor || !critic || !std_ || !obs || !priv || !actions || n <= 0)
    return lrl_set_error(LRL_E_INVALID, "lrl_policy_act: null argument or n <= 0");
  const int nl = encoder->dims[encoder->num_layers];
  if (num_obs + nl > 64 || num_priv > 32 || actor->dims[actor->num_layers] > 16)
    return lrl_set_error(LRL_E_INVALID, "lrl_policy_act: obs+latent > 64, priv > 32 or actions > 16");
  if (actor->dims[0] != num_obs + nl || critic->dims[0] != num_obs + nl || encoder->dims[0] != num_priv)
    return lrl_set_error(LRL_E_INVALID, "lrl_policy_act: layer input widths do not match obs/priv/latent");
  for (const lrl_mlp_desc* d : {encoder, actor, critic}) {
    if (d->num_layers < 1 || d->num_layers > 7) return lrl_set_error(LRL_E_INVALID, "lrl_policy_act: 1..7 layers");
    for (int l = 0; l <= d->num_layers; ++l)
      if (d->dims[l] <= 0 || d->dims[l] > lrl::MAXW)
        return lrl_set_error(LRL_E_INVALID, "lrl_policy_act: layer width must be 1..512");
  }
  if (store && (!store->obs || !store->priv || !store->actions || !store->values || !store->logp || !store->mu ||
                !store->sigma || store->hist_dim < 0))
    return lrl_set_error(LRL_E_INVALID, "lrl_policy_act: incomplete rollout store");
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)lrl::policy_act_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            policy_lds_bytes()) != hipSuccess)
      return lrl_set_error(LRL_E_HIP, "lrl_policy_act: cannot raise the LDS limit");
    attr = true;
  }
  lrl_rollout_store st{};
  if (store) st = *store;
  const int blocks = (n + lrl::PROWS - 1) / lrl::PROWS;
  hipLaunchKernelGGL(lrl::policy_act_kernel, dim3(blocks), dim3(lrl::PTHREADS), policy_lds_bytes(), (hipStream_t)stream,
                     *encoder, *actor, *critic, std_, obs, priv, hist, n, num_obs, num_priv, eps, seed, counter,
                     actions, mu, values, logp, st, store_row, store ? 1 : 0);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : lrl_set_error(LRL_E_HIP, hipGetErrorString(e));
}
