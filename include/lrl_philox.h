/*
 * Counter-based RNG (Philox4x32-10) shared by the HIP kernels and the CPU oracle.
 *
 * The reference draws its randomness from torch's global generator (obs noise rand_like
 * legged_robot.py:392, DR torch.rand :523-560, Normal.sample actor_critic.py:144).  Reproducing a
 * torch stream inside a kernel is not practical, so the product uses a
 * counter-based stream keyed by (seed, global env id, step counter, stream id): trajectories do not
 * depend on the GPU count or the launch geometry.  Parity tests inject the reference's draws.
 */
#ifndef LRL_PHILOX_H_
#define LRL_PHILOX_H_
#include <stdint.h>

#if defined(__HIPCC__)
#define LRL_HD __host__ __device__ __forceinline__
#else
#define LRL_HD static inline
#endif

enum { LRL_RNG_OBS_NOISE = 1, LRL_RNG_DR = 2, LRL_RNG_INIT = 3, LRL_RNG_POLICY = 4, LRL_RNG_RESET = 5, LRL_RNG_PUSH = 6,
       LRL_RNG_TERRAIN = 7 };

typedef struct { uint32_t v[4]; } lrl_u32x4;

LRL_HD uint32_t lrl_mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

/* ctr = (c0, c1, c2, c3), key = seed */
LRL_HD lrl_u32x4 lrl_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = lrl_mulhilo(0xD2511F53u, c0, &hi0);
    uint32_t lo1 = lrl_mulhilo(0xCD9E8D57u, c2, &hi1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  lrl_u32x4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

/* uniform in [0, 1): 24 random bits */
LRL_HD float lrl_u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

/* the k-th uniform of a (env, step, stream) sequence */
LRL_HD float lrl_uniform(uint64_t seed, uint64_t env, uint64_t step, uint32_t stream, uint32_t k) {
  lrl_u32x4 r = lrl_philox((uint32_t)env, (uint32_t)(step & 0xffffffffu),
                           (stream << 16) ^ (uint32_t)(step >> 32), k >> 2, seed);
  return lrl_u01(r.v[k & 3]);
}

#endif /* LRL_PHILOX_H_ */
