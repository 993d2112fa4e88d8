// lrl_curriculum.cpp — native host restatement of the grid-adaptive command curriculum's per-reset work
// (RewardThresholdCurriculum.sample / .update, mini_gym/envs/base/curriculum.py:56-68, 105-115), bit-exact with
// the numpy form in lrl/curriculum.py (which restates the reference with numpy.random.RandomState):
//   * MT19937 exactly as numpy's RandomState (the state is the caller's 624-word key + position, so the numpy
//     generator and this one are interchangeable: lrl/curriculum.py keeps them in sync);
//   * RandomState.choice(indices, n, p=w / w.sum()): numpy's pairwise sum for w.sum(), p = w / sum, cdf = cumsum(p)
//     (sequential), cdf /= cdf[-1], n doubles from random_sample, searchsorted(side='right');
//   * RandomState.uniform(low = c + half, high = c - half) over the [n][3] cells in C order: low + (high - low) * u;
//   * the weight update's clipped +0.2 adds: the listed bins once (fancy assignment from the old values), then every
//     bin of each centre's +-local_range neighbourhood once per centre, in centre order (the reference's loop).
// It runs once per resampled batch on the host, on the upstream-reset path of every env step (legacy_fork=False),
// where the numpy form cost ~0.15 ms per step while the GPU waited.
#pragma clang fp contract(off)
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/lrl.h"

extern "C" int lrl_set_error(int code, const char* msg);  // lrl_capi.cpp

namespace {

constexpr int MT_N = 624, MT_M = 397;

void mt_gen(uint32_t* key) {
  constexpr uint32_t A = 0x9908b0dfu, UP = 0x80000000u, LO = 0x7fffffffu;
  int i = 0;
  for (; i < MT_N - MT_M; ++i) {
    const uint32_t y = (key[i] & UP) | (key[i + 1] & LO);
    key[i] = key[i + MT_M] ^ (y >> 1) ^ (-(y & 1u) & A);
  }
  for (; i < MT_N - 1; ++i) {
    const uint32_t y = (key[i] & UP) | (key[i + 1] & LO);
    key[i] = key[i + (MT_M - MT_N)] ^ (y >> 1) ^ (-(y & 1u) & A);
  }
  const uint32_t y = (key[MT_N - 1] & UP) | (key[0] & LO);
  key[MT_N - 1] = key[MT_M - 1] ^ (y >> 1) ^ (-(y & 1u) & A);
}

struct MT {
  uint32_t* key;
  int pos;
  uint32_t next32() {
    if (pos >= MT_N) {
      mt_gen(key);
      pos = 0;
    }
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  double next_double() {  // random_sample: 53 bits from two draws
    const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
};

// numpy's pairwise summation of a contiguous float64 array (the add.reduce inner loop)
double pairwise_sum(const double* a, int64_t n) {
  if (n < 8) {
    double res = 0.;
    for (int64_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

// np.sum of a 1-D float64 array: the identity plus the pairwise sum of every element (checked against np.sum on
// random arrays, tests/test_curriculum.py)
double np_sum(const double* a, int64_t n) { return 0.0 + pairwise_sum(a, n); }

double clip01(double x) { return std::min(std::max(x, 0.0), 1.0); }

}  // namespace

extern "C" double lrl_np_sum_f64(const double* a, int64_t n) { return np_sum(a, n); }

extern "C" int32_t lrl_curriculum_sample(uint32_t* mt_key, int32_t* mt_pos, const double* weights, int32_t nbins,
                                         const double* grid, const double* half, int32_t n, double* cmds,
                                         int64_t* bins) {
  if (!mt_key || !mt_pos || !weights || !grid || !half || nbins <= 0 || n < 0 || (n > 0 && (!cmds || !bins)))
    return lrl_set_error(LRL_E_INVALID, "lrl_curriculum_sample: bad argument");
  // the normalised cdf depends on the weights alone: reuse the last one while the weights are unchanged (the update
  // before most resamples adds nothing: no bin of the batch passed its thresholds)
  thread_local std::vector<double> cdf, wcopy;
  double* c;
  if ((int)wcopy.size() == nbins && memcmp(wcopy.data(), weights, (size_t)nbins * sizeof(double)) == 0) {
    c = cdf.data();
  } else {
    wcopy.assign(weights, weights + nbins);
    const double S = np_sum(weights, nbins);
    cdf.resize((size_t)nbins);
    c = cdf.data();
    // RandomState.choice's checks on p: NaN, negative entries, and |kahan_sum(p) - 1| > sqrt(eps).  p = w / S with S
    // numpy's own sum of w, so sum(p) is 1 to within nbins ulps (far inside the tolerance) unless S is 0 or not finite,
    // which makes p NaN / inf: those are the cases the sum check can reject, and they are tested here directly.
    bool nan = false, neg = false;
    for (int i = 0; i < nbins; ++i) {
      const double p = weights[i] / S;
      c[i] = p;
      nan |= p != p;
      neg |= p < 0.0;
    }
    if (nan || neg || !(fabs(S) < INFINITY) || S == 0.0) {
      wcopy.clear();  // (no cdf cached for these weights)
      if (nan) return lrl_set_error(LRL_E_INVALID, "probabilities contain NaN");
      if (neg) return lrl_set_error(LRL_E_INVALID, "probabilities are not non-negative");
      return lrl_set_error(LRL_E_INVALID, "probabilities do not sum to 1");
    }
    for (int i = 1; i < nbins; ++i) c[i] = c[i - 1] + c[i];  // cumsum: sequential, as add.accumulate
    const double last = c[nbins - 1];
    for (int i = 0; i < nbins; ++i) c[i] /= last;
  }
  MT mt{mt_key, *mt_pos};
  thread_local std::vector<double> u;
  u.resize((size_t)n);
  for (int j = 0; j < n; ++j) u[(size_t)j] = mt.next_double();
  for (int j = 0; j < n; ++j) bins[j] = (int64_t)(std::upper_bound(c, c + nbins, u[(size_t)j]) - c);
  for (int j = 0; j < n; ++j)
    for (int d = 0; d < 3; ++d) {
      const double g = grid[(int64_t)d * nbins + bins[j]];
      const double lo = g + half[d], hi = g - half[d];
      const double range = hi - lo;
      cmds[(int64_t)j * 3 + d] = lo + range * mt.next_double();
    }
  *mt_pos = mt.pos;
  return 0;
}

// weights: [nx * ny * nz] (bin = (ix * ny + iy) * nz + iz); axes: the three axes' grid values, concatenated
extern "C" int32_t lrl_curriculum_update_weights(double* weights, const double* axes, int32_t nx, int32_t ny,
                                                 int32_t nz, const int64_t* centres, int32_t n, double local_range) {
  if (!weights || !axes || nx <= 0 || ny <= 0 || nz <= 0 || n < 0 || (n > 0 && !centres))
    return lrl_set_error(LRL_E_INVALID, "lrl_curriculum_update_weights: bad argument");
  const int64_t nb = (int64_t)nx * ny * nz;
  for (int j = 0; j < n; ++j)
    if (centres[j] < 0 || centres[j] >= nb) return lrl_set_error(LRL_E_INVALID, "lrl_curriculum_update_weights: bin out of range");
  // weights[centres] = clip(weights[centres] + 0.2, 0, 1): every listed bin from its old value (duplicates agree)
  std::vector<double> nv((size_t)n);
  for (int j = 0; j < n; ++j) nv[(size_t)j] = clip01(weights[centres[j]] + 0.2);
  for (int j = 0; j < n; ++j) weights[centres[j]] = nv[(size_t)j];
  // each centre's neighbourhood (grid >= c - r and grid <= c + r on every axis), one clipped add per centre
  const double* ax[3] = {axes, axes + nx, axes + nx + ny};
  const int len[3] = {nx, ny, nz};
  std::vector<int> memb[3];
  for (int j = 0; j < n; ++j) {
    int64_t rem = centres[j];
    int idx[3];
    idx[2] = (int)(rem % nz);
    rem /= nz;
    idx[1] = (int)(rem % ny);
    idx[0] = (int)(rem / ny);
    for (int d = 0; d < 3; ++d) {
      memb[d].clear();
      const double c = ax[d][idx[d]], lo = c - local_range, hi = c + local_range;
      for (int i = 0; i < len[d]; ++i)
        if (ax[d][i] >= lo && ax[d][i] <= hi) memb[d].push_back(i);
    }
    for (int a : memb[0])
      for (int b : memb[1])
        for (int c : memb[2]) {
          double& w = weights[((int64_t)a * ny + b) * nz + c];
          w = clip01(w + 0.2);
        }
  }
  return 0;
}
