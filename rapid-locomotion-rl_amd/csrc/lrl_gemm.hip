// lrl_gemm.hip — fp32 MFMA GEMM kernels of the PPO update (see lrl_gemm.h for the contract).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/lrl.h"
#include "lrl_gemm.h"

namespace lrl {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GBK = 16;
constexpr int GTHREADS = 256;

template <int BM, int BN, int LAYOUT>
struct GemmTile {
  static constexpr bool AMC = (LAYOUT & 1) != 0;
  static constexpr bool BNC = (LAYOUT & 2) != 0;
  // k-major LDS images; padding keeps the transposing stores of k-contiguous operands conflict-free
  // (row pitch = 2 mod 8 words) and the float4 stores of m/n-contiguous operands 16-B aligned.
  static constexpr int PA = AMC ? 4 : 2;
  static constexpr int PB = BNC ? 4 : 2;
  static constexpr int NA = BM * GBK / 4 / GTHREADS;  // float4 loads per thread per tile
  static constexpr int NB = BN * GBK / 4 / GTHREADS;
};

__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }

// ---- global -> register staging of one BK slice ----
// k-contiguous operand X(r, k) = P[row(r) * ld + k], tile rows r0.., k0..: thread item i covers
// (r = i / 4, k = 4 (i % 4) .. +3).  m/n-contiguous operand X(r, k) = P[krow(k) * ld + r]: item i covers
// (k = i / (R/4), r = 4 (i % (R/4)) .. +3).
template <int R, int NI, bool RCONTIG, bool VEC>
__device__ __forceinline__ void stage_load(float4 (&reg)[NI], const float* __restrict__ P, int64_t ld,
                                           const int64_t* __restrict__ rows, int r0, int R_lim, int k0,
                                           int k_lim) {
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = threadIdx.x + u * GTHREADS;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (!RCONTIG) {
      const int r = i >> 2, k = k0 + 4 * (i & 3);
      const int gr = r0 + r;
      if (gr < R_lim) {
        const int64_t row = rows ? rows[gr] : (int64_t)gr;
        const float* src = P + row * ld + k;
        if (VEC && k + 3 < k_lim) {
          const float4 t = *reinterpret_cast<const float4*>(src);
          v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (k + c < k_lim) v[c] = src[c];
        }
      }
    } else {
      const int r = 4 * (i % (R / 4)), k = k0 + i / (R / 4);
      const int gr = r0 + r;
      if (k < k_lim) {
        const int64_t row = rows ? rows[k] : (int64_t)k;
        const float* src = P + row * ld + gr;
        if (VEC && gr + 3 < R_lim) {
          const float4 t = *reinterpret_cast<const float4*>(src);
          v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (gr + c < R_lim) v[c] = src[c];
        }
      }
    }
    reg[u] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int R, int PAD, int NI, bool RCONTIG>
__device__ __forceinline__ void stage_store(float (*S)[R + PAD], const float4 (&reg)[NI]) {
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = threadIdx.x + u * GTHREADS;
    if (!RCONTIG) {
      const int r = i >> 2, k = 4 * (i & 3);
      S[k + 0][r] = reg[u].x;
      S[k + 1][r] = reg[u].y;
      S[k + 2][r] = reg[u].z;
      S[k + 3][r] = reg[u].w;
    } else {
      const int r = 4 * (i % (R / 4)), k = i / (R / 4);
      *reinterpret_cast<float4*>(&S[k][r]) = reg[u];
    }
  }
}

template <int BM, int BN, int LAYOUT, bool AV, bool BV, int EPI>
__global__ __launch_bounds__(GTHREADS) void gemm_kernel(GemmP p) {
  using T = GemmTile<BM, BN, LAYOUT>;
  __shared__ __attribute__((aligned(16))) float As[2][GBK][BM + T::PA];
  __shared__ __attribute__((aligned(16))) float Bs[2][GBK][BN + T::PB];
  const int g = blockIdx.z / p.splits, s = blockIdx.z - g * p.splits;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kbeg = s * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, h = lane >> 5;
  constexpr int TM = BM / 64, TN = BN / 64;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // bias-gradient partial (weight-gradient products): column sums of A(m, k) over this split's k
  const bool do_bsum = EPI == EPI_PARTIAL && p.bias_part != nullptr && blockIdx.y == 0;
  float bsum = 0.f;

  float4 ra[T::NA], rb[T::NB];
  int k0 = kbeg;
  if (k0 < kend) {
    stage_load<BM, T::NA, T::AMC, AV>(ra, A, p.lda, T::AMC ? nullptr : p.a_rows, m0, p.M, k0, kend);
    stage_load<BN, T::NB, T::BNC, BV>(rb, B, p.ldb, T::BNC ? p.b_rows : nullptr, n0, p.N, k0, kend);
    stage_store<BM, T::PA, T::NA, T::AMC>(As[0], ra);
    stage_store<BN, T::PB, T::NB, T::BNC>(Bs[0], rb);
  }
  __syncthreads();
  int buf = 0;
  for (; k0 < kend; k0 += GBK) {
    const int kn = k0 + GBK;
    if (kn < kend) {
      stage_load<BM, T::NA, T::AMC, AV>(ra, A, p.lda, T::AMC ? nullptr : p.a_rows, m0, p.M, kn, kend);
      stage_load<BN, T::NB, T::BNC, BV>(rb, B, p.ldb, T::BNC ? p.b_rows : nullptr, n0, p.N, kn, kend);
    }
    if (do_bsum && threadIdx.x < BM) {
#pragma unroll
      for (int k = 0; k < GBK; ++k) bsum += As[buf][k][threadIdx.x];
    }
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[buf][kk + h][wm + 32 * i + li];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[buf][kk + h][wn + 32 * j + li];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kn < kend) {
      stage_store<BM, T::PA, T::NA, T::AMC>(As[buf ^ 1], ra);
      stage_store<BN, T::PB, T::NB, T::BNC>(Bs[buf ^ 1], rb);
    }
    __syncthreads();
    buf ^= 1;
  }

  // ---- epilogue ----
  float* __restrict__ C = p.C + g * p.gc;
  if (EPI == EPI_PARTIAL) C += (int64_t)s * p.part_stride;
  const float* __restrict__ bias = p.bias ? p.bias + g * p.gbias : nullptr;
  const float* __restrict__ aux = p.aux ? p.aux + g * p.gaux : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + 32 * j + li;
    if (col >= p.N) continue;
    float bj = 0.f;
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < p.M) {
          float v = acc[i][j][r];
          if (EPI == EPI_BIAS) v += bj;
          if (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
          if (EPI == EPI_DELU) {
            const float x = aux[(int64_t)row * p.ld_aux + col];
            v = x > 0.f ? v : v * (x + 1.f);
          }
          C[(int64_t)row * p.ldc + col] = v;
        }
      }
    }
  }
  // bias partial layout [split][group][M] (contiguous per split, like the C partials)
  if (do_bsum && threadIdx.x < BM && m0 + (int)threadIdx.x < p.M)
    p.bias_part[((int64_t)s * (gridDim.z / p.splits) + g) * p.M + m0 + threadIdx.x] = bsum;
}

template <int BM, int BN, int LAYOUT, int EPI>
static void launch_t(const GemmP& p, bool av, bool bv, dim3 grid, hipStream_t st) {
  if (av && bv)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LAYOUT, true, true, EPI>), grid, dim3(GTHREADS), 0, st, p);
  else if (av)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LAYOUT, true, false, EPI>), grid, dim3(GTHREADS), 0, st, p);
  else if (bv)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LAYOUT, false, true, EPI>), grid, dim3(GTHREADS), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LAYOUT, false, false, EPI>), grid, dim3(GTHREADS), 0, st, p);
}

template <int BM, int BN>
static int launch_bm(const GemmP& p, int layout, int epi, bool av, bool bv, dim3 grid, hipStream_t st) {
  switch (layout) {
    case GEMM_NT:
      switch (epi) {
        case EPI_STORE: launch_t<BM, BN, GEMM_NT, EPI_STORE>(p, av, bv, grid, st); return 0;
        case EPI_BIAS: launch_t<BM, BN, GEMM_NT, EPI_BIAS>(p, av, bv, grid, st); return 0;
        case EPI_BIAS_ELU: launch_t<BM, BN, GEMM_NT, EPI_BIAS_ELU>(p, av, bv, grid, st); return 0;
      }
      break;
    case GEMM_NN:
      switch (epi) {
        case EPI_STORE: launch_t<BM, BN, GEMM_NN, EPI_STORE>(p, av, bv, grid, st); return 0;
        case EPI_DELU: launch_t<BM, BN, GEMM_NN, EPI_DELU>(p, av, bv, grid, st); return 0;
      }
      break;
    case GEMM_TN:
      if (epi == EPI_PARTIAL) {
        launch_t<BM, BN, GEMM_TN, EPI_PARTIAL>(p, av, bv, grid, st);
        return 0;
      }
      break;
  }
  return LRL_E_INVALID;
}

static bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

int gemm_pick_splits(int M, int N, int K, int groups) {
  const int bm = M > 64 ? 128 : 64, bn = N > 64 ? 128 : 64;
  const int tiles = groups * ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int splits = 1;
  // aim for >= 512 workgroups, keep >= 256 rows per split and <= 128 splits
  while (tiles * splits < 512 && splits < 128 && (K / (splits * 2)) >= 256) splits *= 2;
  return splits;
}

int gemm_launch(const GemmP& p0, int layout, int epi, int groups, void* stream) {
  GemmP p = p0;
  if (p.M <= 0 || p.N <= 0 || p.K < 0 || groups <= 0) return LRL_E_INVALID;
  if (p.splits <= 0) p.splits = 1;
  if (p.kps <= 0) p.kps = (p.K + p.splits - 1) / p.splits;
  p.kps = (p.kps + GBK - 1) / GBK * GBK;
  const bool amc = layout & 1, bnc = layout & 2;
  // float4 staging needs the contiguous dimension's pitch and base 16-B aligned (group offsets too)
  const bool av = (p.lda % 4 == 0) && aligned16(p.A) && (p.ga % 4 == 0);
  const bool bv = (p.ldb % 4 == 0) && aligned16(p.B) && (p.gb % 4 == 0);
  (void)amc;
  (void)bnc;
  const int bm = p.M > 64 ? 128 : 64;
  const int bn = p.N > 64 ? 128 : 64;
  dim3 grid((p.M + bm - 1) / bm, (p.N + bn - 1) / bn, groups * p.splits);
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc;
  if (bm == 128 && bn == 128) rc = launch_bm<128, 128>(p, layout, epi, av, bv, grid, st);
  else if (bm == 128) rc = launch_bm<128, 64>(p, layout, epi, av, bv, grid, st);
  else if (bn == 128) rc = launch_bm<64, 128>(p, layout, epi, av, bv, grid, st);
  else rc = launch_bm<64, 64>(p, layout, epi, av, bv, grid, st);
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
}

}  // namespace lrl
