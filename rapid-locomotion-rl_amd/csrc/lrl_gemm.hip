// lrl_gemm.hip — fp32 MFMA GEMM kernels of the PPO update (see lrl_gemm.h for the contract).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>

#include "../../include/lrl.h"
#include "lrl_gemm.h"

namespace lrl {

typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifndef LRL_GBK
#define LRL_GBK 16
#endif
constexpr int GBK = LRL_GBK;  // k-slice per LDS stage
constexpr int KQ = GBK / 4;   // float4 items per k-contiguous row slice
constexpr int GTHREADS = 256;

template <int BM, int BN, int LAYOUT>
struct GemmTile {
  static constexpr bool AMC = (LAYOUT & 1) != 0;
  static constexpr bool BNC = (LAYOUT & 2) != 0;
  // k-major LDS images.  Transposing stores of k-contiguous operands: row pitch = 1 mod 8 words keeps the
  // 32 lanes of a half-wave (4 rows x 8 k-quads) on distinct banks; float4 stores of m/n-contiguous
  // operands need a 16-B aligned pitch.
  static constexpr int PK = GBK == 32 ? 1 : 2;
  static constexpr int PA = AMC ? 4 : PK;
  static constexpr int PB = BNC ? 4 : PK;
  static constexpr int IA = BM * GBK / 4, IB = BN * GBK / 4;  // float4 items per tile
  static constexpr int NA = (IA + GTHREADS - 1) / GTHREADS;   // per thread
  static constexpr int NB = (IB + GTHREADS - 1) / GTHREADS;
  // 4 waves: WM x WN wave grid, each wave TM x TN MFMA tiles of 32x32
  static constexpr int WN = (BM >= 64 && BN >= 64) ? 2 : (BM == 32 ? 4 : 1);
  static constexpr int WM = 4 / WN;
  static constexpr int TM = BM / (32 * WM);
  static constexpr int TN = BN / (32 * WN);
  static_assert(TM >= 1 && TN >= 1, "tile shape");
};

// trace tag of a weight-gradient shape (M x N per group, groups): 1 = the update's largest product, the actor /
// critic layer-2 gradient (256 x 512, 2 groups); 2 = their layer 3 (128 x 256, 2 groups); 3 = their layer 1
// (512 x 60); 4 = the adaptation module's first layer (256 x 630 history); 5 = the env-factor encoder's first
// layer (256 x 18); 6 = its second (128 x 256, 1 group); 0 = any other shape
static int tn_shape_tag(int M, int N, int groups) {
  if (M == 256 && N == 512) return 1;
  if (M == 128 && N == 256) return groups > 1 ? 2 : 6;
  if (M == 512 && N <= 64) return 3;
  if (M == 256 && N >= 600) return 4;
  if (M == 256 && N <= 64) return 5;
  return 0;
}

__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }

// load 4 consecutive floats (all in range) with the widest access the operand's alignment allows
__device__ __forceinline__ float4 load4(const float* __restrict__ src, int vec) {
  if (vec == 4) return *reinterpret_cast<const float4*>(src);
  if (vec == 2) {
    const float2 a = reinterpret_cast<const float2*>(src)[0], b = reinterpret_cast<const float2*>(src)[1];
    return make_float4(a.x, a.y, b.x, b.y);
  }
  return make_float4(src[0], src[1], src[2], src[3]);
}

// ---- global -> register staging of one BK slice ----
// k-contiguous operand X(r, k) = P[row(r) * ld + k]: item i covers (r = i / KQ, k = 4 (i % KQ) .. +3); the
// row pointers (through the gather list when there is one) are resolved once per workgroup.
// r-contiguous operand X(r, k) = P[krow(k) * ld + r]: item i covers (k = i / (R/4), r = 4 (i % (R/4)) .. +3).
template <int R, int NI, bool RCONTIG>
struct Stager {
  static constexpr int ITEMS = R * GBK / 4;
  const float* rowp[NI];  // k-contiguous: source row (nullptr: outside the tile / matrix)
  const float* P;
  const int64_t* rows;
  int64_t ld;
  int vec, r0, R_lim;

  __device__ __forceinline__ void init(const float* P_, int64_t ld_, const int64_t* rows_, int vec_, int r0_,
                                       int R_lim_) {
    P = P_; ld = ld_; rows = rows_; vec = vec_; r0 = r0_; R_lim = R_lim_;
    if (!RCONTIG) {
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = threadIdx.x + u * GTHREADS;
        const int gr = r0 + i / KQ;
        rowp[u] = nullptr;
        if ((ITEMS % GTHREADS == 0 || i < ITEMS) && gr < R_lim)
          rowp[u] = P + (rows ? rows[gr] : (int64_t)gr) * ld + 4 * (i % KQ);
      }
    }
  }

  __device__ __forceinline__ void load(float4 (&reg)[NI], int k0, int k_lim) const {
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = threadIdx.x + u * GTHREADS;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!RCONTIG) {
        const int k = k0 + 4 * (i % KQ);
        if (rowp[u]) {
          const float* src = rowp[u] + k0;
          if (k + 3 < k_lim) {
            v = load4(src, vec);
          } else {
            if (k + 0 < k_lim) v.x = src[0];
            if (k + 1 < k_lim) v.y = src[1];
            if (k + 2 < k_lim) v.z = src[2];
          }
        }
      } else if (ITEMS % GTHREADS == 0 || i < ITEMS) {
        const int r = 4 * (i % (R / 4)), k = k0 + i / (R / 4);
        const int gr = r0 + r;
        if (k < k_lim) {
          const int64_t row = rows ? rows[k] : (int64_t)k;
          const float* src = P + row * ld + gr;
          if (gr + 3 < R_lim) {
            v = load4(src, vec);
          } else {
            if (gr + 0 < R_lim) v.x = src[0];
            if (gr + 1 < R_lim) v.y = src[1];
            if (gr + 2 < R_lim) v.z = src[2];
          }
        }
      }
      reg[u] = v;
    }
  }

  // interior slice of a tile whose rows, columns and k range are all in bounds, float4-aligned operand
  __device__ __forceinline__ void load_fast(float4 (&reg)[NI], int k0) const {
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = threadIdx.x + u * GTHREADS;
      if (ITEMS % GTHREADS != 0 && i >= ITEMS) continue;
      if (!RCONTIG) {
        reg[u] = *reinterpret_cast<const float4*>(rowp[u] + k0);
      } else {
        const int r = 4 * (i % (R / 4)), k = k0 + i / (R / 4);
        const int64_t row = rows ? rows[k] : (int64_t)k;
        reg[u] = *reinterpret_cast<const float4*>(P + row * ld + r0 + r);
      }
    }
  }
};

template <int R, int PAD, int NI, bool RCONTIG>
__device__ __forceinline__ void stage_store(float (*S)[R + PAD], const float4 (&reg)[NI]) {
  constexpr int ITEMS = R * GBK / 4;
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = threadIdx.x + u * GTHREADS;
    if (ITEMS % GTHREADS != 0 && i >= ITEMS) {
    } else if (!RCONTIG) {
      const int r = i / KQ, k = 4 * (i % KQ);
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

template <int BM, int BN, int LAYOUT, int EPI>
__global__ __launch_bounds__(GTHREADS) void gemm_kernel(GemmP p) {
  using T = GemmTile<BM, BN, LAYOUT>;
  __shared__ __attribute__((aligned(16))) float As[2][GBK][BM + T::PA];
  __shared__ __attribute__((aligned(16))) float Bs[2][GBK][BN + T::PB];
  // XCD-aware tile order: the hardware deals workgroup ids round-robin over the 8 XCDs, so id i is
  // renumbered to L with consecutive L on the same XCD; L runs n-tile fastest, then m-tile, then
  // (group, split): the workgroups sharing an A row-panel (or a split's rows) share one XCD's L2.
  const int mt = (p.M + BM - 1) / BM, nt = (p.N + BN - 1) / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, zz = L / (nt * mt);
  const int groups = p.groups;
  const int g = zz / p.splits, s = zz - g * p.splits;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int kbeg = s * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, h = lane >> 5;
  constexpr int TM = T::TM, TN = T::TN;
  const int wm = (w / T::WN) * (BM / T::WM), wn = (w % T::WN) * (BN / T::WN);
  const int64_t* a_rows = T::AMC ? nullptr : p.a_rows;
  const int64_t* b_rows = T::BNC ? p.b_rows : nullptr;

  // NACC independent accumulator chains per output tile (k-steps alternate between them) when a wave owns
  // a single 32x32 tile, so consecutive MFMAs of the wave do not wait on each other's results
#ifndef LRL_GEMM_SPLITACC
#define LRL_GEMM_SPLITACC 1
#endif
  constexpr int NACC = (LRL_GEMM_SPLITACC && TM * TN == 1) ? 2 : 1;
  f32x16 acc[TM][TN], acc2[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = acc2[i][j][r] = 0.f;

  // bias-gradient partial (weight-gradient products): column sums of A(m, k) over this split's k
  const bool do_bsum = EPI == EPI_PARTIAL && p.bias_part != nullptr && tn_ == 0;
  float bsum = 0.f;

  float4 ra[T::NA], rb[T::NB];
  Stager<BM, T::NA, T::AMC> sa;
  Stager<BN, T::NB, T::BNC> sb;
  sa.init(A, p.lda, a_rows, p.avec, m0, p.M);
  sb.init(B, p.ldb, b_rows, p.bvec, n0, p.N);
  // uniform fast path: whole tile in bounds, every k slice full, float4 staging on both operands
  const bool fast = m0 + BM <= p.M && n0 + BN <= p.N && ((kend - kbeg) % GBK) == 0 && p.avec == 4 && p.bvec == 4;
  // backward-data epilogue operand (the layer input, for elu'): fetched up front so its latency hides
  // under the main loop instead of trailing it
  float xaux[EPI == EPI_DELU ? TM : 1][EPI == EPI_DELU ? TN : 1][16];
  if constexpr (EPI == EPI_DELU) {
    const float* __restrict__ ax = p.aux + g * p.gaux;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = min(n0 + wn + 32 * j + li, p.N - 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = min(m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h, p.M - 1);
          xaux[i][j][r] = ax[(int64_t)row * p.ld_aux + col];
        }
    }
  }
  int k0 = kbeg;
  if (k0 < kend) {
    if (fast) {
      sa.load_fast(ra, k0);
      sb.load_fast(rb, k0);
    } else {
      sa.load(ra, k0, kend);
      sb.load(rb, k0, kend);
    }
    stage_store<BM, T::PA, T::NA, T::AMC>(As[0], ra);
    stage_store<BN, T::PB, T::NB, T::BNC>(Bs[0], rb);
  }
  __syncthreads();
  int buf = 0;
  for (; k0 < kend; k0 += GBK) {
    const int kn = k0 + GBK;
    if (kn < kend) {
      if (fast) {
        sa.load_fast(ra, kn);
        sb.load_fast(rb, kn);
      } else {
        sa.load(ra, kn, kend);
        sb.load(rb, kn, kend);
      }
    }
    if (do_bsum && threadIdx.x < BM) {
#pragma unroll
      for (int k = 0; k < GBK; ++k) bsum += As[buf][k][threadIdx.x];
    }
    // all operands of the slice first (GBK/2 x (TM + TN) ds_read_b32), then the MFMAs back to back, so no
    // MFMA waits on an LDS read issued right before it
    float a[GBK / 2][TM], b[GBK / 2][TN];
#pragma unroll
    for (int kk = 0; kk < GBK / 2; ++kk) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[kk][i] = As[buf][2 * kk + h][wm + 32 * i + li];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[kk][j] = Bs[buf][2 * kk + h][wn + 32 * j + li];
    }
    __builtin_amdgcn_sched_barrier(0);
    // MFMAs at raised wave priority: the other waves' staging work fills the MFMA shadow instead of
    // delaying the next MFMA issue (measured +8..17% on the update's shapes, scripts/gemm_bench.py)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < GBK / 2; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (NACC == 2 && (kk & 1))
            acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][i], b[kk][j], acc2[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
    // keep the scheduler from sinking the LDS reads back next to their MFMAs
    __builtin_amdgcn_sched_barrier(0);
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
          float v = NACC == 2 ? acc[i][j][r] + acc2[i][j][r] : acc[i][j][r];
          if (EPI == EPI_BIAS) v += bj;
          if (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
          if constexpr (EPI == EPI_DELU) {
            const float x = xaux[i][j][r];
            v = x > 0.f ? v : v * (x + 1.f);
          }
          C[(int64_t)row * p.ldc + col] = v;
        }
      }
    }
  }
  // bias partial layout [split][group][M] (contiguous per split, like the C partials)
  if (do_bsum && threadIdx.x < BM && m0 + (int)threadIdx.x < p.M)
    p.bias_part[((int64_t)s * groups + g) * p.M + m0 + threadIdx.x] = bsum;
}

// ---------------------------------------------------------------------------------------------------
// LDS-DMA variant for the interior batch-major products (forward NT, backward-data NN) with float4-aligned
// operands: 64x64 tile, 4 waves each owning a 32x32 MFMA tile, BK = 16, a 3-deep ring of LDS stages
// filled by global_load_lds_dwordx4 (no staging registers, no ds_write pass), counted vmcnt waits and a
// raw s_barrier so the loads of slice k+2 stay in flight while slice k is consumed.
//   k-contiguous operands (A; B of NT) land as [row][16 k] images, 16-B chunk c of row r stored in slot
//   c ^ ((r >> 2) & 3) (the swizzle is applied to the SOURCE address, the DMA destination stays lane-linear),
//   and each lane reads its row's 8 k-values (k = 8h .. 8h+7) with two conflict-free ds_read_b128;
//   the n-contiguous B of NN lands as [16 k][64 n] and is read with ds_read_b32 (consecutive n per lane).
// MFMA k-step t of lane half h uses k = 8h + t for both operands, so the sum runs over every k once.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int LAYOUT, int EPI>
__global__ __launch_bounds__(GTHREADS) void gemm_glds_kernel(GemmP p) {
  constexpr int BM = 64, BN = 64, BKD = 16, NST = 3, IMG = 1024;
  constexpr bool BNC = (LAYOUT & 2) != 0;
  static_assert((LAYOUT & 1) == 0, "A must be k-contiguous");
  __shared__ __attribute__((aligned(16))) float S[NST * 2 * IMG];  // [stage][A | B][image], one LDS object
  const int mt = p.M / BM, nt = p.N / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, g = L / (nt * mt);
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const int K = p.K;

  // this lane's DMA sources: A rows 16w + lane/4 (chunk pre-swizzled); B likewise (NT) or k-row 4w + lane/16 (NN)
  const int ar = 16 * w + (lane >> 2);
  const int achunk = (lane & 3) ^ ((ar >> 2) & 3);
  const float* asrc = A + (p.a_rows ? p.a_rows[m0 + ar] : (int64_t)(m0 + ar)) * p.lda + 4 * achunk;
  const float* bsrc;
  if constexpr (!BNC) {
    bsrc = B + (int64_t)(n0 + ar) * p.ldb + 4 * achunk;
  } else {
    bsrc = B + (int64_t)(4 * w + (lane >> 4)) * p.ldb + n0 + 4 * (lane & 15);
  }
  // the DMA is issued from inline asm so the compiler does not track it (it would otherwise drain it with
  // vmcnt(0) before every ds_read); completion is ordered by the counted waits below
  const uint32_t s_lds = (uint32_t)(uintptr_t)(lds_ptr_t)S;
  auto dma = [&](const float* src, uint32_t lds_off) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_off)
                 : "memory");
  };
  auto issue = [&](int st, int k0) {
    const uint32_t base = __builtin_amdgcn_readfirstlane(s_lds + (uint32_t)((st * 2 * IMG + w * 256) * 4));
    dma(asrc + k0, base);
    dma(BNC ? bsrc + (int64_t)k0 * p.ldb : bsrc + k0, base + IMG * 4);
  };

  // backward-data epilogue operand (elu' of the layer input), fetched before the DMA ring starts
  float xaux[16];
  if constexpr (EPI == EPI_DELU) {
    const float* __restrict__ ax = p.aux + g * p.gaux;
    const int col = n0 + wn + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      xaux[r] = ax[(int64_t)row * p.ld_aux + col];
    }
  }

  f32x16 acc, acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;

  const int ns = K / BKD;
  issue(0, 0);
  if (ns > 1) issue(1, BKD);
  const int ai = wm + li, aswz = (ai >> 2) & 3;
  const int bi = wn + li, bswz = (bi >> 2) & 3;
  for (int s = 0; s < ns; ++s) {
    // this wave's DMA of slice s has landed (slice s+1's two loads may stay in flight) ...
    if (s + 1 < ns) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ... and every wave's, and every wave is done reading the stage slice s+2 will overwrite
    __builtin_amdgcn_s_barrier();
    if (s + 2 < ns) issue((s + 2) % NST, (s + 2) * BKD);
    const float* As = S + (s % NST) * 2 * IMG;
    const float* Bs = As + IMG;
    float a[8], b[8];
    {
      const float4 a0 = *reinterpret_cast<const float4*>(As + ai * 16 + 4 * ((2 * h) ^ aswz));
      const float4 a1 = *reinterpret_cast<const float4*>(As + ai * 16 + 4 * ((2 * h + 1) ^ aswz));
      a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
    }
    if constexpr (!BNC) {
      const float4 b0 = *reinterpret_cast<const float4*>(Bs + bi * 16 + 4 * ((2 * h) ^ bswz));
      const float4 b1 = *reinterpret_cast<const float4*>(Bs + bi * 16 + 4 * ((2 * h + 1) ^ bswz));
      b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) b[t] = Bs[(8 * h + t) * BN + bi];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (t & 1) acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], acc2, 0, 0, 0);
      else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], acc, 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }

  float* __restrict__ C = p.C + g * p.gc;
  const int col = n0 + wn + li;
  float bj = 0.f;
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = p.bias[g * p.gbias + col];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h;
    float v = acc[r] + acc2[r];
    if constexpr (EPI == EPI_BIAS) v += bj;
    if constexpr (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
    if constexpr (EPI == EPI_DELU) {
      const float x = xaux[r];
      v = x > 0.f ? v : v * (x + 1.f);
    }
    C[(int64_t)row * p.ldc + col] = v;
  }
}


// BK = 32 variant of the LDS-DMA kernel (k a multiple of 32): 16 MFMAs per wave between barriers instead
// of 8.  [row][32 k] images (128-B rows): 16-B chunk c of row r sits in slot c ^ ((r >> 1) & 7), so the 8
// lanes of a ds_read_b128 group (8 consecutive rows, one chunk) hit 8 distinct 16-B bank groups; DMA d of a
// slice fills rows 8d .. 8d+7 (lane l: row 8d + l / 8, slot l % 8, source chunk pre-swizzled).  The NN B image
// is [32 k][64 n], DMA d filling k-rows 4d .. 4d+3.  Lane half h uses k = 16h .. 16h+15 at MFMA steps 0..15.
template <int LAYOUT, int EPI>
__global__ __launch_bounds__(GTHREADS) void gemm_glds32_kernel(GemmP p) {
  constexpr int BM = 64, BN = 64, BKD = 32, NST = 3, IMG = 2048;
  constexpr bool BNC = (LAYOUT & 2) != 0;
  static_assert((LAYOUT & 1) == 0, "A must be k-contiguous");
  __shared__ __attribute__((aligned(16))) float S[NST * 2 * IMG];
  const int mt = p.M / BM, nt = p.N / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, g = L / (nt * mt);
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const int K = p.K;
  const float* asrc[2];
  const float* bsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = 2 * w + i, row = 8 * d + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    asrc[i] = A + (p.a_rows ? p.a_rows[m0 + row] : (int64_t)(m0 + row)) * p.lda + 4 * chunk;
    if constexpr (!BNC) bsrc[i] = B + (int64_t)(n0 + row) * p.ldb + 4 * chunk;
    else bsrc[i] = B + (int64_t)(4 * d + (lane >> 4)) * p.ldb + n0 + 4 * (lane & 15);
  }
  const uint32_t s_lds = (uint32_t)(uintptr_t)(lds_ptr_t)S;
  auto dma = [&](const float* src, uint32_t lds_off) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_off)
                 : "memory");
  };
  auto issue = [&](int st, int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t base =
          __builtin_amdgcn_readfirstlane(s_lds + (uint32_t)((st * 2 * IMG + (2 * w + i) * 256) * 4));
      dma(asrc[i] + k0, base);
      dma(BNC ? bsrc[i] + (int64_t)k0 * p.ldb : bsrc[i] + k0, base + IMG * 4);
    }
  };
  float xaux[16];
  if constexpr (EPI == EPI_DELU) {
    const float* __restrict__ ax = p.aux + g * p.gaux;
    const int col = n0 + wn + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      xaux[r] = ax[(int64_t)row * p.ld_aux + col];
    }
  }
  f32x16 acc, acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
  const int ns = K / BKD;
  issue(0, 0);
  if (ns > 1) issue(1, BKD);
  const int ai = wm + li, aswz = (ai >> 1) & 7;
  const int bi = wn + li, bswz = (bi >> 1) & 7;
  for (int s = 0; s < ns; ++s) {
    if (s + 1 < ns) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 2 < ns) issue((s + 2) % NST, (s + 2) * BKD);
    const float* As = S + (s % NST) * 2 * IMG;
    const float* Bs = As + IMG;
    float a[16], b[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(As + ai * 32 + 4 * ((4 * h + q) ^ aswz));
      a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
    }
    if constexpr (!BNC) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(Bs + bi * 32 + 4 * ((4 * h + q) ^ bswz));
        b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) b[t] = Bs[(16 * h + t) * BN + bi];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (t & 1) acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], acc2, 0, 0, 0);
      else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], acc, 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  float* __restrict__ C = p.C + g * p.gc;
  const int col = n0 + wn + li;
  float bj = 0.f;
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = p.bias[g * p.gbias + col];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h;
    float v = acc[r] + acc2[r];
    if constexpr (EPI == EPI_BIAS) v += bj;
    if constexpr (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
    if constexpr (EPI == EPI_DELU) {
      const float x = xaux[r];
      v = x > 0.f ? v : v * (x + 1.f);
    }
    C[(int64_t)row * p.ldc + col] = v;
  }
}

// ---- thin products: C[M][N <= 32] = A[M][K] op(B), K = 128 NBK (512 or 1024) ----
// (the latent gradient dY W[:, 42:60] over k = 1024, the 18-/32-wide output layers.)  A register-staged
// 32-wide tile wastes most of its loads here and a split-k launch pays a partial round trip through HBM,
// so: a workgroup's 4 waves take k in quarters; each lane keeps its column of op(B) for the whole quarter
// in registers (loaded once per workgroup; lanes past N hold zeros), the workgroup walks 32-row tiles
// (persistent grid) with A streamed from global memory one 32-k block ahead (lane (i, h) loads row i's
// float4s at k = 8v + 4h, the k-permutation its B registers follow), and the quarter sums are added in
// wave order (fixed, deterministic) before the epilogue.
template <int LAYOUT, int EPI, int NBK>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_thin_kernel(GemmP p) {
  __shared__ float red[3 * 16 * 64];
  constexpr bool BNC = (LAYOUT & 2) != 0;
  const int N = p.N, M = p.M;
  const int g = blockIdx.y;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  float* __restrict__ C = p.C + g * p.gc;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 31, h = lane >> 5;
  const int kbeg = w * 32 * NBK;
  const bool colv = li < N;
  float breg[NBK][16];
#pragma unroll
  for (int kb = 0; kb < NBK; ++kb)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int k = kbeg + 32 * kb + 8 * (t >> 2) + 4 * h + (t & 3);
      breg[kb][t] = colv ? (BNC ? B[(int64_t)k * p.ldb + li] : B[(int64_t)li * p.ldb + k]) : 0.f;
    }
  const int mt = (M + 31) >> 5;
  auto rowp = [&](int t) -> const float* {
    const int row = t * 32 + li;
    if (t >= mt || row >= M) return nullptr;
    return A + (p.a_rows ? p.a_rows[row] : (int64_t)row) * p.lda + kbeg + 4 * h;
  };
  auto load = [&](const float* ar, int kb, float4* dst) {
#pragma unroll
    for (int v = 0; v < 4; ++v)
      dst[v] = ar ? *reinterpret_cast<const float4*>(ar + 32 * kb + 8 * v) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const float* ar = rowp(blockIdx.x);
  float4 cur[4];
  load(ar, 0, cur);
  for (int t = blockIdx.x; t < mt; t += gridDim.x) {
    const float* arn = rowp(t + gridDim.x);
    f32x16 acc, acc2;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
#pragma unroll
    for (int kb = 0; kb < NBK; ++kb) {
      float4 nxt[4];
      if (kb + 1 < NBK) load(ar, kb + 1, nxt);
      else load(arn, 0, nxt);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float av = (s & 3) == 0 ? cur[s >> 2].x : (s & 3) == 1 ? cur[s >> 2].y : (s & 3) == 2 ? cur[s >> 2].z : cur[s >> 2].w;
        if (s & 1) acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, breg[kb][s], acc2, 0, 0, 0);
        else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, breg[kb][s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) cur[v] = nxt[v];
    }
    ar = arn;
    if (w > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((w - 1) * 16 + r) * 64 + lane] = acc[r] + acc2[r];
    }
    __syncthreads();
    if (w == 0) {
      float bj = 0.f;
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = colv ? p.bias[g * p.gbias + li] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = acc[r] + acc2[r];
        v += red[r * 64 + lane];
        v += red[(16 + r) * 64 + lane];
        v += red[(32 + r) * 64 + lane];
        if constexpr (EPI == EPI_BIAS) v += bj;
        if constexpr (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
        const int orow = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (colv && orow < M) C[(int64_t)orow * p.ldc + li] = v;
      }
    }
    __syncthreads();
  }
}

// The same product on 16-row tiles (v_mfma_f32_16x16x4_f32, two 16-column blocks): 1,536 tiles of the 24,576-row
// minibatch deal evenly over the 512-workgroup persistent grid (3 each), where 768 32-row tiles leave half the
// workgroups one tile short.  Lane (h, i) of a wave loads row i's float4 at k = 16 s + 4 h and feeds its four values
// to four consecutive MFMA steps; its B registers hold column i (+16) at the same k.
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int LAYOUT, int EPI, int NBK>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_thin16_kernel(GemmP p) {
  __shared__ float red[3 * 8 * 64];
  constexpr bool BNC = (LAYOUT & 2) != 0;
  constexpr int KS = 2 * NBK;  // 16-k blocks of a wave's quarter (32 NBK k)
  const int N = p.N, M = p.M;
  const int g = blockIdx.y;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  float* __restrict__ C = p.C + g * p.gc;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, h = lane >> 4;
  const int kbeg = w * 32 * NBK;
  float breg[KS][2][4];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kbeg + 16 * s + 4 * h + u, col = i + 16 * cb;
        breg[s][cb][u] = col < N ? (BNC ? B[(int64_t)k * p.ldb + col] : B[(int64_t)col * p.ldb + k]) : 0.f;
      }
  const int mt = (M + 15) >> 4;
  auto rowp = [&](int t) -> const float* {
    const int row = t * 16 + i;
    if (t >= mt || row >= M) return nullptr;
    return A + (p.a_rows ? p.a_rows[row] : (int64_t)row) * p.lda + kbeg + 4 * h;
  };
  auto load = [&](const float* ar, int s0, float4* dst) {  // 4 blocks of 16 k
#pragma unroll
    for (int v = 0; v < 4; ++v)
      dst[v] = ar ? *reinterpret_cast<const float4*>(ar + 16 * (s0 + v)) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const float* ar = rowp(blockIdx.x);
  float4 cur[4];
  load(ar, 0, cur);
  for (int t = blockIdx.x; t < mt; t += gridDim.x) {
    const float* arn = rowp(t + gridDim.x);
    f32x4v acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s0 = 0; s0 < KS; s0 += 4) {
      float4 nxt[4];
      if (s0 + 4 < KS) load(ar, s0 + 4, nxt);
      else load(arn, 0, nxt);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float av[4] = {cur[v].x, cur[v].y, cur[v].z, cur[v].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], breg[s0 + v][0][u], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], breg[s0 + v][1][u], acc1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) cur[v] = nxt[v];
    }
    ar = arn;
    if (w > 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[((w - 1) * 8 + r) * 64 + lane] = acc0[r];
        red[((w - 1) * 8 + 4 + r) * 64 + lane] = acc1[r];
      }
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int col = i + 16 * cb;
        float bj = 0.f;
        if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = col < N ? p.bias[g * p.gbias + col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = cb ? acc1[r] : acc0[r];
          v += red[(4 * cb + r) * 64 + lane];
          v += red[(8 + 4 * cb + r) * 64 + lane];
          v += red[(16 + 4 * cb + r) * 64 + lane];
          if constexpr (EPI == EPI_BIAS) v += bj;
          if constexpr (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
          const int orow = t * 16 + 4 * h + r;
          if (col < N && orow < M) C[(int64_t)orow * p.ldc + col] = v;
        }
      }
    }
    __syncthreads();
  }
}

// (LRL_THIN16=0: development switch back to the 32-row tiles)
static bool thin16_enabled() {
  static const int on = [] {
    const char* e = getenv("LRL_THIN16");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}

template <int LAYOUT, int EPI, int NBK>
static int launch_thin_k(const GemmP& p, int groups, hipStream_t st) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return LRL_E_HIP;
    ncu = prop.multiProcessorCount;
  }
  if (thin16_enabled()) {
    const int mt = (p.M + 15) / 16;
    const int gx = std::max(1, std::min(mt, 2 * ncu / std::max(1, groups)));
    hipLaunchKernelGGL((gemm_thin16_kernel<LAYOUT, EPI, NBK>), dim3(gx, groups), dim3(GTHREADS), 0, st, p);
    return 0;
  }
  const int mt = (p.M + 31) / 32;
  const int gx = std::max(1, std::min(mt, 2 * ncu / std::max(1, groups)));
  hipLaunchKernelGGL((gemm_thin_kernel<LAYOUT, EPI, NBK>), dim3(gx, groups), dim3(GTHREADS), 0, st, p);
  return 0;
}
template <int LAYOUT, int EPI>
static int launch_thin(const GemmP& p, int groups, hipStream_t st) {
  switch (p.K / 128) {
    case 4: return launch_thin_k<LAYOUT, EPI, 4>(p, groups, st);
    case 8: return launch_thin_k<LAYOUT, EPI, 8>(p, groups, st);
  }
  return LRL_E_INVALID;
}

// ---------------------------------------------------------------------------------------------------
// LDS-DMA weight-gradient product (TN, split-k partials): dW[o][i] = sum_b dY[b][o] X[rows(b)][i] over a
// split's rows b.  Both operands are b-major in memory, so a 16-row slice of each is a [16 k][128] image
// that global_load_lds_dwordx4 fills row by row (DMA d of a slice covers k-rows 2d, 2d + 1); a 3-deep ring
// of slices with counted vmcnt waits keeps two slices in flight under the MFMAs.  128x128 tile, 4 waves
// each 64x64 (2x2 MFMA tiles); MFMA operands are ds_read_b32 of [k][m] / [k][n] (consecutive m / n per
// lane).  The split's gathered row list is converted to int32 in LDS once.  Bias-gradient partial: column
// sums of the dY slice (n-tile 0 workgroups).
// SHAPE: trace tag only (the code is the same for every value): each weight-gradient shape of the update gets
// its own symbol, so a kernel trace / PMC pass keys its launches apart (see tn_shape_tag)
template <int NST, int BN, int SHAPE>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_glds_tn_kernel(GemmP p) {
  // BN = 128: 4 waves of 64x64 (2x2 MFMA tiles); BN = 64 (narrow inputs, e.g. the 60-wide actor/critic input):
  // 4 waves of 64x32
  constexpr int BM = 128, BKD = 16, IMGA = BKD * BM, IMGB = BKD * BN, TN = BN / 64;
  constexpr int NB_DMA = IMGB / 256;  // 1 KiB DMAs per B slice (4 or 8): per wave NB_DMA / 4
  extern __shared__ __attribute__((aligned(16))) float S[];  // [NST][A 16x128 | B 16xBN], then int32 rows
  const int mt = p.M / BM, nt = (p.N + BN - 1) / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, zz = L / (nt * mt);
  const int g = zz / p.splits, sp = zz - g * p.splits;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int kbeg = sp * p.kps, kend = min(p.K, kbeg + p.kps);
  const int ns = (kend - kbeg) / BKD;
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ B = p.B + g * p.gb;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * 64, wn = (w & 1) * (BN / 2);
  constexpr int STG = IMGA + IMGB;
  int* rows = reinterpret_cast<int*>(S + NST * STG);
  if (p.b_rows) {
    for (int i = threadIdx.x; i < kend - kbeg; i += GTHREADS) rows[i] = (int)p.b_rows[kbeg + i];
    __syncthreads();
  }
  const uint32_t s_lds = (uint32_t)(uintptr_t)(lds_ptr_t)S;
  auto dma = [&](const float* src, uint32_t lds_off) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_off)
                 : "memory");
  };
  // A: DMA d = 4 i + w (i = 0, 1) fills k-rows 2d + h (128 floats each), 16-B chunk li;
  // B: DMA d = 4 i + w (i < NB_DMA / 4) fills k-rows d * (256 / BN) + lane / (BN / 4), chunk lane % (BN / 4)
  auto issue = [&](int st, int s) {
    const int kl = s * BKD;
    const uint32_t sbase = s_lds + (uint32_t)(st * STG * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int d = 4 * i + w, kr = kl + 2 * d + h;
      dma(A + (int64_t)(kbeg + kr) * p.lda + m0 + 4 * li, __builtin_amdgcn_readfirstlane(sbase + d * 1024));
    }
#pragma unroll
    for (int i = 0; i < NB_DMA / 4; ++i) {
      constexpr int CPR = BN / 4;
      const int d = 4 * i + w, kr = kl + d * (64 / CPR) + lane / CPR;
      const int64_t brow = p.b_rows ? (int64_t)rows[kr] : (int64_t)(kbeg + kr);
      dma(B + brow * p.ldb + n0 + 4 * (lane % CPR), __builtin_amdgcn_readfirstlane(sbase + IMGA * 4 + d * 1024));
    }
  };
  const bool do_bsum = p.bias_part != nullptr && tn_ == 0;
  float bsum = 0.f;
  f32x16 acc[2][TN];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < TN; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
  static_assert(NST == 3, "the counted waits below assume a 3-deep ring");
  if (ns > 0) issue(0, 0);
  if (ns > 1) issue(1, 1);
  for (int s = 0; s < ns; ++s) {
    // this wave's DMAs of slice s have landed (slice s+1's 2 + NB_DMA/4 may stay in flight) ...
    if (s + 1 < ns) {
      if constexpr (NB_DMA == 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + 2 < ns) issue((s + 2) % NST, s + 2);
    const float* As = S + (s % NST) * STG;
    const float* Bs = As + IMGA;
    if (do_bsum && threadIdx.x < BM) {
#pragma unroll
      for (int k = 0; k < BKD; ++k) bsum += As[k * BM + threadIdx.x];
    }
    float av[8][2], bv[8][TN];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
      for (int a = 0; a < 2; ++a) av[t][a] = As[(2 * t + h) * BM + wm + 32 * a + li];
#pragma unroll
      for (int c = 0; c < TN; ++c) bv[t][c] = Bs[(2 * t + h) * BN + wn + 32 * c + li];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < TN; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t][a], bv[t][c], acc[a][c], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  float* __restrict__ C = p.C + g * p.gc + (int64_t)sp * p.part_stride;
#pragma unroll
  for (int c = 0; c < TN; ++c) {
    const int col = n0 + wn + 32 * c + li;
    if (col >= p.N) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        C[(int64_t)row * p.ldc + col] = acc[a][c][r];
      }
  }
  if (do_bsum && threadIdx.x < BM)
    p.bias_part[((int64_t)sp * p.groups + g) * p.M + m0 + threadIdx.x] = bsum;
}

template <int BN, int SHAPE>
static int launch_glds_tn_tag(const GemmP& p, int groups, hipStream_t st) {
  const size_t lds = (size_t)3 * 16 * (128 + BN) * sizeof(float) + (p.b_rows ? (size_t)p.kps * sizeof(int) : 0);
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_glds_tn_kernel<3, BN, SHAPE>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return LRL_E_HIP;
    attr = true;
  }
  dim3 gt((p.M / 128) * ((p.N + BN - 1) / BN) * groups * p.splits);
  hipLaunchKernelGGL((gemm_glds_tn_kernel<3, BN, SHAPE>), gt, dim3(GTHREADS), lds, st, p);
  return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
}

template <int BN>
static int launch_glds_tn(const GemmP& p, int groups, hipStream_t st) {
  switch (tn_shape_tag(p.M, p.N, groups)) {
    case 1: return launch_glds_tn_tag<BN, 1>(p, groups, st);
    case 2: return launch_glds_tn_tag<BN, 2>(p, groups, st);
    case 3: return launch_glds_tn_tag<BN, 3>(p, groups, st);
    case 4: return launch_glds_tn_tag<BN, 4>(p, groups, st);
    case 5: return launch_glds_tn_tag<BN, 5>(p, groups, st);
    case 6: return launch_glds_tn_tag<BN, 6>(p, groups, st);
    default: return launch_glds_tn_tag<BN, 0>(p, groups, st);
  }
}

// ---------------------------------------------------------------------------------------------------
// fp32 products on the bf16 MFMA ("x6"): every operand element is split exactly into three bf16 parts,
// x = hi + mid + lo (truncation: hi takes the top 8 significant bits, mid the next 8 of the exact remainder,
// lo the rest — 24 bits in all, so nothing is lost), and a 32x32x16 k-step sums the six products whose
// order is above 2^-24 (lo*hi, mid*mid, hi*lo, mid*hi, hi*mid, hi*hi, smallest first) into an fp32
// accumulator.  The dropped products (mid*lo, lo*mid, lo*lo) are below 2^-24 of |a b|, so the result is
// as accurate as the fp32 MFMA's (measured: max |C - C_fp64| / sum|a b| 1.6-2.1e-7 for both on the update's
// shapes, scripts/proto_x6.hip), at 6 x 32 cycles per 32x32x16 step instead of 8 x 64 for the fp32 form.
// The split happens once per element while staging: global -> registers (fp32), split, three bf16 plane
// images -> LDS; each MFMA operand is then one ds_read_b128 per plane.
//   k-contiguous operand ([r][k]: A of NT / NN, B of NT): float4 loads, thread i covers row i/4, k-quad i%4;
//   r-contiguous operand ([k][r]: B of NN, A and B of TN): a thread loads a run of R/16 consecutive k of one
//   row r (dword loads, coalesced over r), so its split parts land as one contiguous run of the [r][k] image.
// Plane images are [R][16] bf16 (32-B rows); 16-B chunk c of row r sits in slot c ^ ((r >> 3) & 1), which keeps
// the 16-lane groups of the ds_read_b128 operand reads conflict-free.
// BM x BN tile (64 or 128 each), 4 waves in a 2 x 2 grid, wave tile (BM/2) x (BN/2) = TM x TN MFMA tiles;
// BK = 16, two LDS stages, the next slice's global loads in flight under the current slice's MFMAs.
constexpr int XBK = 16;
#ifndef LRL_X6_PIPE
#define LRL_X6_PIPE 1  // software-pipelined main loop (see gemm_x6_kernel)
#endif
#ifndef LRL_X6_PIPE_VALU
#define LRL_X6_PIPE_VALU 4  // VALU instructions scheduled after each MFMA of the pipelined loop
#endif

__device__ __forceinline__ uint32_t x6_hi_pair(uint32_t u0, uint32_t u1) {
  return __builtin_amdgcn_perm(u1, u0, 0x07060302u);  // (u1 & 0xffff0000) | (u0 >> 16)
}
// (x0, x1) -> the packed bf16 pairs of their hi / mid / lo parts
__device__ __forceinline__ void x6_split2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  uint32_t u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
  h = x6_hi_pair(u0, u1);
  float r0 = x0 - __uint_as_float(u0 & 0xffff0000u), r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
  u0 = __float_as_uint(r0);
  u1 = __float_as_uint(r1);
  m = x6_hi_pair(u0, u1);
  r0 = r0 - __uint_as_float(u0 & 0xffff0000u);
  r1 = r1 - __uint_as_float(u1 & 0xffff0000u);
  l = x6_hi_pair(__float_as_uint(r0), __float_as_uint(r1));
}
__device__ __forceinline__ int x6_off(int r, int c) { return r * XBK + 8 * (c ^ ((r >> 3) & 1)); }

typedef short bf16x8_t __attribute__((ext_vector_type(8)));

template <int R, bool KC, bool KGATHER = false>
struct X6Op {
  static constexpr int PLANE = R * XBK;                 // bf16 elements of one plane image
  static constexpr int NI = KC ? R / 64 : 1;             // float4 items per thread (k-contiguous)
  static constexpr int KR = KC ? 4 : R / 16;             // k-run per thread (r-contiguous): 8 or 4
  static constexpr int NV = KC ? 4 * NI : KR;  // staged values per thread and slice
  const float* rowp[NI];  // k-contiguous: row pointers (nullptr: row outside the operand)
  const float* P;
  const int64_t* krows;
  int64_t ld;
  int ldi, roff;  // r-contiguous: 32-bit element offsets from the (wave-uniform) operand base
  int rr, kb;     // r-contiguous: this thread's row in the tile and k offset of its run
  bool rok;
  bool vec4;      // k-contiguous: rows 16-B aligned (float4 loads); otherwise dword loads

  __device__ __forceinline__ void init(const float* P_, int64_t ld_, const int64_t* rows, const int64_t* krows_,
                                       int r0, int R_lim, bool vec4_ = true) {
    P = P_; ld = ld_; krows = krows_; vec4 = vec4_;
    const int t = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int r = (t >> 2) + 64 * u, gr = r0 + r;
        rowp[u] = gr < R_lim ? P_ + (rows ? rows[gr] : (int64_t)gr) * ld_ + 4 * (t & 3) : nullptr;
      }
    } else {
      rr = t % R;
      kb = __builtin_amdgcn_readfirstlane(KR * (t / R));  // wave-uniform: the run's row list reads are scalar
      rok = r0 + rr < R_lim;
      ldi = (int)ld_;
      roff = r0 + rr;
    }
  }
  __device__ __forceinline__ void load(float (&v)[NV], int k0, int k_lim, bool fast) const {
    if (KC) {
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int k = k0 + 4 * (threadIdx.x & 3);
        float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
        if (fast) {
          q = *reinterpret_cast<const float4*>(rowp[u] + k0);
        } else if (rowp[u]) {
          const float* s = rowp[u] + k0;
          if (k + 3 < k_lim && vec4) {
            q = *reinterpret_cast<const float4*>(s);
          } else if (k + 3 < k_lim) {
            q = make_float4(s[0], s[1], s[2], s[3]);
          } else {
            if (k + 0 < k_lim) q.x = s[0];
            if (k + 1 < k_lim) q.y = s[1];
            if (k + 2 < k_lim) q.z = s[2];
          }
        }
        v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < KR; ++e) {
        const int k = k0 + kb + e;
        // gathered rows index the whole rollout buffer (T * N rows): 64-bit offsets; identity rows are bounded by
        // try_x6's K * ld < 2^31 check, so 32-bit math is exact there
        if constexpr (KGATHER) {
          const int64_t o = krows[k] * ld + roff;
          if (fast) v[e] = P[o];
          else v[e] = (rok && k < k_lim) ? P[o] : 0.f;
        } else if (fast) {
          v[e] = P[k * ldi + roff];
        } else {
          v[e] = (rok && k < k_lim) ? P[k * ldi + roff] : 0.f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(const float (&v)[NV], uint16_t* img) const {
    const int t = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int r = (t >> 2) + 64 * u, j = t & 3;
        uint32_t h0, m0, l0, h1, m1, l1;
        x6_split2(v[4 * u], v[4 * u + 1], h0, m0, l0);
        x6_split2(v[4 * u + 2], v[4 * u + 3], h1, m1, l1);
        const int off = x6_off(r, j >> 1) + 4 * (j & 1);
        *reinterpret_cast<uint2*>(img + off) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(img + PLANE + off) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(img + 2 * PLANE + off) = make_uint2(l0, l1);
      }
    } else if (KR == 8) {
      uint32_t h[4], m[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x6_split2(v[2 * e], v[2 * e + 1], h[e], m[e], l[e]);
      const int off = x6_off(rr, kb >> 3);
      *reinterpret_cast<uint4*>(img + off) = make_uint4(h[0], h[1], h[2], h[3]);
      *reinterpret_cast<uint4*>(img + PLANE + off) = make_uint4(m[0], m[1], m[2], m[3]);
      *reinterpret_cast<uint4*>(img + 2 * PLANE + off) = make_uint4(l[0], l[1], l[2], l[3]);
    } else {
      uint32_t h[2], m[2], l[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) x6_split2(v[2 * e], v[2 * e + 1], h[e], m[e], l[e]);
      const int off = x6_off(rr, kb >> 3) + (kb & 4);
      *reinterpret_cast<uint2*>(img + off) = make_uint2(h[0], h[1]);
      *reinterpret_cast<uint2*>(img + PLANE + off) = make_uint2(m[0], m[1]);
      *reinterpret_cast<uint2*>(img + 2 * PLANE + off) = make_uint2(l[0], l[1]);
    }
  }
  // sum of this thread's staged values (bias-gradient partial of an r-contiguous A)
  __device__ __forceinline__ static float vsum(const float (&v)[NV]) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < NV; ++e) s += v[e];
    return s;
  }
};

// TAG: trace tag only (the weight-gradient shape, tn_shape_tag): each of the update's large weight gradients gets its own
// symbol so a kernel trace / PMC pass keys its launches apart; the code is the same for every value
template <int BM, int BN, int LAYOUT, int EPI, bool FAST, bool BGATHER, int TAG = 0>
__global__ __launch_bounds__(GTHREADS, 3) void gemm_x6_kernel(GemmP p) {  // 3 waves / SIMD: 3 workgroups per CU (LDS 48 KB)
  constexpr bool AKC = (LAYOUT & 1) == 0, BKC = (LAYOUT & 2) == 0;
  constexpr int PA = BM * XBK, PB = BN * XBK, STG = 3 * (PA + PB);
  constexpr int TM = BM / 64, TN = BN / 64;
  __shared__ __attribute__((aligned(16))) uint16_t S[2 * STG];
  const int mt = (p.M + BM - 1) / BM, nt = (p.N + BN - 1) / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, zz = L / (nt * mt);
  const int g = zz / p.splits, sp = zz - g * p.splits;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int kbeg = sp * p.kps, kend = min(p.K, kbeg + p.kps);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  X6Op<BM, AKC> oa;
  X6Op<BN, BKC, BGATHER && !BKC> ob;
  oa.init(p.A + g * p.ga, p.lda, AKC ? p.a_rows : nullptr, nullptr, m0, p.M, p.avec == 4);
  ob.init(p.B + g * p.gb, p.ldb, nullptr, BKC ? nullptr : p.b_rows, n0, p.N, p.bvec == 4);
  // FAST: every tile of the launch is interior and every split's k range a whole number of slices
  constexpr bool fast = FAST;
  const bool do_bsum = EPI == EPI_PARTIAL && p.bias_part != nullptr && tn_ == 0;
  float bsum = 0.f;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  using OA = decltype(oa);
  using OB = decltype(ob);
  // one k-step of the 32x32x16 products on the stage at As: six MFMAs per tile (smallest products first)
  auto compute = [&](const uint16_t* As) {
    const uint16_t* Bs = As + 3 * PA;
    bf16x8_t a[TM][3], b[TN][3];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = *reinterpret_cast<const bf16x8_t*>(As + pl * PA + x6_off(wm + 32 * i + li, h));
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[j][pl] = *reinterpret_cast<const bf16x8_t*>(Bs + pl * PB + x6_off(wn + 32 * j + li, h));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
        acc[i][j] = c;
      }
  };
  if constexpr (LRL_X6_PIPE && FAST) {
  // Software pipeline: slice s + 1 waits split-ready in registers while slice s is multiplied, so its split (VALU)
  // and LDS stores interleave with slice s's MFMAs in one scheduling region; slice s + 2 is in flight meanwhile.
  float va[2][OA::NV], vb[2][OB::NV];
  const int ns = (kend - kbeg + XBK - 1) / XBK;
  if (ns > 0) {
    oa.load(va[0], kbeg, kend, fast);
    ob.load(vb[0], kbeg, kend, fast);
    if (ns > 1) {
      oa.load(va[1], kbeg + XBK, kend, fast);
      ob.load(vb[1], kbeg + XBK, kend, fast);
    }
    if (do_bsum) bsum += OA::vsum(va[0]);
    oa.store(va[0], S);
    ob.store(vb[0], S + 3 * PA);
    if (ns > 2) {
      oa.load(va[0], kbeg + 2 * XBK, kend, fast);
      ob.load(vb[0], kbeg + 2 * XBK, kend, fast);
    }
  }
  __syncthreads();
  // step s: multiply stage s & 1, split + store slice s + 1 (register set (s + 1) & 1) into the other stage, then
  // load slice s + 3 into that register set
  auto step = [&](int s, auto par, auto full) {
    constexpr int P = decltype(par)::value;
    constexpr bool F = decltype(full)::value;  // s + 3 < ns: no guards
    compute(S + P * STG);
    if (F || s + 1 < ns) {
      if (do_bsum) bsum += OA::vsum(va[P ^ 1]);
      oa.store(va[P ^ 1], S + (P ^ 1) * STG);
      ob.store(vb[P ^ 1], S + (P ^ 1) * STG + 3 * PA);
    }
    if (F || s + 3 < ns) {
      oa.load(va[P ^ 1], kbeg + (s + 3) * XBK, kend, fast);
      ob.load(vb[P ^ 1], kbeg + (s + 3) * XBK, kend, fast);
    }
    if constexpr (F) {
      // interleave: the operand reads, then each MFMA followed by split / address VALU, then the stores and loads
      constexpr int NMF = TM * TN * 6;
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * (TM + TN), 0);
#pragma unroll
      for (int q = 0; q < NMF; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, LRL_X6_PIPE_VALU, 0);
      }
    }
    __syncthreads();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  int s = 0;
  for (; s + 4 < ns; s += 2) {
    step(s, I0{}, BT{});
    step(s + 1, I1{}, BT{});
  }
  for (; s < ns; s += 2) {
    step(s, I0{}, BF{});
    if (s + 1 < ns) step(s + 1, I1{}, BF{});
  }
  } else {
  float va[OA::NV], vb[OB::NV];
  if (kbeg < kend) {
    oa.load(va, kbeg, kend, fast);
    ob.load(vb, kbeg, kend, fast);
    if (do_bsum) bsum += OA::vsum(va);
    oa.store(va, S);
    ob.store(vb, S + 3 * PA);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += XBK) {
    const bool more = k0 + XBK < kend;
    if (more) {
      oa.load(va, k0 + XBK, kend, fast);
      ob.load(vb, k0 + XBK, kend, fast);
    }
    compute(S + buf * STG);
    if (more) {
      if (do_bsum) bsum += OA::vsum(va);
      oa.store(va, S + (buf ^ 1) * STG);
      ob.store(vb, S + (buf ^ 1) * STG + 3 * PA);
    }
    __syncthreads();
    buf ^= 1;
  }
  }

  float* __restrict__ C = p.C + g * p.gc;
  if (EPI == EPI_PARTIAL) C += (int64_t)sp * p.part_stride;
  const float* __restrict__ bias = p.bias ? p.bias + g * p.gbias : nullptr;
  // (the backward-data epilogue's layer input is read here, not prefetched: 16 registers per MFMA tile held
  // through the main loop would cost occupancy)
  const float* __restrict__ ax = EPI == EPI_DELU ? p.aux + g * p.gaux : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + 32 * j + li;
    if (!FAST && col >= p.N) continue;
    float bj = 0.f;
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // rows 8q + 4h .. +3 of the MFMA tile: accumulator registers 4q .. 4q+3
        const int row0 = m0 + wm + 32 * i + 8 * q + 4 * h;
        // 32-bit element offsets from per-group base pointers (row * ld < 2^31 for every product here)
        const int ldc = (int)p.ldc, ldx = (int)p.ld_aux;
        float* __restrict__ crow = C + (int64_t)row0 * p.ldc + col;
        float xa[4];
        if constexpr (EPI == EPI_DELU) {
          const float* __restrict__ xrow = ax + (int64_t)row0 * p.ld_aux + col;
#pragma unroll
          for (int r = 0; r < 4; ++r) xa[r] = (FAST || row0 + r < p.M) ? xrow[r * ldx] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (FAST || row0 + r < p.M) {
            float v = acc[i][j][4 * q + r];
            if (EPI == EPI_BIAS) v += bj;
            if (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
            if constexpr (EPI == EPI_DELU) {
              const float x = xa[r];
              v = x > 0.f ? v : v * (x + 1.f);
            }
            crow[r * ldc] = v;
          }
        }
        asm volatile("" ::: "memory");  // (bounds the epilogue's live loads and addresses to one row group)
      }
  }
  if constexpr (EPI == EPI_PARTIAL && !AKC) {
    // bias-gradient partial: the k-runs of one row are spread over GTHREADS / BM threads; add them in thread
    // order through LDS (fixed order: deterministic)
    if (do_bsum) {
      float* red = reinterpret_cast<float*>(S);  // the loop's last barrier has retired every stage read
      red[threadIdx.x] = bsum;
      __syncthreads();
      if (threadIdx.x < BM && m0 + (int)threadIdx.x < p.M) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < GTHREADS / BM; ++q) s += red[q * BM + threadIdx.x];
        p.bias_part[((int64_t)sp * p.groups + g) * p.M + m0 + threadIdx.x] = s;
      }
    }
  }
}

template <int BM, int BN>
static int launch_x6_tile(const GemmP& p, int layout, int epi, int groups, hipStream_t st) {
  dim3 grid(((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN) * groups * p.splits);
  const bool akc = (layout & 1) == 0, bkc = (layout & 2) == 0;
  const bool interior = p.M % BM == 0 && p.N % BN == 0 && p.K % XBK == 0 && p.kps % XBK == 0 &&
                        (!akc || p.avec == 4) && (!bkc || p.bvec == 4);
  const bool bg = p.b_rows != nullptr;
#define LRL_X6G(L, E, G)                                                                                     \
  do {                                                                                                       \
    if (interior) hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, L, E, true, G>), grid, dim3(GTHREADS), 0, st, p); \
    else hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, L, E, false, G>), grid, dim3(GTHREADS), 0, st, p);        \
  } while (0)
#define LRL_X6(L, E) LRL_X6G(L, E, false)
  if (layout == GEMM_NT) {
    if (epi == EPI_STORE) LRL_X6(GEMM_NT, EPI_STORE);
    else if (epi == EPI_BIAS) LRL_X6(GEMM_NT, EPI_BIAS);
    else if (epi == EPI_BIAS_ELU) LRL_X6(GEMM_NT, EPI_BIAS_ELU);
    else return LRL_E_INVALID;
  } else if (layout == GEMM_NN) {
    if (epi == EPI_STORE) LRL_X6(GEMM_NN, EPI_STORE);
    else if (epi == EPI_DELU) LRL_X6(GEMM_NN, EPI_DELU);
    else return LRL_E_INVALID;
  } else if (layout == GEMM_TN && epi == EPI_PARTIAL) {
    const int tag = (BM == 128 && BN == 128 && interior) ? tn_shape_tag(p.M, p.N, groups) : 0;
#define LRL_X6T(G, T) hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, GEMM_TN, EPI_PARTIAL, true, G, T>), grid, dim3(GTHREADS), 0, st, p)
    if (tag == 1) LRL_X6T(false, 1);
    else if (tag == 2) LRL_X6T(false, 2);
    else if (tag == 4) { if (bg) LRL_X6T(true, 4); else LRL_X6T(false, 4); }
    else if (tag == 6) LRL_X6T(false, 6);
    else if (bg) LRL_X6G(GEMM_TN, EPI_PARTIAL, true);
    else LRL_X6G(GEMM_TN, EPI_PARTIAL, false);
#undef LRL_X6T
  } else {
    return LRL_E_INVALID;
  }
#undef LRL_X6
#undef LRL_X6G
  return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
}

// x6 path switch: LRL_GEMM_X6=0 keeps every product on the fp32 MFMA kernels (A/B comparisons)
static bool x6_enabled() {
  static const int on = [] {
    const char* e = getenv("LRL_GEMM_X6");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}

static int try_x6d(const GemmP& p, int layout, int epi, int groups, int bm, int bn, hipStream_t st);

// returns 1 when the product was launched on the x6 kernel (0: not eligible, <0: error)
static int try_x6(const GemmP& p, int layout, int epi, int groups, hipStream_t st) {
  if (!x6_enabled()) return 0;
  // (LRL_X6_MIN: development override of the smallest output side x6 takes — 16 by default)
  static const int min_side = getenv("LRL_X6_MIN") ? atoi(getenv("LRL_X6_MIN")) : 16;
  if (p.N < min_side || (layout == GEMM_TN && p.M < min_side)) return 0;
  // r-contiguous operands (A of TN, B of NN / TN) and the epilogue use 32-bit element offsets from the group base
  // (k * ld + row, row * ldc + col): keep every identity-indexed offset below 2^31 (gathered rows are 64-bit)
  const int64_t lim = int64_t(1) << 31;
  if ((layout & 1) && (int64_t)p.K * p.lda >= lim) return 0;
  if ((layout & 2) && p.b_rows == nullptr && (int64_t)p.K * p.ldb >= lim) return 0;
  if ((int64_t)p.M * p.ldc >= lim || (epi == EPI_DELU && (int64_t)p.M * p.ld_aux >= lim)) return 0;
  int rc;
  if (layout == GEMM_TN) {
    // (both operands r-contiguous: dword loads, any alignment)
    if (epi != EPI_PARTIAL || p.M < 16 || p.N < 16 || p.kps % XBK) return 0;
    const bool m64 = p.M <= 64, n64 = p.N <= 64;
    if (m64 && n64) rc = launch_x6_tile<64, 64>(p, layout, epi, groups, st);
    else if (m64) rc = launch_x6_tile<64, 128>(p, layout, epi, groups, st);
    else if (n64) rc = launch_x6_tile<128, 64>(p, layout, epi, groups, st);
    else rc = launch_x6_tile<128, 128>(p, layout, epi, groups, st);
  } else {
    if (p.splits != 1 || p.N < 16 || p.M < 64 || epi == EPI_PARTIAL) return 0;
    // measured (scripts/gemm_bench.py): one or two 16-k slices do not pay the split / staging set-up, and the
    // thin kernel (B in registers) stays faster for <= 32-wide outputs over k = 512 / 1024
    if (p.K < 32) return 0;
    if (p.N <= 32 && p.K % 128 == 0 && (p.K / 128 == 4 || p.K / 128 == 8) && p.avec == 4 && p.M >= 256) return 0;
    // (LRL_X6_SMALL_WG: development override — below this many 64 x 128 workgroups the product takes 64 x 64 tiles)
    static const int small_wg = getenv("LRL_X6_SMALL_WG") ? atoi(getenv("LRL_X6_SMALL_WG")) : 1024;
    int bn = p.N > 64 ? 128 : 64;
    if (bn == 128 && (int64_t)((p.M + 63) / 64) * ((p.N + 127) / 128) * groups < small_wg) bn = 64;
    // 128-row tiles when they still give two workgroups per CU, 64 otherwise
    const int64_t wg128 = (int64_t)((p.M + 127) / 128) * ((p.N + bn - 1) / bn) * groups;
    const int bm = wg128 >= 512 ? 128 : 64;
    // the same tile on the LDS-DMA kernel where the tiles are interior
    if (int dr = try_x6d(p, layout, epi, groups, bm, bn, st)) return dr;
    if (bm == 128 && bn == 128) rc = launch_x6_tile<128, 128>(p, layout, epi, groups, st);
    else if (bm == 128) rc = launch_x6_tile<128, 64>(p, layout, epi, groups, st);
    else if (bn == 128) rc = launch_x6_tile<64, 128>(p, layout, epi, groups, st);
    else rc = launch_x6_tile<64, 64>(p, layout, epi, groups, st);
  }
  return rc ? rc : 1;
}

// ---------------------------------------------------------------------------------------------------
// x6 with a pre-split B ("x6p", NT / NN products whose B is a weight matrix).  The weights are split into their
// hi / mid / lo bf16 planes once per optimiser step (x6_planes_kernel, op(B) already in [n][k] form — the transpose
// of the backward-data B is taken there), so nothing in the product transposes or splits B.  Both operands then
// stage global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write pass) into a 3-deep ring
// of 16-k stages with counted vmcnt waits and a raw s_barrier, so two stages stay in flight across each barrier;
// only A (fp32 activations) is split, in registers, right after its ds_read: one split per element and reading wave,
// 11 VALU per pair of floats, which the MFMAs of the other workgroup on the SIMD (2 per CU) hide.
//   A image per stage: [BM][16] fp32 (64-B rows), 16-B chunk c of row r in slot c ^ ((r >> 2) & 3); a DMA
//   wave-instruction fills 16 rows (lane l: row l / 4, slot l % 4, source chunk pre-swizzled).
//   B images per stage: 3 planes of [128][16] bf16 (32-B rows), chunk c of row r in slot c ^ ((r >> 3) & 1); a DMA
//   wave-instruction fills 32 rows of one plane.
// Tile BM x 128 (BM = 64 / 128), 4 waves in a 2 x 2 grid, wave tile (BM/2) x 64; the six MFMA products per 32x32x16
// step in the order of gemm_x6_kernel over the same k order, so the result is bit-identical to it.
template <int BM, int EPI, bool GATHER>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_x6p_kernel(GemmP p) {
  constexpr int BN = 128, NST = 3, TM = BM / 64, TN = 2;
  constexpr int AIMG = BM * 64, BIMG = BN * 32, STB = AIMG + 3 * BIMG;  // bytes
  constexpr int NA = BM / 64, NB = 3;  // DMA wave-instructions per wave and stage
  constexpr int NPW = NA + NB;
  static_assert(NPW == 4 || NPW == 5, "vmcnt table");
  __shared__ __attribute__((aligned(16))) uint8_t S[NST * STB];  // the only LDS object (see the glds rules)
  const int mt = p.M / BM, nt = p.N / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, g = L / (nt * mt);
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const float* __restrict__ A = p.A + g * p.ga;
  const uint16_t* __restrict__ Bp = p.bpl + g * p.gbp;
  const float* asrc[NA];
#pragma unroll
  for (int d = 0; d < NA; ++d) {
    const int r = (w * NA + d) * 16 + (lane >> 2), ch = (lane & 3) ^ ((r >> 2) & 3);
    asrc[d] = A + (GATHER ? p.a_rows[m0 + r] : (int64_t)(m0 + r)) * p.lda + 4 * ch;
  }
  const uint16_t* bsrc[NB];
#pragma unroll
  for (int d = 0; d < NB; ++d) {
    const int j = w * NB + d, r = (j & 3) * 32 + (lane >> 1), ch = (lane & 1) ^ ((r >> 3) & 1);
    bsrc[d] = Bp + (j >> 2) * p.bpl_ps + (int64_t)(n0 + r) * p.bpl_ld + 8 * ch;
  }
  const uint32_t s_lds = (uint32_t)(uintptr_t)(lds_ptr_t)S;
  // the DMA is issued from inline asm so the compiler does not track it; completion is ordered by the counted waits
  auto dma = [&](const void* src, uint32_t lds_off) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_off)
                 : "memory");
  };
  auto issue = [&](int st, int k0) {
    const uint32_t base = s_lds + (uint32_t)(st * STB);
#pragma unroll
    for (int d = 0; d < NA; ++d) dma(asrc[d] + k0, __builtin_amdgcn_readfirstlane(base + (w * NA + d) * 1024));
#pragma unroll
    for (int d = 0; d < NB; ++d) dma(bsrc[d] + k0, __builtin_amdgcn_readfirstlane(base + AIMG + (w * NB + d) * 1024));
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ns = p.K / 16;
  issue(0, 0);
  if (ns > 1) issue(1, 16);
  for (int s = 0; s < ns; ++s) {
    // this wave's DMAs of stage s have landed (stage s + 1's may stay in flight) ...
    if (s + 1 < ns) {
      if constexpr (NPW == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // ... and every wave's; every wave is also done reading stage s - 1, whose buffer stage s + 2 refills
    __builtin_amdgcn_s_barrier();
    if (s + 2 < ns) issue((s + 2) % NST, (s + 2) * 16);
    const uint8_t* As = S + (s % NST) * STB;
    const uint8_t* Bs = As + AIMG;
    bf16x8_t a[TM][3], b[TN][3];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = wn + 32 * j + li, off = r * 32 + 16 * (h ^ ((r >> 3) & 1));
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) b[j][pl] = *reinterpret_cast<const bf16x8_t*>(Bs + pl * BIMG + off);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm + 32 * i + li, sw = (r >> 2) & 3;
      const float4 x0 = *reinterpret_cast<const float4*>(As + r * 64 + 16 * ((2 * h) ^ sw));
      const float4 x1 = *reinterpret_cast<const float4*>(As + r * 64 + 16 * ((2 * h + 1) ^ sw));
      uint32_t hh[4], mm[4], ll[4];
      x6_split2(x0.x, x0.y, hh[0], mm[0], ll[0]);
      x6_split2(x0.z, x0.w, hh[1], mm[1], ll[1]);
      x6_split2(x1.x, x1.y, hh[2], mm[2], ll[2]);
      x6_split2(x1.z, x1.w, hh[3], mm[3], ll[3]);
      uint4 vh = make_uint4(hh[0], hh[1], hh[2], hh[3]), vm = make_uint4(mm[0], mm[1], mm[2], mm[3]),
            vl = make_uint4(ll[0], ll[1], ll[2], ll[3]);
      a[i][0] = *reinterpret_cast<bf16x8_t*>(&vh);
      a[i][1] = *reinterpret_cast<bf16x8_t*>(&vm);
      a[i][2] = *reinterpret_cast<bf16x8_t*>(&vl);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
        acc[i][j] = c;
      }
  }

  float* __restrict__ C = p.C + g * p.gc;
  const float* __restrict__ bias = p.bias ? p.bias + g * p.gbias : nullptr;
  const float* __restrict__ ax = EPI == EPI_DELU ? p.aux + g * p.gaux : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + 32 * j + li;
    float bj = 0.f;
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // rows 8q + 4h .. +3 of the MFMA tile: accumulator registers 4q .. 4q+3
        const int row0 = m0 + wm + 32 * i + 8 * q + 4 * h;
        float* __restrict__ crow = C + (int64_t)row0 * p.ldc + col;
        float xa[4];
        if constexpr (EPI == EPI_DELU) {
          const float* __restrict__ xrow = ax + (int64_t)row0 * p.ld_aux + col;
#pragma unroll
          for (int r = 0; r < 4; ++r) xa[r] = xrow[r * p.ld_aux];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][4 * q + r];
          if (EPI == EPI_BIAS) v += bj;
          if (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
          if constexpr (EPI == EPI_DELU) {
            const float x = xa[r];
            v = x > 0.f ? v : v * (x + 1.f);
          }
          crow[r * p.ldc] = v;
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------------
// x6 weight gradient with LDS-DMA staging ("x6t", TN, split-k partials): both operands are [k][r] activations
// (r = the output row / column), so they land as [16 k][128 r] fp32 images by LDS-DMA (a wave-instruction fills two
// k-rows; 16-B chunk c of k-row k sits in slot c ^ (8 * ((k >> 3) & 1)), so the two lane halves of a read, k and
// k + 8, use opposite bank halves), in a 3-deep ring with counted vmcnt and a raw barrier.  Each lane gathers its
// 8 k-values per MFMA operand with ds_read_b32 (immediate offsets) and splits them in registers.  128 x 128 tiles,
// 4 waves of 2 x 2 MFMA tiles, the six products in gemm_x6_kernel's order over the same k order, and the bias
// gradient partial summed in its (row, k-half) order: bit-identical to it.
constexpr int X6T_MAX_GATHER_KPS = 1024;  // gathered-B splits of at most this many rows (the row list in LDS)
template <int BN, int TAG, bool BGATHER>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_x6t_kernel(GemmP p) {
  constexpr int BM = 128, NST = 3, TM = 2, TN = BN / 64;
  constexpr int IMG = 16 * 128 * 4, STB = IMG + 16 * BN * 4;  // bytes: A image [16][128], then B image [16][BN]
  constexpr int NAP = IMG / 1024, NBP = BN / 16;              // DMA pieces (1 KiB wave-instructions) per stage
  constexpr int NPW = (NAP + NBP) / 4;                        // per wave: 4 (BN 128) or 3 (BN 64)
  constexpr int KPP = 256 / BN;                               // k-rows per B piece
  constexpr int XROWS = BGATHER ? X6T_MAX_GATHER_KPS : 0;  // gathered B: the split's row list (int32) after the ring
  __shared__ __attribute__((aligned(16))) uint8_t S[NST * STB + 4 * XROWS];
  const int mt = p.M / BM, nt = (p.N + BN - 1) / BN;  // (ragged n: see try_x6t)
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, zz = L / (nt * mt);
  const int g = zz / p.splits, sp = zz - g * p.splits;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int kbeg = sp * p.kps, kend = min(p.K, kbeg + p.kps);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ Bm = p.B + g * p.gb;
  // this wave's DMA pieces j = NPW w + d: A's first (two k-rows each: lane / 32, slot lane % 32), then B's (KPP k-rows
  // each); the source chunk is pre-swizzled, the LDS destination of piece j is j KiB into the stage
  const float* src[NPW];
  int64_t kstep[NPW];
  int bkr[NPW];
  int* xrows = reinterpret_cast<int*>(S + NST * STB);
  if constexpr (BGATHER) {
    // the split's B row list into LDS before the ring starts (no DMA in flight: a plain barrier is safe)
    for (int t = threadIdx.x; t < kend - kbeg; t += GTHREADS) xrows[t] = (int)p.b_rows[kbeg + t];
    __syncthreads();
  }
#pragma unroll
  for (int d = 0; d < NPW; ++d) {
    const int j = NPW * w + d;
    if (j < NAP) {
      const int kr = 2 * j + (lane >> 5), ch = (lane & 31) ^ (8 * ((kr >> 3) & 1));
      src[d] = A + (int64_t)(kbeg + kr) * p.lda + m0 + 4 * ch;
      kstep[d] = (int64_t)16 * p.lda;
      bkr[d] = -1;
    } else {
      const int kr = KPP * (j - NAP) + lane / (BN / 4), ch = (lane % (BN / 4)) ^ (8 * ((kr >> 3) & 1));
      src[d] = BGATHER ? Bm + n0 + 4 * ch : Bm + (int64_t)(kbeg + kr) * p.ldb + n0 + 4 * ch;
      kstep[d] = (int64_t)16 * p.ldb;
      bkr[d] = kr;
    }
  }
  const uint32_t s_lds = (uint32_t)(uintptr_t)(lds_ptr_t)S;
  auto dma = [&](const void* src, uint32_t lds_off) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_off)
                 : "memory");
  };
  auto issue = [&](int st, int s) {
    const uint32_t base = s_lds + (uint32_t)(st * STB);
#pragma unroll
    for (int d = 0; d < NPW; ++d) {
      const float* sr = (BGATHER && bkr[d] >= 0) ? src[d] + (int64_t)xrows[16 * s + bkr[d]] * p.ldb : src[d] + s * kstep[d];
      dma(sr, __builtin_amdgcn_readfirstlane(base + (NPW * w + d) * 1024));
    }
  };
  const bool do_bsum = p.bias_part != nullptr && tn_ == 0 && wn == 0;
  float bsum[TM] = {0.f, 0.f};
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ns = (kend - kbeg) / 16;
  if (ns > 0) issue(0, 0);
  if (ns > 1) issue(1, 1);
  // lane's element offsets (floats) into an image: k-row 8h + t at + 128 t, row / column r ^ 32 h
  const int sw = 32 * h;
  static_assert(NPW == 3 || NPW == 4, "vmcnt below");
  for (int s = 0; s < ns; ++s) {
    if (s + 1 < ns) {
      if constexpr (NPW == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + 2 < ns) issue((s + 2) % NST, s + 2);
    const float* As = reinterpret_cast<const float*>(S + (s % NST) * STB);
    const float* Bs = As + IMG / 4;
    bf16x8_t a[TM][3], b[TN][3];
    auto gather_split = [&](const float* img, int pitch, int r, bf16x8_t (&o)[3], float* vs) {
      const float* p0 = img + 8 * h * pitch + (r ^ sw);
      float v[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = p0[pitch * t];
      if (vs) {
        float s8 = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) s8 += v[t];
        *vs += s8;
      }
      uint32_t hh[4], mm[4], ll[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x6_split2(v[2 * e], v[2 * e + 1], hh[e], mm[e], ll[e]);
      uint4 vh = make_uint4(hh[0], hh[1], hh[2], hh[3]), vm = make_uint4(mm[0], mm[1], mm[2], mm[3]),
            vl = make_uint4(ll[0], ll[1], ll[2], ll[3]);
      o[0] = *reinterpret_cast<bf16x8_t*>(&vh);
      o[1] = *reinterpret_cast<bf16x8_t*>(&vm);
      o[2] = *reinterpret_cast<bf16x8_t*>(&vl);
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) gather_split(As, 128, wm + 32 * i + li, a[i], do_bsum ? &bsum[i] : nullptr);
#pragma unroll
    for (int j = 0; j < TN; ++j) gather_split(Bs, BN, wn + 32 * j + li, b[j], nullptr);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
        acc[i][j] = c;
      }
  }

  float* __restrict__ C = p.C + g * p.gc + (int64_t)sp * p.part_stride;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + 32 * j + li;
    if (col >= p.N) continue;  // (ragged n: the DMA read the row pitch's padding columns, which no output keeps)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row0 = m0 + wm + 32 * i + 8 * q + 4 * h;
        float* __restrict__ crow = C + (int64_t)row0 * p.ldc + col;
#pragma unroll
        for (int r = 0; r < 4; ++r) crow[r * p.ldc] = acc[i][j][4 * q + r];
      }
  }
  if (p.bias_part != nullptr && tn_ == 0) {
    // bias-gradient partial: row r's two k-halves added in gemm_x6_kernel's order (k-half 0 first, from 0)
    __syncthreads();  // every stage read has retired (no DMA is in flight after the last vmcnt(0))
    float* red = reinterpret_cast<float*>(S);
    if (wn == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i) red[h * BM + wm + 32 * i + li] = bsum[i];
    }
    __syncthreads();
    if (threadIdx.x < BM) {
      float s = 0.f;
      s += red[threadIdx.x];
      s += red[BM + threadIdx.x];
      p.bias_part[((int64_t)sp * p.groups + g) * p.M + m0 + threadIdx.x] = s;
    }
  }
}

// run-time path mask (lrl_debug_gemm_paths: tests compare the paths in one process): bit 0 off = no x6p, bit 1 = no x6t,
// bit 2 = no x6d, bit 3 = x6d on (NT and NN) unless bit 2
static int g_path_off = 0;

// ---------------------------------------------------------------------------------------------------
// x6 forward / backward-data with LDS-DMA staging ("x6d", NT / NN, fp32 operands): gemm_x6t_kernel's structure for
// the batch-major products.  Both operands land fp32 by LDS-DMA in a 3-deep ring of 16-k stages (counted vmcnt, raw
// barrier, two stages in flight across it); each lane reads its 8 k-values per MFMA operand and splits them in
// registers.  k-contiguous operands (A; B of NT): [R][16] images (64-B rows, 16-B chunk c of row r in slot
// c ^ ((r >> 2) & 3)), read with two ds_read_b128; the n-contiguous B of NN: [16][BN] (chunk c of k-row k in slot
// c ^ (8 * ((k >> 3) & 1))), read with ds_read_b32.  Tile shapes as gemm_x6_kernel picks them; the six products in
// its order over the same k order: bit-identical to it.
template <int BM, int BN, int LAYOUT, int EPI, bool GATHER>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_x6d_kernel(GemmP p) {
  constexpr bool BNC = LAYOUT == GEMM_NN;
  constexpr int NST = 3, TM = BM / 64, TN = BN / 64;
  constexpr int AIMG = BM * 64, BIMG = BN * 64, STB = AIMG + BIMG;  // bytes
  constexpr int NAI = BM / 16, NBI = BN / 16, NPW = (NAI + NBI) / 4;  // DMA wave-instructions (per stage; per wave)
  static_assert((NAI + NBI) % 4 == 0 && NPW >= 2 && NPW <= 4, "DMA split");
  __shared__ __attribute__((aligned(16))) uint8_t S[NST * STB];
  const int mt = p.M / BM, nt = p.N / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn_ = L % nt, tm_ = (L / nt) % mt, g = L / (nt * mt);
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const float* __restrict__ A = p.A + g * p.ga;
  const float* __restrict__ Bm = p.B + g * p.gb;
  // this wave's DMA pieces j = NPW w + d: A image pieces first (16 rows each), then B's (16 rows, or 1024 / (4 BN)
  // k-rows of the NN image); the LDS destination of piece j is j KiB into the stage
  const float* src[NPW];
  int64_t kstep[NPW];
#pragma unroll
  for (int d = 0; d < NPW; ++d) {
    const int j = NPW * w + d;
    if (j < NAI) {
      const int r = 16 * j + (lane >> 2), ch = (lane & 3) ^ ((r >> 2) & 3);
      src[d] = A + (GATHER ? p.a_rows[m0 + r] : (int64_t)(m0 + r)) * p.lda + 4 * ch;
      kstep[d] = 16;
    } else if (!BNC) {
      const int r = 16 * (j - NAI) + (lane >> 2), ch = (lane & 3) ^ ((r >> 2) & 3);
      src[d] = Bm + (int64_t)(n0 + r) * p.ldb + 4 * ch;
      kstep[d] = 16;
    } else {
      constexpr int KPP = 256 / BN;  // k-rows per piece
      const int kr = KPP * (j - NAI) + lane / (BN / 4), c = lane % (BN / 4), ch = c ^ (8 * ((kr >> 3) & 1));
      src[d] = Bm + (int64_t)kr * p.ldb + n0 + 4 * ch;
      kstep[d] = 16 * p.ldb;
    }
  }
  const uint32_t s_lds = (uint32_t)(uintptr_t)(lds_ptr_t)S;
  auto dma = [&](const void* s, uint32_t lds_off) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(s), "s"(lds_off)
                 : "memory");
  };
  auto issue = [&](int st, int s) {
    const uint32_t base = s_lds + (uint32_t)(st * STB);
#pragma unroll
    for (int d = 0; d < NPW; ++d)
      dma(src[d] + s * kstep[d], __builtin_amdgcn_readfirstlane(base + (NPW * w + d) * 1024));
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto split8 = [&](const float (&v)[8], bf16x8_t (&o)[3]) {
    uint32_t hh[4], mm[4], ll[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x6_split2(v[2 * e], v[2 * e + 1], hh[e], mm[e], ll[e]);
    uint4 vh = make_uint4(hh[0], hh[1], hh[2], hh[3]), vm = make_uint4(mm[0], mm[1], mm[2], mm[3]),
          vl = make_uint4(ll[0], ll[1], ll[2], ll[3]);
    o[0] = *reinterpret_cast<bf16x8_t*>(&vh);
    o[1] = *reinterpret_cast<bf16x8_t*>(&vm);
    o[2] = *reinterpret_cast<bf16x8_t*>(&vl);
  };
  // k-contiguous image: row r's k-values 8h .. 8h+7
  auto read_kc = [&](const uint8_t* img, int r, float (&v)[8]) {
    const int sw = (r >> 2) & 3;
    const float4 x0 = *reinterpret_cast<const float4*>(img + r * 64 + 16 * ((2 * h) ^ sw));
    const float4 x1 = *reinterpret_cast<const float4*>(img + r * 64 + 16 * ((2 * h + 1) ^ sw));
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
  };

  const int ns = p.K / 16;
  issue(0, 0);
  if (ns > 1) issue(1, 1);
  for (int s = 0; s < ns; ++s) {
    if (s + 1 < ns) {
      if constexpr (NPW == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (NPW == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + 2 < ns) issue((s + 2) % NST, s + 2);
    const uint8_t* As = S + (s % NST) * STB;
    const uint8_t* Bs = As + AIMG;
    bf16x8_t a[TM][3], b[TN][3];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v[8];
      read_kc(As, wm + 32 * i + li, v);
      split8(v, a[i]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float v[8];
      if constexpr (!BNC) {
        read_kc(Bs, wn + 32 * j + li, v);
      } else {
        const float* img = reinterpret_cast<const float*>(Bs) + 8 * h * BN + ((wn + 32 * j + li) ^ (32 * h));
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = img[BN * t];
      }
      split8(v, b[j]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
        acc[i][j] = c;
      }
  }

  float* __restrict__ C = p.C + g * p.gc;
  const float* __restrict__ bias = p.bias ? p.bias + g * p.gbias : nullptr;
  const float* __restrict__ ax = EPI == EPI_DELU ? p.aux + g * p.gaux : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn + 32 * j + li;
    float bj = 0.f;
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) bj = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row0 = m0 + wm + 32 * i + 8 * q + 4 * h;
        float* __restrict__ crow = C + (int64_t)row0 * p.ldc + col;
        float xa[4];
        if constexpr (EPI == EPI_DELU) {
          const float* __restrict__ xrow = ax + (int64_t)row0 * p.ld_aux + col;
#pragma unroll
          for (int r = 0; r < 4; ++r) xa[r] = xrow[r * p.ld_aux];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][4 * q + r];
          if (EPI == EPI_BIAS) v += bj;
          if (EPI == EPI_BIAS_ELU) v = elu_f(v + bj);
          if constexpr (EPI == EPI_DELU) {
            const float x = xa[r];
            v = x > 0.f ? v : v * (x + 1.f);
          }
          crow[r * p.ldc] = v;
        }
      }
  }
}

template <int BM, int BN, int LAYOUT>
static void launch_x6d_l(const GemmP& p, int epi, int groups, hipStream_t st) {
  dim3 grid((unsigned)((p.M / BM) * (p.N / BN) * groups));
  const bool gat = p.a_rows != nullptr;
#define LRL_X6D(E)                                                                                             \
  do {                                                                                                         \
    if (gat) hipLaunchKernelGGL((gemm_x6d_kernel<BM, BN, LAYOUT, E, true>), grid, dim3(GTHREADS), 0, st, p);   \
    else hipLaunchKernelGGL((gemm_x6d_kernel<BM, BN, LAYOUT, E, false>), grid, dim3(GTHREADS), 0, st, p);      \
  } while (0)
  if (LAYOUT == GEMM_NT) {
    if (epi == EPI_STORE) LRL_X6D(EPI_STORE);
    else if (epi == EPI_BIAS) LRL_X6D(EPI_BIAS);
    else LRL_X6D(EPI_BIAS_ELU);
  } else {
    if (epi == EPI_STORE) LRL_X6D(EPI_STORE);
    else LRL_X6D(EPI_DELU);
  }
#undef LRL_X6D
}

// x6d path switch, off by default: measured 1.00-1.05x gemm_x6_kernel on the backward-data products in isolation but
// slower inside the update (79 against 68 us for the 2-group dH1, profiles/r4o_kernel_stats.csv), and 0.79-0.97x on
// the forward ones, whose float4-staged operands gemm_x6_kernel splits once per workgroup instead of once per reading
// wave (profiles/r4n_x6d_vs_x6.jsonl).  LRL_GEMM_X6D=1: the backward-data products, =2: the forward too
static int x6d_mode() {
  static const int m = [] {
    const char* e = getenv("LRL_GEMM_X6D");
    return e ? atoi(e) : 0;
  }();
  const int off = __atomic_load_n(&g_path_off, __ATOMIC_RELAXED);
  return (off & 4) ? 0 : (off & 8) ? 2 : m;
}
static bool x6d_enabled() { return x6d_mode() != 0; }

// returns 1 when launched on the x6d kernel (0: not eligible, <0: error); bm / bn: the tile gemm_x6_kernel would take
static int try_x6d(const GemmP& p, int layout, int epi, int groups, int bm, int bn, hipStream_t st) {
  if (!x6d_enabled() || (layout != GEMM_NT && layout != GEMM_NN) || p.splits != 1) return 0;
  if (layout == GEMM_NT && x6d_mode() != 2) return 0;
  if (layout == GEMM_NT && epi != EPI_STORE && epi != EPI_BIAS && epi != EPI_BIAS_ELU) return 0;
  if (layout == GEMM_NN && epi != EPI_STORE && epi != EPI_DELU) return 0;
  if (p.M % bm || p.N % bn || p.K % 16 || p.K < 32 || p.avec != 4 || p.bvec != 4) return 0;
  if (layout == GEMM_NN && p.b_rows) return 0;
  const int key = (bm == 128 ? 2 : 0) | (bn == 128 ? 1 : 0) | (layout == GEMM_NN ? 4 : 0);
  switch (key) {
    case 0: launch_x6d_l<64, 64, GEMM_NT>(p, epi, groups, st); break;
    case 1: launch_x6d_l<64, 128, GEMM_NT>(p, epi, groups, st); break;
    case 2: launch_x6d_l<128, 64, GEMM_NT>(p, epi, groups, st); break;
    case 3: launch_x6d_l<128, 128, GEMM_NT>(p, epi, groups, st); break;
    case 4: launch_x6d_l<64, 64, GEMM_NN>(p, epi, groups, st); break;
    case 5: launch_x6d_l<64, 128, GEMM_NN>(p, epi, groups, st); break;
    case 6: launch_x6d_l<128, 64, GEMM_NN>(p, epi, groups, st); break;
    default: launch_x6d_l<128, 128, GEMM_NN>(p, epi, groups, st); break;
  }
  return hipGetLastError() == hipSuccess ? 1 : LRL_E_HIP;
}
// x6t path switch: LRL_GEMM_X6T=0 keeps the weight gradients on gemm_x6_kernel
static bool x6t_enabled() {
  static const int on = [] {
    const char* e = getenv("LRL_GEMM_X6T");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0 && !(__atomic_load_n(&g_path_off, __ATOMIC_RELAXED) & 2);
}

// returns 1 when launched on the x6t kernel (0: not eligible, <0: error).  n may be ragged when B's row pitch covers
// the last tile (the DMA reads whole 128-wide tiles); a gathered B keeps its split's row list in LDS
static int try_x6t(const GemmP& p, int layout, int epi, int groups, hipStream_t st) {
  if (!x6t_enabled() || layout != GEMM_TN || epi != EPI_PARTIAL) return 0;
  const int bn = p.N <= 64 ? 64 : 128, nt = (p.N + bn - 1) / bn;
  if (p.M % 128 || p.K % 16 || p.kps % 16 || p.kps < 16 || p.avec != 4 || p.bvec != 4) return 0;
  if ((int64_t)nt * bn > p.ldb) return 0;
  if (p.b_rows && p.kps > X6T_MAX_GATHER_KPS) return 0;
  if ((int64_t)(p.splits - 1) * p.kps >= p.K) return 0;  // (every split has a non-empty range)
  dim3 grid((unsigned)((p.M / 128) * nt * groups * p.splits));  // (stores stop at p.N)
  if (bn == 64) {
    if (p.b_rows) hipLaunchKernelGGL((gemm_x6t_kernel<64, 5, true>), grid, dim3(GTHREADS), 0, st, p);
    else hipLaunchKernelGGL((gemm_x6t_kernel<64, 3, false>), grid, dim3(GTHREADS), 0, st, p);
    return hipGetLastError() == hipSuccess ? 1 : LRL_E_HIP;
  }
  if (p.b_rows) {
    hipLaunchKernelGGL((gemm_x6t_kernel<128, 4, true>), grid, dim3(GTHREADS), 0, st, p);
    return hipGetLastError() == hipSuccess ? 1 : LRL_E_HIP;
  }
  switch (tn_shape_tag(p.M, p.N, groups)) {
    case 1: hipLaunchKernelGGL((gemm_x6t_kernel<128, 1, false>), grid, dim3(GTHREADS), 0, st, p); break;
    case 2: hipLaunchKernelGGL((gemm_x6t_kernel<128, 2, false>), grid, dim3(GTHREADS), 0, st, p); break;
    case 6: hipLaunchKernelGGL((gemm_x6t_kernel<128, 6, false>), grid, dim3(GTHREADS), 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_x6t_kernel<128, 0, false>), grid, dim3(GTHREADS), 0, st, p); break;
  }
  return hipGetLastError() == hipSuccess ? 1 : LRL_E_HIP;
}

// x6p path switch for the update: off unless LRL_GEMM_X6P=1 — measured slower than gemm_x6_kernel on every update
// shape (the 6-byte planes of B cost more DMA issue and LDS traffic than the staging split saves, and A
// is split by both waves that read it); products whose caller hands over planes (lrl_gemm_f32 layout | 0x100) run it
static bool x6p_enabled() {
  static const int on = [] {
    const char* e = getenv("LRL_GEMM_X6P");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return on != 0 && !(__atomic_load_n(&g_path_off, __ATOMIC_RELAXED) & 1);
}

bool gemm_x6p_enabled() { return x6p_enabled(); }

// returns 1 when launched on the x6p kernel (0: not eligible, <0: error)
static int try_x6p(const GemmP& p, int layout, int epi, int groups, hipStream_t st) {
  if (!p.bpl || (__atomic_load_n(&g_path_off, __ATOMIC_RELAXED) & 1) || (layout != GEMM_NT && layout != GEMM_NN) ||
      p.splits != 1)
    return 0;
  if (epi != EPI_STORE && epi != EPI_BIAS && epi != EPI_BIAS_ELU && epi != EPI_DELU) return 0;
  if (p.M % 64 || p.N % 128 || p.K % 16 || p.K < 32 || p.avec != 4 || p.bpl_ld != p.K) return 0;
  if ((reinterpret_cast<uintptr_t>(p.bpl) & 15) || p.gbp % 8 || p.bpl_ps % 8) return 0;
  // 128-row tiles when they give at least three per CU pair of workgroup slots, 64 otherwise
  const int64_t t128 = (int64_t)(p.M / 128) * (p.N / 128) * groups;
  const bool big = p.M % 128 == 0 && t128 >= 768;
  const bool gat = p.a_rows != nullptr;
  dim3 grid((unsigned)((p.M / (big ? 128 : 64)) * (p.N / 128) * groups));
#define LRL_X6P(BMV, E)                                                                                         \
  do {                                                                                                          \
    if (gat) hipLaunchKernelGGL((gemm_x6p_kernel<BMV, E, true>), grid, dim3(GTHREADS), 0, st, p);              \
    else hipLaunchKernelGGL((gemm_x6p_kernel<BMV, E, false>), grid, dim3(GTHREADS), 0, st, p);                 \
  } while (0)
#define LRL_X6P_E(E)      \
  do {                    \
    if (big) LRL_X6P(128, E); \
    else LRL_X6P(64, E);  \
  } while (0)
  switch (epi) {
    case EPI_STORE: LRL_X6P_E(EPI_STORE); break;
    case EPI_BIAS: LRL_X6P_E(EPI_BIAS); break;
    case EPI_BIAS_ELU: LRL_X6P_E(EPI_BIAS_ELU); break;
    default: LRL_X6P_E(EPI_DELU); break;
  }
#undef LRL_X6P_E
#undef LRL_X6P
  return hipGetLastError() == hipSuccess ? 1 : LRL_E_HIP;
}

// ---- weight planes: op(B) of each job split into hi / mid / lo bf16 planes, [3][groups][n][kp] ----
struct PlaneJobs {
  PlaneJob j[MAX_PLANE_JOBS];
  int64_t start[MAX_PLANE_JOBS + 1];  // first element (of one plane) of each job
  int n;
};

__global__ __launch_bounds__(256) void x6_planes_kernel(PlaneJobs J) {
  const int64_t total = J.start[J.n];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    int q = 0;
    while (q + 1 < J.n && e >= J.start[q + 1]) ++q;
    const PlaneJob& jb = J.j[q];
    const int kp = plane_kp(jb), nn = plane_n(jb), kk = jb.trans ? jb.rows : jb.cols;
    const int64_t t = e - J.start[q];
    const int k = (int)(t % kp);
    const int64_t rn = t / kp;
    const int n = (int)(rn % nn), g = (int)(rn / nn);
    float x = 0.f;
    if (k < kk) x = jb.trans ? jb.W[g * jb.gsrc + (int64_t)k * jb.ldw + n] : jb.W[g * jb.gsrc + (int64_t)n * jb.ldw + k];
    // the truncation split of x6_split2, one element
    uint32_t u = __float_as_uint(x);
    const uint16_t hi = (uint16_t)(u >> 16);
    float r = x - __uint_as_float(u & 0xffff0000u);
    u = __float_as_uint(r);
    const uint16_t mid = (uint16_t)(u >> 16);
    r = r - __uint_as_float(u & 0xffff0000u);
    const uint16_t lo = (uint16_t)(__float_as_uint(r) >> 16);
    const int64_t ps = (int64_t)jb.groups * nn * kp;
    jb.dst[t] = hi;
    jb.dst[ps + t] = mid;
    jb.dst[2 * ps + t] = lo;
  }
}

int x6_planes_launch(const PlaneJob* jobs, int n, void* stream) {
  if (n <= 0 || n > MAX_PLANE_JOBS) return LRL_E_INVALID;
  PlaneJobs J{};
  J.n = n;
  J.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    J.j[i] = jobs[i];
    if (!jobs[i].W || !jobs[i].dst || jobs[i].rows <= 0 || jobs[i].cols <= 0 || jobs[i].groups <= 0) return LRL_E_INVALID;
    J.start[i + 1] = J.start[i] + plane_elems(jobs[i]) / 3;
  }
  const int blocks = (int)std::min<int64_t>((J.start[n] + 255) / 256, 2048);
  hipLaunchKernelGGL(x6_planes_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), J);
  return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
}

template <int BM, int BN>
static int launch_bm(const GemmP& p, int layout, int epi, dim3 grid, hipStream_t st) {
#define LRL_GEMM_LAUNCH(L, E) hipLaunchKernelGGL((gemm_kernel<BM, BN, L, E>), grid, dim3(GTHREADS), 0, st, p)
  switch (layout) {
    case GEMM_NT:
      switch (epi) {
        case EPI_STORE: LRL_GEMM_LAUNCH(GEMM_NT, EPI_STORE); return 0;
        case EPI_BIAS: LRL_GEMM_LAUNCH(GEMM_NT, EPI_BIAS); return 0;
        case EPI_BIAS_ELU: LRL_GEMM_LAUNCH(GEMM_NT, EPI_BIAS_ELU); return 0;
      }
      break;
    case GEMM_NN:
      switch (epi) {
        case EPI_STORE: LRL_GEMM_LAUNCH(GEMM_NN, EPI_STORE); return 0;
        case EPI_DELU: LRL_GEMM_LAUNCH(GEMM_NN, EPI_DELU); return 0;
        case EPI_PARTIAL: LRL_GEMM_LAUNCH(GEMM_NN, EPI_PARTIAL); return 0;
      }
      break;
    case GEMM_TN:
      if (epi == EPI_PARTIAL) {
        LRL_GEMM_LAUNCH(GEMM_TN, EPI_PARTIAL);
        return 0;
      }
      break;
  }
#undef LRL_GEMM_LAUNCH
  return LRL_E_INVALID;
}

// widest staging access allowed by the pitch / base / group offset alignment of an operand
static int vec_width(const float* ptr, int64_t ld, int64_t goff) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  if ((a & 15) == 0 && ld % 4 == 0 && goff % 4 == 0) return 4;
  if ((a & 7) == 0 && ld % 2 == 0 && goff % 2 == 0) return 2;
  return 1;
}

// tile shape: 128 where the dimension is long, narrower for the thin layers; at least 4 32x32 tiles
// Measured on MI355X (scripts/gemm_bench.py): 64x64 tiles (4 workgroups/CU, one 32x32 MFMA tile per
// wave) beat 128x128 for the batch-major forward / backward-data products; the split-k weight
// gradients prefer 128x128.
#ifndef LRL_GEMM_BM128
#define LRL_GEMM_BM128 0
#endif
static void pick_tile(int M, int N, bool wgrad, int& bm, int& bn) {
  const int mx = wgrad ? 128 : 64;
  bm = M > 64 && (mx > 64 || LRL_GEMM_BM128) ? 128 : (M > 32 ? 64 : 32);
  bn = N > 64 && mx > 64 ? 128 : (N > 32 ? 64 : 32);
  if (bm == 32 && bn < 128) bn = 128;
  if (bn == 32 && bm < 128) bm = 128;
}

int gemm_pick_splits(int M, int N, int K, int groups) {
  int bm, bn;
  pick_tile(M, N, true, bm, bn);
  const int tiles = groups * ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int splits = 1;
  // aim for >= 1024 workgroups (a split-k workgroup's life is short and latency-bound), keep >= 128 rows
  // per split and <= 256 splits
  // per split; the partial slices (written and re-read once) stay under 12M floats
  const int64_t out = (int64_t)groups * M * N;
  // (LRL_SPLIT_WG / LRL_SPLIT_MAXF: development overrides of the workgroup target and the partial-size cap)
  static const int wg_target = getenv("LRL_SPLIT_WG") ? atoi(getenv("LRL_SPLIT_WG")) : 512;
  static const int64_t max_f = getenv("LRL_SPLIT_MAXF") ? atoll(getenv("LRL_SPLIT_MAXF")) : (12ll << 20);
  // small outputs (<= 64K elements: the encoder / adaptation layers' weight gradients) may split down to
  // LRL_SPLIT_SMALL_ROWS rows per split: their partials are small and their few tiles need the parallelism
  static const int small_rows = getenv("LRL_SPLIT_SMALL_ROWS") ? atoi(getenv("LRL_SPLIT_SMALL_ROWS")) : 128;
  const int min_rows = out <= 65536 ? small_rows : 128;
  while (tiles * splits < wg_target && splits < 256 && (K / (splits * 2)) >= min_rows && out * splits * 2 <= max_f)
    splits *= 2;
  return splits;
}

static thread_local int g_last_path = 0;
int gemm_last_path() { return g_last_path; }

int gemm_launch(const GemmP& p0, int layout, int epi, int groups, void* stream) {
  GemmP p = p0;
  if (p.M <= 0 || p.N <= 0 || p.K < 0 || groups <= 0) return LRL_E_INVALID;
  if (p.splits <= 0) p.splits = 1;
  if (p.kps <= 0) p.kps = (p.K + p.splits - 1) / p.splits;
  p.kps = (p.kps + GBK - 1) / GBK * GBK;
  p.avec = vec_width(p.A, p.lda, p.ga);
  p.bvec = vec_width(p.B, p.ldb, p.gb);
  int bm, bn;
  pick_tile(p.M, p.N, layout == GEMM_TN, bm, bn);
  p.groups = groups;
  dim3 grid(((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn) * groups * p.splits);
  hipStream_t st = static_cast<hipStream_t>(stream);
  static const bool trace = getenv("LRL_GEMM_TRACE") != nullptr;  // shape log for profiling runs
  if (trace)
    fprintf(stderr, "gemm layout=%d epi=%d M=%d N=%d K=%d groups=%d splits=%d avec=%d bvec=%d arows=%d brows=%d\n",
            layout, epi, p.M, p.N, p.K, groups, p.splits, p.avec, p.bvec, p.a_rows != nullptr, p.b_rows != nullptr);
  // weight products with a pre-split B: the LDS-DMA x6p kernel
  g_last_path = 0;
  if (int xr = try_x6p(p, layout, epi, groups, st)) {
    if (xr > 0) g_last_path = 1;
    return xr > 0 ? 0 : xr;
  }
  if (int xr = try_x6t(p, layout, epi, groups, st)) {
    if (xr > 0) g_last_path = 2;
    return xr > 0 ? 0 : xr;
  }
  // fp32 on the bf16 MFMA (exact split, fp32-class error) wherever the tile shapes fit
  if (int xr = try_x6(p, layout, epi, groups, st)) return xr > 0 ? 0 : xr;
  // LDS-DMA path: batch-major product, every tile interior, float4-aligned operands, single split
  if (layout != GEMM_TN && p.splits == 1 && p.M % 64 == 0 && p.N % 64 == 0 && p.K % 16 == 0 && p.K >= 32 &&
      p.avec == 4 && p.bvec == 4 && epi != EPI_PARTIAL && (layout == GEMM_NT || layout == GEMM_NN)) {
    dim3 g1((p.M / 64) * (p.N / 64) * groups);
#ifndef LRL_GLDS_BK32
#define LRL_GLDS_BK32 1
#endif
    const bool bk32 = LRL_GLDS_BK32 && p.K % 32 == 0 && p.K >= 64;
#define LRL_GLDS(L, E)                                                                      \
  do {                                                                                      \
    if (bk32) hipLaunchKernelGGL((gemm_glds32_kernel<L, E>), g1, dim3(GTHREADS), 0, st, p); \
    else hipLaunchKernelGGL((gemm_glds_kernel<L, E>), g1, dim3(GTHREADS), 0, st, p);        \
  } while (0)
    if (layout == GEMM_NT) {
      if (epi == EPI_STORE) LRL_GLDS(GEMM_NT, EPI_STORE);
      else if (epi == EPI_BIAS) LRL_GLDS(GEMM_NT, EPI_BIAS);
      else LRL_GLDS(GEMM_NT, EPI_BIAS_ELU);
    } else {
      if (epi == EPI_STORE) LRL_GLDS(GEMM_NN, EPI_STORE);
      else LRL_GLDS(GEMM_NN, EPI_DELU);
    }
#undef LRL_GLDS
    return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
  }
  // LDS-DMA weight gradient: 128-row m tiles, 128-wide n tiles whose reads stay inside the row pitch,
  // whole 16-row slices in every split, float4-aligned operands
#ifndef LRL_GLDS_TN
#define LRL_GLDS_TN 1
#endif
  if (LRL_GLDS_TN && layout == GEMM_TN && epi == EPI_PARTIAL && p.M % 128 == 0 && p.K % 16 == 0 &&
      p.kps % 16 == 0 && p.avec == 4 && p.bvec == 4 && p.kps <= 8192) {
    if (p.N <= 64 && p.ldb >= 64) return launch_glds_tn<64>(p, groups, st);
    if ((int64_t)((p.N + 127) / 128) * 128 <= p.ldb) return launch_glds_tn<128>(p, groups, st);
  }
  // thin output (N <= 32): B staged whole in LDS, k split over the workgroup's waves
  const int kb128 = p.K / 128;
  if (layout != GEMM_TN && p.splits == 1 && p.N <= 32 && p.K % 128 == 0 && p.avec == 4 && p.M >= 256 &&
      (kb128 == 4 || kb128 == 8) &&  // (shorter k: the register-staged 128 x 32 tile is as fast)
      (epi == EPI_STORE || epi == EPI_BIAS || epi == EPI_BIAS_ELU)) {
    int trc = LRL_E_INVALID;
    if (layout == GEMM_NT) {
      if (epi == EPI_STORE) trc = launch_thin<GEMM_NT, EPI_STORE>(p, groups, st);
      else if (epi == EPI_BIAS) trc = launch_thin<GEMM_NT, EPI_BIAS>(p, groups, st);
      else trc = launch_thin<GEMM_NT, EPI_BIAS_ELU>(p, groups, st);
    } else {
      if (epi == EPI_STORE) trc = launch_thin<GEMM_NN, EPI_STORE>(p, groups, st);
      else if (epi == EPI_BIAS) trc = launch_thin<GEMM_NN, EPI_BIAS>(p, groups, st);
      else trc = launch_thin<GEMM_NN, EPI_BIAS_ELU>(p, groups, st);
    }
    if (trc) return trc;
    return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
  }
  int rc = LRL_E_INVALID;
  if (bm == 128 && bn == 128) rc = launch_bm<128, 128>(p, layout, epi, grid, st);
  else if (bm == 128 && bn == 64) rc = launch_bm<128, 64>(p, layout, epi, grid, st);
  else if (bm == 64 && bn == 128) rc = launch_bm<64, 128>(p, layout, epi, grid, st);
  else if (bm == 64 && bn == 64) rc = launch_bm<64, 64>(p, layout, epi, grid, st);
  else if (bm == 128 && bn == 32) rc = launch_bm<128, 32>(p, layout, epi, grid, st);
  else if (bm == 32 && bn == 128) rc = launch_bm<32, 128>(p, layout, epi, grid, st);
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : LRL_E_HIP;
}

}  // namespace lrl

extern "C" int32_t lrl_debug_gemm_paths(int32_t disable_mask) {
  return __atomic_exchange_n(&lrl::g_path_off, (int)disable_mask, __ATOMIC_RELAXED);
}
