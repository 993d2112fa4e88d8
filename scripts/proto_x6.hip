// Prototype (timing / numerics experiment, not product): fp32 GEMM on the bf16 MFMA with the exact 3-way split
// x = hi + mid + lo done while staging (each operand element split once per workgroup, three bf16 planes in LDS),
// six products per k-step (hh hm mh hl mm lh; dropped terms <= 2^-24 relative), fp32 accumulation.
// 128x128 tile, 4 waves of 64x64 (2x2 v_mfma_f32_32x32x16_bf16 tiles), BK = 16, two LDS stages, register prefetch.
// Operands: KC = row-major [r][k] (float4 loads), RC = k-major [k][r] (dword loads of 8 consecutive k per lane).
//   NT forward:        A KC (row gather), B KC
//   NN backward-data:  A KC, B RC
//   TN weight grad:    A RC, B RC (k-row gather on B), split-k partials
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/proto_x6.hip -o scripts/proto_x6.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 128, BN = 128, BK = 16, TH = 256;
constexpr int PLANE = 128 * BK;          // bf16 elements per plane image
constexpr int OPER = 3 * PLANE;          // per operand
constexpr int STAGE = 2 * OPER;          // per stage (A then B)

struct P {
  const float* A; const float* B; float* C;
  const int* a_rows;  // KC A row gather (NT) or null
  const int* b_rows;  // RC B k-row gather (TN) or null
  int M, N, K, lda, ldb, ldc, kps;
  int64_t part_stride;
};

__device__ __forceinline__ uint32_t hi16pair(uint32_t u0, uint32_t u1) {
  return __builtin_amdgcn_perm(u1, u0, 0x07060302u);
}
// (x0, x1) -> packed bf16 pairs of the hi / mid / lo parts (truncation split: exact)
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  uint32_t u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
  h = hi16pair(u0, u1);
  float r0 = x0 - __uint_as_float(u0 & 0xffff0000u), r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
  u0 = __float_as_uint(r0); u1 = __float_as_uint(r1);
  m = hi16pair(u0, u1);
  r0 = r0 - __uint_as_float(u0 & 0xffff0000u); r1 = r1 - __uint_as_float(u1 & 0xffff0000u);
  l = hi16pair(__float_as_uint(r0), __float_as_uint(r1));
}

// swizzled offset (bf16 elements) of 8-element chunk c (0/1) of row r in a [128][16] plane image
__device__ __forceinline__ int chunk_off(int r, int c) { return r * BK + 8 * (c ^ ((r >> 3) & 1)); }

template <bool KC>
struct Op {
  // KC: 2 float4 per thread (rows t/4 and 64 + t/4, k-quad t%4); RC: 8 dwords (row t%128, k = 8 (t/128) + e)
  float v[8];
  const float* base[KC ? 2 : 1];
  const float* P_;
  const int* krows;
  int ld, r0;
  __device__ __forceinline__ void init(const float* Pp, int ldp, const int* rrows, const int* kr, int r0p) {
    P_ = Pp; ld = ldp; krows = kr; r0 = r0p;
    const int t = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = (t >> 2) + 64 * u;
        const int gr = rrows ? rrows[r0 + r] : r0 + r;
        base[u] = Pp + (int64_t)gr * ldp + 4 * (t & 3);
      }
    } else {
      base[0] = Pp + r0 + (t & 127);
    }
  }
  __device__ __forceinline__ void load(int k0) {
    const int t = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 q = *reinterpret_cast<const float4*>(base[u] + k0);
        v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
      }
    } else {
      const int kb = k0 + 8 * (t >> 7);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = kb + e;
        const int64_t kr = krows ? krows[k] : k;
        v[e] = base[0][kr * ld];
      }
    }
  }
  __device__ __forceinline__ void store(uint16_t* img) const {
    const int t = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = (t >> 2) + 64 * u, j = t & 3;
        uint32_t h0, m0, l0, h1, m1, l1;
        split2(v[4 * u], v[4 * u + 1], h0, m0, l0);
        split2(v[4 * u + 2], v[4 * u + 3], h1, m1, l1);
        const int off = chunk_off(r, j >> 1) + 4 * (j & 1);
        *reinterpret_cast<uint2*>(img + off) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(img + PLANE + off) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(img + 2 * PLANE + off) = make_uint2(l0, l1);
      }
    } else {
      const int r = t & 127, c = t >> 7;
      uint32_t h[4], m[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split2(v[2 * e], v[2 * e + 1], h[e], m[e], l[e]);
      const int off = chunk_off(r, c);
      *reinterpret_cast<uint4*>(img + off) = make_uint4(h[0], h[1], h[2], h[3]);
      *reinterpret_cast<uint4*>(img + PLANE + off) = make_uint4(m[0], m[1], m[2], m[3]);
      *reinterpret_cast<uint4*>(img + 2 * PLANE + off) = make_uint4(l[0], l[1], l[2], l[3]);
    }
  }
};

template <bool AKC, bool BKC, bool PART>
__global__ __launch_bounds__(TH, 2) void x6_kernel(P p) {
  __shared__ __attribute__((aligned(16))) uint16_t S[2 * STAGE];
  const int mt = p.M / BM, nt = p.N / BN;
  int L;
  {
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tn = L % nt, tm = (L / nt) % mt, sp = L / (nt * mt);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = PART ? sp * p.kps : 0, kend = PART ? min(p.K, kbeg + p.kps) : p.K;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 31, h = lane >> 5;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  Op<AKC> oa;
  Op<BKC> ob;
  oa.init(p.A, p.lda, AKC ? p.a_rows : nullptr, nullptr, m0);
  ob.init(p.B, p.ldb, nullptr, BKC ? nullptr : p.b_rows, n0);
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  oa.load(kbeg);
  ob.load(kbeg);
  oa.store(S);
  ob.store(S + OPER);
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) {
      oa.load(k0 + BK);
      ob.load(k0 + BK);
    }
    const uint16_t* As = S + buf * STAGE;
    const uint16_t* Bs = As + OPER;
    bf16x8 a[2][3], b[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ra = wm + 32 * i + li, rb = wn + 32 * i + li;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        a[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * PLANE + chunk_off(ra, h));
        b[i][pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * PLANE + chunk_off(rb, h));
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
        acc[i][j] = c;
      }
    if (more) {
      oa.store(S + (buf ^ 1) * STAGE);
      ob.store(S + (buf ^ 1) * STAGE + OPER);
    }
    __syncthreads();
    buf ^= 1;
  }
  float* C = p.C + (PART ? (int64_t)sp * p.part_stride : 0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        const int col = n0 + wn + 32 * j + li;
        C[(int64_t)row * p.ldc + col] = acc[i][j][q];
      }
}

static uint64_t s_rng = 12345;
static double rnd() { s_rng = s_rng * 6364136223846793005ull + 1442695040888963407ull; return ((s_rng >> 40) / 16777216.0) * 2 - 1; }

// layout 0 NT: A[M][K] (rows gathered from M+64), B[N][K]; 2 NN: A[M][K], B[K][N]; 3 TN: A[K][M], B[K+64][N] gathered
int run(int layout, int M, int N, int K, int splits) {
  const bool gather = layout != 2;
  const int arows_n = layout == 0 ? M + 64 : 0, krows_n = layout == 3 ? K + 64 : 0;
  std::vector<float> hA(layout == 0 ? (size_t)arows_n * K : (size_t)M * K), hB(layout == 3 ? (size_t)krows_n * N : (size_t)N * K);
  for (auto& v : hA) v = (float)(rnd() * (rnd() > 0 ? 1.0 : 0.01));
  for (auto& v : hB) v = (float)(rnd() * 0.1);
  const int nsrc = layout == 0 ? arows_n : krows_n, nrows = layout == 0 ? M : (layout == 3 ? K : 0);
  std::vector<int> perm(nsrc > 0 ? nsrc : 0);
  for (size_t i = 0; i < perm.size(); ++i) perm[i] = (int)i;
  for (size_t i = perm.size(); i > 1; --i) { size_t j = (size_t)((rnd() * 0.5 + 0.5) * (i - 1)); std::swap(perm[i - 1], perm[j]); }
  std::vector<int> rows(perm.begin(), perm.begin() + nrows);
  (void)gather;
  float *dA, *dB, *dC; int* dR = nullptr;
  hipMalloc(&dA, hA.size() * 4); hipMalloc(&dB, hB.size() * 4);
  const size_t csz = (size_t)M * N * (layout == 3 ? splits : 1);
  hipMalloc(&dC, csz * 4);
  hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice);
  if (!rows.empty()) { hipMalloc(&dR, rows.size() * 4); hipMemcpy(dR, rows.data(), rows.size() * 4, hipMemcpyHostToDevice); }
  P p{};
  p.A = dA; p.B = dB; p.C = dC; p.M = M; p.N = N; p.K = K; p.ldc = N;
  p.kps = K / splits; p.part_stride = (int64_t)M * N;
  if (layout == 0) { p.lda = K; p.ldb = K; p.a_rows = dR; }
  if (layout == 2) { p.lda = K; p.ldb = N; }
  if (layout == 3) { p.lda = M; p.ldb = N; p.b_rows = dR; }
  dim3 grid((M / BM) * (N / BN) * (layout == 3 ? splits : 1));
  auto launch = [&]() {
    if (layout == 0) hipLaunchKernelGGL((x6_kernel<true, true, false>), grid, dim3(TH), 0, 0, p);
    else if (layout == 2) hipLaunchKernelGGL((x6_kernel<true, false, false>), grid, dim3(TH), 0, 0, p);
    else hipLaunchKernelGGL((x6_kernel<false, false, true>), grid, dim3(TH), 0, 0, p);
  };
  for (int it = 0; it < 5; ++it) launch();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int reps = 50;
  hipEventRecord(e0, 0);
  for (int it = 0; it < reps; ++it) launch();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= reps;
  std::vector<float> hc(csz);
  hipMemcpy(hc.data(), dC, csz * 4, hipMemcpyDeviceToHost);
  double emax = 0;
  for (int smp = 0; smp < 3000; ++smp) {
    const int m = (int)((rnd() * 0.5 + 0.5) * (M - 1)), n = (int)((rnd() * 0.5 + 0.5) * (N - 1));
    double ref = 0, mag = 0, got = 0;
    for (int k = 0; k < K; ++k) {
      double a, b;
      if (layout == 0) { a = hA[(size_t)rows[m] * K + k]; b = hB[(size_t)n * K + k]; }
      else if (layout == 2) { a = hA[(size_t)m * K + k]; b = hB[(size_t)k * N + n]; }
      else { a = hA[(size_t)k * M + m]; b = hB[(size_t)rows[k] * N + n]; }
      ref += a * b; mag += fabs(a * b);
    }
    if (layout == 3) for (int s = 0; s < splits; ++s) got += hc[(size_t)s * M * N + (size_t)m * N + n];
    else got = hc[(size_t)m * N + n];
    emax = fmax(emax, fabs(got - ref) / mag);
  }
  const double flop = 2.0 * M * N * K;
  printf("{\"layout\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"splits\": %d, \"us\": %.1f, \"tf\": %.1f, \"maxrel\": %.3g}\n",
         layout, M, N, K, splits, ms * 1e3, flop / (ms * 1e-3) / 1e12, emax);
  hipFree(dA); hipFree(dB); hipFree(dC); if (dR) hipFree(dR);
  return 0;
}

int main() {
  run(0, 24576, 256, 512, 1);
  run(0, 24576, 512, 512, 1);
  run(0, 24576, 256, 640, 1);
  run(0, 24576, 1024, 64, 1);
  run(2, 24576, 512, 256, 1);
  run(2, 24576, 1024, 256, 1);
  run(3, 256, 512, 24576, 48);
  run(3, 256, 512, 24576, 24);
  run(3, 256, 640, 24576, 24);
  return 0;
}
