// Prototype (timing / numerics experiment, not product): fp32 NT GEMM C[m][n] = sum_k A[m][k] W[n][k] on
// bf16 MFMA with the exact 3-way split x = hi + mid + lo (truncation: each part a bf16, the remainders exact) and
// the six products whose order is <= 2^-16 (hh, hm, mh, hl, mm, lh), fp32 accumulation — against the same tile
// structure on the fp32 MFMA, on the update's largest forward shape.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/proto_bf16x6.hip -o /tmp/proto_bf16x6
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 128, BN = 128, BK = 32, PITCH = BK + 4, THREADS = 256;

// hi / mid / lo bf16 parts of 8 floats (exact: x = hi + mid + lo)
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t u = __float_as_uint(x[j]);
    const uint32_t uh = u & 0xffff0000u;
    const float r1 = x[j] - __uint_as_float(uh);
    const uint32_t u1 = __float_as_uint(r1);
    const uint32_t um = u1 & 0xffff0000u;
    const float r2 = r1 - __uint_as_float(um);
    h[j] = (short)(uh >> 16);
    m[j] = (short)(um >> 16);
    l[j] = (short)(__float_as_uint(r2) >> 16);
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(THREADS, 2) void gemm_nt(const float* __restrict__ A, const float* __restrict__ W,
                                                      float* __restrict__ C, int M, int N, int K) {
  __shared__ float As[2][BM][PITCH];
  __shared__ float Bs[2][BN][PITCH];
  const int nt = N / BN;
  const int tm = blockIdx.x / nt, tn = blockIdx.x % nt;
  const int m0 = tm * BM, n0 = tn * BN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int r = lane & 31, h = lane >> 5;
  // staging: 128 rows x 32 k = 1024 float4, 4 per thread
  float4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = t + u * THREADS, row = i >> 3, c = (i & 7) * 4;
      ra[u] = *reinterpret_cast<const float4*>(A + (int64_t)(m0 + row) * K + k0 + c);
      rb[u] = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + row) * K + k0 + c);
    }
  };
  auto sstore = [&](int b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = t + u * THREADS, row = i >> 3, c = (i & 7) * 4;
      *reinterpret_cast<float4*>(&As[b][row][c]) = ra[u];
      *reinterpret_cast<float4*>(&Bs[b][row][c]) = rb[u];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  gload(0);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += BK) {
    if (k0 + BK < K) gload(k0 + BK);
    if constexpr (SPLIT) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float x[8];
          const float4 v0 = *reinterpret_cast<const float4*>(&As[buf][wm + 32 * i + r][16 * ks + 8 * h]);
          const float4 v1 = *reinterpret_cast<const float4*>(&As[buf][wm + 32 * i + r][16 * ks + 8 * h + 4]);
          x[0] = v0.x; x[1] = v0.y; x[2] = v0.z; x[3] = v0.w; x[4] = v1.x; x[5] = v1.y; x[6] = v1.z; x[7] = v1.w;
          split8(x, ah[i], am[i], al[i]);
          const float4 w0 = *reinterpret_cast<const float4*>(&Bs[buf][wn + 32 * i + r][16 * ks + 8 * h]);
          const float4 w1 = *reinterpret_cast<const float4*>(&Bs[buf][wn + 32 * i + r][16 * ks + 8 * h + 4]);
          x[0] = w0.x; x[1] = w0.y; x[2] = w0.z; x[3] = w0.w; x[4] = w1.x; x[5] = w1.y; x[6] = w1.z; x[7] = w1.w;
          split8(x, bh[i], bm[i], bl[i]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x16 c = acc[i][j];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], c, 0, 0, 0);
            acc[i][j] = c;
          }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        float a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          a[i] = As[buf][wm + 32 * i + r][2 * kk + h];
          b[i] = Bs[buf][wn + 32 * i + r][2 * kk + h];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
    if (k0 + BK < K) {
      sstore(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        const int col = n0 + wn + 32 * j + r;
        C[(int64_t)row * N + col] = acc[i][j][q];
      }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 24576, N = argc > 2 ? atoi(argv[2]) : 512, K = argc > 3 ? atoi(argv[3]) : 512;
  std::vector<float> hA((size_t)M * K), hW((size_t)N * K);
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return ((s >> 40) / 16777216.0) * 2 - 1; };
  for (auto& v : hA) v = (float)(rnd() * (rnd() > 0 ? 1.0 : 0.01));  // mixed magnitudes (post-ELU-like)
  for (auto& v : hW) v = (float)(rnd() * 0.1);
  float *dA, *dW, *dC1, *dC2;
  hipMalloc(&dA, hA.size() * 4);
  hipMalloc(&dW, hW.size() * 4);
  hipMalloc(&dC1, (size_t)M * N * 4);
  hipMalloc(&dC2, (size_t)M * N * 4);
  hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dW, hW.data(), hW.size() * 4, hipMemcpyHostToDevice);
  dim3 grid((M / BM) * (N / BN));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms[2];
  for (int v = 0; v < 2; ++v) {
    for (int it = 0; it < 3; ++it) {
      if (v == 0) hipLaunchKernelGGL(gemm_nt<false>, grid, dim3(THREADS), 0, 0, dA, dW, dC1, M, N, K);
      else hipLaunchKernelGGL(gemm_nt<true>, grid, dim3(THREADS), 0, 0, dA, dW, dC2, M, N, K);
    }
    hipEventRecord(e0, 0);
    const int reps = 50;
    for (int it = 0; it < reps; ++it) {
      if (v == 0) hipLaunchKernelGGL(gemm_nt<false>, grid, dim3(THREADS), 0, 0, dA, dW, dC1, M, N, K);
      else hipLaunchKernelGGL(gemm_nt<true>, grid, dim3(THREADS), 0, 0, dA, dW, dC2, M, N, K);
    }
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[v], e0, e1);
    ms[v] /= reps;
  }
  std::vector<float> c1((size_t)M * N), c2((size_t)M * N);
  hipMemcpy(c1.data(), dC1, c1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(c2.data(), dC2, c2.size() * 4, hipMemcpyDeviceToHost);
  // error vs an fp64 reference on sampled outputs, scaled by sum |a b|
  double e_f32 = 0, e_x6 = 0;
  for (int smp = 0; smp < 4000; ++smp) {
    const int m = (int)((rnd() * 0.5 + 0.5) * (M - 1)), n = (int)((rnd() * 0.5 + 0.5) * (N - 1));
    double ref = 0, mag = 0;
    for (int k = 0; k < K; ++k) {
      ref += (double)hA[(size_t)m * K + k] * hW[(size_t)n * K + k];
      mag += fabs((double)hA[(size_t)m * K + k] * hW[(size_t)n * K + k]);
    }
    e_f32 = fmax(e_f32, fabs(c1[(size_t)m * N + n] - ref) / mag);
    e_x6 = fmax(e_x6, fabs(c2[(size_t)m * N + n] - ref) / mag);
  }
  const double flop = 2.0 * M * N * K;
  printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"f32_us\": %.1f, \"f32_tf\": %.1f, \"bf16x6_us\": %.1f, \"bf16x6_tf\": %.1f, "
         "\"maxrel_f32\": %.3g, \"maxrel_bf16x6\": %.3g}\n",
         M, N, K, ms[0] * 1e3, flop / (ms[0] * 1e-3) / 1e12, ms[1] * 1e3, flop / (ms[1] * 1e-3) / 1e12, e_f32, e_x6);
  return 0;
}
