// Calibration (development tool): cycles per v_mfma_f32_32x32x16_bf16 on this box in the x6 kernel's arrangement —
// 256-thread workgroups, 4 waves, 3 workgroups per CU, each wave 2x2 output tiles x 6 products per k-step —
// (a) operands in registers only, (b) operands re-read from LDS each k-step (12 ds_read_b128 per 24 MFMAs),
// with random operand bits or with small normal values.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/proto_mfma_rate.hip -o scripts/proto_mfma_rate.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <bool LDS>
__global__ __launch_bounds__(256, 3) void rate_kernel(const uint16_t* __restrict__ src, float* out, int steps) {
  __shared__ __attribute__((aligned(16))) uint16_t S[2 * 3 * 2 * 128 * 16];  // 48 KB like the x6 stage pair
  for (int i = threadIdx.x; i < (int)(sizeof(S) / 2); i += 256) S[i] = src[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, li = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  bf16x8 a[2][3], b[2][3];
  for (int i = 0; i < 2; ++i)
    for (int p = 0; p < 3; ++p) {
      a[i][p] = *reinterpret_cast<const bf16x8*>(S + p * 2048 + (64 * (w >> 1) + 32 * i + li) * 16 + 8 * h);
      b[i][p] = *reinterpret_cast<const bf16x8*>(S + 6144 + p * 2048 + (64 * (w & 1) + 32 * i + li) * 16 + 8 * h);
    }
  for (int s = 0; s < steps; ++s) {
    if (LDS) {
      const uint16_t* As = S + (s & 1) * 12288;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          a[i][p] = *reinterpret_cast<const bf16x8*>(As + p * 2048 + (64 * (w >> 1) + 32 * i + li) * 16 + 8 * h);
          b[i][p] = *reinterpret_cast<const bf16x8*>(As + 6144 + p * 2048 + (64 * (w & 1) + 32 * i + li) * 16 + 8 * h);
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
  }
  float t = 0.f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int q = 0; q < 16; ++q) t += acc[i][j][q];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main() {
  const int n = 2 * 3 * 2 * 128 * 16, wgs = 768, steps = 512;
  uint16_t* h = new uint16_t[n];
  float *dout;
  uint16_t *dsrc;
  hipMalloc(&dsrc, n * 2);
  hipMalloc(&dout, wgs * 256 * 4);
  for (int mode = 0; mode < 2; ++mode) {
    uint64_t st = 99;
    for (int i = 0; i < n; ++i) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      const uint32_t r = (uint32_t)(st >> 33);
      // mode 0: random bits (any exponent, NaN / inf included); mode 1: normal values in [0.5, 2) with random sign
      h[i] = mode == 0 ? (uint16_t)r : (uint16_t)(((r & 1u) << 15) | ((126u + ((r >> 1) & 1u)) << 7) | ((r >> 2) & 0x7fu));
    }
    hipMemcpy(dsrc, h, n * 2, hipMemcpyHostToDevice);
    for (int lds = 0; lds < 2; ++lds) {
      auto launch = [&]() {
        if (lds) hipLaunchKernelGGL(rate_kernel<true>, dim3(wgs), dim3(256), 0, 0, dsrc, dout, steps);
        else hipLaunchKernelGGL(rate_kernel<false>, dim3(wgs), dim3(256), 0, 0, dsrc, dout, steps);
      };
      for (int it = 0; it < 3; ++it) launch();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0, 0);
      for (int it = 0; it < 10; ++it) launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 10;
      const double mfma = (double)wgs * 4 * steps * 24;  // per launch
      const double per_simd = mfma / 1024.0;              // 256 CUs x 4 SIMDs
      printf("{\"operands\": \"%s\", \"lds\": %d, \"ms\": %.4f, \"ns_per_mfma_per_simd\": %.3f, \"bf16_TF\": %.1f}\n",
             mode == 0 ? "random bits" : "normal", lds, ms, ms * 1e6 / per_simd, mfma * 32768.0 / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
