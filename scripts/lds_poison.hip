// Determinism probe helper (scripts/determinism_probe.py): fills the LDS of every CU with a chosen 32-bit pattern
// before a launch, so a kernel that reads LDS it never wrote this launch sees that pattern instead of whatever the
// previous workgroup on the CU left there.  Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC lds_poison.hip -o
// liblds_poison.so
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr int POISON_WORDS = 40960;  // all 160 KiB of a CU's LDS per workgroup (one resident per CU)

__global__ __launch_bounds__(256) void lds_poison_kernel(uint32_t pattern, uint32_t* sink) {
  __shared__ uint32_t buf[POISON_WORDS];
  for (int i = threadIdx.x; i < POISON_WORDS; i += blockDim.x) buf[i] = pattern;
  __syncthreads();
  // keep the stores: one word read back and written out under a condition the host never meets
  if (buf[(threadIdx.x * 61) % POISON_WORDS] == pattern + 1u) sink[blockIdx.x] = 1u;
}

extern "C" int lds_poison(uint32_t pattern, void* sink, void* stream) {
  hipLaunchKernelGGL(lds_poison_kernel, dim3(256 * 4), dim3(256), 0, (hipStream_t)stream, pattern, (uint32_t*)sink);
  return (int)hipGetLastError();
}
