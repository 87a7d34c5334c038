// Store-path probe for the coarse z kernels: 65536 rays x 128 samples of fp32
// (33.5 MB) written as one float4 per thread, (a) constant values, (b) values
// from one Philox4x32-10 block per thread (the sampling kernels' draw), (c) as
// (b) but four float4 per thread. Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y, (uint32_t)p0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__global__ void __launch_bounds__(256) k_const(float4* z, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) z[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

__global__ void __launch_bounds__(256) k_philox(float4* z, int64_t n4, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const uint4 r = philox(make_uint4((uint32_t)(i >> 5), 0u, (uint32_t)(i & 31), 0x1001u),
                         make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float s = 5.9604644775390625e-08f;
  z[i] = make_float4((r.x >> 8) * s, (r.y >> 8) * s, (r.z >> 8) * s, (r.w >> 8) * s);
}

__global__ void __launch_bounds__(256) k_philox4(float4* z, int64_t n4, uint64_t seed) {
  const int64_t base = ((int64_t)blockIdx.x * blockDim.x) * 4 + threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t i = base + q * blockDim.x;
    if (i >= n4) return;
    const uint4 r = philox(make_uint4((uint32_t)(i >> 5), 0u, (uint32_t)(i & 31), 0x1001u),
                           make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const float s = 5.9604644775390625e-08f;
    z[i] = make_float4((r.x >> 8) * s, (r.y >> 8) * s, (r.z >> 8) * s, (r.w >> 8) * s);
  }
}

int main() {
  const int64_t n4 = 65536ll * 128 / 4;
  float4* z;
  CK(hipMalloc(&z, n4 * sizeof(float4)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned g1 = (unsigned)((n4 + 255) / 256), g4 = (unsigned)((n4 + 1023) / 1024);
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int it = 0; it < 50; ++it) {
        if (v == 0) k_const<<<g1, 256>>>(z, n4);
        else if (v == 1) k_philox<<<g1, 256>>>(z, n4, 7 + it);
        else k_philox4<<<g4, 256>>>(z, n4, 7 + it);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s %.2f us/launch %.0f GB/s\n", v == 0 ? "const" : v == 1 ? "philox" : "philox4", ms * 1e3 / 50,
             n4 * 16.0 / (ms * 1e-3 / 50) / 1e9);
    }
  }
  CK(hipFree(z));
  return 0;
}
