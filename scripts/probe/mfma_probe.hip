// MFMA throughput/power probe: back-to-back v_mfma_f32_16x16x32_f16 vs
// v_mfma_f32_32x32x16_f16 on every SIMD (4 waves per SIMD), same FLOPs per
// wave, operands changing from one MFMA to the next (random fp16 bits) or, with
// "const", the same operands for every MFMA. Prints
// TFLOP/s per shape; run under scripts/gpu_power.sh (CMD=...) to compare the
// board power each draws. Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ half8 rnd8(unsigned s) {
  half8 h;
  for (int i = 0; i < 8; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = (_Float16)((float)(s >> 8) * (1.0f / 16777216.0f) - 0.5f);
  }
  return h;
}

__global__ void __launch_bounds__(256) mfma16(float* out, int iters, int same) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const half8 a0 = rnd8(t * 8 + 1), a1 = rnd8(t * 8 + 2 - same), a2 = rnd8(t * 8 + 3 - 2 * same),
              a3 = rnd8(t * 8 + 4 - 3 * same);
  const half8 b0 = rnd8(t * 8 + 5), b1 = rnd8(t * 8 + 6 - same), b2 = rnd8(t * 8 + 7 - 2 * same),
              b3 = rnd8(t * 8 + 8 - 3 * same);
  floatx4 c[4] = {};
  for (int it = 0; it < iters; ++it) {   // asm: keeps the compiler from shuffling the loop-carried accumulators
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %4, %8, %0\n\t"
                 "v_mfma_f32_16x16x32_f16 %1, %5, %9, %1\n\t"
                 "v_mfma_f32_16x16x32_f16 %2, %6, %10, %2\n\t"
                 "v_mfma_f32_16x16x32_f16 %3, %7, %11, %3"
                 : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3])
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
  }
  const floatx4 s = c[0] + c[1] + c[2] + c[3];
  out[t] = s[0] + s[1] + s[2] + s[3];
}

__global__ void __launch_bounds__(256) mfma32(float* out, int iters, int same) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const half8 a0 = rnd8(t * 8 + 1), a1 = rnd8(t * 8 + 2 - same), b0 = rnd8(t * 8 + 5), b1 = rnd8(t * 8 + 6 - same);
  floatx16 c0 = {}, c1 = {};
  for (int it = 0; it < iters; ++it) {   // 2 x 32x32x16 = 4 x 16x16x32 in FLOPs
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %4, %0\n\t"
                 "v_mfma_f32_32x32x16_f16 %1, %3, %5, %1"
                 : "+v"(c0), "+v"(c1) : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  out[t] = s;
}

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200000;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int same = argc > 3 && argv[3][0] == 'c';   // "const": the same operands for every MFMA
  const int blocks = 256 * 4, threads = 256;   // 4 waves per SIMD on 256 CUs
  float* out;
  CK(hipMalloc(&out, sizeof(float) * blocks * threads));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int shape = 0; shape < 2; ++shape) {
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      if (shape == 0) mfma16<<<blocks, threads>>>(out, iters, same);
      else mfma32<<<blocks, threads>>>(out, iters, same);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double flops = 4.0 * 16384.0 * iters * (blocks * threads / 64);
      printf("%s %s %.1f ms %.1f TFLOP/s\n", shape ? "32x32x16" : "16x16x32", same ? "const" : "random", ms,
             flops / ms / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(out));
  return 0;
}
