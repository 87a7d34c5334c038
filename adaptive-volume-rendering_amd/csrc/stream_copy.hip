// Streaming device copy and fill: the "achievable HBM" yardsticks of the bench
// (each HBM-bound kernel is reported against the 8 TB/s peak and
// against what a plain copy reaches on the same box). 16 B per lane, four
// independent loads in flight per lane before the stores, every wave
// instruction a contiguous 1 KiB; one pass, no grid-stride loop.
#include "avr_common.h"

namespace avr {

constexpr int kCopyThreads = 256;
constexpr int kCopyUnroll = 4;

__global__ void __launch_bounds__(kCopyThreads) stream_copy_kernel(const uint4* __restrict__ src,
                                                                   uint4* __restrict__ dst, int64_t n16) {
  const int64_t base = (int64_t)blockIdx.x * (kCopyThreads * kCopyUnroll) + threadIdx.x;
  uint4 v[kCopyUnroll];
#pragma unroll
  for (int k = 0; k < kCopyUnroll; ++k) {
    const int64_t i = base + (int64_t)k * kCopyThreads;
    if (i < n16) v[k] = src[i];
  }
#pragma unroll
  for (int k = 0; k < kCopyUnroll; ++k) {
    const int64_t i = base + (int64_t)k * kCopyThreads;
    if (i < n16) dst[i] = v[k];
  }
}

// write-only twin: the same 1 KiB per wave instruction, four stores per lane
__global__ void __launch_bounds__(kCopyThreads) stream_fill_kernel(uint4* __restrict__ dst, int64_t n16, uint32_t w) {
  const int64_t base = (int64_t)blockIdx.x * (kCopyThreads * kCopyUnroll) + threadIdx.x;
  const uint4 v = make_uint4(w, w, w, w);
#pragma unroll
  for (int k = 0; k < kCopyUnroll; ++k) {
    const int64_t i = base + (int64_t)k * kCopyThreads;
    if (i < n16) dst[i] = v;
  }
}

}  // namespace avr

using namespace avr;

extern "C" int avr_stream_copy(const void* src, void* dst, int64_t n_bytes, void* stream) {
  AVR_REQUIRE(n_bytes >= 0 && n_bytes % 16 == 0, "avr_stream_copy: n_bytes must be a non-negative multiple of 16");
  if (n_bytes == 0) return AVR_OK;
  AVR_REQUIRE(src && dst, "avr_stream_copy: null pointer");
  AVR_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "avr_stream_copy: pointers must be 16-B aligned");
  const int64_t n16 = n_bytes / 16;
  const int64_t per = kCopyThreads * kCopyUnroll;
  const int64_t blocks = (n16 + per - 1) / per;
  AVR_REQUIRE(blocks < (1ll << 31), "avr_stream_copy: too large");
  stream_copy_kernel<<<(unsigned)blocks, kCopyThreads, 0, as_stream(stream)>>>(reinterpret_cast<const uint4*>(src),
                                                                              reinterpret_cast<uint4*>(dst), n16);
  return check_launch("stream_copy_kernel");
}

extern "C" int avr_stream_fill(void* dst, int64_t n_bytes, uint32_t word, void* stream) {
  AVR_REQUIRE(n_bytes >= 0 && n_bytes % 16 == 0, "avr_stream_fill: n_bytes must be a non-negative multiple of 16");
  if (n_bytes == 0) return AVR_OK;
  AVR_REQUIRE(dst, "avr_stream_fill: null pointer");
  AVR_REQUIRE(((uintptr_t)dst & 15) == 0, "avr_stream_fill: pointer must be 16-B aligned");
  const int64_t n16 = n_bytes / 16;
  const int64_t per = kCopyThreads * kCopyUnroll;
  const int64_t blocks = (n16 + per - 1) / per;
  AVR_REQUIRE(blocks < (1ll << 31), "avr_stream_fill: too large");
  stream_fill_kernel<<<(unsigned)blocks, kCopyThreads, 0, as_stream(stream)>>>(reinterpret_cast<uint4*>(dst), n16, word);
  return check_launch("stream_fill_kernel");
}
