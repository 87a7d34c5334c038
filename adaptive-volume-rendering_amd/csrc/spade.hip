// The spade product rule's backward over row-major rows (avr.layer_train; models.py:585-587: X' = S * X + T
// before block b < n_lin_z): from the gradient g at X', the scale_z rows' gradient gs = g * X and the gradient
// carried on to X, g_out = S * g, plus max |gs| for the scale_z weight gradient's scale -- one pass (three
// reads, two writes) where torch took two products and a reduction (three more passes). Each product is the
// same single fp32 rounding torch's mul makes, so both outputs are bit-identical to it. HBM-bound: float4 per
// lane, a grid of at most kSpadeBlocks workgroups walking the values so the maximum is one publish per wave.
#include "avr_common.h"

namespace avr {

constexpr int kSpadeThreads = 256;
constexpr int kSpadeBlocks = 4096;

__global__ void __launch_bounds__(kSpadeThreads) spade_bwd_rows_kernel(int64_t n4, const floatx4* __restrict__ g,
                                                                      const floatx4* __restrict__ x,
                                                                      const floatx4* __restrict__ s,
                                                                      floatx4* __restrict__ gs,
                                                                      floatx4* __restrict__ g_out, unsigned* gs_max) {
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kSpadeThreads;
  for (int64_t i = (int64_t)blockIdx.x * kSpadeThreads + threadIdx.x; i < n4; i += stride) {
    const floatx4 gv = g[i], xv = x[i], sv = s[i];
    floatx4 a, b;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = fmul(gv[e], xv[e]);
      b[e] = fmul(sv[e], gv[e]);
      m = fmaxf(m, fabsf(a[e]));
    }
    gs[i] = a;
    g_out[i] = b;
  }
  if (gs_max) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) m = fmaxf(m, lane_xor(m, d, lane));
    if (lane == 0) publish_max(gs_max, m);
  }
}

}  // namespace avr

using namespace avr;

extern "C" int avr_spade_bwd_rows(int64_t n, const float* g, const float* x, const float* s, float* gs, float* g_out,
                                  uint32_t* gs_max, void* stream) {
  AVR_REQUIRE(n >= 0 && n % 4 == 0, "avr_spade_bwd_rows: n %lld (a multiple of 4)", (long long)n);
  if (n == 0) return AVR_OK;
  AVR_REQUIRE(g && x && s && gs && g_out, "avr_spade_bwd_rows: null pointer");
  AVR_REQUIRE(((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(s) |
                reinterpret_cast<uintptr_t>(gs) | reinterpret_cast<uintptr_t>(g_out)) & 15) == 0,
              "avr_spade_bwd_rows: 16-B aligned arrays");
  const int64_t n4 = n / 4;
  int64_t blocks = (n4 + kSpadeThreads - 1) / kSpadeThreads;
  if (blocks > kSpadeBlocks) blocks = kSpadeBlocks;
  spade_bwd_rows_kernel<<<(unsigned)blocks, kSpadeThreads, 0, as_stream(stream)>>>(
      n4, reinterpret_cast<const floatx4*>(g), reinterpret_cast<const floatx4*>(x),
      reinterpret_cast<const floatx4*>(s), reinterpret_cast<floatx4*>(gs), reinterpret_cast<floatx4*>(g_out), gs_max);
  return check_launch("spade_bwd_rows_kernel");
}
