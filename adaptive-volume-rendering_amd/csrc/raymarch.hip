// LSTM ray marcher of Raymarcher / AdaptiveVolumeRenderer (renderers.py:313-351,
// :380-432): starting at ro + rd * d0, `steps` times
//   v      = latent features at the current point (phi(..., return_features=True),
//            models.py:753-823: pixel-aligned bilinear lookup, no MLP)
//   (h, c) = LSTMCell(v, (h, c))            hidden 16, gates i f g o (torch order)
//   sd     = out_layer(h)                   Linear(16, 1)
//   x      = x + rd * sd
// then the final distance (x - ro)_x / rd_x (quirk kept: x component only,
// renderers.py:490; rd_x = 0 gives inf / NaN as in the reference).
//
// The input projection W_ih v is linear in the bilinearly interpolated latent,
// so it is applied once per latent texel (gate table P = latent^T W_ih^T, 64
// floats per texel, computed by the caller) and interpolated per step: 4 x 256 B
// of gathers per ray and step instead of 4 x 2 KB plus a 512 x 64 GEMV.
// One ray per 16 lanes; lane k owns hidden unit k (its 4 gate rows of W_hh
// stay in registers, h_j comes in by 16-lane shuffles).
#include "field_common.h"

namespace avr {

constexpr int kHid = 16;           // LSTMCell hidden size (renderers.py:301, :370)
constexpr int kGates = 4 * kHid;   // i, f, g, o

__device__ __forceinline__ float sigmoid_(float x) { return fdiv(1.0f, fadd(1.0f, expf(-x))); }

__global__ void __launch_bounds__(256) raymarch_kernel(View v, const float* __restrict__ table,
                                                       const float* __restrict__ w_hh, const float* __restrict__ b_ih,
                                                       const float* __restrict__ b_hh, const float* __restrict__ w_out,
                                                       const float* __restrict__ b_out, const float* __restrict__ ro,
                                                       const float* __restrict__ rd, const float* __restrict__ d0,
                                                       int64_t n_rays, int steps, float* __restrict__ world,
                                                       float* __restrict__ final_dist, float* __restrict__ trace) {
  const int k = threadIdx.x & (kHid - 1);
  const int64_t ray_raw = (int64_t)blockIdx.x * (blockDim.x / kHid) + threadIdx.x / kHid;
  const bool live = ray_raw < n_rays;
  const int64_t ray = live ? ray_raw : n_rays - 1;   // keep the 16-lane group whole for the shuffles
  float wr[4][kHid], bias[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int j = 0; j < kHid; ++j) wr[q][j] = w_hh[(q * kHid + k) * kHid + j];
    bias[q] = fadd(b_ih[q * kHid + k], b_hh[q * kHid + k]);
  }
  const float wo = w_out[k], bo = b_out[0];
  const float r0 = ro[3 * ray], r1 = ro[3 * ray + 1], r2 = ro[3 * ray + 2];
  const float e0 = rd[3 * ray], e1 = rd[3 * ray + 1], e2 = rd[3 * ray + 2];
  const float dist0 = d0[ray];
  float x0 = fadd(r0, fmul(e0, dist0)), x1 = fadd(r1, fmul(e1, dist0)), x2 = fadd(r2, fmul(e2, dist0));
  if (trace && live && k < 3) trace[3 * ray + k] = k == 0 ? x0 : (k == 1 ? x1 : x2);
  float h = 0.f, c = 0.f;
  for (int s = 0; s < steps; ++s) {
    const Bilinear bl = bilinear_at(v, x0, x1, x2);
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // W_ih v + b_ih: bilinear blend of the per-texel projections
      const int row = q * kHid + k;
      const float p = ((table[(int64_t)bl.tex[0] * kGates + row] * bl.w[0] +
                        table[(int64_t)bl.tex[1] * kGates + row] * bl.w[1]) +
                       table[(int64_t)bl.tex[2] * kGates + row] * bl.w[2]) +
                      table[(int64_t)bl.tex[3] * kGates + row] * bl.w[3];
      g[q] = p + bias[q];
    }
#pragma unroll
    for (int j = 0; j < kHid; ++j) {
      const float hj = __shfl(h, j, kHid);
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] = fmaf(wr[q][j], hj, g[q]);
    }
    const float ig = sigmoid_(g[0]), fg = sigmoid_(g[1]), gg = tanhf(g[2]), og = sigmoid_(g[3]);
    c = fadd(fmul(fg, c), fmul(ig, gg));
    h = fmul(og, tanhf(c));
    float sd = fmul(wo, h);
#pragma unroll
    for (int d = kHid / 2; d > 0; d >>= 1) sd = fadd(sd, __shfl_xor(sd, d, kHid));
    sd = fadd(sd, bo);
    x0 = fadd(x0, fmul(e0, sd));   // world_coords + rds * signed_distance (renderers.py:341, :432)
    x1 = fadd(x1, fmul(e1, sd));
    x2 = fadd(x2, fmul(e2, sd));
    if (trace && live && k < 3) trace[(int64_t)(s + 1) * n_rays * 3 + 3 * ray + k] = k == 0 ? x0 : (k == 1 ? x1 : x2);
  }
  if (!live) return;
  if (k < 3) world[3 * ray + k] = k == 0 ? x0 : (k == 1 ? x1 : x2);
  if (k == 0 && final_dist) final_dist[ray] = fdiv(fsub(x0, r0), e0);   // renderers.py:490 (x component only)
}

}  // namespace avr

using namespace avr;

extern "C" int avr_raymarch(const avr_view_desc* view, const float* gate_table, const float* w_hh, const float* b_ih,
                            const float* b_hh, const float* w_out, const float* b_out, const float* ro,
                            const float* rd, const float* init_dist, int64_t n_rays, int steps, float* world,
                            float* final_dist, float* trace, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && steps >= 0, "avr_raymarch: negative size");
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(view && gate_table && w_hh && b_ih && b_hh && w_out && b_out && ro && rd && init_dist && world,
              "avr_raymarch: null pointer");
  AVR_REQUIRE(view->latent_h > 0 && view->latent_w > 0, "avr_raymarch: bad latent size");
  View v;
  view_from_desc(view, &v);
  const int per_block = 256 / kHid;
  raymarch_kernel<<<(unsigned)((n_rays + per_block - 1) / per_block), 256, 0, as_stream(stream)>>>(
      v, gate_table, w_hh, b_ih, b_hh, w_out, b_out, ro, rd, init_dist, n_rays, steps, world, final_dist, trace);
  return check_launch("raymarch_kernel");
}
