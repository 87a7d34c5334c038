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

// ------------------------------------------------------------------ training (ABI 11)
// The same march with autograd for train.py (AdaptiveVolumeRenderer / Raymarcher training: the reference
// backpropagates through 10 LSTMCell steps on grid_sample'd 512-channel features, renderers.py:413-432,
// :320-343, ~half of the train step in torch.profiler, profiles/r04b_train_profile_adaptive_mv.log).
// Forward: the kernel above over SB scenes (ray r of scene r / n_per_scene, its view and gate table), storing
// per step the point, h, c and the four gate activations. Backward, one ray per 16 lanes in reverse step order:
//   dsd = rd . dx;  dh = clamp(w_out dsd + W_hh^T dg_next, -10, 10)   (the reference's hook on state[0])
//   LSTMCell backward -> dg (64 gate pre-activations)
//   d table[texel] += w_corner dg (fixed-point int64 sums, below: W_ih's gradient is then dT^T latent, the
//   latent's W_ih^T dT)
//   dx += R^T d(xc) of the bilinear lookup's position gradient (grid_sample border / align_corners=True
//         backward: zero where the coordinate was clipped)
// with W_hh, the biases and out_layer's gradients summed per workgroup.
struct MarchScenes {
  View v[AVR_MAX_SCENES];
};
constexpr int kMarchState = 6 * kHid;   // per ray and step: h, c, i, f, g, o

// Lookup geometry of a point with the derivatives of the continuous texel coordinates (ix, iy) with respect
// to the camera point xc (models.py:753-760, SpatialEncoder.index :260-273, grid_sample align_corners=True,
// border: clipped coordinates have zero gradient, torch's clip_coordinates_set_grad).
struct LookupGrad {
  Bilinear bl;
  float wx0, wx1, wy0, wy1;
  float dix[3], diy[3];   // d ix / d xc, d iy / d xc (0 where clipped)
};

__device__ __forceinline__ LookupGrad lookup_grad(const View& v, float x0, float x1, float x2) {
  LookupGrad L;
  const float xr0 = dot3(v.R + 0, x0, x1, x2), xr1 = dot3(v.R + 3, x0, x1, x2), xr2 = dot3(v.R + 6, x0, x1, x2);
  const float xc0 = fadd(xr0, v.t[0]), xc1 = fadd(xr1, v.t[1]), xc2 = fadd(xr2, v.t[2]);
  const float u = fadd(fmul(fdiv(-xc0, xc2), v.focal[0]), v.c[0]);
  const float w = fadd(fmul(fdiv(-xc1, xc2), v.focal[1]), v.c[1]);
  const float gx = fsub(fmul(u, v.scale[0]), 1.0f), gy = fsub(fmul(w, v.scale[1]), 1.0f);
  const float ixr = fmul(fdiv(fadd(gx, 1.0f), 2.0f), (float)(v.W - 1));
  const float iyr = fmul(fdiv(fadd(gy, 1.0f), 2.0f), (float)(v.H - 1));
  const float ix = fminf(fmaxf(ixr, 0.f), (float)(v.W - 1));
  const float iy = fminf(fmaxf(iyr, 0.f), (float)(v.H - 1));
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  L.wx1 = fsub(ix, fx0); L.wy1 = fsub(iy, fy0);
  L.wx0 = fsub(fadd(fx0, 1.0f), ix); L.wy0 = fsub(fadd(fy0, 1.0f), iy);
  const int X0 = (int)fx0, Y0 = (int)fy0;
  const int X1 = X0 + 1 < v.W ? X0 + 1 : v.W - 1, Y1 = Y0 + 1 < v.H ? Y0 + 1 : v.H - 1;
  L.bl.tex[0] = Y0 * v.W + X0; L.bl.w[0] = fmul(L.wx0, L.wy0);
  L.bl.tex[1] = Y0 * v.W + X1; L.bl.w[1] = fmul(L.wx1, L.wy0);
  L.bl.tex[2] = Y1 * v.W + X0; L.bl.w[2] = fmul(L.wx0, L.wy1);
  L.bl.tex[3] = Y1 * v.W + X1; L.bl.w[3] = fmul(L.wx1, L.wy1);
  const bool cx = ixr > 0.f && ixr < (float)(v.W - 1), cy = iyr > 0.f && iyr < (float)(v.H - 1);
  const float ax = cx ? 0.5f * (float)(v.W - 1) * v.scale[0] * v.focal[0] : 0.f;
  const float ay = cy ? 0.5f * (float)(v.H - 1) * v.scale[1] * v.focal[1] : 0.f;
  // a clipped coordinate (ax / ay = 0) passes exactly zero, also where 1 / xc2 is infinite (a point on the
  // source camera's plane: 0 * inf would be NaN)
  const float iz = 1.0f / xc2;
  L.dix[0] = ax != 0.f ? -ax * iz : 0.f; L.dix[1] = 0.f; L.dix[2] = ax != 0.f ? ax * xc0 * iz * iz : 0.f;
  L.diy[0] = 0.f; L.diy[1] = ay != 0.f ? -ay * iz : 0.f; L.diy[2] = ay != 0.f ? ay * xc1 * iz * iz : 0.f;
  return L;
}

__global__ void __launch_bounds__(256) raymarch_train_kernel(MarchScenes sc, const float* __restrict__ tables,
                                                             int64_t table_stride, const float* __restrict__ w_hh,
                                                             const float* __restrict__ b_ih,
                                                             const float* __restrict__ b_hh,
                                                             const float* __restrict__ w_out,
                                                             const float* __restrict__ b_out,
                                                             const float* __restrict__ ro,
                                                             const float* __restrict__ rd,
                                                             const float* __restrict__ d0, int64_t n_per_scene,
                                                             int64_t n_rays, int steps, float* __restrict__ world,
                                                             float* __restrict__ trace, float* __restrict__ state) {
  const int k = threadIdx.x & (kHid - 1);
  const int64_t ray_raw = (int64_t)blockIdx.x * (blockDim.x / kHid) + threadIdx.x / kHid;
  const bool live = ray_raw < n_rays;
  const int64_t ray = live ? ray_raw : n_rays - 1;
  const int scene = (int)(ray / n_per_scene);
  const View& v = sc.v[scene];
  const float* table = tables + scene * table_stride;
  float wr[4][kHid], bias[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int j = 0; j < kHid; ++j) wr[q][j] = w_hh[(q * kHid + k) * kHid + j];
    bias[q] = fadd(b_ih[q * kHid + k], b_hh[q * kHid + k]);
  }
  const float wo = w_out[k], bo = b_out[0];
  const float e0 = rd[3 * ray], e1 = rd[3 * ray + 1], e2 = rd[3 * ray + 2];
  const float dist0 = d0[ray];
  float x0 = fadd(ro[3 * ray], fmul(e0, dist0)), x1 = fadd(ro[3 * ray + 1], fmul(e1, dist0));
  float x2 = fadd(ro[3 * ray + 2], fmul(e2, dist0));
  if (live && k < 3) trace[3 * ray + k] = k == 0 ? x0 : (k == 1 ? x1 : x2);
  float h = 0.f, c = 0.f;
  for (int s = 0; s < steps; ++s) {
    const Bilinear bl = bilinear_at(v, x0, x1, x2);
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
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
    if (live) {
      float* st = state + ((int64_t)s * n_rays + ray) * kMarchState;
      st[k] = h; st[kHid + k] = c;
      st[2 * kHid + k] = ig; st[3 * kHid + k] = fg; st[4 * kHid + k] = gg; st[5 * kHid + k] = og;
    }
    float sd = fmul(wo, h);
#pragma unroll
    for (int d = kHid / 2; d > 0; d >>= 1) sd = fadd(sd, __shfl_xor(sd, d, kHid));
    sd = fadd(sd, bo);
    x0 = fadd(x0, fmul(e0, sd));
    x1 = fadd(x1, fmul(e1, sd));
    x2 = fadd(x2, fmul(e2, sd));
    if (live && k < 3) trace[(int64_t)(s + 1) * n_rays * 3 + 3 * ray + k] = k == 0 ? x0 : (k == 1 ? x1 : x2);
  }
  if (live && k < 3) world[3 * ray + k] = k == 0 ? x0 : (k == 1 ? x1 : x2);
}

// Gradient accumulators of one workgroup: d W_hh (64 x 16), d bias (64; b_ih and b_hh alike), d w_out (16),
// d b_out (1).
constexpr int kMarchGrads = kGates * kHid + kGates + kHid + 1;
constexpr int kMarchRays = 256 / kHid;   // rays per workgroup

// Bit-deterministic backward (ABI 15): no floating-point atomics anywhere.
//  * raymarch_bwd_kernel runs the reverse recursion per ray and stores, per step and ray, the 64 gate-gradient
//    values dg and the lookup's 4 texels and weights (instead of scattering them), plus max |dg| over the finite
//    values (an unsigned max of the float bits: order-independent) and a flag for non-finite ones. The parameter
//    gradients are summed in a fixed order -- the 4 rays of a wave by two xor shuffles (commutative adds: every
//    lane ends with the same bits), the 4 waves of a workgroup in wave order through LDS, the workgroups in block
//    order by raymarch_grads_reduce_kernel.
//  * raymarch_table_scatter_kernel adds every contribution w_corner * dg to the table gradient as an int64 fixed-
//    point value under one power-of-two scale 2^s per launch, chosen from max |dg| and the number of contributions
//    so no sum can overflow. Integer addition is associative: the sums are the same bits in any atomic order.
//    Each contribution is the exact double product w * dg rounded once to the fixed-point grid (an error of at
//    most 2^(cbits - 62) of max |dg|, 2^-45 with the 2^17 contributions of a train.py step): far below fp32
//    resolution relative to the largest gradient, which is how the table gradient is consumed (W_ih's gradient
//    sums over every texel; the latent's is compared at that scale).
//  * raymarch_table_finish_kernel converts the sums to fp32 (ldexp(sum, -s), rounded once); an entry that a
//    non-finite dg reached is NaN (the reference's scatter would carry the NaN there too).
// Round 5 summed the table gradient in fp64 atomics instead: order-dependent at 2^-53, so one fp32 rounding in a
// great many could differ run to run, and one Adam step amplifies such a bit.
struct MarchCtl {
  unsigned max_bits;   // max |dg| over finite values, float bits
  unsigned bad;        // nonzero if some dg was NaN / inf
};

__global__ void __launch_bounds__(256) raymarch_bwd_kernel(MarchScenes sc, const float* __restrict__ tables,
                                                           int64_t table_stride, const float* __restrict__ w_hh,
                                                           const float* __restrict__ w_out,
                                                           const float* __restrict__ rd,
                                                           const float* __restrict__ trace,
                                                           const float* __restrict__ state,
                                                           const float* __restrict__ grad_world, int64_t n_per_scene,
                                                           int64_t n_rays, int steps, int pos_grad,
                                                           float* __restrict__ dg_rows, float* __restrict__ lk_rows,
                                                           MarchCtl* __restrict__ ctl,
                                                           float* __restrict__ grad_partials) {
  // W_hh^T dg per step: red (ray, unit k, column j); after the loop the same LDS holds the per-wave parameter
  // sums wsum (the loop's last barrier ends every read of red)
  static_assert(kMarchRays * kHid * (kHid + 1) <= 4 * kMarchGrads, "red fits the wsum area");
  __shared__ float smem[4 * kMarchGrads];
  float (*red)[kHid][kHid + 1] = reinterpret_cast<float (*)[kHid][kHid + 1]>(smem);
  float (*wsum)[kMarchGrads] = reinterpret_cast<float (*)[kMarchGrads]>(smem);
  const int k = threadIdx.x & (kHid - 1), rl = threadIdx.x / kHid;
  const int64_t ray_raw = (int64_t)blockIdx.x * kMarchRays + rl;
  const bool live = ray_raw < n_rays;
  const int64_t ray = live ? ray_raw : n_rays - 1;
  const int scene = (int)(ray / n_per_scene);
  const View& v = sc.v[scene];
  const float* table = tables + scene * table_stride;
  float wr[4][kHid];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < kHid; ++j) wr[q][j] = w_hh[(q * kHid + k) * kHid + j];
  const float wo = w_out[k];
  const float e0 = rd[3 * ray], e1 = rd[3 * ray + 1], e2 = rd[3 * ray + 2];
  float dx0 = live ? grad_world[3 * ray] : 0.f, dx1 = live ? grad_world[3 * ray + 1] : 0.f;
  float dx2 = live ? grad_world[3 * ray + 2] : 0.f;
  float dWhh[4][kHid], db[4] = {0.f, 0.f, 0.f, 0.f}, dwo = 0.f, dbo = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < kHid; ++j) dWhh[q][j] = 0.f;
  float dh_next = 0.f, dc_next = 0.f;
  float dg_max = 0.f;
  bool dg_bad = false;
  for (int s = steps - 1; s >= 0; --s) {
    const float* st = state + ((int64_t)s * n_rays + ray) * kMarchState;
    const float h = st[k], c = st[kHid + k];
    const float ig = st[2 * kHid + k], fg = st[3 * kHid + k], gg = st[4 * kHid + k], og = st[5 * kHid + k];
    const float c_prev = s > 0 ? state[((int64_t)(s - 1) * n_rays + ray) * kMarchState + kHid + k] : 0.f;
    const float h_prev = s > 0 ? state[((int64_t)(s - 1) * n_rays + ray) * kMarchState + k] : 0.f;
    // x_{s+1} = x_s + rd * sd_s;  sd_s = w_out . h_s + b_out
    const float dsd = e0 * dx0 + e1 * dx1 + e2 * dx2;
    dwo += dsd * h;
    dbo += dsd;
    float dh = wo * dsd + dh_next;
    // state[0].register_hook(clamp(-10, 10)); a NaN stays NaN, as torch.clamp keeps it (fminf / fmaxf alone
    // would turn it into -10 and hide it from the LSTM's gradients)
    dh = dh != dh ? dh : fminf(fmaxf(dh, -10.f), 10.f);
    const float tc = tanhf(c);
    const float dc = dh * og * (1.f - tc * tc) + dc_next;
    float dg[4];
    dg[0] = dc * gg * ig * (1.f - ig);                // i
    dg[1] = dc * c_prev * fg * (1.f - fg);            // f
    dg[2] = dc * ig * (1.f - gg * gg);                // g
    dg[3] = dh * tc * og * (1.f - og);                // o
    dc_next = dc * fg;
#pragma unroll
    for (int q = 0; q < 4; ++q) db[q] += dg[q];
    // W_hh^T dg -> dh of step s - 1 (unit j), and d W_hh += dg h_{s-1}^T
    float part[kHid];
#pragma unroll
    for (int j = 0; j < kHid; ++j) {
      const float hj = __shfl(h_prev, j, kHid);
      part[j] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        part[j] = fmaf(wr[q][j], dg[q], part[j]);
        dWhh[q][j] = fmaf(dg[q], hj, dWhh[q][j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kHid; ++j) red[rl][k][j] = part[j];
    // the lookup at x_s: its table gradient is scattered later (dg and the lookup stored), the position gradient
    // here
    const float* xs = trace + (int64_t)s * n_rays * 3 + 3 * ray;
    const LookupGrad L = lookup_grad(v, xs[0], xs[1], xs[2]);
    float gix = 0.f, giy = 0.f;
    const int64_t rs = (int64_t)s * n_rays + ray;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = q * kHid + k;
      const float tnw = table[(int64_t)L.bl.tex[0] * kGates + row], tne = table[(int64_t)L.bl.tex[1] * kGates + row];
      const float tsw = table[(int64_t)L.bl.tex[2] * kGates + row], tse = table[(int64_t)L.bl.tex[3] * kGates + row];
      gix += dg[q] * (L.wy0 * (tne - tnw) + L.wy1 * (tse - tsw));
      giy += dg[q] * (L.wx0 * (tsw - tnw) + L.wx1 * (tse - tne));
      if (live) {
        dg_rows[rs * kGates + row] = dg[q];
        const float a = fabsf(dg[q]);
        if (a <= 3.402823466e38f) dg_max = fmaxf(dg_max, a);   // finite (a NaN fails the compare)
        else dg_bad = true;
      }
    }
    if (live && k < 8) lk_rows[rs * 8 + k] = k < 4 ? __int_as_float(L.bl.tex[k]) : L.bl.w[k - 4];
#pragma unroll
    for (int d = kHid / 2; d > 0; d >>= 1) {
      gix += __shfl_xor(gix, d, kHid);
      giy += __shfl_xor(giy, d, kHid);
    }
    const float dxc0 = gix * L.dix[0] + giy * L.diy[0];
    const float dxc1 = gix * L.dix[1] + giy * L.diy[1];
    const float dxc2 = gix * L.dix[2] + giy * L.diy[2];
    // xc = R x + t: dx += R^T dxc (x_s feeds the lookup and, by identity, x_{s+1}); not with stop_encoder_grad,
    // whose detached latent cuts the lookup from the points (models.py:810-811)
    if (pos_grad) {
      dx0 += v.R[0] * dxc0 + v.R[3] * dxc1 + v.R[6] * dxc2;
      dx1 += v.R[1] * dxc0 + v.R[4] * dxc1 + v.R[7] * dxc2;
      dx2 += v.R[2] * dxc0 + v.R[5] * dxc1 + v.R[8] * dxc2;
    }
    __syncthreads();   // red written
    float acc = 0.f;
#pragma unroll
    for (int kk = 0; kk < kHid; ++kk) acc += red[rl][kk][k];
    dh_next = acc;
    __syncthreads();   // red read before the next step overwrites it
  }
  // max |dg| and the non-finite flag of the wave: one unsigned max / or per wave (order-independent)
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    dg_max = fmaxf(dg_max, __shfl_xor(dg_max, d));
    dg_bad = __shfl_xor((int)dg_bad, d) | (int)dg_bad;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&ctl->max_bits, __float_as_uint(dg_max));
    if (dg_bad) atomicOr(&ctl->bad, 1u);
  }
  // this workgroup's parameter gradients (dead rays contribute nothing), summed in a fixed order
  if (!live) {
    dwo = dbo = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      db[q] = 0.f;
#pragma unroll
      for (int j = 0; j < kHid; ++j) dWhh[q][j] = 0.f;
    }
  }
  const auto wave_sum = [](float x) {   // the wave's 4 rays (lanes 16 r + k), same bits on every lane
    x += __shfl_xor(x, 16);
    return x + __shfl_xor(x, 32);
  };
  const int wave = threadIdx.x >> 6;
  float* ws = wsum[wave];
  const bool writer = (threadIdx.x & 63) < kHid;   // ray 0 of the wave writes the wave's sums
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int j = 0; j < kHid; ++j) {
      const float t = wave_sum(dWhh[q][j]);
      if (writer) ws[(q * kHid + k) * kHid + j] = t;
    }
    const float t = wave_sum(db[q]);
    if (writer) ws[kGates * kHid + q * kHid + k] = t;
  }
  dwo = wave_sum(dwo);
  dbo = wave_sum(dbo);
  if (writer) ws[kGates * kHid + kGates + k] = dwo;
  if (writer && k == 0) ws[kGates * kHid + kGates + kHid] = dbo;
  __syncthreads();
  float* out = grad_partials + (int64_t)blockIdx.x * kMarchGrads;
  for (int i = threadIdx.x; i < kMarchGrads; i += blockDim.x)
    out[i] = ((wsum[0][i] + wsum[1][i]) + wsum[2][i]) + wsum[3][i];
}

// d_grads[i] = sum over the workgroups' partials in block order
__global__ void __launch_bounds__(256) raymarch_grads_reduce_kernel(const float* __restrict__ partials, int n_blocks,
                                                                    float* __restrict__ d_grads) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kMarchGrads) return;
  float s = 0.f;
  for (int b = 0; b < n_blocks; ++b) s += partials[(int64_t)b * kMarchGrads + i];
  d_grads[i] = s;
}

// The fixed-point exponent: every |w * dg| <= max |dg| < 2^e, so |w * dg * 2^s| < 2^(62 - cbits) and a sum of
// at most 2^cbits contributions stays below 2^62.
__device__ __forceinline__ int march_fixed_exp(const MarchCtl* ctl, int cbits) {
  const float m = __uint_as_float(ctl->max_bits);
  if (!(m > 0.f)) return 0;
  int e;
  frexpf(m, &e);   // m = f 2^e, f in [0.5, 1)
  return 62 - cbits - e;
}

// One wave per (step, ray): lane r adds w_c * dg[r] into the 4 corner texels' row r (64 consecutive int64 per
// corner: coalesced atomics).
__global__ void __launch_bounds__(256) raymarch_table_scatter_kernel(const float* __restrict__ dg_rows,
                                                                     const float* __restrict__ lk_rows,
                                                                     const MarchCtl* __restrict__ ctl,
                                                                     int64_t n_rays, int64_t n_per_scene,
                                                                     int64_t table_stride, int64_t n_rs, int cbits,
                                                                     unsigned long long* __restrict__ acc,
                                                                     float* __restrict__ d_tables) {
  const int64_t rs = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (rs >= n_rs) return;
  const int r = threadIdx.x & 63;
  const int64_t ray = rs % n_rays;
  const int64_t base = (ray / n_per_scene) * table_stride;
  const int sc = march_fixed_exp(ctl, cbits);
  const float g = dg_rows[rs * kGates + r];
  const bool finite = fabsf(g) <= 3.402823466e38f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int tex = __float_as_int(lk_rows[rs * 8 + c]);
    const float w = lk_rows[rs * 8 + 4 + c];
    const int64_t i = base + (int64_t)tex * kGates + r;
    if (finite) {
      const double prod = (double)w * (double)g;                 // exact (two fp32 factors)
      const long long q = (long long)rint(ldexp(prod, sc));     // one rounding onto the fixed-point grid
      if (q != 0) atomicAdd(acc + i, (unsigned long long)q);    // two's complement: signed sums
    } else {
      d_tables[i] = __int_as_float(0x7fc00000);                 // NaN marker (every writer stores the same bits)
    }
  }
}

__global__ void __launch_bounds__(256) raymarch_table_finish_kernel(const unsigned long long* __restrict__ acc,
                                                                    const MarchCtl* __restrict__ ctl, int64_t n,
                                                                    int cbits, float* __restrict__ d_tables) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int sc = march_fixed_exp(ctl, cbits);
  const bool bad = ctl->bad != 0u;
  if (bad && d_tables[i] != d_tables[i]) return;               // a non-finite contribution reached this entry
  d_tables[i] = (float)ldexp((double)(long long)acc[i], -sc);
}

}  // namespace avr

using namespace avr;

static int march_scenes(const avr_view_desc* views, int n_scenes, MarchScenes* sc, const char* what) {
  AVR_REQUIRE(views && n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES, "%s: 1..%d scenes", what, AVR_MAX_SCENES);
  for (int s = 0; s < n_scenes; ++s) {
    AVR_REQUIRE(views[s].latent_h == views[0].latent_h && views[s].latent_w == views[0].latent_w &&
                    views[s].latent_h > 0 && views[s].latent_w > 0,
                "%s: scenes need latent maps of one (positive) size", what);
    view_from_desc(&views[s], &sc->v[s]);
  }
  return AVR_OK;
}

extern "C" int avr_raymarch_train(const avr_view_desc* views, int n_scenes, const float* gate_tables,
                                  const float* w_hh, const float* b_ih, const float* b_hh, const float* w_out,
                                  const float* b_out, const float* ro, const float* rd, const float* init_dist,
                                  int64_t n_per_scene, int steps, float* world, float* trace, float* state,
                                  void* stream) {
  AVR_REQUIRE(n_per_scene >= 0 && steps >= 0, "avr_raymarch_train: negative size");
  if (n_per_scene == 0) return AVR_OK;
  MarchScenes sc;
  int rc = march_scenes(views, n_scenes, &sc, "avr_raymarch_train");
  if (rc) return rc;
  AVR_REQUIRE(gate_tables && w_hh && b_ih && b_hh && w_out && b_out && ro && rd && init_dist && world && trace &&
                  (state || steps == 0),
              "avr_raymarch_train: null pointer");
  const int64_t n = n_per_scene * n_scenes;
  const int64_t stride = (int64_t)views[0].latent_h * views[0].latent_w * kGates;
  const int per_block = 256 / kHid;
  raymarch_train_kernel<<<(unsigned)((n + per_block - 1) / per_block), 256, 0, as_stream(stream)>>>(
      sc, gate_tables, stride, w_hh, b_ih, b_hh, w_out, b_out, ro, rd, init_dist, n_per_scene, n, steps, world,
      trace, state);
  return check_launch("raymarch_train_kernel");
}

// scratch regions of avr_raymarch_bwd, 256-B aligned: the int64 table accumulators, dg rows, lookup rows,
// the workgroups' parameter partials, the control words
struct MarchScratch {
  int64_t acc, dg, lk, partials, ctl, total;
};

static MarchScratch march_scratch(int64_t n_rays, int steps, int64_t table_entries) {
  const auto up = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  MarchScratch m;
  m.acc = 0;
  m.dg = m.acc + up(table_entries * 8);
  m.lk = m.dg + up((int64_t)steps * n_rays * kGates * 4);
  m.partials = m.lk + up((int64_t)steps * n_rays * 8 * 4);
  m.ctl = m.partials + up(((n_rays + kMarchRays - 1) / kMarchRays) * kMarchGrads * 4);
  m.total = m.ctl + up(sizeof(MarchCtl));
  return m;
}

extern "C" int avr_raymarch_bwd_scratch_bytes(int64_t n_rays, int steps, int64_t table_entries, int64_t* n_bytes) {
  AVR_REQUIRE(n_rays >= 0 && steps >= 0 && table_entries >= 0 && n_bytes,
              "avr_raymarch_bwd_scratch_bytes: bad arguments");
  *n_bytes = march_scratch(n_rays, steps, table_entries).total;
  return AVR_OK;
}

extern "C" int avr_raymarch_bwd(const avr_view_desc* views, int n_scenes, const float* gate_tables,
                                const float* w_hh, const float* w_out, const float* rd, const float* trace,
                                const float* state, const float* grad_world, int64_t n_per_scene, int steps,
                                int lookup_grad, float* d_tables, float* d_grads, void* scratch,
                                int64_t scratch_bytes, void* stream) {
  AVR_REQUIRE(n_per_scene >= 0 && steps >= 0, "avr_raymarch_bwd: negative size");
  if (n_per_scene == 0 || steps == 0) {   // nothing marched: every gradient is zero (written whole, as below)
    hipStream_t s = as_stream(stream);
    bool ok = !d_grads || hipMemsetAsync(d_grads, 0, kMarchGrads * sizeof(float), s) == hipSuccess;
    if (d_tables && views && n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES)
      ok = ok && hipMemsetAsync(d_tables, 0, (size_t)views[0].latent_h * views[0].latent_w * kGates * n_scenes *
                                                 sizeof(float), s) == hipSuccess;
    return ok ? AVR_OK : fail(AVR_E_HIP, "avr_raymarch_bwd: memset");
  }
  MarchScenes sc;
  int rc = march_scenes(views, n_scenes, &sc, "avr_raymarch_bwd");
  if (rc) return rc;
  AVR_REQUIRE(gate_tables && w_hh && w_out && rd && trace && state && grad_world && d_tables && d_grads && scratch,
              "avr_raymarch_bwd: null pointer");
  const int64_t n = n_per_scene * n_scenes;
  const int64_t stride = (int64_t)views[0].latent_h * views[0].latent_w * kGates;
  const int64_t entries = stride * n_scenes;
  const int64_t blocks = (n + kMarchRays - 1) / kMarchRays;
  const int64_t n_rs = (int64_t)steps * n;
  AVR_REQUIRE(blocks < (1ll << 31) && (n_rs + 3) / 4 < (1ll << 31), "avr_raymarch_bwd: too many rays");
  // every table entry receives at most n_rs * 4 contributions (4 corners per lookup)
  int cbits = 0;
  while (cbits < 40 && (1ll << cbits) < n_rs * 4) ++cbits;
  AVR_REQUIRE(cbits <= 30, "avr_raymarch_bwd: too many ray steps for the fixed-point sums");
  const MarchScratch m = march_scratch(n, steps, entries);
  AVR_REQUIRE(scratch_bytes >= m.total, "avr_raymarch_bwd: scratch of %lld bytes < %lld",
              (long long)scratch_bytes, (long long)m.total);
  char* sb = static_cast<char*>(scratch);
  auto* acc = reinterpret_cast<unsigned long long*>(sb + m.acc);
  auto* dg_rows = reinterpret_cast<float*>(sb + m.dg);
  auto* lk_rows = reinterpret_cast<float*>(sb + m.lk);
  auto* partials = reinterpret_cast<float*>(sb + m.partials);
  auto* ctl = reinterpret_cast<MarchCtl*>(sb + m.ctl);
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(acc, 0, (size_t)entries * 8, s) != hipSuccess ||
      hipMemsetAsync(ctl, 0, sizeof(MarchCtl), s) != hipSuccess ||
      hipMemsetAsync(d_tables, 0, (size_t)entries * 4, s) != hipSuccess)
    return fail(AVR_E_HIP, "avr_raymarch_bwd: memset");
  raymarch_bwd_kernel<<<(unsigned)blocks, 256, 0, s>>>(sc, gate_tables, stride, w_hh, w_out, rd, trace, state,
                                                       grad_world, n_per_scene, n, steps, lookup_grad ? 1 : 0,
                                                       dg_rows, lk_rows, ctl, partials);
  rc = check_launch("raymarch_bwd_kernel");
  if (rc) return rc;
  raymarch_grads_reduce_kernel<<<(kMarchGrads + 255) / 256, 256, 0, s>>>(partials, (int)blocks, d_grads);
  rc = check_launch("raymarch_grads_reduce_kernel");
  if (rc) return rc;
  raymarch_table_scatter_kernel<<<(unsigned)((n_rs + 3) / 4), 256, 0, s>>>(dg_rows, lk_rows, ctl, n, n_per_scene,
                                                                            stride, n_rs, cbits, acc, d_tables);
  rc = check_launch("raymarch_table_scatter_kernel");
  if (rc) return rc;
  raymarch_table_finish_kernel<<<(unsigned)((entries + 255) / 256), 256, 0, s>>>(acc, ctl, entries, cbits, d_tables);
  return check_launch("raymarch_table_finish_kernel");
}

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
