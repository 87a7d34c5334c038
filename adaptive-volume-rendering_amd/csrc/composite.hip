// Alpha compositing with cumulative transmittance — volume_integral,
// renderers.py:69-119, and its gradient w.r.t. (rgb, sigma).
//
// One wave64 per ray, samples dealt round-robin (sample n -> lane n % 64,
// round n / 64) so every field/z load is a coalesced 1 KiB / 256 B wave
// access. The exclusive product T_n = prod_{m<n} (1 - a_m + 1e-10) is a wave
// scan in fp64 with a carry between rounds (the reference's ATen cumprod also
// accumulates in fp64) and is rounded to fp32 before w = a * T, exactly as the
// reference does. The white-background sum uses the torch-CPU cascade order.
#include "avr_common.h"

namespace avr {

constexpr int kCompWaves = 4;

__device__ float cascade_sum_wave_c(const float* x, int N, int lane, float* scratch) {
  const int nvec = N >> 3, ngrp = nvec >> 2;
  if (lane < 32) {
    float p = 0.f;
    for (int i = 0; i < ngrp; ++i) p = fadd(p, x[32 * i + lane]);
    scratch[lane] = p;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane < 8) {
    float a0 = scratch[lane];
    for (int v = ngrp * 4; v < nvec; ++v) a0 = fadd(a0, x[8 * v + lane]);
    scratch[32 + lane] = fadd(fadd(fadd(a0, scratch[8 + lane]), scratch[16 + lane]), scratch[24 + lane]);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane == 0) {
    float s = 0.f;
    for (int k = nvec * 8; k < N; ++k) s = fadd(s, x[k]);
    for (int l = 0; l < 8; ++l) s = fadd(s, scratch[32 + l]);
    scratch[40] = s;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return scratch[40];
}

struct SampleTerms {
  float d, e, alpha, t, zz;
};

__device__ __forceinline__ SampleTerms sample_terms(const float* __restrict__ zr, int n, int N, float sigma,
                                                    float infinity) {
  SampleTerms s;
  const float z0 = zr[n];
  const bool last = (n == N - 1);
  const float z1 = last ? 0.f : zr[n + 1];
  s.d = last ? 1e10f : fsub(z1, z0);
  s.zz = last ? infinity : z1;
  s.e = expf(-fmul(sigma, s.d));
  s.alpha = fsub(1.0f, s.e);
  s.t = fadd(fsub(1.0f, s.alpha), 1e-10f);
  return s;
}

// Forward: lane l owns the K consecutive samples [K l, K l + K) of its ray
// (K = ceil(N / 64)), so the transmittance needs ONE wave scan: a sequential
// fp64 product over the lane's own samples, a DPP exclusive product scan of
// the lane totals, and the lane-local expansion. rgb / dist are fp64 lane sums
// reduced by a DPP scan; the white-background sum reads w back from LDS in the
// torch-CPU cascade order. No block barriers: every ray is one wave.
template <int K>
__global__ void __launch_bounds__(256) composite_fwd_kernel(const float* __restrict__ z,
                                                            const float4* __restrict__ field, int64_t n_rays, int N,
                                                            int white_back, float infinity, float* __restrict__ rgb,
                                                            float* __restrict__ dist, float* __restrict__ w_out,
                                                            const float* __restrict__ ro,
                                                            const float* __restrict__ rd,
                                                            const double* __restrict__ depth_row,
                                                            float* __restrict__ depth) {
  extern __shared__ float smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ray = (int64_t)blockIdx.x * kCompWaves + wid;
  if (ray >= n_rays) return;  // wave-uniform; no block barriers below
  float* wbuf = smem + wid * (N + 64);
  float* scratch = wbuf + N;
  const float* zr = z + ray * N;
  const float4* fr = field + ray * N;
  const int n0 = K * lane;
  // depth epilogue inputs, loaded up front so their latency hides under the ray's work
  double4 drow = make_double4(0.0, 0.0, 0.0, 0.0);
  float o3[3] = {0.f, 0.f, 0.f}, d3[3] = {0.f, 0.f, 0.f};
  if (depth && lane == 0) {
    drow = reinterpret_cast<const double4*>(depth_row)[ray];
#pragma unroll
    for (int q = 0; q < 3; ++q) { o3[q] = ro[3 * ray + q]; d3[q] = rd[3 * ray + q]; }
  }
  float4 f[K];
  float zv[K + 1];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int n = n0 + k;
    f[k] = n < N ? fr[n] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k <= K; ++k) zv[k] = n0 + k < N ? zr[n0 + k] : 0.f;
  float alpha[K], zz[K];
  double P[K + 1];     // P[k] = prod of t over the lane's samples before k (sequential fp64)
  P[0] = 1.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int n = n0 + k;
    const bool ok = n < N;
    const bool last = (n == N - 1);
    const float d = last ? 1e10f : fsub(zv[k + 1], zv[k]);
    zz[k] = last ? infinity : zv[k + 1];
    const float e = expf(-fmul(f[k].w, d));
    alpha[k] = ok ? fsub(1.0f, e) : 0.f;
    const float t = ok ? fadd(fsub(1.0f, alpha[k]), 1e-10f) : 1.f;
    P[k + 1] = P[k] * (double)t;
  }
  double total;
  const double excl = wave_excl_prod_dpp(P[K], total);
  double r = 0.0, g = 0.0, b = 0.0, dd = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int n = n0 + k;
    const float T = (float)(excl * P[k]);
    const float w = fmul(alpha[k], T);
    if (n < N) {
      wbuf[n] = w;
      if (w_out) w_out[ray * N + n] = w;
      r += (double)w * f[k].x;
      g += (double)w * f[k].y;
      b += (double)w * f[k].z;
      dd += (double)w * zz[k];
    }
  }
  r = wave_total_sum_dpp(r);
  g = wave_total_sum_dpp(g);
  b = wave_total_sum_dpp(b);
  dd = wave_total_sum_dpp(dd);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  float acc = 0.f;
  if (white_back) acc = cascade_sum_wave_c(wbuf, N, lane, scratch);
  if (lane == 0) {
    float cr = (float)r, cg = (float)g, cb = (float)b;
    if (white_back) {
      const float bg = fsub(1.0f, acc);
      cr = fadd(cr, bg);
      cg = fadd(cg, bg);
      cb = fadd(cb, bg);
    }
    rgb[3 * ray] = cr;
    rgb[3 * ray + 1] = cg;
    rgb[3 * ray + 2] = cb;
    const float dist_f = (float)dd;
    dist[ray] = dist_f;
    if (depth) {   // depth_from_world(ro + rd * dist, cam2world), utils.py:358-361, as depth_kernel computes it
      double zc = drow.w;
      zc += drow.x * (double)fadd(o3[0], fmul(d3[0], dist_f));
      zc += drow.y * (double)fadd(o3[1], fmul(d3[1], dist_f));
      zc += drow.z * (double)fadd(o3[2], fmul(d3[2], dist_f));
      depth[ray] = (float)(-zc);
    }
  }
}

// dL/d(rgb_n) = G * w_n
// g_w_n  = G.c_n + Gd * zz_n + gw_n - wb * sum(G)
// S_n    = sum_{m>n} g_w_m w_m
// dL/da_n = g_w_n T_n - S_n / t_n           (cumprod backward, no zero inputs: t >= 1e-10)
// dL/dsigma_n = dL/da_n * exp(-sigma_n d_n) * d_n
// z (AdaptiveVolumeRenderer trains its band through it): d_n = z_{n+1} - z_n
// (n < N-1), zz_n = z_{n+1}; with gd_n = dL/da_n * exp(-sigma_n d_n) * sigma_n,
// dL/dz_m = [m >= 1] (gd_{m-1} + Gd w_{m-1}) - [m <= N-2] gd_m.
__global__ void __launch_bounds__(256) composite_bwd_kernel(const float* __restrict__ z,
                                                            const float4* __restrict__ field, int64_t n_rays, int N,
                                                            int white_back, float infinity,
                                                            const float* __restrict__ grad_rgb,
                                                            const float* __restrict__ grad_dist,
                                                            const float* __restrict__ grad_w,
                                                            float4* __restrict__ grad_field,
                                                            float* __restrict__ grad_z) {
  extern __shared__ double dsm[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ray = (int64_t)blockIdx.x * kCompWaves + wid;
  if (ray >= n_rays) return;
  double* qpre = dsm + (size_t)wid * N * 2;  // inclusive prefix of q = g_w * w
  float* Tbuf = reinterpret_cast<float*>(qpre + N);
  const float* zr = z + ray * N;
  const float4* fr = field + ray * N;
  const float G0 = grad_rgb[3 * ray], G1 = grad_rgb[3 * ray + 1], G2 = grad_rgb[3 * ray + 2];
  const float Gd = grad_dist ? grad_dist[ray] : 0.f;
  const float Gbg = white_back ? fadd(fadd(G0, G1), G2) : 0.f;
  double carryT = 1.0, carryQ = 0.0;
  for (int base = 0; base < N; base += 64) {
    const int n = base + lane;
    const bool ok = n < N;
    float4 f = ok ? fr[n] : make_float4(0.f, 0.f, 0.f, 0.f);
    SampleTerms s = ok ? sample_terms(zr, n, N, f.w, infinity) : SampleTerms{0.f, 1.f, 0.f, 1.f, 0.f};
    const double incl = wave_incl_scan_mul((double)s.t, lane) * carryT;
    double excl = __shfl_up(incl, 1, 64);
    if (lane == 0) excl = carryT;
    carryT = __shfl(incl, 63, 64);
    const float T = (float)excl;
    const float w = fmul(s.alpha, T);
    double gw = (double)G0 * f.x + (double)G1 * f.y + (double)G2 * f.z + (double)Gd * s.zz - (double)Gbg;
    if (grad_w && ok) gw += (double)grad_w[ray * N + n];
    const double q = ok ? gw * (double)w : 0.0;
    const double qi = wave_incl_scan_add(q, lane) + carryQ;
    carryQ = __shfl(qi, 63, 64);
    if (ok) {
      qpre[n] = qi;
      Tbuf[n] = T;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const double Q = carryQ;
  double carryZ = 0.0;   // gd + Gd w of the previous round's last sample
  for (int base = 0; base < N; base += 64) {
    const int n = base + lane;
    const bool ok = n < N;
    double vz = 0.0, gd = 0.0;
    if (ok) {
      const float4 f = fr[n];
      const SampleTerms s = sample_terms(zr, n, N, f.w, infinity);
      const float T = Tbuf[n];
      const float w = fmul(s.alpha, T);
      const double gw = (double)G0 * f.x + (double)G1 * f.y + (double)G2 * f.z + (double)Gd * s.zz - (double)Gbg +
                        (grad_w ? (double)grad_w[ray * N + n] : 0.0);
      const double S = Q - qpre[n];
      const double ga = gw * (double)T - S / (double)s.t;
      const double gs = ga * (double)s.e * (double)s.d;
      grad_field[ray * N + n] = make_float4(fmul(G0, w), fmul(G1, w), fmul(G2, w), (float)gs);
      if (n < N - 1) gd = ga * (double)s.e * (double)f.w;
      vz = gd + (n < N - 1 ? (double)Gd * w : 0.0);
    }
    if (grad_z) {   // wave-uniform
      double prev = __shfl_up(vz, 1, 64);
      if (lane == 0) prev = carryZ;
      carryZ = __shfl(vz, 63, 64);
      if (ok) grad_z[ray * N + n] = (float)((n >= 1 ? prev : 0.0) - gd);
    }
  }
}

}  // namespace avr

using namespace avr;

static int composite_fwd(const float* z, const float* field, int64_t n_rays, int n_samples, int white_back,
                         float infinity, float* rgb, float* dist, float* weights, const float* ro, const float* rd,
                         const double* depth_row, float* depth, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples <= 1024, "avr_composite_fwd: n_samples must be in [1,1024]");
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(z && field && rgb && dist, "avr_composite_fwd: null pointer");
  AVR_REQUIRE(!depth || (ro && rd && depth_row), "avr_composite_fwd_depth: null ro / rd / depth_row");
  const size_t shm = (size_t)kCompWaves * (n_samples + 64) * sizeof(float);
  const unsigned grid = (unsigned)((n_rays + kCompWaves - 1) / kCompWaves);
  const float4* f4 = reinterpret_cast<const float4*>(field);
  hipStream_t st = as_stream(stream);
#define AVR_COMP_K(KK)                                                                                          \
  case KK:                                                                                                      \
    composite_fwd_kernel<KK><<<grid, 64 * kCompWaves, shm, st>>>(z, f4, n_rays, n_samples, white_back, infinity, \
                                                                 rgb, dist, weights, ro, rd, depth_row, depth); \
    break;
  switch ((n_samples + 63) / 64) {
    AVR_COMP_K(1) AVR_COMP_K(2) AVR_COMP_K(3) AVR_COMP_K(4) AVR_COMP_K(5) AVR_COMP_K(6) AVR_COMP_K(7) AVR_COMP_K(8)
    AVR_COMP_K(9) AVR_COMP_K(10) AVR_COMP_K(11) AVR_COMP_K(12) AVR_COMP_K(13) AVR_COMP_K(14) AVR_COMP_K(15)
    AVR_COMP_K(16)
  }
#undef AVR_COMP_K
  return check_launch("composite_fwd_kernel");
}

extern "C" int avr_composite_fwd(const float* z, const float* field, int64_t n_rays, int n_samples, int white_back,
                                 float infinity, float* rgb, float* dist, float* weights, void* stream) {
  return composite_fwd(z, field, n_rays, n_samples, white_back, infinity, rgb, dist, weights, nullptr, nullptr,
                       nullptr, nullptr, stream);
}

extern "C" int avr_composite_fwd_depth(const float* z, const float* field, int64_t n_rays, int n_samples,
                                       int white_back, float infinity, const float* ro, const float* rd,
                                       const double* depth_row, float* rgb, float* dist, float* weights, float* depth,
                                       void* stream) {
  AVR_REQUIRE(n_rays == 0 || depth, "avr_composite_fwd_depth: null depth");
  return composite_fwd(z, field, n_rays, n_samples, white_back, infinity, rgb, dist, weights, ro, rd, depth_row,
                       depth, stream);
}

extern "C" int avr_composite_bwd(const float* z, const float* field, int64_t n_rays, int n_samples, int white_back,
                                 float infinity, const float* grad_rgb, const float* grad_dist,
                                 const float* grad_weights, float* grad_field, float* grad_z, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples <= 1024, "avr_composite_bwd: n_samples must be in [1,1024]");
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(z && field && grad_rgb && grad_field, "avr_composite_bwd: null pointer");
  const size_t shm = (size_t)kCompWaves * n_samples * (sizeof(double) + sizeof(double));
  const unsigned grid = (unsigned)((n_rays + kCompWaves - 1) / kCompWaves);
  composite_bwd_kernel<<<grid, 64 * kCompWaves, shm, as_stream(stream)>>>(
      z, reinterpret_cast<const float4*>(field), n_rays, n_samples, white_back, infinity, grad_rgb, grad_dist,
      grad_weights, reinterpret_cast<float4*>(grad_field), grad_z);
  return check_launch("composite_bwd_kernel");
}
