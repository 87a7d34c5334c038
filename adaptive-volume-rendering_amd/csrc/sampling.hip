// Stratified (coarse) and inverse-CDF (fine) sampling.
//   sample_coarse renderers.py:4-24
//   sample_fine   renderers.py:27-54   (+ sample_depth :56-66, clamp :255,
//                                        sort(cat(...)) :257-258)
//
// sample_fine runs one wave64 per ray with the ray's state in LDS:
//   w' = w + 1e-5, s = torch-CPU cascade sum (8 lanes x ILP 4, bit-exact),
//   pdf = w'/s (IEEE), cdf = [0, fp64 prefix sum] (wave scan; the fp64 partial
//   sums of these fp32 terms are exact, so the scan order cannot change a bit),
//   idx = #{cdf <= u} - 1 by binary search, z = near + (far-near)*((idx+u2)/Nc),
//   then a bitonic sort of [z_coarse | z_fine | z_depth] padded to 2^k with +inf.
#include <float.h>

#include "avr_common.h"

namespace avr {

constexpr uint32_t kStreamCoarse = 0x1001u, kStreamU = 0x2002u, kStreamU2 = 0x3003u, kStreamDepth = 0x4004u;

__global__ void __launch_bounds__(256) sample_coarse_kernel(float near_, float far_, int64_t n_rays, int n,
                                                            const float* __restrict__ noise, uint64_t seed,
                                                            uint64_t offset, float* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rays * n) return;
  const int64_t r = i / n;
  const int s = (int)(i - r * n);
  const float span = fsub(far_, near_);
  const float step = fdiv((float)s, (float)n);
  const float u = noise ? noise[i] : philox_uniform(seed, offset + (uint64_t)r, (uint32_t)s, kStreamCoarse);
  // z = (near + span*step) + (u*span)/n   (two separate einsums, renderers.py:13-14)
  z[i] = fadd(fadd(near_, fmul(span, step)), fdiv(fmul(u, span), (float)n));
}

// sample_coarse with per-ray bounds (AdaptiveVolumeRenderer's band around the
// raymarched distance, renderers.py:492-493: near = d - eps, far = d + eps).
__global__ void __launch_bounds__(256) sample_coarse_rays_kernel(const float* __restrict__ near_,
                                                                 const float* __restrict__ far_, int64_t n_rays,
                                                                 int n, const float* __restrict__ noise,
                                                                 uint64_t seed, uint64_t offset,
                                                                 float* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rays * n) return;
  const int64_t r = i / n;
  const int s = (int)(i - r * n);
  const float nr = near_[r];
  const float span = fsub(far_[r], nr);
  const float step = fdiv((float)s, (float)n);
  const float u = noise ? noise[i] : philox_uniform(seed, offset + (uint64_t)r, (uint32_t)s, kStreamCoarse);
  z[i] = fadd(fadd(nr, fmul(span, step)), fdiv(fmul(u, span), (float)n));
}

// torch-CPU fp32 row sum (ATen vectorised reduction): four 8-lane accumulators
// over full groups of four 8-vectors, leftover vectors into accumulator 0,
// ((a0+a1)+a2)+a3, then the scalar tail, then the 8 lanes in order.
// `x` is the ray's row in LDS; computed by lanes 0..31 then lane 0.
__device__ float cascade_sum_wave(const float* x, int N, int lane, float* scratch) {
  const int nvec = N >> 3;
  const int ngrp = nvec >> 2;          // full groups of 4 vectors
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
    const float a = fadd(fadd(fadd(a0, scratch[8 + lane]), scratch[16 + lane]), scratch[24 + lane]);
    scratch[32 + lane] = a;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  float s = 0.f;
  if (lane == 0) {
    for (int k = nvec * 8; k < N; ++k) s = fadd(s, x[k]);
    for (int l = 0; l < 8; ++l) s = fadd(s, scratch[32 + l]);
    scratch[40] = s;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return scratch[40];
}

// Per-wave LDS: cdf[kMaxCoarse+1] | scratch[64] | sort buffer[kMaxSort]
constexpr int kMaxCoarse = 256;
constexpr int kMaxSort = 512;
constexpr int kFineWaves = 4;
constexpr int kWaveLds = (kMaxCoarse + 1 + 64 + kMaxSort);

__global__ void __launch_bounds__(256) sample_fine_kernel(
    const float* __restrict__ weights, const float* __restrict__ z_coarse, float near_, float far_, int64_t n_rays,
    int Nc, int Nf, int Nd, float depth_std, const float* __restrict__ u_in, const float* __restrict__ u2_in,
    const float* __restrict__ nd_in, uint64_t seed, uint64_t offset, int sort_n, float* __restrict__ z_sorted,
    int32_t* __restrict__ idx_out, float* __restrict__ z_fine_out) {
  __shared__ float lds[kFineWaves * kWaveLds];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ray = (int64_t)blockIdx.x * kFineWaves + wid;
  const bool active = ray < n_rays;  // wave-uniform
  float* cdf = lds + wid * kWaveLds;   // [0 .. Nc]
  float* scratch = cdf + kMaxCoarse + 1;
  float* sbuf = scratch + 64;
  const int Ntot = Nc + Nf + Nd;
  const float span = fsub(far_, near_);

  if (active) {
    // 1) w' = w + 1e-5 into cdf[1..Nc] (temporarily), cascade sum.
    const float* w = weights + ray * Nc;
    for (int k = lane; k < Nc; k += 64) cdf[1 + k] = fadd(w[k], 1e-5f);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const float s = cascade_sum_wave(cdf + 1, Nc, lane, scratch);
    // 2) pdf and fp64 inclusive prefix sum -> cdf[1..Nc], cdf[0] = 0.
    double carry = 0.0;
    for (int base = 0; base < Nc; base += 64) {
      const int k = base + lane;
      const double p = (k < Nc) ? (double)fdiv(cdf[1 + k], s) : 0.0;
      const double incl = wave_incl_scan_add(p, lane) + carry;
      carry = __shfl(incl, 63, 64);
      if (k < Nc) cdf[1 + k] = (float)incl;
    }
    if (lane == 0) cdf[0] = 0.f;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  __syncthreads();
  if (active) {
    // 3) importance samples: idx = upper_bound(cdf[0..Nc], u) - 1, clamped >= 0
    const float* zc = z_coarse + ray * Nc;
    for (int f = lane; f < Nf; f += 64) {
      const float u = u_in ? u_in[ray * Nf + f] : philox_uniform(seed, offset + (uint64_t)ray, f, kStreamU);
      const float u2 = u2_in ? u2_in[ray * Nf + f] : philox_uniform(seed, offset + (uint64_t)ray, f, kStreamU2);
      int lo = 0, hi = Nc + 1;  // count of cdf entries <= u
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
      }
      const int idx = lo > 0 ? lo - 1 : 0;
      const float steps = fdiv(fadd((float)idx, u2), (float)Nc);
      const float zf = fadd(near_, fmul(span, steps));
      if (idx_out) idx_out[ray * Nf + f] = idx;
      if (z_fine_out) z_fine_out[ray * Nf + f] = zf;
      sbuf[Nc + f] = zf;
    }
    for (int k = lane; k < Nc; k += 64) sbuf[k] = zc[k];
    // 4) depth samples: clamp(randn * std, near, far)  (quirk Q6)
    for (int d = lane; d < Nd; d += 64) {
      const float n = nd_in ? nd_in[ray * Nd + d] : philox_normal(seed, offset + (uint64_t)ray, d, kStreamDepth);
      sbuf[Nc + Nf + d] = fminf(fmaxf(fmul(n, depth_std), near_), far_);
    }
    for (int k = Ntot + lane; k < sort_n; k += 64) sbuf[k] = FLT_MAX;
  }
  __syncthreads();
  // 5) bitonic sort of sbuf[0..sort_n) ascending (sort_n power of two <= 512)
  for (int size = 2; size <= sort_n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (active) {
        for (int t = lane; t < (sort_n >> 1); t += 64) {
          const int i = 2 * t - (t & (stride - 1));
          const int j = i + stride;
          const float a = sbuf[i], b = sbuf[j];
          const bool up = ((i & size) == 0);
          if ((a > b) == up) { sbuf[i] = b; sbuf[j] = a; }
        }
      }
      __syncthreads();
    }
  }
  if (active) {
    float* out = z_sorted + ray * Ntot;
    for (int k = lane; k < Ntot; k += 64) out[k] = sbuf[k];
  }
}

}  // namespace avr

using namespace avr;

extern "C" int avr_sample_coarse(float near_, float far_, int64_t n_rays, int n_samples, const float* noise,
                                 uint64_t seed, uint64_t offset, float* z, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0, "avr_sample_coarse: bad sizes");
  const int64_t n = n_rays * n_samples;
  if (n == 0) return AVR_OK;
  AVR_REQUIRE(z, "avr_sample_coarse: null output");
  sample_coarse_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(near_, far_, n_rays, n_samples,
                                                                                 noise, seed, offset, z);
  return check_launch("sample_coarse_kernel");
}

extern "C" int avr_sample_coarse_rays(const float* near_, const float* far_, int64_t n_rays, int n_samples,
                                      const float* noise, uint64_t seed, uint64_t offset, float* z, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0, "avr_sample_coarse_rays: bad sizes");
  const int64_t n = n_rays * n_samples;
  if (n == 0) return AVR_OK;
  AVR_REQUIRE(near_ && far_ && z, "avr_sample_coarse_rays: null pointer");
  sample_coarse_rays_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(near_, far_, n_rays,
                                                                                       n_samples, noise, seed,
                                                                                       offset, z);
  return check_launch("sample_coarse_rays_kernel");
}

extern "C" int avr_sample_fine(const float* weights, const float* z_coarse, float near_, float far_, int64_t n_rays,
                               int n_coarse, int n_importance, int n_depth, float depth_std, const float* u,
                               const float* u2, const float* noise_depth, uint64_t seed, uint64_t offset,
                               float* z_sorted, int32_t* idx, float* z_fine, void* stream) {
  AVR_REQUIRE(n_rays >= 0, "avr_sample_fine: negative n_rays");
  AVR_REQUIRE(n_rays == 0 || (weights && z_coarse && z_sorted), "avr_sample_fine: null pointer");
  AVR_REQUIRE(n_coarse > 0 && n_coarse <= kMaxCoarse, "avr_sample_fine: n_coarse must be in [1, %d]", kMaxCoarse);
  AVR_REQUIRE(n_importance >= 0 && n_depth >= 0, "avr_sample_fine: negative sample count");
  const int ntot = n_coarse + n_importance + n_depth;
  AVR_REQUIRE(ntot <= kMaxSort, "avr_sample_fine: total samples %d > %d", ntot, kMaxSort);
  const bool explicit_noise = (u != nullptr);
  AVR_REQUIRE(explicit_noise == (u2 != nullptr) && (n_depth == 0 || explicit_noise == (noise_depth != nullptr)),
              "avr_sample_fine: u, u2, noise_depth must be all given or all NULL");
  if (n_rays == 0) return AVR_OK;
  int sort_n = 2;
  while (sort_n < ntot) sort_n <<= 1;
  const unsigned grid = (unsigned)((n_rays + kFineWaves - 1) / kFineWaves);
  sample_fine_kernel<<<grid, 64 * kFineWaves, 0, as_stream(stream)>>>(
      weights, z_coarse, near_, far_, n_rays, n_coarse, n_importance, n_depth, depth_std, u, u2, noise_depth, seed,
      offset, sort_n, z_sorted, idx, z_fine);
  return check_launch("sample_fine_kernel");
}
