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

// Four consecutive samples per thread: one Philox4x32 block gives all four
// uniforms (the same values philox_uniform draws one at a time), one 16-B store.
__device__ __forceinline__ float coarse_z(float near_, float span, int s, int n, float u) {
  // z = (near + span*step) + (u*span)/n   (two separate einsums, renderers.py:13-14)
  const float step = fdiv((float)s, (float)n);
  return fadd(fadd(near_, fmul(span, step)), fdiv(fmul(u, span), (float)n));
}

// near + span * (s / n) depends on s only: each workgroup tabulates it once in
// LDS (kCoarseTab entries; larger n computes it per sample), so a sample costs
// one IEEE division. 32-bit index arithmetic when the sample count allows.
constexpr int kCoarseTab = 1024;

__global__ void __launch_bounds__(256) sample_coarse_kernel(float near_, float far_, int64_t n_rays, int n,
                                                            const float* __restrict__ noise, uint64_t seed,
                                                            uint64_t offset, const int64_t* __restrict__ ray_ids,
                                                            float* __restrict__ z) {
  __shared__ float base_tab[kCoarseTab];
  const int nq = (n + 3) >> 2;                           // 4-sample blocks per ray
  const float span = fsub(far_, near_);
  const bool tab = n <= kCoarseTab;
  if (tab)
    for (int s = threadIdx.x; s < n; s += blockDim.x) base_tab[s] = fadd(near_, fmul(span, fdiv((float)s, (float)n)));
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = n_rays * nq;
  if (i >= total) return;
  int64_t r;
  int q;
  if (total < (1ll << 32)) {
    const unsigned ui = (unsigned)i, ur = ui / (unsigned)nq;
    r = ur;
    q = (int)(ui - ur * (unsigned)nq);
  } else {
    r = i / nq;
    q = (int)(i - r * nq);
  }
  float u[4];
  if (noise) {
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = 4 * q + k < n ? noise[r * n + 4 * q + k] : 0.f;
  } else {
    const uint64_t key = offset + (uint64_t)(ray_ids ? ray_ids[r] : r);
    const float4 v = philox_uniform4(seed, key, (uint32_t)q, kStreamCoarse);
    u[0] = v.x; u[1] = v.y; u[2] = v.z; u[3] = v.w;
  }
  float o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int s = 4 * q + k;
    o[k] = tab ? fadd(base_tab[s < n ? s : 0], fdiv(fmul(u[k], span), (float)n)) : coarse_z(near_, span, s, n, u[k]);
  }
  float* zr = z + r * n + 4 * q;
  if ((n & 3) == 0) {
    *reinterpret_cast<float4*>(zr) = make_float4(o[0], o[1], o[2], o[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * q + k < n) zr[k] = o[k];
  }
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

constexpr int kMaxCoarse = 256;
constexpr int kMaxSort = 512;
constexpr int kFineWaves = 4;

// Per-wave LDS (floats): cdf[Nc + 1] | scratch[64] | sbuf[sort_n] | obuf[Ntot]
__host__ __device__ inline int fine_wave_floats(int Nc, int sort_n, int Ntot) { return Nc + 1 + 64 + sort_n + Ntot; }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// #{L[i] < x} (LT) or #{L[i] <= x} over the sorted LDS list L[0..n); n is wave-uniform.
template <bool LT>
__device__ __forceinline__ int count_below(const float* L, int n, float x) {
  int lo = 0;
  while (n > 0) {
    const int half = n >> 1;
    const float v = L[lo + half];
    const bool go = LT ? (v < x) : (v <= x);
    lo = go ? lo + half + 1 : lo;
    n = go ? n - half - 1 : half;
  }
  return lo;
}

// Ascending bitonic sort of one float per lane across the wave (64 values).
__device__ __forceinline__ float wave_sort64(float v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const float o = __shfl_xor(v, j, 64);
      const bool up = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == up) ? fminf(v, o) : fmaxf(v, o);
    }
  }
  return v;
}

// One wave per ray; no block barriers (each wave owns its LDS slice).
//   1) w' = w + 1e-5, s = torch-CPU cascade sum (bit-exact);
//   2) pdf = w'/s (IEEE), cdf = [0, fp64 prefix sum]: lane l sums its K
//      consecutive entries sequentially, one DPP exclusive scan joins the lanes
//      (these fp64 partial sums of fp32 terms are exact: order cannot change a bit);
//   3) idx = #{cdf <= u} - 1 (binary search), z = near + (far-near)*((idx+u2)/Nc);
//   4) depth samples clamp(randn * std, near, far) (quirk Q6);
//   5) values-only sort of [z_coarse | z_fine | z_depth]: when z_coarse is
//      ascending (stratified: always, barring fp32 ties) and Nf, Nd <= 64, the
//      fine and depth lists are sorted in registers and the three sorted lists
//      merged by rank (own index + counts below in the other lists, ties broken
//      coarse < fine < depth); otherwise a wave-local bitonic sort.
__global__ void __launch_bounds__(256) sample_fine_kernel(
    const float* __restrict__ weights, const float* __restrict__ z_coarse, float near_, float far_, int64_t n_rays,
    int Nc, int Nf, int Nd, float depth_std, const float* __restrict__ u_in, const float* __restrict__ u2_in,
    const float* __restrict__ nd_in, uint64_t seed, uint64_t offset, const int64_t* __restrict__ ray_ids, int sort_n,
    float* __restrict__ z_sorted,
    int32_t* __restrict__ idx_out, float* __restrict__ z_fine_out) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ray = (int64_t)blockIdx.x * kFineWaves + wid;
  if (ray >= n_rays) return;  // wave-uniform
  const int Ntot = Nc + Nf + Nd;
  float* cdf = lds + (size_t)wid * fine_wave_floats(Nc, sort_n, Ntot);   // [0 .. Nc]
  float* scratch = cdf + Nc + 1;
  float* sbuf = scratch + 64;   // lists: coarse [0, Nc) | fine [Nc, Nc+Nf) | depth [Nc+Nf, Ntot)
  float* obuf = sbuf + sort_n;
  const float span = fsub(far_, near_);
  const uint64_t key = offset + (uint64_t)(ray_ids ? ray_ids[ray] : ray);   // Philox counter of this ray

  // 1) + 2)
  const float* w = weights + ray * Nc;
  const float* zc = z_coarse + ray * Nc;
  bool coarse_sorted = true;
  for (int k = lane; k < Nc; k += 64) {
    cdf[1 + k] = fadd(w[k], 1e-5f);
    sbuf[k] = zc[k];
  }
  wave_sync();
  for (int k = lane; k + 1 < Nc; k += 64) coarse_sorted &= sbuf[k] <= sbuf[k + 1];
  coarse_sorted = __all(coarse_sorted);
  const float s = cascade_sum_wave(cdf + 1, Nc, lane, scratch);
  {
    const int K = (Nc + 63) >> 6, k0 = K * lane;
    double part = 0.0;
    for (int k = 0; k < K; ++k)
      if (k0 + k < Nc) part += (double)fdiv(cdf[1 + k0 + k], s);
    double run = wave_excl_sum_dpp(part);
    wave_sync();   // every pdf read before any cdf write
    for (int k = 0; k < K; ++k)
      if (k0 + k < Nc) {
        run += (double)fdiv(cdf[1 + k0 + k], s);
        cdf[1 + k0 + k] = (float)run;
      }
    if (lane == 0) cdf[0] = 0.f;
  }
  wave_sync();

  // 3) importance samples
  float zf_mine = FLT_MAX;
  for (int f = lane; f < Nf; f += 64) {
    const float u = u_in ? u_in[ray * Nf + f] : philox_uniform(seed, key, f, kStreamU);
    const float u2 = u2_in ? u2_in[ray * Nf + f] : philox_uniform(seed, key, f, kStreamU2);
    const int cnt = count_below<false>(cdf, Nc + 1, u);   // #{cdf <= u}
    const int idx = cnt > 0 ? cnt - 1 : 0;
    const float steps = fdiv(fadd((float)idx, u2), (float)Nc);
    const float zf = fadd(near_, fmul(span, steps));
    if (idx_out) idx_out[ray * Nf + f] = idx;
    if (z_fine_out) z_fine_out[ray * Nf + f] = zf;
    sbuf[Nc + f] = zf;
    zf_mine = zf;
  }
  // 4) depth samples: clamp(randn * std, near, far)  (quirk Q6)
  float zd_mine = FLT_MAX;
  for (int d = lane; d < Nd; d += 64) {
    const float n = nd_in ? nd_in[ray * Nd + d] : philox_normal(seed, key, d, kStreamDepth);
    zd_mine = fminf(fmaxf(fmul(n, depth_std), near_), far_);
    sbuf[Nc + Nf + d] = zd_mine;
  }
  wave_sync();

  // 5) sort
  float* out = z_sorted + ray * Ntot;
  if (coarse_sorted && Nf <= 64 && Nd <= 64) {
    const float* A = sbuf;
    float* B = sbuf + Nc;
    float* D = sbuf + Nc + Nf;
    const float bf = wave_sort64(zf_mine, lane);
    const float bd = Nd > 0 ? wave_sort64(zd_mine, lane) : FLT_MAX;
    wave_sync();   // the unsorted lists are read by nobody past this point
    if (lane < Nf) B[lane] = bf;
    if (lane < Nd) D[lane] = bd;
    wave_sync();
    for (int k = lane; k < Nc; k += 64) {
      const float x = A[k];
      obuf[k + count_below<true>(B, Nf, x) + count_below<true>(D, Nd, x)] = x;
    }
    if (lane < Nf) obuf[lane + count_below<false>(A, Nc, bf) + count_below<true>(D, Nd, bf)] = bf;
    if (lane < Nd) obuf[lane + count_below<false>(A, Nc, bd) + count_below<false>(B, Nf, bd)] = bd;
    wave_sync();
    for (int k = lane; k < Ntot; k += 64) out[k] = obuf[k];
    return;
  }
  for (int k = Ntot + lane; k < sort_n; k += 64) sbuf[k] = FLT_MAX;
  wave_sync();
  for (int size = 2; size <= sort_n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = lane; t < (sort_n >> 1); t += 64) {
        const int i = 2 * t - (t & (stride - 1));
        const int j = i + stride;
        const float a = sbuf[i], b = sbuf[j];
        const bool up = ((i & size) == 0);
        if ((a > b) == up) { sbuf[i] = b; sbuf[j] = a; }
      }
      wave_sync();
    }
  }
  for (int k = lane; k < Ntot; k += 64) out[k] = sbuf[k];
}

}  // namespace avr

using namespace avr;

extern "C" int avr_sample_coarse(float near_, float far_, int64_t n_rays, int n_samples, const float* noise,
                                 uint64_t seed, uint64_t offset, const int64_t* ray_ids, float* z, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0, "avr_sample_coarse: bad sizes");
  const int64_t n = n_rays * n_samples;
  if (n == 0) return AVR_OK;
  AVR_REQUIRE(z, "avr_sample_coarse: null output");
  const int64_t threads = n_rays * ((n_samples + 3) / 4);
  sample_coarse_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, as_stream(stream)>>>(near_, far_, n_rays,
                                                                                       n_samples, noise, seed,
                                                                                       offset, ray_ids, z);
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
                               const int64_t* ray_ids, float* z_sorted, int32_t* idx, float* z_fine, void* stream) {
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
  const size_t shm = (size_t)kFineWaves * fine_wave_floats(n_coarse, sort_n, ntot) * sizeof(float);
  sample_fine_kernel<<<grid, 64 * kFineWaves, shm, as_stream(stream)>>>(
      weights, z_coarse, near_, far_, n_rays, n_coarse, n_importance, n_depth, depth_std, u, u2, noise_depth, seed,
      offset, ray_ids, sort_n, z_sorted, idx, z_fine);
  return check_launch("sample_fine_kernel");
}
