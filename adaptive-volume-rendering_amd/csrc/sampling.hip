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
//   then the values-only merge of [z_coarse | z_fine | z_depth] (register
//   bitonic sorts of the short lists + slot ranks; a wave-local bitonic sort of
//   the list padded to 2^k with +inf when z_coarse is not ascending).
#include <float.h>

#include "avr_common.h"

namespace avr {

// Philox streams: coarse noise; the fine pass's (u, u2) pair (one block per fine
// sample: u = .x, u2 = .y); the depth samples' normals.
constexpr uint32_t kStreamCoarse = 0x1001u, kStreamFine = 0x2002u, kStreamDepth = 0x4004u;

// Four consecutive samples per thread: one Philox4x32 block gives all four
// uniforms (the same values philox_uniform draws one at a time), one 16-B store.
template <bool POW2>
__device__ __forceinline__ float coarse_z(float near_, float span, int s, int n, float u, float inv_n) {
  // z = (near + span*step) + (u*span)/n   (two separate einsums, renderers.py:13-14)
  const float step = div_count<POW2>((float)s, (float)n, inv_n);
  return fadd(fadd(near_, fmul(span, step)), div_count<POW2>(fmul(u, span), (float)n, inv_n));
}

// near + span * (s / n) depends on s only: each workgroup tabulates it once in
// LDS (kCoarseTab entries; larger n computes it per sample), so a sample costs
// one IEEE division. 32-bit index arithmetic when the sample count allows.
constexpr int kCoarseTab = 1024;

template <bool POW2>
__global__ void __launch_bounds__(256) sample_coarse_kernel(float near_, float far_, int64_t n_rays, int n,
                                                            const float* __restrict__ noise, uint64_t seed,
                                                            uint64_t offset, const int64_t* __restrict__ ray_ids,
                                                            float* __restrict__ z) {
  __shared__ float base_tab[kCoarseTab];
  const int nq = (n + 3) >> 2;                           // 4-sample blocks per ray
  const float span = fsub(far_, near_);
  const bool tab = n <= kCoarseTab;
  const float inv_n = 1.0f / (float)n;                   // exact when POW2 (the only case it is used)
  if (tab)
    for (int s = threadIdx.x; s < n; s += blockDim.x)
      base_tab[s] = fadd(near_, fmul(span, div_count<POW2>((float)s, (float)n, inv_n)));
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
    o[k] = tab ? fadd(base_tab[s < n ? s : 0], div_count<POW2>(fmul(u[k], span), (float)n, inv_n))
               : coarse_z<POW2>(near_, span, s, n, u[k], inv_n);
  }
  float* zr = z + r * n + 4 * q;
  if ((n & 3) == 0) {
    *reinterpret_cast<floatx4*>(zr) = floatx4{o[0], o[1], o[2], o[3]};   // one 16-B store (not x3 + x1)
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
  const float u = noise ? noise[i] : philox_uniform(seed, offset + (uint64_t)r, (uint32_t)s, kStreamCoarse);
  z[i] = coarse_z<false>(nr, span, s, n, u, 0.f);
}

// get_world_rays (utils.py:315-336) + sample_coarse (renderers.py:4-24) in one
// launch, plus each ray's depth row for the composite epilogue. A workgroup
// owns kRaysPerBlock (64) consecutive rays: wave 0 builds ro, rd with one lane
// per ray (and, if asked, row 2 of inverse(cam2world) in fp64: depth = -(row .
// [x, 1]), utils.py:358-361) while waves 1-7 write the rays' z in 4-sample
// quads, consecutive threads on consecutive quads (coalesced 16-B stores): z
// does not depend on the geometry, so the fp64 latency of wave 0 overlaps the
// z stores instead of preceding them.
constexpr int kRaysPerBlock = 64;
#ifndef AVR_RAYS_THREADS
#define AVR_RAYS_THREADS 512
#endif
constexpr int kRaysThreads = AVR_RAYS_THREADS;   // wave 0 geometry + 7 z waves (13.0-13.5 vs 13.9 us with 3)

struct CoarseQuads {
  float near_, span, inv_n;
  int n, nq, lg_nq;
  bool tab;
  const float* noise;
  uint64_t seed, offset;
  const int64_t* ray_ids;
  float* z;
  const float* base_tab;
};

// the 4 z of quad `it` (ray r0 + it / nq, samples 4q..4q+3)
template <bool POW2>
__device__ __forceinline__ void coarse_quad(const CoarseQuads& c, int64_t r0, int it, int64_t& ray, int& q,
                                            float (&o)[4]) {
  const int rl = POW2 && c.n >= 4 ? it >> c.lg_nq : it / c.nq;
  q = it - rl * c.nq;
  ray = r0 + rl;
  float u[4];
  if (c.noise) {
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = 4 * q + k < c.n ? c.noise[ray * c.n + 4 * q + k] : 0.f;
  } else {
    const uint64_t key = c.offset + (uint64_t)(c.ray_ids ? c.ray_ids[ray] : ray);
    const float4 v = philox_uniform4(c.seed, key, (uint32_t)q, kStreamCoarse);
    u[0] = v.x; u[1] = v.y; u[2] = v.z; u[3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int s = 4 * q + k;
    o[k] = c.tab ? fadd(c.base_tab[s < c.n ? s : 0], div_count<POW2>(fmul(u[k], c.span), (float)c.n, c.inv_n))
                 : coarse_z<POW2>(c.near_, c.span, s, c.n, u[k], c.inv_n);
  }
}

template <bool V4>
__device__ __forceinline__ void store_quad(const CoarseQuads& c, int64_t ray, int q, const float (&o)[4]) {
  float* zr = c.z + ray * c.n + 4 * q;
  if constexpr (V4) {
    *reinterpret_cast<floatx4*>(zr) = floatx4{o[0], o[1], o[2], o[3]};
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * q + k < c.n) zr[k] = o[k];
  }
}

// quads it0, it0 + stride, ... < items; AVR_COARSE_ILP quads per pass (independent Philox chains in flight)
#ifndef AVR_COARSE_ILP
#define AVR_COARSE_ILP 1
#endif
template <bool POW2, bool V4>
__device__ __forceinline__ void coarse_quad_loop(const CoarseQuads& c, int64_t r0, int it0, int stride, int items) {
  constexpr int P = AVR_COARSE_ILP;
  int it = it0;
  for (; it + (P - 1) * stride < items; it += P * stride) {
    int64_t ray[P];
    int q[P];
    float o[P][4];
#pragma unroll
    for (int p = 0; p < P; ++p) coarse_quad<POW2>(c, r0, it + p * stride, ray[p], q[p], o[p]);
#pragma unroll
    for (int p = 0; p < P; ++p) store_quad<V4>(c, ray[p], q[p], o[p]);
  }
  for (; it < items; it += stride) {
    int64_t ray;
    int q;
    float o[4];
    coarse_quad<POW2>(c, r0, it, ray, q, o);
    store_quad<V4>(c, ray, q, o);
  }
}

template <bool POW2>
__global__ void __launch_bounds__(kRaysThreads) rays_coarse_kernel(
    const float* __restrict__ x_pix, const float* __restrict__ K, const float* __restrict__ c2w, int64_t sb_stride,
    int64_t ray_stride, int64_t n_sb, int64_t n_rays, float near_, float far_, int n, const float* __restrict__ noise,
    uint64_t seed, uint64_t offset, const int64_t* __restrict__ ray_ids, float* __restrict__ ro,
    float* __restrict__ rd, double* __restrict__ depth_row, float* __restrict__ z) {
  __shared__ float base_tab[kCoarseTab];
  const int64_t total = n_sb * n_rays;
  const int64_t r0 = (int64_t)blockIdx.x * kRaysPerBlock;
  const float span = fsub(far_, near_);
  const float inv_n = 1.0f / (float)n;
  // a power-of-two count computes near + span * (s / n) directly (an exact
  // scaling, no table and no barrier); otherwise the table saves a division
  const bool tab = !POW2 && n <= kCoarseTab;
  if (tab) {
    for (int s = threadIdx.x; s < n; s += blockDim.x)
      base_tab[s] = fadd(near_, fmul(span, div_count<POW2>((float)s, (float)n, inv_n)));
    __syncthreads();   // base_tab
  }
  if (threadIdx.x < 64) {   // wave 0: the rays' geometry, one lane per ray
    if (threadIdx.x >= kRaysPerBlock || r0 + threadIdx.x >= total) return;
    const int64_t i = r0 + threadIdx.x;
    const int64_t sb = i / n_rays, r = i - sb * n_rays;
    double k[3][3], ki[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) k[a][b] = (double)K[sb * 9 + a * 3 + b];
    invert<3>(k, ki);
    const double hx = x_pix[2 * i], hy = x_pix[2 * i + 1];
    float cam[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double kf0 = (double)(float)ki[a][0], kf1 = (double)(float)ki[a][1], kf2 = (double)(float)ki[a][2];
      cam[a] = (float)(kf0 * hx + kf1 * hy + kf2);
    }
    cam[0] = (-cam[0]) * -1.0f;   // unproject: x negated, then scaled by z = -1 (utils.py:262-265)
    cam[1] = cam[1] * -1.0f;
    cam[2] = cam[2] * -1.0f;
    const float nrm = (float)sqrt((double)cam[0] * cam[0] + (double)cam[1] * cam[1] + (double)cam[2] * cam[2]);
    const float d0 = fdiv(cam[0], nrm), d1 = fdiv(cam[1], nrm), d2 = fdiv(cam[2], nrm);
    const float* T = c2w + sb * sb_stride + r * ray_stride;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      rd[3 * i + a] = (float)((double)T[4 * a] * d0 + (double)T[4 * a + 1] * d1 + (double)T[4 * a + 2] * d2);
      ro[3 * i + a] = T[4 * a + 3];
    }
    if (depth_row) {
      double m[4][4], inv[4][4];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) m[p][q] = (double)T[4 * p + q];
      invert<4>(m, inv);
      reinterpret_cast<double4*>(depth_row)[i] = make_double4(inv[2][0], inv[2][1], inv[2][2], inv[2][3]);
    }
    return;
  }
  const int nq = (n + 3) >> 2;
  const int lg_nq = POW2 && n >= 4 ? __builtin_ctz((unsigned)nq) : 0;   // nq a power of two too
  const int64_t nr_blk = total - r0 < kRaysPerBlock ? total - r0 : kRaysPerBlock;
  const int items = (int)nr_blk * nq;
  const CoarseQuads cq{near_, span, inv_n, n, nq, lg_nq, tab, noise, seed, offset, ray_ids, z, base_tab};
  // waves 1-7: z. The whole-quad store is chosen once for the loop, not per quad (a per-quad branch let
  // the compiler merge the 16-B store with the ragged path's scalar stores into x3 + x1 stores)
  if ((n & 3) == 0) coarse_quad_loop<POW2, true>(cq, r0, threadIdx.x - 64, blockDim.x - 64, items);
  else coarse_quad_loop<POW2, false>(cq, r0, threadIdx.x - 64, blockDim.x - 64, items);
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
constexpr int kMaxK = kMaxCoarse / 64;   // coarse samples per lane

// cascade_sum_wave for N a multiple of 64 from registers: lane l holds
// x[l + 64m], m < K = N/64. Same additions in the same order: lane l < 32
// sums x[32i + l] over i (x[l + 64m], then lane l+32's x[l + 32 + 64m]), lane
// l < 8 adds the partials of lanes l+8, l+16, l+24, and the 8 lane sums are
// added in lane order. No LDS round trips or wave barriers.
__device__ __forceinline__ float cascade_sum_regs(const float (&x)[kMaxK], int K, int lane) {
  float p = 0.f;
#pragma unroll
  for (int m = 0; m < kMaxK; ++m)
    if (m < K) {
      p = fadd(p, x[m]);
      p = fadd(p, lane_xor(x[m], 32, lane));
    }
  const float q8 = lane_xor(p, 8, lane);
  const float a = fadd(fadd(fadd(p, q8), lane_xor(p, 16, lane)), lane_xor(q8, 16, lane));
  float s = 0.f;
#pragma unroll
  for (int l = 0; l < 8; ++l) s = fadd(s, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), l)));
  return s;
}
constexpr int kMaxSort = 512;
constexpr int kFineWaves = 4;

// Per-wave LDS (floats): cdf[Nc + 1] | scratch[64] | sbuf[sort_n] | obuf[Ntot]
__host__ __device__ inline int fine_wave_floats(int Nc, int sort_n, int Ntot) { return Nc + 1 + 64 + sort_n + Ntot; }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// #{L[i] < x} (LT) or #{L[i] <= x} over the sorted LDS list L[0..n). The
// probe sequence depends on n only (base += half when L[base + half - 1]
// passes): a uniform n keeps the loop scalar and the lanes converged.
template <bool LT>
__device__ __forceinline__ int count_below(const float* L, int n, float x) {
  if (n <= 0) return 0;
  int base = 0;
  for (int len = n; len > 1;) {
    const int half = len >> 1;
    const float v = L[base + half - 1];
    base = (LT ? v < x : v <= x) ? base + half : base;
    len -= half;
  }
  const float v = L[base];
  return base + ((LT ? v < x : v <= x) ? 1 : 0);
}

// lanes of a bitonic stage (k, j) that keep the minimum: ((l & k) == 0) == ((l & j) == 0)
__host__ __device__ constexpr uint64_t bitonic_min_lanes(int k, int j) {
  uint64_t m = 0;
  for (int l = 0; l < 64; ++l)
    if (((l & k) == 0) == ((l & j) == 0)) m |= 1ull << l;
  return m;
}

// partner value of lane l ^ J for the sort: quad-permute DPP (J = 1, 2; left
// to the compiler to fold into the min/max), a ds_swizzle xor within 32 lanes
// (J = 4, 8, 16: LDS crossbar, no memory traffic, one instruction instead of
// two DPP rows and a select), the permlane32 swap for J = 32
template <int J>
__device__ __forceinline__ float sort_partner(float v, int lane) {
  const int b = __float_as_int(v);
  if constexpr (J == 1) return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0xB1, 0xf, 0xf, false));
  else if constexpr (J == 2) return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0x4E, 0xf, 0xf, false));
  else if constexpr (J <= 16) return __int_as_float(__builtin_amdgcn_ds_swizzle(b, 0x1F | (J << 10)));
  else return lane_xor(v, J, lane);
}

template <int K, int J>
__device__ __forceinline__ float bitonic_stages(float v, int lane) {
  // keep v where (v < o) == (lane keeps the minimum), else o: one compare
  // (into a lane mask), a scalar xnor with the stage's constant, one select;
  // equal values are interchangeable (values-only sort, no NaN, no -0)
  const float o = sort_partner<J>(v, lane);
  const uint64_t keep_v = ~(__ballot(v < o) ^ bitonic_min_lanes(K, J));
  v = mask_select(keep_v, o, v);
  if constexpr (J > 1) return bitonic_stages<K, J / 2>(v, lane);
  else return v;
}

template <int K>
__device__ __forceinline__ float bitonic_from(float v, int lane) {
  v = bitonic_stages<K, K / 2>(v, lane);
  if constexpr (K < 64) return bitonic_from<2 * K>(v, lane);
  else return v;
}

// Ascending bitonic sort of one float per lane across the wave (64 values);
// partners through lane_xor (DPP / permlane swaps, no LDS round trips), the
// min/max choice by a constant lane mask.
__device__ __forceinline__ float wave_sort64(float v, int lane) { return bitonic_from<2>(v, lane); }

// count_below over the sorted list L[0..n) from a guess g of the answer: when
// L[g-2] and L[g+2] bracket x (checked), the count is g - 1 plus the entries
// of the window [g-1, g+2) that pass — five independent reads instead of a
// dependent search chain; otherwise the full binary search. Exact either way.
template <bool LT>
__device__ __forceinline__ int count_below_near(const float* L, int n, float x, int g) {
  const auto pass = [&](float v) { return LT ? v < x : v <= x; };
  const int lo = g - 1 < 0 ? 0 : (g - 1 > n ? n : g - 1);
  const int hi = g + 2 > n ? n : (g + 2 < lo ? lo : g + 2);
  const int last = n - 1;
  const float before = L[lo > 0 ? lo - 1 : 0], after = L[hi < n ? hi : last];
  const float w0 = L[lo < last ? lo : last], w1 = L[lo + 1 < last ? lo + 1 : last], w2 = L[lo + 2 < last ? lo + 2 : last];
  const bool below_lo = lo == 0 || pass(before);   // every index < lo counts
  const bool above_hi = hi == n || !pass(after);   // no index >= hi counts
  const int c = lo + (lo < hi && pass(w0)) + (lo + 1 < hi && pass(w1)) + (lo + 2 < hi && pass(w2));
  if (below_lo && above_hi) return c;
  return count_below<LT>(L, n, x);
}

// One wave per ray; no block barriers (each wave owns its LDS slice).
//   1) w' = w + 1e-5, s = torch-CPU cascade sum (bit-exact);
//   2) pdf = w'/s (IEEE, once per entry), cdf = [0, fp64 prefix sum]: lane l
//      sums its K consecutive entries sequentially, one DPP exclusive scan
//      joins the lanes (these fp64 partial sums of fp32 terms are exact:
//      order cannot change a bit);
//   3) idx = #{cdf <= u} - 1 (binary search), z = near + (far-near)*((idx+u2)/Nc);
//   4) depth samples clamp(randn * std, near, far) (quirk Q6);
//   5) values-only sort of [z_coarse | z_fine | z_depth]: when z_coarse is
//      ascending (stratified: always, barring fp32 ties) and Nf, Nd <= 64, the
//      fine and depth lists are sorted in registers and the three sorted lists
//      merged by rank (own index + counts below in the other lists, ties broken
//      coarse < fine < depth; a fine value's count in the coarse list starts
//      from its stratified bin; with no depth samples, the coarse values fill
//      the slots the fine values leave, in order); otherwise a wave-local
//      bitonic sort.
// NC, NF, ND > 0: the sample counts as compile-time constants (the renderer's
// 128 -> 64 shape: loops unrolled, no loop or exec-mask bookkeeping); 0: runtime.
template <bool POW2, int NC = 0, int NF = 0, int ND = 0>
__global__ void __launch_bounds__(256) sample_fine_kernel(
    const float* __restrict__ weights, const float* __restrict__ z_coarse, float near_, float far_, int64_t n_rays,
    int Nc_, int Nf_, int Nd_, float depth_std, const float* __restrict__ u_in, const float* __restrict__ u2_in,
    const float* __restrict__ nd_in, uint64_t seed, uint64_t offset, const int64_t* __restrict__ ray_ids, int sort_n,
    float* __restrict__ z_sorted, int32_t* __restrict__ idx_out, float* __restrict__ z_fine_out) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wid, ray: scalars
  const int64_t ray = (int64_t)blockIdx.x * kFineWaves + wid;
  if (ray >= n_rays) return;  // wave-uniform
  const int Nc = NC ? NC : Nc_, Nf = NC ? NF : Nf_, Nd = NC ? ND : Nd_;
  const int Ntot = Nc + Nf + Nd;
  float* cdf = lds + (size_t)wid * fine_wave_floats(Nc, sort_n, Ntot);   // [0 .. Nc]
  float* scratch = cdf + Nc + 1;
  float* sbuf = scratch + 64;   // lists: coarse [0, Nc) | fine [Nc, Nc+Nf) | depth [Nc+Nf, Ntot)
  float* obuf = sbuf + sort_n;
  const float span = fsub(far_, near_);
  const uint64_t key = offset + (uint64_t)(ray_ids ? ray_ids[ray] : ray);   // Philox counter of this ray
  const float inv_nc = 1.0f / (float)Nc;

  // 1) + 2)
  const float* w = weights + ray * Nc;
  const float* zc = z_coarse + ray * Nc;
  bool coarse_sorted = true;
  float wv[kMaxK], zv[kMaxK];
#pragma unroll
  for (int m = 0; m < kMaxK; ++m) {
    const int k = lane + 64 * m;
    wv[m] = k < Nc ? w[k] : 0.f;
    zv[m] = k < Nc ? zc[k] : 0.f;
  }
  // the in-kernel (u, u2) draw of this lane's fine sample does not depend on
  // the weights: it runs while their loads are in flight (one sample per lane)
  float4 draw = {0.f, 0.f, 0.f, 0.f};
  if (!u_in && Nf <= 64 && lane < Nf) draw = philox_uniform4(seed, key, (uint32_t)lane, kStreamFine);
  float xr[kMaxK];
#pragma unroll
  for (int m = 0; m < kMaxK; ++m) {
    const int k = lane + 64 * m;
    xr[m] = 0.f;
    if (k < Nc) {
      xr[m] = fadd(wv[m], 1e-5f);
      cdf[1 + k] = xr[m];
      sbuf[k] = zv[m];
    }
  }
  float s;
  if ((Nc & 63) == 0) {
    s = cascade_sum_regs(xr, Nc >> 6, lane);
    wave_sync();
  } else {
    wave_sync();
    s = cascade_sum_wave(cdf + 1, Nc, lane, scratch);
  }
  for (int k = lane; k + 1 < Nc; k += 64) coarse_sorted &= sbuf[k] <= sbuf[k + 1];
  coarse_sorted = __all(coarse_sorted);
  {
    const int K = (Nc + 63) >> 6, k0 = K * lane;
    float pv[kMaxK];
    double part = 0.0;
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) {
      pv[k] = (k < K && k0 + k < Nc) ? fdiv(cdf[1 + k0 + k], s) : 0.f;
      part += (double)pv[k];
    }
    double run = wave_excl_sum_dpp(part);
    wave_sync();   // every pdf read before any cdf write
#pragma unroll
    for (int k = 0; k < kMaxK; ++k)
      if (k < K && k0 + k < Nc) {
        run += (double)pv[k];
        cdf[1 + k0 + k] = (float)run;
      }
    if (lane == 0) cdf[0] = 0.f;
  }
  wave_sync();

  // 3) importance samples
  float zf_mine = FLT_MAX;
  for (int f = lane; f < Nf; f += 64) {
    float u, u2;
    if (u_in) {
      u = u_in[ray * Nf + f];
      u2 = u2_in[ray * Nf + f];
    } else {
      const float4 v = Nf <= 64 ? draw : philox_uniform4(seed, key, (uint32_t)f, kStreamFine);
      u = v.x;
      u2 = v.y;
    }
    const int cnt = count_below<false>(cdf, Nc + 1, u);   // #{cdf <= u}
    const int idx = cnt > 0 ? cnt - 1 : 0;
    const float steps = div_count<POW2>(fadd((float)idx, u2), (float)Nc, inv_nc);
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
  if (coarse_sorted && Nf <= 64 && Nd == 0) {
    // two lists: the fine values take slots lane + #{A <= bf} (increasing in
    // lane); the coarse values fill the other slots in order. A slot's list
    // index = the number of fine slots before it (ballot + mbcnt) or the rest.
    const float* A = sbuf;
    float* B = sbuf + Nc;
    int* marks = reinterpret_cast<int*>(obuf);
    for (int k = lane; k < Ntot; k += 64) marks[k] = 0;
    const float bf = wave_sort64(zf_mine, lane);
    wave_sync();   // the unsorted fine list is read by nobody past this point
    if (lane < Nf) {
      B[lane] = bf;
      const float t = (bf - near_) * ((float)Nc * __builtin_amdgcn_rcpf(span));   // a guess: verified below
      const int g = t > 0.f ? (t < (float)Nc ? (int)t : Nc) : 0;
      marks[lane + count_below_near<false>(A, Nc, bf, g)] = 1;
    }
    wave_sync();
    int base = 0;
    for (int s0 = 0; s0 < Ntot; s0 += 64) {
      const int k = s0 + lane;
      const bool fine = k < Ntot && marks[k] != 0;
      const uint64_t mask = __ballot(fine);
      const int before = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
      if (k < Ntot) out[k] = sbuf[fine ? Nc + before : k - before];   // B[before] or A[k - before]: one read
      base += __popcll(mask);
    }
    return;
  }
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
    if (lane < Nf) {
      // stratified coarse lists put #{A <= bf} within a step of bf's bin
      const float t = (bf - near_) * ((float)Nc * __builtin_amdgcn_rcpf(span));   // a guess: verified below
      const int g = t > 0.f ? (t < (float)Nc ? (int)t : Nc) : 0;
      obuf[lane + count_below_near<false>(A, Nc, bf, g) + count_below<true>(D, Nd, bf)] = bf;
    }
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

// AdaptiveVolumeRenderer's band in training (renderers.py:490-496 and the band points, :497-508): per ray the
// marched distance d = (world_x - ro_x) / rd_x, z_i = (near + span * (i / n)) + (noise_i * span) / n with near =
// d - eps, far = d + eps, span = far - near (sample_coarse's fp32 operations, renderers.py:10-14, in torch's
// order), z sorted ascending (torch.sort: rounding can swap neighbours), pts = ro + rd * z. One thread per ray.
constexpr int kBandMax = 64;

__global__ void __launch_bounds__(256) band_fwd_kernel(int64_t R, int n, const float* __restrict__ world,
                                                       const float* __restrict__ ro, const float* __restrict__ rd,
                                                       const float* __restrict__ noise, float eps,
                                                       float* __restrict__ z, float* __restrict__ pts) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const float o0 = ro[3 * r], o1 = ro[3 * r + 1], o2 = ro[3 * r + 2];
  const float d0 = rd[3 * r], d1 = rd[3 * r + 1], d2 = rd[3 * r + 2];
  const float d = fdiv(fsub(world[3 * r], o0), d0);
  const float near_ = fsub(d, eps), far_ = fadd(d, eps), span = fsub(far_, near_);
  const float fn = (float)n;
  float zz[kBandMax];
  for (int i = 0; i < n; ++i) {
    const float v = fadd(fadd(near_, fmul(span, fdiv((float)i, fn))), fdiv(fmul(noise[r * n + i], span), fn));
    int k = i;
    for (; k > 0 && v < zz[k - 1]; --k) zz[k] = zz[k - 1];   // insertion: ascending, ties keep their order
    zz[k] = v;
  }
  for (int i = 0; i < n; ++i) {
    const float v = zz[i];
    z[r * n + i] = v;
    float* p = pts + 3 * (r * n + i);
    p[0] = fadd(o0, fmul(d0, v));
    p[1] = fadd(o1, fmul(d1, v));
    p[2] = fadd(o2, fmul(d2, v));
  }
}

// Its adjoint: every z_i moves with d (dz_i / dd = 1: near and far both do, span does not), pts with z along rd, so
// d loss / d world_x = sum_i (gz_i + gpts_i . rd) / rd_x; world_y, world_z and ro / rd get nothing.
__global__ void __launch_bounds__(256) band_bwd_kernel(int64_t R, int n, const float* __restrict__ rd,
                                                       const float* __restrict__ gz, const float* __restrict__ gpts,
                                                       float* __restrict__ gworld) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const float d0 = rd[3 * r], d1 = rd[3 * r + 1], d2 = rd[3 * r + 2];
  float s = 0.f;
  for (int i = 0; i < n; ++i) {
    float g = gz ? gz[r * n + i] : 0.f;
    if (gpts) {
      const float* q = gpts + 3 * (r * n + i);
      g = fadd(g, fadd(fadd(fmul(q[0], d0), fmul(q[1], d1)), fmul(q[2], d2)));
    }
    s = fadd(s, g);
  }
  gworld[3 * r] = fdiv(s, d0);
  gworld[3 * r + 1] = 0.f;
  gworld[3 * r + 2] = 0.f;
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
  const unsigned grid = (unsigned)((threads + 255) / 256);
  if ((n_samples & (n_samples - 1)) == 0)
    sample_coarse_kernel<true><<<grid, 256, 0, as_stream(stream)>>>(near_, far_, n_rays, n_samples, noise, seed,
                                                                   offset, ray_ids, z);
  else
    sample_coarse_kernel<false><<<grid, 256, 0, as_stream(stream)>>>(near_, far_, n_rays, n_samples, noise, seed,
                                                                    offset, ray_ids, z);
  return check_launch("sample_coarse_kernel");
}

extern "C" int avr_rays_sample_coarse(const float* x_pix, const float* K, const float* c2w, int64_t c2w_sb_stride,
                                      int64_t c2w_ray_stride, int64_t n_sb, int64_t n_rays, float near_, float far_,
                                      int n_samples, const float* noise, uint64_t seed, uint64_t offset,
                                      const int64_t* ray_ids, float* ro, float* rd, double* depth_row, float* z,
                                      void* stream) {
  AVR_REQUIRE(n_sb >= 0 && n_rays >= 0 && n_samples > 0, "avr_rays_sample_coarse: bad sizes");
  const int64_t total = n_sb * n_rays;
  if (total == 0) return AVR_OK;
  AVR_REQUIRE(x_pix && K && c2w && ro && rd && z, "avr_rays_sample_coarse: null pointer");
  const int64_t blocks = (total + kRaysPerBlock - 1) / kRaysPerBlock;
  AVR_REQUIRE(blocks < (1ll << 31), "avr_rays_sample_coarse: too many rays");
  auto* kern = (n_samples & (n_samples - 1)) == 0 ? rays_coarse_kernel<true> : rays_coarse_kernel<false>;
  kern<<<(unsigned)blocks, kRaysThreads, 0, as_stream(stream)>>>(x_pix, K, c2w, c2w_sb_stride, c2w_ray_stride, n_sb, n_rays,
                                                        near_, far_, n_samples, noise, seed, offset, ray_ids, ro, rd,
                                                        depth_row, z);
  return check_launch("rays_coarse_kernel");
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
  auto* kern = (n_coarse & (n_coarse - 1)) == 0 ? sample_fine_kernel<true> : sample_fine_kernel<false>;
  if (n_coarse == 128 && n_importance == 64 && n_depth == 0) kern = sample_fine_kernel<true, 128, 64, 0>;
  kern<<<grid, 64 * kFineWaves, shm, as_stream(stream)>>>(
      weights, z_coarse, near_, far_, n_rays, n_coarse, n_importance, n_depth, depth_std, u, u2, noise_depth, seed,
      offset, ray_ids, sort_n, z_sorted, idx, z_fine);
  return check_launch("sample_fine_kernel");
}

extern "C" int avr_band_fwd(int64_t n_rays, int n_samples, const float* world, const float* ro, const float* rd,
                            const float* noise, float eps, float* z, float* pts, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples <= kBandMax, "avr_band_fwd: bad sizes (1..%d samples)",
              kBandMax);
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(world && ro && rd && noise && z && pts, "avr_band_fwd: null pointer");
  band_fwd_kernel<<<(unsigned)((n_rays + 255) / 256), 256, 0, as_stream(stream)>>>(n_rays, n_samples, world, ro, rd,
                                                                                   noise, eps, z, pts);
  return check_launch("band_fwd_kernel");
}

extern "C" int avr_band_bwd(int64_t n_rays, int n_samples, const float* rd, const float* grad_z,
                            const float* grad_pts, float* grad_world, void* stream) {
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples <= kBandMax, "avr_band_bwd: bad sizes (1..%d samples)",
              kBandMax);
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(rd && grad_world, "avr_band_bwd: null pointer");
  band_bwd_kernel<<<(unsigned)((n_rays + 255) / 256), 256, 0, as_stream(stream)>>>(n_rays, n_samples, rd, grad_z,
                                                                                   grad_pts, grad_world);
  return check_launch("band_bwd_kernel");
}
