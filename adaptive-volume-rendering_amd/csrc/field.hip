// Radiance field: NewPixelNeRFNet.forward (models.py:739-863) fused into one
// kernel on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact f32 products).
//
// Transposed formulation: every layer computes Y^T = W . X^T with the hidden
// features on the MFMA rows and 16 samples on the MFMA columns, so a layer's
// 16x16 accumulator tile (lane l: sample l&15, features 4(l>>4)+0..3) is
// already in the lane order the next layer's B operand wants:
//   k-step (t, r) uses feature 16t + 4g + r from lane group g = l>>4.
// Weights are repacked once (avr_field_pack) into that fragment order,
// [t][ot][lane] float4 = W[16ot + (l&15)][16t + 4(l>>4) + 0..3], so each lane
// streams 16 B per 4 MFMAs with fully coalesced 1 KiB wave loads.
//
// One wave = 16 samples; a lane keeps the residual stream h and the block
// temporary t for its 16x(d_hidden) slice in registers (2 x d_hidden/4 VGPRs),
// and a 1 KiB-per-tile LDS slab (per wave, no cross-wave traffic, no barriers)
// turns an accumulator tile into the next layer's B operand with one
// ds_write_b128 / ds_read_b128 per tile.
//
// lin_z is applied to the latent map per texel (avr_field_latent_table) and
// bilinearly interpolated per sample; every bias (b_in + bz0, b1 + bz_{b+1},
// ...) is pre-summed at pack time.
#include <mutex>

#include "field_common.h"

namespace avr {

// ----------------------------------------------------------------- layout
static int make_layout(const avr_field_dims* d, Layout* L) {
  AVR_REQUIRE(d, "field: null dims");
  AVR_REQUIRE(d->d_hidden == 64 || d->d_hidden == 128 || d->d_hidden == 256 || d->d_hidden == 512,
              "field: d_hidden must be 64/128/256/512 (got %d)", d->d_hidden);
  AVR_REQUIRE(d->d_latent > 0 && d->d_latent % 16 == 0 && d->d_latent <= 1024,
              "field: d_latent must be a positive multiple of 16 <= 1024 (got %d)", d->d_latent);
  AVR_REQUIRE(d->n_blocks >= 1 && d->n_blocks <= AVR_MAX_BLOCKS, "field: n_blocks must be in [1, %d]",
              AVR_MAX_BLOCKS);
  AVR_REQUIRE(d->n_lin_z >= 0 && d->n_lin_z <= d->n_blocks, "field: n_lin_z must be in [0, n_blocks]");
  AVR_REQUIRE(d->num_freqs >= 0 && 3 + 6 * d->num_freqs + 3 == d->d_in && d->d_in <= 16 * kInTiles,
              "field: d_in %d != 6*num_freqs+6 or > 48 (fused path supports PE(xyz)+raw viewdirs)", d->d_in);
  const int NT = d->d_hidden / 16, KC = d->d_hidden / 32;
  L->NT = NT;
  L->KTl = d->d_latent / 16;
  const int64_t tile = 64 * 4;  // floats per (t, ot) fp32 fragment block
  const int64_t tile16 = 64 * 8;  // floats per (c, ft) fp16 hi/lo fragment block (64 lanes x 32 B)
  int64_t o = 0;
  L->w_in = o; o += (int64_t)kInTiles * NT * tile;
  for (int b = 0; b < d->n_blocks; ++b) {
    L->fc0[b] = o; o += (int64_t)NT * NT * tile;
    L->fc1[b] = o; o += (int64_t)NT * NT * tile;
  }
  L->w_out = o; o += (int64_t)NT * tile;
  for (int b = 0; b < d->n_lin_z; ++b) { L->lin_z[b] = o; o += (int64_t)L->KTl * NT * tile; }
  L->b_in = o; o += d->d_hidden;
  for (int b = 0; b < d->n_blocks; ++b) {
    L->b_fc0[b] = o; o += d->d_hidden;
    L->b_fc1[b] = o; o += d->d_hidden;
  }
  L->b_out = o; o += 16;
  o = (o + 63) & ~(int64_t)63;
  L->x3_hdr = o; o += 64;
  L->x3_in = o; o += (int64_t)kX3InChunks * NT * tile16;
  for (int b = 0; b < d->n_blocks; ++b) {
    L->x3_fc0[b] = o; o += (int64_t)KC * NT * tile16;
    L->x3_fc1[b] = o; o += (int64_t)KC * NT * tile16;
  }
  L->x3_out = o; o += (int64_t)KC * tile16;
  AVR_REQUIRE(d->bn == 0 || d->bn == 1, "field: bn must be 0 or 1");
  L->bn = d->bn;
  for (int b = 0; b < d->n_blocks; ++b) {
    L->bn_a[b] = L->bn_c[b] = 0;
    if (d->bn) { L->bn_a[b] = o; o += d->d_hidden; L->bn_c[b] = o; o += d->d_hidden; }
  }
  AVR_REQUIRE(d->spade == 0 || d->spade == 1, "field: spade must be 0 or 1");
  AVR_REQUIRE(d->beta >= 0.f && d->beta < 1e30f, "field: beta must be >= 0 (0: ReLU)");
  AVR_REQUIRE(!(d->beta > 0.f && d->bn), "field: Softplus with BatchNorm runs on the module path");
  AVR_REQUIRE(!(d->spade && d->bn), "field: use_spade with BatchNorm runs on the module path");
  L->spade = d->spade;
  L->n_lin_z = d->n_lin_z;
  L->n_tables = d->n_lin_z * (d->spade ? 2 : 1);
  for (int b = 0; b < AVR_MAX_BLOCKS; ++b) L->scale_z[b] = 0;
  for (int t = 0; t < 2 * AVR_MAX_BLOCKS; ++t) L->b_tab[t] = 0;
  if (d->spade) {
    for (int b = 0; b < d->n_lin_z; ++b) { L->scale_z[b] = o; o += (int64_t)L->KTl * NT * tile; }
    for (int t = 0; t < L->n_tables; ++t) { L->b_tab[t] = o; o += d->d_hidden; }
  }
  L->x3_tables = d->d_latent % 64 == 0 && d->d_latent <= 512;
  for (int t = 0; t < 2 * AVR_MAX_BLOCKS; ++t) L->x3_tab[t] = 0;
  for (int t = 0; L->x3_tables && t < L->n_tables; ++t) {
    L->x3_tab[t] = o;
    o += (int64_t)(d->d_latent / 32) * NT * tile16;
  }
  L->total = o;
  return AVR_OK;
}

static int make_bwd_layout(const avr_field_dims* d, BwdLayout* LB) {
  const int64_t S = (int64_t)(d->d_hidden / 32) * (d->d_hidden / 16) * 64 * 8;   // floats per x3 hidden layer
  int64_t o = 64;
  for (int b = 0; b < d->n_blocks; ++b) {
    LB->fc0t[b] = o; o += S;
    LB->fc1t[b] = o; o += S;
  }
  // lin_z[b]^T (d_latent x d_hidden after the transpose: a hidden layer's shape when d_latent == d_hidden) for
  // avr_bn_layer_run's transposed products (the point gradient's sum_b Gz[b] . W_z[b])
  for (int b = 0; b < AVR_MAX_BLOCKS; ++b) {
    LB->lzt[b] = -1;
    if (b < d->n_lin_z && d->d_latent == d->d_hidden && !d->spade) { LB->lzt[b] = o; o += S; }
  }
  LB->total = o;
  return AVR_OK;
}

int field_layout(const avr_field_dims* d, Layout* L) { return make_layout(d, L); }
int field_bwd_layout(const avr_field_dims* d, BwdLayout* LB) {
  Layout L;
  const int rc = make_layout(d, &L);
  return rc ? rc : make_bwd_layout(d, LB);
}

// ----------------------------------------------------------------- packing
// fp32 fragments: dst[(t*NTo + ot)*64 + l][r] = W[16ot + (l&15)][16t + 4(l>>4) + r] (zero padded);
// bias vectors: dst[i] = a[i] + b[i] (b may be null), zero beyond n.
// The fp32 fragments and bias vectors of a pack in two launches (blockIdx.y = job), not one launch each:
// the pack runs in every training step (the weights change).
struct LinJob {
  const float* W;
  float* dst;
  int out_dim, in_dim, NTo, KTi;
};
struct LinBatch {
  LinJob j[2 + 4 * AVR_MAX_BLOCKS];
  int count;
};
struct BiasJob {
  const float* a;
  const float* b;
  float* dst;
  int n, n_pad;
};
struct BiasBatch {
  BiasJob j[2 + 8 * AVR_MAX_BLOCKS];
  int count;
};

__global__ void pack_linear_batch_kernel(LinBatch bt) {
  const LinJob& J = bt.j[blockIdx.y];
  const int64_t n = (int64_t)J.KTi * J.NTo * 256;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i & 3);
    const int l = (int)((i >> 2) & 63);
    const int64_t blk = i >> 8;
    const int ot = (int)(blk % J.NTo), t = (int)(blk / J.NTo);
    const int row = 16 * ot + (l & 15), col = 16 * t + 4 * (l >> 4) + r;
    J.dst[i] = (row < J.out_dim && col < J.in_dim) ? J.W[(int64_t)row * J.in_dim + col] : 0.f;
  }
}

__global__ void pack_bias_batch_kernel(BiasBatch bt) {
  const BiasJob& J = bt.j[blockIdx.y];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < J.n_pad; i += gridDim.x * blockDim.x)
    J.dst[i] = (i < J.n) ? (J.b ? fadd(J.a[i], J.b[i]) : J.a[i]) : 0.f;
}


// x3 fragments: dst[((c*FTt + ft)*2 + {0, 1})*512 + 8l + e] = (hi, lo) of
// (a tile's 64 hi lanes, then its 64 lo lanes: each 16-B-per-lane load of one
// half reads 1 KiB contiguous, whole 128-B lines)
// W[16ft + (l&15)][32c + (e<4 ? 4g+e : 16+4g+e-4)] * s_w, g = l>>4, with
// s_w = 2^(14 - ceil-exponent of max|W|) from the layer's header word.
// (rs, cs) = element strides of W's rows / columns: (in_dim, 1) for W, (1, ld) for W^T.
__device__ __forceinline__ void pack_x3_elem(const float* __restrict__ W, int out_dim, int in_dim, int64_t rs,
                                             int64_t cs, int FTt, const unsigned* __restrict__ maxbits,
                                             _Float16* __restrict__ dst, int64_t i) {
  const int e = (int)(i & 7);
  const int l = (int)((i >> 3) & 63);
  const int64_t blk = i >> 9;
  const int ft = (int)(blk % FTt), c = (int)(blk / FTt);
  const int g = l >> 4;
  const int row = 16 * ft + (l & 15);
  const int col = 32 * c + (e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4));
  const float sw = pow2_scale_for(__uint_as_float(*maxbits));
  const float v = (row < out_dim && col < in_dim) ? W[(int64_t)row * rs + (int64_t)col * cs] * sw : 0.f;
  const _Float16 hi = (_Float16)v;
  const _Float16 lo = (_Float16)(v - (float)hi);
  const int64_t base = ((int64_t)c * FTt + ft) * 2 * 64 * 8 + l * 8;
  dst[base + e] = hi;
  dst[base + 64 * 8 + e] = lo;
}

// Every layer of a pack in two launches (max |W| of each layer, then its
// fragments; blockIdx.y = layer) instead of two per layer: the weight pack
// runs in every training step.
struct X3PackJob {
  const float* W;
  unsigned* maxbits;
  _Float16* dst;
  int64_t rs, cs, nw, n;
  int out_dim, in_dim, FTt;
};
struct X3PackBatch {
  X3PackJob j[kX3PackJobs];
  int count;
};

// max|W| of each layer as float bits (atomicMax on non-negative floats = on their bits)
// (one atomic per workgroup: a few dozen per layer, not one per wave)
__global__ void absmax_batch_kernel(X3PackBatch b) {
  __shared__ float wm[4];
  const X3PackJob& J = b.j[blockIdx.y];
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < J.nw; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(J.W[i]));
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(J.maxbits, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}

__global__ void pack_x3_batch_kernel(X3PackBatch b) {
  const X3PackJob& J = b.j[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < J.n; i += (int64_t)gridDim.x * blockDim.x)
    pack_x3_elem(J.W, J.out_dim, J.in_dim, J.rs, J.cs, J.FTt, J.maxbits, J.dst, i);
}

// ----------------------------------------------------------------- fp32 MFMA tiles
// acc[ot] += sum_t sum_r A(ot,t,r) B(t,r); A from packed global [t][ot][lane]
// through a P-deep register ring that runs ahead across t iterations, B from
// the wave's LDS slab [t][lane].
// NTOT: output tiles per K tile in the packed layout (NT < NTOT: this call
// computes the NT tiles starting at W, a slice of them)
template <int NT, int P, int NTOT = NT>
__device__ __forceinline__ void gemm_tiles(floatx4 (&acc)[NT], const floatx4* __restrict__ W, int KT,
                                           const floatx4* slab, int lane) {
  static_assert(NT % P == 0 && P % 2 == 0, "ring must divide the tile count");
  const floatx4* wl = W + lane;
  floatx4 ring[P];
#pragma unroll
  for (int p = 0; p < P; ++p) ring[p] = wl[p * 64];
  for (int t = 0; t < KT; ++t) {
    const floatx4 bv = slab[t * 64 + lane];
    const floatx4* cur = wl + (int64_t)t * NTOT * 64;
    const floatx4* nxt = wl + (int64_t)(t + 1 < KT ? t + 1 : t) * NTOT * 64;
#pragma unroll
    for (int ot = 0; ot < NT; ot += 2) {
      const floatx4 a0 = ring[ot % P];
      const floatx4 a1 = ring[(ot + 1) % P];
      ring[ot % P] = (ot + P < NT) ? cur[(ot + P) * 64] : nxt[(ot + P - NT) * 64];
      ring[(ot + 1) % P] = (ot + 1 + P < NT) ? cur[(ot + 1 + P) * 64] : nxt[(ot + 1 + P - NT) * 64];
      acc[ot] = mfma4(a0.x, bv.x, acc[ot]);
      acc[ot + 1] = mfma4(a1.x, bv.x, acc[ot + 1]);
      acc[ot] = mfma4(a0.y, bv.y, acc[ot]);
      acc[ot + 1] = mfma4(a1.y, bv.y, acc[ot + 1]);
      acc[ot] = mfma4(a0.z, bv.z, acc[ot]);
      acc[ot + 1] = mfma4(a1.z, bv.z, acc[ot + 1]);
      acc[ot] = mfma4(a0.w, bv.w, acc[ot]);
      acc[ot + 1] = mfma4(a1.w, bv.w, acc[ot + 1]);
    }
  }
}

template <int NT>
__device__ __forceinline__ void load_bias(floatx4 (&acc)[NT], const float* __restrict__ bias, int g) {
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = *reinterpret_cast<const floatx4*>(bias + 16 * ot + 4 * g);
}

template <int NT>
__device__ __forceinline__ void add_bias(floatx4 (&acc)[NT], const float* __restrict__ bias, int g) {
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] += *reinterpret_cast<const floatx4*>(bias + 16 * ot + 4 * g);
}

// acc += sum_c w_c * Z[texel_c][features of this lane]
template <int NT>
__device__ __forceinline__ void add_interp(floatx4 (&acc)[NT], const float* __restrict__ Z, const Bilinear& bl,
                                           int g) {
  constexpr int CH = NT < 8 ? NT : 8;
#pragma unroll
  for (int o0 = 0; o0 < NT; o0 += CH) {
    floatx4 v[CH][4];
#pragma unroll
    for (int k = 0; k < CH; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[k][c] = *reinterpret_cast<const floatx4*>(Z + (int64_t)bl.tex[c] * (NT * 16) + 16 * (o0 + k) + 4 * g);
#pragma unroll
    for (int k = 0; k < CH; ++k)
      acc[o0 + k] += ((bl.w[0] * v[k][0] + bl.w[1] * v[k][1]) + bl.w[2] * v[k][2]) + bl.w[3] * v[k][3];
  }
}

template <int NT>
__device__ __forceinline__ void store_relu(floatx4* slab, const floatx4 (&acc)[NT], int lane) {
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) {
    floatx4 v = acc[ot];
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    slab[ot * 64 + lane] = v;
  }
}

template <int NT>
__global__ void __launch_bounds__(256, 1) field_fwd_kernel(FieldArgs a) {
  extern __shared__ floatx4 lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  floatx4* slab = lds + (size_t)wid * (NT > kInTiles ? NT : kInTiles) * 64;
  const int64_t m = ((int64_t)blockIdx.x * kFieldWaves + wid) * kSPW + j;
  const bool valid = m < a.M;
  const int64_t mm = valid ? m : a.M - 1;

  // ---- sample geometry, z_feature (features 16t + 4g + r of this lane's sample -> slab[t][lane])
  const SampleGeom sg = sample_geom(a, mm);
#pragma unroll
  for (int t = 0; t < kInTiles; ++t) {
    float f[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = z_feature(sg, 16 * t + 4 * g + r, a.num_freqs, a.freq_factor);
    slab[t * 64 + lane] = floatx4{f[0], f[1], f[2], f[3]};
  }
  const Bilinear& bl = sg.bl;

  const floatx4* P4 = reinterpret_cast<const floatx4*>(a.packed);
  floatx4 h[NT], tt[NT];
  constexpr int P = NT >= 16 ? 16 : NT;

  // ---- lin_in (+ lin_z[0] + both biases)
  load_bias<NT>(h, a.packed + a.L.b_in, g);
  if (a.n_lin_z > 0) add_interp<NT>(h, a.table, bl, g);
  gemm_tiles<NT, P>(h, P4 + a.L.w_in / 4, kInTiles, slab, lane);

  // ---- ResnetBlockFC x n_blocks
  for (int b = 0; b < a.n_blocks; ++b) {
    store_relu<NT>(slab, h, lane);
    load_bias<NT>(tt, a.packed + a.L.b_fc0[b], g);
    gemm_tiles<NT, P>(tt, P4 + a.L.fc0[b] / 4, NT, slab, lane);
    store_relu<NT>(slab, tt, lane);
    add_bias<NT>(h, a.packed + a.L.b_fc1[b], g);
    if (b + 1 < a.n_lin_z) add_interp<NT>(h, a.table + (b + 1) * a.table_stride, bl, g);
    gemm_tiles<NT, P>(h, P4 + a.L.fc1[b] / 4, NT, slab, lane);
  }

  // ---- lin_out(relu(h)) -> (sigmoid rgb, relu sigma)
  store_relu<NT>(slab, h, lane);
  floatx4 o0 = *reinterpret_cast<const floatx4*>(a.packed + a.L.b_out + 4 * g);
  floatx4 o1 = {0.f, 0.f, 0.f, 0.f};
  const floatx4* wo = P4 + a.L.w_out / 4 + lane;
#pragma unroll 4
  for (int t = 0; t < NT; t += 2) {
    const floatx4 A0 = wo[t * 64], A1 = wo[(t + 1) * 64];
    const floatx4 B0 = slab[t * 64 + lane], B1 = slab[(t + 1) * 64 + lane];
    o0 = mfma4(A0.x, B0.x, o0); o1 = mfma4(A1.x, B1.x, o1);
    o0 = mfma4(A0.y, B0.y, o0); o1 = mfma4(A1.y, B1.y, o1);
    o0 = mfma4(A0.z, B0.z, o0); o1 = mfma4(A1.z, B1.z, o1);
    o0 = mfma4(A0.w, B0.w, o0); o1 = mfma4(A1.w, B1.w, o1);
  }
  const floatx4 o = o0 + o1;
  if (g == 0 && valid) a.out[m] = make_float4(sigmoidf_(o.x), sigmoidf_(o.y), sigmoidf_(o.z), fmaxf(o.w, 0.f));
}

// Table t's weights: lin_z[t], then (use_spade) scale_z[t - n_lin_z].
__device__ __forceinline__ int64_t table_weights(const Layout& L, int t) {
  return t < L.n_lin_z ? L.lin_z[t] : L.scale_z[t - L.n_lin_z];
}

// table[b][texel][f] = sum_c Wz_b[f][c] latent[c][texel]  (16 texels per wave)
// (+ the table's bias with use_spade)
template <int NT>
__global__ void __launch_bounds__(256, 1) latent_table_kernel(const float* __restrict__ packed, Layout L,
                                                              const float* __restrict__ latent, int HW,
                                                              float* __restrict__ table) {
  extern __shared__ floatx4 lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int b = blockIdx.y;
  floatx4* slab = lds + (size_t)wid * L.KTl * 64;
  const int64_t texel = ((int64_t)blockIdx.x * kFieldWaves + wid) * kSPW + j;
  const bool valid = texel < HW;
  const int64_t tx = valid ? texel : HW - 1;
  for (int t = 0; t < L.KTl; ++t) {
    const int c0 = 16 * t + 4 * g;
    slab[t * 64 + lane] = floatx4{latent[(int64_t)c0 * HW + tx], latent[(int64_t)(c0 + 1) * HW + tx],
                                  latent[(int64_t)(c0 + 2) * HW + tx], latent[(int64_t)(c0 + 3) * HW + tx]};
  }
  floatx4 acc[NT];
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = floatx4{0.f, 0.f, 0.f, 0.f};
  constexpr int P = NT >= 16 ? 16 : NT;
  gemm_tiles<NT, P>(acc, reinterpret_cast<const floatx4*>(packed + table_weights(L, b)), L.KTl, slab, lane);
  if (L.spade) {
#pragma unroll
    for (int ot = 0; ot < NT; ++ot) acc[ot] += *reinterpret_cast<const floatx4*>(packed + L.b_tab[b] + 16 * ot + 4 * g);
  }
  if (valid) {
    float* dst = table + ((int64_t)b * HW + texel) * (NT * 16) + 4 * g;
#pragma unroll
    for (int ot = 0; ot < NT; ++ot) *reinterpret_cast<floatx4*>(dst + 16 * ot) = acc[ot];
  }
}

// The same table with the output tiles split over the workgroup's waves
// (NT >= 8): a workgroup owns 16 texels, their latent columns are staged in
// LDS once (32 KB at d_latent 512) and wave w computes output tiles
// [w NT/4, (w+1) NT/4). Four times the workgroups of latent_table_kernel at a
// quarter of the LDS each, so a 4096-texel table fills the chip.
template <int NT>
__global__ void __launch_bounds__(256) latent_table_split_kernel(const float* __restrict__ packed, Layout L,
                                                                 const float* __restrict__ latent, int HW,
                                                                 float* __restrict__ table) {
  constexpr int NWT = NT / kFieldWaves;          // output tiles per wave
  constexpr int P = NWT >= 16 ? 16 : NWT;
  extern __shared__ floatx4 lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int b = blockIdx.y;
  const int64_t texel = (int64_t)blockIdx.x * kSPW + j;
  const bool valid = texel < HW;
  const int64_t tx = valid ? texel : HW - 1;
  for (int t = wid; t < L.KTl; t += kFieldWaves) {
    const int c0 = 16 * t + 4 * g;
    lds[t * 64 + lane] = floatx4{latent[(int64_t)c0 * HW + tx], latent[(int64_t)(c0 + 1) * HW + tx],
                                 latent[(int64_t)(c0 + 2) * HW + tx], latent[(int64_t)(c0 + 3) * HW + tx]};
  }
  __syncthreads();
  floatx4 acc[NWT];
#pragma unroll
  for (int ot = 0; ot < NWT; ++ot) acc[ot] = floatx4{0.f, 0.f, 0.f, 0.f};
  gemm_tiles<NWT, P, NT>(acc, reinterpret_cast<const floatx4*>(packed + table_weights(L, b)) + NWT * wid * 64, L.KTl,
                         lds, lane);
  if (L.spade) {
#pragma unroll
    for (int ot = 0; ot < NWT; ++ot)
      acc[ot] += *reinterpret_cast<const floatx4*>(packed + L.b_tab[b] + 16 * (NWT * wid + ot) + 4 * g);
  }
  if (valid) {
    float* dst = table + ((int64_t)b * HW + texel) * (NT * 16) + 16 * NWT * wid + 4 * g;
#pragma unroll
    for (int ot = 0; ot < NWT; ++ot) *reinterpret_cast<floatx4*>(dst + 16 * ot) = acc[ot];
  }
}

// ----------------------------------------------------------------- host side
static int pack_linear(const float* W, int out_dim, int in_dim, int NTo, int KTi, float* dst, LinBatch& bt) {
  AVR_REQUIRE(W, "avr_field_pack: null weight tensor");
  AVR_REQUIRE(bt.count < (int)(sizeof(bt.j) / sizeof(bt.j[0])), "avr_field_pack: too many layers");
  bt.j[bt.count++] = LinJob{W, dst, out_dim, in_dim, NTo, KTi};
  return AVR_OK;
}

// one layer into a batch (W is (out_dim, in_dim) row-major; transpose: (in_dim,
// out_dim), and the fragments hold W^T)
static int add_x3(X3PackBatch& bt, const float* W, int out_dim, int in_dim, int KC, int FTt, unsigned* maxbits,
                  float* dst, bool transpose = false) {
  AVR_REQUIRE(W, "avr_field_pack: null weight tensor");
  AVR_REQUIRE(bt.count < kX3PackJobs, "avr_field_pack: too many layers");
  X3PackJob& J = bt.j[bt.count++];
  J.W = W;
  J.maxbits = maxbits;
  J.dst = reinterpret_cast<_Float16*>(dst);
  J.rs = transpose ? 1 : in_dim;
  J.cs = transpose ? out_dim : 1;
  J.nw = (int64_t)out_dim * in_dim;
  J.n = (int64_t)KC * FTt * 64 * 8;
  J.out_dim = out_dim;
  J.in_dim = in_dim;
  J.FTt = FTt;
  return AVR_OK;
}

static int run_x3(const X3PackBatch& bt, hipStream_t s) {
  if (bt.count == 0) return AVR_OK;
  int64_t nw = 0, n = 0;
  for (int k = 0; k < bt.count; ++k) {
    nw = bt.j[k].nw > nw ? bt.j[k].nw : nw;
    n = bt.j[k].n > n ? bt.j[k].n : n;
  }
  const unsigned ga = (unsigned)((nw + 4095) / 4096 < 64 ? (nw + 4095) / 4096 : 64);   // >= 16 values per thread
  absmax_batch_kernel<<<dim3(ga, bt.count), 256, 0, s>>>(bt);
  int rc = check_launch("absmax_batch_kernel");
  if (rc) return rc;
  const unsigned gp = (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
  pack_x3_batch_kernel<<<dim3(gp, bt.count), 256, 0, s>>>(bt);
  return check_launch("pack_x3_batch_kernel");
}

static int pack_bias(const float* a, const float* b, int n, int n_pad, float* dst, BiasBatch& bt) {
  AVR_REQUIRE(a, "avr_field_pack: null bias tensor");
  AVR_REQUIRE(bt.count < (int)(sizeof(bt.j) / sizeof(bt.j[0])), "avr_field_pack: too many vectors");
  bt.j[bt.count++] = BiasJob{a, b, dst, n, n_pad};
  return AVR_OK;
}

static int run_fp32_packs(const LinBatch& lb, const BiasBatch& bb, hipStream_t s) {
  int64_t n = 0;
  for (int k = 0; k < lb.count; ++k) {
    const int64_t nk = (int64_t)lb.j[k].KTi * lb.j[k].NTo * 256;
    n = nk > n ? nk : n;
  }
  if (lb.count) {
    pack_linear_batch_kernel<<<dim3((unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024), lb.count), 256, 0,
                               s>>>(lb);
    const int rc = check_launch("pack_linear_batch_kernel");
    if (rc) return rc;
  }
  int nb = 0;
  for (int k = 0; k < bb.count; ++k) nb = bb.j[k].n_pad > nb ? bb.j[k].n_pad : nb;
  if (bb.count == 0) return AVR_OK;
  pack_bias_batch_kernel<<<dim3((unsigned)((nb + 255) / 256), bb.count), 256, 0, s>>>(bb);
  return check_launch("pack_bias_batch_kernel");
}

template <int NT>
static int launch_field(const FieldArgs& a, hipStream_t s) {
  const size_t shm = (size_t)kFieldWaves * (NT > kInTiles ? NT : kInTiles) * 64 * sizeof(floatx4);
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&field_fwd_kernel<NT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return fail(AVR_E_HIP, "field_fwd_kernel: cannot set dynamic LDS to %zu", shm);
    attr = true;
  }
  const int64_t per_block = kFieldWaves * kSPW;
  const int64_t blocks = (a.M + per_block - 1) / per_block;
  AVR_REQUIRE(blocks < (1ll << 31), "field: too many points");
  field_fwd_kernel<NT><<<(unsigned)blocks, 64 * kFieldWaves, shm, s>>>(a);
  return check_launch("field_fwd_kernel");
}

template <int NT>
static int launch_table(const float* packed, const Layout& L, const float* latent, int HW, int n_lin_z,
                        float* table, hipStream_t s) {
  if constexpr (NT >= 8) {
    const size_t shm = (size_t)L.KTl * 64 * sizeof(floatx4);
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&latent_table_split_kernel<NT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return fail(AVR_E_HIP, "latent_table_split_kernel: cannot set dynamic LDS to %zu", shm);
    dim3 grid((HW + kSPW - 1) / kSPW, n_lin_z);
    latent_table_split_kernel<NT><<<grid, 64 * kFieldWaves, shm, s>>>(packed, L, latent, HW, table);
    return check_launch("latent_table_split_kernel");
  }
  const size_t shm = (size_t)kFieldWaves * L.KTl * 64 * sizeof(floatx4);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&latent_table_kernel<NT>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
    return fail(AVR_E_HIP, "latent_table_kernel: cannot set dynamic LDS to %zu", shm);
  const int per_block = kFieldWaves * kSPW;
  dim3 grid((HW + per_block - 1) / per_block, n_lin_z);
  latent_table_kernel<NT><<<grid, 64 * kFieldWaves, shm, s>>>(packed, L, latent, HW, table);
  return check_launch("latent_table_kernel");
}

static int field_common(const avr_field_dims* dims, const avr_view_desc* view, const float* packed,
                        const float* table, FieldArgs* a) {
  Layout L;
  int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(view && packed, "field: null view/packed");
  AVR_REQUIRE(dims->n_lin_z == 0 || table, "field: null latent table");
  AVR_REQUIRE(view->latent_h > 0 && view->latent_w > 0, "field: bad latent size");
  a->packed = packed;
  a->table = table;
  a->table_stride = (int64_t)view->latent_h * view->latent_w * dims->d_hidden;
  a->L = L;
  view_from_desc(view, &a->v);
  a->n_blocks = dims->n_blocks;
  a->n_lin_z = dims->n_lin_z;
  a->num_freqs = dims->num_freqs;
  a->freq_factor = dims->freq_factor;
  a->beta = dims->beta;
  a->b_begin = 0;
  a->b_end = dims->n_blocks;
  a->h_out = nullptr;
  a->h_in = nullptr;
  return AVR_OK;
}

// The precision each blob was packed for (avr_field_pack): an AVR_FIELD_X3 blob holds no fp32 fragments of
// lin_in / fc_0 / fc_1, so the fp32 kernel must not run on it. A small host-side table keyed by the blob's
// address (the last kPackTags packs; the device header is not read back: that would synchronise the stream).
namespace {
constexpr int kPackTags = 128;
struct PackTag {
  const float* p;
  int precision;
};
std::mutex g_pack_mu;
PackTag g_pack_tags[kPackTags] = {};
int g_pack_next = 0;

void record_pack(const float* p, int precision) {
  std::lock_guard<std::mutex> lock(g_pack_mu);
  for (PackTag& t : g_pack_tags)
    if (t.p == p) {
      t.precision = precision;
      return;
    }
  g_pack_tags[g_pack_next] = PackTag{p, precision};
  g_pack_next = (g_pack_next + 1) % kPackTags;
}

int packed_precision(const float* p) {   // -1: not packed by this library instance (or evicted)
  std::lock_guard<std::mutex> lock(g_pack_mu);
  for (const PackTag& t : g_pack_tags)
    if (t.p == p) return t.precision;
  return -1;
}
}  // namespace

static int dispatch_field(const avr_field_dims* dims, const FieldArgs& a, hipStream_t s) {
  const int d_hidden = dims->d_hidden;
  if (dims->precision == AVR_FIELD_X3) return dispatch_field_x3(d_hidden, a, s);
  AVR_REQUIRE(packed_precision(a.packed) != AVR_FIELD_X3,
              "field: the blob was packed for AVR_FIELD_X3 (no fp32 lin_in / fc_0 / fc_1 fragments): pack it with "
              "AVR_FIELD_FP32 to run the fp32 kernel");
  AVR_REQUIRE(!dims->bn, "field: BatchNorm nets run on the x3 path only");
  AVR_REQUIRE(!dims->spade && !(dims->beta > 0.f), "field: use_spade / Softplus nets run on the x3 path only");
  AVR_REQUIRE(dims->precision == AVR_FIELD_FP32, "field: unknown precision %d", dims->precision);
  switch (d_hidden) {
    case 64: return launch_field<4>(a, s);
    case 128: return launch_field<8>(a, s);
    case 256: return launch_field<16>(a, s);
    case 512: return launch_field<32>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "field: d_hidden %d", d_hidden);
}

}  // namespace avr

using namespace avr;

#ifdef AVR_STAMPS
static unsigned long long* g_stamps = nullptr;
extern "C" void avr_debug_set_stamps(void* p) { g_stamps = reinterpret_cast<unsigned long long*>(p); }
static int g_debug = 0;
extern "C" void avr_debug_set_flags(int f) { g_debug = f; }
#endif

extern "C" int avr_field_packed_floats(const avr_field_dims* dims, int64_t* n_floats) {
  Layout L;
  const int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(n_floats, "avr_field_packed_floats: null output");
  *n_floats = L.total;
  return AVR_OK;
}

extern "C" int avr_field_pack(const avr_field_dims* dims, const avr_resnetfc_weights* w, float* packed,
                              void* stream) {
  Layout L;
  int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(w && packed, "avr_field_pack: null pointer");
  hipStream_t s = as_stream(stream);
  const int H = dims->d_hidden, NT = L.NT;
  // the fp32 fragments the x3 kernels never read (lin_in, fc_0, fc_1) are packed only for an fp32 blob; the
  // lin_z / scale_z ones always (the exact-fp32 tables)
  const bool fp32 = dims->precision != AVR_FIELD_X3, fp32_tab = true;
  LinBatch lb{};
  BiasBatch bb{};
  if (fp32 && (rc = pack_linear(w->lin_in_w, H, dims->d_in, NT, kInTiles, packed + L.w_in, lb))) return rc;
  if ((rc = pack_linear(w->lin_out_w, 4, H, 1, NT, packed + L.w_out, lb))) return rc;   // also the backward's
  for (int b = 0; b < dims->n_blocks; ++b) {
    if (fp32 && (rc = pack_linear(w->fc0_w[b], H, H, NT, NT, packed + L.fc0[b], lb))) return rc;
    if (fp32 && (rc = pack_linear(w->fc1_w[b], H, H, NT, NT, packed + L.fc1[b], lb))) return rc;
    if ((rc = pack_bias(w->fc0_b[b], nullptr, H, H, packed + L.b_fc0[b], bb))) return rc;
    const float* bz = (b + 1 < dims->n_lin_z && !dims->spade) ? w->lin_z_b[b + 1] : nullptr;
    if ((rc = pack_bias(w->fc1_b[b], bz, H, H, packed + L.b_fc1[b], bb))) return rc;
  }
  for (int b = 0; fp32_tab && b < dims->n_lin_z; ++b)
    if ((rc = pack_linear(w->lin_z_w[b], H, dims->d_latent, NT, L.KTl, packed + L.lin_z[b], lb))) return rc;
  if ((rc = pack_bias(w->lin_in_b, dims->n_lin_z > 0 && !dims->spade ? w->lin_z_b[0] : nullptr, H, H,
                      packed + L.b_in, bb)))
    return rc;
  for (int b = 0; dims->spade && b < dims->n_lin_z; ++b) {
    AVR_REQUIRE(w->scale_z_w[b] && w->scale_z_b[b] && w->lin_z_b[b],
                "avr_field_pack: use_spade needs scale_z weight / bias and lin_z bias of every lin_z block");
    if (fp32_tab && (rc = pack_linear(w->scale_z_w[b], H, dims->d_latent, NT, L.KTl, packed + L.scale_z[b], lb)))
      return rc;
    if ((rc = pack_bias(w->lin_z_b[b], nullptr, H, H, packed + L.b_tab[b], bb))) return rc;
    if ((rc = pack_bias(w->scale_z_b[b], nullptr, H, H, packed + L.b_tab[dims->n_lin_z + b], bb))) return rc;
  }
  if ((rc = pack_bias(w->lin_out_b, nullptr, 4, 16, packed + L.b_out, bb))) return rc;
  for (int b = 0; dims->bn && b < dims->n_blocks; ++b) {
    AVR_REQUIRE(w->bn_scale[b] && w->bn_shift[b], "avr_field_pack: bn needs bn_scale / bn_shift of every block");
    if ((rc = pack_bias(w->bn_scale[b], nullptr, H, H, packed + L.bn_a[b], bb))) return rc;
    if ((rc = pack_bias(w->bn_shift[b], nullptr, H, H, packed + L.bn_c[b], bb))) return rc;
  }
  if ((rc = run_fp32_packs(lb, bb, s))) return rc;
  // split-fp16 fragments (header word per layer: 0 lin_in, 1 lin_out, 2+2b fc0[b], 3+2b fc1[b])
  unsigned* hdr = reinterpret_cast<unsigned*>(packed + L.x3_hdr);
  if (hipMemsetAsync(hdr, 0, 64 * sizeof(float), s) != hipSuccess) return fail(AVR_E_HIP, "avr_field_pack: memset");
  const int KC = H / 32;
  X3PackBatch bt{};
  if ((rc = add_x3(bt, w->lin_in_w, H, dims->d_in, kX3InChunks, NT, hdr + 0, packed + L.x3_in))) return rc;
  if ((rc = add_x3(bt, w->lin_out_w, 4, H, KC, 1, hdr + 1, packed + L.x3_out))) return rc;
  for (int b = 0; b < dims->n_blocks; ++b) {
    if ((rc = add_x3(bt, w->fc0_w[b], H, H, KC, NT, hdr + 2 + 2 * b, packed + L.x3_fc0[b]))) return rc;
    if ((rc = add_x3(bt, w->fc1_w[b], H, H, KC, NT, hdr + 3 + 2 * b, packed + L.x3_fc1[b]))) return rc;
  }
  // the table weights for the x3 table kernel (lin_z[t], then scale_z with use_spade)
  for (int t = 0; L.x3_tables && t < L.n_tables; ++t) {
    const float* Wt = t < dims->n_lin_z ? w->lin_z_w[t] : w->scale_z_w[t - dims->n_lin_z];
    if ((rc = add_x3(bt, Wt, H, dims->d_latent, dims->d_latent / 32, NT, hdr + kX3TabHdr + t, packed + L.x3_tab[t])))
      return rc;
  }
  if ((rc = run_x3(bt, s))) return rc;
  record_pack(packed, dims->precision);
  return AVR_OK;
}

extern "C" int avr_field_bwd_packed_floats(const avr_field_dims* dims, int64_t* n_floats) {
  Layout L;
  BwdLayout LB;
  const int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(n_floats, "avr_field_bwd_packed_floats: null output");
  make_bwd_layout(dims, &LB);
  *n_floats = LB.total;
  return AVR_OK;
}

extern "C" int avr_field_pack_bwd(const avr_field_dims* dims, const avr_resnetfc_weights* w, float* packed_bwd,
                                  void* stream) {
  Layout L;
  BwdLayout LB;
  int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(w && packed_bwd, "avr_field_pack_bwd: null pointer");
  make_bwd_layout(dims, &LB);
  hipStream_t s = as_stream(stream);
  unsigned* hdr = reinterpret_cast<unsigned*>(packed_bwd);
  if (hipMemsetAsync(hdr, 0, 64 * sizeof(float), s) != hipSuccess) return fail(AVR_E_HIP, "avr_field_pack_bwd: memset");
  const int H = dims->d_hidden, KC = H / 32, NT = H / 16;
  X3PackBatch bt{};
  for (int b = 0; b < dims->n_blocks; ++b) {
    if ((rc = add_x3(bt, w->fc0_w[b], H, H, KC, NT, hdr + 2 + 2 * b, packed_bwd + LB.fc0t[b], true))) return rc;
    if ((rc = add_x3(bt, w->fc1_w[b], H, H, KC, NT, hdr + 3 + 2 * b, packed_bwd + LB.fc1t[b], true))) return rc;
  }
  for (int b = 0; b < AVR_MAX_BLOCKS; ++b)
    if (LB.lzt[b] >= 0 &&
        (rc = add_x3(bt, w->lin_z_w[b], H, H, KC, NT, hdr + kBwdLinZHdr + b, packed_bwd + LB.lzt[b], true)))
      return rc;
  return run_x3(bt, s);
}

extern "C" int avr_field_train_sizes(const avr_field_dims* dims, int n_scenes, int64_t n_points, int64_t* act_floats,
                                     int64_t* mask_words_out) {
  Layout L;
  const int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(n_scenes >= 1 && n_points >= 0 && act_floats && mask_words_out, "avr_field_train_sizes: bad argument");
  const int64_t layers = 2 * dims->n_blocks + 1;
  const int64_t blocks = n_scenes * ((n_points + kX3Samples - 1) / kX3Samples);
  *act_floats = layers * n_scenes * n_points * dims->d_hidden;
  *mask_words_out = layers * blocks * 4 * mask_words(dims->d_hidden / 64) * 64;
  return AVR_OK;
}

extern "C" int avr_field_fwd_points_train(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                                          const float* packed, const float* tables, const float* xyz,
                                          const float* viewdirs, int64_t n_points, float* out, float* act,
                                          int64_t act_rows, uint32_t* mask, uint32_t* act_max, float* z_feature,
                                          int ld_z, uint32_t* z_max, void* stream) {
  FieldArgs a{};
  AVR_REQUIRE(views && n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES,
              "avr_field_fwd_points_train: 1..%d scenes per call", AVR_MAX_SCENES);
  int rc = field_common(dims, views, packed, tables, &a);
  if (rc) return rc;
  AVR_REQUIRE(dims->precision == AVR_FIELD_X3, "avr_field_fwd_points_train: the training path is x3 only");
  AVR_REQUIRE(!dims->bn && !dims->spade,
              "avr_field_fwd_points_train: BatchNorm nets train on avr_bn_layer_run, use_spade nets on the module path");
  AVR_REQUIRE(n_points >= 0, "avr_field_fwd_points_train: bad size");
  AVR_REQUIRE(n_points == 0 || (xyz && viewdirs && out && act && mask), "avr_field_fwd_points_train: null pointer");
  AVR_REQUIRE(act_rows >= n_scenes * n_points, "avr_field_fwd_points_train: act_rows < n_scenes * n_points");
  for (int s = 0; s < n_scenes; ++s) {
    AVR_REQUIRE(views[s].latent_h == views[0].latent_h && views[s].latent_w == views[0].latent_w,
                "avr_field_fwd_points_train: scenes need latent maps of one size");
    view_from_desc(&views[s], &a.views[s]);
  }
  a.xyz = xyz; a.vd = viewdirs; a.n_samples = 1;
  a.M = n_points;
  a.out = reinterpret_cast<float4*>(out);
  a.act = act;
  a.act_stride = act_rows * dims->d_hidden;
  a.mask = mask;
  a.act_max = act_max;
  AVR_REQUIRE(!z_feature || ld_z >= dims->d_in, "avr_field_fwd_points_train: ld_z %d < d_in %d", ld_z, dims->d_in);
  a.zf = z_feature;
  a.zf_ld = ld_z;
  a.zf_max = z_max;
  a.n_scenes = n_scenes;
  a.blocks_per_scene = (n_points + kX3Samples - 1) / kX3Samples;
  a.table_scene_stride = (int64_t)(a.L.n_tables > 0 ? a.L.n_tables : 1) * a.table_stride;
  if (a.M == 0) return AVR_OK;
  return dispatch_field_x3(dims->d_hidden, a, as_stream(stream));
}

extern "C" int avr_field_bwd(const avr_field_dims* dims, const float* packed, const float* packed_bwd, int n_scenes,
                             int64_t n_points, const float* out, const float* grad_out, const uint32_t* mask,
                             const float* act, int64_t act_rows, float* grads, int64_t grads_rows,
                             uint32_t* grads_max, void* stream) {
  BwdArgs a{};
  int rc = make_layout(dims, &a.L);
  if (rc) return rc;
  AVR_REQUIRE(dims->precision == AVR_FIELD_X3, "avr_field_bwd: the training path is x3 only");
  AVR_REQUIRE(!dims->bn && !dims->spade,
              "avr_field_bwd: BatchNorm nets train on avr_bn_layer_run, use_spade nets on the module path");
  AVR_REQUIRE(!(dims->beta > 0.f) || (act && act_rows >= (int64_t)n_scenes * n_points),
              "avr_field_bwd: Softplus nets need the forward's act rows (act_rows >= n_scenes * n_points)");
  a.act = act;
  a.act_stride = act_rows * dims->d_hidden;
  a.beta = dims->beta;
  AVR_REQUIRE(n_points >= 0 && n_scenes >= 1, "avr_field_bwd: bad size");
  if (n_points == 0) return AVR_OK;
  AVR_REQUIRE(packed && packed_bwd && out && grad_out && mask && grads, "avr_field_bwd: null pointer");
  AVR_REQUIRE(grads_rows >= n_scenes * n_points, "avr_field_bwd: grads_rows < n_scenes * n_points");
  make_bwd_layout(dims, &a.LB);
  a.packed = packed;
  a.packed_bwd = packed_bwd;
  a.n_blocks = dims->n_blocks;
  a.M = n_points;
  a.n_scenes = n_scenes;
  a.blocks_per_scene = (n_points + kX3Samples - 1) / kX3Samples;
  a.out = reinterpret_cast<const float4*>(out);
  a.grad_out = reinterpret_cast<const float4*>(grad_out);
  a.mask = mask;
  a.G = grads;
  a.g_stride = grads_rows * dims->d_hidden;
  a.g_max = grads_max;
  return dispatch_field_bwd_x3(dims->d_hidden, a, as_stream(stream));
}

extern "C" int avr_field_latent_table(const avr_field_dims* dims, const float* packed, const float* latent, int H,
                                      int W, float* table, void* stream) {
  Layout L;
  int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(packed && latent && table, "avr_field_latent_table: null pointer");
  AVR_REQUIRE(H > 0 && W > 0, "avr_field_latent_table: bad latent size");
  if (L.n_tables == 0) return AVR_OK;
  hipStream_t s = as_stream(stream);
  // AVR_FIELD_X3: tables on the split-fp16 GEMM (the training path, which recomputes them every step);
  // AVR_FIELD_FP32: exact fp32 products (inference: computed once per latent map)
  if (dims->precision == AVR_FIELD_X3 && L.x3_tables)
    return dispatch_table_x3(packed, L, latent, H * W, dims->d_latent, dims->d_hidden, table, 1, s);
  switch (dims->d_hidden) {
    case 64: return launch_table<4>(packed, L, latent, H * W, L.n_tables, table, s);
    case 128: return launch_table<8>(packed, L, latent, H * W, L.n_tables, table, s);
    case 256: return launch_table<16>(packed, L, latent, H * W, L.n_tables, table, s);
    case 512: return launch_table<32>(packed, L, latent, H * W, L.n_tables, table, s);
  }
  return fail(AVR_E_UNSUPPORTED, "field: d_hidden %d", dims->d_hidden);
}

extern "C" int avr_field_latent_table_batch(const avr_field_dims* dims, const float* packed, const float* latent,
                                            int n_scenes, int H, int W, float* table, void* stream) {
  Layout L;
  int rc = make_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(n_scenes >= 1, "avr_field_latent_table_batch: n_scenes must be >= 1");
  AVR_REQUIRE(packed && latent && table, "avr_field_latent_table_batch: null pointer");
  AVR_REQUIRE(H > 0 && W > 0, "avr_field_latent_table_batch: bad latent size");
  if (L.n_tables == 0) return AVR_OK;
  if (dims->precision == AVR_FIELD_X3 && L.x3_tables)
    return dispatch_table_x3(packed, L, latent, H * W, dims->d_latent, dims->d_hidden, table, n_scenes,
                             as_stream(stream));
  const int64_t lat_stride = (int64_t)dims->d_latent * H * W, tab_stride = (int64_t)L.n_tables * H * W * dims->d_hidden;
  for (int sc = 0; sc < n_scenes; ++sc)
    if ((rc = avr_field_latent_table(dims, packed, latent + sc * lat_stride, H, W, table + sc * tab_stride, stream)))
      return rc;
  return AVR_OK;
}

extern "C" int avr_field_fwd_rays(const avr_field_dims* dims, const avr_view_desc* view, const float* packed,
                                  const float* table, const float* ro, const float* rd, const float* z,
                                  int64_t n_rays, int n_samples, float* out, void* stream) {
  FieldArgs a{};
  int rc = field_common(dims, view, packed, table, &a);
  if (rc) return rc;
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0, "avr_field_fwd_rays: bad sizes");
  AVR_REQUIRE(n_rays == 0 || (ro && rd && z && out), "avr_field_fwd_rays: null pointer");
  a.ro = ro; a.rd = rd; a.z = z; a.n_samples = n_samples;
#ifdef AVR_STAMPS
  a.stamps = g_stamps;
  a.debug = g_debug;
#endif
  a.M = n_rays * n_samples;
  a.out = reinterpret_cast<float4*>(out);
  if (a.M == 0) return AVR_OK;
  return dispatch_field(dims, a, as_stream(stream));
}

// Several scenes in one launch (x3 path): scene s's samples are rows s * per_scene .. of the inputs, its lin_z
// tables at tables + s * max(n_tables, 1) * H*W * d_hidden (FusedField.tables_batch), its view views[s].
static int field_batch(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes, const float* packed,
                       const float* tables, FieldArgs* a, int64_t per_scene, const char* what) {
  AVR_REQUIRE(views && n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES, "%s: 1..%d scenes per call", what,
              AVR_MAX_SCENES);
  AVR_REQUIRE(dims && dims->precision == AVR_FIELD_X3, "%s: the multi-scene launch is x3 only", what);
  int rc = field_common(dims, views, packed, tables, a);
  if (rc) return rc;
  for (int s = 0; s < n_scenes; ++s) {
    AVR_REQUIRE(views[s].latent_h == views[0].latent_h && views[s].latent_w == views[0].latent_w,
                "%s: scenes need latent maps of one size", what);
    view_from_desc(&views[s], &a->views[s]);
  }
  a->M = per_scene;
  a->n_scenes = n_scenes;
  a->blocks_per_scene = (per_scene + kX3Samples - 1) / kX3Samples;
  a->table_scene_stride = (int64_t)(a->L.n_tables > 0 ? a->L.n_tables : 1) * a->table_stride;
  return AVR_OK;
}

extern "C" int avr_field_fwd_rays_batch(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                                        const float* packed, const float* tables, const float* ro, const float* rd,
                                        const float* z, int64_t n_rays, int n_samples, float* out, void* stream) {
  FieldArgs a{};
  AVR_REQUIRE(n_rays >= 0 && n_samples > 0, "avr_field_fwd_rays_batch: bad sizes");
  int rc = field_batch(dims, views, n_scenes, packed, tables, &a, n_rays * n_samples, "avr_field_fwd_rays_batch");
  if (rc) return rc;
  AVR_REQUIRE(n_rays == 0 || (ro && rd && z && out), "avr_field_fwd_rays_batch: null pointer");
  a.ro = ro; a.rd = rd; a.z = z; a.n_samples = n_samples;
  a.out = reinterpret_cast<float4*>(out);
  if (a.M == 0) return AVR_OK;
  return dispatch_field_x3(dims->d_hidden, a, as_stream(stream));
}

extern "C" int avr_field_fwd_points_batch(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                                          const float* packed, const float* tables, const float* xyz,
                                          const float* viewdirs, int64_t n_points, float* out, void* stream) {
  FieldArgs a{};
  AVR_REQUIRE(n_points >= 0, "avr_field_fwd_points_batch: bad size");
  int rc = field_batch(dims, views, n_scenes, packed, tables, &a, n_points, "avr_field_fwd_points_batch");
  if (rc) return rc;
  AVR_REQUIRE(n_points == 0 || (xyz && viewdirs && out), "avr_field_fwd_points_batch: null pointer");
  a.xyz = xyz; a.vd = viewdirs; a.n_samples = 1;
  a.out = reinterpret_cast<float4*>(out);
  if (a.M == 0) return AVR_OK;
  return dispatch_field_x3(dims->d_hidden, a, as_stream(stream));
}

extern "C" int avr_field_fwd_points_split(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                                          const float* packed, const float* tables, const float* xyz,
                                          const float* viewdirs, int64_t n_points, int b_begin, int b_end,
                                          const float* h_in, float* h_out, float* out, void* stream) {
  FieldArgs a{};
  AVR_REQUIRE(n_points >= 0, "avr_field_fwd_points_split: bad size");
  int rc = field_batch(dims, views, n_scenes, packed, tables, &a, n_points, "avr_field_fwd_points_split");
  if (rc) return rc;
  const bool first = b_begin == 0;
  if (first) {
    AVR_REQUIRE(b_end > 0 && b_end < dims->n_blocks && b_end >= dims->n_lin_z,
                "avr_field_fwd_points_split: first launch needs n_lin_z <= b_end < n_blocks (got %d)", b_end);
    AVR_REQUIRE(n_points == 0 || (xyz && viewdirs && h_out), "avr_field_fwd_points_split: null pointer");
  } else {
    AVR_REQUIRE(b_begin >= dims->n_lin_z && b_begin < dims->n_blocks && b_end == dims->n_blocks,
                "avr_field_fwd_points_split: second launch needs n_lin_z <= b_begin < b_end == n_blocks");
    AVR_REQUIRE(n_points == 0 || (h_in && out), "avr_field_fwd_points_split: null pointer");
  }
  a.xyz = xyz; a.vd = viewdirs; a.n_samples = 1;
  a.b_begin = b_begin;
  a.b_end = b_end;
  a.h_in = first ? nullptr : h_in;
  a.h_out = first ? h_out : nullptr;
  a.out = reinterpret_cast<float4*>(out);
  if (a.M == 0) return AVR_OK;
  return dispatch_field_x3(dims->d_hidden, a, as_stream(stream));
}

extern "C" int avr_field_fwd_points(const avr_field_dims* dims, const avr_view_desc* view, const float* packed,
                                    const float* table, const float* xyz, const float* viewdirs, int64_t n_points,
                                    float* out, void* stream) {
  FieldArgs a{};
  int rc = field_common(dims, view, packed, table, &a);
  if (rc) return rc;
  AVR_REQUIRE(n_points >= 0, "avr_field_fwd_points: bad size");
  AVR_REQUIRE(n_points == 0 || (xyz && viewdirs && out), "avr_field_fwd_points: null pointer");
  a.xyz = xyz; a.vd = viewdirs; a.n_samples = 1;
  a.M = n_points;
  a.out = reinterpret_cast<float4*>(out);
  if (a.M == 0) return AVR_OK;
  return dispatch_field(dims, a, as_stream(stream));
}
