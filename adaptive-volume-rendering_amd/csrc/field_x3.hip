// Radiance field on split-fp16 MFMA ("x3"): the same function as
// field_fwd_kernel (models.py:739-863) with every ResnetFC product computed as
//   W.x ~= Wh.xh + Wh.xl + Wl.xh        (v_mfma_f32_16x16x32_f16, fp32 accumulate)
// where W*s_w = Wh + Wl and x*s_x = xh + xl are fp16 hi/lo splits under
// power-of-two scales (s_w per layer at pack time from max|W|; s_x per layer
// and per workgroup from max|x| at run time, so neither part can overflow and
// the lo parts stay normal). Products of fp16 values are exact in fp32, the
// dropped Wl.xl term and the split residuals are ~2^-22 relative: the result
// tracks the fp32 kernel to fp32 accumulation noise (tests/test_gpu_parity.py),
// at 16/3 x the fp32 MFMA rate.
//
// Work split: a 256-thread workgroup owns 64 samples; wave w owns output
// features [HID/4 * w, HID/4 * (w+1)) for all 64 samples, so each weight byte
// is fetched once per workgroup (each wave streams its own quarter of W from
// L2 straight into registers, double-buffered one K-chunk ahead). The layer
// input X (64 samples x HID, fp32) lives in LDS in B-fragment order
// [chunk][half][g][sample][4]: one conflict-free ds_read_b128 pair per
// (chunk, sample group), and accumulator tiles store back with one
// ds_write_b128 each. Two barriers per layer.
#include "field_common.h"

namespace avr {

struct FragX3 {
  half8 hi, lo;
};

__device__ __forceinline__ FragX3 load_frag(const uint4* p) {
  FragX3 f;
  const uint4 a = p[0], b = p[1];
  f.hi = __builtin_bit_cast(half8, a);
  f.lo = __builtin_bit_cast(half8, b);
  return f;
}

__device__ __forceinline__ void split8(const float4& x0, const float4& x1, float s, half8& hi, half8& lo) {
  const float v[8] = {x0.x * s, x0.y * s, x0.z * s, x0.w * s, x1.x * s, x1.y * s, x1.z * s, x1.w * s};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const _Float16 h = (_Float16)v[e];
    hi[e] = h;
    lo[e] = (_Float16)(v[e] - (float)h);
  }
}

// X element (chunk c, half, lane group g, sample s) as float4 index
__device__ __forceinline__ int xidx(int c, int half, int g, int s) { return ((c * 2 + half) * 4 + g) * 64 + s; }

// One K-chunk: for each sample group, split its B fragment once and run the
// three products into each feature tile's accumulator. A single accumulation
// chain of v_mfma_f32_16x16x32_f16 issues back to back at full rate
// (MI355X_MICROARCH.md), so the three products may target the same tile.
template <int FT>
__device__ __forceinline__ void chunk_mfma(floatx4 (&acc)[FT][4], const FragX3 (&A)[FT], const float4* X4, int c,
                                           float s_x, int g, int j) {
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    half8 bh, bl;
    split8(X4[xidx(c, 0, g, 16 * sg + j)], X4[xidx(c, 1, g, 16 * sg + j)], s_x, bh, bl);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      acc[ft][sg] = mfma32h(A[ft].hi, bh, acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].hi, bl, acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].lo, bh, acc[ft][sg]);
    }
  }
}

// acc[ft][sg] += sum over KC chunks; W points at this wave's first fragment of
// chunk 0, consecutive chunks are `cstride` fragments apart (32 B each).
template <int FT>
__device__ __forceinline__ void gemm_x3(floatx4 (&acc)[FT][4], const uint4* __restrict__ W, int KC, int cstride,
                                        const float4* X4, float s_x, int lane) {
  const int g = lane >> 4, j = lane & 15;
  const uint4* wl = W + 2 * lane;
  FragX3 A0[FT], A1[FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) A0[ft] = load_frag(wl + 2 * 64 * ft);
  for (int c = 0; c < KC; c += 2) {
    const uint4* w1 = wl + (int64_t)2 * (c + 1) * cstride;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) A1[ft] = load_frag(w1 + 2 * 64 * ft);
    chunk_mfma<FT>(acc, A0, X4, c, s_x, g, j);
    const uint4* w2 = wl + (int64_t)2 * (c + 2 < KC ? c + 2 : c + 1) * cstride;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) A0[ft] = load_frag(w2 + 2 * 64 * ft);
    chunk_mfma<FT>(acc, A1, X4, c + 1, s_x, g, j);
  }
}

// Store relu(acc * inv) into X (this wave's feature tiles), return local max.
template <int FT>
__device__ __forceinline__ float store_x(float4* X4, const floatx4 (&acc)[FT][4], float inv, int wid, int g, int j) {
  float mx = 0.f;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const int ftg = FT * wid + ft;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 v = acc[ft][sg] * inv;
      const float4 r = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
      mx = fmaxf(mx, fmaxf(fmaxf(r.x, r.y), fmaxf(r.z, r.w)));
      X4[xidx(ftg >> 1, ftg & 1, g, 16 * sg + j)] = r;
    }
  }
  return mx;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = fmaxf(v, __shfl_xor(v, d, 64));
  return v;
}

// acc = ((ACCUM ? acc : 0) + bias [+ interp(Z)]) * S for this wave's features
template <int FT, bool ACCUM>
__device__ __forceinline__ void init_acc(floatx4 (&acc)[FT][4], const float* __restrict__ bias,
                                         const float* __restrict__ Z, const int* bil_tex, const float* bil_w,
                                         float S, int wid, int g, int j) {
  constexpr int HID = 64 * FT;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const floatx4 b = *reinterpret_cast<const floatx4*>(bias + 16 * (FT * wid + ft) + 4 * g);
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) acc[ft][sg] = ACCUM ? acc[ft][sg] + b : b;
  }
  if (Z) {
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const int s = 16 * sg + j;
      int tex[4];
      float w[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) { tex[c] = bil_tex[4 * s + c]; w[c] = bil_w[4 * s + c]; }
      floatx4 v[FT][4];
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          v[ft][c] = *reinterpret_cast<const floatx4*>(Z + (int64_t)tex[c] * HID + 16 * (FT * wid + ft) + 4 * g);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
        acc[ft][sg] += ((w[0] * v[ft][0] + w[1] * v[ft][1]) + w[2] * v[ft][2]) + w[3] * v[ft][3];
    }
  }
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) acc[ft][sg] *= S;
}

__device__ __forceinline__ float layer_scale(const float* packed, const Layout& L, int layer) {
  return pow2_scale_for(__uint_as_float(reinterpret_cast<const unsigned*>(packed + L.x3_hdr)[layer]));
}

template <int FT>
__global__ void __launch_bounds__(256, 1) field_x3_kernel(FieldArgs a) {
  constexpr int KC = 2 * FT;                       // K chunks of a hidden layer (HID / 32)
  constexpr int KCX = KC > kX3InChunks ? KC : kX3InChunks;
  constexpr int NTT = 4 * FT;                      // feature tiles of a hidden layer
  extern __shared__ float lds[];
  float4* X4 = reinterpret_cast<float4*>(lds);
  int* bil_tex = reinterpret_cast<int*>(lds + KCX * 2048);
  float* bil_w = reinterpret_cast<float*>(bil_tex + 256);
  float* red = bil_w + 256;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t base = (int64_t)blockIdx.x * kX3Samples;
  const Layout& L = a.L;
  const uint4* P16 = reinterpret_cast<const uint4*>(a.packed);  // 16-B units

  // ---- prologue: wave w prepares samples 16w + j (lanes g share the geometry)
  {
    const int s = 16 * wid + j;
    const int64_t m = base + s;
    const SampleGeom geo = sample_geom(a, m < a.M ? m : a.M - 1);
    if (g == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) { bil_tex[4 * s + c] = geo.bl.tex[c]; bil_w[4 * s + c] = geo.bl.w[c]; }
    }
    float mx = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // features 16g + 4q + e -> X[c = g>>1][half = g&1][q][s][e]
      float f[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = z_feature(geo, 16 * g + 4 * q + e, a.num_freqs, a.freq_factor);
        mx = fmaxf(mx, fabsf(f[e]));
      }
      X4[xidx(g >> 1, g & 1, q, s)] = make_float4(f[0], f[1], f[2], f[3]);
    }
    mx = wave_max(mx);
    if (lane == 0) red[wid] = mx;
  }
  __syncthreads();
  float s_x = pow2_scale_for(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));

  floatx4 h[FT][4], t[FT][4];

  // ---- lin_in (+ lin_z[0] + biases)
  {
    const float S = layer_scale(a.packed, L, 0) * s_x;
    init_acc<FT, false>(h, a.packed + L.b_in, a.n_lin_z > 0 ? a.table : nullptr, bil_tex, bil_w, S, wid, g, j);
    gemm_x3<FT>(h, P16 + L.x3_in / 4 + 2 * 64 * FT * wid, kX3InChunks, 64 * NTT, X4, s_x, lane);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) h[ft][sg] *= 1.0f / S;
  }

  for (int b = 0; b < a.n_blocks; ++b) {
    // relu(h) -> X
    __syncthreads();
    float mx = wave_max(store_x<FT>(X4, h, 1.0f, wid, g, j));
    if (lane == 0) red[wid] = mx;
    __syncthreads();
    s_x = pow2_scale_for(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
    // fc_0
    float S = layer_scale(a.packed, L, 2 + 2 * b) * s_x;
    init_acc<FT, false>(t, a.packed + L.b_fc0[b], nullptr, bil_tex, bil_w, S, wid, g, j);
    gemm_x3<FT>(t, P16 + L.x3_fc0[b] / 4 + 2 * 64 * FT * wid, KC, 64 * NTT, X4, s_x, lane);
    // relu(t) -> X
    __syncthreads();
    mx = wave_max(store_x<FT>(X4, t, 1.0f / S, wid, g, j));
    if (lane == 0) red[wid] = mx;
    __syncthreads();
    s_x = pow2_scale_for(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
    // fc_1 accumulates onto the residual (+ b1 + bz[b+1] + interp(Z[b+1]))
    S = layer_scale(a.packed, L, 3 + 2 * b) * s_x;
    init_acc<FT, true>(h, a.packed + L.b_fc1[b], (b + 1 < a.n_lin_z) ? a.table + (b + 1) * a.table_stride : nullptr,
                 bil_tex, bil_w, S, wid, g, j);
    gemm_x3<FT>(h, P16 + L.x3_fc1[b] / 4 + 2 * 64 * FT * wid, KC, 64 * NTT, X4, s_x, lane);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) h[ft][sg] *= 1.0f / S;
  }

  // ---- lin_out(relu(h)): wave w computes the 16-row output tile for samples 16w + j
  __syncthreads();
  float mx = wave_max(store_x<FT>(X4, h, 1.0f, wid, g, j));
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  s_x = pow2_scale_for(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  const float S = layer_scale(a.packed, L, 1) * s_x;
  floatx4 o = *reinterpret_cast<const floatx4*>(a.packed + L.b_out + 4 * g) * S;
  {
    const uint4* wo = P16 + L.x3_out / 4 + 2 * lane;
    for (int c = 0; c < KC; ++c) {
      const FragX3 A = load_frag(wo + (int64_t)2 * 64 * c);
      half8 bh, bl;
      const int s = 16 * wid + j;
      split8(X4[xidx(c, 0, g, s)], X4[xidx(c, 1, g, s)], s_x, bh, bl);
      o = mfma32h(A.hi, bh, o);
      o = mfma32h(A.hi, bl, o);
      o = mfma32h(A.lo, bh, o);
    }
  }
  o *= 1.0f / S;
  const int64_t m = base + 16 * wid + j;
  if (g == 0 && m < a.M) a.out[m] = make_float4(sigmoidf_(o.x), sigmoidf_(o.y), sigmoidf_(o.z), fmaxf(o.w, 0.f));
}

template <int FT>
static int launch_x3(const FieldArgs& a, hipStream_t s) {
  constexpr int KC = 2 * FT;
  constexpr int KCX = KC > kX3InChunks ? KC : kX3InChunks;
  const size_t shm = (size_t)KCX * 2048 * sizeof(float) + 512 * sizeof(float) + 64;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&field_x3_kernel<FT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return fail(AVR_E_HIP, "field_x3_kernel: cannot set dynamic LDS to %zu", shm);
    attr = true;
  }
  const int64_t blocks = (a.M + kX3Samples - 1) / kX3Samples;
  AVR_REQUIRE(blocks < (1ll << 31), "field: too many points");
  field_x3_kernel<FT><<<(unsigned)blocks, 64 * kFieldWaves, shm, s>>>(a);
  return check_launch("field_x3_kernel");
}

int dispatch_field_x3(int d_hidden, const FieldArgs& a, hipStream_t s) {
  switch (d_hidden) {
    case 64: return launch_x3<1>(a, s);
    case 128: return launch_x3<2>(a, s);
    case 256: return launch_x3<4>(a, s);
    case 512: return launch_x3<8>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "field x3: d_hidden %d", d_hidden);
}

}  // namespace avr
