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
// input X (64 samples x HID) lives in LDS already split into fp16 hi/lo in
// B-fragment order [chunk][hi|lo][g][sample][8 x fp16]: one conflict-free
// ds_read_b128 pair per (chunk, sample group). Each layer's epilogue reads its
// accumulators once, applies bias/relu/scale, reduces the max for the next
// power-of-two scale, and writes the split operand (two barriers per layer).
// Accumulators stay in their scaled domain between layers (no unscale pass),
// and the bilinear lin_z gather for block b+1 streams in during block b's fc_0
// MFMAs (issued one K-chunk ahead, added into the residual).
#include "field_common.h"

// Contraction is fine for the field's own arithmetic (bias / interpolation /
// scaling); the geometry helpers use __f*_rn intrinsics, which never contract.
#pragma clang fp contract(fast)

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

// LDS X: 16-B slot (chunk c, part 0 = hi / 1 = lo, lane group g, sample s)
// holding the 8 fp16 B-operand elements e of that lane: feature
// 32c + 16*(e>>2) + 4g + (e&3). Writers place a tile's 4 values at byte 8*(tile&1).
__device__ __forceinline__ int xidx(int c, int part, int g, int s) { return ((c * 2 + part) * 4 + g) * 64 + s; }

struct BPair {
  half8 hi, lo;
};

__device__ __forceinline__ BPair read_b(const uint4* X16, int c, int sg, int g, int j) {
  BPair b;
  b.hi = __builtin_bit_cast(half8, X16[xidx(c, 0, g, 16 * sg + j)]);
  b.lo = __builtin_bit_cast(half8, X16[xidx(c, 1, g, 16 * sg + j)]);
  return b;
}

__device__ __forceinline__ void split4(const floatx4& x, uint2& hi, uint2& lo) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  half4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (_Float16)x[e];
    l[e] = (_Float16)(x[e] - (float)h[e]);
  }
  hi = __builtin_bit_cast(uint2, h);
  lo = __builtin_bit_cast(uint2, l);
}

// One K-chunk on resident A fragments: per sample group, the three products
// into each feature tile (one accumulation chain of v_mfma_f32_16x16x32_f16
// issues back to back at full rate, MI355X_MICROARCH.md). The B fragment of
// the next (chunk, sample group) is read from LDS one group ahead.
template <int FT, bool ZERO>
__device__ __forceinline__ void chunk_mfma(floatx4 (&acc)[FT][4], const FragX3 (&A)[FT], const uint4* X16, int c,
                                           int cn, BPair& B, int g, int j) {
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    const BPair Bn = read_b(X16, sg < 3 ? c : cn, (sg + 1) & 3, g, j);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      acc[ft][sg] = mfma32h(A[ft].hi, B.hi, ZERO ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].hi, B.lo, acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].lo, B.hi, acc[ft][sg]);
    }
    __builtin_amdgcn_sched_barrier(0);
    B = Bn;
  }
}

// acc += W . X over KC chunks (KC even, runtime). W points at this wave's
// first fragment of chunk 0; consecutive chunks are `cstride` fragments
// (32 B each) apart. A is double-buffered one chunk ahead in registers.
template <int FT>
__device__ __forceinline__ void gemm_x3(floatx4 (&acc)[FT][4], const uint4* __restrict__ W, int KC, int cstride,
                                        const uint4* X16, int lane) {
  const int g = lane >> 4, j = lane & 15;
  const uint4* wl = W + 2 * lane;
  FragX3 A0[FT], A1[FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) A0[ft] = load_frag(wl + 2 * 64 * ft);
  BPair B = read_b(X16, 0, 0, g, j);
  for (int c = 0; c < KC; c += 2) {
    const uint4* w1 = wl + (int64_t)2 * (c + 1) * cstride;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) A1[ft] = load_frag(w1 + 2 * 64 * ft);
    __builtin_amdgcn_sched_barrier(0);
    const int c2 = c + 2 < KC ? c + 2 : c + 1;
    chunk_mfma<FT, false>(acc, A0, X16, c, c + 1, B, g, j);
    const uint4* w2 = wl + (int64_t)2 * c2 * cstride;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) A0[ft] = load_frag(w2 + 2 * 64 * ft);
    __builtin_amdgcn_sched_barrier(0);
    chunk_mfma<FT, false>(acc, A1, X16, c + 1, c2, B, g, j);
  }
}

// Bilinear lin_z gather for one (feature tile, sample group) pair: 4 corner
// rows of this lane's 4 features.
struct Gath {
  floatx4 v[4];
};

__device__ __forceinline__ Gath issue_gather(const float* __restrict__ Zw, const int* bil_tex, int s) {
  const int4 tex = *reinterpret_cast<const int4*>(bil_tex + 4 * s);
  Gath G;
  G.v[0] = *reinterpret_cast<const floatx4*>(Zw + tex.x);
  G.v[1] = *reinterpret_cast<const floatx4*>(Zw + tex.y);
  G.v[2] = *reinterpret_cast<const floatx4*>(Zw + tex.z);
  G.v[3] = *reinterpret_cast<const floatx4*>(Zw + tex.w);
  return G;
}

__device__ __forceinline__ floatx4 blend(const Gath& G, const float* bil_w, int s, float scale) {
  const float4 w = *reinterpret_cast<const float4*>(bil_w + 4 * s);
  return (((G.v[0] * w.x + G.v[1] * w.y) + G.v[2] * w.z) + G.v[3] * w.w) * scale;
}

// t = W . X over KC = 2 FT chunks (compile-time, fully unrolled) starting from
// zero, while the lin_z gather of the next block streams into the residual h:
// chunk c issues the corner loads of pairs 2c, 2c+1 (feature tile c/2, sample
// groups 2(c&1), 2(c&1)+1) before its 96 MFMAs and blends them into h after.
// `Zw` = this lane's feature base of the next lin_z table (null: no gather);
// `zs` = h's accumulator scale.
template <int FT>
__device__ __forceinline__ void gemm_x3_fc0(floatx4 (&acc)[FT][4], floatx4 (&h)[FT][4], const uint4* __restrict__ W,
                                            int cstride, const uint4* X16, int lane, const float* __restrict__ Zw,
                                            const int* bil_tex, const float* bil_w, float zs) {
  constexpr int KC = 2 * FT;
  const int g = lane >> 4, j = lane & 15;
  const uint4* wl = W + 2 * lane;
  FragX3 A[2][FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) A[0][ft] = load_frag(wl + 2 * 64 * ft);
  BPair B = read_b(X16, 0, 0, g, j);
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int cur = c & 1, nxt = cur ^ 1;
    const int cn = c + 1 < KC ? c + 1 : c;
    const int ftp = c >> 1, sg0 = 2 * (c & 1);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) A[nxt][ft] = load_frag(wl + (int64_t)2 * cn * cstride + 2 * 64 * ft);
    Gath G0, G1;
    if (Zw) {
      G0 = issue_gather(Zw + 16 * ftp, bil_tex, 16 * sg0 + j);
      G1 = issue_gather(Zw + 16 * ftp, bil_tex, 16 * (sg0 + 1) + j);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (c == 0)
      chunk_mfma<FT, true>(acc, A[cur], X16, c, cn, B, g, j);
    else
      chunk_mfma<FT, false>(acc, A[cur], X16, c, cn, B, g, j);
    if (Zw) {
      h[ftp][sg0] += blend(G0, bil_w, 16 * sg0 + j, zs);
      h[ftp][sg0 + 1] += blend(G1, bil_w, 16 * (sg0 + 1) + j, zs);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// h += scale * interp(Z) for all of this wave's tiles (blocking, one sample group per batch)
template <int FT>
__device__ __forceinline__ void add_interp(floatx4 (&h)[FT][4], const float* __restrict__ Zw, const int* bil_tex,
                                           const float* bil_w, float scale, int j) {
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    Gath G[FT];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) G[ft] = issue_gather(Zw + 16 * ft, bil_tex, 16 * sg + j);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) h[ft][sg] += blend(G[ft], bil_w, 16 * sg + j, scale);
  }
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = fmaxf(v, __shfl_xor(v, d, 64));
  return v;
}

// v = relu(acc * f [+ bias]) (one read of the accumulators), returns the wave max
template <int FT, bool BIAS>
__device__ __forceinline__ float prep_input(floatx4 (&v)[FT][4], const floatx4 (&acc)[FT][4], float f,
                                            const float* __restrict__ bias, int wid, int g) {
  float mx = 0.f;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    floatx4 b = {0.f, 0.f, 0.f, 0.f};
    if (BIAS) b = *reinterpret_cast<const floatx4*>(bias + 16 * (FT * wid + ft) + 4 * g);
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      floatx4 x = BIAS ? acc[ft][sg] * f + b : acc[ft][sg] * f;
      x.x = fmaxf(x.x, 0.f); x.y = fmaxf(x.y, 0.f); x.z = fmaxf(x.z, 0.f); x.w = fmaxf(x.w, 0.f);
      v[ft][sg] = x;
      mx = fmaxf(fmaxf(mx, x.x), fmaxf(fmaxf(x.y, x.z), x.w));
    }
  }
  return wave_max(mx);
}

// X <- split(v * s_x) for this wave's feature tiles
template <int FT>
__device__ __forceinline__ void store_split(uint4* X16, const floatx4 (&v)[FT][4], float s_x, int wid, int g, int j) {
  char* base = reinterpret_cast<char*>(X16);
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const int ftg = FT * wid + ft;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      uint2 hi, lo;
      split4(v[ft][sg] * s_x, hi, lo);
      const int s = 16 * sg + j;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 0, g, s) * 16 + (ftg & 1) * 8) = hi;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 1, g, s) * 16 + (ftg & 1) * 8) = lo;
    }
  }
}

__device__ __forceinline__ float layer_scale(const float* packed, const Layout& L, int layer) {
  return pow2_scale_for(__uint_as_float(reinterpret_cast<const unsigned*>(packed + L.x3_hdr)[layer]));
}

__device__ __forceinline__ float red_max(const float* red) {
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// relu'd layer input -> LDS (two barriers: all reads of the previous X done /
// all writes of the new X visible); returns the operand scale s_x
template <int FT>
__device__ __forceinline__ float publish(uint4* X16, const floatx4 (&v)[FT][4], float mx, float* red, int wid,
                                         int lane, int g, int j) {
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  const float s_x = pow2_scale_for(red_max(red));
  store_split<FT>(X16, v, s_x, wid, g, j);
  __syncthreads();
  return s_x;
}

template <int FT>
__global__ void __launch_bounds__(256, 1) field_x3_kernel(FieldArgs a) {
  constexpr int KC = 2 * FT;                       // K chunks of a hidden layer (HID / 32)
  constexpr int KCX = KC > kX3InChunks ? KC : kX3InChunks;
  constexpr int NTT = 4 * FT;                      // feature tiles of a hidden layer
  constexpr int HID = 64 * FT;
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);      // KCX * 512 slots of 16 B
  int* bil_tex = reinterpret_cast<int*>(lds + KCX * 2048);   // [64][4] element offsets into a table
  float* bil_w = reinterpret_cast<float*>(bil_tex + 256);    // [64][4]
  float* red = bil_w + 256;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t base = (int64_t)blockIdx.x * kX3Samples;
  const Layout& L = a.L;
  const uint4* P16 = reinterpret_cast<const uint4*>(a.packed);  // 16-B units
  const int zoff = 16 * FT * wid + 4 * g;         // this lane's feature offset inside a table row

  AVR_STAMP(0);
  // ---- prologue: wave w prepares samples 16w + j (lanes g share the geometry);
  // lane g computes z_feature 16g .. 16g+15 of that sample (K = 64 padded input)
  floatx4 f[4];
  float mx = 0.f;
  {
    const int s = 16 * wid + j;
    const int64_t m = base + s;
    const SampleGeom geo = sample_geom(a, m < a.M ? m : a.M - 1);
    if (g == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) { bil_tex[4 * s + c] = geo.bl.tex[c] * HID; bil_w[4 * s + c] = geo.bl.w[c]; }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[q][e] = z_feature(geo, 16 * g + 4 * q + e, a.num_freqs, a.freq_factor);
        mx = fmaxf(mx, fabsf(f[q][e]));
      }
    mx = wave_max(mx);
  }
  AVR_STAMP(1);
  float s_x;
  {
    if (lane == 0) red[wid] = mx;
    __syncthreads();
    s_x = pow2_scale_for(red_max(red));
    // feature 16g + 4q + e: chunk g>>1, tile parity g&1, lane group q
    char* xb = reinterpret_cast<char*>(X16);
    const int s = 16 * wid + j;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint2 hi, lo;
      split4(f[q] * s_x, hi, lo);
      *reinterpret_cast<uint2*>(xb + xidx(g >> 1, 0, q, s) * 16 + (g & 1) * 8) = hi;
      *reinterpret_cast<uint2*>(xb + xidx(g >> 1, 1, q, s) * 16 + (g & 1) * 8) = lo;
    }
    __syncthreads();
  }

  AVR_STAMP(2);
  floatx4 h[FT][4], t[FT][4], v[FT][4];

  // ---- lin_in: h = (b_in + bz0 + interp(Z0)) * S + W_in . X ; h stays scaled by S_h
  float S_h = layer_scale(a.packed, L, 0) * s_x;
  {
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const floatx4 b = *reinterpret_cast<const floatx4*>(a.packed + L.b_in + 16 * (FT * wid + ft) + 4 * g);
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) h[ft][sg] = b * S_h;
    }
    if (a.n_lin_z > 0) add_interp<FT>(h, a.table + zoff, bil_tex, bil_w, S_h, j);
    AVR_STAMP(3);
    gemm_x3<FT>(h, P16 + L.x3_in / 4 + 2 * 64 * FT * wid, kX3InChunks, 64 * NTT, X16, lane);
    AVR_STAMP(4);
  }

  for (int b = 0; b < a.n_blocks; ++b) {
    // fc_0 input relu(h)
    mx = prep_input<FT, false>(v, h, 1.0f / S_h, nullptr, wid, g);
    s_x = publish<FT>(X16, v, mx, red, wid, lane, g, j);
    AVR_STAMP(5 + 5 * (b & 3));
    // fc_0 (from zero)
    const float S_t = layer_scale(a.packed, L, 2 + 2 * b) * s_x;
    const float* Zw = (b + 1 < a.n_lin_z) ? a.table + (b + 1) * a.table_stride + zoff : nullptr;
    gemm_x3_fc0<FT>(t, h, P16 + L.x3_fc0[b] / 4 + 2 * 64 * FT * wid, 64 * NTT, X16, lane, nullptr, bil_tex, bil_w,
                    S_h);
    AVR_STAMP(6 + 5 * (b & 3));
    // fc_1 input relu(t + b0)
    mx = prep_input<FT, true>(v, t, 1.0f / S_t, a.packed + L.b_fc0[b], wid, g);
    s_x = publish<FT>(X16, v, mx, red, wid, lane, g, j);
    AVR_STAMP(7 + 5 * (b & 3));
    // fc_1 accumulates onto the residual, rescaled to this layer's scale (+ b1 + bz[b+1])
    const float S1 = layer_scale(a.packed, L, 3 + 2 * b) * s_x;
    const float r = S1 / S_h;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const floatx4 bb = *reinterpret_cast<const floatx4*>(a.packed + L.b_fc1[b] + 16 * (FT * wid + ft) + 4 * g);
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) h[ft][sg] = h[ft][sg] * r + bb * S1;
    }
    if (Zw) add_interp<FT>(h, Zw, bil_tex, bil_w, S1, j);
    S_h = S1;
    AVR_STAMP(8 + 5 * (b & 3));
    gemm_x3<FT>(h, P16 + L.x3_fc1[b] / 4 + 2 * 64 * FT * wid, KC, 64 * NTT, X16, lane);
    AVR_STAMP(9 + 5 * (b & 3));
  }

  // ---- lin_out(relu(h)): wave w computes the 16-row output tile for samples 16w + j.
  FragX3 Ao[KC];
  {
    const uint4* wo = P16 + L.x3_out / 4 + 2 * lane;
#pragma unroll
    for (int c = 0; c < KC; ++c) Ao[c] = load_frag(wo + (int64_t)2 * 64 * c);
  }
  mx = prep_input<FT, false>(v, h, 1.0f / S_h, nullptr, wid, g);
  s_x = publish<FT>(X16, v, mx, red, wid, lane, g, j);
  AVR_STAMP(25);
  const float S = layer_scale(a.packed, L, 1) * s_x;
  floatx4 o = *reinterpret_cast<const floatx4*>(a.packed + L.b_out + 4 * g) * S;
  {
    const int s = 16 * wid + j;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const half8 bh = __builtin_bit_cast(half8, X16[xidx(c, 0, g, s)]);
      const half8 bl = __builtin_bit_cast(half8, X16[xidx(c, 1, g, s)]);
      o = mfma32h(Ao[c].hi, bh, o);
      o = mfma32h(Ao[c].hi, bl, o);
      o = mfma32h(Ao[c].lo, bh, o);
    }
  }
  o *= 1.0f / S;
  AVR_STAMP(26);
  const int64_t m = base + 16 * wid + j;
  if (g == 0 && m < a.M) a.out[m] = make_float4(sigmoidf_(o.x), sigmoidf_(o.y), sigmoidf_(o.z), fmaxf(o.w, 0.f));
}

template <int FT>
static int launch_x3(const FieldArgs& a, hipStream_t s) {
  constexpr int KC = 2 * FT;
  constexpr int KCX = KC > kX3InChunks ? KC : kX3InChunks;
  const size_t shm = (size_t)KCX * 2048 * sizeof(float) + 512 * sizeof(float) + 64;  // X + bilinear + red
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
