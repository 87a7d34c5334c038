// Split-fp16 ("x3") MFMA building blocks shared by the field forward
// (field_x3.hip) and backward (field_bwd.hip) kernels: the LDS operand layout,
// the hi/lo split, the K-chunk GEMM loop with weights streamed one chunk ahead,
// and the publish step that turns a layer's register values into the next
// GEMM's LDS operand.
#pragma once
#include "field_common.h"

// Contraction is fine for the field's own arithmetic (bias / interpolation /
// scaling); the geometry helpers use __f*_rn intrinsics, which never contract.
#pragma clang fp contract(fast)

namespace avr {

struct FragX3 {
  half8 hi, lo;
};

// p = tile base + lane (uint4 units); the tile holds its 64 lanes' hi halves,
// then their lo halves (pack_x3_kernel), so each half loads 1 KiB contiguous.
__device__ __forceinline__ FragX3 load_frag(const uint4* p) {
  FragX3 f;
  const uint4 a = p[0], b = p[64];
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

// hi = fp16(x*s), lo = fp16(x*s - hi): one packed convert per pair for hi and
// one v_fma_mix{lo,hi}_f16 per value for lo (x*s is exact: s is a power of two)
__device__ __forceinline__ void split4(const floatx4& x, float s, uint2& hi, uint2& lo) {
  const floatx4 y = x * s;
  unsigned h0, h1, l0, l1;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h0) : "v"(y.x), "v"(y.y));
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h1) : "v"(y.z), "v"(y.w));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l0) : "v"(x.x), "v"(s), "v"(h0));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l0) : "v"(x.y), "v"(s), "v"(h0));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l1) : "v"(x.z), "v"(s), "v"(h1));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l1) : "v"(x.w), "v"(s), "v"(h1));
  hi = make_uint2(h0, h1);
  lo = make_uint2(l0, l1);
}

// Side task of a GEMM (the backward kernel, RowSideH): copy the GEMM's own operand X out of
// LDS as fp32 rows while the MFMAs run, so the row stores spread over the K
// loop instead of bursting ahead of it (a burst queues in front of the next
// weight loads: vmcnt retires in order). NoSide: inference.
struct NoSide {
  __device__ __forceinline__ void load(const uint4*, int) {}
  __device__ __forceinline__ void store(int) {}
};

// Lane (g, j) of wave w copies slot pair (chunk c, g, sample 16 w + j) of X:
// features 32c + 4g .. +3 and 32c + 16 + 4g .. +3 of that sample, each value
// (hi + lo) / s_x -- the operand the GEMM multiplies (exact in fp32: hi and lo
// hold <= 22 significant bits together; 1 / s_x is a power of two). Only
// wave-uniform fields (SGPRs): the lane's sample and group are re-derived
// from its id at each use, so the task holds just the 8 VGPRs in flight.
struct RowSide {
  __amdgpu_buffer_rsrc_t rows;   // rows of the workgroup's samples 0 .. nvalid-1 (raw buffer: stores
                                 // past the last existing row are dropped by the hardware, no branch)
  float inv;                     // 1 / s_x
  int wid;
  uint4 h, l;
  template <int HID>
  __device__ __forceinline__ void init(float* rows0, float s_x, int64_t nrows, int w) {
    const int nvalid = nrows < 64 ? (int)nrows : 64;
    rows = __builtin_amdgcn_make_buffer_rsrc(rows0, 0, nvalid * HID * 4, 0x00020000);
    inv = 1.0f / s_x;
    wid = w;
  }
  __device__ __forceinline__ void load(const uint4* X16, int c) {
    const int lane = __lane_id(), s = 16 * wid + (lane & 15), g = lane >> 4;
    h = X16[xidx(c, 0, g, s)];
    l = X16[xidx(c, 1, g, s)];
  }
  template <int HID>
  __device__ __forceinline__ void store_hid(int c) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int lane = __lane_id(), s = 16 * wid + (lane & 15), g = lane >> 4;
    const half8 hh = __builtin_bit_cast(half8, h), ll = __builtin_bit_cast(half8, l);
    floatx4 a, b;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = ((float)hh[e] + (float)ll[e]) * inv;
      b[e] = ((float)hh[e + 4] + (float)ll[e + 4]) * inv;
    }
    const int off = 4 * (s * HID + 32 * c + 4 * g);
    // non-temporal (aux bit 1 = nt): the rows stream through once; allocated in L2 they evict the weights
    // (scripts/gpu_train_prof.sh sweep of sc0 / sc1 / nt: nt alone is fastest, 3.69 -> 2.94 ms per
    // default_mv fine-pass backward)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rows, off, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), rows, off + 64, 0, 2);
  }
};

template <int HID>
struct RowSideH : RowSide {
  __device__ __forceinline__ void store(int c) { store_hid<HID>(c); }
};

// One K-chunk on resident fragments A (this wave's FT tiles) and B (the 4
// sample groups), in feature-tile pairs: pair p issues its 3 x 2 x 4 chained
// v_mfma_f32_16x16x32_f16 (each accumulation chain issues back to back at full
// rate, MI355X_MICROARCH.md) and the global loads of pair p of the NEXT chunk
// into An, one load per few MFMAs (sched_group_barrier), so every A load has a
// whole chunk of MFMAs to land in and its issue hides in the MFMA gaps. In the
// last pair each B[sg] is refilled with the next chunk's fragment as soon as
// its MFMAs have issued. The side task reads its slots of chunk cc in pair 0
// and converts / stores them in pair 1 (in pair 0's tail for a single pair).
template <int FT, bool ZERO, typename Side = NoSide>
__device__ __forceinline__ void chunk_step(floatx4 (&acc)[FT][4], const FragX3 (&A)[FT], FragX3 (&An)[FT],
                                           const uint4* wn, BPair (&B)[4], const uint4* X16, int cn, int g, int j,
                                           Side& side, int cc) {
  constexpr int GS = FT >= 2 ? 2 : 1;       // tiles per group
  constexpr int NG = FT / GS;
  constexpr int NMF = 3 * GS * 4;           // MFMAs per group
  constexpr int NLD = 2 * GS;               // global loads per group
  constexpr int PER = NMF / (NLD + 1);
#pragma unroll
  for (int p = 0; p < NG; ++p) {
    if (p == 0) side.load(X16, cc);
#pragma unroll
    for (int q = 0; q < GS; ++q) An[GS * p + q] = load_frag(wn + 2 * 64 * (GS * p + q));
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
#pragma unroll
      for (int q = 0; q < GS; ++q) {
        const int ft = GS * p + q;
        acc[ft][sg] = mfma32h(A[ft].hi, B[sg].hi, ZERO ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[ft][sg]);
        acc[ft][sg] = mfma32h(A[ft].hi, B[sg].lo, acc[ft][sg]);
        acc[ft][sg] = mfma32h(A[ft].lo, B[sg].hi, acc[ft][sg]);
      }
      if (p == NG - 1) B[sg] = read_b(X16, cn, sg, g, j);
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NLD * PER, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  side.store(cc);
}

// acc (+)= W . X over KC chunks (KC even, runtime; ZERO: acc starts from 0).
// W points at this wave's first fragment of chunk 0; consecutive chunks are
// `cstride` fragments (32 B each) apart. A is double-buffered one chunk ahead
// in registers (the last chunk reloads itself: harmless, keeps the pattern).
// This wave's chunk-0 A fragments of a layer, loaded ahead of the layer
// (before the publish that precedes it) so the GEMM starts on landed data.
// Only the first kPrefetch tiles (the first group of chunk 0) are prefetched:
// more would push the epilogue into spills, and a scratch store waits for
// every outstanding load.
// (The 8-wave layout, 4 tiles per wave, prefetches all of them: NPF = FT.)
constexpr int kPrefetch = 2;

template <int FT, int NPF = kPrefetch>
__device__ __forceinline__ void prefetch_a(FragX3 (&A0)[FT], const uint4* __restrict__ W, int lane) {
#pragma unroll
  for (int ft = 0; ft < (FT < NPF ? FT : NPF); ++ft) A0[ft] = load_frag(W + (unsigned)(lane + 2 * 64 * ft));
}

// A0 holds chunk 0 (prefetch_a). side: an optional side task per K-chunk (RowSide).
template <int FT, bool ZERO, bool SYNC, typename Side = NoSide>
__device__ __forceinline__ void gemm_x3(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* __restrict__ W, int KC,
                                        int cstride, const uint4* X16, int lane, Side side = Side{}) {
  const int g = lane >> 4, j = lane & 15;
  const uint4* wl = W + lane;
  FragX3 A1[FT];
  BPair B[4];
#pragma unroll
  for (int ft = kPrefetch; ft < FT; ++ft) A0[ft] = load_frag(wl + 2 * 64 * ft);
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) B[sg] = read_b(X16, 0, sg, g, j);
  __builtin_amdgcn_sched_barrier(0);
  for (int c = 0; c < KC; c += 2) {
    const int c2 = c + 2 < KC ? c + 2 : c + 1;
    const uint4* w1 = wl + (int64_t)2 * (c + 1) * cstride;
    const uint4* w2 = wl + (int64_t)2 * c2 * cstride;
    if (ZERO && c == 0)
      chunk_step<FT, true>(acc, A0, A1, w1, B, X16, c + 1, g, j, side, c);
    else
      chunk_step<FT, false>(acc, A0, A1, w1, B, X16, c + 1, g, j, side, c);
    chunk_step<FT, false>(acc, A1, A0, w2, B, X16, c2, g, j, side, c + 1);
    // two waves per SIMD: the older one would otherwise win the MFMA pipe and
    // run a whole layer ahead, leaving its partner's epilogue unoverlapped;
    // a plain barrier every two chunks keeps them in step (the MFMA pipe stays
    // busy with the lagging wave meanwhile)
    if (SYNC) __builtin_amdgcn_s_barrier();
  }
}

// 8-wave variant of the K-chunk loop (256 registers per wave): sample groups
// outermost, so only the current and the next B fragment pair are resident
// (16 registers instead of 32); the next chunk's A fragment of tile sg loads
// during sample group sg (FT == 4: one tile per group).
template <int FT, bool ZERO>
__device__ __forceinline__ void chunk_step_sg(floatx4 (&acc)[FT][4], const FragX3 (&A)[FT], FragX3 (&An)[FT],
                                              const uint4* __restrict__ wn, unsigned lo, BPair& B, const uint4* X16,
                                              int c, int cn, int g, int j) {
  static_assert(FT == 4, "one next-chunk tile per sample group");
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    const BPair Bn = sg < 3 ? read_b(X16, c, sg + 1, g, j) : read_b(X16, cn, 0, g, j);
    An[sg] = load_frag(wn + (lo + 2 * 64 * sg));   // wave-uniform base + 32-bit lane offset
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      acc[ft][sg] = mfma32h(A[ft].hi, B.hi, ZERO ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].hi, B.lo, acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].lo, B.hi, acc[ft][sg]);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    B = Bn;
  }
}

// A0 holds chunk 0's first NPF tiles (prefetch_a<FT, NPF>). No barrier in the
// loop: the two waves of a SIMD drift apart by priority (field_x3_kernel).
template <int FT, bool ZERO, int NPF = FT>
__device__ __forceinline__ void gemm_x3_sg(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* __restrict__ W,
                                           int KC, int cstride, const uint4* X16, int lane) {
  const int g = lane >> 4, j = lane & 15;
  const unsigned lo = lane;          // W (wave-uniform) + lo: this lane's fragment
  FragX3 A1[FT];
#pragma unroll
  for (int ft = NPF; ft < FT; ++ft) A0[ft] = load_frag(W + (lo + 2 * 64 * ft));
  BPair B = read_b(X16, 0, 0, g, j);
  __builtin_amdgcn_sched_barrier(0);
  for (int c = 0; c < KC; c += 2) {
    const int c2 = c + 2 < KC ? c + 2 : c + 1;
    const uint4* w1 = W + (int64_t)2 * (c + 1) * cstride;
    const uint4* w2 = W + (int64_t)2 * c2 * cstride;
    if (ZERO && c == 0)
      chunk_step_sg<FT, true>(acc, A0, A1, w1, lo, B, X16, c, c + 1, g, j);
    else
      chunk_step_sg<FT, false>(acc, A0, A1, w1, lo, B, X16, c, c + 1, g, j);
    chunk_step_sg<FT, false>(acc, A1, A0, w2, lo, B, X16, c + 1, c2, g, j);
  }
}

// The 8-wave K loop with a side task (the backward chain's G rows, RowSide8): chunk_step_sg plus the task's LDS
// read of chunk c in sample group 0 and its row stores in sample group 2.
template <int FT, bool ZERO, typename Side>
__device__ __forceinline__ void chunk_step_sg_side(floatx4 (&acc)[FT][4], const FragX3 (&A)[FT], FragX3 (&An)[FT],
                                                   const uint4* __restrict__ wn, unsigned lo, BPair& B,
                                                   const uint4* X16, int c, int cn, int g, int j, Side& side) {
  static_assert(FT == 4, "one next-chunk tile per sample group");
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    if (sg == 0) side.load(X16, c);
    const BPair Bn = sg < 3 ? read_b(X16, c, sg + 1, g, j) : read_b(X16, cn, 0, g, j);
    An[sg] = load_frag(wn + (lo + 2 * 64 * sg));
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      acc[ft][sg] = mfma32h(A[ft].hi, B.hi, ZERO ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].hi, B.lo, acc[ft][sg]);
      acc[ft][sg] = mfma32h(A[ft].lo, B.hi, acc[ft][sg]);
    }
    if (sg == 2) side.store(c);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    B = Bn;
  }
}

template <int FT, bool ZERO, typename Side>
__device__ __forceinline__ void gemm_x3_sg_side(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* __restrict__ W,
                                                int KC, int cstride, const uint4* X16, int lane, Side side) {
  const int g = lane >> 4, j = lane & 15;
  const unsigned lo = lane;
  FragX3 A1[FT];
  BPair B = read_b(X16, 0, 0, g, j);
  __builtin_amdgcn_sched_barrier(0);
  for (int c = 0; c < KC; c += 2) {
    const int c2 = c + 2 < KC ? c + 2 : c + 1;
    const uint4* w1 = W + (int64_t)2 * (c + 1) * cstride;
    const uint4* w2 = W + (int64_t)2 * c2 * cstride;
    if (ZERO && c == 0)
      chunk_step_sg_side<FT, true>(acc, A0, A1, w1, lo, B, X16, c, c + 1, g, j, side);
    else
      chunk_step_sg_side<FT, false>(acc, A0, A1, w1, lo, B, X16, c, c + 1, g, j, side);
    chunk_step_sg_side<FT, false>(acc, A1, A0, w2, lo, B, X16, c + 1, c2, g, j, side);
  }
}

// RowSide for 8 waves: waves w and w + 4 share sample 16 (w & 3) + j; wave w copies the K-chunks of parity w >> 2
template <int HID>
struct RowSide8 : RowSide {
  int par;
  __device__ __forceinline__ void init8(float* rows0, float s_x, int64_t nrows, int w) {
    init<HID>(rows0, s_x, nrows, w & 3);
    par = w >> 2;
  }
  __device__ __forceinline__ void load(const uint4* X16, int c) {
    if ((c & 1) == par) RowSide::load(X16, c);
  }
  __device__ __forceinline__ void store(int c) {
    if ((c & 1) == par) store_hid<HID>(c);
  }
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not
// for its outstanding global loads (the next layer's weight prefetch stays in
// flight; __syncthreads would drain it).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = fmaxf(v, __shfl_xor(v, d, 64));
  return v;
}

// The MLP's activation (models.py:442-445, 536-537): ACT 0 = ReLU, 1 = Softplus(beta) as torch computes it in
// fp32 (x where beta * x > 20, else log1p(exp(beta * x)) / beta).
template <int ACT>
__device__ __forceinline__ float act1(float x, float beta) {
  if constexpr (ACT == 0) {
    return fmaxf(x, 0.f);
  } else {
    const float bx = x * beta;
    return bx > 20.f ? x : log1pf(expf(bx)) / beta;
  }
}

template <int ACT>
__device__ __forceinline__ floatx4 act4(floatx4 x, float beta) {
  if constexpr (ACT == 0) {
    x.x = fmaxf(x.x, 0.f); x.y = fmaxf(x.y, 0.f); x.z = fmaxf(x.z, 0.f); x.w = fmaxf(x.w, 0.f);
    return x;
  } else {
    return floatx4{act1<1>(x.x, beta), act1<1>(x.y, beta), act1<1>(x.z, beta), act1<1>(x.w, beta)};
  }
}

// Upper bound of act over values whose max(0, max) is m (both activations increase monotonically): the
// operand scale of a layer input from the max-of-relu its epilogue reduces.
template <int ACT>
__device__ __forceinline__ float act_bound(float m, float beta) {
  return ACT == 0 ? m : act1<1>(m, beta);
}

// v = act(acc * f [+ bias]) (one read of the accumulators), returns the wave max of max(0, acc * f [+ bias])
// (act_bound gives the bound of v)
template <int FT, bool BIAS, int ACT = 0>
__device__ __forceinline__ float prep_input(floatx4 (&v)[FT][4], const floatx4 (&acc)[FT][4], float f,
                                            const float* __restrict__ bias, int wid, int g, float beta = 0.f) {
  float mx = 0.f;
  floatx4 bv[FT];   // all bias loads first (one wait, not one per tile)
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
    bv[ft] = BIAS ? *reinterpret_cast<const floatx4*>(bias + 16 * (FT * wid + ft) + 4 * g) : floatx4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const floatx4 b = bv[ft];
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 x = BIAS ? acc[ft][sg] * f + b : acc[ft][sg] * f;
      const floatx4 y = act4<ACT>(x, beta);
      v[ft][sg] = y;
      const floatx4 m = ACT == 0 ? y : x;   // mx starts at 0: max relu (ReLU: from the stored values)
      mx = fmaxf(fmaxf(mx, m.x), fmaxf(fmaxf(m.y, m.z), m.w));
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
      split4(v[ft][sg], s_x, hi, lo);
      const int s = 16 * sg + j;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 0, g, s) * 16 + (ftg & 1) * 8) = hi;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 1, g, s) * 16 + (ftg & 1) * 8) = lo;
    }
  }
}

// ---- Two-pass epilogue (8-wave workgroups, 256 registers per wave: no room
// for a materialised copy v of the layer input). Pass 1 reduces the max of
// relu(acc * f + b); pass 2 recomputes each value and writes its split.
template <int FT, bool BIAS>
__device__ __forceinline__ void load_bias(floatx4 (&bv)[FT], const float* __restrict__ bias, int wid, int g) {
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
    bv[ft] = BIAS ? *reinterpret_cast<const floatx4*>(bias + 16 * (FT * wid + ft) + 4 * g) : floatx4{0.f, 0.f, 0.f, 0.f};
}

template <bool BIAS, int ACT = 0>
__device__ __forceinline__ floatx4 relu_affine(const floatx4& a, float f, const floatx4& b, float beta = 0.f) {
  return act4<ACT>(BIAS ? a * f + b : a * f, beta);
}

// max relu(x_i) = max(0, max x_i): no per-value relu (mx starts at 0)
template <int FT, bool BIAS>
__device__ __forceinline__ float max_relu_affine(const floatx4 (&acc)[FT][4], float f, const floatx4 (&bv)[FT]) {
  float mx = 0.f;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 x = BIAS ? acc[ft][sg] * f + bv[ft] : acc[ft][sg] * f;
      mx = fmaxf(mx, fmaxf(x.x, x.y));
      mx = fmaxf(mx, fmaxf(x.z, x.w));
    }
  return wave_max(mx);
}

// X <- split(act(acc * f + b) * s_x) for this wave's feature tiles
template <int FT, bool BIAS, int ACT = 0>
__device__ __forceinline__ void store_split_affine(uint4* X16, const floatx4 (&acc)[FT][4], float f,
                                                   const floatx4 (&bv)[FT], float s_x, int wid, int g, int j,
                                                   float beta = 0.f) {
  char* base = reinterpret_cast<char*>(X16);
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const int ftg = FT * wid + ft;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      uint2 hi, lo;
      split4(relu_affine<BIAS, ACT>(acc[ft][sg], f, bv[ft], beta), s_x, hi, lo);
      const int s = 16 * sg + j;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 0, g, s) * 16 + (ftg & 1) * 8) = hi;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 1, g, s) * 16 + (ftg & 1) * 8) = lo;
    }
  }
}

// ---- Eval-mode BatchNorm in front of fc_0's relu (train.py --bn; ResnetBlockFC.bn_0,
// models.py:456-458): relu(a * x + c) per feature of the residual stream x = acc * f,
// with this lane's (a, c) loaded per feature tile (bn_a / bn_c: d_hidden floats in the
// packed blob). The second bn_0 (in front of fc_1's relu) is folded into fc_0 at pack time.
template <int FT>
__device__ __forceinline__ void bn_tile(floatx4& a4, floatx4& c4, const float* __restrict__ bn_a,
                                        const float* __restrict__ bn_c, float f, int wid, int ft, int g) {
  const int o = 16 * (FT * wid + ft) + 4 * g;
  a4 = *reinterpret_cast<const floatx4*>(bn_a + o) * f;
  c4 = *reinterpret_cast<const floatx4*>(bn_c + o);
}

template <int FT>
__device__ __forceinline__ float max_relu_bn(const floatx4 (&acc)[FT][4], float f, const float* __restrict__ bn_a,
                                             const float* __restrict__ bn_c, int wid, int g) {
  float mx = 0.f;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    floatx4 a4, c4;
    bn_tile<FT>(a4, c4, bn_a, bn_c, f, wid, ft, g);
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 x = acc[ft][sg] * a4 + c4;
      mx = fmaxf(mx, fmaxf(x.x, x.y));
      mx = fmaxf(mx, fmaxf(x.z, x.w));
    }
  }
  return wave_max(mx);
}

// v = relu(acc * f * a + c) (4-wave layouts, materialised layer input); returns the wave max
template <int FT>
__device__ __forceinline__ float prep_bn(floatx4 (&v)[FT][4], const floatx4 (&acc)[FT][4], float f,
                                         const float* __restrict__ bn_a, const float* __restrict__ bn_c, int wid,
                                         int g) {
  float mx = 0.f;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    floatx4 a4, c4;
    bn_tile<FT>(a4, c4, bn_a, bn_c, f, wid, ft, g);
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      floatx4 x = acc[ft][sg] * a4 + c4;
      x.x = fmaxf(x.x, 0.f); x.y = fmaxf(x.y, 0.f); x.z = fmaxf(x.z, 0.f); x.w = fmaxf(x.w, 0.f);
      v[ft][sg] = x;
      mx = fmaxf(fmaxf(mx, x.x), fmaxf(fmaxf(x.y, x.z), x.w));
    }
  }
  return wave_max(mx);
}

__device__ __forceinline__ float layer_scale(const float* packed, const Layout& L, int layer) {
  return pow2_scale_for(__uint_as_float(reinterpret_cast<const unsigned*>(packed + L.x3_hdr)[layer]));
}

template <int NW>
__device__ __forceinline__ float red_max(const float* red) {
  float m = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
  return m;
}

// relu'd layer input -> LDS (two barriers: all reads of the previous X done /
// all writes of the new X visible); returns the operand scale s_x
// wgmax (training kernels): wave 0 records the workgroup's max there (LDS)
template <int FT, int NW>
__device__ __forceinline__ float publish(uint4* X16, const floatx4 (&v)[FT][4], float mx, float* red, int wid,
                                         int lane, int g, int j, float* wgmax = nullptr) {
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float m = red_max<NW>(red);
  if (wgmax && wid == 0 && lane == 0) *wgmax = m;
  const float s_x = pow2_scale_for(m);
  store_split<FT>(X16, v, s_x, wid, g, j);
  lds_barrier();
  return s_x;
}

// Two-pass publish of relu(acc * f * a + c) per feature (mx from max_relu_bn); returns s_x
template <int FT, int NW>
__device__ __forceinline__ float publish_bn(uint4* X16, const floatx4 (&acc)[FT][4], float f,
                                            const float* __restrict__ bn_a, const float* __restrict__ bn_c, float mx,
                                            float* red, int wid, int lane, int g, int j) {
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float s_x = pow2_scale_for(red_max<NW>(red));
  char* base = reinterpret_cast<char*>(X16);
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    floatx4 a4, c4;
    bn_tile<FT>(a4, c4, bn_a, bn_c, f, wid, ft, g);
    const int ftg = FT * wid + ft;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      floatx4 x = acc[ft][sg] * a4 + c4;
      x.x = fmaxf(x.x, 0.f); x.y = fmaxf(x.y, 0.f); x.z = fmaxf(x.z, 0.f); x.w = fmaxf(x.w, 0.f);
      uint2 hi, lo;
      split4(x, s_x, hi, lo);
      const int s = 16 * sg + j;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 0, g, s) * 16 + (ftg & 1) * 8) = hi;
      *reinterpret_cast<uint2*>(base + xidx(ftg >> 1, 1, g, s) * 16 + (ftg & 1) * 8) = lo;
    }
  }
  lds_barrier();
  return s_x;
}

// Two-pass publish of act(acc * f + b) (mx: a bound of the values, act_bound of max_relu_affine); returns s_x
template <int FT, int NW, bool BIAS, int ACT = 0>
__device__ __forceinline__ float publish_affine(uint4* X16, const floatx4 (&acc)[FT][4], float f,
                                                const floatx4 (&bv)[FT], float mx, float* red, int wid, int lane,
                                                int g, int j, float beta = 0.f) {
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float s_x = pow2_scale_for(red_max<NW>(red));
  store_split_affine<FT, BIAS, ACT>(X16, acc, f, bv, s_x, wid, g, j, beta);
  lds_barrier();
  return s_x;
}

}  // namespace avr
