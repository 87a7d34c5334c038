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
#include <stdlib.h>

#include "x3_gemm.h"

namespace avr {

// ---- lin_z interpolation through LDS.
// The 64 samples x 4 bilinear corners of a workgroup touch few distinct
// texels (samples run along one ray: ~40-60 of 256 at the bench geometry).
// They are deduplicated once per workgroup (LDS hash table, slots numbered in
// first-occurrence order), the distinct rows of each lin_z table are copied
// into LDS by LDS-DMA (global_load_lds_dwordx4, no VGPRs), and every lane
// blends its 4 features x 4 corners from LDS with ds_read_b128. Rows are
// padded by 16 B so consecutive slots start in different bank quads. More
// distinct texels than the stage holds are handled in passes.

// Per-workgroup bookkeeping at the top of the LDS allocation.
struct ZTail {
  int tex[256];          // [sample][corner] texel index
  float w[256];          // [sample][corner] bilinear weight
  int slot[256];         // [sample][corner] distinct-texel slot
  unsigned ht_key[512];  // hash table: texel
  unsigned ht_min[512];  //             first entry holding it
  int first_slot[256];   // [entry] slot, for first occurrences
  int uniq[256];         // [slot] texel
  float red[16];
  int wtot[4];
  float lmax[kX3MaxLayers];   // training forward: max of each saved layer over the workgroup
  float zmax;                 //                   and of the z_feature rows
};
constexpr unsigned kEmpty = 0xffffffffu;

// Entry e = threadIdx.x (sample e>>2, corner e&3); tail->tex complete and
// ht_key/ht_min initialised before the first barrier inside. Returns the
// number of distinct texels; tail->slot is complete after the last barrier.
// Entries live in threads 0..255 (waves 0..3); other waves only join the barriers.
__device__ __forceinline__ int dedup_texels(ZTail* tail, int lane, int wid) {
  const int e = threadIdx.x;
  const bool ent = e < 256;
  __syncthreads();
  const unsigned tex = ent ? (unsigned)tail->tex[e] : 0u;
  unsigned b = (tex * 2654435761u) >> 23;  // 9-bit bucket
  if (ent) {
    for (;;) {
      const unsigned old = atomicCAS(&tail->ht_key[b], kEmpty, tex);
      if (old == kEmpty || old == tex) break;
      b = (b + 1) & 511;
    }
    atomicMin(&tail->ht_min[b], (unsigned)e);
  }
  __syncthreads();
  const int first = ent ? (int)tail->ht_min[b] : -1;
  const bool is_first = ent && first == e;
  const unsigned long long m = __ballot(is_first);
  const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
  if (ent && lane == 0) tail->wtot[wid] = __popcll(m);
  __syncthreads();
  int off = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) off += w < wid ? tail->wtot[w] : 0;
  const int D = tail->wtot[0] + tail->wtot[1] + tail->wtot[2] + tail->wtot[3];
  if (is_first) {
    tail->uniq[off + pos] = (int)tex;
    tail->first_slot[e] = off + pos;
  }
  __syncthreads();
  if (ent) tail->slot[e] = tail->first_slot[first];
  return D;
}

// Copy table rows uniq[lo .. lo+n) (row = HID floats) to stage rows 0 .. n
// (stride RS bytes) by LDS-DMA; wave w takes pieces w, w+NW, ... of 1 KiB.
// The row indices are read from LDS up front (lane i holds the row of the
// wave's i-th piece): an LDS read between two LDS-DMA issues would make the
// compiler wait for the earlier DMA to land.
template <int HID, int NW>
__device__ __forceinline__ void stage_rows(char* stage, const float* __restrict__ table, const ZTail* tail, int lo,
                                           int n, int RS, int lane, int wid, int dst0 = 0) {
  constexpr int ROWB = 4 * HID;                                  // bytes per row
  constexpr int PPR = ROWB >= 1024 ? ROWB / 1024 : 1;            // pieces per row
  constexpr int LANES = ROWB >= 1024 ? 64 : ROWB / 16;           // active lanes per piece
  const int npc = n * PPR;
  const int mine = (npc - wid + NW - 1) / NW;                    // pieces of this wave (<= 64)
  int rowv = 0;
  {
    const int pc = wid + NW * lane;
    if (lane < mine) rowv = tail->uniq[lo + pc / PPR];
  }
  for (int i = 0; i < mine; ++i) {
    const int pc = wid + NW * i;
    const int r = pc / PPR, q = pc - r * PPR;
    const int row = __builtin_amdgcn_readlane(rowv, i);
    const char* src = reinterpret_cast<const char*>(table + (int64_t)row * HID) + 1024 * q + 16 * lane;
    auto* dst = (__attribute__((address_space(3))) void*)(stage + (dst0 + r) * RS + 1024 * q);
    if (lane < LANES) __builtin_amdgcn_global_load_lds((const void*)src, dst, 16, 0, 0);
  }
}

typedef __attribute__((address_space(3))) char lds_char;

template <int FT, bool ZERO, bool TWO>
__device__ __forceinline__ void gemm(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* __restrict__ W, int KC,
                                     int cstride, const uint4* X16, int lane) {
  if constexpr (TWO)
    gemm_x3_sg<FT, ZERO, FT>(acc, A0, W, KC, cstride, X16, lane);
  else
    gemm_x3<FT, ZERO, false>(acc, A0, W, KC, cstride, X16, lane);
}

// h += S * sum_c w_c * row(slot_c) over the corners whose slot is in [lo, lo+n).
// PREP: also v = act(h * f) and the running max of max(0, h * f) for the next
// publish (the fc_0 input of the block), from the same register read of h.
template <int FT, bool PREP, bool STOREV = true, int ACT = 0>
__device__ __forceinline__ void blend_stage(floatx4 (&h)[FT][4], floatx4 (&v)[FT][4], float& mx, const char* stage_g,
                                            const ZTail* tail, int lo, int n, int RS, float S, float f, int wid, int g,
                                            int j, float beta = 0.f) {
  const lds_char* stage = (const lds_char*)stage_g;
  const unsigned fo = 64u * FT * wid + 16u * g;   // this lane's feature offset in a row
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    const int s = 16 * sg + j;
    const int4 sl = *reinterpret_cast<const int4*>(tail->slot + 4 * s);
    const float4 w = *reinterpret_cast<const float4*>(tail->w + 4 * s);
    const int sc0 = sl.x - lo, sc1 = sl.y - lo, sc2 = sl.z - lo, sc3 = sl.w - lo;
    const bool i0 = (unsigned)sc0 < (unsigned)n, i1 = (unsigned)sc1 < (unsigned)n;
    const bool i2 = (unsigned)sc2 < (unsigned)n, i3 = (unsigned)sc3 < (unsigned)n;
    const unsigned o0 = (i0 ? sc0 : 0) * RS + fo, o1 = (i1 ? sc1 : 0) * RS + fo;
    const unsigned o2 = (i2 ? sc2 : 0) * RS + fo, o3 = (i3 ? sc3 : 0) * RS + fo;
    const float w0 = i0 ? w.x * S : 0.f, w1 = i1 ? w.y * S : 0.f, w2 = i2 ? w.z * S : 0.f, w3 = i3 ? w.w * S : 0.f;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const floatx4 v0 = *reinterpret_cast<const __attribute__((address_space(3))) floatx4*>(stage + o0 + 64 * ft);
      const floatx4 v1 = *reinterpret_cast<const __attribute__((address_space(3))) floatx4*>(stage + o1 + 64 * ft);
      const floatx4 v2 = *reinterpret_cast<const __attribute__((address_space(3))) floatx4*>(stage + o2 + 64 * ft);
      const floatx4 v3 = *reinterpret_cast<const __attribute__((address_space(3))) floatx4*>(stage + o3 + 64 * ft);
      const floatx4 hn = h[ft][sg] + (((v0 * w0 + v1 * w1) + v2 * w2) + v3 * w3);
      h[ft][sg] = hn;
      if (PREP) {
        floatx4 x = hn * f;
        if (STOREV) {
          const floatx4 y = act4<ACT>(x, beta);
          v[ft][sg] = y;
          if (ACT == 0) x = y;   // ReLU: the max from the stored values
        }
        // mx starts at 0: max relu(x_i) = max(0, max x_i)
        mx = fmaxf(mx, fmaxf(x.x, x.y));
        mx = fmaxf(mx, fmaxf(x.z, x.w));
      }
      if (ft & 1) __builtin_amdgcn_sched_barrier(0);  // bound the LDS reads in flight (register pressure)
    }
  }
}

// LDS plan: X (KCX chunks x 8 KiB) from byte 0; the lin_z stage aliases X
// (rows of RS bytes from byte 0); ZTail at the top of the allocation.
template <int HID>
struct LdsPlan {
  static constexpr int KC = HID / 32;
  static constexpr int KCX = KC > kX3InChunks ? KC : kX3InChunks;
  static constexpr int XB = KCX * 8192;
  static constexpr int RS = 4 * HID + 16;
  static constexpr int TAIL = (int)((sizeof(ZTail) + 15) / 16 * 16);
  static constexpr int WANT = (XB > 96 * RS ? XB : 96 * RS) + TAIL;
  static constexpr int BYTES = WANT < 160 * 1024 ? WANT : 160 * 1024;
  static constexpr int CAP = (BYTES - TAIL) / RS;
  static constexpr int IN_ROWS0 = (kX3InChunks * 8192 + RS - 1) / RS;   // first row clear of lin_in's X
  static_assert(XB + TAIL <= BYTES, "X and tail must fit");
  static_assert(CAP * (4 * HID >= 1024 ? HID / 256 : 1) <= 4 * 64, "stage_rows: one lane per piece");
};

#if defined(AVR_STAMPS)
#define DBG_B(b) ((a.debug & 1) ? 0 : (b))
#else
#define DBG_B(b) (b)
#endif

// Training forward: GEMM input `layer` (relu'd, true scale) -> act rows and
// its relu mask bits -> mask (both consumed by the backward pass); the
// workgroup's max of the layer goes to tail->lmax (publish). Called after the
// next GEMM's weight prefetch (vmcnt retires in order: the first weight waits
// then do not wait for these stores). The rows are stored non-temporally: 4 B
// per value of every layer stream through once (4.4 GB per default_mv fine
// pass), and allocating them in L2 evicts the weights (same-box A/B,
// scripts/gpu_train_prof.sh: 5.16 -> 3.88 ms per fine-pass launch).
template <int FT, int NW>
__device__ __forceinline__ void save_layer(const FieldArgs& a, int layer, const floatx4 (&v)[FT][4], int64_t base,
                                           int64_t roff, int wid, int g, int j, int lane) {
  constexpr int HID = 16 * FT * NW, MW = mask_words(FT);
  float* act = a.act + (int64_t)layer * a.act_stride + roff * HID;
  unsigned bits[MW];
#pragma unroll
  for (int q = 0; q < MW; ++q) bits[q] = 0u;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 x = v[ft][sg];
      const int64_t m = base + 16 * sg + j;
      if (m < a.M) __builtin_nontemporal_store(x, reinterpret_cast<floatx4*>(act + m * HID + 16 * (FT * wid + ft) + 4 * g));
      const int idx = (ft * 4 + sg) * 4;
      const unsigned nib = (x.x > 0.f ? 1u : 0u) | (x.y > 0.f ? 2u : 0u) | (x.z > 0.f ? 4u : 0u) | (x.w > 0.f ? 8u : 0u);
      bits[idx >> 5] |= nib << (idx & 31);
    }
  unsigned* mk = a.mask + (((int64_t)layer * gridDim.x + blockIdx.x) * NW + wid) * MW * 64 + lane;
#pragma unroll
  for (int q = 0; q < MW; ++q) mk[q * 64] = bits[q];
}

// Training forward on the 8-wave layout (d_hidden 512: FT 4 x NW 8, two waves per SIMD as in inference; the
// 4-wave layout's materialised layer input v does not fit its 256 registers): the two-pass publish of
// act(acc * f [+ b]) also stores each value as its act row and its relu mask bit, the bits in the 4-wave
// layout's mask words (field_bwd_x3_kernel<8, 4> reads them: the 16-feature tile 4 wid + ft is tile
// 4 (wid & 1) + ft of 4-wave wave wid >> 1, word 2 (wid & 1) + ft / 2 there); the workgroup's max goes to *lmax.
template <int FT, int NW, bool BIAS>
__device__ __forceinline__ float publish_affine_save(uint4* X16, const floatx4 (&acc)[FT][4], float f,
                                                     const floatx4 (&bv)[FT], float mx, float* red, int wid, int lane,
                                                     int g, int j, const FieldArgs& a, int layer, int64_t base,
                                                     int64_t roff, float* lmax) {
  static_assert(FT == 4 && NW == 8, "8-wave training forward: d_hidden 512");
  constexpr int HID = 16 * FT * NW;
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float m = red_max<NW>(red);
  if (wid == 0 && lane == 0) *lmax = m;
  const float s_x = pow2_scale_for(m);
  char* xb = reinterpret_cast<char*>(X16);
  // the tile's rows from a wave-uniform base, 32-bit lane offsets recomputed here from an opaque lane id (hoisted
  // out of the block loop, the per-row addresses would stay live across it and spill)
  int ln = lane;
  asm volatile("" : "+v"(ln));
  g = ln >> 4;
  j = ln & 15;
  float* act = a.act + (int64_t)layer * a.act_stride + (roff + base) * HID;
  const int nval = a.M - base < 64 ? (int)(a.M - base) : 64;
  unsigned bits[2] = {0u, 0u};
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const int ftg = FT * wid + ft;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 y = relu_affine<BIAS, 0>(acc[ft][sg], f, bv[ft]);
      uint2 hi, lo;
      split4(y, s_x, hi, lo);
      const int s = 16 * sg + j;
      *reinterpret_cast<uint2*>(xb + xidx(ftg >> 1, 0, g, s) * 16 + (ftg & 1) * 8) = hi;
      *reinterpret_cast<uint2*>(xb + xidx(ftg >> 1, 1, g, s) * 16 + (ftg & 1) * 8) = lo;
      if (s < nval) __builtin_nontemporal_store(y, reinterpret_cast<floatx4*>(act + (unsigned)(s * HID + 16 * ftg + 4 * g)));
      const int idx = (ft * 4 + sg) * 4;
      bits[idx >> 5] |= ((y.x > 0.f ? 1u : 0u) | (y.y > 0.f ? 2u : 0u) | (y.z > 0.f ? 4u : 0u) | (y.w > 0.f ? 8u : 0u))
                        << (idx & 31);
    }
  }
  unsigned* mk = a.mask + ((((int64_t)layer * gridDim.x + blockIdx.x) * 4 + (wid >> 1)) * 4 + 2 * (wid & 1)) * 64 + ln;
  mk[0] = bits[0];
  mk[64] = bits[1];
  lds_barrier();
  return s_x;
}

// Work split: NW waves (4: one per SIMD; 8: two per SIMD, which doubles the
// VALU issue rate of the epilogues and hides one wave's stalls behind the
// other); wave w owns the FT 16-row feature tiles FT*w .. FT*w + FT-1.
// SAVE (training forward): also write every GEMM input and its relu mask.
// BN: eval-mode BatchNorm nets (x3_gemm.h max_relu_bn): the block input is relu(a * h + c).
// SPADE: use_spade nets (models.py:585-587): before block b < n_lin_z, h = scale_z[b](z) * h + lin_z[b](z);
// the scale table is staged and blended first (into t, free between blocks), h is scaled, then the lin_z
// table follows as for every net (its bias is in the table, not folded into the previous layer).
// ACT: the MLP's activation (x3_gemm.h act1: 0 ReLU, 1 Softplus(a.beta)); the split scale of a layer input
// comes from act_bound of the max of max(0, pre-activation), its epilogue's usual reduction.
template <int FT, int NW, bool SAVE, bool BN = false, bool SPADE = false, int ACT = 0>
__global__ void __launch_bounds__(64 * NW, 1) field_x3_kernel(FieldArgs a) {
  constexpr int HID = 16 * FT * NW;
  using P = LdsPlan<HID>;
  constexpr int KC = P::KC;
  constexpr int NTT = FT * NW;                     // feature tiles of a hidden layer
  constexpr int PES = (6 * 7 + NW - 1) / NW;       // PE slots per lane (6 * num_freqs <= 42)
  // 8 waves (256 registers each): two-pass epilogues instead of a materialised layer input v
  constexpr bool TWO = NW > 4;
  constexpr int NPF = TWO ? FT : kPrefetch;   // chunk-0 weight tiles loaded ahead of each layer's publish
  static_assert(!(SAVE && TWO) || (FT == 4 && ACT == 0 && !SPADE), "8-wave training forward: ReLU, d_hidden 512");
  static_assert(!(SAVE && BN), "BatchNorm nets train on the module path");
  static_assert(!(SAVE && SPADE) && !(BN && SPADE), "use_spade: inference without BatchNorm only");
  static_assert(ACT == 0 || !BN, "Softplus: without BatchNorm only");
  const float beta = a.beta;
  const floatx4 bz[FT] = {};
  // 8 waves: waves 0-3 at priority 1 leave each GEMM first, so their epilogue VALU overlaps the last MFMAs of
  // waves 4-7 on the same SIMDs (measured against no priority, priority for waves 4-7, and a barrier every one
  // or two K-chunk pairs inside the GEMM: this was the fastest)
  if constexpr (TWO) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) < 256) __builtin_amdgcn_s_setprio(1);
  }
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);      // KCX * 512 slots of 16 B
  char* stage = reinterpret_cast<char*>(lds);
  ZTail* tail = reinterpret_cast<ZTail*>(reinterpret_cast<char*>(lds) + (P::BYTES - P::TAIL));
  float* red = tail->red;
  // wid through readfirstlane: the compiler then knows it is wave-uniform and keeps
  // wid-derived addresses (weight fragments, bias rows) in SGPRs
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int gg = g + 4 * (wid >> 2);               // prologue: sub-lane of sample 16 (wid & 3) + j
  // SAVE: one training launch covers every scene of the batch (scene of this workgroup, its rows)
  // (inference over several scenes in one launch likewise: n_scenes > 1)
  const bool multi = SAVE || a.n_scenes > 1;
  int scene = 0;
  int64_t lblk = blockIdx.x;
  if (multi) {
    scene = (int)(blockIdx.x / a.blocks_per_scene);
    lblk = blockIdx.x - (int64_t)scene * a.blocks_per_scene;
  }
  const int64_t base = lblk * kX3Samples;
  const int64_t roff = (int64_t)scene * a.M;
  const Layout& L = a.L;
  const uint4* P16 = reinterpret_cast<const uint4*>(a.packed);  // 16-B units

  floatx4 h[FT][4], t[FT][4], v[FT][4];
  FragX3 A0[FT];   // chunk 0 of the next GEMM's weights, prefetched before the publish ahead of it
  float S_h = 1.0f, s_x = 1.0f, mx = 0.f;
  // 8 waves: stage rows of the next lin_z table that are already in flight
  // ([p0, p1), issued while the preceding GEMM still read other parts of X)
  int p0 = 0, p1 = 0, D = 0;
  if (a.h_in == nullptr) {
    AVR_STAMP(0);
    // ---- prologue: waves w and w+4 prepare samples 16 (w & 3) + j (the lanes
    // share the geometry). The 6 * num_freqs sines of a sample are spread over
    // its NW sub-lanes gg (PE entries gg, gg + NW, ...; sub-lanes 0-2 also own
    // xyz_rot[gg] / R viewdir[gg]), then each value is written as fp16 hi/lo
    // into its B-fragment slot; the padding features d_in .. 63 stay zero.
    {
      for (int i = threadIdx.x; i < 2 * kX3InChunks * 256; i += 64 * NW) X16[i] = make_uint4(0u, 0u, 0u, 0u);
      for (int i = threadIdx.x; i < 512; i += 64 * NW) { tail->ht_key[i] = kEmpty; tail->ht_min[i] = kEmpty; }
    }
    const int npe = 6 * a.num_freqs;
    float xr[3], vr[3];
    {
      const int s = 16 * (wid & 3) + j;
      const int64_t m = base + s;
      const int64_t mm = m < a.M ? m : a.M - 1;
      const SampleGeom geo = SAVE ? sample_geom_pts(a.views[scene], a.xyz + 3 * roff, a.vd + 3 * roff, mm)
                                  : sample_geom_scene(a, multi ? a.views[scene] : a.v, roff, mm);
      if (g == 0 && wid < 4) {
        *reinterpret_cast<int4*>(tail->tex + 4 * s) = make_int4(geo.bl.tex[0], geo.bl.tex[1], geo.bl.tex[2], geo.bl.tex[3]);
        *reinterpret_cast<float4*>(tail->w + 4 * s) = make_float4(geo.bl.w[0], geo.bl.w[1], geo.bl.w[2], geo.bl.w[3]);
      }
#pragma unroll
      for (int d = 0; d < 3; ++d) { xr[d] = geo.xr[d]; vr[d] = geo.vr[d]; }
    }
    AVR_STAMP(27);
    D = a.n_lin_z > 0 ? dedup_texels(tail, lane, wid) : 0;
    AVR_STAMP(28);
  #ifdef AVR_STAMPS
    if (a.stamps && threadIdx.x == 0) a.stamps[(int64_t)blockIdx.x * 64 + 31] = (unsigned long long)D;
  #endif
    float pe[PES], xo = 0.f, vo = 0.f;
    {
      // straight-line: every slot computes (selects, no branches); slots past
      // npe are zeroed; the rare |argument| > 8192 takes sinf (uniform branch)
      float arg[PES];
      bool big = false;
#pragma unroll
      for (int i = 0; i < PES; ++i) {
        const int q = gg + NW * i, jj = q / 3, dd = q - 3 * jj;
        const float x = dd == 0 ? xr[0] : (dd == 1 ? xr[1] : xr[2]);
        const float freq = fmul(a.freq_factor, __builtin_ldexpf(1.0f, jj >> 1));
        const float phase = (jj & 1) ? 1.5707963705062866f : 0.f;  // fp32(pi/2)
        arg[i] = fadd(phase, fmul(x, freq));
        pe[i] = pe_sin_fast(arg[i]);
        big |= q < npe && fabsf(arg[i]) > 8192.f;
      }
      if (__builtin_expect(__any(big), 0)) {
#pragma unroll
        for (int i = 0; i < PES; ++i)
          if (fabsf(arg[i]) > 8192.f) pe[i] = sinf(arg[i]);
      }
#pragma unroll
      for (int i = 0; i < PES; ++i) {
        pe[i] = gg + NW * i < npe ? pe[i] : 0.f;
        mx = fmaxf(mx, fabsf(pe[i]));
      }
      if (gg < 3) { xo = gg == 0 ? xr[0] : (gg == 1 ? xr[1] : xr[2]); vo = gg == 0 ? vr[0] : (gg == 1 ? vr[1] : vr[2]); }
      mx = fmaxf(mx, fmaxf(fabsf(xo), fabsf(vo)));
      mx = wave_max(mx);
    }
    const uint4* Win = P16 + L.x3_in / 4 + 2 * 64 * FT * wid;
    prefetch_a<FT, NPF>(A0, Win, lane);
    AVR_STAMP(1);
    if (SAVE && a.zf) {
      // the training forward also keeps z_feature (lin_in's input, the operand of its weight gradient): the
      // values this lane owns, the padding columns up to zf_ld as zeros
      const int64_t m = base + 16 * (wid & 3) + j;
      if (m < a.M) {
        float* zr = a.zf + (roff + m) * a.zf_ld;
#pragma unroll
        for (int i = 0; i < PES; ++i)
          if (gg + NW * i < npe) __builtin_nontemporal_store(pe[i], zr + 3 + gg + NW * i);
        if (gg < 3) {
          __builtin_nontemporal_store(xo, zr + gg);
          __builtin_nontemporal_store(vo, zr + 3 + npe + gg);
        }
        for (int k = 6 + npe + gg; k < a.zf_ld; k += NW) __builtin_nontemporal_store(0.f, zr + k);   // sub-lanes gg < NW
      }
    }
    {
      if (lane == 0) red[wid] = mx;
      lds_barrier();
      s_x = pow2_scale_for(red_max<NW>(red));
      if (SAVE && threadIdx.x == 0) tail->zmax = red_max<NW>(red);
      const int s = 16 * (wid & 3) + j;
      char* xb = reinterpret_cast<char*>(X16);
      // feature k -> chunk k>>5, lane group (k>>2)&3, element 4*((k>>4)&1) + (k&3)
      const auto put = [&](int k, float val) {
        const int c = k >> 5, gg = (k >> 2) & 3, e = 4 * ((k >> 4) & 1) + (k & 3);
        const float y = val * s_x;
        const _Float16 hi = (_Float16)y;
        *reinterpret_cast<_Float16*>(xb + xidx(c, 0, gg, s) * 16 + 2 * e) = hi;
        *reinterpret_cast<_Float16*>(xb + xidx(c, 1, gg, s) * 16 + 2 * e) = (_Float16)(y - (float)hi);
      };
#pragma unroll
      for (int i = 0; i < PES; ++i)
        if (gg + NW * i < npe) put(3 + gg + NW * i, pe[i]);
      if (gg < 3) { put(gg, xo); put(3 + npe + gg, vo); }
      lds_barrier();
    }

    AVR_STAMP(2);
    // ---- lin_in: h = (b_in + W_in . X) * S_h ; h stays scaled by S_h
    S_h = layer_scale(a.packed, L, 0) * s_x;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const floatx4 b = *reinterpret_cast<const floatx4*>(a.packed + L.b_in + 16 * (FT * wid + ft) + 4 * g);
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) h[ft][sg] = b * S_h;
    }
    AVR_STAMP(3);
    // 8 waves: stage rows of the next lin_z table that are already in flight
    // ([p0, p1), issued while the preceding GEMM still read other parts of X)
    // 8 waves: block 0's lin_z stage rows that do not overlap lin_in's X are DMA'd before the lin_in GEMM
    constexpr bool PRE0 = TWO;
    if (PRE0 && a.n_lin_z > 0 && D <= P::CAP && D > P::IN_ROWS0) {
      // the first table block 0 blends: lin_z[0], or scale_z[0] (table n_lin_z) with use_spade
      stage_rows<HID, NW>(stage, a.table + (SPADE ? a.n_lin_z : 0) * a.table_stride + scene * a.table_scene_stride,
                          tail, P::IN_ROWS0, D - P::IN_ROWS0, P::RS, lane, wid, P::IN_ROWS0);
      p0 = P::IN_ROWS0;
      p1 = D;
    }
    gemm<FT, false, TWO>(h, A0, Win, kX3InChunks, 64 * NTT, X16, lane);
    AVR_STAMP(4);
  } else {
    // the second half of a split pass (NS > 1 source views: avr_field_fwd_points_split): h = the combined
    // residual stream at block b_begin's input, fp32 rows (scale 1); no geometry, no lin_z (b >= n_lin_z)
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const int64_t m = base + 16 * sg + j;
        const int64_t mm = m < a.M ? m : a.M - 1;
        h[ft][sg] = *reinterpret_cast<const floatx4*>(a.h_in + (roff + mm) * HID + 16 * (FT * wid + ft) + 4 * g);
      }
  }

  for (int b = a.b_begin; b < a.b_end; ++b) {
    // + lin_z[b](interp latent) (models.py ResnetFC: x = x + lin_z[b](z) before block b)
    // (fused with the fc_0 input prep: v = relu(h), mx)
    if (b < a.n_lin_z) lds_barrier();  // every wave is done reading X (the stage aliases it)
    if constexpr (SPADE) {
      if (b < a.n_lin_z) {
        // t = sum_c w_c * scale_z row_c (all passes), then h *= t (h's scale S_h is unchanged)
        const float* stab = a.table + (a.n_lin_z + b) * a.table_stride + scene * a.table_scene_stride;
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
          for (int sg = 0; sg < 4; ++sg) t[ft][sg] = floatx4{0.f, 0.f, 0.f, 0.f};
        float unused = 0.f;
        for (int lo = 0; lo < D; lo += P::CAP) {
          const int n = D - lo < P::CAP ? D - lo : P::CAP;
          if (lo > 0) __syncthreads();
          if (p0 > 0) stage_rows<HID, NW>(stage, stab, tail, 0, p0, P::RS, lane, wid, 0);
          if (p0 > 0 || p1 > 0) {   // pass 0 of a single-pass set, partly staged before lin_in
            if (p1 < n) stage_rows<HID, NW>(stage, stab, tail, p1, n - p1, P::RS, lane, wid, p1);
          } else {
            stage_rows<HID, NW>(stage, stab, tail, lo, n, P::RS, lane, wid);
          }
          p0 = p1 = 0;
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          blend_stage<FT, false>(t, v, unused, stage, tail, lo, n, P::RS, 1.0f, 1.0f, wid, g, j);
        }
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
          for (int sg = 0; sg < 4; ++sg) h[ft][sg] *= t[ft][sg];
        __syncthreads();   // every wave is done with the scale rows before the lin_z rows replace them
      }
    }
    const float* table = a.table + b * a.table_stride + scene * a.table_scene_stride;
    if (b < a.n_lin_z && D <= P::CAP) {
      if (p0 > 0) stage_rows<HID, NW>(stage, table, tail, 0, p0, P::RS, lane, wid, 0);
      if (p1 < D) stage_rows<HID, NW>(stage, table, tail, p1, D - p1, P::RS, lane, wid, p1);
      p0 = p1 = 0;
      AVR_STAMP(29);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      AVR_STAMP(30);
      mx = 0.f;
      blend_stage<FT, true, !TWO, ACT>(h, v, mx, stage, tail, 0, D, P::RS, S_h, 1.0f / S_h, wid, g, j, beta);
      mx = wave_max(mx);
    } else {
      for (int lo = 0; b < a.n_lin_z && lo < D; lo += P::CAP) {   // more distinct texels than the stage holds
        const int n = D - lo < P::CAP ? D - lo : P::CAP;
        if (lo > 0) __syncthreads();
        stage_rows<HID, NW>(stage, table, tail, lo, n, P::RS, lane, wid);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        blend_stage<FT, false>(h, v, mx, stage, tail, lo, n, P::RS, S_h, 1.0f / S_h, wid, g, j);
      }
      mx = TWO ? max_relu_affine<FT, false>(h, 1.0f / S_h, bz)
               : prep_input<FT, false, ACT>(v, h, 1.0f / S_h, nullptr, wid, g, beta);
    }
    mx = act_bound<ACT>(mx, beta);   // (BN nets are ReLU only: their max below replaces this)
    const float* bn_a = a.packed + L.bn_a[b];
    const float* bn_c = a.packed + L.bn_c[b];
    if constexpr (BN) {   // the block input is relu(bn_0(h)) (models.py:456-458), not relu(h)
      if constexpr (TWO) mx = max_relu_bn<FT>(h, 1.0f / S_h, bn_a, bn_c, wid, g);
      else mx = prep_bn<FT>(v, h, 1.0f / S_h, bn_a, bn_c, wid, g);
    }
    AVR_STAMP(5 + 5 * (b & 3));
    const uint4* W0 = P16 + L.x3_fc0[DBG_B(b)] / 4 + 2 * 64 * FT * wid;
    const uint4* W1 = P16 + L.x3_fc1[DBG_B(b)] / 4 + 2 * 64 * FT * wid;
    prefetch_a<FT, NPF>(A0, W0, lane);
    if constexpr (TWO) {
      // the fc_1 bias loads are issued before the t publish, whose barriers cover their latency
      if constexpr (BN) s_x = publish_bn<FT, NW>(X16, h, 1.0f / S_h, bn_a, bn_c, mx, red, wid, lane, g, j);
      else if constexpr (SAVE)
        s_x = publish_affine_save<FT, NW, false>(X16, h, 1.0f / S_h, bz, mx, red, wid, lane, g, j, a, 2 * b, base,
                                                 roff, &tail->lmax[2 * b]);
      else s_x = publish_affine<FT, NW, false, ACT>(X16, h, 1.0f / S_h, bz, mx, red, wid, lane, g, j, beta);
      AVR_STAMP(6 + 5 * (b & 3));
      const float S_t = layer_scale(a.packed, L, 2 + 2 * b) * s_x;
      gemm<FT, true, TWO>(t, A0, W0, KC, 64 * NTT, X16, lane);
      AVR_STAMP(7 + 5 * (b & 3));
      floatx4 bv[FT];
      load_bias<FT, true>(bv, a.packed + L.b_fc0[b], wid, g);
      mx = act_bound<ACT>(max_relu_affine<FT, true>(t, 1.0f / S_t, bv), beta);
      if (b == 1) AVR_STAMP(20);
      floatx4 bb[FT];
      load_bias<FT, true>(bb, a.packed + L.b_fc1[b], wid, g);
      prefetch_a<FT, NPF>(A0, W1, lane);
      if (b == 1) AVR_STAMP(21);
      if constexpr (SAVE)
        s_x = publish_affine_save<FT, NW, true>(X16, t, 1.0f / S_t, bv, mx, red, wid, lane, g, j, a, 2 * b + 1, base,
                                                roff, &tail->lmax[2 * b + 1]);
      else s_x = publish_affine<FT, NW, true, ACT>(X16, t, 1.0f / S_t, bv, mx, red, wid, lane, g, j, beta);
      AVR_STAMP(8 + 5 * (b & 3));
      // fc_1 accumulates onto the residual, rescaled to this layer's scale (+ b1)
      const float S1 = layer_scale(a.packed, L, 3 + 2 * b) * s_x;
      const float r = S1 / S_h;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) h[ft][sg] = h[ft][sg] * r + bb[ft] * S1;
      S_h = S1;
      gemm<FT, false, TWO>(h, A0, W1, KC, 64 * NTT, X16, lane);
    } else {
      if (SAVE) save_layer<FT, NW>(a, 2 * b, v, base, roff, wid, g, j, lane);
      s_x = publish<FT, NW>(X16, v, mx, red, wid, lane, g, j, SAVE ? &tail->lmax[2 * b] : nullptr);
      AVR_STAMP(6 + 5 * (b & 3));
      // fc_0 (from zero)
      const float S_t = layer_scale(a.packed, L, 2 + 2 * b) * s_x;
      gemm<FT, true, TWO>(t, A0, W0, KC, 64 * NTT, X16, lane);
      AVR_STAMP(7 + 5 * (b & 3));
      // fc_1 input relu(t + b0)
      mx = act_bound<ACT>(prep_input<FT, true, ACT>(v, t, 1.0f / S_t, a.packed + L.b_fc0[b], wid, g, beta), beta);
      prefetch_a<FT, NPF>(A0, W1, lane);
      if (SAVE) save_layer<FT, NW>(a, 2 * b + 1, v, base, roff, wid, g, j, lane);
      s_x = publish<FT, NW>(X16, v, mx, red, wid, lane, g, j, SAVE ? &tail->lmax[2 * b + 1] : nullptr);
      AVR_STAMP(8 + 5 * (b & 3));
      // fc_1 accumulates onto the residual, rescaled to this layer's scale (+ b1)
      const float S1 = layer_scale(a.packed, L, 3 + 2 * b) * s_x;
      const float r = S1 / S_h;
      floatx4 bb[FT];   // all bias loads first (one wait, not one per tile)
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
        bb[ft] = *reinterpret_cast<const floatx4*>(a.packed + L.b_fc1[b] + 16 * (FT * wid + ft) + 4 * g) * S1;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) h[ft][sg] = h[ft][sg] * r + bb[ft];
      S_h = S1;
      gemm<FT, false, TWO>(h, A0, W1, KC, 64 * NTT, X16, lane);
    }
    AVR_STAMP(9 + 5 * (b & 3));
  }
  if (a.h_out) {
    // the first half of a split pass: the residual stream after block b_end - 1, fp32 rows (h / S_h), for the
    // caller's combine over the source views (combine_interleaved, models.py:566-579 / utils.py:71-81)
    const float f = 1.0f / S_h;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const int64_t m = base + 16 * sg + j;
        if (m < a.M)
          __builtin_nontemporal_store(h[ft][sg] * f, reinterpret_cast<floatx4*>(a.h_out + (roff + m) * HID +
                                                                                16 * (FT * wid + ft) + 4 * g));
      }
    return;
  }

  if constexpr (TWO) {
    // ---- lin_out(relu(h)) without publishing X: every wave multiplies its own 64
    // features (its 2 K-chunks) into a partial 4 x 64 output under a wave-local split
    // scale, the partials meet in LDS (the dead dedup area of the tail) and waves 0-3
    // sum them in wave order for samples 16w + j.
    const uint4* wo = P16 + L.x3_out / 4 + lane;
    FragX3 Aw[2];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) Aw[cc] = load_frag(wo + 2 * 64 * (2 * wid + cc));
    const float f = 1.0f / S_h;
    const float mxw = act_bound<ACT>(max_relu_affine<FT, false>(h, f, bz), beta);
    const float s_w = pow2_scale_for(mxw);
    floatx4 part[4];
    // SAVE: lin_out's input (layer 2 n_blocks) as act rows and mask bits (publish_affine_save's layout), the
    // workgroup's max through red
    unsigned sbits[2] = {0u, 0u};
    const int lout = 2 * a.n_blocks;
    if constexpr (SAVE) {
      float* sact = a.act + (int64_t)lout * a.act_stride + (roff + base) * HID;
      const int snval = a.M - base < 64 ? (int)(a.M - base) : 64;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        part[sg] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
          uint2 h0, l0, h1, l1;
          const floatx4 y0 = relu_affine<false, ACT>(h[2 * cc][sg], f, bz[0], beta);
          const floatx4 y1 = relu_affine<false, ACT>(h[2 * cc + 1][sg], f, bz[0], beta);
          if constexpr (SAVE) {
            const int srow = 16 * sg + j;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const floatx4 y = q ? y1 : y0;
              const int ft = 2 * cc + q, ftg = FT * wid + ft;
              if (srow < snval)
                __builtin_nontemporal_store(y, reinterpret_cast<floatx4*>(sact + (unsigned)(srow * HID + 16 * ftg + 4 * g)));
              const int idx = (ft * 4 + sg) * 4;
              sbits[idx >> 5] |= ((y.x > 0.f ? 1u : 0u) | (y.y > 0.f ? 2u : 0u) | (y.z > 0.f ? 4u : 0u) |
                                  (y.w > 0.f ? 8u : 0u)) << (idx & 31);
            }
          }
          split4(y0, s_w, h0, l0);
          split4(y1, s_w, h1, l1);
          const half8 bh = __builtin_bit_cast(half8, make_uint4(h0.x, h0.y, h1.x, h1.y));
          const half8 bl = __builtin_bit_cast(half8, make_uint4(l0.x, l0.y, l1.x, l1.y));
          part[sg] = mfma32h(Aw[cc].hi, bh, part[sg]);
          part[sg] = mfma32h(Aw[cc].hi, bl, part[sg]);
          part[sg] = mfma32h(Aw[cc].lo, bh, part[sg]);
        }
      }
    } else {
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        part[sg] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
          uint2 h0, l0, h1, l1;
          split4(relu_affine<false, ACT>(h[2 * cc][sg], f, bz[0], beta), s_w, h0, l0);
          split4(relu_affine<false, ACT>(h[2 * cc + 1][sg], f, bz[0], beta), s_w, h1, l1);
          const half8 bh = __builtin_bit_cast(half8, make_uint4(h0.x, h0.y, h1.x, h1.y));
          const half8 bl = __builtin_bit_cast(half8, make_uint4(l0.x, l0.y, l1.x, l1.y));
          part[sg] = mfma32h(Aw[cc].hi, bh, part[sg]);
          part[sg] = mfma32h(Aw[cc].hi, bl, part[sg]);
          part[sg] = mfma32h(Aw[cc].lo, bh, part[sg]);
        }
      }
    }
    const float un = 1.0f / (layer_scale(a.packed, L, 1) * s_w);
    float4* pbuf = reinterpret_cast<float4*>(tail);   // [wave][sample] (r, g, b, sigma) partials: 8 KiB
    if (g == 0) {
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const floatx4 o = part[sg] * un;
        pbuf[wid * 64 + 16 * sg + j] = make_float4(o.x, o.y, o.z, o.w);
      }
    }
    if constexpr (SAVE) {
      unsigned* mk = a.mask + ((((int64_t)lout * gridDim.x + blockIdx.x) * 4 + (wid >> 1)) * 4 + 2 * (wid & 1)) * 64 +
                     lane;
      mk[0] = sbits[0];
      mk[64] = sbits[1];
      if (lane == 0) red[wid] = mxw;
    }
    lds_barrier();
    AVR_STAMP(25);
    if (wid >= 4) return;
    if constexpr (SAVE) {
      // the layer maxima: one atomic per workgroup and layer (lin_out's input: the waves' maxima met in red)
      const int nl = 2 * a.n_blocks + 1;
      if (a.act_max && wid == 0 && lane < nl)
        publish_max(a.act_max + lane, lane == nl - 1 ? red_max<NW>(red) : tail->lmax[lane]);
      if (a.zf_max && threadIdx.x == 64) publish_max(a.zf_max, tail->zmax);
    }
    const int s = 16 * wid + j;
    const int64_t m = base + s;
    if (g == 0 && m < a.M) {
      float4 o = *reinterpret_cast<const float4*>(a.packed + L.b_out);
#pragma unroll
      for (int v = 0; v < NW; ++v) {
        const float4 p = pbuf[v * 64 + s];
        o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
      }
      AVR_STAMP(26);
      a.out[roff + m] = make_float4(sigmoidf_(o.x), sigmoidf_(o.y), sigmoidf_(o.z), fmaxf(o.w, 0.f));
    }
    return;
  }
  // ---- lin_out(relu(h)): waves 0-3 compute the 16-row output tile for samples 16w + j.
  // (a quarter of lin_out's A fragments are loaded ahead of the publish, the rest after)
  FragX3 Ao[KC];
  const uint4* wo = P16 + L.x3_out / 4;
  const unsigned wlo = lane;
  if (wid < 4) {
#pragma unroll
    for (int c = 0; c < KC / 4; ++c) Ao[c] = load_frag(wo + (wlo + 2 * 64 * c));
  }
  if constexpr (TWO) {
    mx = act_bound<ACT>(max_relu_affine<FT, false>(h, 1.0f / S_h, bz), beta);
    s_x = publish_affine<FT, NW, false, ACT>(X16, h, 1.0f / S_h, bz, mx, red, wid, lane, g, j, beta);
  } else {
    mx = act_bound<ACT>(prep_input<FT, false, ACT>(v, h, 1.0f / S_h, nullptr, wid, g, beta), beta);
    if (SAVE) save_layer<FT, NW>(a, 2 * a.n_blocks, v, base, roff, wid, g, j, lane);
    s_x = publish<FT, NW>(X16, v, mx, red, wid, lane, g, j, SAVE ? &tail->lmax[2 * a.n_blocks] : nullptr);
  }
  if (wid < 4) {
#pragma unroll
    for (int c = KC / 4; c < KC; ++c) Ao[c] = load_frag(wo + (wlo + 2 * 64 * c));
  }
  AVR_STAMP(25);
  if (wid >= 4) return;
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
  if (g == 0 && m < a.M)
    a.out[roff + m] = make_float4(sigmoidf_(o.x), sigmoidf_(o.y), sigmoidf_(o.z), fmaxf(o.w, 0.f));
  if constexpr (SAVE) {
    // the layer maxima: one atomic per workgroup and layer, issued last (nothing waits on them here;
    // one per wave and layer in front of the weight loads cost ~1 ms per default_mv fine pass)
    const int nl = 2 * a.n_blocks + 1;
    if (a.act_max && wid == 0 && lane < nl) publish_max(a.act_max + lane, tail->lmax[lane]);
    if (a.zf_max && threadIdx.x == 64) publish_max(a.zf_max, tail->zmax);
  }
}

// ---- lin_z / scale_z tables on the same split-fp16 GEMM (x3 fields; the fp32 field keeps
// latent_table_split_kernel's exact products): table[t][texel][f] = sum_c W_t[f][c] latent[c][texel]
// (+ the table's bias with use_spade), for the 64 texels of a workgroup. The latent columns (CHW: one
// coalesced 256-B row per channel) are split into X under one power-of-two scale per workgroup, then
// KCL = d_latent / 32 K-chunks of the hidden layers' GEMM; blockIdx.y = table. ALL: one workgroup makes every
// table of its texels from the one staged operand (the latent read once instead of once per table, and each
// table's stores drain under the next table's GEMM), for grids that fill the chip without the table dimension.
template <int FT, int NW, bool ALL = false>
__global__ void __launch_bounds__(64 * NW, 1) table_x3_kernel(const float* __restrict__ packed, Layout L,
                                                              const float* __restrict__ latent, int HW, int d_latent,
                                                              float* __restrict__ table, int64_t lat_stride,
                                                              int64_t tab_stride) {
  latent += blockIdx.z * lat_stride;   // scene blockIdx.z of a batch
  table += blockIdx.z * tab_stride;
  constexpr int HID = 16 * FT * NW, NTT = FT * NW;
  constexpr bool TWO = NW > 4;
  constexpr int MAXQ = 512 / 4 / NW;               // 4-channel groups per wave (d_latent <= 512)
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);
  const int KCL = d_latent >> 5;
  float* red = lds + KCL * 2048;                   // after X (8 KiB per chunk)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int t_first = ALL ? 0 : blockIdx.y, t_end = ALL ? L.n_tables : t_first + 1;
  const int64_t t0 = (int64_t)blockIdx.x * kX3Samples;
  const auto wtab = [&](int t) {
    return reinterpret_cast<const uint4*>(packed) + L.x3_tab[t] / 4 + 2 * 64 * FT * wid;
  };
  FragX3 A0[FT];
  prefetch_a<FT, TWO ? FT : kPrefetch>(A0, wtab(t_first), lane);
  // lane = texel; wave w loads channel groups w, w + NW, ...
  const int64_t tx = t0 + lane < HW ? t0 + lane : HW - 1;
  floatx4 xv[MAXQ];
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < MAXQ; ++i) {
    const int k = 4 * (wid + NW * i);
    xv[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (k < d_latent) {
#pragma unroll
      for (int r = 0; r < 4; ++r) xv[i][r] = latent[(int64_t)(k + r) * HW + tx];
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(xv[i].x), fabsf(xv[i].y)), fmaxf(fabsf(xv[i].z), fabsf(xv[i].w))));
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float s_x = pow2_scale_for(red_max<NW>(red));
  char* xb = reinterpret_cast<char*>(X16);
#pragma unroll
  for (int i = 0; i < MAXQ; ++i) {
    const int k = 4 * (wid + NW * i);
    if (k < d_latent) {
      uint2 hi, lo;
      split4(xv[i], s_x, hi, lo);
      const int c = k >> 5, gq = (k >> 2) & 3, half = (k >> 4) & 1;
      *reinterpret_cast<uint2*>(xb + xidx(c, 0, gq, lane) * 16 + 8 * half) = hi;
      *reinterpret_cast<uint2*>(xb + xidx(c, 1, gq, lane) * 16 + 8 * half) = lo;
    }
  }
  lds_barrier();
  for (int t = t_first; t < t_end; ++t) {
    floatx4 acc[FT][4];
    gemm<FT, true, TWO>(acc, A0, wtab(t), KCL, 64 * NTT, X16, lane);
    if (t + 1 < t_end) prefetch_a<FT, TWO ? FT : kPrefetch>(A0, wtab(t + 1), lane);   // under this epilogue
    const float inv = 1.0f / (layer_scale(packed, L, kX3TabHdr + t) * s_x);
    float* dst = table + (int64_t)t * HW * HID;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const int f0 = 16 * (FT * wid + ft) + 4 * g;
      const floatx4 b =
          L.spade ? *reinterpret_cast<const floatx4*>(packed + L.b_tab[t] + f0) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const int64_t texel = t0 + 16 * sg + j;
        if (texel < HW) *reinterpret_cast<floatx4*>(dst + texel * HID + f0) = acc[ft][sg] * inv + b;
      }
    }
  }
}

template <int FT, int NW, bool ALL>
static int launch_table_x3_k(const float* packed, const Layout& L, const float* latent, int HW, int d_latent,
                             float* table, int n_scenes, hipStream_t s) {
  const size_t shm = (size_t)(d_latent / 32) * 8192 + 64;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&table_x3_kernel<FT, NW, ALL>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 8192 * 4 + 64) != hipSuccess)
      return fail(AVR_E_HIP, "table_x3_kernel: cannot set dynamic LDS");
    attr = true;
  }
  const dim3 grid((unsigned)((HW + kX3Samples - 1) / kX3Samples), ALL ? 1u : (unsigned)L.n_tables, (unsigned)n_scenes);
  const int64_t tab_stride = (int64_t)(L.n_tables > 0 ? L.n_tables : 1) * HW * (16 * FT * NW);
  table_x3_kernel<FT, NW, ALL><<<grid, 64 * NW, shm, s>>>(packed, L, latent, HW, d_latent, table,
                                                          (int64_t)d_latent * HW, tab_stride);
  return check_launch("table_x3_kernel");
}

// every table per workgroup once the texel blocks alone give a workgroup to each CU (AVR_TABLE_ALL=0|1 forces
// the choice, for A/B)
static bool table_all(int64_t blocks, int n_tables) {
  const char* e = getenv("AVR_TABLE_ALL");
  if (e) return e[0] == '1' && n_tables > 1;
  return n_tables > 1 && blocks >= 256;
}

template <int FT, int NW>
static int launch_table_x3(const float* packed, const Layout& L, const float* latent, int HW, int d_latent,
                           float* table, int n_scenes, hipStream_t s) {
  const int64_t blocks = (int64_t)((HW + kX3Samples - 1) / kX3Samples) * n_scenes;
  if (table_all(blocks, L.n_tables))
    return launch_table_x3_k<FT, NW, true>(packed, L, latent, HW, d_latent, table, n_scenes, s);
  return launch_table_x3_k<FT, NW, false>(packed, L, latent, HW, d_latent, table, n_scenes, s);
}

int dispatch_table_x3(const float* packed, const Layout& L, const float* latent, int HW, int d_latent, int d_hidden,
                      float* table, int n_scenes, hipStream_t s) {
  AVR_REQUIRE(L.x3_tables && d_latent % 64 == 0 && d_latent <= 512, "table x3: d_latent %d", d_latent);
  switch (d_hidden) {
    case 64: return launch_table_x3<1, 4>(packed, L, latent, HW, d_latent, table, n_scenes, s);
    case 128: return launch_table_x3<2, 4>(packed, L, latent, HW, d_latent, table, n_scenes, s);
    case 256: return launch_table_x3<4, 4>(packed, L, latent, HW, d_latent, table, n_scenes, s);
    case 512: return launch_table_x3<4, 8>(packed, L, latent, HW, d_latent, table, n_scenes, s);
  }
  return fail(AVR_E_UNSUPPORTED, "table x3: d_hidden %d", d_hidden);
}

template <int FT, int NW, bool SAVE, bool BN = false, bool SPADE = false, int ACT = 0>
static int launch_x3(const FieldArgs& a, hipStream_t s) {
  const size_t shm = LdsPlan<16 * FT * NW>::BYTES;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&field_x3_kernel<FT, NW, SAVE, BN, SPADE, ACT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return fail(AVR_E_HIP, "field_x3_kernel: cannot set dynamic LDS to %zu", shm);
    attr = true;
  }
  const int64_t blocks = (SAVE || a.n_scenes > 1) ? a.blocks_per_scene * a.n_scenes
                                                  : (a.M + kX3Samples - 1) / kX3Samples;
  AVR_REQUIRE(blocks < (1ll << 31), "field: too many points");
  field_x3_kernel<FT, NW, SAVE, BN, SPADE, ACT><<<(unsigned)blocks, 64 * NW, shm, s>>>(a);
  return check_launch("field_x3_kernel");
}

// AVR_X3_WAVES (diagnostics), read per launch so a test can switch layouts in one process
static int x3_waves() {
  const char* e = getenv("AVR_X3_WAVES");
  return (e && atoi(e) == 4) ? 4 : 8;
}

static int save_waves() {
  const char* e = getenv("AVR_X3_SAVE_WAVES");
  return (e && atoi(e) == 4) ? 4 : 8;
}

int dispatch_field_x3(int d_hidden, const FieldArgs& a, hipStream_t s) {
  // inference at d_hidden 512: 8 waves x 4 tiles (+2.7-4.7 % over the 4-wave layout on the same box);
  // AVR_X3_WAVES=4 selects the 4-wave layout (diagnostics)
  if (a.L.bn) {   // eval-mode BatchNorm (inference only)
    AVR_REQUIRE(!a.act, "field x3: BatchNorm nets train on the module path");
    switch (d_hidden) {
      case 64: return launch_x3<1, 4, false, true>(a, s);
      case 128: return launch_x3<2, 4, false, true>(a, s);
      case 256: return launch_x3<4, 4, false, true>(a, s);
      case 512: return x3_waves() == 8 ? launch_x3<4, 8, false, true>(a, s) : launch_x3<8, 4, false, true>(a, s);
    }
    return fail(AVR_E_UNSUPPORTED, "field x3: d_hidden %d", d_hidden);
  }
  if (a.beta > 0.f && !a.L.spade && a.act) {   // Softplus training forward (4-wave SAVE layout, ABI 11)
    switch (d_hidden) {
      case 64: return launch_x3<1, 4, true, false, false, 1>(a, s);
      case 128: return launch_x3<2, 4, true, false, false, 1>(a, s);
      case 256: return launch_x3<4, 4, true, false, false, 1>(a, s);
      case 512: return launch_x3<8, 4, true, false, false, 1>(a, s);
    }
    return fail(AVR_E_UNSUPPORTED, "field x3: d_hidden %d", d_hidden);
  }
  if (a.L.spade || a.beta > 0.f) {   // use_spade and / or Softplus (inference)
    AVR_REQUIRE(!a.act, "field x3: use_spade nets train on the module path");
    const int v = (a.L.spade ? 1 : 0) | (a.beta > 0.f ? 2 : 0);
#define AVR_X3_OPT(FT, NW)                                      \
  switch (v) {                                                  \
    case 1: return launch_x3<FT, NW, false, false, true, 0>(a, s);  \
    case 2: return launch_x3<FT, NW, false, false, false, 1>(a, s); \
    default: return launch_x3<FT, NW, false, false, true, 1>(a, s); \
  }
    switch (d_hidden) {
      case 64: AVR_X3_OPT(1, 4)
      case 128: AVR_X3_OPT(2, 4)
      case 256: AVR_X3_OPT(4, 4)
      case 512: AVR_X3_OPT(4, 8)
    }
#undef AVR_X3_OPT
    return fail(AVR_E_UNSUPPORTED, "field x3: d_hidden %d", d_hidden);
  }
  if (d_hidden == 512 && !a.act && x3_waves() == 8) return launch_x3<4, 8, false>(a, s);
  // training forward at d_hidden 512: the 8-wave layout too (AVR_X3_SAVE_WAVES=4: the 4-wave one, A/B)
  if (d_hidden == 512 && a.act && save_waves() == 8) return launch_x3<4, 8, true>(a, s);
  switch (d_hidden) {
    case 64: return a.act ? launch_x3<1, 4, true>(a, s) : launch_x3<1, 4, false>(a, s);
    case 128: return a.act ? launch_x3<2, 4, true>(a, s) : launch_x3<2, 4, false>(a, s);
    case 256: return a.act ? launch_x3<4, 4, true>(a, s) : launch_x3<4, 4, false>(a, s);
    case 512: return a.act ? launch_x3<8, 4, true>(a, s) : launch_x3<8, 4, false>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "field x3: d_hidden %d", d_hidden);
}

}  // namespace avr
