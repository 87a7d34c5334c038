// Training-mode BatchNorm of ResnetFC(bn=True) on the HIP path: train.py --bn (train.py:210, :265) builds
// ResnetBlockFC(bn=True), whose forward is relu(bn_0(x)) -> fc_0 -> relu(bn_0(net)) -> fc_1, + x
// (models.py:454-461; bn_0 applied twice, bn_1 unused), with batch statistics over every row of the field
// call in training mode.
//
// The fused field kernels carry a 64-sample tile through every layer in one workgroup; batch statistics are a
// reduction over all rows between two GEMMs, so this net runs layer by layer. One launch per GEMM over
// row-major fp32 rows (bn_layer_kernel): the operand -- the layer input normalised and relu'd (forward), or
// the BatchNorm backward of the gradient (backward) -- is built in the prologue straight from the rows in the
// fused kernels' B-fragment order (each lane loads exactly its fragment columns), split into fp16 hi/lo under
// one power-of-two scale per workgroup and written to LDS; the K loop is theirs (x3: three
// v_mfma_f32_16x16x32_f16 per product, fp32 accumulate, weights streamed one chunk ahead); the epilogue works in
// the accumulator layout -- adds bias / residual / lin_z rows (forward) or applies the relu mask (backward,
// recomputed from the pre-BN rows: the relu'd operands are never stored; ABI 14: lin_z^T layers without a mask,
// an added residual gradient and the stored rows' max), stores the rows and reduces this workgroup's column
// statistics. A finalize launch between
// layers (bn_stats_kernel / bn_grad_stats_kernel) combines the workgroups' partials in fp64.
#include "x3_gemm.h"

namespace avr {

struct BnArgs {
  int64_t M;
  int prologue, kin, K;
  const float* src; int64_t ld_src;
  const float* src_pre; const float* src_res;
  const float* in_mu; const float* in_scale; const float* in_shift;
  const float* in_m1; const float* in_m2; const float* in_invstd;
  float* opnd_out; unsigned* opnd_max;
  const float* w;               // this layer's x3 fragments (chunk 0, tile 0)
  const unsigned* hdr; int hdr_idx;   // the blob header's max |W| bits of the layer (the pack's power-of-two scale)
  int KC;
  const float* bias; const float* add1; const float* add2;
  float* out;
  const float* pre_rows; const float* out_mu; const float* out_invstd; const float* out_scale; const float* out_shift;
  float* part;
  // forward: the lin_z rows gathered in the epilogue (row m of scene m / zrows: the bilinear blend of
  // ztab + scene * ztab_stride at zxyz[m] in zviews[scene]), or ztab = null
  const float* ztab; int64_t ztab_stride, zrows;
  const float* zxyz;
  unsigned* out_max;            // backward: max |out| of the stored rows, or null
  View zviews[AVR_MAX_SCENES];
};

__device__ __forceinline__ floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

// 16 lanes of one lane group g (lanes 16g .. 16g + 15): sum over j, the same bits in every lane (xor butterfly on
// DPP / row shifts: no LDS round trip, unlike __shfl_xor's ds_bpermute)
__device__ __forceinline__ floatx4 sum16(floatx4 v) {
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] += lane_xor(v[t], d, 0);
  }
  return v;
}

// Row lines <-> fragment pairs. Lane (g, j) of a 16-row group works on the 16-B groups x0 (columns c + 4g .. +3)
// and x1 (c + 16 + 4g .. +3) of row j: each row's 128-B line is split over lanes g and both halves. In memory it
// is moved as two instructions of 8 rows x 128 B -- lane j takes row j & 7 (A) and row 8 + (j & 7) (B), columns
// c + 16 (j >> 3) + 4g .. +3 -- so that every instruction covers whole lines, and lanes j and j ^ 8 swap one
// value through one DPP row rotation (row_ror:8).
__device__ __forceinline__ floatx4 ror8(floatx4 v) {
  floatx4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[t]), 0x128, 0xf, 0xf, false));
  return r;
}
__device__ __forceinline__ void lines_to_pair(floatx4 A, floatx4 B, bool lo, floatx4& x0, floatx4& x1) {
  const floatx4 r = ror8(lo ? B : A);
  x0 = lo ? A : r;
  x1 = lo ? r : B;
}
__device__ __forceinline__ void pair_to_lines(floatx4 x0, floatx4 x1, bool lo, floatx4& A, floatx4& B) {
  const floatx4 r = ror8(lo ? x1 : x0);
  A = lo ? x0 : r;
  B = lo ? r : x1;
}

template <int FT, int NW, bool TWO>
__device__ __forceinline__ void bn_gemm(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* __restrict__ W, int KC,
                                        int cstride, const uint4* X16, int lane) {
  if constexpr (TWO)
    gemm_x3_sg<FT, true, FT>(acc, A0, W, KC, cstride, X16, lane);
  else
    gemm_x3<FT, true, false>(acc, A0, W, KC, cstride, X16, lane);
}

// MODE 0 forward, 1 backward; KK = K (64: lin_in, or d_hidden). Workgroup = 64 rows, NW waves, no fp32 stage and
// no epilogue barrier:
// * operand: the K columns are 4 KK / 32 items (32-column chunk c, sample group sg of 16 rows); wave w takes IPW
//   consecutive items; lane (g, j) needs, for each, exactly its B-fragment columns 32c + 4g .. +3 and
//   32c + 16 + 4g .. +3 of row 16 sg + j, loaded as whole 128-B row lines and exchanged (lines_to_pair); it
//   applies the prologue's transform and keeps the values in registers until the workgroup's max |operand| is
//   met in LDS; then one 16-B hi and one 16-B lo LDS write per item put them in the fused kernels' X slots
//   (conflict-free: consecutive j, consecutive slots).
// * GEMM: the fused kernels' K loop; lane (g, j) of wave w ends with features 16 (FT w + ft) + 4g .. +3 of rows
//   16 sg + j.
// * epilogue straight from the accumulators: the addend / pre-BN loads and the row stores move whole lines
//   (pair_to_lines), and since a wave owns its columns for all 64 rows, a column's statistics are in-lane sums
//   over the four sample groups and a 16-lane DPP reduction over j -- no LDS, no barrier, so each wave starts its
//   epilogue as soon as its own GEMM ends.
template <int FT, int NW, int MODE, int KK>
// (4-wave layouts: two workgroups per CU, so at most 256 registers a lane)
__global__ void __launch_bounds__(64 * NW, NW > 4 ? 1 : 2) bn_layer_kernel(BnArgs a) {
  constexpr int HID = 16 * FT * NW;
  constexpr bool TWO = NW > 4;
  constexpr int IPW = 4 * (KK / 32) / NW;    // operand items per wave
  constexpr int IPC = IPW < 4 ? IPW : 4;     // items per chunk of this wave
  constexpr int NCH = IPW / IPC;             // chunks of this wave
  static_assert(IPW >= 1 && IPW * NW == 4 * (KK / 32) && NCH * IPC == IPW, "operand items per wave");
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);
  float* red = lds + 64 * KK;                // past X (64 samples x KK x (hi + lo) fp16)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int64_t m0 = (int64_t)blockIdx.x * kX3Samples;
  const int nvalid = a.M - m0 < kX3Samples ? (int)(a.M - m0) : kX3Samples;
  const uint4* W = reinterpret_cast<const uint4*>(a.w) + 2 * 64 * FT * wid;
  FragX3 A0[FT];
  prefetch_a<FT, TWO ? FT : kPrefetch>(A0, W, lane);

  // ---------------------------------------------------------------- operand
  // item i of this wave: chunk (IPW w + i) / 4, sample group (IPW w + i) % 4; its row r = 16 sg + j (rows past
  // the end load row m0 and become zeros); half h: columns 32 c + 16 h + 4 g .. +3
  const int i0 = IPW * wid;
  const auto chunk = [&](int i) { return (i0 + i) >> 2; };
  const auto row_r = [&](int i) { return 16 * ((i0 + i) & 3) + j; };
  const auto col_k = [&](int i, int h) { return 32 * chunk(i) + 16 * h + 4 * g; };
  // the item's rows as lines (see lines_to_pair): line row lr(i, half), columns 32 c + 16 (j >> 3) + 4 g
  const bool lo = j < 8;
  const auto lr = [&](int i, int half) { return 16 * ((i0 + i) & 3) + 8 * half + (j & 7); };
  const auto lrow = [&](int i, int half) -> int64_t { return m0 + (lr(i, half) < nvalid ? lr(i, half) : 0); };
  const auto lcol = [&](int i) { return 32 * chunk(i) + 16 * (j >> 3) + 4 * g; };
  const auto srow = [&](int i) -> int64_t { return m0 + (row_r(i) < nvalid ? row_r(i) : 0); };
  floatx4 xv[IPW][2];
  if (KK != 64 || a.kin == KK) {   // whole 16-B groups (every hidden layer): a batch's loads back to back, branch-free
    if (a.prologue == AVR_BN_GRAD) {
      // three rows per value (gradient, pre-BN, residual): one chunk's parameters and two items per batch, the
      // residual's presence decided once (a null check per load would keep each load behind its own branch)
      const auto grad = [&](auto res_t) {
        constexpr bool RES = decltype(res_t)::value;
#pragma unroll
        for (int cc = 0; cc < NCH; ++cc) {
          floatx4 pp[5][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = col_k(cc * IPC, h);
            pp[0][h] = ld4(a.in_mu + k); pp[1][h] = ld4(a.in_invstd + k); pp[2][h] = ld4(a.in_m1 + k);
            pp[3][h] = ld4(a.in_m2 + k); pp[4][h] = ld4(a.in_scale + k);
          }
          constexpr int GB = IPC < 2 ? IPC : 2;   // items per batch
#pragma unroll
          for (int q0 = 0; q0 < IPC; q0 += GB) {
            floatx4 sv[GB][2], pv[GB][2], rv[GB][2];
#pragma unroll
            for (int q = 0; q < GB; ++q)
#pragma unroll
              for (int e = 0; e < 2; ++e) {   // line e (A / B)
                const int i = cc * IPC + q0 + q;
                const int64_t o = lrow(i, e) * a.ld_src + lcol(i);
                sv[q][e] = ld4(a.src + o);
                pv[q][e] = ld4(a.src_pre + o);
                if constexpr (RES) rv[q][e] = ld4(a.src_res + o);
              }
#pragma unroll
            for (int q = 0; q < GB; ++q) {
              lines_to_pair(sv[q][0], sv[q][1], lo, sv[q][0], sv[q][1]);
              lines_to_pair(pv[q][0], pv[q][1], lo, pv[q][0], pv[q][1]);
              if constexpr (RES) lines_to_pair(rv[q][0], rv[q][1], lo, rv[q][0], rv[q][1]);
            }
#pragma unroll
            for (int q = 0; q < GB; ++q)
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const floatx4 xh = (pv[q][h] - pp[0][h]) * pp[1][h];
                floatx4 v = (sv[q][h] - pp[2][h] - xh * pp[3][h]) * pp[4][h];
                if constexpr (RES) v += rv[q][h];
                xv[cc * IPC + q0 + q][h] = v;
              }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      };
      if (a.src_res) grad(std::true_type{});
      else grad(std::false_type{});
    } else {
#pragma unroll
      for (int i = 0; i < IPW; ++i)
#pragma unroll
        for (int e = 0; e < 2; ++e) xv[i][e] = ld4(a.src + lrow(i, e) * a.ld_src + lcol(i));
#pragma unroll
      for (int i = 0; i < IPW; ++i) lines_to_pair(xv[i][0], xv[i][1], lo, xv[i][0], xv[i][1]);
      if (a.prologue == AVR_BN_RELU) {
#pragma unroll
        for (int cc = 0; cc < NCH; ++cc)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = col_k(cc * IPC, h);
            const floatx4 mu = ld4(a.in_mu + k), sc = ld4(a.in_scale + k), sh = ld4(a.in_shift + k);
#pragma unroll
            for (int q = 0; q < IPC; ++q) xv[cc * IPC + q][h] = bn_relu4(xv[cc * IPC + q][h], mu, sc, sh);
          }
      }
    }
  } else {             // lin_in's z_feature rows (in_valid < in_dim, PLAIN): columns past in_valid are zeros
#pragma unroll
    for (int i = 0; i < IPW; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = col_k(i, h);
        const float* p = a.src + srow(i) * a.ld_src + k;
        floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
        if (k + 4 <= a.kin) {
          v = ld4(p);
        } else if (k < a.kin) {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = k + t < a.kin ? p[t] : 0.f;
        }
        xv[i][h] = v;
      }
  }
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const bool live = row_r(i) < nvalid;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!live) xv[i][h] = floatx4{0.f, 0.f, 0.f, 0.f};
      const floatx4 v = xv[i][h];
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float wgmax = red_max<NW>(red);
  if (a.opnd_max && wid == 0 && lane == 0) publish_max(a.opnd_max, wgmax);
  const float s_x = pow2_scale_for(wgmax);
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    uint2 hi0, lo0, hi1, lo1;
    split4(xv[i][0], s_x, hi0, lo0);
    split4(xv[i][1], s_x, hi1, lo1);
    X16[xidx(chunk(i), 0, g, row_r(i))] = make_uint4(hi0.x, hi0.y, hi1.x, hi1.y);
    X16[xidx(chunk(i), 1, g, row_r(i))] = make_uint4(lo0.x, lo0.y, lo1.x, lo1.y);
  }
  if (a.opnd_out) {    // after every prologue load: a store ahead of a load would hold its wait
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      floatx4 L[2];
      pair_to_lines(xv[i][0], xv[i][1], lo, L[0], L[1]);
#pragma unroll
      for (int e = 0; e < 2; ++e)
        if (lr(i, e) < nvalid)
          __builtin_nontemporal_store(L[e], reinterpret_cast<floatx4*>(a.opnd_out + (m0 + lr(i, e)) * KK + lcol(i)));
    }
  }
  lds_barrier();

  // ---------------------------------------------------------------- GEMM
  floatx4 acc[FT][4];
  bn_gemm<FT, NW, TWO>(acc, A0, W, KK / 32, 64 * FT * NW, X16, lane);
  const float inv = 1.0f / (pow2_scale_for(__uint_as_float(a.hdr[a.hdr_idx])) * s_x);

  // ---------------------------------------------------------------- epilogue
  const auto feat = [&](int ft) { return 16 * (FT * wid + ft) + 4 * g; };
  const auto live = [&](int sg) { return 16 * sg + j < nvalid; };
  const auto orow = [&](int sg) -> int64_t { return (m0 + (live(sg) ? 16 * sg + j : 0)) * HID; };
  // the rows' lines (FT even: tiles 2p, 2p + 1 are one 128-B line of a row; lines_to_pair): line row
  // 16 sg + 8 e + (j & 7), columns 16 (FT w + 2p) + 16 (j >> 3) + 4g
  const auto er = [&](int sg, int e) { return 16 * sg + 8 * e + (j & 7); };
  const auto eoff = [&](int sg, int e, int p) -> int64_t {
    return (m0 + (er(sg, e) < nvalid ? er(sg, e) : 0)) * HID + 16 * (FT * wid + 2 * p) + 16 * (j >> 3) + 4 * g;
  };
  // t = this lane's tiles of the rows at base (all loads issued, then the exchanges)
  const auto load_rows = [&](const float* base, floatx4 (&t)[FT][4]) {
    if constexpr (FT % 2 == 0) {
#pragma unroll
      for (int p = 0; p < FT / 2; ++p)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) {
          t[2 * p][sg] = ld4(base + eoff(sg, 0, p));
          t[2 * p + 1][sg] = ld4(base + eoff(sg, 1, p));
        }
#pragma unroll
      for (int p = 0; p < FT / 2; ++p)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) lines_to_pair(t[2 * p][sg], t[2 * p + 1][sg], lo, t[2 * p][sg], t[2 * p + 1][sg]);
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) t[ft][sg] = ld4(base + orow(sg) + feat(ft));
    }
  };
  const auto store_rows = [&](float* base, const floatx4 (&t)[FT][4]) {
    if constexpr (FT % 2 == 0) {
#pragma unroll
      for (int p = 0; p < FT / 2; ++p)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) {
          floatx4 L[2];
          pair_to_lines(t[2 * p][sg], t[2 * p + 1][sg], lo, L[0], L[1]);
#pragma unroll
          for (int e = 0; e < 2; ++e)
            if (er(sg, e) < nvalid) *reinterpret_cast<floatx4*>(base + eoff(sg, e, p)) = L[e];
        }
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg)
          if (live(sg)) *reinterpret_cast<floatx4*>(base + orow(sg) + feat(ft)) = t[ft][sg];
    }
  };
  const floatx4 zero4 = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 s1[FT], s2[FT];
  if constexpr (MODE == AVR_BN_FWD) {
    // out = W . op + bias (+ add1) (+ add2) (+ lin_z rows), added in that order (acc * inv is exact: a power of 2)
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const floatx4 b = a.bias ? ld4(a.bias + feat(ft)) : zero4;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) acc[ft][sg] = acc[ft][sg] * inv + b;
    }
    if (a.add1) {
      floatx4 t[FT][4];
      load_rows(a.add1, t);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) acc[ft][sg] += t[ft][sg];
    }
    if (a.add2) {
      floatx4 t[FT][4];
      load_rows(a.add2, t);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) acc[ft][sg] += t[ft][sg];
    }
    if (a.ztab) {   // the rows' lin_z features: avr_latent_features' lookup and blend order, bit for bit
      float px[4][3];
#pragma unroll
      for (int sg = 0; sg < 4; ++sg)
#pragma unroll
        for (int d = 0; d < 3; ++d) px[sg][d] = a.zxyz[3 * (orow(sg) / HID) + d];
      const int64_t sc0 = m0 / a.zrows;      // the workgroup's first scene (rows are scene-major)
      Bilinear bl[4];
      int64_t sc[4];
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const int64_t row = orow(sg) / HID;
        sc[sg] = sc0;
        while (row >= (sc[sg] + 1) * a.zrows) ++sc[sg];
        bl[sg] = bilinear_at(a.zviews[sc[sg]], px[sg][0], px[sg][1], px[sg][2]);
      }
      // one sample group's corners in flight at a time (all four would not fit beside the accumulators)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const float* tab = a.ztab + sc[sg] * a.ztab_stride;
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) {
          const int f = feat(ft);
          const floatx4 c0 = ld4(tab + (int64_t)bl[sg].tex[0] * HID + f);
          const floatx4 c1 = ld4(tab + (int64_t)bl[sg].tex[1] * HID + f);
          const floatx4 c2 = ld4(tab + (int64_t)bl[sg].tex[2] * HID + f);
          const floatx4 c3 = ld4(tab + (int64_t)bl[sg].tex[3] * HID + f);
          floatx4 z;
#pragma unroll
          for (int t = 0; t < 4; ++t)
            z[t] = fadd(fadd(fadd(fmul(c0[t], bl[sg].w[0]), fmul(c1[t], bl[sg].w[1])), fmul(c2[t], bl[sg].w[2])),
                        fmul(c3[t], bl[sg].w[3]));
          acc[ft][sg] += z;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    store_rows(a.out, acc);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      s1[ft] = zero4;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg)
        if (live(sg)) s1[ft] += acc[ft][sg];
    }
    // this workgroup's column means, then M2 about them (two-pass)
    const float rn = 1.0f / (float)nvalid;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      s1[ft] = sum16(s1[ft]) * rn;
      s2[ft] = zero4;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        if (live(sg)) {
          const floatx4 d = acc[ft][sg] - s1[ft];
          s2[ft] += d * d;
        }
      }
      s2[ft] = sum16(s2[ft]);
    }
  } else if (!a.pre_rows) {   // lin_z[b]^T (ABI 14): no mask, no statistics; add1 / the store below are shared
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      s1[ft] = zero4;
      s2[ft] = zero4;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) acc[ft][sg] = acc[ft][sg] * inv;
    }
  } else {
    // gp = (W^T . op) * relu mask of the forward operand, recomputed from the pre-BN row (bn_relu4, as the
    // forward did); the pre-BN rows also give xhat for the statistics (sums of gp and of gp * xhat)
    floatx4 pv[FT][4];
    load_rows(a.pre_rows, pv);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const int f = feat(ft);
      const floatx4 mu = ld4(a.out_mu + f), is = ld4(a.out_invstd + f);
      const floatx4 sc = ld4(a.out_scale + f), sh = ld4(a.out_shift + f);
      s1[ft] = zero4;
      s2[ft] = zero4;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const floatx4 z = bn_relu4(pv[ft][sg], mu, sc, sh);
        const floatx4 v = acc[ft][sg] * inv;
        floatx4 gp;
        gp.x = z.x > 0.f ? v.x : 0.f; gp.y = z.y > 0.f ? v.y : 0.f;
        gp.z = z.z > 0.f ? v.z : 0.f; gp.w = z.w > 0.f ? v.w : 0.f;
        acc[ft][sg] = gp;
        if (live(sg)) {
          const floatx4 xh = (pv[ft][sg] - mu) * is;
          s1[ft] += gp;
          s2[ft] += gp * xh;
        }
      }
      s1[ft] = sum16(s1[ft]);
      s2[ft] = sum16(s2[ft]);
    }
  }
  if constexpr (MODE == AVR_BN_BWD) {
    if (a.add1) {   // a residual gradient added to the stored rows (the statistics are of gp alone)
      floatx4 t[FT][4];
      load_rows(a.add1, t);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) acc[ft][sg] += t[ft][sg];
    }
    store_rows(a.out, acc);
    if (a.out_max) {   // the stored rows only (dead rows hold row m0's addend)
      float m = 0.f;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < 4; ++sg)
          if (live(sg)) {
            const floatx4 v = acc[ft][sg];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          }
      m = wave_max(m);
      if (lane == 0) publish_max(a.out_max, m);
    }
  }
  if (j == 0) {
    float* part = a.part + (int64_t)blockIdx.x * 2 * HID;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      *reinterpret_cast<floatx4*>(part + feat(ft)) = s1[ft];
      *reinterpret_cast<floatx4*>(part + HID + feat(ft)) = s2[ft];
    }
  }
}

template <int FT, int NW, int MODE, int KK>
static int launch_bn_layer(const BnArgs& a, hipStream_t s) {
  const size_t shm = (size_t)64 * KK * 4 + 64;   // X (64 samples x KK x hi + lo fp16) + the wave maxima
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bn_layer_kernel<FT, NW, MODE, KK>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return fail(AVR_E_HIP, "bn_layer_kernel: cannot set dynamic LDS");
    attr = true;
  }
  const int64_t blocks = (a.M + kX3Samples - 1) / kX3Samples;
  AVR_REQUIRE(blocks < (1ll << 31), "avr_bn_layer_run: too many rows");
  bn_layer_kernel<FT, NW, MODE, KK><<<(unsigned)blocks, 64 * NW, shm, s>>>(a);
  return check_launch("bn_layer_kernel");
}

// K is lin_in's 64 (forward) or d_hidden
template <int FT, int NW, int MODE>
static int launch_bn_layer_k(const BnArgs& a, hipStream_t s) {
  constexpr int HID = 16 * FT * NW;
  if (a.K == HID) return launch_bn_layer<FT, NW, MODE, HID>(a, s);
  if constexpr (MODE == AVR_BN_FWD && HID != 64) {
    if (a.K == 64) return launch_bn_layer<FT, NW, MODE, 64>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "avr_bn_layer_run: in_dim %d with d_hidden %d", a.K, HID);
}

template <int MODE>
static int dispatch_bn_layer(int H, const BnArgs& a, hipStream_t s) {
  switch (H) {
    case 64: return launch_bn_layer_k<1, 4, MODE>(a, s);
    case 128: return launch_bn_layer_k<2, 4, MODE>(a, s);
    case 256: return launch_bn_layer_k<4, 4, MODE>(a, s);
    case 512: return launch_bn_layer_k<4, 8, MODE>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "avr_bn_layer_run: d_hidden %d", H);
}

// ------------------------------------------------------------------ finalize
// Stage 2: block = 16 waves over 64 columns, wave q folds rows q, q + 16, ... of the stage-1 sums (two rows in
// flight per step), LDS meets the 16 wave sums in order (a 4-wave fold was a 40-step load-add chain, 15 µs).
constexpr int kBnFoldWaves = 16;

__device__ __forceinline__ void fold_rows(const double* __restrict__ fold, int nfold, int N, int c, double& a,
                                          double& b) {
  __shared__ double sa[64 * kBnFoldWaves], sb[64 * kBnFoldWaves];
  const int q = threadIdx.x >> 6;
  double a0 = 0.0, b0 = 0.0, a1 = 0.0, b1 = 0.0;
  if (c < N) {
    int f = q;
    for (; f + kBnFoldWaves < nfold; f += 2 * kBnFoldWaves) {
      a0 += fold[(int64_t)f * 2 * N + c];
      b0 += fold[(int64_t)f * 2 * N + N + c];
      a1 += fold[(int64_t)(f + kBnFoldWaves) * 2 * N + c];
      b1 += fold[(int64_t)(f + kBnFoldWaves) * 2 * N + N + c];
    }
    if (f < nfold) {
      a0 += fold[(int64_t)f * 2 * N + c];
      b0 += fold[(int64_t)f * 2 * N + N + c];
    }
  }
  sa[threadIdx.x] = a0 + a1;
  sb[threadIdx.x] = b0 + b1;
  __syncthreads();
  a = 0.0; b = 0.0;
#pragma unroll
  for (int w = 0; w < kBnFoldWaves; ++w) {
    a += sa[64 * w + (threadIdx.x & 63)];
    b += sb[64 * w + (threadIdx.x & 63)];
  }
}

__global__ void __launch_bounds__(64 * kBnFoldWaves) bn_stats_kernel(const double* __restrict__ fold, int nfold,
                                                                    int64_t M, int N,
                                                       const float* __restrict__ gamma, float eps, float momentum,
                                                       float* running_mean, float* running_var, float* mu_out,
                                                       float* invstd_out, float* scale_out) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double a, b;
  fold_rows(fold, nfold, N, c, a, b);
  if (threadIdx.x >= 64 || c >= N) return;
  const double n = (double)M, mean = a / n;
  const double m2 = fmax(b - n * mean * mean, 0.0);
  const double var = m2 / n;                                    // biased: the normalisation (torch)
  const float istd = (float)(1.0 / sqrt(var + (double)eps));
  mu_out[c] = (float)mean;
  invstd_out[c] = istd;
  scale_out[c] = gamma[c] * istd;
  if (running_mean) {                                           // torch: unbiased variance in the running stat
    const float unb = (float)(n > 1.0 ? m2 / (n - 1.0) : var);
    running_mean[c] = momentum * (float)mean + (1.0f - momentum) * running_mean[c];
    running_var[c] = momentum * unb + (1.0f - momentum) * running_var[c];
  }
}

__global__ void __launch_bounds__(64 * kBnFoldWaves) bn_grad_stats_kernel(const double* __restrict__ fold, int nfold,
                                                                         int64_t M,
                                                            int N, const float* __restrict__ gamma,
                                                            const float* __restrict__ invstd, float* coef, float* m1,
                                                            float* m2, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double a, b;
  fold_rows(fold, nfold, N, c, a, b);
  if (threadIdx.x >= 64 || c >= N) return;
  m1[c] = (float)(a / (double)M);
  m2[c] = (float)(b / (double)M);
  coef[c] = gamma[c] * invstd[c];
  dbeta[c] += (float)a;       // bn_0 is applied twice per block: both applications add into its gradients
  dgamma[c] += (float)b;
}

// Grid (column groups of 4 x 64, rows / 16): thread (x, y) handles column group 64 blockIdx.x + (x & 63) of rows
// 16 blockIdx.y + (x >> 6) + 4 k, k < 4: coalesced 1-KB row segments, the column parameters loaded once per
// thread, and all twelve row loads issued before the first store (out is __restrict__: nothing orders them).
__global__ void __launch_bounds__(256) bn_grad_rows_kernel(int64_t n_rows, int N4, const floatx4* __restrict__ gr,
                                                           const floatx4* __restrict__ pre,
                                                           const floatx4* __restrict__ res,
                                                           const floatx4* __restrict__ coef,
                                                           const floatx4* __restrict__ m1,
                                                           const floatx4* __restrict__ m2,
                                                           const floatx4* __restrict__ mu,
                                                           const floatx4* __restrict__ invstd,
                                                           floatx4* __restrict__ out, unsigned* out_max) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int64_t r0 = (int64_t)blockIdx.y * 16 + (threadIdx.x >> 6);
  float mx = 0.f;
  if (c < N4) {
    const floatx4 cf = coef[c], a1 = m1[c], a2 = m2[c], u = mu[c], is = invstd[c];
    floatx4 g[4], p[4], q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t r = r0 + 4 * k < n_rows ? r0 + 4 * k : n_rows - 1;   // clamped rows are loaded, not stored
      const int64_t i = r * N4 + c;
      g[k] = gr[i];
      p[k] = pre[i];
      q[k] = res ? res[i] : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (r0 + 4 * k < n_rows) {
        floatx4 v = (g[k] - a1 - (p[k] - u) * is * a2) * cf;
        if (res) v += q[k];
        out[(r0 + 4 * k) * N4 + c] = v;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    }
  }
  // one publish per block (publish_max: thousands of blocks' atomics on one word serialise at its L2 channel;
  // one per wave took most of this kernel's time)
  __shared__ float red[4];
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0 && out_max) {
    publish_max(out_max, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// Two-stage finalize: stage 1 (grid column blocks x row groups of 16 partials, one wave each: lane = column,
// coalesced 256-B partial rows) folds 16 workgroups' partials into fp64 sums; stage 2 (one wave per 64 columns)
// folds those. Forward partials are per-workgroup (mean, M2) of n_i rows: A1 = sum n_i mean_i and
// A2 = sum (M2_i + n_i mean_i^2), then M2 = A2 - n mean^2 (fp64: no Chan divisions, no cancellation at fp32
// scale). Backward partials are plain sums.
constexpr int kBnFold = 16;

template <bool FWD>
__global__ void __launch_bounds__(64) bn_fold_kernel(const float* __restrict__ part, int64_t M, int N,
                                                     double* __restrict__ fold) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  const int64_t nwg = (M + kX3Samples - 1) / kX3Samples;
  double a = 0.0, b = 0.0;
  if (c < N) {
#pragma unroll 8
    for (int64_t w = (int64_t)blockIdx.y * kBnFold; w < nwg && w < (int64_t)(blockIdx.y + 1) * kBnFold; ++w) {
      const float p0 = part[w * 2 * N + c], p1 = part[w * 2 * N + N + c];
      if constexpr (FWD) {
        const double n = (double)(M - w * kX3Samples < kX3Samples ? M - w * kX3Samples : kX3Samples);
        a += n * (double)p0;
        b += (double)p1 + n * (double)p0 * (double)p0;
      } else {
        a += (double)p0;
        b += (double)p1;
      }
    }
    fold[(int64_t)blockIdx.y * 2 * N + c] = a;
    fold[(int64_t)blockIdx.y * 2 * N + N + c] = b;
  }
}

}  // namespace avr


using namespace avr;

extern "C" int avr_bn_layer_run(const avr_field_dims* dims, const avr_bn_layer* l, void* stream) {
  Layout L;
  int rc = field_layout(dims, &L);
  if (rc) return rc;
  AVR_REQUIRE(l, "avr_bn_layer_run: null layer");
  // use_spade blobs too (ABI 13: avr.layer_train runs spade / NS > 1 nets layer by layer; the layer reads only
  // lin_in / fc_0 / fc_1 fragments and the header, whose offsets the layout computes for either)
  AVR_REQUIRE(dims->precision == AVR_FIELD_X3 && !dims->bn && !(dims->beta > 0.f),
              "avr_bn_layer_run: an x3 blob packed without eval-BN folding (dims->bn = 0), ReLU");
  AVR_REQUIRE(l->mode == AVR_BN_FWD || l->mode == AVR_BN_BWD, "avr_bn_layer_run: bad mode %d", l->mode);
  AVR_REQUIRE(l->prologue >= AVR_BN_PLAIN && l->prologue <= AVR_BN_GRAD, "avr_bn_layer_run: bad prologue");
  AVR_REQUIRE(l->n_rows >= 0, "avr_bn_layer_run: bad row count");
  if (l->n_rows == 0) return AVR_OK;
  const int H = dims->d_hidden, nb = dims->n_blocks;
  BnArgs a{};
  a.M = l->n_rows;
  a.prologue = l->prologue;
  a.K = l->in_dim;
  a.kin = l->in_valid;
  a.KC = l->in_dim / 32;
  AVR_REQUIRE(l->in_dim % 64 == 0 && l->in_dim >= 64 && l->in_dim <= 512 && l->in_dim / 4 % (H == 512 ? 8 : 4) == 0,
              "avr_bn_layer_run: in_dim %d", l->in_dim);
  AVR_REQUIRE(l->in_valid > 0 && l->in_valid <= l->in_dim && (l->in_valid == l->in_dim || l->in_dim == 64),
              "avr_bn_layer_run: in_valid %d (< in_dim only for lin_in's 64 columns)", l->in_valid);
  AVR_REQUIRE(l->src && l->out && l->partial && l->blob, "avr_bn_layer_run: null pointer");
  AVR_REQUIRE(l->ld_src >= l->in_valid && l->ld_src % 4 == 0,
              "avr_bn_layer_run: ld_src %lld (>= in_valid, a multiple of 4: 16-B rows)", (long long)l->ld_src);
  AVR_REQUIRE(l->prologue != AVR_BN_RELU || (l->in_mu && l->in_scale && l->in_shift),
              "avr_bn_layer_run: AVR_BN_RELU needs in_mu / in_scale / in_shift");
  AVR_REQUIRE(l->prologue != AVR_BN_GRAD || (l->src_pre && l->in_mu && l->in_scale && l->in_m1 && l->in_m2 &&
                                             l->in_invstd),
              "avr_bn_layer_run: AVR_BN_GRAD needs src_pre, in_mu / scale / m1 / m2 / invstd");
  a.src = l->src; a.ld_src = l->ld_src; a.src_pre = l->src_pre; a.src_res = l->src_res;
  a.in_mu = l->in_mu; a.in_scale = l->in_scale; a.in_shift = l->in_shift;
  a.in_m1 = l->in_m1; a.in_m2 = l->in_m2; a.in_invstd = l->in_invstd;
  a.opnd_out = l->operand_out;
  a.opnd_max = l->operand_max;
  // the layer's fragments and its header word (0 lin_in, 2 + 2b fc_0[b], 3 + 2b fc_1[b])
  const int ly = l->layer;
  const bool lzt = l->mode == AVR_BN_BWD && ly >= AVR_BN_LAYER_LIN_Z_T && ly < AVR_BN_LAYER_LIN_Z_T + dims->n_lin_z;
  AVR_REQUIRE(ly == 0 || (ly >= 2 && ly < 2 + 2 * nb) || lzt, "avr_bn_layer_run: layer %d", ly);
  const unsigned* hdr;
  if (l->mode == AVR_BN_FWD) {
    AVR_REQUIRE(ly != 0 || l->in_dim == 64, "avr_bn_layer_run: lin_in's operand is 64 columns");
    AVR_REQUIRE(ly == 0 || l->in_dim == H, "avr_bn_layer_run: a hidden layer's operand is d_hidden columns");
    a.w = l->blob + (ly == 0 ? L.x3_in : (ly % 2 == 0 ? L.x3_fc0[(ly - 2) / 2] : L.x3_fc1[(ly - 2) / 2]));
    hdr = reinterpret_cast<const unsigned*>(l->blob + L.x3_hdr);
    AVR_REQUIRE(!l->out_max, "avr_bn_layer_run: out_max is a backward-mode field");
    a.bias = l->bias; a.add1 = l->add1; a.add2 = l->add2;
    if (l->lin_z_table) {
      AVR_REQUIRE(l->xyz && l->views && l->n_views >= 1 && l->n_views <= AVR_MAX_SCENES && l->rows_per_scene > 0 &&
                      l->rows_per_scene * l->n_views == l->n_rows && l->lin_z_scene_stride >= 0 &&
                      l->lin_z_scene_stride % 4 == 0 && reinterpret_cast<uintptr_t>(l->lin_z_table) % 16 == 0,
                  "avr_bn_layer_run: lin_z_table needs xyz, 1..%d views of rows_per_scene rows each (n_rows in "
                  "all), a 16-B aligned table", AVR_MAX_SCENES);
      for (int v = 0; v < l->n_views; ++v) {
        AVR_REQUIRE(l->views[v].latent_h > 0 && l->views[v].latent_w > 0, "avr_bn_layer_run: view %d latent size", v);
        view_from_desc(&l->views[v], &a.zviews[v]);
      }
      a.ztab = l->lin_z_table; a.ztab_stride = l->lin_z_scene_stride; a.zrows = l->rows_per_scene; a.zxyz = l->xyz;
    }
  } else {
    AVR_REQUIRE(ly >= 2 && l->in_dim == H,
                "avr_bn_layer_run: the backward runs fc_0 / fc_1 / lin_z (d_hidden columns)");
    BwdLayout LB;
    if ((rc = field_bwd_layout(dims, &LB))) return rc;
    if (lzt) {
      AVR_REQUIRE(LB.lzt[ly - AVR_BN_LAYER_LIN_Z_T] >= 0,
                  "avr_bn_layer_run: lin_z^T needs d_latent == d_hidden (%d, %d) and no use_spade", dims->d_latent, H);
      AVR_REQUIRE(!l->pre_rows && !l->out_mu && !l->out_invstd && !l->out_scale && !l->out_shift,
                  "avr_bn_layer_run: lin_z^T has no relu mask (pre_rows / out_* NULL)");
      a.w = l->blob + LB.lzt[ly - AVR_BN_LAYER_LIN_Z_T];
    } else {
      AVR_REQUIRE(l->pre_rows && l->out_mu && l->out_invstd && l->out_scale && l->out_shift,
                  "avr_bn_layer_run: AVR_BN_BWD needs pre_rows, out_mu, out_invstd, out_scale, out_shift");
      a.w = l->blob + (ly % 2 == 0 ? LB.fc0t[(ly - 2) / 2] : LB.fc1t[(ly - 2) / 2]);
    }
    hdr = reinterpret_cast<const unsigned*>(l->blob);
    AVR_REQUIRE(!l->add2 && !l->lin_z_table, "avr_bn_layer_run: AVR_BN_BWD adds add1 only");
    a.pre_rows = l->pre_rows; a.out_mu = l->out_mu; a.out_invstd = l->out_invstd;
    a.out_scale = l->out_scale; a.out_shift = l->out_shift;
    a.add1 = l->add1;
    a.out_max = l->out_max;
  }
  a.hdr = hdr;
  a.hdr_idx = ly;
  a.out = l->out;
  a.part = l->partial;
  hipStream_t s = as_stream(stream);   // the weight scale is read on the device (the pack launch wrote it)
  return l->mode == AVR_BN_FWD ? dispatch_bn_layer<AVR_BN_FWD>(H, a, s) : dispatch_bn_layer<AVR_BN_BWD>(H, a, s);
}

// The fold scratch (fp64, 2 x n_cols per 16 partials) lives in the partial buffer past the partials
// (avr_bn_partial_floats sizes it), so the entry points allocate nothing.
static int64_t bn_n_fold(int64_t n_rows) { return ((n_rows + kX3Samples - 1) / kX3Samples + kBnFold - 1) / kBnFold; }

extern "C" int avr_bn_partial_floats(int64_t n_rows, int n_cols, int64_t* n_floats) {
  AVR_REQUIRE(n_rows >= 0 && n_cols > 0 && n_floats, "avr_bn_partial_floats: bad argument");
  const int64_t nwg = (n_rows + kX3Samples - 1) / kX3Samples;
  // partials (nwg, 2, n_cols) fp32, then 8-B aligned fold rows (n_fold, 2, n_cols) fp64
  *n_floats = (nwg * 2 * n_cols + 1) / 2 * 2 + bn_n_fold(n_rows) * 2 * n_cols * 2;
  return AVR_OK;
}

static const float* bn_fold(const float* partial, int64_t n_rows, int n_cols, bool fwd, double** fold,
                            hipStream_t s) {
  const int64_t nwg = (n_rows + kX3Samples - 1) / kX3Samples;
  *fold = reinterpret_cast<double*>(const_cast<float*>(partial) + (nwg * 2 * n_cols + 1) / 2 * 2);
  const dim3 grid((unsigned)((n_cols + 63) / 64), (unsigned)bn_n_fold(n_rows));
  if (fwd)
    bn_fold_kernel<true><<<grid, 64, 0, s>>>(partial, n_rows, n_cols, *fold);
  else
    bn_fold_kernel<false><<<grid, 64, 0, s>>>(partial, n_rows, n_cols, *fold);
  return partial;
}

extern "C" int avr_bn_stats(const float* partial, int64_t n_rows, int n_cols, const float* gamma, float eps,
                            float momentum, float* running_mean, float* running_var, float* mu, float* invstd,
                            float* scale, void* stream) {
  AVR_REQUIRE(n_rows >= 2, "avr_bn_stats: BatchNorm in training mode needs more than 1 value per channel");
  AVR_REQUIRE(n_cols > 0 && partial && gamma && mu && invstd && scale, "avr_bn_stats: bad argument");
  AVR_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "avr_bn_stats: running mean / var together");
  hipStream_t s = as_stream(stream);
  double* fold;
  bn_fold(partial, n_rows, n_cols, true, &fold, s);
  int rc = check_launch("bn_fold_kernel");
  if (rc) return rc;
  bn_stats_kernel<<<(unsigned)((n_cols + 63) / 64), 64 * kBnFoldWaves, 0, s>>>(fold, (int)bn_n_fold(n_rows), n_rows,
                                                                             n_cols, gamma,
                                                                 eps, momentum, running_mean, running_var, mu, invstd,
                                                                 scale);
  return check_launch("bn_stats_kernel");
}

extern "C" int avr_bn_grad_stats(const float* partial, int64_t n_rows, int n_cols, const float* gamma,
                                 const float* invstd, float* coef, float* m1, float* m2, float* dgamma, float* dbeta,
                                 void* stream) {
  AVR_REQUIRE(n_rows >= 1 && n_cols > 0, "avr_bn_grad_stats: bad sizes");
  AVR_REQUIRE(partial && gamma && invstd && coef && m1 && m2 && dgamma && dbeta, "avr_bn_grad_stats: null pointer");
  hipStream_t s = as_stream(stream);
  double* fold;
  bn_fold(partial, n_rows, n_cols, false, &fold, s);
  int rc = check_launch("bn_fold_kernel");
  if (rc) return rc;
  bn_grad_stats_kernel<<<(unsigned)((n_cols + 63) / 64), 64 * kBnFoldWaves, 0, s>>>(fold, (int)bn_n_fold(n_rows),
                                                                                  n_rows, n_cols,
                                                                      gamma, invstd, coef, m1, m2, dgamma, dbeta);
  return check_launch("bn_grad_stats_kernel");
}

extern "C" int avr_bn_grad_rows(int64_t n_rows, int n_cols, const float* g, const float* pre, const float* res,
                                const float* coef, const float* m1, const float* m2, const float* mu,
                                const float* invstd, float* out, uint32_t* out_max, void* stream) {
  AVR_REQUIRE(n_rows >= 0 && n_cols > 0 && n_cols % 4 == 0, "avr_bn_grad_rows: bad sizes");
  if (n_rows == 0) return AVR_OK;
  AVR_REQUIRE(g && pre && coef && m1 && m2 && mu && invstd && out, "avr_bn_grad_rows: null pointer");
  const int N4 = n_cols / 4;
  const dim3 grid((unsigned)((N4 + 63) / 64), (unsigned)((n_rows + 15) / 16));
  bn_grad_rows_kernel<<<grid, 256, 0, as_stream(stream)>>>(
      n_rows, N4, reinterpret_cast<const floatx4*>(g), reinterpret_cast<const floatx4*>(pre),
      reinterpret_cast<const floatx4*>(res), reinterpret_cast<const floatx4*>(coef),
      reinterpret_cast<const floatx4*>(m1), reinterpret_cast<const floatx4*>(m2),
      reinterpret_cast<const floatx4*>(mu), reinterpret_cast<const floatx4*>(invstd),
      reinterpret_cast<floatx4*>(out), out_max);
  return check_launch("bn_grad_rows_kernel");
}
