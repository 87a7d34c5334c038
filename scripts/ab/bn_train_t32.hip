// REJECTED A/B variant (not built by the Makefile; profiles/r05ab_bn_t32_rejected.txt): bn_train.hip with 32-row tiles on
// 4-wave workgroups at d_hidden 512, two workgroups per CU. Correct (BN / layer-train GPU tests green) but slower than the
// one-tile 64-row kernel: fc_1 forward 488 vs 427 us, --bn step 29.9 vs 27.9 ms (the doubled weight stream per row).
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
// recomputed from the pre-BN rows: the relu'd operands are never stored), stores the rows and
// reduces this workgroup's column statistics. A finalize launch between
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

// A layer GEMM over tiles of NSG sample groups (16 rows each), in three parts shared by the two kernels below.
// NG waves share a tile; wave gw of the group holds the output features 16 (FT gw + ft) + 4g .. +3 of rows
// 16 sg + j (lane = (g, j)). MODE 0 forward, 1 backward; KK = K (64: lin_in, or d_hidden).
// * operand (bn_operand): the K columns of the tile are KK / 32 * NSG items (32-column chunk c, sample group sg);
//   wave gw takes IPW consecutive items; lane (g, j) needs, for each, exactly its B-fragment columns 32c + 4g .. +3
//   and 32c + 16 + 4g .. +3 of row 16 sg + j, loaded as whole 128-B row lines and exchanged (lines_to_pair), with
//   the prologue's transform applied. The values wait in registers until the tile's max |operand| is known; then
//   (bn_split) one 16-B hi and one 16-B lo LDS write per item put them in the GEMM's X slots (xslot: conflict-free,
//   consecutive j in consecutive slots).
// * GEMM: the fused kernels' split-fp16 K loop on those slots.
// * epilogue (bn_epilogue) straight from the accumulators: the addend / pre-BN loads and the row stores move
//   whole lines (pair_to_lines), and since a wave owns its columns for all rows of the tile, a column's statistics
//   are in-lane sums over the sample groups and a 16-lane DPP reduction over j -- no LDS, no barrier.
template <int NSG>
__device__ __forceinline__ int xslot(int c, int part, int g, int s) { return ((c * 2 + part) * 4 + g) * (16 * NSG) + s; }

template <int NG, int KK, int NSG>
struct BnItems {
  static constexpr int NIT = KK / 32 * NSG;                 // operand items of a tile
  static constexpr int IPW = (NIT + NG - 1) / NG;            // items per wave (the last waves may have fewer)
  static constexpr bool CHUNKED = IPW % NSG == 0;            // a wave's items are whole chunks
};

// item i of wave gw: it = IPW gw + i (< NIT), chunk it / NSG, sample group it % NSG, row r = 16 sg + j (rows past
// the end load row m0 and become zeros); half h: columns 32 c + 16 h + 4 g .. +3. Returns the lane's max |value|.
template <int NG, int KK, int NSG>
__device__ __forceinline__ float bn_operand(const BnArgs& a, int64_t m0, int nvalid, int gw, int lane,
                                            floatx4 (&xv)[BnItems<NG, KK, NSG>::IPW][2]) {
  using It = BnItems<NG, KK, NSG>;
  constexpr int IPW = It::IPW;
  const int g = lane >> 4, j = lane & 15;
  const int i0 = IPW * gw;
  const auto has = [&](int i) { return IPW * NG == It::NIT || i0 + i < It::NIT; };   // wave-uniform
  const auto chunk = [&](int i) { return (i0 + i) / NSG; };
  const auto sgi = [&](int i) { return (i0 + i) % NSG; };
  const auto row_r = [&](int i) { return 16 * sgi(i) + j; };
  const auto col_k = [&](int i, int h) { return 32 * chunk(i) + 16 * h + 4 * g; };
  // the item's rows as lines (see lines_to_pair): line row lr(i, half), columns 32 c + 16 (j >> 3) + 4 g
  const bool lo = j < 8;
  const auto lr = [&](int i, int half) { return 16 * sgi(i) + 8 * half + (j & 7); };
  // offsets (32-bit, per lane) from the tile's first row (a wave-uniform base: one SGPR pair, not a 64-bit
  // address per load)
  const int ld = (int)a.ld_src;
  const auto lcol = [&](int i) { return 32 * chunk(i) + 16 * (j >> 3) + 4 * g; };
  const auto loff = [&](int i, int half) { return (unsigned)((lr(i, half) < nvalid ? lr(i, half) : 0) * ld + lcol(i)); };
  const auto soff = [&](int i) { return (unsigned)((row_r(i) < nvalid ? row_r(i) : 0) * ld); };
  const float* src = a.src + m0 * a.ld_src;
  const float* src_pre = a.src_pre + m0 * a.ld_src;
  const float* src_res = a.src_res + m0 * a.ld_src;
#pragma unroll
  for (int i = 0; i < IPW; ++i) xv[i][0] = xv[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (KK != 64 || a.kin == KK) {   // whole 16-B groups (every hidden layer): a batch's loads back to back, branch-free
    if (a.prologue == AVR_BN_GRAD) {
      // three rows per value (gradient, pre-BN, residual): one chunk's parameters and two items per batch, the
      // residual's presence decided once (a null check per load would keep each load behind its own branch)
      static_assert(KK == 64 || It::CHUNKED, "hidden layers: whole chunks per wave");
      const auto grad = [&](auto res_t) {
        constexpr bool RES = decltype(res_t)::value;
        constexpr int PC = It::CHUNKED ? NSG : 1;   // items sharing one parameter load
#pragma unroll
        for (int c0 = 0; c0 < IPW; c0 += PC) {
          if (!has(c0)) break;
          floatx4 pp[5][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = col_k(c0, h);
            pp[0][h] = ld4(a.in_mu + k); pp[1][h] = ld4(a.in_invstd + k); pp[2][h] = ld4(a.in_m1 + k);
            pp[3][h] = ld4(a.in_m2 + k); pp[4][h] = ld4(a.in_scale + k);
          }
          constexpr int GB = PC < 2 ? PC : 2;   // items per batch
#pragma unroll
          for (int q0 = 0; q0 < PC; q0 += GB) {
            constexpr int GBq = GB;
            floatx4 sv[GBq][2], pv[GBq][2], rv[GBq][2];
            const int nq = q0 + GB <= PC ? GB : PC - q0;
#pragma unroll
            for (int q = 0; q < GBq; ++q)
#pragma unroll
              for (int e = 0; e < 2; ++e) {   // line e (A / B); past the chunk's items: item c0's rows again
                const int i = c0 + (q < nq ? q0 + q : 0);
                const unsigned o = loff(i, e);
                sv[q][e] = ld4(src + o);
                pv[q][e] = ld4(src_pre + o);
                if constexpr (RES) rv[q][e] = ld4(src_res + o);
              }
#pragma unroll
            for (int q = 0; q < GBq; ++q) {
              lines_to_pair(sv[q][0], sv[q][1], lo, sv[q][0], sv[q][1]);
              lines_to_pair(pv[q][0], pv[q][1], lo, pv[q][0], pv[q][1]);
              if constexpr (RES) lines_to_pair(rv[q][0], rv[q][1], lo, rv[q][0], rv[q][1]);
            }
#pragma unroll
            for (int q = 0; q < GBq; ++q) {
              if (q >= nq) break;
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const floatx4 xh = (pv[q][h] - pp[0][h]) * pp[1][h];
                floatx4 v = (sv[q][h] - pp[2][h] - xh * pp[3][h]) * pp[4][h];
                if constexpr (RES) v += rv[q][h];
                xv[c0 + q0 + q][h] = v;
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      };
      if (a.src_res) grad(std::true_type{});
      else grad(std::false_type{});
    } else {
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const int ii = has(i) ? i : 0;     // (a wave past the last item loads its first item's rows again)
#pragma unroll
        for (int e = 0; e < 2; ++e) xv[i][e] = ld4(src + loff(ii, e));
      }
#pragma unroll
      for (int i = 0; i < IPW; ++i) lines_to_pair(xv[i][0], xv[i][1], lo, xv[i][0], xv[i][1]);
      if (a.prologue == AVR_BN_RELU) {
        constexpr int PC = It::CHUNKED ? NSG : 1;
#pragma unroll
        for (int c0 = 0; c0 < IPW; c0 += PC)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = col_k(c0, h);
            const floatx4 mu = ld4(a.in_mu + k), sc = ld4(a.in_scale + k), sh = ld4(a.in_shift + k);
#pragma unroll
            for (int q = 0; q < PC; ++q) xv[c0 + q][h] = bn_relu4(xv[c0 + q][h], mu, sc, sh);
          }
      }
    }
  } else {             // lin_in's z_feature rows (in_valid < in_dim, PLAIN): columns past in_valid are zeros
#pragma unroll
    for (int i = 0; i < IPW; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = col_k(i, h);
        const float* p = src + soff(has(i) ? i : 0) + k;
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
    const bool live = has(i) && row_r(i) < nvalid;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!live) xv[i][h] = floatx4{0.f, 0.f, 0.f, 0.f};
      const floatx4 v = xv[i][h];
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  }
  return mx;
}

// xv -> the X slots under the scale s_x (and the operand rows to opnd_out: after every operand load, since a
// store ahead of a load would hold that load's wait)
template <int NG, int KK, int NSG>
__device__ __forceinline__ void bn_split(const BnArgs& a, uint4* X16,
                                         const floatx4 (&xv)[BnItems<NG, KK, NSG>::IPW][2], float s_x, int64_t m0,
                                         int nvalid, int gw, int lane) {
  using It = BnItems<NG, KK, NSG>;
  constexpr int IPW = It::IPW;
  const int g = lane >> 4, j = lane & 15;
  const int i0 = IPW * gw;
  const auto has = [&](int i) { return IPW * NG == It::NIT || i0 + i < It::NIT; };
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    if (!has(i)) break;
    uint2 hi0, lo0, hi1, lo1;
    split4(xv[i][0], s_x, hi0, lo0);
    split4(xv[i][1], s_x, hi1, lo1);
    const int c = (i0 + i) / NSG, r = 16 * ((i0 + i) % NSG) + j;
    X16[xslot<NSG>(c, 0, g, r)] = make_uint4(hi0.x, hi0.y, hi1.x, hi1.y);
    X16[xslot<NSG>(c, 1, g, r)] = make_uint4(lo0.x, lo0.y, lo1.x, lo1.y);
  }
  if (a.opnd_out) {
    const bool lo = j < 8;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if (!has(i)) break;
      floatx4 L[2];
      pair_to_lines(xv[i][0], xv[i][1], lo, L[0], L[1]);
      const int col = 32 * ((i0 + i) / NSG) + 16 * (j >> 3) + 4 * g;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int r = 16 * ((i0 + i) % NSG) + 8 * e + (j & 7);
        if (r < nvalid)
          __builtin_nontemporal_store(L[e], reinterpret_cast<floatx4*>(a.opnd_out + (m0 + r) * KK + col));
      }
    }
  }
}

// acc (W . X, unscaled) -> the layer's rows and this tile's column statistics (part row `tile`). PB: line pairs
// per load batch (the addend / pre-BN rows of PB pairs in flight beside the accumulators).
// ZT: the lin_z gather (ztab) compiled in (at 512 columns only in the one-tile kernel: beside the persistent
// kernel's two roles it does not fit the registers)
template <int FT, int NG, int MODE, int NSG, int PB, bool ZT = true>
__device__ __forceinline__ void bn_epilogue(const BnArgs& a, floatx4 (&acc)[FT][NSG], float inv, int64_t m0,
                                            int nvalid, int gw, int lane, int64_t tile) {
  constexpr int HID = 16 * FT * NG;
  const int g = lane >> 4, j = lane & 15;
  const bool lo = j < 8;
  const auto feat = [&](int ft) { return 16 * (FT * gw + ft) + 4 * g; };
  const auto live = [&](int sg) { return 16 * sg + j < nvalid; };
  // offsets (32-bit, per lane) from the tile's first row: base + m0 * HID is wave-uniform
  const auto orow = [&](int sg) { return (unsigned)((live(sg) ? 16 * sg + j : 0) * HID); };
  // the rows' lines (FT even: tiles 2p, 2p + 1 are one 128-B line of a row; lines_to_pair): line row
  // 16 sg + 8 e + (j & 7), columns 16 (FT gw + 2p) + 16 (j >> 3) + 4g
  const auto er = [&](int sg, int e) { return 16 * sg + 8 * e + (j & 7); };
  const auto eoff = [&](int sg, int e, int p) {
    return (unsigned)((er(sg, e) < nvalid ? er(sg, e) : 0) * HID + 16 * (FT * gw + 2 * p) + 16 * (j >> 3) + 4 * g);
  };
  // f(ft, sg, t) for every tile with t = the lane's value of the rows at base; loads of PB line pairs in flight
  const auto with_rows = [&](const float* base0, auto f) {
    const float* base = base0 + m0 * HID;
    if constexpr (FT % 2 == 0) {
      constexpr int NP = FT / 2, B = PB < NP ? PB : NP;
#pragma unroll
      for (int p0 = 0; p0 < NP; p0 += B) {
        floatx4 t[B][2][NSG];
#pragma unroll
        for (int q = 0; q < B; ++q)
#pragma unroll
          for (int sg = 0; sg < NSG; ++sg) {
            t[q][0][sg] = ld4(base + eoff(sg, 0, p0 + q));
            t[q][1][sg] = ld4(base + eoff(sg, 1, p0 + q));
          }
#pragma unroll
        for (int q = 0; q < B; ++q)
#pragma unroll
          for (int sg = 0; sg < NSG; ++sg) {
            lines_to_pair(t[q][0][sg], t[q][1][sg], lo, t[q][0][sg], t[q][1][sg]);
            f(2 * (p0 + q), sg, t[q][0][sg]);
            f(2 * (p0 + q) + 1, sg, t[q][1][sg]);
          }
      }
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) f(ft, sg, ld4(base + orow(sg) + feat(ft)));
    }
  };
  const auto store_rows = [&](float* base0) {
    float* base = base0 + m0 * HID;
    if constexpr (FT % 2 == 0) {
#pragma unroll
      for (int p = 0; p < FT / 2; ++p)
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
          floatx4 L[2];
          pair_to_lines(acc[2 * p][sg], acc[2 * p + 1][sg], lo, L[0], L[1]);
#pragma unroll
          for (int e = 0; e < 2; ++e)
            if (er(sg, e) < nvalid) *reinterpret_cast<floatx4*>(base + eoff(sg, e, p)) = L[e];
        }
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg)
          if (live(sg)) *reinterpret_cast<floatx4*>(base + orow(sg) + feat(ft)) = acc[ft][sg];
    }
  };
  const floatx4 zero4 = floatx4{0.f, 0.f, 0.f, 0.f};
  float* part = a.part + tile * 2 * HID;
  const auto put_stats = [&](int ft, floatx4 t1, floatx4 t2) {
    if (j == 0) {
      *reinterpret_cast<floatx4*>(part + feat(ft)) = t1;
      *reinterpret_cast<floatx4*>(part + HID + feat(ft)) = t2;
    }
  };
  if constexpr (MODE == AVR_BN_FWD) {
    // out = W . op + bias (+ add1) (+ add2) (+ lin_z rows), added in that order (acc * inv is exact: a power of 2)
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const floatx4 b = a.bias ? ld4(a.bias + feat(ft)) : zero4;
#pragma unroll
      for (int sg = 0; sg < NSG; ++sg) acc[ft][sg] = acc[ft][sg] * inv + b;
    }
    const auto add = [&](int ft, int sg, floatx4 t) { acc[ft][sg] += t; };
    if (a.add1) with_rows(a.add1, add);
    if (a.add2) with_rows(a.add2, add);
    if (ZT && a.ztab) {   // the rows' lin_z features: avr_latent_features' lookup and blend order, bit for bit
      if constexpr (NSG == 4) {
        // every sample group's bilinear first (the lane's scene by a per-lane search), then one sample group's
        // corners in flight at a time
        float px[NSG][3];
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg)
#pragma unroll
          for (int d = 0; d < 3; ++d) px[sg][d] = a.zxyz[3 * (m0 + orow(sg) / HID) + d];
        const int64_t sc0 = m0 / a.zrows;      // the tile's first scene (rows are scene-major)
        Bilinear bl[NSG];
        int64_t sc[NSG];
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
          const int64_t row = m0 + orow(sg) / HID;
          sc[sg] = sc0;
          while (row >= (sc[sg] + 1) * a.zrows) ++sc[sg];
          bl[sg] = bilinear_at(a.zviews[sc[sg]], px[sg][0], px[sg][1], px[sg][2]);
        }
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
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
      } else {
        // one sample group's bilinear at a time, the corners of ZB tiles in flight (all of them would not fit beside
        // the accumulators). The scenes a sample group spans are a wave-uniform range (rows are scene-major): the
        // views are read with uniform indices, each lane keeping the one of its row's scene.
        constexpr int ZB = FT < 2 ? FT : 2;
  #pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
          const int64_t row = m0 + orow(sg) / HID;
          const int last = 16 * sg + 15 < nvalid - 1 ? 16 * sg + 15 : nvalid - 1;
          const int64_t s_lo = (m0 + (16 * sg < nvalid ? 16 * sg : 0)) / a.zrows, s_hi = (m0 + (last > 0 ? last : 0)) / a.zrows;
          Bilinear bl{};
          int64_t scn = s_lo;
          for (int64_t sc = s_lo; sc <= s_hi; ++sc) {
            if (row >= sc * a.zrows && row < (sc + 1) * a.zrows) {
              bl = bilinear_at(a.zviews[sc], a.zxyz[3 * row], a.zxyz[3 * row + 1], a.zxyz[3 * row + 2]);
              scn = sc;
            }
          }
          const float* tab = a.ztab + scn * a.ztab_stride;
  #pragma unroll
          for (int f0 = 0; f0 < FT; f0 += ZB) {
  #pragma unroll
            for (int ft = f0; ft < f0 + ZB; ++ft) {
              const int f = feat(ft);
              const floatx4 c0 = ld4(tab + (unsigned)(bl.tex[0] * HID + f)), c1 = ld4(tab + (unsigned)(bl.tex[1] * HID + f));
              const floatx4 c2 = ld4(tab + (unsigned)(bl.tex[2] * HID + f)), c3 = ld4(tab + (unsigned)(bl.tex[3] * HID + f));
              floatx4 z;
  #pragma unroll
              for (int t = 0; t < 4; ++t)
                z[t] = fadd(fadd(fadd(fmul(c0[t], bl.w[0]), fmul(c1[t], bl.w[1])), fmul(c2[t], bl.w[2])),
                            fmul(c3[t], bl.w[3]));
              acc[ft][sg] += z;
            }
            asm volatile("" ::: "memory");   // (the next group's corner loads stay behind this group's use)
          }
        }
      }
    }
    store_rows(a.out);
    // this tile's column means, then M2 about them (two-pass), a tile column group at a time
    const float rn = 1.0f / (float)nvalid;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      floatx4 m = zero4, m2 = zero4;
#pragma unroll
      for (int sg = 0; sg < NSG; ++sg)
        if (live(sg)) m += acc[ft][sg];
      m = sum16(m) * rn;
#pragma unroll
      for (int sg = 0; sg < NSG; ++sg) {
        if (live(sg)) {
          const floatx4 d = acc[ft][sg] - m;
          m2 += d * d;
        }
      }
      put_stats(ft, m, sum16(m2));
    }
  } else {
    // gp = (W^T . op) * relu mask of the forward operand, recomputed from the pre-BN row (bn_relu4, as the
    // forward did); the pre-BN rows also give xhat for the statistics (sums of gp and of gp * xhat). A group of
    // tiles at a time (its pre-BN lines and column parameters), its statistics written as soon as they are done.
    constexpr int FG = FT % 2 == 0 ? 2 : 1;
#pragma unroll
    for (int f0 = 0; f0 < FT; f0 += FG) {
      floatx4 pv[FG][NSG];
      if constexpr (FG == 2) {
        const float* base = a.pre_rows + m0 * HID;
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
          pv[0][sg] = ld4(base + eoff(sg, 0, f0 / 2));
          pv[1][sg] = ld4(base + eoff(sg, 1, f0 / 2));
        }
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) lines_to_pair(pv[0][sg], pv[1][sg], lo, pv[0][sg], pv[1][sg]);
      } else {
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) pv[0][sg] = ld4(a.pre_rows + m0 * HID + orow(sg) + feat(f0));
      }
#pragma unroll
      for (int q = 0; q < FG; ++q) {
        const int ft = f0 + q, f = feat(ft);
        const floatx4 mu = ld4(a.out_mu + f), is = ld4(a.out_invstd + f);
        const floatx4 sc = ld4(a.out_scale + f), sh = ld4(a.out_shift + f);
        floatx4 m = zero4, m2 = zero4;
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
          const floatx4 z = bn_relu4(pv[q][sg], mu, sc, sh);
          const floatx4 v = acc[ft][sg] * inv;
          floatx4 gp;
          gp.x = z.x > 0.f ? v.x : 0.f; gp.y = z.y > 0.f ? v.y : 0.f;
          gp.z = z.z > 0.f ? v.z : 0.f; gp.w = z.w > 0.f ? v.w : 0.f;
          acc[ft][sg] = gp;
          if (live(sg)) {
            m += gp;
            m2 += gp * ((pv[q][sg] - mu) * is);
          }
        }
        put_stats(ft, sum16(m), sum16(m2));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    store_rows(a.out);
  }
}

// acc = W . X of a wave: FT tiles x NSG sample groups; A rolls (tile ft's next-chunk fragment loads into
// its registers as soon as its 3 NSG MFMAs of this chunk have issued, landing while the other tiles compute), B
// refilled in the last tile.
template <int FT, int NSG>
__device__ __forceinline__ void gemm_roll(floatx4 (&acc)[FT][NSG], FragX3 (&A)[FT], const uint4* __restrict__ W,
                                          int KC, int cstride, const uint4* X16, int lane) {
  const int g = lane >> 4, j = lane & 15;
  const uint4* wl = W + lane;
  BPair B[NSG];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int sg = 0; sg < NSG; ++sg) acc[ft][sg] = floatx4{0.f, 0.f, 0.f, 0.f};
  const auto rb = [&](int c, int sg) {
    BPair b;
    b.hi = __builtin_bit_cast(half8, X16[xslot<NSG>(c, 0, g, 16 * sg + j)]);
    b.lo = __builtin_bit_cast(half8, X16[xslot<NSG>(c, 1, g, 16 * sg + j)]);
    return b;
  };
#pragma unroll
  for (int sg = 0; sg < NSG; ++sg) B[sg] = rb(0, sg);
  for (int c = 0; c < KC; ++c) {
    const int cn = c + 1 < KC ? c + 1 : c;   // the last chunk reloads itself (harmless, branch-free)
    const uint4* wn = wl + (int64_t)2 * cn * cstride;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
#pragma unroll
      for (int sg = 0; sg < NSG; ++sg) {
        acc[ft][sg] = mfma32h(A[ft].hi, B[sg].hi, acc[ft][sg]);
        acc[ft][sg] = mfma32h(A[ft].hi, B[sg].lo, acc[ft][sg]);
        acc[ft][sg] = mfma32h(A[ft].lo, B[sg].hi, acc[ft][sg]);
        if (ft == FT - 1) B[sg] = rb(cn, sg);
      }
      A[ft] = load_frag(wn + 2 * 64 * ft);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// d_hidden 64 / 128 / 256: one 64-row tile per 4-wave workgroup, two workgroups per CU (so at most 256 registers a
// lane): one workgroup's row traffic runs under the other's MFMAs.
template <int FT, int MODE, int KK>
__global__ void __launch_bounds__(256, 2) bn_layer_kernel(BnArgs a) {
  constexpr int NW = 4;
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);
  float* red = lds + 64 * KK;                // past X (64 samples x KK x (hi + lo) fp16)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * kX3Samples;
  const int nvalid = a.M - m0 < kX3Samples ? (int)(a.M - m0) : kX3Samples;
  const uint4* W = reinterpret_cast<const uint4*>(a.w) + 2 * 64 * FT * wid;
  FragX3 A0[FT];
  prefetch_a<FT, kPrefetch>(A0, W, lane);
  floatx4 xv[BnItems<NW, KK, 4>::IPW][2];
  float mx = wave_max(bn_operand<NW, KK, 4>(a, m0, nvalid, wid, lane, xv));
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float wgmax = red_max<NW>(red);
  if (a.opnd_max && wid == 0 && lane == 0) publish_max(a.opnd_max, wgmax);
  const float s_x = pow2_scale_for(wgmax);
  bn_split<NW, KK, 4>(a, X16, xv, s_x, m0, nvalid, wid, lane);
  lds_barrier();
  floatx4 acc[FT][4];
  gemm_x3<FT, true, false>(acc, A0, W, KK / 32, 64 * FT * NW, X16, lane);
  const float inv = 1.0f / (pow2_scale_for(__uint_as_float(a.hdr[a.hdr_idx])) * s_x);
  bn_epilogue<FT, NW, MODE, 4, FT / 2>(a, acc, inv, m0, nvalid, wid, lane, blockIdx.x);
}

// d_hidden 512: 32-row tiles (2 sample groups) on 4-wave workgroups (FT 8: 128 features a wave), two workgroups per CU
// (X 64 KB each; acc 64 + rolling A 64 + B 16 registers of the 256 two waves per SIMD leave), so one workgroup's row
// traffic runs under the other's MFMAs. The weight stream per row is twice the 64-row kernel's (L2-resident).
constexpr int kT32Sg = 2, kT32Rows = 16 * kT32Sg;

template <int MODE, int KK>
__global__ void __launch_bounds__(256, 2) bn_layer_t32_kernel(BnArgs a) {
  constexpr int FT = 8, NW = 4, NSG = kT32Sg, TR = kT32Rows;
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);
  float* red = lds + TR * KK;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * TR;
  const int nvalid = a.M - m0 < TR ? (int)(a.M - m0) : TR;
  const uint4* W = reinterpret_cast<const uint4*>(a.w) + 2 * 64 * FT * wid;
  floatx4 xv[BnItems<NW, KK, NSG>::IPW][2];
  float mx = wave_max(bn_operand<NW, KK, NSG>(a, m0, nvalid, wid, lane, xv));
  // chunk 0's weights after the operand loads (in flight beside them, they would not fit the registers)
  FragX3 A[FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) A[ft] = load_frag(W + (unsigned)(lane + 2 * 64 * ft));
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float wgmax = red_max<NW>(red);
  if (a.opnd_max && wid == 0 && lane == 0) publish_max(a.opnd_max, wgmax);
  const float s_x = pow2_scale_for(wgmax);
  bn_split<NW, KK, NSG>(a, X16, xv, s_x, m0, nvalid, wid, lane);
  lds_barrier();
  floatx4 acc[FT][NSG];
  gemm_roll<FT, NSG>(acc, A, W, KK / 32, 64 * FT * NW, X16, lane);
  const float inv = 1.0f / (pow2_scale_for(__uint_as_float(a.hdr[a.hdr_idx])) * s_x);
  bn_epilogue<FT, NW, MODE, NSG, 1>(a, acc, inv, m0, nvalid, wid, lane, blockIdx.x);
}

// rows of a statistics partial (one per tile of avr_bn_layer_run's kernel for that width)
static int bn_tile_rows(int n_cols) { return n_cols == 512 ? kT32Rows : kX3Samples; }

template <int FT, int MODE, int KK>
static int launch_bn_layer(const BnArgs& a, hipStream_t s) {
  constexpr int HID = 16 * FT * 4;
  const int64_t tr = bn_tile_rows(FT == 8 ? 512 : HID);
  const int64_t tiles = (a.M + tr - 1) / tr;
  AVR_REQUIRE(tiles < (1ll << 31), "avr_bn_layer_run: too many rows");
  if constexpr (FT == 8) {
    const size_t shm = (size_t)kT32Rows * KK * 4 + 64;   // X (32 samples x KK x hi + lo fp16) + the wave maxima
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bn_layer_t32_kernel<MODE, KK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
        return fail(AVR_E_HIP, "bn_layer_t32_kernel: cannot set dynamic LDS");
      attr = true;
    }
    bn_layer_t32_kernel<MODE, KK><<<(unsigned)tiles, 256, shm, s>>>(a);
    return check_launch("bn_layer_t32_kernel");
  } else {
    const size_t shm = (size_t)64 * KK * 4 + 64;   // X (64 samples x KK x hi + lo fp16) + the wave maxima
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bn_layer_kernel<FT, MODE, KK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
        return fail(AVR_E_HIP, "bn_layer_kernel: cannot set dynamic LDS");
      attr = true;
    }
    bn_layer_kernel<FT, MODE, KK><<<(unsigned)tiles, 256, shm, s>>>(a);
    return check_launch("bn_layer_kernel");
  }
}

// K is lin_in's 64 (forward) or d_hidden
template <int FT, int MODE>
static int launch_bn_layer_k(const BnArgs& a, hipStream_t s) {
  constexpr int HID = 16 * FT * 4;
  if (a.K == HID) return launch_bn_layer<FT, MODE, HID>(a, s);
  if constexpr (MODE == AVR_BN_FWD && HID != 64) {
    if (a.K == 64) return launch_bn_layer<FT, MODE, 64>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "avr_bn_layer_run: in_dim %d with d_hidden %d", a.K, HID);
}

template <int MODE>
static int dispatch_bn_layer(int H, const BnArgs& a, hipStream_t s) {
  switch (H) {
    case 64: return launch_bn_layer_k<1, MODE>(a, s);
    case 128: return launch_bn_layer_k<2, MODE>(a, s);
    case 256: return launch_bn_layer_k<4, MODE>(a, s);
    case 512: return launch_bn_layer_k<8, MODE>(a, s);
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
__global__ void __launch_bounds__(64) bn_fold_kernel(const float* __restrict__ part, int64_t M, int N, int tr,
                                                     double* __restrict__ fold) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  const int64_t nwg = (M + tr - 1) / tr;
  double a = 0.0, b = 0.0;
  if (c < N) {
#pragma unroll 8
    for (int64_t w = (int64_t)blockIdx.y * kBnFold; w < nwg && w < (int64_t)(blockIdx.y + 1) * kBnFold; ++w) {
      const float p0 = part[w * 2 * N + c], p1 = part[w * 2 * N + N + c];
      if constexpr (FWD) {
        const double n = (double)(M - w * tr < tr ? M - w * tr : tr);
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
  AVR_REQUIRE(ly == 0 || (ly >= 2 && ly < 2 + 2 * nb), "avr_bn_layer_run: layer %d", ly);
  const unsigned* hdr;
  if (l->mode == AVR_BN_FWD) {
    AVR_REQUIRE(ly != 0 || l->in_dim == 64, "avr_bn_layer_run: lin_in's operand is 64 columns");
    AVR_REQUIRE(ly == 0 || l->in_dim == H, "avr_bn_layer_run: a hidden layer's operand is d_hidden columns");
    a.w = l->blob + (ly == 0 ? L.x3_in : (ly % 2 == 0 ? L.x3_fc0[(ly - 2) / 2] : L.x3_fc1[(ly - 2) / 2]));
    hdr = reinterpret_cast<const unsigned*>(l->blob + L.x3_hdr);
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
    AVR_REQUIRE(ly >= 2 && l->in_dim == H, "avr_bn_layer_run: the backward runs fc_0 / fc_1 (d_hidden columns)");
    AVR_REQUIRE(l->pre_rows && l->out_mu && l->out_invstd && l->out_scale && l->out_shift,
                "avr_bn_layer_run: AVR_BN_BWD needs pre_rows, out_mu, out_invstd, out_scale, out_shift");
    BwdLayout LB;
    if ((rc = field_bwd_layout(dims, &LB))) return rc;
    a.w = l->blob + (ly % 2 == 0 ? LB.fc0t[(ly - 2) / 2] : LB.fc1t[(ly - 2) / 2]);
    hdr = reinterpret_cast<const unsigned*>(l->blob);
    a.pre_rows = l->pre_rows; a.out_mu = l->out_mu; a.out_invstd = l->out_invstd;
    a.out_scale = l->out_scale; a.out_shift = l->out_shift;
  }
  a.hdr = hdr;
  a.hdr_idx = ly;
  a.out = l->out;
  a.part = l->partial;
  hipStream_t s = as_stream(stream);   // the weight scale is read on the device (the pack launch wrote it)
  return l->mode == AVR_BN_FWD ? dispatch_bn_layer<AVR_BN_FWD>(H, a, s) : dispatch_bn_layer<AVR_BN_BWD>(H, a, s);
}

// The fold scratch (fp64, 2 x n_cols per 16 partials) lives in the partial buffer past the partials
// (avr_bn_partial_floats sizes it), so the entry points allocate nothing. One partial per tile of the layer
// kernel of that width (bn_tile_rows: 48 rows at 512 columns, 64 otherwise).
static int64_t bn_n_tiles(int64_t n_rows, int n_cols) { return (n_rows + bn_tile_rows(n_cols) - 1) / bn_tile_rows(n_cols); }
static int64_t bn_n_fold(int64_t n_rows, int n_cols) { return (bn_n_tiles(n_rows, n_cols) + kBnFold - 1) / kBnFold; }

extern "C" int avr_bn_partial_floats(int64_t n_rows, int n_cols, int64_t* n_floats) {
  AVR_REQUIRE(n_rows >= 0 && n_cols > 0 && n_floats, "avr_bn_partial_floats: bad argument");
  const int64_t nwg = bn_n_tiles(n_rows, n_cols);
  // partials (nwg, 2, n_cols) fp32, then 8-B aligned fold rows (n_fold, 2, n_cols) fp64
  *n_floats = (nwg * 2 * n_cols + 1) / 2 * 2 + bn_n_fold(n_rows, n_cols) * 2 * n_cols * 2;
  return AVR_OK;
}

static const float* bn_fold(const float* partial, int64_t n_rows, int n_cols, bool fwd, double** fold,
                            hipStream_t s) {
  const int64_t nwg = bn_n_tiles(n_rows, n_cols);
  *fold = reinterpret_cast<double*>(const_cast<float*>(partial) + (nwg * 2 * n_cols + 1) / 2 * 2);
  const dim3 grid((unsigned)((n_cols + 63) / 64), (unsigned)bn_n_fold(n_rows, n_cols));
  const int tr = bn_tile_rows(n_cols);
  if (fwd)
    bn_fold_kernel<true><<<grid, 64, 0, s>>>(partial, n_rows, n_cols, tr, *fold);
  else
    bn_fold_kernel<false><<<grid, 64, 0, s>>>(partial, n_rows, n_cols, tr, *fold);
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
  bn_stats_kernel<<<(unsigned)((n_cols + 63) / 64), 64 * kBnFoldWaves, 0, s>>>(fold, (int)bn_n_fold(n_rows, n_cols), n_rows,
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
  bn_grad_stats_kernel<<<(unsigned)((n_cols + 63) / 64), 64 * kBnFoldWaves, 0, s>>>(fold, (int)bn_n_fold(n_rows, n_cols),
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
