// Training-mode BatchNorm of ResnetFC(bn=True) on the HIP path: train.py --bn (train.py:210, :265) builds
// ResnetBlockFC(bn=True), whose forward is relu(bn_0(x)) -> fc_0 -> relu(bn_0(net)) -> fc_1, + x
// (models.py:454-461; bn_0 applied twice, bn_1 unused), with batch statistics over every row of the field
// call in training mode.
//
// The fused field kernels carry a 64-sample tile through every layer in one workgroup; batch statistics are a
// reduction over all rows between two GEMMs, so this net runs layer by layer. One launch per GEMM over
// row-major fp32 rows (bn_layer_kernel): the operand -- the layer input normalised and relu'd (forward), or
// the BatchNorm backward of the gradient (backward) -- is built in the prologue from the rows, split into
// fp16 hi/lo under one power-of-two scale per workgroup and staged in LDS in the fused kernels' B-fragment
// order; the K loop is theirs (x3: three v_mfma_f32_16x16x32_f16 per product, fp32 accumulate, weights
// streamed one chunk ahead); the epilogue adds bias / residual / lin_z rows (forward) or applies the relu mask
// (backward, recomputed from the pre-BN rows: the relu'd operands are never stored), stores the rows and
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

// 16 lanes of one lane group g (lanes 16g .. 16g + 15): sum over j
__device__ __forceinline__ floatx4 sum16(floatx4 v) {
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) {
    v.x += __shfl_xor(v.x, d, 64);
    v.y += __shfl_xor(v.y, d, 64);
    v.z += __shfl_xor(v.z, d, 64);
    v.w += __shfl_xor(v.w, d, 64);
  }
  return v;
}

template <int FT, int NW, bool TWO>
__device__ __forceinline__ void bn_gemm(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* __restrict__ W, int KC,
                                        int cstride, const uint4* X16, int lane) {
  if constexpr (TWO)
    gemm_x3_sg<FT, true, FT>(acc, A0, W, KC, cstride, X16, lane);
  else
    gemm_x3<FT, true, false>(acc, A0, W, KC, cstride, X16, lane);
}

// MODE 0 forward, 1 backward. Workgroup = 64 rows; lane = row in the prologue (wave w builds the operand
// columns [K/NW * w, K/NW * (w + 1)) of all 64 rows: one 16-B load per row and column group, written into
// the slots of its sample -- conflict-free LDS stores), then the fused kernels' GEMM and register layout:
// lane (g, j) of wave w holds features 16 (FT w + ft) + 4 g .. +3 of rows 16 sg + j.
template <int FT, int NW, int MODE>
__global__ void __launch_bounds__(64 * NW, 1) bn_layer_kernel(BnArgs a) {
  constexpr int HID = 16 * FT * NW, NTT = FT * NW;
  constexpr bool TWO = NW > 4;
  constexpr int MAXQ = 512 / 4 / NW;        // operand column groups per wave (K <= 512)
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);
  // the stages (prologue K + 4, epilogue HID + 4 floats a row; X aliases them), the column sums, then red
  const int stage_f = kX3Samples * ((a.K > HID ? a.K : HID) + 4);
  float* red = lds + stage_f + NW * HID;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int64_t m0 = (int64_t)blockIdx.x * kX3Samples;
  const int nvalid = a.M - m0 < kX3Samples ? (int)(a.M - m0) : kX3Samples;
  const uint4* W = reinterpret_cast<const uint4*>(a.w) + 2 * 64 * FT * wid;
  FragX3 A0[FT];
  prefetch_a<FT, TWO ? FT : kPrefetch>(A0, W, lane);

  // ---------------------------------------------------------------- operand
  // Phase A, coalesced: wave w takes rows w, w + NW, ...; lane l column groups l, l + 64, ... of the row (one
  // 1-KB row segment per load), applies the prologue's transform with its columns' parameters and writes the
  // fp32 values into an LDS stage, row stride 4 K + 16 B. Phase B: lane = row reads its operand columns back
  // (the +16 B row pad spreads the 64 rows over the banks) and splits them into X, which aliases the stage
  // (the values wait in registers across the barrier).
  const int G4 = a.K / 4;                    // column groups of a row
  const int rs = a.K + 4;                    // stage row stride (floats)
  float mx = 0.f;
  // pair i of this lane: row wid + NW (i >> 1), column group lane + 64 (i & 1) (K <= 512: <= 2 per row). In
  // batches of PB pairs, every load of a batch issued before the batch's first store: a load cannot move above a
  // store that may alias it, and the in-order memory counter makes a wait on a load also wait on every store
  // issued before it -- one round trip per pair otherwise. The lane's two column groups' parameters are loaded
  // once (RELU: mu, scale, shift; GRAD: mu, invstd, m1, m2, scale).
  floatx4 pp[5][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = 4 * (lane + 64 * h) < a.kin ? 4 * (lane + 64 * h) : 0;
    if (a.prologue == AVR_BN_RELU) {
      pp[0][h] = ld4(a.in_mu + k); pp[1][h] = ld4(a.in_scale + k); pp[2][h] = ld4(a.in_shift + k);
    } else if (a.prologue == AVR_BN_GRAD) {
      pp[0][h] = ld4(a.in_mu + k); pp[1][h] = ld4(a.in_invstd + k); pp[2][h] = ld4(a.in_m1 + k);
      pp[3][h] = ld4(a.in_m2 + k); pp[4][h] = ld4(a.in_scale + k);
    }
  }
  // (the backward's GRAD prologue holds three rows per pair: smaller batches keep it within the registers)
  constexpr int PB = MAXQ < 8 ? MAXQ : (MODE == AVR_BN_FWD ? 8 : 4);
#pragma unroll
  for (int b0 = 0; b0 < MAXQ; b0 += PB) {
    floatx4 sv[PB], pv[PB], rv[PB];
    // pair jb's source offset (rows past the end read row m0, columns past the row column 0: every load is
    // unconditional, so none waits behind a branch); its values are dropped below where they do not belong
    const auto src_off = [&](int jb) -> int64_t {
      const int i = b0 + jb, r = wid + NW * (i >> 1), q = lane + 64 * (i & 1);
      const bool ok = r < kX3Samples && q < G4 && 4 * q + 4 <= a.kin;
      return (m0 + (r < nvalid && ok ? r : 0)) * a.ld_src + (ok ? 4 * q : 0);
    };
    if (a.kin == a.K) {   // whole 16-B groups (every hidden layer): the batch's loads back to back
#pragma unroll
      for (int jb = 0; jb < PB; ++jb) sv[jb] = ld4(a.src + src_off(jb));
      if (a.prologue == AVR_BN_GRAD) {
#pragma unroll
        for (int jb = 0; jb < PB; ++jb) pv[jb] = ld4(a.src_pre + src_off(jb));
        if (a.src_res) {
#pragma unroll
          for (int jb = 0; jb < PB; ++jb) rv[jb] = ld4(a.src_res + src_off(jb));
        }
      }
    } else {              // lin_in's z_feature rows (in_valid < in_dim, PLAIN)
#pragma unroll
      for (int jb = 0; jb < PB; ++jb) {
        const int i = b0 + jb, r = wid + NW * (i >> 1), q = lane + 64 * (i & 1);
        sv[jb] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (r < kX3Samples && q < G4) {
          const int64_t row = m0 + (r < nvalid ? r : 0);
          const int k = 4 * q;
          if (k + 4 <= a.kin) {
            sv[jb] = ld4(a.src + row * a.ld_src + k);
          } else if (k < a.kin) {
#pragma unroll
            for (int t = 0; t < 4; ++t) sv[jb][t] = k + t < a.kin ? a.src[row * a.ld_src + k + t] : 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int jb = 0; jb < PB; ++jb) {
      const int i = b0 + jb, r = wid + NW * (i >> 1), q = lane + 64 * (i & 1), h = i & 1;
      if (r < kX3Samples && q < G4) {
        const bool live = r < nvalid;
        const int64_t row = m0 + (live ? r : 0);
        const int k = 4 * q;
        floatx4 v = sv[jb];
        if (k < a.kin) {
          if (a.prologue == AVR_BN_RELU) {
            v = bn_relu4(v, pp[0][h], pp[1][h], pp[2][h]);
          } else if (a.prologue == AVR_BN_GRAD) {
            const floatx4 xh = (pv[jb] - pp[0][h]) * pp[1][h];
            v = (v - pp[2][h] - xh * pp[3][h]) * pp[4][h];
            if (a.src_res) v += rv[jb];
          }
        }
        if (!live) v = floatx4{0.f, 0.f, 0.f, 0.f};
        else if (a.opnd_out) __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(a.opnd_out + row * a.K + k));
        *reinterpret_cast<floatx4*>(lds + r * rs + k) = v;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  lds_barrier();
  const float wgmax = red_max<NW>(red);
  if (a.opnd_max && wid == 0 && lane == 0) publish_max(a.opnd_max, wgmax);
  const float s_x = pow2_scale_for(wgmax);
  const int qpw = a.K / 4 / NW;              // phase B: column groups of this wave
  floatx4 xv[MAXQ];
#pragma unroll
  for (int i = 0; i < MAXQ; ++i)
    if (i < qpw) xv[i] = *reinterpret_cast<const floatx4*>(lds + lane * rs + 4 * (qpw * wid + i));
  lds_barrier();
  char* xb = reinterpret_cast<char*>(X16);
#pragma unroll
  for (int i = 0; i < MAXQ; ++i) {
    if (i < qpw) {
      const int k = 4 * (qpw * wid + i);
      uint2 hi, lo;
      split4(xv[i], s_x, hi, lo);
      const int c = k >> 5, gq = (k >> 2) & 3, half = (k >> 4) & 1;
      *reinterpret_cast<uint2*>(xb + xidx(c, 0, gq, lane) * 16 + 8 * half) = hi;
      *reinterpret_cast<uint2*>(xb + xidx(c, 1, gq, lane) * 16 + 8 * half) = lo;
    }
  }
  lds_barrier();

  // ---------------------------------------------------------------- GEMM
  floatx4 acc[FT][4];
  bn_gemm<FT, NW, TWO>(acc, A0, W, a.KC, 64 * NTT, X16, lane);
  const float inv = 1.0f / (pow2_scale_for(__uint_as_float(a.hdr[a.hdr_idx])) * s_x);

  // ---------------------------------------------------------------- epilogue
  // The accumulators (feature-major in the registers) go to an fp32 stage in LDS (row-major, aliasing X), and
  // the rows are finished like the prologue's: wave = rows, lane = column groups, so the addend / mask / pre-BN
  // row loads and the row stores are coalesced 1-KB segments. The workgroup's column statistics are per-lane
  // sums over the wave's rows, met across the waves in LDS.
  constexpr int EQ = HID / 4;                // column groups of an output row
  constexpr int es = HID + 4;                // stage row stride (floats)
  float* colred = lds + stage_f;             // (NW, HID) per-wave column sums, past the stages
  __syncthreads();                           // every wave has left the GEMM (the stage overwrites X)
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const int f0 = 16 * (FT * wid + ft) + 4 * g;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) *reinterpret_cast<floatx4*>(lds + (16 * sg + j) * es + f0) = acc[ft][sg] * inv;
  }
  __syncthreads();
  floatx4 yv[MAXQ];
  floatx4 s1[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}}, s2[2] = {s1[0], s1[0]};
  floatx4 cp0[2], cp1[2], cp2[2], cp3[2];    // per-column parameters of the lane's two groups
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = 4 * (lane + 64 * h) < HID ? 4 * (lane + 64 * h) : 0;
    if constexpr (MODE == AVR_BN_FWD) {
      cp0[h] = a.bias ? ld4(a.bias + f) : floatx4{0.f, 0.f, 0.f, 0.f};
      cp1[h] = cp2[h] = cp3[h] = cp0[h];
    } else {
      cp0[h] = ld4(a.out_mu + f);
      cp1[h] = ld4(a.out_invstd + f);
      cp2[h] = ld4(a.out_scale + f);
      cp3[h] = ld4(a.out_shift + f);
    }
  }
  // pair i as in the prologue; every load of the epilogue is issued before its first store (see there)
  const auto valid = [&](int i) { return wid + NW * (i >> 1) < kX3Samples && lane + 64 * (i & 1) < EQ; };
  const auto live = [&](int i) { return wid + NW * (i >> 1) < nvalid; };
  const auto row_of = [&](int i) -> int64_t { return m0 + (live(i) ? wid + NW * (i >> 1) : 0); };
  const auto col_of = [&](int i) { return 4 * (lane + 64 * (i & 1)); };
  // an always-valid offset for pair i's row loads (past the row: column 0), so the loads need no branch
  const auto off_of = [&](int i) -> int64_t { return row_of(i) * HID + (valid(i) ? col_of(i) : 0); };
  const auto staged = [&](int i) {
    return valid(i) ? *reinterpret_cast<const floatx4*>(lds + (wid + NW * (i >> 1)) * es + col_of(i))
                    : floatx4{0.f, 0.f, 0.f, 0.f};
  };
  if constexpr (MODE == AVR_BN_FWD) {
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) yv[i] = staged(i);
    // out = W . op + bias (+ add1) (+ add2) (+ lin_z rows), added in that order
#pragma unroll
    for (int i = 0; i < MAXQ; ++i)
      if (valid(i)) yv[i] += cp0[i & 1];
    const floatx4 zero4 = floatx4{0.f, 0.f, 0.f, 0.f};
    if (a.add1) {
      floatx4 t[MAXQ];
#pragma unroll
      for (int i = 0; i < MAXQ; ++i) t[i] = ld4(a.add1 + off_of(i));
#pragma unroll
      for (int i = 0; i < MAXQ; ++i) yv[i] += valid(i) ? t[i] : zero4;
    }
    if (a.add2) {
      floatx4 t[MAXQ];
#pragma unroll
      for (int i = 0; i < MAXQ; ++i) t[i] = ld4(a.add2 + off_of(i));
#pragma unroll
      for (int i = 0; i < MAXQ; ++i) yv[i] += valid(i) ? t[i] : zero4;
    }
    if (a.ztab) {   // the rows' lin_z features: avr_latent_features' lookup and blend order, bit for bit
      // the points of the wave's rows first (one load each, all in flight together), then per row its corners
      float px[MAXQ / 2][3];
#pragma unroll
      for (int i = 0; i < MAXQ; i += 2)
#pragma unroll
        for (int d = 0; d < 3; ++d) px[i >> 1][d] = a.zxyz[3 * row_of(i) + d];
      const int64_t sc0 = m0 / a.zrows;      // the workgroup's first scene (rows are scene-major)
#pragma unroll
      for (int i = 0; i < MAXQ; i += 2) {
        if (wid + NW * (i >> 1) < kX3Samples) {
          int64_t sc = sc0;
          while (row_of(i) >= (sc + 1) * a.zrows) ++sc;
          const Bilinear bl = bilinear_at(a.zviews[sc], px[i >> 1][0], px[i >> 1][1], px[i >> 1][2]);
          const float* tab = a.ztab + sc * a.ztab_stride;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int f = valid(i + h) ? col_of(i + h) : 0;
            const floatx4 c0 = ld4(tab + (int64_t)bl.tex[0] * HID + f), c1 = ld4(tab + (int64_t)bl.tex[1] * HID + f);
            const floatx4 c2 = ld4(tab + (int64_t)bl.tex[2] * HID + f), c3 = ld4(tab + (int64_t)bl.tex[3] * HID + f);
            floatx4 z;
#pragma unroll
            for (int t = 0; t < 4; ++t)
              z[t] = fadd(fadd(fadd(fmul(c0[t], bl.w[0]), fmul(c1[t], bl.w[1])), fmul(c2[t], bl.w[2])),
                          fmul(c3[t], bl.w[3]));
            if (valid(i + h)) yv[i + h] += z;
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) {
      if (valid(i) && live(i)) {
        *reinterpret_cast<floatx4*>(a.out + row_of(i) * HID + col_of(i)) = yv[i];
        s1[i & 1] += yv[i];
      }
    }
  } else {
    // gp = (W^T . op) * relu mask of the forward operand, recomputed from the pre-BN row (bn_relu4, as the
    // forward did); the pre-BN rows also give xhat for the statistics
    floatx4 pv[MAXQ];
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) pv[i] = ld4(a.pre_rows + off_of(i));
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) {
      if (valid(i) && live(i)) {
        const floatx4 z = bn_relu4(pv[i], cp0[i & 1], cp2[i & 1], cp3[i & 1]);
        const floatx4 v = staged(i);
        floatx4 gp;
        gp.x = z.x > 0.f ? v.x : 0.f; gp.y = z.y > 0.f ? v.y : 0.f;
        gp.z = z.z > 0.f ? v.z : 0.f; gp.w = z.w > 0.f ? v.w : 0.f;
        *reinterpret_cast<floatx4*>(a.out + row_of(i) * HID + col_of(i)) = gp;
        const floatx4 xh = (pv[i] - cp0[i & 1]) * cp1[i & 1];
        s1[i & 1] += gp;
        s2[i & 1] += gp * xh;
      }
    }
  }
  float* part = a.part + (int64_t)blockIdx.x * 2 * HID;
  // the waves' column sums meet in one LDS slot (NW x HID), used twice: sums of y (-> the means, needed by
  // every lane for the squared deviations) or of gp, then M2 or the sums of gp * xhat
  const auto put = [&](const floatx4 (&v)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (lane + 64 * h < EQ) *reinterpret_cast<floatx4*>(colred + wid * HID + 4 * (lane + 64 * h)) = v[h];
  };
  const auto total = [&](int h) {
    floatx4 t = floatx4{0.f, 0.f, 0.f, 0.f};
    if (lane + 64 * h < EQ)
      for (int w = 0; w < NW; ++w) t += *reinterpret_cast<const floatx4*>(colred + w * HID + 4 * (lane + 64 * h));
    return t;
  };
  put(s1);
  __syncthreads();
  floatx4 t1[2] = {total(0), total(1)};
  __syncthreads();
  if constexpr (MODE == AVR_BN_FWD) {
    const float rn = 1.0f / (float)nvalid;
    t1[0] *= rn;                             // this workgroup's column means
    t1[1] *= rn;
#pragma unroll
    for (int i = 0; i < MAXQ; ++i) {
      const int r = wid + NW * (i >> 1);
      if (r < nvalid) {
        const floatx4 d = yv[i] - t1[i & 1];
        s2[i & 1] += d * d;
      }
    }
  }
  put(s2);
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const floatx4 t2 = total(h);
      const int f = 4 * (lane + 64 * h);
      if (f < HID) {
        *reinterpret_cast<floatx4*>(part + f) = t1[h];
        *reinterpret_cast<floatx4*>(part + HID + f) = t2;
      }
    }
  }
}

template <int FT, int NW, int MODE>
static int launch_bn_layer(const BnArgs& a, hipStream_t s) {
  // the larger of the prologue's and the epilogue's fp32 stage (X aliases them) + the column sums + red
  constexpr int HID = 16 * FT * NW;
  const size_t stage = (size_t)kX3Samples * ((a.K > HID ? a.K : HID) + 4) * 4;
  const size_t shm = stage + (size_t)NW * HID * 4 + 64;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bn_layer_kernel<FT, NW, MODE>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            kX3Samples * (512 + 4) * 4 + NW * HID * 4 + 64) != hipSuccess)
      return fail(AVR_E_HIP, "bn_layer_kernel: cannot set dynamic LDS");
    attr = true;
  }
  const int64_t blocks = (a.M + kX3Samples - 1) / kX3Samples;
  AVR_REQUIRE(blocks < (1ll << 31), "avr_bn_layer_run: too many rows");
  bn_layer_kernel<FT, NW, MODE><<<(unsigned)blocks, 64 * NW, shm, s>>>(a);
  return check_launch("bn_layer_kernel");
}

template <int MODE>
static int dispatch_bn_layer(int H, const BnArgs& a, hipStream_t s) {
  switch (H) {
    case 64: return launch_bn_layer<1, 4, MODE>(a, s);
    case 128: return launch_bn_layer<2, 4, MODE>(a, s);
    case 256: return launch_bn_layer<4, 4, MODE>(a, s);
    case 512: return launch_bn_layer<4, 8, MODE>(a, s);
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
  AVR_REQUIRE(l->in_valid > 0 && l->in_valid <= l->in_dim, "avr_bn_layer_run: in_valid %d", l->in_valid);
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
