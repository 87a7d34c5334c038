// Backward of the radiance field's ResnetFC: the input-gradient chain of
// autograd through models.py:856-862 (sigmoid rgb, relu sigma), lin_out
// (:592), every ResnetBlockFC (:454-470, dx = fc_1(relu(fc_0(relu(x)))),
// out = x + dx) and the lin_z residual adds (:578-581), in reverse:
//   dx  = W_out^T d_out  (x) [a_out > 0]                      (G[2 nb] is written last)
//   per block b = nb-1 .. 0:
//     G1_b = dx                                               -> G[2b + 1]
//     G0_b = (W1_b^T G1_b) (x) [r_b > 0]                      -> G[2b]
//     dx   = dx + (W0_b^T G0_b) (x) [a_b > 0]                 (gradient at block b's input)
//   G_in = dx                                                 -> G[2 nb]
// G[l] pairs with the forward's saved GEMM input act[l] (a_b = act[2b],
// r_b = act[2b+1], a_out = act[2 nb]): dW = G[l]^T act[l] and db = sum G[l]
// are plain GEMMs / reductions over the samples, done by the caller.
//
// The two 512x512 products per block run on the forward's split-fp16 MFMA
// machinery (x3_gemm.h) with W^T packed in the same fragment order
// (avr_field_pack_bwd). Per 64-sample workgroup the chain needs only the relu
// masks of the forward (1 bit per value, 16 B per lane and layer), so nothing
// but the gradients themselves goes through HBM.
#include "x3_gemm.h"

namespace avr {

template <int FT>
__device__ __forceinline__ floatx4 masked(const floatx4& v, const unsigned* mb, int ft, int sg) {
  const int idx = (ft * 4 + sg) * 4;
  const unsigned bits = mb[idx >> 5] >> (idx & 31);
  floatx4 r;
  r.x = (bits & 1u) ? v.x : 0.f;
  r.y = (bits & 2u) ? v.y : 0.f;
  r.z = (bits & 4u) ? v.z : 0.f;
  r.w = (bits & 8u) ? v.w : 0.f;
  return r;
}

// (8 waves, d_hidden 512: the masks are in the 4-wave layout -- wave w's tile 4 w + ft is tile 4 (w & 1) + ft of
// 4-wave wave w >> 1, its words 2 (w & 1) + q there)
template <int FT, int NW>
__device__ __forceinline__ void load_mask(unsigned (&mb)[mask_words(FT)], const unsigned* mask, int layer, int lane,
                                          int wid) {
  constexpr int MW = mask_words(FT);
  const unsigned* mk = NW == 8 ? mask + ((((int64_t)layer * gridDim.x + blockIdx.x) * 4 + (wid >> 1)) * 4 +
                                         2 * (wid & 1)) * 64 + lane
                               : mask + (((int64_t)layer * gridDim.x + blockIdx.x) * NW + wid) * MW * 64 + lane;
#pragma unroll
  for (int q = 0; q < MW; ++q) mb[q] = mk[q * 64];
}

// d act(x) / dx applied to v: ReLU from the forward's mask bits; Softplus(beta) from the saved activation
// y = softplus(x) of row m, features f0 .. f0+3 of layer `layer`: torch's softplus_backward is
// g * sigmoid(beta x) = g * (1 - exp(-beta y)) (-expm1: no cancellation where the slope is tiny; where torch
// takes the linear branch, beta x > 20, this is 1 to fp32 precision)
template <int FT, int ACT>
__device__ __forceinline__ floatx4 dact(const floatx4& v, const unsigned* mb, const BwdArgs& a, int layer,
                                        int64_t row, int f0, int ft, int sg) {
  if constexpr (ACT == 0) {
    return masked<FT>(v, mb, ft, sg);
  } else {
    const floatx4 y = *reinterpret_cast<const floatx4*>(a.act + (int64_t)layer * a.act_stride + row + f0);
    floatx4 r;
    r.x = v.x * -expm1f(-a.beta * y.x);
    r.y = v.y * -expm1f(-a.beta * y.y);
    r.z = v.z * -expm1f(-a.beta * y.z);
    r.w = v.w * -expm1f(-a.beta * y.w);
    return r;
  }
}

template <int FT, int NW>
__device__ __forceinline__ void store_rows(float* G, const floatx4 (&v)[FT][4], int64_t base, int64_t M, int wid,
                                           int g, int j) {
  constexpr int HID = 16 * FT * NW;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const int64_t m = base + 16 * sg + j;
      if (m < M) __builtin_nontemporal_store(v[ft][sg], reinterpret_cast<floatx4*>(G + m * HID + 16 * (FT * wid + ft) + 4 * g));
    }
}

// G rows of `layer` copied out of the LDS operand by a GEMM side task (x3_gemm.h RowSideH): lane (g, j)
// of wave w copies sample 16 w + j
template <int HID>
__device__ __forceinline__ RowSideH<HID> grad_side(const BwdArgs& a, int layer, float s_x, int64_t base, int64_t roff,
                                                   int wid) {
  RowSideH<HID> rs;
  rs.template init<HID>(a.G + (int64_t)layer * a.g_stride + (roff + base) * HID, s_x, a.M - base, wid);
  return rs;
}

template <int HID>
__device__ __forceinline__ RowSide8<HID> grad_side8(const BwdArgs& a, int layer, float s_x, int64_t base, int64_t roff,
                                                    int wid) {
  RowSide8<HID> rs;
  rs.init8(a.G + (int64_t)layer * a.g_stride + (roff + base) * HID, s_x, a.M - base, wid);
  return rs;
}

// the K loop of one backward GEMM: 4 waves (gemm_x3 with the row side task) or 8 (gemm_x3_sg_side)
template <int FT, int NW, int HID>
__device__ __forceinline__ void bwd_gemm(floatx4 (&acc)[FT][4], FragX3 (&A0)[FT], const uint4* W, const uint4* X16,
                                         int lane, const BwdArgs& a, int layer, float s_x, int64_t base, int64_t roff,
                                         int wid) {
  constexpr int KC = HID / 32, NTT = FT * NW;
  if constexpr (NW == 8)
    gemm_x3_sg_side<FT, true>(acc, A0, W, KC, 64 * NTT, X16, lane, grad_side8<HID>(a, layer, s_x, base, roff, wid));
  else
    gemm_x3<FT, true, false>(acc, A0, W, KC, 64 * NTT, X16, lane, grad_side<HID>(a, layer, s_x, base, roff, wid));
}

template <int FT>
__device__ __forceinline__ float absmax(const floatx4 (&v)[FT][4]) {
  float mx = 0.f;
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 x = v[ft][sg];
      mx = fmaxf(fmaxf(mx, fabsf(x.x)), fmaxf(fabsf(x.y), fmaxf(fabsf(x.z), fabsf(x.w))));
    }
  return wave_max(mx);
}

__device__ __forceinline__ float bwd_scale(const float* packed_bwd, int layer) {
  return pow2_scale_for(__uint_as_float(reinterpret_cast<const unsigned*>(packed_bwd)[layer]));
}

template <int FT, int NW, int ACT>
__global__ void __launch_bounds__(64 * NW, 1) field_bwd_x3_kernel(BwdArgs a) {
  constexpr int HID = 16 * FT * NW;
  constexpr int KC = HID / 32;
  constexpr int MW = mask_words(FT);
  extern __shared__ float lds[];
  uint4* X16 = reinterpret_cast<uint4*>(lds);   // KC chunks x 8 KiB, the forward's operand layout
  float* red = lds + KC * 2048;
  float* lmax = red + 16;                       // per-layer workgroup max |G| (kX3MaxLayers)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, j = lane & 15;
  const int scene = (int)(blockIdx.x / a.blocks_per_scene);   // the forward's workgroup -> scene map
  const int64_t base = (int64_t)(blockIdx.x - (int64_t)scene * a.blocks_per_scene) * kX3Samples;
  const int64_t roff = (int64_t)scene * a.M;
  const int nb = a.n_blocks;
  const uint4* PB = reinterpret_cast<const uint4*>(a.packed_bwd);
  // Softplus: offset of the saved activation row of sample group sg (rows past M read the last row: unused)
  const auto arow = [&](int sg) -> int64_t {
    const int64_t m = base + 16 * sg + j;
    return (roff + (m < a.M ? m : a.M - 1)) * HID;
  };

  floatx4 dx[FT][4], t[FT][4];
  unsigned mb[MW];
  // ---- d out: sigmoid' from the saved output (torch: g * (1 - y) * y), relu' (y > 0)
  float d4[4][4];
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    const int64_t m = base + 16 * sg + j;
    const bool ok = m < a.M;
    const float4 o = a.out[roff + (ok ? m : a.M - 1)], go = a.grad_out[roff + (ok ? m : a.M - 1)];
    d4[sg][0] = ok ? go.x * ((1.f - o.x) * o.x) : 0.f;
    d4[sg][1] = ok ? go.y * ((1.f - o.y) * o.y) : 0.f;
    d4[sg][2] = ok ? go.z * ((1.f - o.z) * o.z) : 0.f;
    d4[sg][3] = ok && o.w > 0.f ? go.w : 0.f;
  }
  load_mask<FT, NW>(mb, a.mask, 2 * nb, lane, wid);
  // ---- lin_out^T: W_out (4 x HID) from the fp32 fragments, row k of tile `tile` at lane k + 16 g
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const int tile = FT * wid + ft;
    floatx4 w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = *reinterpret_cast<const floatx4*>(a.packed + a.L.w_out + ((int64_t)tile * 64 + k + 16 * g) * 4);
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const floatx4 acc = ((w[0] * d4[sg][0] + w[1] * d4[sg][1]) + w[2] * d4[sg][2]) + w[3] * d4[sg][3];
      dx[ft][sg] = dact<FT, ACT>(acc, mb, a, 2 * nb, arow(sg), 16 * tile + 4 * g, ft, sg);
    }
  }

  FragX3 A0[FT];
  for (int b = nb - 1; b >= 0; --b) {
    // ---- fc_1^T
    // G[2b + 1] = dx and G[2b] are the operands of the two GEMMs: their rows are copied out of
    // LDS during those GEMMs (RowSide), not stored as a burst ahead of the weight loads
    float mx = absmax<FT>(dx);
    const uint4* W1 = PB + a.LB.fc1t[b] / 4 + 2 * 64 * FT * wid;
    prefetch_a<FT, NW == 8 ? FT : kPrefetch>(A0, W1, lane);
    float s_x = publish<FT, NW>(X16, dx, mx, red, wid, lane, g, j, &lmax[2 * b + 1]);
    load_mask<FT, NW>(mb, a.mask, 2 * b + 1, lane, wid);
    bwd_gemm<FT, NW, HID>(t, A0, W1, X16, lane, a, 2 * b + 1, s_x, base, roff, wid);
    float inv = 1.0f / (bwd_scale(a.packed_bwd, 3 + 2 * b) * s_x);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg)
        t[ft][sg] = dact<FT, ACT>(t[ft][sg] * inv, mb, a, 2 * b + 1, arow(sg), 16 * (FT * wid + ft) + 4 * g, ft, sg);
    mx = absmax<FT>(t);
    // ---- fc_0^T
    const uint4* W0 = PB + a.LB.fc0t[b] / 4 + 2 * 64 * FT * wid;
    prefetch_a<FT, NW == 8 ? FT : kPrefetch>(A0, W0, lane);
    s_x = publish<FT, NW>(X16, t, mx, red, wid, lane, g, j, &lmax[2 * b]);
    load_mask<FT, NW>(mb, a.mask, 2 * b, lane, wid);
    bwd_gemm<FT, NW, HID>(t, A0, W0, X16, lane, a, 2 * b, s_x, base, roff, wid);
    inv = 1.0f / (bwd_scale(a.packed_bwd, 2 + 2 * b) * s_x);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int sg = 0; sg < 4; ++sg)
        dx[ft][sg] += dact<FT, ACT>(t[ft][sg] * inv, mb, a, 2 * b, arow(sg), 16 * (FT * wid + ft) + 4 * g, ft, sg);
  }
  // G_in (nothing waits on these stores any more), then the layer maxima: one atomic per workgroup and
  // layer for the GEMM operands (the workgroup max publish recorded), one per wave for G_in
  store_rows<FT, NW>(a.G + 2 * nb * a.g_stride + roff * HID, dx, base, a.M, wid, g, j);
  if (a.g_max) {
    const float mx_in = absmax<FT>(dx);
    if (lane == 0) publish_max(a.g_max + 2 * nb, mx_in);
    if (wid == 0 && lane < 2 * nb) publish_max(a.g_max + lane, lmax[lane]);
  }
}

template <int FT, int NW, int ACT>
static int launch_bwd(const BwdArgs& a, hipStream_t s) {
  constexpr int HID = 16 * FT * NW;
  const size_t shm = (size_t)(HID / 32) * 8192 + 64 + 4 * kX3MaxLayers;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&field_bwd_x3_kernel<FT, NW, ACT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return fail(AVR_E_HIP, "field_bwd_x3_kernel: cannot set dynamic LDS to %zu", shm);
    attr = true;
  }
  const int64_t blocks = a.blocks_per_scene * a.n_scenes;
  AVR_REQUIRE(blocks < (1ll << 31), "field backward: too many points");
  field_bwd_x3_kernel<FT, NW, ACT><<<(unsigned)blocks, 64 * NW, shm, s>>>(a);
  return check_launch("field_bwd_x3_kernel");
}

// d_hidden 512, ReLU: 8 waves x 4 tiles, two waves per SIMD as the forward (AVR_X3_BWD_WAVES=4: the 4-wave
// layout, A/B); Softplus keeps the 4-wave layout (its slopes come from the act rows)
static int bwd_waves() {
  const char* e = getenv("AVR_X3_BWD_WAVES");
  return (e && atoi(e) == 4) ? 4 : 8;
}

template <int ACT>
static int dispatch_bwd_act(int d_hidden, const BwdArgs& a, hipStream_t s) {
  switch (d_hidden) {
    case 64: return launch_bwd<1, 4, ACT>(a, s);
    case 128: return launch_bwd<2, 4, ACT>(a, s);
    case 256: return launch_bwd<4, 4, ACT>(a, s);
    case 512:
      if constexpr (ACT == 0) {
        if (bwd_waves() == 8) return launch_bwd<4, 8, ACT>(a, s);
      }
      return launch_bwd<8, 4, ACT>(a, s);
  }
  return fail(AVR_E_UNSUPPORTED, "field backward: d_hidden %d", d_hidden);
}

int dispatch_field_bwd_x3(int d_hidden, const BwdArgs& a, hipStream_t s) {
  return a.beta > 0.f ? dispatch_bwd_act<1>(d_hidden, a, s) : dispatch_bwd_act<0>(d_hidden, a, s);
}

}  // namespace avr
