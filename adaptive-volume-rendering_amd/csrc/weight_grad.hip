// Weight gradients of the field's linear layers (the dW = G^T X, db = sum G
// half of autograd through nn.Linear, models.py:541-592) as one batched
// split-K GEMM on split-fp16 MFMA. For every layer l and K-range k of the
// samples:
//   partial[l][k][o][i]   = sum_{m in k} G_l[m][o] * X_l[m][i]
//   bias_partial[l][k][o] = sum_{m in k} G_l[m][o]
// G (gradient at the layer output) and X (the layer input) are fp32 rows, one
// per sample, as the training forward / backward kernels write them.
//
// The contraction runs over the ROW index of both operands, so the MFMA
// operands are k-strided in memory: each workgroup stages 32-sample chunks of
// its 128-column G and X slices in LDS as row-major fp16 hi/lo images
// (padded 288-B rows) and reads the A and B fragments of
// v_mfma_f32_16x16x32_f16 with gfx950's transposing ds_read_b64_tr_b16.
// Products are W-split x3 (Gh.Xh + Gh.Xl + Gl.Xh, fp32 accumulate) under
// per-layer power-of-two scales from the max |G| / |X| the producing kernels
// tracked, the same arithmetic as the forward's GEMMs. A layer may name a
// per-column BatchNorm-relu transform of X (the training-mode BN path's
// operands, rebuilt from the pre-BN rows in the staging instead of stored).
//
// Work split: workgroup = one 128 x 128 output tile of one layer over one
// K-range; 4 waves of 64 x 64 (4 x 4 MFMA tiles). Consecutive workgroups on
// one XCD take the tiles of the same K-range, so the G / X rows they share are
// read from that XCD's L2.
#include "x3_gemm.h"

namespace avr {

constexpr int kDwTile = 256;                 // output tile (o x i) per workgroup
constexpr int kDwK = 32;
constexpr int kDwRow = 256 + 32;             // bytes per row of a 128-column half image (padded: 9 x 32 B)
constexpr int kDwHalf = kDwK * kDwRow;       // one 128-column half image (32 rows)
constexpr int kDwImg = 2 * kDwHalf;          // one fp16 image of 256 columns
constexpr int kDwStage = 4 * kDwImg;         // G hi, G lo, X hi, X lo
constexpr int kDwXf = 3 * kDwTile * 4;        // XF: the tile's BatchNorm column parameters (mu, scale, shift)

struct DwLayerDev {
  const float* g;
  const float* x;
  int64_t ldg, ldx;
  int O, I, nIt, tile0;
  const unsigned* gmax;
  const unsigned* xmax;
  float* part;
  float* bpart;
  const float* xmu; const float* xscale; const float* xshift;   // NULL, or X = relu((x - mu) * scale + shift)
  int xrelu;                                                     // (xmu NULL) X = relu(x)
};

struct DwArgs {
  DwLayerDev L[AVR_WGRAD_MAX_LAYERS];
  int n_layers, tiles, ksplit;
  int64_t M, kper;
};

typedef short short4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) floatx4 lds_floatx4;

// byte offset of column col of row r in a 256-column image (two 128-column
// halves of padded 288-B rows: 8 consecutive rows start in 8 different 32-B
// bank groups, so the transposed reads below are conflict-free with no swizzle
// and a fragment's address is affine in its column: one lane base + an immediate)
__device__ __forceinline__ int img_off_col(int r, int col) { return kDwHalf * (col >> 7) + kDwRow * r + 2 * (col & 127); }

// Lane base of the transposed operand reads: lane l (g = l >> 4, i = l & 15,
// q = i >> 2, p = i & 3) supplies row 4g + q, columns 4p .. 4p+3 of a 16-column
// block; the second read takes row 16 + 4g + q.
__device__ __forceinline__ int tr_base(int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  return kDwRow * (4 * g + q) + 8 * p;
}

// MFMA operand fragment of 16 columns col0 .. col0+15 of an image (col0 a
// compile-time multiple of 16 after unrolling): lane l gets column col0 + (l & 15),
// K rows {4g .. 4g+3, 16+4g .. 16+4g+3} (g = l >> 4). The same K permutation on
// both operands leaves every product sum unchanged.
__device__ __forceinline__ half8 tr_frag(const lds_char* img_full, int col0_full, int base) {
  const lds_char* img = img_full + kDwHalf * (col0_full >> 7) + 2 * (col0_full & 127) + base;
  typedef __attribute__((address_space(3))) short4_t lds_short4;
  const short4_t r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)img);
  const short4_t r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(img + 16 * kDwRow));
  const short4_t both[2] = {r0, r1};
  return __builtin_bit_cast(half8, both);
}

// NW = 4: one wave per SIMD, 128 x 128 per wave (512 registers: the
// accumulators fill the AGPRs). NW = 8: two waves per SIMD, 128 x 64 per wave
// (256 registers), so one wave's MFMAs run while the other waits on LDS or
// the barrier.
//
// PIPE: the split of chunk c + 1 into its (free) stage and the loads of chunk
// c + 2 are interleaved with chunk c's MFMAs instead of following them after
// the barrier, so the two waves of a SIMD never both sit in a split phase.
// XF: some layer of the launch names a BatchNorm-relu transform of X (its own instantiation: the staging
// registers of the default one are at the limit).
template <int NW, bool PIPE = false, bool XF = false>
__global__ void __launch_bounds__(NW * 64, 1) weight_grad_kernel(DwArgs a) {
  constexpr int WI = NW / 2;                 // waves across the 256 input columns
  constexpr int TO = 8, TI = 16 / WI;        // 16 x 16 MFMA tiles per wave: output rows x input columns
  constexpr int NU = kDwK / NW;              // staged rows per thread and chunk
  extern __shared__ float lds_f[];
  lds_char* lds = (lds_char*)lds_f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // XCD-aware order: blocks b = x, x+8, ... run on XCD x; give them consecutive logical indices
  const int nb = gridDim.x, b = blockIdx.x, x = b & 7, per = nb >> 3, rem = nb & 7;
  const int lg = x * per + (x < rem ? x : rem) + (b >> 3);
  const int krange = lg / a.tiles, tile = lg - krange * a.tiles;
  int l = 0;
  while (l + 1 < a.n_layers && tile >= a.L[l + 1].tile0) ++l;
  const DwLayerDev D = a.L[l];   // one copy in SGPRs (the fields are read in the loop)
  const int local = tile - D.tile0, ot = local / D.nIt, it = local - ot * D.nIt;
  const int o0 = ot * kDwTile, i0 = it * kDwTile;
  const int64_t k0 = (int64_t)krange * a.kper;
  const int64_t k1 = k0 + a.kper < a.M ? k0 + a.kper : a.M;
  const int nch = k1 > k0 ? (int)((k1 - k0 + kDwK - 1) / kDwK) : 0;
  const float sG = pow2_scale_for(__uint_as_float(*D.gmax)), sX = pow2_scale_for(__uint_as_float(*D.xmax));
  const bool bias = D.bpart && it == 0;

  // staging: thread -> 4-column group cc, rows rb + NW u of each 32-row chunk.
  // Columns past O / I read column 0 instead (finite values whose products
  // land in output rows / columns that are never stored), so every load is
  // unconditional: a uniform chunk base (SGPRs) plus a 32-bit lane offset.
  const int cc = threadIdx.x & 63, rb = threadIdx.x >> 6;
  const int ldg = (int)D.ldg, ldx = (int)D.ldx;
  const int gcol = o0 + 4 * cc < D.O ? o0 + 4 * cc : 0;
  const int xcol = i0 + 4 * cc < D.I ? i0 + 4 * cc : 0;
  floatx4 bsum = {0.f, 0.f, 0.f, 0.f};
  // Rows of chunk c that exist: rows past the K-range's end (its ragged last
  // chunk, and the chunks past it that the branch-free pipeline below also
  // loads) read row k1 - 1 and contribute G = 0. `last` is wave-uniform.
  const auto chunk_last = [&](int c) -> int {
    const int64_t n = k1 - 1 - (k0 + (int64_t)kDwK * c);
    return n < kDwK - 1 ? (int)n : kDwK - 1;
  };
  floatx4 gn[NU], xn[NU];
  // row group u (row rb + NW u) of chunk c -> registers (no branches: the
  // pipeline's loads stay in flight across the MFMAs that follow them)
  const auto load_u = [&](int c, int u) {
    const int64_t row0 = k0 + (int64_t)kDwK * c;
    const int last = chunk_last(c);
    const int r = rb + NW * u < last ? rb + NW * u : last;
    gn[u] = *reinterpret_cast<const floatx4*>(D.g + row0 * D.ldg + (r * ldg + gcol));
    xn[u] = *reinterpret_cast<const floatx4*>(D.x + row0 * D.ldx + (r * ldx + xcol));
  };

  const int wo = wid / WI, wi = wid % WI;
  const int trb = tr_base(lane);
  floatx4 acc[TO][TI];
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int u = 0; u < TI; ++u) acc[t][u] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Row group u of chunk c (registers gn / xn) -> LDS stage c & 1, split into
  // fp16 hi / lo; G of rows past the K-range as 0 (also out of the bias sum).
  const auto put = [&](int c, int u) {
    lds_char* st = lds + (c & 1) * kDwStage;
    const int r = rb + NW * u, off = img_off_col(r, 4 * cc);
    const floatx4 g = r > chunk_last(c) ? floatx4{0.f, 0.f, 0.f, 0.f} : gn[u];
    uint2 hi, lo;
    split4(g, sG, hi, lo);
    *(lds_u32x2*)(st + off) = u32x2{hi.x, hi.y};
    *(lds_u32x2*)(st + kDwImg + off) = u32x2{lo.x, lo.y};
    floatx4 xv = xn[u];
    if constexpr (XF) {
      if (D.xmu) {   // block-uniform; the parameters from LDS (a global load here would make the wait for it
                     // also wait for the chunk loads in flight behind it: the counter is in order)
        const lds_floatx4* P = (const lds_floatx4*)(lds + 2 * kDwStage);
        xv = bn_relu4(xv, P[cc], P[64 + cc], P[128 + cc]);
      } else if (D.xrelu) {   // identity statistics: bn_relu4's result with mu 0, scale 1, shift 0, no parameters
        xv = floatx4{fmaxf(xv.x, 0.f), fmaxf(xv.y, 0.f), fmaxf(xv.z, 0.f), fmaxf(xv.w, 0.f)};
      }
    }
    split4(xv, sX, hi, lo);
    *(lds_u32x2*)(st + 2 * kDwImg + off) = u32x2{hi.x, hi.y};
    *(lds_u32x2*)(st + 3 * kDwImg + off) = u32x2{lo.x, lo.y};
    if (bias) bsum += g;
  };

  // Chunk c: the loads of chunk c + 2 are issued first (their registers were
  // split into LDS at the end of chunk c - 1), then the MFMAs on stage c & 1,
  // one barrier, and chunk c + 2 is split into stage c & 1, which nobody reads
  // any more; chunk c + 1 (stage (c + 1) & 1, split at the end of chunk c - 1)
  // was made visible by that barrier. A chunk's loads have the whole MFMA phase
  // to land. Chunks past nch are harmless (rows clamped, G = 0, never read).
  // Scheduling barriers keep each row tile's fragment reads next to its MFMAs.
  const auto step = [&](int c) {
    const lds_char* st = lds + (c & 1) * kDwStage;
#pragma unroll
    for (int u = 0; u < NU; ++u) load_u(c + 2, u);
    half8 bh[TI], bl[TI];
#pragma unroll
    for (int u = 0; u < TI; ++u) {
      bh[u] = tr_frag(st + 2 * kDwImg, (256 / WI) * wi + 16 * u, trb);
      bl[u] = tr_frag(st + 3 * kDwImg, (256 / WI) * wi + 16 * u, trb);
    }
    half8 ah = tr_frag(st, 128 * wo, trb), al = tr_frag(st + kDwImg, 128 * wo, trb);
#pragma unroll
    for (int t = 0; t < TO; ++t) {
      half8 ahn = ah, aln = al;
      if (t + 1 < TO) {
        ahn = tr_frag(st, 128 * wo + 16 * (t + 1), trb);
        aln = tr_frag(st + kDwImg, 128 * wo + 16 * (t + 1), trb);
      }
#pragma unroll
      for (int u = 0; u < TI; ++u) {
        acc[t][u] = mfma32h(ah, bh[u], acc[t][u]);
        acc[t][u] = mfma32h(ah, bl[u], acc[t][u]);
        acc[t][u] = mfma32h(al, bh[u], acc[t][u]);
      }
      __builtin_amdgcn_sched_barrier(0);
      ah = ahn;
      al = aln;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NU; ++u) put(c + 2, u);
  };

  // Pipelined chunk c: stage c & 1 holds chunk c (visible since the last
  // barrier); stage (c + 1) & 1 was last read in chunk c - 1, so row group u
  // of chunk c + 1 (registers gn / xn, loaded during chunk c - 1) is split into
  // it beside row tile 2u's MFMAs (TO / NU = 2 row tiles per row group), and
  // the same registers are refilled with chunk c + 2 beside row tile 2u + 1.
  // One LDS-only barrier per chunk (the loads stay in flight across it).
  const auto step_pipe = [&](int c) {
    const lds_char* st = lds + (c & 1) * kDwStage;
    half8 bh[TI], bl[TI];
#pragma unroll
    for (int u = 0; u < TI; ++u) {
      bh[u] = tr_frag(st + 2 * kDwImg, (256 / WI) * wi + 16 * u, trb);
      bl[u] = tr_frag(st + 3 * kDwImg, (256 / WI) * wi + 16 * u, trb);
    }
    half8 ah = tr_frag(st, 128 * wo, trb), al = tr_frag(st + kDwImg, 128 * wo, trb);
#pragma unroll
    for (int t = 0; t < TO; ++t) {
      half8 ahn = ah, aln = al;
      if (t + 1 < TO) {
        ahn = tr_frag(st, 128 * wo + 16 * (t + 1), trb);
        aln = tr_frag(st + kDwImg, 128 * wo + 16 * (t + 1), trb);
      }
#pragma unroll
      for (int u = 0; u < TI; ++u) {
        acc[t][u] = mfma32h(ah, bh[u], acc[t][u]);
        acc[t][u] = mfma32h(ah, bl[u], acc[t][u]);
        acc[t][u] = mfma32h(al, bh[u], acc[t][u]);
      }
      constexpr int TPU = TO / NU;
      if (t % TPU == 0) {
        put(c + 1, t / TPU);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // DS write
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * TI - 8, 0);
      } else if (t % TPU == 1) {
        load_u(c + 2, t / TPU);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);     // VMEM read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * TI - 8, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      ah = ahn;
      al = aln;
    }
    lds_barrier();
  };

  if constexpr (XF) {
    if (D.xmu && nch > 0) {
      if (threadIdx.x < 192) {
        const int k = threadIdx.x >> 6;
        const float* src = k == 0 ? D.xmu : (k == 1 ? D.xscale : D.xshift);
        ((lds_floatx4*)(lds + 2 * kDwStage))[threadIdx.x] = *reinterpret_cast<const floatx4*>(src + xcol);
      }
      __syncthreads();
    }
  }
  if (nch > 0) {
#pragma unroll
    for (int u = 0; u < NU; ++u) load_u(0, u);
#pragma unroll
    for (int u = 0; u < NU; ++u) put(0, u);
#pragma unroll
    for (int u = 0; u < NU; ++u) load_u(1, u);
    if constexpr (!PIPE) {
#pragma unroll
      for (int u = 0; u < NU; ++u) put(1, u);
    }
    __syncthreads();
  }
  if constexpr (PIPE) {
    static_assert(TO == 2 * NU, "two row tiles per staged row group");
    for (int c = 0; c < nch; ++c) step_pipe(c);
  } else {
    for (int c = 0; c < nch; ++c) step(c);
  }

  // ---- partial dW: lane holds rows 4 (lane >> 4) + r, column lane & 15 of each 16 x 16 tile
  const float inv = (1.0f / sG) * (1.0f / sX);
  float* part = D.part + (int64_t)krange * D.O * D.I;
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int u = 0; u < TI; ++u) {
      const int i = i0 + (256 / WI) * wi + 16 * u + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + 128 * wo + 16 * t + 4 * (lane >> 4) + r;
        if (o < D.O && i < D.I) part[(int64_t)o * D.I + i] = acc[t][u][r] * inv;
      }
    }
  // ---- partial db: the NW row groups' column sums through LDS
  if (bias) {
    __syncthreads();
    float* red = lds_f;   // [NW][256]
    *reinterpret_cast<floatx4*>(red + rb * kDwTile + 4 * cc) = bsum;
    __syncthreads();
    if (threadIdx.x < kDwTile && o0 + (int)threadIdx.x < D.O) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) s += red[q * kDwTile + threadIdx.x];
      D.bpart[(int64_t)krange * D.O + o0 + threadIdx.x] = s;
    }
  }
}

// ---- dW = sum_k partial[k], db = sum_k bias_partial[k] of every layer in one launch (float4 per thread,
// the splits summed in order k = 0 .. n_split - 1): one job per output array, jobs laid end to end in
// float4 units.
constexpr int kDwRedJobs = 2 * AVR_WGRAD_MAX_LAYERS;

struct DwReduceArgs {
  const floatx4* src[kDwRedJobs];
  floatx4* dst[kDwRedJobs];
  int64_t n4[kDwRedJobs];       // float4 per split
  int64_t start[kDwRedJobs + 1];
  int jobs, ksplit;
};

__global__ void __launch_bounds__(256) weight_grad_reduce_kernel(DwReduceArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.start[a.jobs]) return;
  int j = 0;
  while (i >= a.start[j + 1]) ++j;
  const int64_t e = i - a.start[j], n = a.n4[j];
  const floatx4* p = a.src[j] + e;
  floatx4 s = __builtin_nontemporal_load(p);
  for (int k = 1; k < a.ksplit; ++k) s += __builtin_nontemporal_load(p + k * n);
  a.dst[j][e] = s;
}

}  // namespace avr

using namespace avr;

extern "C" int avr_weight_grads_reduce(const avr_wgrad_layer* layers, int n_layers, int n_split, float* const* dw,
                                       float* const* db, void* stream) {
  AVR_REQUIRE(layers && dw && n_layers >= 1 && n_layers <= AVR_WGRAD_MAX_LAYERS,
              "avr_weight_grads_reduce: bad layer list");
  AVR_REQUIRE(n_split >= 1, "avr_weight_grads_reduce: n_split must be >= 1");
  DwReduceArgs a{};
  a.ksplit = n_split;
  int64_t total = 0;
  for (int l = 0; l < n_layers; ++l) {
    const avr_wgrad_layer& s = layers[l];
    AVR_REQUIRE(s.partial && dw[l], "avr_weight_grads_reduce: null pointer (layer %d)", l);
    AVR_REQUIRE(s.out_dim > 0 && s.in_dim > 0 && s.out_dim % 4 == 0 && s.in_dim % 4 == 0,
                "avr_weight_grads_reduce: layer %d dims must be positive multiples of 4", l);
    const bool want_b = s.bias_partial != nullptr;
    AVR_REQUIRE(!want_b || (db && db[l]), "avr_weight_grads_reduce: layer %d has bias partials but no db", l);
    const float* srcs[2] = {s.partial, s.bias_partial};
    float* dsts[2] = {dw[l], want_b ? db[l] : nullptr};
    const int64_t ns[2] = {(int64_t)s.out_dim * s.in_dim / 4, (int64_t)s.out_dim / 4};
    for (int q = 0; q < (want_b ? 2 : 1); ++q) {
      AVR_REQUIRE((reinterpret_cast<uintptr_t>(srcs[q]) | reinterpret_cast<uintptr_t>(dsts[q])) % 16 == 0,
                  "avr_weight_grads_reduce: layer %d buffers must be 16-B aligned", l);
      a.src[a.jobs] = reinterpret_cast<const floatx4*>(srcs[q]);
      a.dst[a.jobs] = reinterpret_cast<floatx4*>(dsts[q]);
      a.n4[a.jobs] = ns[q];
      a.start[a.jobs] = total;
      total += ns[q];
      ++a.jobs;
    }
  }
  a.start[a.jobs] = total;
  weight_grad_reduce_kernel<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(a);
  return check_launch("weight_grad_reduce_kernel");
}

extern "C" int avr_weight_grads(const avr_wgrad_layer* layers, int n_layers, int64_t n_rows, int n_split,
                                void* stream) {
  AVR_REQUIRE(layers && n_layers >= 1 && n_layers <= AVR_WGRAD_MAX_LAYERS, "avr_weight_grads: bad layer list");
  AVR_REQUIRE(n_rows >= 0 && n_split >= 1, "avr_weight_grads: bad sizes");
  DwArgs a{};
  a.n_layers = n_layers;
  a.M = n_rows;
  a.ksplit = n_split;
  const int64_t per = (n_rows + n_split - 1) / n_split;
  a.kper = ((per + kDwK - 1) / kDwK) * kDwK;
  if (a.kper == 0) a.kper = kDwK;
  int tiles = 0;
  bool xf = false;
  for (int l = 0; l < n_layers; ++l) {
    const avr_wgrad_layer& s = layers[l];
    AVR_REQUIRE(s.grad && s.input && s.partial && s.grad_max && s.input_max, "avr_weight_grads: null pointer (layer %d)", l);
    AVR_REQUIRE(s.out_dim > 0 && s.in_dim > 0 && s.out_dim % 4 == 0 && s.in_dim % 4 == 0 && s.ld_grad >= s.out_dim &&
                    s.ld_input >= s.in_dim && s.ld_grad % 4 == 0 && s.ld_input % 4 == 0,
                "avr_weight_grads: layer %d dims must be multiples of 4 within their row strides", l);
    DwLayerDev& D = a.L[l];
    D.g = s.grad; D.x = s.input; D.ldg = s.ld_grad; D.ldx = s.ld_input;
    D.O = s.out_dim; D.I = s.in_dim;
    D.nIt = (s.in_dim + kDwTile - 1) / kDwTile;
    D.tile0 = tiles;
    D.gmax = s.grad_max; D.xmax = s.input_max;
    D.part = s.partial; D.bpart = s.bias_partial;
    AVR_REQUIRE((!s.in_mu && !s.in_scale && !s.in_shift) ||
                    (s.in_mu && s.in_scale && s.in_shift &&
                     ((reinterpret_cast<uintptr_t>(s.in_mu) | reinterpret_cast<uintptr_t>(s.in_scale) |
                       reinterpret_cast<uintptr_t>(s.in_shift)) % 16) == 0),
                "avr_weight_grads: layer %d: in_mu / in_scale / in_shift all NULL or all set (16-B aligned)", l);
    AVR_REQUIRE(!s.input_relu || !s.in_mu, "avr_weight_grads: layer %d: input_relu with in_mu / in_scale / in_shift",
                l);
    D.xmu = s.in_mu; D.xscale = s.in_scale; D.xshift = s.in_shift;
    D.xrelu = s.input_relu;
    xf = xf || s.in_mu || s.input_relu;
    tiles += ((s.out_dim + kDwTile - 1) / kDwTile) * D.nIt;
  }
  a.tiles = tiles;
  const int64_t blocks = (int64_t)tiles * n_split;
  AVR_REQUIRE(blocks < (1ll << 31), "avr_weight_grads: too many tiles");
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&weight_grad_kernel<4>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kDwStage) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&weight_grad_kernel<8>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kDwStage) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&weight_grad_kernel<8, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kDwStage) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&weight_grad_kernel<8, true, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kDwStage + kDwXf) != hipSuccess)
      return fail(AVR_E_HIP, "weight_grad_kernel: cannot set dynamic LDS");
    attr = true;
  }
  const char* e = getenv("AVR_WGRAD_WAVES");   // 8 (default) or 4, read per call
  // AVR_WGRAD_PIPE=0: the 8-wave kernel with the split after the MFMAs (the round-2 schedule, kept for A/B;
  // the pipelined one is 3-6 % faster, profiles/r03g_wgrad_pipe_ab.txt)
  const char* pe = getenv("AVR_WGRAD_PIPE");
  if (xf)   // BatchNorm-relu inputs: the pipelined 8-wave kernel with the transform (no A/B variants)
    weight_grad_kernel<8, true, true><<<(unsigned)blocks, 512, 2 * kDwStage + kDwXf, as_stream(stream)>>>(a);
  else if (e && atoi(e) == 4)
    weight_grad_kernel<4><<<(unsigned)blocks, 256, 2 * kDwStage, as_stream(stream)>>>(a);
  else if (pe && atoi(pe) == 0)
    weight_grad_kernel<8, false><<<(unsigned)blocks, 512, 2 * kDwStage, as_stream(stream)>>>(a);
  else
    weight_grad_kernel<8, true><<<(unsigned)blocks, 512, 2 * kDwStage, as_stream(stream)>>>(a);
  return check_launch("weight_grad_kernel");
}
