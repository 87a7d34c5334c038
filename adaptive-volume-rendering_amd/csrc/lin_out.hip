// lin_out over row-major rows, the output layer of the layer-by-layer training paths (avr.bn_train,
// avr.layer_train): forward out = act(relu(x) . W^T + b) (models.py:592, 856-862: sigmoid rgb, relu sigma) and
// its backward d_raw = d out * act'(raw), g = (d_raw . W) where pre > 0 (the relu's threshold_backward), each in
// one pass over the (n_rows, d_hidden) rows. Both are HBM-bound (4 B per hidden value read, plus 4 B per value
// written by the backward; 4 x d_hidden FMAs per row): 16 lanes per row, four rows per wave, W held in registers,
// each lane's float4 columns j + 16 i so a wave instruction reads four 256-B row segments; the 4 sums of a row
// reduce over its 16 lanes with DPP (lane_xor 1, 2, 4, 8 stay inside a DPP row). A grid of at most kLinOutBlocks
// workgroups walks the rows, so the max |.| words (relu(x) forward, d_raw backward) take one publish per wave.
#include "avr_common.h"

namespace avr {

constexpr int kLinOutThreads = 256;
constexpr int kLinOutBlocks = 2048;

__device__ __forceinline__ floatx4 ld4g(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

__device__ __forceinline__ float sum16(float v, int lane) {
  v += lane_xor(v, 1, lane);
  v += lane_xor(v, 2, lane);
  v += lane_xor(v, 4, lane);
  v += lane_xor(v, 8, lane);
  return v;
}

__device__ __forceinline__ float max64(float v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v = fmaxf(v, lane_xor(v, d, lane));
  return v;
}

// QL = d_hidden / 64 float4 columns per lane; RR rows per lane group per pass (independent loads in flight)
template <int QL, int RR>
__global__ void __launch_bounds__(kLinOutThreads) lin_out_fwd_rows_kernel(int64_t M, const float* __restrict__ x,
                                                                         int64_t ld, const float* __restrict__ w,
                                                                         const float* __restrict__ b,
                                                                         float* __restrict__ out, unsigned* xmax) {
  constexpr int H = 64 * QL;
  const int lane = threadIdx.x & 63, j = lane & 15, rs = lane >> 4;
  floatx4 wv[4][QL];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < QL; ++i) wv[k][i] = ld4g(w + k * H + 4 * (j + 16 * i));
  const floatx4 bias = ld4g(b);
  float amax = 0.f;
  const int64_t nw = (int64_t)gridDim.x * (kLinOutThreads / 64);
  for (int64_t r0 = ((int64_t)blockIdx.x * (kLinOutThreads / 64) + (threadIdx.x >> 6)) * 4 * RR; r0 < M;
       r0 += nw * 4 * RR) {
    floatx4 xv[RR][QL];
#pragma unroll
    for (int q = 0; q < RR; ++q) {
      const int64_t row = r0 + 4 * q + rs;
#pragma unroll
      for (int i = 0; i < QL; ++i)
        xv[q][i] = row < M ? ld4g(x + row * ld + 4 * (j + 16 * i)) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < RR; ++q) {
      const int64_t row = r0 + 4 * q + rs;
      float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < QL; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = fmaxf(xv[q][i][e], 0.f);
          amax = fmaxf(amax, a);
#pragma unroll
          for (int k = 0; k < 4; ++k) s[k] = __builtin_fmaf(a, wv[k][i][e], s[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] = sum16(s[k], lane);
      if (row < M && j == 0) {
        floatx4 o;
#pragma unroll
        for (int k = 0; k < 3; ++k) o[k] = fdiv(1.f, fadd(1.f, expf(-fadd(s[k], bias[k]))));
        o[3] = fmaxf(fadd(s[3], bias[3]), 0.f);
        *reinterpret_cast<floatx4*>(out + 4 * row) = o;
      }
    }
  }
  if (xmax) {
    amax = max64(amax, lane);
    if (lane == 0) publish_max(xmax, amax);
  }
}

template <int QL, int RR>
__global__ void __launch_bounds__(kLinOutThreads) lin_out_bwd_rows_kernel(
    int64_t M, const float* __restrict__ gout, const float* __restrict__ y, const float* __restrict__ w,
    const float* __restrict__ pre, int64_t ld, float* __restrict__ draw, float* __restrict__ g, unsigned* dmax) {
  constexpr int H = 64 * QL;
  const int lane = threadIdx.x & 63, j = lane & 15, rs = lane >> 4;
  floatx4 wv[4][QL];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < QL; ++i) wv[k][i] = ld4g(w + k * H + 4 * (j + 16 * i));
  float m = 0.f;
  const int64_t nw = (int64_t)gridDim.x * (kLinOutThreads / 64);
  for (int64_t r0 = ((int64_t)blockIdx.x * (kLinOutThreads / 64) + (threadIdx.x >> 6)) * 4 * RR; r0 < M;
       r0 += nw * 4 * RR) {
    floatx4 pv[RR][QL], d[RR];
#pragma unroll
    for (int q = 0; q < RR; ++q) {
      const int64_t row = r0 + 4 * q + rs;
      const int64_t rr = row < M ? row : M - 1;   // a row past the end reloads the last (never stored)
      const floatx4 go = ld4g(gout + 4 * rr), yv = ld4g(y + 4 * rr);
#pragma unroll
      for (int i = 0; i < QL; ++i) pv[q][i] = ld4g(pre + rr * ld + 4 * (j + 16 * i));
      // aten's sigmoid_backward ((go (1 - y)) y, left to right) and ReluBackward's threshold_backward (a select:
      // go where y > 0, else 0 -- a NaN / inf go on an inactive sigma gives 0, as torch's)
#pragma unroll
      for (int k = 0; k < 3; ++k) d[q][k] = fmul(fmul(go[k], fsub(1.f, yv[k])), yv[k]);
      d[q][3] = yv[3] > 0.f ? go[3] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < RR; ++q) {
      const int64_t row = r0 + 4 * q + rs;
      if (row >= M) continue;   // no cross-lane exchange below
      if (j == 0) *reinterpret_cast<floatx4*>(draw + 4 * row) = d[q];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(d[q][0]), fabsf(d[q][1])), fmaxf(fabsf(d[q][2]), fabsf(d[q][3]))));
#pragma unroll
      for (int i = 0; i < QL; ++i) {
        floatx4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = __builtin_fmaf(d[q][3], wv[3][i][e], __builtin_fmaf(d[q][2], wv[2][i][e],
                                         __builtin_fmaf(d[q][1], wv[1][i][e], fmul(d[q][0], wv[0][i][e]))));
          o[e] = pv[q][i][e] <= 0.f ? 0.f : v;   // aten threshold_backward(v, pre, 0)
        }
        __builtin_nontemporal_store(o, reinterpret_cast<floatx4*>(g + row * H + 4 * (j + 16 * i)));
      }
    }
  }
  if (dmax) {
    m = max64(m, lane);
    if (lane == 0) publish_max(dmax, m);
  }
}

// The activations' backward alone (the fused training path, whose chain kernel applies lin_out^T itself): d_raw
// = [sigmoid_backward(go, y) rgb, threshold_backward(go, y, 0) sigma] per row as lin_out_bwd_rows_kernel computes
// it, and max |d_raw| (the weight gradient's scale input). One thread per row.
__global__ void __launch_bounds__(256) lin_out_act_bwd_kernel(int64_t M, const float* __restrict__ gout,
                                                              const float* __restrict__ y, float* __restrict__ draw,
                                                              unsigned* dmax) {
  const int lane = threadIdx.x & 63;
  float m = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x; row < M; row += (int64_t)gridDim.x * 256) {
    const floatx4 go = ld4g(gout + 4 * row), yv = ld4g(y + 4 * row);
    floatx4 d;
#pragma unroll
    for (int k = 0; k < 3; ++k) d[k] = fmul(fmul(go[k], fsub(1.f, yv[k])), yv[k]);
    d[3] = yv[3] > 0.f ? go[3] : 0.f;
    *reinterpret_cast<floatx4*>(draw + 4 * row) = d;
    m = fmaxf(m, fmaxf(fmaxf(fabsf(d[0]), fabsf(d[1])), fmaxf(fabsf(d[2]), fabsf(d[3]))));
  }
  if (dmax) {
    m = max64(m, lane);
    if (lane == 0) publish_max(dmax, m);
  }
}

// rows per lane group per pass: the forward one, the backward two (scripts/lin_out_bench.py at 131 072 / 98 304
// rows: forward 54 / 45 us with one row, 56 / 49 with two; backward 91 / 78 with one, 88 / 66 with two);
// AVR_LIN_OUT_RR=1|2 sets both (A/B)
static int lin_out_rr(int dflt) {
  const char* e = getenv("AVR_LIN_OUT_RR");
  return e ? (atoi(e) == 1 ? 1 : 2) : dflt;
}

static unsigned lin_out_grid(int64_t M) {
  const int64_t waves = (M + 3) / 4;
  const int64_t blocks = (waves + kLinOutThreads / 64 - 1) / (kLinOutThreads / 64);
  return (unsigned)(blocks < kLinOutBlocks ? blocks : kLinOutBlocks);
}

}  // namespace avr

using namespace avr;

#define AVR_LIN_OUT_CASES(RR, KERNEL, ...)                                         \
  switch (H) {                                                                     \
    case 64: KERNEL<1, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;    \
    case 128: KERNEL<2, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;   \
    case 192: KERNEL<3, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;   \
    case 256: KERNEL<4, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;   \
    case 320: KERNEL<5, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;   \
    case 384: KERNEL<6, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;   \
    case 448: KERNEL<7, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;   \
    default: KERNEL<8, RR><<<grid, kLinOutThreads, 0, s>>>(__VA_ARGS__); break;    \
  }
#define AVR_LIN_OUT_DISPATCH(RR_DEFAULT, KERNEL, ...)            \
  if (lin_out_rr(RR_DEFAULT) == 1) {                              \
    AVR_LIN_OUT_CASES(1, KERNEL, __VA_ARGS__)                     \
  } else {                                                        \
    AVR_LIN_OUT_CASES(2, KERNEL, __VA_ARGS__)                     \
  }

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

extern "C" int avr_lin_out_fwd_rows(int64_t n_rows, int d_hidden, const float* x, int64_t ld_x, const float* weight,
                                    const float* bias, float* out, uint32_t* x_max, void* stream) {
  AVR_REQUIRE(n_rows >= 0 && d_hidden >= 64 && d_hidden <= 512 && d_hidden % 64 == 0,
              "avr_lin_out_fwd_rows: d_hidden %d (64 .. 512, a multiple of 64)", d_hidden);
  if (n_rows == 0) return AVR_OK;
  AVR_REQUIRE(x && weight && bias && out, "avr_lin_out_fwd_rows: null pointer");
  AVR_REQUIRE(ld_x >= d_hidden && ld_x % 4 == 0 && aligned16(x) && aligned16(weight) && aligned16(bias) &&
                  aligned16(out),
              "avr_lin_out_fwd_rows: 16-B aligned rows and tensors (ld_x %lld)", (long long)ld_x);
  const unsigned grid = lin_out_grid(n_rows);
  hipStream_t s = as_stream(stream);
  const int H = d_hidden;
  AVR_LIN_OUT_DISPATCH(1, lin_out_fwd_rows_kernel, n_rows, x, ld_x, weight, bias, out, x_max)
  return check_launch("lin_out_fwd_rows_kernel");
}

extern "C" int avr_lin_out_bwd_rows(int64_t n_rows, int d_hidden, const float* grad_out, const float* out,
                                    const float* weight, const float* pre, int64_t ld_pre, float* d_raw, float* g,
                                    uint32_t* d_raw_max, void* stream) {
  AVR_REQUIRE(n_rows >= 0 && d_hidden >= 64 && d_hidden <= 512 && d_hidden % 64 == 0,
              "avr_lin_out_bwd_rows: d_hidden %d (64 .. 512, a multiple of 64)", d_hidden);
  if (n_rows == 0) return AVR_OK;
  AVR_REQUIRE(grad_out && out && weight && pre && d_raw && g, "avr_lin_out_bwd_rows: null pointer");
  AVR_REQUIRE(ld_pre >= d_hidden && ld_pre % 4 == 0 && aligned16(grad_out) && aligned16(out) && aligned16(weight) &&
                  aligned16(pre) && aligned16(d_raw) && aligned16(g),
              "avr_lin_out_bwd_rows: 16-B aligned rows and tensors (ld_pre %lld)", (long long)ld_pre);
  const unsigned grid = lin_out_grid(n_rows);
  hipStream_t s = as_stream(stream);
  const int H = d_hidden;
  AVR_LIN_OUT_DISPATCH(2, lin_out_bwd_rows_kernel, n_rows, grad_out, out, weight, pre, ld_pre, d_raw, g, d_raw_max)
  return check_launch("lin_out_bwd_rows_kernel");
}

extern "C" int avr_lin_out_act_bwd_rows(int64_t n_rows, const float* grad_out, const float* out, float* d_raw,
                                        uint32_t* d_raw_max, void* stream) {
  AVR_REQUIRE(n_rows >= 0, "avr_lin_out_act_bwd_rows: n_rows %lld", (long long)n_rows);
  if (n_rows == 0) return AVR_OK;
  AVR_REQUIRE(grad_out && out && d_raw, "avr_lin_out_act_bwd_rows: null pointer");
  AVR_REQUIRE(aligned16(grad_out) && aligned16(out) && aligned16(d_raw),
              "avr_lin_out_act_bwd_rows: 16-B aligned tensors");
  const int64_t blocks = (n_rows + 255) / 256;
  lin_out_act_bwd_kernel<<<(unsigned)(blocks < 2048 ? blocks : 2048), 256, 0, as_stream(stream)>>>(
      n_rows, grad_out, out, d_raw, d_raw_max);
  return check_launch("lin_out_act_bwd_kernel");
}
