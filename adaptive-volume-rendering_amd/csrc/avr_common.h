// Shared device/host helpers for libavr_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avr.h"

namespace avr {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// relu(bn_0(x)) of a training-mode BatchNorm (models.py:456-461) per column: relu((x - mu) * scale + shift),
// scale = gamma * invstd, shift = beta, one explicit fma per value. The BN layers' prologue, their backward's
// relu mask and the weight-gradient staging each recompute it from the pre-BN rows and must agree bit for bit.
__device__ __forceinline__ floatx4 bn_relu4(floatx4 x, floatx4 mu, floatx4 scale, floatx4 shift) {
  const floatx4 d = x - mu;
  return floatx4{fmaxf(__builtin_fmaf(d.x, scale.x, shift.x), 0.f), fmaxf(__builtin_fmaf(d.y, scale.y, shift.y), 0.f),
                 fmaxf(__builtin_fmaf(d.z, scale.z, shift.z), 0.f), fmaxf(__builtin_fmaf(d.w, scale.w, shift.w), 0.f)};
}

// atomicMax on a max-|x| word (non-negative float bits) only where v would raise it: every workgroup of a
// large grid publishing into one word (or one cache line) serialises at its L2 channel; after the first
// workgroups almost all of them only read. A stale read only costs an atomic that changes nothing.
__device__ __forceinline__ void publish_max(unsigned* p, float v) {
  const unsigned b = __float_as_uint(v);
  if (v > 0.f && b > __atomic_load_n(p, __ATOMIC_RELAXED)) atomicMax(p, b);
}

// ------------------------------------------------------------------ errors
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);

#define AVR_REQUIRE(cond, ...)                                   \
  do {                                                           \
    if (!(cond)) return ::avr::fail(AVR_E_INVALID, __VA_ARGS__); \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

// ------------------------------------------------------------------ fp32 ops
// Explicit round-to-nearest primitives so hipcc never contracts an a*b+c that
// the reference evaluates as two roundings (the build also uses -ffp-contract=off).
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fdiv(float a, float b) { return __fdiv_rn(a, b); }

// Gauss-Jordan inverse with partial pivoting in fp64 (torch.inverse is an LU
// solve; fp64 here keeps the fp32-rounded results at the oracle's values).
template <int N>
__device__ __forceinline__ void invert(double (&a)[N][N], double (&inv)[N][N]) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) inv[i][j] = (i == j) ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < N; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
#pragma unroll
    for (int r = c + 1; r < N; ++r) {
      const double v = fabs(a[r][c]);
      if (v > best) { best = v; p = r; }
    }
#pragma unroll
    for (int r = c + 1; r < N; ++r) {  // swap rows c and p (branch-free on the unrolled index)
      if (r == p) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          double t = a[c][j]; a[c][j] = a[r][j]; a[r][j] = t;
          t = inv[c][j]; inv[c][j] = inv[r][j]; inv[r][j] = t;
        }
      }
    }
    const double d = 1.0 / a[c][c];
#pragma unroll
    for (int j = 0; j < N; ++j) { a[c][j] *= d; inv[c][j] *= d; }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      if (r == c) continue;
      const double f = a[r][c];
#pragma unroll
      for (int j = 0; j < N; ++j) { a[r][j] -= f * a[c][j]; inv[r][j] -= f * inv[c][j]; }
    }
  }
}

// per-lane select by a wave-uniform lane mask (bit l set: lane l takes `set`)
__device__ __forceinline__ float mask_select(uint64_t m, float clear, float set) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(clear), "v"(set), "s"(m));
  return r;
}

// ------------------------------------------------------------------ Philox4x32-10
// Counter-based RNG for in-kernel noise (no noise bytes read from HBM).
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one v_mad_u64_u32 per product gives both halves (32-bit integer multiplies are
    // the slow part of the generator; separate mul_lo / mul_hi would double them)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// 4 uniforms in [0,1) (24-bit grid) for (ray, block of 4 samples, stream).
__device__ __forceinline__ float4 philox_uniform4(uint64_t seed, uint64_t ray, uint32_t block4, uint32_t stream) {
  const uint4 r = philox4x32(make_uint4((uint32_t)ray, (uint32_t)(ray >> 32), block4, stream),
                             make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float s = 5.9604644775390625e-08f;  // 2^-24
  return make_float4((r.x >> 8) * s, (r.y >> 8) * s, (r.z >> 8) * s, (r.w >> 8) * s);
}

__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t ray, uint32_t idx, uint32_t stream) {
  const float4 v = philox_uniform4(seed, ray, idx >> 2, stream);
  switch (idx & 3) {
    case 0: return v.x;
    case 1: return v.y;
    case 2: return v.z;
    default: return v.w;
  }
}

// x / n for the sampling formulas: an exact power-of-two n makes the division an
// exact scaling, i.e. bit-identical to x * (1/n) (also for subnormal results).
// POW2 is a template argument of the kernels so the IEEE division is not even
// emitted on the power-of-two path (a runtime select would compute both).
template <bool POW2>
__device__ __forceinline__ float div_count(float x, float n, float inv_n) {
  if constexpr (POW2) return x * inv_n;
  else return fdiv(x, n);
}

// The value of lane l ^ J (J a power of two < 64) without LDS traffic: DPP
// quad permutes for 1 and 2, row shifts for 4 and 8, gfx950's
// v_permlane16/32_swap for 16 and 32 (unlike __shfl_xor's ds_bpermute).
__device__ __forceinline__ float lane_xor(float v, int J, int lane) {
  const int b = __float_as_int(v);
  switch (J) {
    case 1: return __int_as_float(__builtin_amdgcn_update_dpp(b, b, 0xB1, 0xf, 0xf, false));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(b, b, 0x4E, 0xf, 0xf, false));
    case 4: {
      const int up = __builtin_amdgcn_update_dpp(b, b, 0x104, 0xf, 0xf, false);   // row_shl:4 (lane + 4)
      const int dn = __builtin_amdgcn_update_dpp(b, b, 0x114, 0xf, 0xf, false);   // row_shr:4 (lane - 4)
      return mask_select(0xF0F0F0F0F0F0F0F0ull, __int_as_float(up), __int_as_float(dn));   // lane & 4
    }
    case 8: {
      const int up = __builtin_amdgcn_update_dpp(b, b, 0x108, 0xf, 0xf, false);
      const int dn = __builtin_amdgcn_update_dpp(b, b, 0x118, 0xf, 0xf, false);
      return mask_select(0xFF00FF00FF00FF00ull, __int_as_float(up), __int_as_float(dn));
    }
    case 16: {
      const auto r = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
      return mask_select(0xFFFF0000FFFF0000ull, __uint_as_float(r[1]), __uint_as_float(r[0]));
    }
    default: {
      const auto r = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
      return mask_select(0xFFFFFFFF00000000ull, __uint_as_float(r[1]), __uint_as_float(r[0]));
    }
  }
}

// Standard normal via Box-Muller on two Philox uniforms.
__device__ __forceinline__ float philox_normal(uint64_t seed, uint64_t ray, uint32_t idx, uint32_t stream) {
  const float4 v = philox_uniform4(seed, ray, idx, stream);
  const float u1 = fmaxf(v.x, 1e-7f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * v.y);
}

// ------------------------------------------------------------------ wave primitives
__device__ __forceinline__ double shfl_up_d(double v, int d) {
  return __shfl_up(v, d, kWave);
}

// Inclusive wave64 scan of doubles (sum).
__device__ __forceinline__ double wave_incl_scan_add(double v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const double o = __shfl_up(v, d, kWave);
    if (lane >= d) v += o;
  }
  return v;
}

// Inclusive wave64 scan of doubles (product).
__device__ __forceinline__ double wave_incl_scan_mul(double v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const double o = __shfl_up(v, d, kWave);
    if (lane >= d) v *= o;
  }
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ---- DPP wave64 scans (no LDS traffic, unlike __shfl's ds_bpermute).
// dpp_d: the double of the lane named by CTRL (row_shr:n, row_bcast:15/31,
// wave_shr:1); lanes without a source (or outside ROW_MASK) get `ident`.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v, double ident) {
  const unsigned long long b = __double_as_longlong(v), e = __double_as_longlong(ident);
  const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)e, (int)(unsigned)b, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(e >> 32), (int)(unsigned)(b >> 32), CTRL, ROW_MASK, 0xf,
                                             false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143, kDppWaveShr1 = 0x138;

// Inclusive scan (Hillis-Steele in rows of 16, then row broadcasts); OP(a, b).
template <typename OP>
__device__ __forceinline__ double wave_incl_scan_dpp(double v, double ident, OP op) {
  v = op(v, dpp_d<kDppRowShr1>(v, ident));
  v = op(v, dpp_d<kDppRowShr2>(v, ident));
  v = op(v, dpp_d<kDppRowShr4>(v, ident));
  v = op(v, dpp_d<kDppRowShr8>(v, ident));
  v = op(v, dpp_d<kDppRowBcast15, 0xa>(v, ident));
  v = op(v, dpp_d<kDppRowBcast31, 0xc>(v, ident));
  return v;
}

// Exclusive product scan of doubles (lane 0 gets 1) and the wave total.
__device__ __forceinline__ double wave_excl_prod_dpp(double v, double& total) {
  const double incl = wave_incl_scan_dpp(v, 1.0, [](double a, double b) { return a * b; });
  total = readlane_d(incl, 63);
  return dpp_d<kDppWaveShr1>(incl, 1.0);
}

// dpp_d with identity 0 for the shifts (row_shr, wave_shr) that name a lane for
// every destination or none: bound_ctrl zero-fills the lanes without a source,
// so no old value has to be materialised first.
template <int CTRL>
__device__ __forceinline__ double dpp_d0(double v) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

__device__ __forceinline__ double wave_incl_sum_dpp(double v) {
  v += dpp_d0<kDppRowShr1>(v);
  v += dpp_d0<kDppRowShr2>(v);
  v += dpp_d0<kDppRowShr4>(v);
  v += dpp_d0<kDppRowShr8>(v);
  v += dpp_d<kDppRowBcast15, 0xa>(v, 0.0);
  v += dpp_d<kDppRowBcast31, 0xc>(v, 0.0);
  return v;
}

// Exclusive sum scan of doubles (lane 0 gets 0).
__device__ __forceinline__ double wave_excl_sum_dpp(double v) { return dpp_d0<kDppWaveShr1>(wave_incl_sum_dpp(v)); }

__device__ __forceinline__ double wave_total_sum_dpp(double v) { return readlane_d(wave_incl_sum_dpp(v), 63); }

}  // namespace avr
