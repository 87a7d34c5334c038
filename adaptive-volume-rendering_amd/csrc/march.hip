// Early ray termination for the fine pass (BASELINE config 4, SURVEY §8d:
// "stop when T < T_stop, apply it to the fine pass only"; not in the
// reference, which always evaluates every sample).
//
// The fine samples of a ray are consumed front to back in chunks of C (= 64,
// one field workgroup). After each chunk the per-ray compositing state
// (transmittance T in fp64 exactly as composite_fwd_kernel carries it between
// its 64-sample rounds, and fp64 sums of w*rgb, w*zz, w) is updated and rays
// whose T fell below T_stop are dropped from the active list, so the field
// is evaluated only where it can still change the pixel: the dropped tail
// contributes at most T_stop to rgb (and T_stop * max zz to the distance).
//
//   march_init      T = 1, sums = 0, active = 0 .. R-1
//   march_gather    (ro, rd, z[c0 .. c0+C)) of the active rays -> contiguous
//   <field>         forward_rays on the gathered chunk
//   march_composite one wave per active ray: terms, fp64 product scan with
//                   carry T, sums; survivors appended to the next active list
//   march_finish    rgb (+ white background 1 - sum w), distance
#include "avr_common.h"

namespace avr {

constexpr int kMarchWaves = 4;

struct MarchState {  // per ray, fp64
  double T, r, g, b, d, w;
};

__global__ void march_init_kernel(int64_t n_rays, MarchState* __restrict__ st, int32_t* __restrict__ active) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rays) return;
  st[i] = MarchState{1.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  active[i] = (int32_t)i;
}

__global__ void march_gather_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                    const float* __restrict__ z, const int32_t* __restrict__ active, int64_t n_act,
                                    int N, int c0, int C, float* __restrict__ ro_c, float* __restrict__ rd_c,
                                    float* __restrict__ z_c) {
  const int64_t a = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (a >= n_act) return;
  const int64_t r = active[a];
  for (int k = lane; k < C; k += 64) z_c[a * C + k] = z[r * N + c0 + k];
  if (lane < 3) {
    ro_c[3 * a + lane] = ro[3 * r + lane];
    rd_c[3 * a + lane] = rd[3 * r + lane];
  }
}

// One wave per active ray; lane k holds chunk sample c0 + k (C <= 64).
__global__ void __launch_bounds__(64 * kMarchWaves) march_composite_kernel(
    const float* __restrict__ z, const float4* __restrict__ field, const int32_t* __restrict__ active, int64_t n_act,
    int N, int c0, int C, float infinity, float t_stop, MarchState* __restrict__ st, int32_t* __restrict__ next,
    int32_t* __restrict__ n_next) {
  const int lane = threadIdx.x & 63;
  const int64_t a = (int64_t)blockIdx.x * kMarchWaves + (threadIdx.x >> 6);
  if (a >= n_act) return;  // wave-uniform
  const int64_t ray = active[a];
  const float* zr = z + ray * N;
  const int n = c0 + lane;
  const bool ok = lane < C;
  float4 f = ok ? field[a * C + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  float alpha = 0.f, t = 1.f, zz = 0.f;
  if (ok) {  // same terms and rounding points as composite_fwd_kernel (renderers.py:79-111)
    const bool last = n == N - 1;
    const float z0 = zr[n];
    const float z1 = last ? 0.f : zr[n + 1];
    const float d = last ? 1e10f : fsub(z1, z0);
    zz = last ? infinity : z1;
    alpha = fsub(1.0f, expf(-fmul(f.w, d)));
    t = fadd(fsub(1.0f, alpha), 1e-10f);
  }
  MarchState s = st[ray];
  const double incl = wave_incl_scan_mul((double)t, lane) * s.T;
  double excl = __shfl_up(incl, 1, 64);
  if (lane == 0) excl = s.T;
  const double Tn = __shfl(incl, 63, 64);
  const float w = fmul(alpha, (float)excl);
  const double r = wave_sum_d(ok ? (double)w * f.x : 0.0);
  const double g = wave_sum_d(ok ? (double)w * f.y : 0.0);
  const double b = wave_sum_d(ok ? (double)w * f.z : 0.0);
  const double dd = wave_sum_d(ok ? (double)w * zz : 0.0);
  const double ws = wave_sum_d(ok ? (double)w : 0.0);
  if (lane == 0) {
    s.T = Tn;
    s.r += r; s.g += g; s.b += b; s.d += dd; s.w += ws;
    st[ray] = s;
    if (c0 + C < N && (float)Tn >= t_stop) next[atomicAdd(n_next, 1)] = (int32_t)ray;
  }
}

__global__ void march_finish_kernel(const MarchState* __restrict__ st, int64_t n_rays, int white_back,
                                    float* __restrict__ rgb, float* __restrict__ dist) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rays) return;
  const MarchState s = st[i];
  float cr = (float)s.r, cg = (float)s.g, cb = (float)s.b;
  if (white_back) {
    const float bg = fsub(1.0f, (float)s.w);
    cr = fadd(cr, bg); cg = fadd(cg, bg); cb = fadd(cb, bg);
  }
  rgb[3 * i] = cr; rgb[3 * i + 1] = cg; rgb[3 * i + 2] = cb;
  dist[i] = (float)s.d;
}

}  // namespace avr

using namespace avr;

extern "C" int avr_march_state_bytes(int64_t n_rays, int64_t* n_bytes) {
  AVR_REQUIRE(n_bytes, "march: null output");
  AVR_REQUIRE(n_rays >= 0, "march: n_rays %lld < 0", (long long)n_rays);
  *n_bytes = n_rays * (int64_t)sizeof(MarchState);
  return AVR_OK;
}

extern "C" int avr_march_init(int64_t n_rays, void* state, int32_t* active, void* stream) {
  AVR_REQUIRE(n_rays >= 0, "march_init: n_rays %lld < 0", (long long)n_rays);
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(state && active, "march_init: null pointer");
  march_init_kernel<<<(unsigned)((n_rays + 255) / 256), 256, 0, as_stream(stream)>>>(
      n_rays, reinterpret_cast<MarchState*>(state), active);
  return check_launch("march_init_kernel");
}

extern "C" int avr_march_gather(const float* ro, const float* rd, const float* z, const int32_t* active,
                                int64_t n_act, int n_samples, int c0, int chunk, float* ro_c, float* rd_c, float* z_c,
                                void* stream) {
  AVR_REQUIRE(n_act >= 0 && n_samples > 0 && chunk > 0 && chunk <= 64 && c0 >= 0 && c0 + chunk <= n_samples,
              "march_gather: bad sizes (n_act %lld, N %d, c0 %d, C %d)", (long long)n_act, n_samples, c0, chunk);
  if (n_act == 0) return AVR_OK;
  AVR_REQUIRE(ro && rd && z && active && ro_c && rd_c && z_c, "march_gather: null pointer");
  march_gather_kernel<<<(unsigned)((n_act + 3) / 4), 256, 0, as_stream(stream)>>>(ro, rd, z, active, n_act,
                                                                                 n_samples, c0, chunk, ro_c, rd_c,
                                                                                 z_c);
  return check_launch("march_gather_kernel");
}

extern "C" int avr_march_composite(const float* z, const float* field_c, const int32_t* active, int64_t n_act,
                                   int n_samples, int c0, int chunk, float infinity, float t_stop, void* state,
                                   int32_t* active_next, int32_t* n_next, void* stream) {
  AVR_REQUIRE(n_act >= 0 && n_samples > 0 && chunk > 0 && chunk <= 64 && c0 >= 0 && c0 + chunk <= n_samples,
              "march_composite: bad sizes (n_act %lld, N %d, c0 %d, C %d)", (long long)n_act, n_samples, c0, chunk);
  if (n_act == 0) return AVR_OK;
  AVR_REQUIRE(z && field_c && active && state && active_next && n_next, "march_composite: null pointer");
  march_composite_kernel<<<(unsigned)((n_act + kMarchWaves - 1) / kMarchWaves), 64 * kMarchWaves, 0,
                           as_stream(stream)>>>(z, reinterpret_cast<const float4*>(field_c), active, n_act,
                                                n_samples, c0, chunk, infinity, t_stop,
                                                reinterpret_cast<MarchState*>(state), active_next, n_next);
  return check_launch("march_composite_kernel");
}

extern "C" int avr_march_finish(const void* state, int64_t n_rays, int white_back, float* rgb, float* dist,
                                void* stream) {
  AVR_REQUIRE(n_rays >= 0, "march_finish: n_rays %lld < 0", (long long)n_rays);
  if (n_rays == 0) return AVR_OK;
  AVR_REQUIRE(state && rgb && dist, "march_finish: null pointer");
  march_finish_kernel<<<(unsigned)((n_rays + 255) / 256), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const MarchState*>(state), n_rays, white_back, rgb, dist);
  return check_launch("march_finish_kernel");
}
