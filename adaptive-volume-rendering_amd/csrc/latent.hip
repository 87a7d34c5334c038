// Pixel-aligned latent features at points: SpatialEncoder.index
// (models.py:245-274: project into the source view, uv * scale - 1, grid_sample
// bilinear / border / align_corners=True) as NewPixelNeRFNet.forward calls it
// (models.py:753-810) — the `latent` half of the MLP input, which the lin_z
// weight gradients contract against, and phi(..., return_features=True).
//
// The map is read channels-last, (H*W, C): one wave per point, each lane
// blends 8 channels of the 4 corner rows (2 x 16-B loads per corner, the rows
// of neighbouring points mostly L2 hits) and writes them with two 16-B stores,
// so a point costs one 2 KB row out (C = 512) and the output is row-major
// (n_points, C) with no transpose pass.
#include "field_common.h"

namespace avr {

// Scenes of a batch: blockIdx.y = scene s, its view, map lat_hwc + s * lat_stride, points xyz + 3 s n_points,
// rows out + s * n_points * C. The rows stream out non-temporally (they are read once, by the weight-gradient
// kernel, after every other kernel of the backward).
struct LatBatch {
  View v[AVR_MAX_SCENES];
};

__global__ void __launch_bounds__(256) latent_features_kernel(LatBatch vb, const float* __restrict__ lat_hwc,
                                                              int64_t lat_stride, int C, const float* __restrict__ xyz,
                                                              int64_t n_points, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= n_points) return;
  const int s = blockIdx.y;
  lat_hwc += s * lat_stride;
  xyz += 3 * s * n_points;
  out += s * n_points * C;
  const Bilinear bl = bilinear_at(vb.v[s], xyz[3 * m], xyz[3 * m + 1], xyz[3 * m + 2]);
  // two 256-channel groups per pass, both gathered before either is stored (a load behind a store waits for it)
  for (int c0 = 4 * lane; c0 < C; c0 += 512) {
    floatx4 acc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = c0 + 256 * u;
      if (c < C) {
        const floatx4 a = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[0] * C + c);
        const floatx4 b = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[1] * C + c);
        const floatx4 d = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[2] * C + c);
        const floatx4 e = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[3] * C + c);
        // grid_sample's order: nw, ne, sw, se
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[u][t] = fadd(fadd(fadd(fmul(a[t], bl.w[0]), fmul(b[t], bl.w[1])), fmul(d[t], bl.w[2])), fmul(e[t], bl.w[3]));
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (c0 + 256 * u < C) __builtin_nontemporal_store(acc[u], reinterpret_cast<floatx4*>(out + m * C + c0 + 256 * u));
  }
}

}  // namespace avr

using namespace avr;

extern "C" int avr_latent_features(const avr_view_desc* view, const float* latent_hwc, int channels,
                                   const float* xyz, int64_t n_points, float* out, void* stream) {
  AVR_REQUIRE(n_points >= 0 && channels > 0 && channels % 4 == 0, "avr_latent_features: bad sizes");
  if (n_points == 0) return AVR_OK;
  AVR_REQUIRE(view && latent_hwc && xyz && out, "avr_latent_features: null pointer");
  AVR_REQUIRE(view->latent_h > 0 && view->latent_w > 0, "avr_latent_features: bad latent size");
  LatBatch vb;
  view_from_desc(view, &vb.v[0]);
  latent_features_kernel<<<dim3((unsigned)((n_points + 3) / 4), 1), 256, 0, as_stream(stream)>>>(
      vb, latent_hwc, 0, channels, xyz, n_points, out);
  return check_launch("latent_features_kernel");
}

extern "C" int avr_latent_features_batch(const avr_view_desc* views, int n_scenes, const float* latent_hwc,
                                         int channels, const float* xyz, int64_t n_points, float* out,
                                         void* stream) {
  AVR_REQUIRE(n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES, "avr_latent_features_batch: 1..%d scenes per call",
              AVR_MAX_SCENES);
  AVR_REQUIRE(n_points >= 0 && channels > 0 && channels % 4 == 0, "avr_latent_features_batch: bad sizes");
  if (n_points == 0) return AVR_OK;
  AVR_REQUIRE(views && latent_hwc && xyz && out, "avr_latent_features_batch: null pointer");
  LatBatch vb;
  for (int s = 0; s < n_scenes; ++s) {
    AVR_REQUIRE(views[s].latent_h == views[0].latent_h && views[s].latent_w == views[0].latent_w &&
                    views[s].latent_h > 0 && views[s].latent_w > 0,
                "avr_latent_features_batch: scenes need latent maps of one (positive) size");
    view_from_desc(&views[s], &vb.v[s]);
  }
  const int64_t stride = (int64_t)views[0].latent_h * views[0].latent_w * channels;
  latent_features_kernel<<<dim3((unsigned)((n_points + 3) / 4), (unsigned)n_scenes), 256, 0, as_stream(stream)>>>(
      vb, latent_hwc, stride, channels, xyz, n_points, out);
  return check_launch("latent_features_kernel");
}

// ---- d loss / d xyz through the lookup (the adaptive renderer's band points carry a gradient): torch's
// grid_sample grid gradient (bilinear, border padding, align_corners=True: a clipped coordinate passes none)
// chained through grid = uv * scale - 1, uv = (-xc_xy / xc_z) * focal + c, xc = R x + t (models.py:753-810,
// :260-273). One wave per point: lane l sums channels 4l, 4l + 256, ... of
//   gix = sum_c g_c ((ne - nw) wy0 + (se - sw) wy1),  giy = sum_c g_c ((sw - nw) wx0 + (se - ne) wx1)
// over the corner rows of latent_hwc (H*W, C) and the feature gradient row g (C), then lane 0 applies the
// chain. The corners and weights are the forward's (bilinear_from_rot's operations); a corner past the edge
// only occurs with a zero weight or a clipped (zero-gradient) coordinate, so its clamped texel changes nothing.
namespace avr {

__device__ __forceinline__ float lane_sum(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// The summed rows: term t contributes sum_c g_t[c] (corner differences of map_t)[c], map_t (H*W, C) of scene s at
// map[t] + s * map_scene_stride, g_t the point's row at g[t] + row * ldg[t]. One term (the looked-up latent and
// its feature gradient: avr_latent_features_grad_points) or one per linear layer fed by the lookup with that
// layer's per-texel table and output gradient (avr_latent_tables_grad_points).
struct GradTerms {
  const float* map[AVR_LOOKUP_GRAD_TERMS];
  const float* g[AVR_LOOKUP_GRAD_TERMS];
  int64_t ldg[AVR_LOOKUP_GRAD_TERMS];
  int64_t map_scene_stride;
  int n;
};

__global__ void __launch_bounds__(256) latent_features_grad_points_kernel(LatBatch vb, GradTerms T, int C,
                                                                          const float* __restrict__ xyz,
                                                                          int64_t n_points,
                                                                          float* __restrict__ gxyz) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= n_points) return;
  const int s = blockIdx.y;
  const View& v = vb.v[s];
  const int64_t row = s * n_points + m;
  const float x0 = xyz[3 * row], x1 = xyz[3 * row + 1], x2 = xyz[3 * row + 2];
  const float xr[3] = {dot3(v.R + 0, x0, x1, x2), dot3(v.R + 3, x0, x1, x2), dot3(v.R + 6, x0, x1, x2)};
  const Bilinear bl = bilinear_from_rot(v, xr);
  // the forward's coordinates again, for the weights and the clip masks
  const float xc0 = fadd(xr[0], v.t[0]), xc1 = fadd(xr[1], v.t[1]), xc2 = fadd(xr[2], v.t[2]);
  const float u = fadd(fmul(fdiv(-xc0, xc2), v.focal[0]), v.c[0]);
  const float w = fadd(fmul(fdiv(-xc1, xc2), v.focal[1]), v.c[1]);
  const float gx = fsub(fmul(u, v.scale[0]), 1.0f), gy = fsub(fmul(w, v.scale[1]), 1.0f);
  const float ixr = fmul(fdiv(fadd(gx, 1.0f), 2.0f), (float)(v.W - 1));
  const float iyr = fmul(fdiv(fadd(gy, 1.0f), 2.0f), (float)(v.H - 1));
  const float ix = fminf(fmaxf(ixr, 0.f), (float)(v.W - 1)), iy = fminf(fmaxf(iyr, 0.f), (float)(v.H - 1));
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const float wx1 = fsub(ix, fx0), wy1 = fsub(iy, fy0);
  const float wx0 = fsub(fadd(fx0, 1.0f), ix), wy0 = fsub(fadd(fy0, 1.0f), iy);
  float sx = 0.f, sy = 0.f;
  for (int t = 0; t < T.n; ++t) {
    const float* lat_hwc = T.map[t] + s * T.map_scene_stride;
    const float* g = T.g[t] + row * T.ldg[t];
    for (int c = 4 * lane; c < C; c += 256) {
      const floatx4 gv = *reinterpret_cast<const floatx4*>(g + c);
      const floatx4 nw = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[0] * C + c);
      const floatx4 ne = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[1] * C + c);
      const floatx4 sw = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[2] * C + c);
      const floatx4 se = *reinterpret_cast<const floatx4*>(lat_hwc + (int64_t)bl.tex[3] * C + c);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sx += gv[q] * ((ne[q] - nw[q]) * wy0 + (se[q] - sw[q]) * wy1);
        sy += gv[q] * ((sw[q] - nw[q]) * wx0 + (se[q] - ne[q]) * wx1);
      }
    }
  }
  sx = lane_sum(sx);
  sy = lane_sum(sy);
  if (lane == 0) {
    // d grid -> d uv (the clip passes no gradient at or past either edge) -> d xc -> d x = R^T d xc
    const float mxk = ixr > 0.f && ixr < (float)(v.W - 1) ? 1.f : 0.f;
    const float myk = iyr > 0.f && iyr < (float)(v.H - 1) ? 1.f : 0.f;
    const float gu = sx * (0.5f * (float)(v.W - 1)) * mxk * v.scale[0];
    const float gw = sy * (0.5f * (float)(v.H - 1)) * myk * v.scale[1];
    const float a0 = gu * v.focal[0], a1 = gw * v.focal[1];
    const float inv_z = 1.0f / xc2;
    // a clipped coordinate passes exactly zero: at a point on the source camera's plane (xc2 = 0: the lookup
    // is clipped, 1 / xc2 = inf) the chain would otherwise give 0 * inf = NaN (torch's autograd does: the
    // r04q adaptive train step hit a band point at world z = -1.3f, camera z 0, profiles/r05d_*)
    const float num = a0 * xc0 + a1 * xc1;
    const float d0 = a0 != 0.f ? -a0 * inv_z : 0.f, d1 = a1 != 0.f ? -a1 * inv_z : 0.f;
    const float d2 = num != 0.f ? num * inv_z * inv_z : 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) gxyz[3 * row + j] = v.R[j] * d0 + v.R[3 + j] * d1 + v.R[6 + j] * d2;
  }
}

// z_feature's position adjoint for the fused family (models.py:753-794 with PositionalEncoding :41-87): z = R x
// (normalize_z), zf = [z, sin(f_k z + 0), sin(f_k z + pi/2) for k < F (3 each), R d]; given g = d loss / d zf's
// first 3 + 6F columns, d z_c = g_c + sum_j f_j cos(phase_j + f_j z_c) g[3 + 3j + c] (j < 2F, f_j = f_(j/2) =
// freq_factor 2^(j/2)) and d x = R^T d z -- torch autograd's chain (sin', addcmul', bmm') in one thread per point.
__global__ void __launch_bounds__(256) zfeature_grad_points_kernel(LatBatch vb, const float* __restrict__ xyz,
                                                                   int64_t n_points, const float* __restrict__ g,
                                                                   int64_t ldg, int F, float freq_factor,
                                                                   int accumulate, float* __restrict__ gxyz) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= n_points) return;
  const int s = blockIdx.y;
  const View& v = vb.v[s];
  const int64_t row = s * n_points + m;
  const float x0 = xyz[3 * row], x1 = xyz[3 * row + 1], x2 = xyz[3 * row + 2];
  const float z[3] = {dot3(v.R + 0, x0, x1, x2), dot3(v.R + 3, x0, x1, x2), dot3(v.R + 6, x0, x1, x2)};
  const float* gr = g + row * ldg;
  float dz[3] = {gr[0], gr[1], gr[2]};
  constexpr float kHalfPi = 1.57079632679489662f;
  for (int j = 0; j < 2 * F; ++j) {
    const float f = ldexpf(freq_factor, j >> 1);   // freq_factor * 2^k exactly (models.py:45, fp32)
    const float ph = (j & 1) ? kHalfPi : 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) dz[c] += gr[3 + 3 * j + c] * cosf(ph + z[c] * f) * f;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float d = v.R[k] * dz[0] + v.R[3 + k] * dz[1] + v.R[6 + k] * dz[2];
    gxyz[3 * row + k] = accumulate ? gxyz[3 * row + k] + d : d;
  }
}

}  // namespace avr

static int lookup_views(const avr_view_desc* views, int n_scenes, LatBatch* vb, const char* what) {
  AVR_REQUIRE(n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES, "%s: 1..%d scenes per call", what, AVR_MAX_SCENES);
  for (int s = 0; s < n_scenes; ++s) {
    AVR_REQUIRE(views[s].latent_h == views[0].latent_h && views[s].latent_w == views[0].latent_w &&
                    views[s].latent_h > 0 && views[s].latent_w > 0,
                "%s: scenes need latent maps of one (positive) size", what);
    view_from_desc(&views[s], &vb->v[s]);
  }
  return AVR_OK;
}

extern "C" int avr_latent_features_grad_points(const avr_view_desc* views, int n_scenes, const float* latent_hwc,
                                               int channels, const float* xyz, int64_t n_points,
                                               const float* grad_features, float* grad_xyz, void* stream) {
  AVR_REQUIRE(n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES,
              "avr_latent_features_grad_points: 1..%d scenes per call", AVR_MAX_SCENES);
  AVR_REQUIRE(n_points >= 0 && channels > 0 && channels % 4 == 0, "avr_latent_features_grad_points: bad sizes");
  if (n_points == 0) return AVR_OK;
  AVR_REQUIRE(views && latent_hwc && xyz && grad_features && grad_xyz, "avr_latent_features_grad_points: null pointer");
  LatBatch vb;
  int rc = lookup_views(views, n_scenes, &vb, "avr_latent_features_grad_points");
  if (rc) return rc;
  GradTerms T{};
  T.n = 1;
  T.map[0] = latent_hwc;
  T.g[0] = grad_features;
  T.ldg[0] = channels;
  T.map_scene_stride = (int64_t)views[0].latent_h * views[0].latent_w * channels;
  latent_features_grad_points_kernel<<<dim3((unsigned)((n_points + 3) / 4), (unsigned)n_scenes), 256, 0,
                                       as_stream(stream)>>>(vb, T, channels, xyz, n_points, grad_xyz);
  return check_launch("latent_features_grad_points_kernel");
}

extern "C" int avr_latent_tables_grad_points(const avr_view_desc* views, int n_scenes, const float* tables,
                                             int64_t table_scene_stride, int64_t table_stride, int n_tables,
                                             int channels, const float* xyz, int64_t n_points,
                                             const float* const* grads, int64_t ld_grad, float* grad_xyz,
                                             void* stream) {
  AVR_REQUIRE(n_points >= 0 && channels > 0 && channels % 4 == 0 && ld_grad >= channels && ld_grad % 4 == 0 &&
                  n_tables >= 1 && n_tables <= AVR_LOOKUP_GRAD_TERMS && table_stride >= 0 && table_scene_stride >= 0,
              "avr_latent_tables_grad_points: bad sizes");
  if (n_points == 0) return AVR_OK;
  AVR_REQUIRE(views && tables && xyz && grads && grad_xyz, "avr_latent_tables_grad_points: null pointer");
  LatBatch vb;
  int rc = lookup_views(views, n_scenes, &vb, "avr_latent_tables_grad_points");
  if (rc) return rc;
  const int64_t hw = (int64_t)views[0].latent_h * views[0].latent_w;
  AVR_REQUIRE((table_stride >= hw * channels || n_tables == 1) && (table_scene_stride >= n_tables * hw * channels ||
                                                                    n_scenes == 1),
              "avr_latent_tables_grad_points: overlapping tables");
  GradTerms T{};
  T.n = n_tables;
  T.map_scene_stride = table_scene_stride;
  for (int t = 0; t < n_tables; ++t) {
    AVR_REQUIRE(grads[t], "avr_latent_tables_grad_points: null gradient rows %d", t);
    T.map[t] = tables + t * table_stride;
    T.g[t] = grads[t];
    T.ldg[t] = ld_grad;
  }
  latent_features_grad_points_kernel<<<dim3((unsigned)((n_points + 3) / 4), (unsigned)n_scenes), 256, 0,
                                       as_stream(stream)>>>(vb, T, channels, xyz, n_points, grad_xyz);
  return check_launch("latent_features_grad_points_kernel");
}

extern "C" int avr_zfeature_grad_points(const avr_view_desc* views, int n_scenes, const float* xyz, int64_t n_points,
                                        const float* grad_zf, int64_t ld_grad, int num_freqs, float freq_factor,
                                        int accumulate, float* grad_xyz, void* stream) {
  AVR_REQUIRE(n_scenes >= 1 && n_scenes <= AVR_MAX_SCENES, "avr_zfeature_grad_points: 1..%d scenes per call",
              AVR_MAX_SCENES);
  AVR_REQUIRE(n_points >= 0 && num_freqs >= 0 && num_freqs <= 32 && ld_grad >= 3 + 6 * num_freqs,
              "avr_zfeature_grad_points: bad sizes");
  if (n_points == 0) return AVR_OK;
  AVR_REQUIRE(views && xyz && grad_zf && grad_xyz, "avr_zfeature_grad_points: null pointer");
  LatBatch vb;
  for (int s = 0; s < n_scenes; ++s) view_from_desc(&views[s], &vb.v[s]);   // only R is read
  avr::zfeature_grad_points_kernel<<<dim3((unsigned)((n_points + 255) / 256), (unsigned)n_scenes), 256, 0,
                                     as_stream(stream)>>>(vb, xyz, n_points, grad_zf, ld_grad, num_freqs, freq_factor,
                                                          accumulate ? 1 : 0, grad_xyz);
  return check_launch("zfeature_grad_points_kernel");
}
