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
