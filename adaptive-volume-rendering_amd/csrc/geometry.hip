// Ray generation and depth conversion (one thread per ray; HBM-bound, tiny).
//   get_world_rays   utils.py:315-336  (unproject :246-267, :309-312, :297-307)
//   depth_from_world utils.py:358-361  (transform_world2cam :270-281)
#include "avr_common.h"

namespace avr {

__global__ void __launch_bounds__(256) world_rays_kernel(const float* __restrict__ x_pix,
                                                         const float* __restrict__ K,
                                                         const float* __restrict__ c2w, int64_t sb_stride,
                                                         int64_t ray_stride, int64_t n_sb, int64_t n_rays,
                                                         float* __restrict__ ro, float* __restrict__ rd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_sb * n_rays) return;
  const int64_t sb = i / n_rays, r = i - sb * n_rays;
  double k[3][3], ki[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) k[a][b] = (double)K[sb * 9 + a * 3 + b];
  invert<3>(k, ki);
  const double hx = x_pix[2 * i], hy = x_pix[2 * i + 1];
  float cam[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double kf0 = (double)(float)ki[a][0], kf1 = (double)(float)ki[a][1], kf2 = (double)(float)ki[a][2];
    cam[a] = (float)(kf0 * hx + kf1 * hy + kf2);
  }
  // unproject: x negated, then everything scaled by z = -1 (utils.py:262-265)
  cam[0] = (-cam[0]) * -1.0f;
  cam[1] = cam[1] * -1.0f;
  cam[2] = cam[2] * -1.0f;
  const float nrm = (float)sqrt((double)cam[0] * cam[0] + (double)cam[1] * cam[1] + (double)cam[2] * cam[2]);
  const float d0 = fdiv(cam[0], nrm), d1 = fdiv(cam[1], nrm), d2 = fdiv(cam[2], nrm);
  const float* T = c2w + sb * sb_stride + r * ray_stride;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    rd[3 * i + a] = (float)((double)T[4 * a] * d0 + (double)T[4 * a + 1] * d1 + (double)T[4 * a + 2] * d2);
    ro[3 * i + a] = T[4 * a + 3];
  }
}

__global__ void __launch_bounds__(256) depth_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                                    const float* __restrict__ dist, const float* __restrict__ c2w,
                                                    int64_t sb_stride, int64_t ray_stride, int64_t n_sb,
                                                    int64_t n_rays, float* __restrict__ depth,
                                                    float* __restrict__ ddepth) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_sb * n_rays) return;
  const int64_t sb = i / n_rays, r = i - sb * n_rays;
  const float* T = c2w + sb * sb_stride + r * ray_stride;
  double a[4][4], inv[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) a[p][q] = (double)T[4 * p + q];
  invert<4>(a, inv);
  double z = inv[2][3];
  if (rd) {
    const float d = dist[i];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float w = fadd(ro[3 * i + q], fmul(rd[3 * i + q], d));  // ros + rds * dist (renderers.py:274)
      z += inv[2][q] * (double)w;
    }
  } else {  // ro holds world points (renderers.py:346, :459: depth of the raymarcher's final coords)
#pragma unroll
    for (int q = 0; q < 3; ++q) z += inv[2][q] * (double)ro[3 * i + q];
  }
  depth[i] = (float)(-z);
  if (ddepth && rd)
    ddepth[i] = (float)(-(inv[2][0] * rd[3 * i] + inv[2][1] * rd[3 * i + 1] + inv[2][2] * rd[3 * i + 2]));
}

}  // namespace avr

using namespace avr;

extern "C" int avr_world_rays(const float* x_pix, const float* K, const float* c2w, int64_t c2w_sb_stride,
                              int64_t c2w_ray_stride, int64_t n_sb, int64_t n_rays, float* ro, float* rd,
                              void* stream) {
  AVR_REQUIRE(n_sb >= 0 && n_rays >= 0, "avr_world_rays: negative size");
  const int64_t n = n_sb * n_rays;
  if (n == 0) return AVR_OK;
  AVR_REQUIRE(x_pix && K && c2w && ro && rd, "avr_world_rays: null pointer");
  world_rays_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(
      x_pix, K, c2w, c2w_sb_stride, c2w_ray_stride, n_sb, n_rays, ro, rd);
  return check_launch("world_rays_kernel");
}

extern "C" int avr_depth_from_world(const float* ro, const float* rd, const float* dist, const float* c2w,
                                    int64_t c2w_sb_stride, int64_t c2w_ray_stride, int64_t n_sb, int64_t n_rays,
                                    float* depth, float* ddepth_ddist, void* stream) {
  AVR_REQUIRE(n_sb >= 0 && n_rays >= 0, "avr_depth_from_world: negative size");
  const int64_t n = n_sb * n_rays;
  if (n == 0) return AVR_OK;
  AVR_REQUIRE(ro && (!rd || dist) && c2w && depth, "avr_depth_from_world: null pointer");
  depth_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(ro, rd, dist, c2w, c2w_sb_stride,
                                                                           c2w_ray_stride, n_sb, n_rays, depth,
                                                                           ddepth_ddist);
  return check_launch("depth_kernel");
}
