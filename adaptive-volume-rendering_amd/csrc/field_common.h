// Shared pieces of the radiance-field kernels (field.hip: fp32 MFMA path and
// packing; field_x3.hip: split-fp16 MFMA path).
#pragma once
#include <math.h>

#include "avr_common.h"

namespace avr {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int kFieldWaves = 4;   // 256-thread workgroups, one wave per SIMD
constexpr int kSPW = 16;         // fp32 path: samples per wave (MFMA column count)
constexpr int kInTiles = 3;      // fp32 path: lin_in K = 42 features padded to 48
constexpr int kX3Samples = 64;   // x3 path: samples per workgroup (4 MFMA column groups)
constexpr int kX3InChunks = 2;   // x3 path: lin_in K padded to 64 = 2 chunks of 32
constexpr int kPeSlots = 11;     // x3 prologue: PE entries per lane (6 * num_freqs <= 42)
constexpr int kX3MaxLayers = 2 + 2 * AVR_MAX_BLOCKS;

// Packed blob (floats). fp32 part: [t][ot][lane] float4 fragments for
// v_mfma_f32_16x16x4_f32 (also used by the latent-table kernel for lin_z).
// x3 part: [c][ft][hi | lo][lane][8 x fp16] fragments for
// v_mfma_f32_16x16x32_f16, scaled by 2^e per layer (header holds max|W| bits).
struct Layout {
  int NT;                 // d_hidden / 16
  int KTl;                // d_latent / 16
  int64_t w_in, w_out, fc0[AVR_MAX_BLOCKS], fc1[AVR_MAX_BLOCKS], lin_z[AVR_MAX_BLOCKS];
  int64_t b_in, b_out, b_fc0[AVR_MAX_BLOCKS], b_fc1[AVR_MAX_BLOCKS];
  int64_t x3_hdr, x3_in, x3_out, x3_fc0[AVR_MAX_BLOCKS], x3_fc1[AVR_MAX_BLOCKS];
  int64_t bn_a[AVR_MAX_BLOCKS], bn_c[AVR_MAX_BLOCKS];   // eval BatchNorm affine of block b (bn != 0)
  int bn;
  // use_spade: scale_z[b] fp32 fragments (like lin_z); the per-texel tables carry their biases
  // (b_tab[t]: table t = lin_z[t] for t < n_lin_z, scale_z[t - n_lin_z] after)
  int spade, n_lin_z, n_tables;
  int64_t scale_z[AVR_MAX_BLOCKS], b_tab[2 * AVR_MAX_BLOCKS];
  // x3 fragments of table t's weights (lin_z / scale_z, d_latent a multiple of 64 up to 512: the x3 table
  // kernel's latent tile fits the LDS), header word kX3TabHdr + t
  int x3_tables;
  int64_t x3_tab[2 * AVR_MAX_BLOCKS];
  int64_t total;          // floats
};
constexpr int kX3TabHdr = kX3MaxLayers;                        // header words 18 .. 33
constexpr int kX3PackJobs = kX3MaxLayers + 2 * AVR_MAX_BLOCKS;  // layers of one pack batch

// Backward blob (avr_field_pack_bwd): header (64 words, max|W| bits per layer
// in the forward's numbering) + x3 fragments of fc_0[b]^T and fc_1[b]^T in the
// forward's [c][ft][lane] order, then (ABI 14, d_latent == d_hidden) lin_z[b]^T
// (header word kBwdLinZHdr + b; -1 when absent).
struct BwdLayout {
  int64_t fc0t[AVR_MAX_BLOCKS], fc1t[AVR_MAX_BLOCKS];
  int64_t lzt[AVR_MAX_BLOCKS];
  int64_t total;          // floats
};
constexpr int kBwdLinZHdr = AVR_BN_LAYER_LIN_Z_T;   // header words 34 .. 41

// Training forward / backward (x3 path): relu masks of the 2 * n_blocks + 1
// GEMM inputs, one bit per (feature, sample) a lane holds, bit
// (ft * 4 + sg) * 4 + r; words [layer][workgroup][wave][word][lane].
__host__ __device__ constexpr int mask_words(int FT) { return (FT * 16 + 31) / 32; }

struct View {
  float R[9], t[3];
  float focal[2], c[2], scale[2];
  int H, W;
};

// Source view for the latent lookup (poses = world->camera [R | t], models.py:719-727).
inline void view_from_desc(const avr_view_desc* d, View* v) {
  for (int i = 0; i < 3; ++i) {
    for (int k = 0; k < 3; ++k) v->R[3 * i + k] = d->poses[4 * i + k];
    v->t[i] = d->poses[4 * i + 3];
  }
  for (int i = 0; i < 2; ++i) {
    v->focal[i] = d->focal[i];
    v->c[i] = d->c[i];
    v->scale[i] = d->latent_scaling[i] / d->image_shape[i];  // models.py:263 (fp32 div)
  }
  v->H = d->latent_h;
  v->W = d->latent_w;
}

struct FieldArgs {
  const float* packed;
  const float* table;
  int64_t table_stride;  // floats per lin_z table (HW * d_hidden)
  Layout L;
  View v;
  int n_blocks, n_lin_z, num_freqs;
  float freq_factor;
  float beta;            // > 0: Softplus(beta) activation (x3 inference), 0: ReLU
  // split passes (NS > 1 source views, x3 inference): blocks [b_begin, b_end); h_out: store the residual stream
  // after block b_end - 1 instead of running lin_out; h_in: start from those rows instead of lin_in
  int b_begin, b_end;
  float* h_out;
  const float* h_in;
  // sample source: rays (z != null) or explicit points
  const float* ro; const float* rd; const float* z; int n_samples;
  const float* xyz; const float* vd;
  int64_t M;
  float4* out;
  float* act;                  // training forward: GEMM inputs, layer l at act + l * act_stride, (M, d_hidden)
  int64_t act_stride;          //   floats between layers
  unsigned* mask;              //   their relu masks (see mask_words)
  unsigned* act_max;           //   per-layer max |act| as float bits (atomicMax), or null
  float* zf;                   //   the lin_in input z_feature rows (ld zf_ld, zero padded), or null
  int zf_ld;
  unsigned* zf_max;            //   max |z_feature| as float bits (atomicMax), or null
  // training forward over several scenes in one launch: workgroup b works on
  // scene b / blocks_per_scene (M points each, rows scene * M + m), with that
  // scene's view and lin_z tables (table + scene * table_scene_stride)
  int n_scenes;
  int64_t blocks_per_scene;
  int64_t table_scene_stride;
  View views[AVR_MAX_SCENES];
  unsigned long long* stamps;  // diagnostic builds (-DAVR_STAMPS) only: per-block phase clocks (waves 0, 4)
  int debug;                   // diagnostic builds only: experiment flags (1: every fc layer uses block 0's weights)
};

#ifdef AVR_STAMPS
#define AVR_STAMP(k)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long _t;                                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");              \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (a.stamps && (threadIdx.x & 255) == 0)                                                 \
      a.stamps[(int64_t)blockIdx.x * 64 + 32 * (threadIdx.x >> 8) + (k)] = _t;                \
  } while (0)
#else
#define AVR_STAMP(k) do { } while (0)
#endif

struct Bilinear {
  int tex[4];   // texel index of the 4 corners
  float w[4];
};

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ floatx4 mfma32h(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float dot3(const float* R, float a, float b, float c) {
  return fadd(fadd(fmul(R[0], a), fmul(R[1], b)), fmul(R[2], c));
}

__device__ __forceinline__ float sigmoidf_(float x) { return fdiv(1.0f, fadd(1.0f, expf(-x))); }

// Per-sample geometry of NewPixelNeRFNet.forward (models.py:753-808):
// xyz_rot = R xyz, camera point = xyz_rot + t, R viewdir, and the bilinear
// corners of SpatialEncoder.index (models.py:260-273: uv*scale - 1, then
// grid_sample bilinear / border / align_corners=True).
struct SampleGeom {
  float xr[3], vr[3];
  Bilinear bl;
};

// Rotated point xr = R x -> bilinear corners/weights of the source-view latent:
// camera point xr + t, pinhole uv, uv * scale - 1, then grid_sample bilinear /
// border / align_corners=True (models.py:753-760, SpatialEncoder.index :260-273).
__device__ __forceinline__ Bilinear bilinear_from_rot(const View& v, const float* xr_in) {
  Bilinear bl;
  const float xc0 = fadd(xr_in[0], v.t[0]), xc1 = fadd(xr_in[1], v.t[1]), xc2 = fadd(xr_in[2], v.t[2]);
  const float u = fadd(fmul(fdiv(-xc0, xc2), v.focal[0]), v.c[0]);
  const float w = fadd(fmul(fdiv(-xc1, xc2), v.focal[1]), v.c[1]);
  const float gx = fsub(fmul(u, v.scale[0]), 1.0f), gy = fsub(fmul(w, v.scale[1]), 1.0f);
  float ix = fmul(fdiv(fadd(gx, 1.0f), 2.0f), (float)(v.W - 1));
  float iy = fmul(fdiv(fadd(gy, 1.0f), 2.0f), (float)(v.H - 1));
  ix = fminf(fmaxf(ix, 0.f), (float)(v.W - 1));
  iy = fminf(fmaxf(iy, 0.f), (float)(v.H - 1));
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const float wx1 = fsub(ix, fx0), wy1 = fsub(iy, fy0);
  const float wx0 = fsub(fadd(fx0, 1.0f), ix), wy0 = fsub(fadd(fy0, 1.0f), iy);
  const int X0 = (int)fx0, Y0 = (int)fy0;
  const int X1 = X0 + 1 < v.W ? X0 + 1 : v.W - 1, Y1 = Y0 + 1 < v.H ? Y0 + 1 : v.H - 1;
  bl.tex[0] = Y0 * v.W + X0; bl.w[0] = fmul(wx0, wy0);
  bl.tex[1] = Y0 * v.W + X1; bl.w[1] = fmul(wx1, wy0);
  bl.tex[2] = Y1 * v.W + X0; bl.w[2] = fmul(wx0, wy1);
  bl.tex[3] = Y1 * v.W + X1; bl.w[3] = fmul(wx1, wy1);
  return bl;
}

// Explicit points: xyz / viewdir of point mm under view v.
__device__ __forceinline__ SampleGeom sample_geom_pts(const View& v, const float* xyz, const float* vd, int64_t mm) {
  const float x0 = xyz[3 * mm], x1 = xyz[3 * mm + 1], x2 = xyz[3 * mm + 2];
  const float d0 = vd[3 * mm], d1 = vd[3 * mm + 1], d2 = vd[3 * mm + 2];
  SampleGeom s;
  s.xr[0] = dot3(v.R + 0, x0, x1, x2); s.xr[1] = dot3(v.R + 3, x0, x1, x2); s.xr[2] = dot3(v.R + 6, x0, x1, x2);
  s.vr[0] = dot3(v.R + 0, d0, d1, d2); s.vr[1] = dot3(v.R + 3, d0, d1, d2); s.vr[2] = dot3(v.R + 6, d0, d1, d2);
  s.bl = bilinear_from_rot(v, s.xr);
  return s;
}

__device__ __forceinline__ SampleGeom sample_geom(const FieldArgs& a, int64_t mm) {
  float x0, x1, x2, d0, d1, d2;
  if (a.z) {
    const int64_t r = mm / a.n_samples;
    const float zz = a.z[mm];
    d0 = a.rd[3 * r]; d1 = a.rd[3 * r + 1]; d2 = a.rd[3 * r + 2];
    x0 = fadd(a.ro[3 * r], fmul(d0, zz));      // ros + rds * z (renderers.py:171, :260)
    x1 = fadd(a.ro[3 * r + 1], fmul(d1, zz));
    x2 = fadd(a.ro[3 * r + 2], fmul(d2, zz));
  } else {
    x0 = a.xyz[3 * mm]; x1 = a.xyz[3 * mm + 1]; x2 = a.xyz[3 * mm + 2];
    d0 = a.vd[3 * mm]; d1 = a.vd[3 * mm + 1]; d2 = a.vd[3 * mm + 2];
  }
  const View& v = a.v;
  SampleGeom s;
  s.xr[0] = dot3(v.R + 0, x0, x1, x2); s.xr[1] = dot3(v.R + 3, x0, x1, x2); s.xr[2] = dot3(v.R + 6, x0, x1, x2);
  s.vr[0] = dot3(v.R + 0, d0, d1, d2); s.vr[1] = dot3(v.R + 3, d0, d1, d2); s.vr[2] = dot3(v.R + 6, d0, d1, d2);
  s.bl = bilinear_from_rot(v, s.xr);
  return s;
}

// sample_geom for scene `scene` of a multi-scene launch: its samples are rows
// roff .. roff + M of the z / xyz arrays (roff = scene * M), its rays rows
// roff / n_samples onward, viewed from v (that scene's source view).
__device__ __forceinline__ SampleGeom sample_geom_scene(const FieldArgs& a, const View& v, int64_t roff, int64_t mm) {
  float x0, x1, x2, d0, d1, d2;
  const int64_t g = roff + mm;
  if (a.z) {
    const int64_t r = g / a.n_samples;
    const float zz = a.z[g];
    d0 = a.rd[3 * r]; d1 = a.rd[3 * r + 1]; d2 = a.rd[3 * r + 2];
    x0 = fadd(a.ro[3 * r], fmul(d0, zz));      // ros + rds * z (renderers.py:171, :260)
    x1 = fadd(a.ro[3 * r + 1], fmul(d1, zz));
    x2 = fadd(a.ro[3 * r + 2], fmul(d2, zz));
  } else {
    x0 = a.xyz[3 * g]; x1 = a.xyz[3 * g + 1]; x2 = a.xyz[3 * g + 2];
    d0 = a.vd[3 * g]; d1 = a.vd[3 * g + 1]; d2 = a.vd[3 * g + 2];
  }
  SampleGeom s;
  s.xr[0] = dot3(v.R + 0, x0, x1, x2); s.xr[1] = dot3(v.R + 3, x0, x1, x2); s.xr[2] = dot3(v.R + 6, x0, x1, x2);
  s.vr[0] = dot3(v.R + 0, d0, d1, d2); s.vr[1] = dot3(v.R + 3, d0, d1, d2); s.vr[2] = dot3(v.R + 6, d0, d1, d2);
  s.bl = bilinear_from_rot(v, s.xr);
  return s;
}

// World point -> bilinear corners of the source-view latent (models.py:753-760, :260-273).
__device__ __forceinline__ Bilinear bilinear_at(const View& v, float x0, float x1, float x2) {
  const float xr[3] = {dot3(v.R + 0, x0, x1, x2), dot3(v.R + 3, x0, x1, x2), dot3(v.R + 6, x0, x1, x2)};
  return bilinear_from_rot(v, xr);
}

// Feature k of z_feature (models.py:763-789): [xyz_rot (3), PE (6*num_freqs),
// R viewdir (3)], zero beyond. PE entry q = 3*jj + dd is
// sin(phase_jj + x_dd * freq_jj) with jj = 2*freq_index + {0: sin, 1: pi/2}.
__device__ __forceinline__ float z_feature(const SampleGeom& s, int k, int num_freqs, float freq_factor) {
  // selects instead of runtime-indexed arrays keep everything in registers (no scratch)
  const int npe = 6 * num_freqs;
  const auto pick = [](const float* v, int i) { return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]); };
  if (k < 3) return pick(s.xr, k);
  if (k < 3 + npe) {
    const int q = k - 3, jj = q / 3, dd = q - 3 * jj;
    const float freq = fmul(freq_factor, exp2f((float)(jj >> 1)));
    const float phase = (jj & 1) ? 1.5707963705062866f : 0.f;  // fp32(pi/2)
    return sinf(fadd(phase, fmul(pick(s.xr, dd), freq)));
  }
  if (k < 6 + npe) return pick(s.vr, k - 3 - npe);
  return 0.f;
}

// sin(a) for the positional encoding, ~1.5 ulp for |a| <= 8192 (numpy's
// float32 sin: ~1.45): Cody-Waite reduction by pi/2 (3-term split, fma) +
// Cephes minimax polynomials on [-pi/4, pi/4], straight-line (~25 VALU ops).
// Callers route |a| > 8192 to sinf.
__device__ __forceinline__ float pe_sin_fast(float a) {
  const float j = __builtin_rintf(a * 0.6366197466850281f);
  float r = __builtin_fmaf(-j, 1.5707963705062866f, a);
  r = __builtin_fmaf(-j, -4.371138828673793e-08f, r);
  r = __builtin_fmaf(-j, -1.7151245100058819e-15f, r);
  const float z = r * r;
  const float ps = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  const float S = __builtin_fmaf(r * z, ps, r);
  const float pc = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                                  4.166664568298827e-2f);
  const float C = __builtin_fmaf(z * z, pc, __builtin_fmaf(-0.5f, z, 1.0f));
  const int q = (int)j & 3;
  const float v = (q & 1) ? C : S;
  return (q & 2) ? -v : v;
}

// Power-of-two scale that maps max|x| to [2^13, 2^14] (fp16 split operands).
// The exponent is clamped to [-60, 60] so scale products stay finite.
__device__ __forceinline__ float pow2_scale_for(float maxabs) {
  if (!(maxabs > 0.f) || !isfinite(maxabs)) return 1.0f;
  int e;
  frexpf(maxabs, &e);   // maxabs = m * 2^e, m in [0.5, 1)
  const int k = 14 - e;
  return ldexpf(1.0f, k < -60 ? -60 : (k > 60 ? 60 : k));
}

int dispatch_field_x3(int d_hidden, const FieldArgs& a, hipStream_t s);
// The packed blob's layout for dims (field.hip make_layout / make_bwd_layout), for the kernels of other units
// (bn_train.hip: the layer-by-layer BatchNorm training GEMMs read the same fragments).
int field_layout(const avr_field_dims* d, Layout* L);
int field_bwd_layout(const avr_field_dims* d, BwdLayout* LB);
// lin_z / scale_z tables on the x3 GEMM (L.x3_tables): table[t][texel][d_hidden], t < L.n_tables, for
// n_scenes latent maps (stride d_latent * HW) into tables back to back (stride max(n_tables, 1) * HW * d_hidden)
int dispatch_table_x3(const float* packed, const Layout& L, const float* latent, int HW, int d_latent, int d_hidden,
                      float* table, int n_scenes, hipStream_t s);

struct BwdArgs {
  const float* packed;      // forward blob: lin_out fp32 fragments
  const float* packed_bwd;  // backward blob (BwdLayout)
  Layout L;
  BwdLayout LB;
  int n_blocks;
  int64_t M;
  const float4* out;        // field output (sigmoid rgb, relu sigma)
  const float4* grad_out;
  const unsigned* mask;
  float* G;                 // layer-output gradients, layer l at G + l * g_stride, (M, d_hidden)
  int64_t g_stride;
  unsigned* g_max;          // per-layer max |G| as float bits (atomicMax), or null
  int n_scenes;             // M points per scene, rows scene * M + m
  int64_t blocks_per_scene; // workgroup b: scene b / blocks_per_scene (the forward's map)
  // Softplus(beta) nets (beta > 0, ABI 11): the activation's derivative from the forward's saved GEMM inputs
  // y = softplus(x) (act, layer l at act + l * act_stride): sigmoid(beta x) = 1 - exp(-beta y), no masks
  const float* act;
  int64_t act_stride;
  float beta;
};

int dispatch_field_bwd_x3(int d_hidden, const BwdArgs& a, hipStream_t s);

}  // namespace avr
