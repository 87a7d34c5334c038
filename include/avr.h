/*
 * avr.h — C ABI of libavr_hip.so, the MI355X (gfx950) kernels for the
 * coarse/fine volume-rendering hot path of yankeesong/adaptive-volume-rendering.
 *
 * Every entry point:
 *   - takes DEVICE pointers owned by the caller (fp32, contiguous, ray-major,
 *     sample-minor, channel-innermost unless stated) and an explicit HIP stream
 *     (hipStream_t passed as void*; NULL = legacy default stream);
 *   - allocates nothing, is stateless and re-entrant, and only enqueues work;
 *   - returns 0 (AVR_OK) or an error code; avr_last_error_string() describes
 *     the last failure on the calling thread.
 *
 * The reference is pure Python/PyTorch, so there is no foreign binding to
 * replace; each function below replaces one stage of the reference's Python
 * call chain (file:line in /root/reference) and is bound from Python by
 * ctypes (adaptive-volume-rendering_amd/avr/_lib.py).
 */
#ifndef AVR_H_
#define AVR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVR_ABI_VERSION 16
#define AVR_MAX_BLOCKS 8
#define AVR_LOOKUP_GRAD_TERMS 8   /* tables per avr_latent_tables_grad_points call */
#define AVR_MAX_SCENES 16   /* scenes per training-forward launch */

enum {
  AVR_OK = 0,
  AVR_E_INVALID = 1001,     /* bad argument (null pointer, size out of range) */
  AVR_E_UNSUPPORTED = 1002, /* configuration the kernels do not implement     */
  AVR_E_HIP = 1003          /* a HIP runtime call failed                       */
};

int avr_version(void);
const char* avr_last_error_string(void);
/* Number of HIP devices visible (0 when no GPU); never fails. */
int avr_device_count(void);

/* ---------------------------------------------------------------- geometry
 * get_world_rays — utils.py:315-336 (unproject :246-267, normalisation
 * :309-312, transform_rigid :297-307).
 *   x_pix  (n_sb, n_rays, 2)      pixel coordinates
 *   K      (n_sb, 3, 3)           intrinsics
 *   c2w    element (sb, r) at c2w + sb*c2w_sb_stride + r*c2w_ray_stride
 *          (strides in floats; ray stride 0 = one pose per batch, the
 *          stride-0 `expand` the reference's callers pass)
 *   ro, rd (n_sb, n_rays, 3)      outputs                                      */
int avr_world_rays(const float* x_pix, const float* K, const float* c2w, int64_t c2w_sb_stride,
                   int64_t c2w_ray_stride, int64_t n_sb, int64_t n_rays, float* ro, float* rd, void* stream);

/* depth_from_world(ro + rd*dist, c2w) — renderers.py:274-275, utils.py:358-361
 * (transform_world2cam :270-281, a general 4x4 inverse per ray).
 *   dist (n_sb, n_rays) -> depth (n_sb, n_rays)
 *   ddepth_ddist (n_sb, n_rays) or NULL: d depth / d dist, for autograd.
 *   rd = NULL: ro holds world points (dist unused) — depth_from_world of the
 *   raymarcher's final coordinates (renderers.py:346, :459).                   */
int avr_depth_from_world(const float* ro, const float* rd, const float* dist, const float* c2w,
                         int64_t c2w_sb_stride, int64_t c2w_ray_stride, int64_t n_sb, int64_t n_rays,
                         float* depth, float* ddepth_ddist, void* stream);

/* ---------------------------------------------------------------- sampling
 * sample_coarse — renderers.py:4-24 (infinity == -1 branch).
 *   z (n_rays, n_samples) = near + (far-near)*i/N + U*(far-near)/N
 *   noise (n_rays, n_samples) U[0,1) draws, or NULL: counter-based Philox
 *   keyed on (seed, offset + id(ray), sample).
 *   ray_ids (n_rays) int64 or NULL: id(ray) = ray_ids[ray] instead of ray --
 *   a rank's share of a sharded frame keyed by each ray's index in the whole
 *   frame, so the draws do not depend on how the frame was dealt out.          */
int avr_sample_coarse(float near_, float far_, int64_t n_rays, int n_samples, const float* noise,
                      uint64_t seed, uint64_t offset, const int64_t* ray_ids, float* z, void* stream);

/* get_world_rays + sample_coarse in one launch (utils.py:315-336,
 * renderers.py:4-24; the renderer's stage order): the inputs of
 * avr_world_rays, then near / far / n_samples / noise / seed / offset /
 * ray_ids of avr_sample_coarse -> ro, rd (n_sb, n_rays, 3), z (n_sb * n_rays,
 * n_samples), and, if depth_row is not NULL, row 2 of inverse(cam2world) per
 * ray in fp64 (n_sb * n_rays, 4 doubles) for avr_composite_fwd_depth.
 * Outputs equal avr_world_rays + avr_sample_coarse bit for bit.               */
int avr_rays_sample_coarse(const float* x_pix, const float* K, const float* c2w, int64_t c2w_sb_stride,
                           int64_t c2w_ray_stride, int64_t n_sb, int64_t n_rays, float near_, float far_, int n_samples,
                           const float* noise, uint64_t seed, uint64_t offset, const int64_t* ray_ids, float* ro,
                           float* rd, double* depth_row, float* z, void* stream);

/* sample_coarse with per-ray near/far (n_rays) — AdaptiveVolumeRenderer's band
 * around the raymarched distance (renderers.py:492-493).                        */
int avr_sample_coarse_rays(const float* near_, const float* far_, int64_t n_rays, int n_samples,
                           const float* noise, uint64_t seed, uint64_t offset, float* z, void* stream);
/* ABI 16: AdaptiveVolumeRenderer's band for training (renderers.py:490-508): per ray d = (world_x - ro_x) / rd_x,
 * z = sample_coarse(d - eps, d + eps, n_samples) with the given noise (renderers.py:10-14's fp32 operations in
 * torch's order), sorted ascending per ray (torch.sort), and the band points pts = ro + rd * z. world / ro / rd
 * (n_rays, 3), noise / z (n_rays, n_samples), pts (n_rays * n_samples, 3); n_samples <= 64. avr_band_bwd: its
 * adjoint, grad_world (n_rays, 3) = ((sum_i grad_z_i + grad_pts_i . rd) / rd_x, 0, 0); grad_z or grad_pts may be
 * NULL (no gradient).                                                                                            */
int avr_band_fwd(int64_t n_rays, int n_samples, const float* world, const float* ro, const float* rd,
                 const float* noise, float eps, float* z, float* pts, void* stream);
int avr_band_bwd(int64_t n_rays, int n_samples, const float* rd, const float* grad_z, const float* grad_pts,
                 float* grad_world, void* stream);

/* sample_fine + sample_depth + clamp + sort(cat(...)) — renderers.py:27-54,
 * :56-66, :252-258.
 *   weights  (n_rays, n_coarse)  coarse weights (detached)
 *   z_coarse (n_rays, n_coarse)
 *   u, u2    (n_rays, n_importance) the rand / rand_like draws,
 *   noise_depth (n_rays, n_depth)   the randn_like draw;
 *            all three NULL together => in-kernel Philox (seed, offset + id(ray)),
 *            ray_ids as for avr_sample_coarse.
 *   z_sorted (n_rays, n_coarse + n_importance + n_depth) ascending
 *   idx      (n_rays, n_importance) int32 inverse-CDF bin (may be NULL)
 *   z_fine   (n_rays, n_importance) unsorted importance z (may be NULL)
 * n_coarse <= 256, total samples <= 512.                                       */
int avr_sample_fine(const float* weights, const float* z_coarse, float near_, float far_, int64_t n_rays,
                    int n_coarse, int n_importance, int n_depth, float depth_std, const float* u, const float* u2,
                    const float* noise_depth, uint64_t seed, uint64_t offset, const int64_t* ray_ids,
                    float* z_sorted, int32_t* idx, float* z_fine, void* stream);

/* --------------------------------------------------------------- composite
 * volume_integral — renderers.py:69-119.
 *   z (n_rays, N), field (n_rays, N, 4) = (r, g, b, sigma) per sample
 *   rgb (n_rays, 3), dist (n_rays), weights (n_rays, N) or NULL.
 * N <= 1024.                                                                   */
int avr_composite_fwd(const float* z, const float* field, int64_t n_rays, int n_samples, int white_back,
                      float infinity, float* rgb, float* dist, float* weights, void* stream);

/* avr_composite_fwd + depth_from_world(ro + rd * dist, cam2world) in the
 * epilogue (renderers.py:274-275, utils.py:358-361) from the depth rows of
 * avr_rays_sample_coarse: depth (n_rays), equal to avr_depth_from_world bit
 * for bit. ro, rd (n_rays, 3).                                                 */
int avr_composite_fwd_depth(const float* z, const float* field, int64_t n_rays, int n_samples, int white_back,
                            float infinity, const float* ro, const float* rd, const double* depth_row, float* rgb,
                            float* dist, float* weights, float* depth, void* stream);

/* Gradient of volume_integral (autograd of renderers.py:78-112).
 *   grad_rgb (n_rays,3), grad_dist (n_rays) or NULL, grad_weights (n_rays,N)
 *   or NULL -> grad_field (n_rays, N, 4) = d/d(r, g, b, sigma), and grad_z
 *   (n_rays, N) or NULL = d/dz (VolumeRenderer's z carries no gradient;
 *   AdaptiveVolumeRenderer's band does, renderers.py:492-508).               */
int avr_composite_bwd(const float* z, const float* field, int64_t n_rays, int n_samples, int white_back,
                      float infinity, const float* grad_rgb, const float* grad_dist, const float* grad_weights,
                      float* grad_field, float* grad_z, void* stream);

/* ----------------------------------------------- fine pass, early termination
 * BASELINE config 4 (not in the reference; SURVEY §8d "C4 early termination":
 * stop when T < T_stop, fine pass only). The fine samples z (n_rays, N) are
 * consumed front to back in chunks [c0, c0 + C) (C <= 64): gather the active
 * rays' (ro, rd, z chunk), evaluate the field on them, composite the chunk
 * into the per-ray state (fp64 T and sums, the same terms and T carry as
 * avr_composite_fwd) and append the rays with T >= t_stop to active_next
 * (*n_next counts them; zero it first). finish writes rgb (+ 1 - sum w on a
 * white background) and dist. The skipped tail changes rgb by <= t_stop.
 * state: opaque, avr_march_state_bytes(n_rays) bytes of device memory.        */
int avr_march_state_bytes(int64_t n_rays, int64_t* n_bytes);
int avr_march_init(int64_t n_rays, void* state, int32_t* active, void* stream);
int avr_march_gather(const float* ro, const float* rd, const float* z, const int32_t* active, int64_t n_act,
                     int n_samples, int c0, int chunk, float* ro_c, float* rd_c, float* z_c, void* stream);
int avr_march_composite(const float* z, const float* field_c, const int32_t* active, int64_t n_act,
                        int n_samples, int c0, int chunk, float infinity, float t_stop, void* state,
                        int32_t* active_next, int32_t* n_next, void* stream);
int avr_march_finish(const void* state, int64_t n_rays, int white_back, float* rgb, float* dist, void* stream);

/* ------------------------------------------------------------------- field
 * NewPixelNeRFNet.forward — models.py:739-863 with PositionalEncoding :41-87,
 * SpatialEncoder.index :245-274 (bilinear, border, align_corners=True),
 * ResnetFC :541-592, ResnetBlockFC :454-470 — for the default.conf family:
 * use_encoder, use_xyz, normalize_z, PE on xyz only (include_input), raw
 * viewdirs, ReLU, NS = 1, and (x3 inference) eval-mode BatchNorm (dims->bn)
 * and use_spade (dims->spade).
 *
 * The lin_z projections are applied to the latent map once per texel
 * (avr_field_latent_table) and bilinearly interpolated per sample: the
 * interpolation and lin_z are both linear, so this is the same function with
 * one third fewer per-sample FLOPs.                                            */
typedef struct {
  int d_in;        /* MLP input width without latent: 3 + 6*num_freqs + 3 */
  int d_latent;    /* latent channels (multiple of 16, <= 1024)           */
  int d_hidden;    /* 64, 128, 256 or 512                                 */
  int n_blocks;    /* ResnetBlockFC count (<= AVR_MAX_BLOCKS)             */
  int n_lin_z;     /* min(combine_layer, n_blocks)                        */
  int num_freqs;   /* positional-encoding frequencies                     */
  float freq_factor;
  int precision;   /* AVR_FIELD_FP32: v_mfma_f32_16x16x4_f32;
                      AVR_FIELD_X3: split-fp16 v_mfma_f32_16x16x32_f16 (3 products, fp32 accumulate) */
  int bn;          /* 1: eval-mode BatchNorm in every block (train.py --bn, models.py:430-432, 456-461):
                      ResnetBlockFC applies bn_0 in front of BOTH relus (the reference's bn_0-twice quirk).
                      The caller folds the second one into fc_0 (fc0_w := diag(a) W0, fc0_b := a*b0 + c) and
                      passes the per-feature affine y = a*x + c of bn_0 as bn_scale / bn_shift; the kernel
                      applies it to the residual stream in front of fc_0's relu. x3 inference only.       */
  int spade;       /* 1: ResnetFC(use_spade=True) (models.py:528-534, 585-587): before block b < n_lin_z the
                      residual stream becomes scale_z[b](z) * x + lin_z[b](z). Both projections are per-texel
                      tables with their biases included (avr_field_latent_table writes 2 * n_lin_z tables:
                      lin_z then scale_z), so the lin_z biases are NOT folded into lin_in / fc_1 here.
                      x3 inference only, not with bn.                                                      */
  float beta;      /* > 0: ResnetFC(beta=beta) — every ReLU of the MLP is Softplus(beta) (models.py:442-445,
                      536-537; torch: x where beta*x > 20, else log1p(exp(beta*x)) / beta). 0: ReLU.
                      x3 inference only, not with bn.                                                      */
} avr_field_dims;

#define AVR_FIELD_FP32 0
#define AVR_FIELD_X3 1

/* One ResnetFC's nn.Linear tensors, PyTorch layout (out, in) row-major. */
typedef struct {
  const float* lin_in_w;  const float* lin_in_b;
  const float* lin_out_w; const float* lin_out_b;
  const float* fc0_w[AVR_MAX_BLOCKS]; const float* fc0_b[AVR_MAX_BLOCKS];
  const float* fc1_w[AVR_MAX_BLOCKS]; const float* fc1_b[AVR_MAX_BLOCKS];
  const float* lin_z_w[AVR_MAX_BLOCKS]; const float* lin_z_b[AVR_MAX_BLOCKS];
  /* dims->bn only: eval BatchNorm1d bn_0 of block b as a per-feature affine (d_hidden floats each):
     a = weight / sqrt(running_var + eps), c = bias - running_mean * a                                 */
  const float* bn_scale[AVR_MAX_BLOCKS]; const float* bn_shift[AVR_MAX_BLOCKS];
  /* dims->spade only: ResnetFC.scale_z[b] (d_hidden, d_latent) and its bias, b < n_lin_z             */
  const float* scale_z_w[AVR_MAX_BLOCKS]; const float* scale_z_b[AVR_MAX_BLOCKS];
} avr_resnetfc_weights;

/* Source-view buffers set by NewPixelNeRFNet.encode (models.py:705-734) and
 * SpatialEncoder.forward (models.py:326-328). Host struct, passed by pointer. */
typedef struct {
  float poses[12];        /* world->cam rows [R | t], 3x4 row-major */
  float focal[2];         /* (fx, -fy) as stored by encode           */
  float c[2];
  float image_shape[2];   /* (W, H)                                  */
  float latent_scaling[2];
  int latent_h, latent_w;
} avr_view_desc;

/* Floats needed for one packed ResnetFC (fragment-ordered weights + biases). */
int avr_field_packed_floats(const avr_field_dims* dims, int64_t* n_floats);
/* Repack one ResnetFC into MFMA fragment order (device -> device). dims->precision selects what is packed:
 * AVR_FIELD_FP32 both the fp32 and the split-fp16 fragments, AVR_FIELD_X3 only what the x3 kernels and the
 * tables read (ABI 9) -- run the field kernels with the precision the blob was packed for: the fp32 field
 * entry points reject a blob this library packed for AVR_FIELD_X3 (AVR_E_INVALID; host-side record of the
 * last 128 packs, round 4). */
int avr_field_pack(const avr_field_dims* dims, const avr_resnetfc_weights* w, float* packed, void* stream);
/* table (n_lin_z, H*W, d_hidden) = lin_z[b].weight @ latent[:, texel] (no bias;
 * the bias is folded into the packed biases). latent (d_latent, H, W).
 * dims->spade: (2 * n_lin_z, H*W, d_hidden) — lin_z[b] tables, then scale_z[b]
 * tables, each with its bias added. dims->precision: AVR_FIELD_FP32 exact fp32
 * products, AVR_FIELD_X3 the split-fp16 GEMM (d_latent a multiple of 64 up to
 * 512; ABI 9 -- the training path, which recomputes the tables every step).    */
int avr_field_latent_table(const avr_field_dims* dims, const float* packed, const float* latent, int H, int W,
                           float* table, void* stream);
/* The same for n_scenes maps in one launch (ABI 9): latent (n_scenes, d_latent, H, W), table (n_scenes,
 * max(n_tables, 1), H*W, d_hidden) -- the layout avr_field_fwd_*_batch / _train read.                   */
int avr_field_latent_table_batch(const avr_field_dims* dims, const float* packed, const float* latent, int n_scenes,
                                 int H, int W, float* table, void* stream);
/* Field at xyz = ro[r] + rd[r] * z[r, s], viewdir = rd[r]; out (n_rays*n_samples, 4)
 * = (sigmoid rgb, relu sigma).                                                 */
int avr_field_fwd_rays(const avr_field_dims* dims, const avr_view_desc* view, const float* packed,
                       const float* table, const float* ro, const float* rd, const float* z, int64_t n_rays,
                       int n_samples, float* out, void* stream);
/* Field at explicit points: xyz, viewdirs (n_points, 3) -> out (n_points, 4). */
int avr_field_fwd_points(const avr_field_dims* dims, const avr_view_desc* view, const float* packed,
                         const float* table, const float* xyz, const float* viewdirs, int64_t n_points,
                         float* out, void* stream);

/* Several scenes (<= AVR_MAX_SCENES) in one launch, x3 path only: scene s has
 * its own view views[s] (host array) and lin_z tables (tables + s *
 * max(n_lin_z, 1) * H*W * d_hidden: the per-scene tables back to back), and
 * its samples at rows s * n_rays * n_samples (rays: ro / rd rows s * n_rays)
 * or s * n_points (points) of the inputs and of out. The same results as one
 * avr_field_fwd_rays / _points call per scene (the VolumeRenderer's SB > 1
 * batches, renderers.py:171-174 over models.py:739-863 per object).           */
/* NS > 1 source views per object (NewPixelNeRFNet.num_views_per_obj, models.py:749-853; the MLP combines
 * the views at combine_layer, ResnetFC.forward :566-579 with combine_interleaved, utils.py:71-81): x3
 * inference as two launches around the caller's combine.
 *   b_begin == 0 < b_end < n_blocks (b_end >= n_lin_z): lin_in and blocks [0, b_end) of n_scenes
 *     (object, source view) pairs laid out as avr_field_fwd_points_batch's scenes (view s's pose, focal,
 *     principal point and lin_z tables); h_out (n_scenes * n_points, d_hidden) receives the residual
 *     stream entering block b_end instead of an output.
 *   n_lin_z <= b_begin < b_end == n_blocks: blocks [b_begin, n_blocks) and lin_out of n_scenes objects
 *     from h_in rows (the combined stream); out (n_scenes * n_points, 4). views / tables are checked as
 *     in the batch call but not read; xyz / viewdirs may be NULL.                                      */
int avr_field_fwd_points_split(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                               const float* packed, const float* tables, const float* xyz, const float* viewdirs,
                               int64_t n_points, int b_begin, int b_end, const float* h_in, float* h_out, float* out,
                               void* stream);

int avr_field_fwd_rays_batch(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                             const float* packed, const float* tables, const float* ro, const float* rd,
                             const float* z, int64_t n_rays, int n_samples, float* out, void* stream);
int avr_field_fwd_points_batch(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                               const float* packed, const float* tables, const float* xyz, const float* viewdirs,
                               int64_t n_points, float* out, void* stream);

/* ---------------------------------------------------------- field training
 * Autograd of NewPixelNeRFNet.forward for train.py:108-114 (loss.backward()
 * through the ResnetFC: models.py:541-592, :454-470, :856-862), on the x3
 * path (dims->precision must be AVR_FIELD_X3).
 *
 * Both take a batch of n_scenes (<= AVR_MAX_SCENES) scenes of n_points points
 * each in one launch: views[n_scenes] (host array), tables = the scenes'
 * avr_field_latent_table outputs back to back, xyz / viewdirs (n_scenes,
 * n_points, 3), out (n_scenes * n_points, 4); rows r = scene * n_points + m.
 * Forward: avr_field_fwd_points_train = avr_field_fwd_points that also writes
 *   act  (2 n_blocks + 1) layers of (rows, d_hidden) fp32, layer l at
 *        act + l * act_rows * d_hidden (act_rows >= n_scenes * n_points, so
 *        calls for more scenes can fill one buffer): the relu'd input of every
 *        hidden GEMM, act[2b] = relu(x) into fc_0 of block b, act[2b+1] =
 *        relu(fc_0 out) into fc_1, act[2 n_blocks] = relu(x) into lin_out;
 *   mask (mask_words) their relu masks (opaque, read by avr_field_bwd);
 *   act_max (2 n_blocks + 1) or NULL: atomicMax of max |act[l]| (float bits;
 *        zero it first), the split scales of avr_weight_grads;
 *   z_feature (rows, ld_z >= d_in) or NULL (ABI 9): lin_in's input rows as the
 *        kernel computed them (xyz_rot, PE, viewdir_rot, models.py:763-789),
 *        columns d_in .. ld_z-1 zero; z_max (1 word) or NULL: their max |.|.
 * Backward: avr_field_bwd, given the forward's out and d loss / d out
 * (n_points, 4), writes grads (layer l at grads + l * grads_rows * d_hidden,
 * grads_max as act_max):
 *   grads[2b]   = d loss / d fc_0[b] output (pre-relu),
 *   grads[2b+1] = d loss / d fc_1[b] output,
 *   grads[2 n_blocks] = d loss / d lin_in output.
 * so that dW = grads[l]^T act[l] and db = column sums of grads[l] (fc layers;
 * lin_in with the MLP input, lin_z[b] with the interpolated latent and
 * grads[2b-1] (b >= 1) or grads[2 n_blocks] (b = 0), the gradient at block
 * b's input). packed_bwd: avr_field_bwd_packed_floats floats, filled by
 * avr_field_pack_bwd (fc_0 / fc_1 transposed, x3 fragments).                    */
int avr_field_train_sizes(const avr_field_dims* dims, int n_scenes, int64_t n_points, int64_t* act_floats,
                          int64_t* mask_words);
int avr_field_bwd_packed_floats(const avr_field_dims* dims, int64_t* n_floats);
int avr_field_pack_bwd(const avr_field_dims* dims, const avr_resnetfc_weights* w, float* packed_bwd, void* stream);
int avr_field_fwd_points_train(const avr_field_dims* dims, const avr_view_desc* views, int n_scenes,
                               const float* packed, const float* tables, const float* xyz, const float* viewdirs,
                               int64_t n_points, float* out, float* act, int64_t act_rows, uint32_t* mask,
                               uint32_t* act_max, float* z_feature, int ld_z, uint32_t* z_max, void* stream);
/* ABI 11: act / act_rows = the forward's act buffer and its rows per layer (as passed to
 * avr_field_fwd_points_train): read for Softplus(beta) nets (dims->beta > 0), whose activation derivative
 * comes from the saved activations instead of the relu masks; may be NULL for ReLU nets. */
int avr_field_bwd(const avr_field_dims* dims, const float* packed, const float* packed_bwd, int n_scenes,
                  int64_t n_points, const float* out, const float* grad_out, const uint32_t* mask, const float* act,
                  int64_t act_rows, float* grads, int64_t grads_rows, uint32_t* grads_max, void* stream);

/* Weight gradients of linear layers, dW = G^T X and db = sum_rows G (the
 * parameter half of nn.Linear's autograd, models.py:541-592), for up to
 * AVR_WGRAD_MAX_LAYERS layers in one launch: split-K over the rows (n_split
 * ranges), split-fp16 MFMA (3 products, fp32 accumulate) under power-of-two
 * scales from grad_max / input_max (max |.| as float bits, device; the
 * training kernels above accumulate them with atomicMax). The caller sums
 * the partials over the split: dW = sum_k partial[k], db = sum_k bias_partial[k]. */
#define AVR_WGRAD_MAX_LAYERS 16
typedef struct {
  const float* grad;        /* (n_rows, ld_grad): d loss / d layer output, columns [0, out_dim) */
  int64_t ld_grad;
  const float* input;       /* (n_rows, ld_input): the layer input, columns [0, in_dim) */
  int64_t ld_input;
  int out_dim, in_dim;      /* multiples of 4 */
  const uint32_t* grad_max;
  const uint32_t* input_max;
  float* partial;           /* (n_split, out_dim, in_dim) */
  float* bias_partial;      /* (n_split, out_dim) or NULL */
  /* ABI 12: NULL, or the layer input is relu((input - in_mu) * in_scale + in_shift) per column (in_dim each,
   * 16-B aligned) -- a training-mode BatchNorm's operand rebuilt from its pre-BN rows (avr_bn_layer's
   * AVR_BN_RELU, bit for bit); input_max is then the max of the rebuilt values. */
  const float* in_mu; const float* in_scale; const float* in_shift;
  /* ABI 14: nonzero (in_mu / in_scale / in_shift NULL): the layer input is relu(input) (the layer-by-layer path's
   * identity statistics without their column parameters); input_max is then the max of relu(input). */
  int input_relu;
} avr_wgrad_layer;
int avr_weight_grads(const avr_wgrad_layer* layers, int n_layers, int64_t n_rows, int n_split, void* stream);
/* The caller's sum above, for the whole layer list in one launch (ABI 9): dw[l] (out_dim, in_dim) =
 * sum_k layers[l].partial[k], and db[l] (out_dim) = sum_k layers[l].bias_partial[k] where bias_partial is
 * not NULL, the splits added in order k = 0 .. n_split - 1 in fp32 (replaces torch's partial.sum(0) per
 * layer; train.py's loss.backward() fills .grad from these). 16-B aligned buffers. */
int avr_weight_grads_reduce(const avr_wgrad_layer* layers, int n_layers, int n_split, float* const* dw,
                            float* const* db, void* stream);

/* ------------------------------------------------ training-mode BatchNorm (ABI 11, 12)
 * train.py --bn (train.py:210, :265) builds ResnetBlockFC(bn=True): relu(bn_0(x)) -> fc_0 -> relu(bn_0(net))
 * -> fc_1 (+ x), bn_0 twice per block with batch statistics over every row of the field call
 * (models.py:430-432, 454-461; bn_1 is unused). The statistics are a reduction over all rows between two
 * GEMMs, so this path runs the MLP layer by layer over row-major fp32 rows (n_rows, in_dim / out_dim):
 *
 * avr_bn_layer: one x3 GEMM of a layer over all rows (split-fp16 MFMA, fp32 accumulate, as the fused kernels).
 *   mode AVR_BN_FWD: out = W . op + bias (+ add1) (+ add2) with W = the forward blob's layer `layer` (header
 *     numbering: 0 lin_in, 2 + 2b fc_0[b], 3 + 2b fc_1[b]; pack with dims->bn = 0: no eval-BN folding; ABI 13:
 *     a use_spade blob as well -- avr.layer_train runs use_spade / NS > 1 nets on these layers with identity
 *     statistics, in_mu = out_mu = shift = 0, scale = invstd = 1: op = relu(src), mask = [pre_rows > 0]);
 *     partial (n_wg, 2, out_dim) = per 64-row workgroup (mean, sum of squared deviations) of out's columns.
 *   mode AVR_BN_BWD: gp = (W^T . op) * [(pre_rows - out_mu) * out_scale + out_shift > 0] with W^T from the
 *     backward blob (avr_field_pack_bwd): the relu mask of the forward's AVR_BN_RELU operand, recomputed from
 *     the pre-BN rows (ABI 12; the relu'd operands need not be stored); out = gp (+ add1: ABI 14, a residual
 *     gradient, ld d_hidden; add2 / lin_z_table must be NULL); partial = per workgroup (sum gp, sum gp * xhat),
 *     xhat = (pre_rows - out_mu) * out_invstd. ABI 14: layer AVR_BN_LAYER_LIN_Z_T + b (b < n_lin_z, d_latent ==
 *     d_hidden, no use_spade) is lin_z[b]^T with no mask (pre_rows and the out_* vectors NULL): out = W_z[b]^T .
 *     op (+ add1), the point gradient's sum_b Gz[b] . W_z[b] one layer at a time; the partial is zeros.
 *   The operand op (n_rows, in_dim), read from src (columns >= in_valid are 0):
 *     AVR_BN_PLAIN op = src;
 *     AVR_BN_RELU  op = relu((src - in_mu) * in_scale + in_shift)                 (forward: relu(bn_0(x)));
 *     AVR_BN_GRAD  op = src_res + in_scale * (src - in_m1 - (src_pre - in_mu) * in_invstd * in_m2)
 *                  (src = d loss / d bn output, torch's batch_norm backward; src_res may be NULL).
 *   operand_out (ld in_dim) / operand_max (float bits, atomicMax): the operand as the GEMM used it, or NULL.
 * avr_bn_stats: the forward partials -> batch mean / invstd (folded in fp64: sum n mean, sum M2 + n mean^2),
 *   scale = gamma * invstd, and
 *   the running statistics updated as torch does (momentum; unbiased variance).
 * avr_bn_grad_stats: the backward partials -> m1 = mean gp, m2 = mean gp * xhat, coef = gamma * invstd, and
 *   dgamma += sum gp * xhat, dbeta += sum gp.
 * avr_bn_grad_rows: out = res + coef * (g - m1 - (pre - mu) * invstd * m2) (the last BN backward, no GEMM after
 *   it), out_max as operand_max; out must not overlap g, pre or res.                                                                               */
#define AVR_BN_FWD 0
#define AVR_BN_BWD 1
#define AVR_BN_LAYER_LIN_Z_T 34   /* + b: lin_z[b]^T from the backward blob (AVR_BN_BWD, ABI 14; see below) */
#define AVR_BN_PLAIN 0
#define AVR_BN_RELU 1
#define AVR_BN_GRAD 2
typedef struct {
  int64_t n_rows;
  int mode, prologue;
  int in_dim, in_valid;     /* in_dim: 32 * chunks (64 for lin_in, d_hidden otherwise); in_valid <= in_dim  */
  const float* src; int64_t ld_src;
  const float* src_pre;     /* AVR_BN_GRAD: pre-BN rows (ld ld_src) */
  const float* src_res;     /* AVR_BN_GRAD: rows added (ld ld_src) or NULL */
  const float* in_mu; const float* in_scale; const float* in_shift;
  const float* in_m1; const float* in_m2; const float* in_invstd;
  float* operand_out; uint32_t* operand_max;
  const float* blob; int layer;
  const float* bias; const float* add1; const float* add2;   /* AVR_BN_FWD; add1 also BWD (rows ld d_hidden) */
  float* out;                                                 /* (n_rows, d_hidden) */
  const float* pre_rows;                                      /* AVR_BN_BWD (ld d_hidden) */
  const float* out_mu; const float* out_invstd; const float* out_scale; const float* out_shift;
  float* partial;           /* (ceil(n_rows / 64), 2, d_hidden), within avr_bn_partial_floats floats */
  /* AVR_BN_FWD (ABI 12): NULL, or lin_z rows added last, gathered in the epilogue: row m of scene
   * s = m / rows_per_scene (n_views scenes, n_rows = n_views * rows_per_scene) adds the bilinear blend of the table
   * lin_z_table + s * lin_z_scene_stride ((latent_h * latent_w, d_hidden), e.g. avr_field_latent_table's) at the
   * world point xyz[m] (n_rows, 3) in views[s] -- avr_latent_features' lookup and blend, bit for bit. */
  const float* lin_z_table; int64_t lin_z_scene_stride;
  const float* xyz; const avr_view_desc* views; int n_views; int64_t rows_per_scene;
  /* AVR_BN_BWD (ABI 14): NULL, or max |out| over the stored rows as float bits, max with what is there (the next
   * weight gradient's scale without a reduction pass over the rows) */
  uint32_t* out_max;
} avr_bn_layer;
int avr_bn_layer_run(const avr_field_dims* dims, const avr_bn_layer* l, void* stream);
/* Floats of an avr_bn_layer partial buffer for n_rows rows of n_cols columns: the per-workgroup partials
 * followed by the fp64 scratch avr_bn_stats / avr_bn_grad_stats fold them through (no allocation inside). */
int avr_bn_partial_floats(int64_t n_rows, int n_cols, int64_t* n_floats);
int avr_bn_stats(const float* partial, int64_t n_rows, int n_cols, const float* gamma, float eps, float momentum,
                 float* running_mean, float* running_var, float* mu, float* invstd, float* scale, void* stream);
int avr_bn_grad_stats(const float* partial, int64_t n_rows, int n_cols, const float* gamma, const float* invstd,
                      float* coef, float* m1, float* m2, float* dgamma, float* dbeta, void* stream);
int avr_bn_grad_rows(int64_t n_rows, int n_cols, const float* g, const float* pre, const float* res,
                     const float* coef, const float* m1, const float* m2, const float* mu, const float* invstd,
                     float* out, uint32_t* out_max, void* stream);
/* lin_out over row-major rows (ABI 14), the layer-by-layer paths' output layer (avr.bn_train, avr.layer_train;
 * replaces their torch relu / addmm / sigmoid / threshold_backward, models.py:592, 856-862), d_hidden 64 .. 512
 * (a multiple of 64), every pointer 16-B aligned, weight (4, d_hidden) and bias (4) as nn.Linear holds them:
 * avr_lin_out_fwd_rows: out (n_rows, 4) = [sigmoid(raw[0:3]), relu(raw[3])], raw = relu(x) . weight^T + bias,
 *   x (n_rows, ld_x); x_max (or NULL): max relu(x) as float bits, max with what is there.
 * avr_lin_out_bwd_rows: d_raw (n_rows, 4) = [(grad_out (1 - y)) y rgb, sigma: grad_out where y > 0 else 0] with
 *   y = out (aten's sigmoid_backward and ReluBackward's threshold_backward, bit for bit), g (n_rows, d_hidden) = d_raw . weight where pre > 0, else 0 (aten
 *   threshold_backward; pre (n_rows, ld_pre) = lin_out's input before its relu); d_raw_max (or NULL): max |d_raw|
 *   as float bits, max with what is there. */
/* The spade product rule's backward (ABI 14; avr.layer_train, models.py:585-587: X' = S * X + T): over n values
 * (a multiple of 4, 16-B aligned arrays) gs = g * x and g_out = s * g, each one fp32 product as torch's mul (bit
 * for bit); gs_max (or NULL): max |gs| as float bits, max with what is there. */
int avr_spade_bwd_rows(int64_t n, const float* g, const float* x, const float* s, float* gs, float* g_out,
                       uint32_t* gs_max, void* stream);
int avr_lin_out_fwd_rows(int64_t n_rows, int d_hidden, const float* x, int64_t ld_x, const float* weight,
                         const float* bias, float* out, uint32_t* x_max, void* stream);
int avr_lin_out_bwd_rows(int64_t n_rows, int d_hidden, const float* grad_out, const float* out, const float* weight,
                         const float* pre, int64_t ld_pre, float* d_raw, float* g, uint32_t* d_raw_max, void* stream);
/* ABI 16: the activations' backward alone, d_raw (n_rows, 4) and d_raw_max as avr_lin_out_bwd_rows computes them
 * (no lin_out^T: the fused training path's chain kernel applies it); 16-B aligned (n_rows, 4) rows. */
int avr_lin_out_act_bwd_rows(int64_t n_rows, const float* grad_out, const float* out, float* d_raw,
                             uint32_t* d_raw_max, void* stream);

/* Latent features at points — SpatialEncoder.index (models.py:245-274) as
 * NewPixelNeRFNet.forward uses it (models.py:753-810): bilinear / border /
 * align_corners=True lookup of latent_hwc (H*W, channels), the source view's
 * map channels-last, at world points xyz (n_points, 3) -> out (n_points,
 * channels). channels multiple of 4.                                           */
int avr_latent_features(const avr_view_desc* view, const float* latent_hwc, int channels, const float* xyz,
                        int64_t n_points, float* out, void* stream);
/* n_scenes (<= AVR_MAX_SCENES) views in one launch (ABI 9): latent_hwc (n_scenes, H*W, channels), xyz
 * (n_scenes, n_points, 3), out (n_scenes * n_points, channels).                                         */
int avr_latent_features_batch(const avr_view_desc* views, int n_scenes, const float* latent_hwc, int channels,
                              const float* xyz, int64_t n_points, float* out, void* stream);
/* ABI 12: the adjoint of that lookup with respect to the points -- grad_xyz (n_scenes * n_points, 3) = d loss /
 * d xyz given grad_features (n_scenes * n_points, channels) = d loss / d features: grid_sample's grid gradient
 * (bilinear, border padding -- a clipped coordinate passes no gradient --, align_corners=True) through the
 * projection uv = (-xc_xy / xc_z) * focal + c, xc = R xyz + t (models.py:753-810, :260-273). Replaces the torch
 * autograd of SpatialEncoder.index for the adaptive renderer's band points (renderers.py:492-508).           */
int avr_latent_features_grad_points(const avr_view_desc* views, int n_scenes, const float* latent_hwc, int channels,
                                    const float* xyz, int64_t n_points, const float* grad_features, float* grad_xyz,
                                    void* stream);
/* ABI 15: the same position gradient where the looked-up features feed only linear maps whose per-texel images are
 * at hand -- the lin_z tables (avr_field_latent_table: table_b = lin_z[b].weight @ latent, no bias): sum_b
 * grad_b . lin_z[b](interp(latent, p)) = sum_b grad_b . interp(table_b, p) (both linear), so the gradient through
 * the lookup needs no d loss / d features = sum_b grad_b W_z[b] (a d_hidden x d_latent product per point per
 * table) -- the corner differences of each table dotted with its row of grad_b. tables: scene s, table b at
 * tables + s * table_scene_stride + b * table_stride, (H*W, channels) each; grads[b] (n_scenes * n_points, ld_grad)
 * the gradient at lin_z[b]'s output (d loss / d block-b input); grad_xyz (n_scenes * n_points, 3) written.
 * 1 <= n_tables <= AVR_LOOKUP_GRAD_TERMS. Replaces the torch autograd of SpatialEncoder.index for points whose
 * latent map needs no gradient (the adaptive renderer's band, renderers.py:492-508). */
int avr_latent_tables_grad_points(const avr_view_desc* views, int n_scenes, const float* tables,
                                  int64_t table_scene_stride, int64_t table_stride, int n_tables, int channels,
                                  const float* xyz, int64_t n_points, const float* const* grads, int64_t ld_grad,
                                  float* grad_xyz, void* stream);
/* ABI 16: the position gradient through z_feature for the fused family (use_xyz, normalize_z, PositionalEncoding
 * with include_input on z = R xyz, raw view directions after it; models.py:753-794, :41-87): grad_zf (n_scenes *
 * n_points rows of ld_grad >= 3 + 6 num_freqs) = d loss / d z_feature's first 3 + 6 num_freqs columns; grad_xyz
 * (n_scenes * n_points, 3) = R_s^T d loss / d z, written (accumulate = 0) or added to (accumulate = 1: after the
 * lookup's gradient). Replaces the torch autograd of z_feature for the adaptive renderer's band points.        */
int avr_zfeature_grad_points(const avr_view_desc* views, int n_scenes, const float* xyz, int64_t n_points,
                             const float* grad_zf, int64_t ld_grad, int num_freqs, float freq_factor, int accumulate,
                             float* grad_xyz, void* stream);

/* --------------------------------------------------------- LSTM ray marcher
 * Raymarcher / AdaptiveVolumeRenderer march (renderers.py:313-351, :380-432):
 * x = ro + rd * init_dist, then `steps` x { v = latent features at x
 * (bilinear, models.py:753-823), (h, c) = LSTMCell(v, (h, c)) with hidden 16,
 * sd = out_layer(h), x += rd * sd }; world (n_rays, 3) = final x, final_dist
 * (n_rays) or NULL = (x - ro)_x / rd_x (renderers.py:490, quirk kept), trace
 * ((steps + 1), n_rays, 3) or NULL = every x. gate_table (H*W, 64) =
 * latent (C, H*W)^T . weight_ih^T (C = feature channels), the input projection
 * per texel; w_hh (64, 16), b_ih / b_hh (64), w_out (16), b_out (1) are the
 * LSTMCell / Linear parameters in torch layout.                               */
int avr_raymarch(const avr_view_desc* view, const float* gate_table, const float* w_hh, const float* b_ih,
                 const float* b_hh, const float* w_out, const float* b_out, const float* ro, const float* rd,
                 const float* init_dist, int64_t n_rays, int steps, float* world, float* final_dist, float* trace,
                 void* stream);

/* Training (ABI 11): the march with autograd for train.py's AdaptiveVolumeRenderer / Raymarcher step
 * (renderers.py:413-432, :320-343). n_scenes (<= AVR_MAX_SCENES) scenes of n_per_scene rays each (ray r in
 * scene r / n_per_scene, its view and gate table; gate_tables (n_scenes, H*W, 64)). Forward: world (n, 3),
 * trace ((steps + 1), n, 3) = every point, state (steps, n, 96) = h, c, i, f, g, o per step (the backward's
 * input). Backward, given grad_world (n, 3): d_tables (n_scenes, H*W, 64), fp32, = d loss / d gate table
 * (written whole; W_ih's gradient is then sum_s d_tables[s]^T latent_s^T, the latent's W_ih^T d_tables[s]),
 * d_grads (64*16 + 64 + 16 + 1) = d W_hh, d (b_ih = b_hh), d w_out, d b_out, with the reference's clamp(-10, 10)
 * of every h gradient (state[0].register_hook) and grid_sample's border / align_corners=True position gradient.
 * ABI 15: bit-deterministic by construction, no floating-point atomics -- the table gradient summed as int64
 * fixed-point values under one power-of-two scale per call (chosen from max |dg| so no sum can overflow; integer
 * sums do not depend on the order), then rounded once to fp32 (an entry a NaN / inf gate gradient reached is
 * NaN); the parameter gradients summed in a fixed order. `scratch` holds avr_raymarch_bwd_scratch_bytes(n, steps,
 * n_scenes * H*W * 64) bytes (n = n_scenes * n_per_scene; the accumulators, the stored gate gradients and
 * lookups, the workgroups' partials), scratch_bytes its size; lookup_grad 1 =
 * the lookup's position gradient flows into the points (models.py:753-823 with stop_encoder_grad False), 0 = it
 * does not (stop_encoder_grad True detaches the looked-up latent, models.py:810-811: W_ih, the LSTM and
 * out_layer still get theirs, the points only through x += rd * sd).                                          */
int avr_raymarch_train(const avr_view_desc* views, int n_scenes, const float* gate_tables, const float* w_hh,
                       const float* b_ih, const float* b_hh, const float* w_out, const float* b_out, const float* ro,
                       const float* rd, const float* init_dist, int64_t n_per_scene, int steps, float* world,
                       float* trace, float* state, void* stream);
int avr_raymarch_bwd_scratch_bytes(int64_t n_rays, int steps, int64_t table_entries, int64_t* n_bytes);
int avr_raymarch_bwd(const avr_view_desc* views, int n_scenes, const float* gate_tables, const float* w_hh,
                     const float* w_out, const float* rd, const float* trace, const float* state,
                     const float* grad_world, int64_t n_per_scene, int steps, int lookup_grad, float* d_tables,
                     float* d_grads, void* scratch, int64_t scratch_bytes, void* stream);

/* ------------------------------------------------------------ measurement
 * Streaming device copy dst[0, n_bytes) = src[0, n_bytes) (16-B aligned,
 * n_bytes a multiple of 16): the achievable-HBM yardstick bench.py reports
 * every renderer kernel against. Not on the rendering path.      */
int avr_stream_copy(const void* src, void* dst, int64_t n_bytes, void* stream);

/* Streaming device fill: every 32-bit word of dst[0, n_bytes) = word (16-B
 * aligned, n_bytes a multiple of 16): the write-only yardstick (the ceiling
 * of store-dominated kernels such as the stratified sampler). Not on the
 * rendering path (ABI 10).                                                    */
int avr_stream_fill(void* dst, int64_t n_bytes, uint32_t word, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AVR_H_ */
