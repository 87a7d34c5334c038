/* Host-side argument checks of the C ABI (include/avr.h) under AddressSanitizer
 * (SURVEY §5 "Race detection / sanitizers": a host -fsanitize=address build of
 * the library, `make -C adaptive-volume-rendering_amd asan`). Every call below
 * must be rejected (AVR_E_INVALID / AVR_E_UNSUPPORTED) or be a no-op (zero
 * work) BEFORE any HIP call, so the harness runs without a GPU; ASan checks
 * the validation code itself (struct reads, error-string formatting).
 * Exit status: number of failed checks. Run by tests/test_asan_cpu.py.      */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "avr.h"

static int failures = 0;

static void expect(const char* what, int got, int want) {
  if (got != want) {
    fprintf(stderr, "FAIL %s: got %d want %d (%s)\n", what, got, want, avr_last_error_string());
    ++failures;
  } else if (want != AVR_OK && strlen(avr_last_error_string()) == 0) {
    fprintf(stderr, "FAIL %s: no error string\n", what);
    ++failures;
  }
}

static void check(const char* what, int cond) {
  if (!cond) {
    fprintf(stderr, "FAIL %s\n", what);
    ++failures;
  }
}

int main(void) {
  float buf[64] = {0};
  int64_t n = 0;
  check("version", avr_version() == AVR_ABI_VERSION);
  check("device_count>=0", avr_device_count() >= 0);

  /* geometry / sampling */
  expect("world_rays null", avr_world_rays(NULL, NULL, NULL, 0, 0, 1, 4, NULL, NULL, NULL), AVR_E_INVALID);
  expect("world_rays empty", avr_world_rays(NULL, NULL, NULL, 0, 0, 1, 0, NULL, NULL, NULL), AVR_OK);
  expect("depth null", avr_depth_from_world(NULL, NULL, NULL, NULL, 0, 0, 1, 3, NULL, NULL, NULL), AVR_E_INVALID);
  expect("coarse bad n", avr_sample_coarse(0.8f, 1.8f, 4, 0, NULL, 0, 0, NULL, buf, NULL), AVR_E_INVALID);
  expect("coarse neg rays", avr_sample_coarse(0.8f, 1.8f, -1, 8, NULL, 0, 0, NULL, buf, NULL), AVR_E_INVALID);
  expect("coarse null z", avr_sample_coarse(0.8f, 1.8f, 4, 8, NULL, 0, 0, NULL, NULL, NULL), AVR_E_INVALID);
  expect("coarse empty", avr_sample_coarse(0.8f, 1.8f, 0, 8, NULL, 0, 0, NULL, NULL, NULL), AVR_OK);
  expect("rays_coarse null", avr_rays_sample_coarse(NULL, NULL, NULL, 0, 0, 1, 8, 0.8f, 1.8f, 16, NULL, 0, 0, NULL,
                                                    NULL, NULL, NULL, NULL, NULL), AVR_E_INVALID);
  expect("coarse_rays null", avr_sample_coarse_rays(NULL, NULL, 4, 8, NULL, 0, 0, NULL, NULL), AVR_E_INVALID);
  expect("fine null", avr_sample_fine(NULL, NULL, 0.8f, 1.8f, 4, 64, 32, 0, 0.01f, NULL, NULL, NULL, 0, 0, NULL,
                                      NULL, NULL, NULL, NULL), AVR_E_INVALID);
  expect("fine nc too big", avr_sample_fine(buf, buf, 0.8f, 1.8f, 4, 257, 32, 0, 0.01f, NULL, NULL, NULL, 0, 0,
                                            NULL, buf, NULL, NULL, NULL), AVR_E_INVALID);
  expect("fine total too big", avr_sample_fine(buf, buf, 0.8f, 1.8f, 4, 256, 200, 100, 0.01f, NULL, NULL, NULL, 0,
                                               0, NULL, buf, NULL, NULL, NULL), AVR_E_INVALID);
  expect("fine half noise", avr_sample_fine(buf, buf, 0.8f, 1.8f, 4, 64, 32, 0, 0.01f, buf, NULL, NULL, 0, 0, NULL,
                                            buf, NULL, NULL, NULL), AVR_E_INVALID);
  expect("fine empty", avr_sample_fine(NULL, NULL, 0.8f, 1.8f, 0, 64, 32, 0, 0.01f, NULL, NULL, NULL, 0, 0, NULL,
                                       NULL, NULL, NULL, NULL), AVR_OK);

  /* compositing */
  expect("composite null", avr_composite_fwd(NULL, NULL, 4, 8, 1, 1.8f, NULL, NULL, NULL, NULL), AVR_E_INVALID);
  expect("composite_depth null", avr_composite_fwd_depth(NULL, NULL, 4, 8, 1, 1.8f, NULL, NULL, NULL, NULL, NULL,
                                                         NULL, NULL, NULL), AVR_E_INVALID);
  expect("composite_bwd null", avr_composite_bwd(NULL, NULL, 4, 8, 1, 1.8f, NULL, NULL, NULL, NULL, NULL, NULL),
         AVR_E_INVALID);
  expect("march bytes null", avr_march_state_bytes(16, NULL), AVR_E_INVALID);
  expect("march bytes", avr_march_state_bytes(16, &n), AVR_OK);
  check("march bytes >0", n > 0);

  /* field */
  avr_field_dims d;
  memset(&d, 0, sizeof d);
  d.d_in = 42; d.d_latent = 512; d.d_hidden = 384; d.n_blocks = 3; d.n_lin_z = 3; d.num_freqs = 6;
  d.freq_factor = 1.5f; d.precision = AVR_FIELD_X3;
  expect("packed_floats bad hidden", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.d_hidden = 512;
  expect("packed_floats", avr_field_packed_floats(&d, &n), AVR_OK);
  int64_t plain = n;
  d.bn = 1;
  expect("packed_floats bn", avr_field_packed_floats(&d, &n), AVR_OK);
  check("bn adds 2 x d_hidden per block", n - plain == 2 * 512 * 3);
  d.bn = 2;
  expect("packed_floats bad bn", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.bn = 0;
  d.n_blocks = AVR_MAX_BLOCKS + 1;
  expect("packed_floats too many blocks", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.n_blocks = 3;
  d.d_in = 40;
  expect("packed_floats bad d_in", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.d_in = 42;
  expect("packed_floats null out", avr_field_packed_floats(&d, NULL), AVR_E_INVALID);
  avr_resnetfc_weights w;
  memset(&w, 0, sizeof w);
  expect("pack null blob", avr_field_pack(&d, &w, NULL, NULL), AVR_E_INVALID);
  expect("pack null dims", avr_field_pack(NULL, &w, buf, NULL), AVR_E_INVALID);
  avr_view_desc v;
  memset(&v, 0, sizeof v);
  expect("fwd_rays bad latent", avr_field_fwd_rays(&d, &v, buf, buf, NULL, NULL, NULL, 4, 8, NULL, NULL),
         AVR_E_INVALID);
  v.latent_h = v.latent_w = 8;
  expect("fwd_rays null ro", avr_field_fwd_rays(&d, &v, buf, buf, NULL, NULL, NULL, 4, 8, NULL, NULL),
         AVR_E_INVALID);
  expect("fwd_rays empty", avr_field_fwd_rays(&d, &v, buf, buf, NULL, NULL, NULL, 0, 8, NULL, NULL), AVR_OK);
  expect("fwd_points empty", avr_field_fwd_points(&d, &v, buf, buf, NULL, NULL, 0, NULL, NULL), AVR_OK);
  expect("batch too many scenes", avr_field_fwd_rays_batch(&d, &v, AVR_MAX_SCENES + 1, buf, buf, NULL, NULL, NULL,
                                                           4, 8, NULL, NULL), AVR_E_INVALID);
  d.precision = AVR_FIELD_FP32;
  d.bn = 1;
  expect("bn on fp32 rejected", avr_field_fwd_points(&d, &v, buf, buf, buf, buf, 4, buf, NULL), AVR_E_INVALID);
  d.precision = AVR_FIELD_X3;
  expect("bn training rejected", avr_field_fwd_points_train(&d, &v, 1, buf, buf, buf, buf, 4, buf, buf, 4,
                                                            (uint32_t*)buf, NULL, NULL, 0, NULL, NULL), AVR_E_INVALID);
  d.bn = 0;
  expect("train ld_z < d_in", avr_field_fwd_points_train(&d, &v, 1, buf, buf, buf, buf, 4, buf, buf, 4,
                                                         (uint32_t*)buf, NULL, buf, 8, NULL, NULL), AVR_E_INVALID);
  /* use_spade / Softplus (ABI 8): the scale_z fragments and the 2 * n_lin_z table biases; x3 inference only */
  d.spade = 1;
  expect("packed_floats spade", avr_field_packed_floats(&d, &n), AVR_OK);
  /* fp32 scale_z fragments, their x3 fragments (the x3 table kernel, ABI 9) and the table biases */
  check("spade adds scale_z fragments + table biases", n - plain == 2 * 3 * (int64_t)512 * 512 + 6 * 512);
  d.bn = 1;
  expect("spade with bn rejected", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.bn = 0;
  d.spade = 2;
  expect("bad spade", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.spade = 0;
  d.beta = -1.f;
  expect("negative beta", avr_field_packed_floats(&d, &n), AVR_E_INVALID);
  d.beta = 0.f; d.spade = 1;   /* use_spade trains on the module path (Softplus trains on HIP since ABI 11) */
  expect("spade training rejected", avr_field_fwd_points_train(&d, &v, 1, buf, buf, buf, buf, 4, buf, buf, 4,
                                                               (uint32_t*)buf, NULL, NULL, 0, NULL, NULL), AVR_E_INVALID);
  d.spade = 0; d.beta = 2.f;
  expect("softplus backward without act rows", avr_field_bwd(&d, buf, buf, 1, 4, buf, buf, (uint32_t*)buf, NULL, 0,
                                                             buf, 4, NULL, NULL), AVR_E_INVALID);
  d.precision = AVR_FIELD_FP32;
  expect("softplus on fp32 rejected", avr_field_fwd_points(&d, &v, buf, buf, buf, buf, 4, buf, NULL), AVR_E_INVALID);
  d.precision = AVR_FIELD_X3;
  d.beta = 0.f;
  /* NS > 1 split passes */
  d.n_lin_z = 2;
  expect("split bad b_end", avr_field_fwd_points_split(&d, &v, 1, buf, buf, buf, buf, 4, 0, 3, NULL, buf, NULL, NULL),
         AVR_E_INVALID);
  expect("split b_end < n_lin_z", avr_field_fwd_points_split(&d, &v, 1, buf, buf, buf, buf, 4, 0, 1, NULL, buf, NULL,
                                                             NULL), AVR_E_INVALID);
  expect("split first null h_out", avr_field_fwd_points_split(&d, &v, 1, buf, buf, buf, buf, 4, 0, 2, NULL, NULL,
                                                              NULL, NULL), AVR_E_INVALID);
  expect("split second null h_in", avr_field_fwd_points_split(&d, &v, 1, buf, buf, NULL, NULL, 4, 2, 3, NULL, NULL,
                                                               buf, NULL), AVR_E_INVALID);
  expect("split second before n_lin_z", avr_field_fwd_points_split(&d, &v, 1, buf, buf, NULL, NULL, 4, 1, 3, buf,
                                                                    NULL, buf, NULL), AVR_E_INVALID);
  expect("split empty", avr_field_fwd_points_split(&d, &v, 1, buf, buf, NULL, NULL, 0, 2, 3, NULL, NULL, NULL, NULL),
         AVR_OK);
  d.n_lin_z = 3;
  int64_t act = 0, mw = 0;
  expect("train sizes", avr_field_train_sizes(&d, 2, 100, &act, &mw), AVR_OK);
  check("train sizes act", act == (int64_t)7 * 2 * 100 * 512);
  expect("train sizes bad", avr_field_train_sizes(&d, 0, 100, &act, &mw), AVR_E_INVALID);
  expect("latent_table null", avr_field_latent_table(&d, NULL, NULL, 8, 8, NULL, NULL), AVR_E_INVALID);
  expect("wgrad no layers", avr_weight_grads(NULL, 0, 0, 1, NULL), AVR_E_INVALID);
  {
    avr_wgrad_layer wl;
    memset(&wl, 0, sizeof(wl));
    wl.out_dim = 8; wl.in_dim = 8; wl.partial = buf; wl.bias_partial = buf;
    float* dwp[1] = {buf};
    float* dbp[1] = {NULL};
    expect("wgrad reduce no layers", avr_weight_grads_reduce(NULL, 0, 1, dwp, dbp, NULL), AVR_E_INVALID);
    expect("wgrad reduce bad split", avr_weight_grads_reduce(&wl, 1, 0, dwp, dbp, NULL), AVR_E_INVALID);
    expect("wgrad reduce bias without db", avr_weight_grads_reduce(&wl, 1, 1, dwp, dbp, NULL), AVR_E_INVALID);
    expect("wgrad reduce null db list", avr_weight_grads_reduce(&wl, 1, 1, dwp, NULL, NULL), AVR_E_INVALID);
    wl.in_dim = 6;
    expect("wgrad reduce odd dims", avr_weight_grads_reduce(&wl, 1, 1, dwp, dbp, NULL), AVR_E_INVALID);
    wl.in_dim = 8; wl.grad = buf; wl.input = buf; wl.ld_grad = 8; wl.ld_input = 8;
    wl.grad_max = (const uint32_t*)buf; wl.input_max = (const uint32_t*)buf; wl.in_mu = buf;
    expect("wgrad half a BN transform", avr_weight_grads(&wl, 1, 64, 1, NULL), AVR_E_INVALID);
  }
  expect("latent_features null view", avr_latent_features(NULL, NULL, 4, NULL, 3, NULL, NULL), AVR_E_INVALID);
  expect("latent_features_batch too many scenes",
         avr_latent_features_batch(&v, AVR_MAX_SCENES + 1, buf, 4, buf, 3, buf, NULL), AVR_E_INVALID);
  expect("latent_features_batch null", avr_latent_features_batch(&v, 1, NULL, 4, buf, 3, buf, NULL), AVR_E_INVALID);
  expect("latent_features_batch odd channels", avr_latent_features_batch(&v, 1, buf, 6, buf, 3, buf, NULL),
         AVR_E_INVALID);
  expect("latent_grad_points too many scenes",
         avr_latent_features_grad_points(&v, AVR_MAX_SCENES + 1, buf, 4, buf, 3, buf, buf, NULL), AVR_E_INVALID);
  expect("latent_grad_points null", avr_latent_features_grad_points(&v, 1, buf, 4, buf, 3, NULL, buf, NULL),
         AVR_E_INVALID);
  expect("latent_grad_points empty", avr_latent_features_grad_points(&v, 1, buf, 4, buf, 0, buf, buf, NULL), AVR_OK);
  expect("zfeature_grad_points scenes", avr_zfeature_grad_points(&v, 0, buf, 3, buf, 39, 6, 3.14159f, 0, buf, NULL),
         AVR_E_INVALID);
  expect("zfeature_grad_points ld", avr_zfeature_grad_points(&v, 1, buf, 3, buf, 38, 6, 3.14159f, 0, buf, NULL),
         AVR_E_INVALID);
  expect("zfeature_grad_points null", avr_zfeature_grad_points(&v, 1, buf, 3, NULL, 39, 6, 3.14159f, 1, buf, NULL),
         AVR_E_INVALID);
  expect("lin_out_act_bwd null", avr_lin_out_act_bwd_rows(4, buf, NULL, buf, NULL, NULL), AVR_E_INVALID);
  expect("lin_out_act_bwd rows", avr_lin_out_act_bwd_rows(-1, buf, buf, buf, NULL, NULL), AVR_E_INVALID);
  expect("lin_out_act_bwd empty", avr_lin_out_act_bwd_rows(0, NULL, NULL, NULL, NULL, NULL), AVR_OK);
  expect("zfeature_grad_points empty", avr_zfeature_grad_points(&v, 1, buf, 0, buf, 39, 6, 3.14159f, 0, buf, NULL),
         AVR_OK);
  expect("latent_table_batch null", avr_field_latent_table_batch(&d, NULL, NULL, 2, 8, 8, NULL, NULL), AVR_E_INVALID);
  expect("latent_table_batch no scenes", avr_field_latent_table_batch(&d, buf, buf, 0, 8, 8, buf, NULL),
         AVR_E_INVALID);
  expect("raymarch null", avr_raymarch(NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 4, 10, NULL, NULL,
                                       NULL, NULL), AVR_E_INVALID);

  /* training-mode BatchNorm (ABI 11): argument checks, no launch */
  d.d_hidden = 512; d.bn = 0; d.spade = 0; d.beta = 0.f; d.precision = AVR_FIELD_X3;
  {
    avr_bn_layer l;
    memset(&l, 0, sizeof l);
    l.n_rows = 100; l.mode = AVR_BN_FWD; l.prologue = AVR_BN_PLAIN; l.in_dim = 512; l.in_valid = 512;
    l.src = buf; l.ld_src = 512; l.blob = buf; l.layer = 2; l.out = buf; l.partial = buf;
    expect("bn_layer null layer", avr_bn_layer_run(&d, NULL, NULL), AVR_E_INVALID);
    l.mode = 7;
    expect("bn_layer bad mode", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.mode = AVR_BN_FWD; l.in_dim = 96;
    expect("bn_layer bad in_dim", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.in_dim = 512; l.ld_src = 510;
    expect("bn_layer bad ld", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.ld_src = 512; l.prologue = AVR_BN_RELU;
    expect("bn_layer relu without stats", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.prologue = AVR_BN_PLAIN; l.layer = 2 + 2 * d.n_blocks;
    expect("bn_layer bad layer", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.layer = 2; l.mode = AVR_BN_BWD;
    expect("bn_layer bwd without pre rows", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.mode = AVR_BN_FWD; l.lin_z_table = buf; l.n_views = 1; l.rows_per_scene = 100;
    expect("bn_layer lin_z without points", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.xyz = buf; l.views = &v; l.rows_per_scene = 50;
    expect("bn_layer lin_z rows", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    l.lin_z_table = NULL; l.xyz = NULL; l.views = NULL; l.n_views = 0; l.rows_per_scene = 0;
    d.bn = 1;
    expect("bn_layer folded blob", avr_bn_layer_run(&d, &l, NULL), AVR_E_INVALID);
    d.bn = 0; l.n_rows = 0;
    expect("bn_layer empty", avr_bn_layer_run(&d, &l, NULL), AVR_OK);
  }
  expect("bn_stats one row", avr_bn_stats(buf, 1, 512, buf, 1e-5f, 0.1f, NULL, NULL, buf, buf, buf, NULL),
         AVR_E_INVALID);
  expect("bn_stats half running", avr_bn_stats(buf, 8, 512, buf, 1e-5f, 0.1f, buf, NULL, buf, buf, buf, NULL),
         AVR_E_INVALID);
  expect("bn_grad_stats null", avr_bn_grad_stats(buf, 8, 512, NULL, buf, buf, buf, buf, buf, buf, NULL), AVR_E_INVALID);
  expect("bn_grad_rows odd cols", avr_bn_grad_rows(8, 6, buf, buf, NULL, buf, buf, buf, buf, buf, buf, NULL, NULL),
         AVR_E_INVALID);
  expect("bn_grad_rows empty", avr_bn_grad_rows(0, 8, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL),
         AVR_OK);
  /* LSTM march training (ABI 11) */
  expect("raymarch_train too many scenes",
         avr_raymarch_train(&v, AVR_MAX_SCENES + 1, buf, buf, buf, buf, buf, buf, buf, buf, buf, 4, 10, buf, buf, buf,
                            NULL), AVR_E_INVALID);
  expect("raymarch_train null", avr_raymarch_train(&v, 1, buf, NULL, buf, buf, buf, buf, buf, buf, buf, 4, 10, buf, buf,
                                                   buf, NULL), AVR_E_INVALID);
  expect("raymarch_bwd null", avr_raymarch_bwd(&v, 1, buf, buf, buf, buf, buf, buf, NULL, 4, 10, 1, buf, buf,
                                               buf, 1 << 20, NULL), AVR_E_INVALID);
  expect("raymarch_bwd no scratch", avr_raymarch_bwd(&v, 1, buf, buf, buf, buf, buf, buf, buf, 4, 10, 1, buf,
                                                     buf, NULL, 1 << 20, NULL), AVR_E_INVALID);
  expect("raymarch_bwd scratch too small", avr_raymarch_bwd(&v, 1, buf, buf, buf, buf, buf, buf, buf, 4, 10, 1, buf,
                                                            buf, buf, 64, NULL), AVR_E_INVALID);
  expect("raymarch_bwd no steps", avr_raymarch_bwd(&v, 1, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 4, 0, 1, NULL,
                                                   NULL, NULL, 0, NULL), AVR_OK);
  {
    /* ABI 15: int64 accumulators (8 B per table entry), dg rows (64 floats per ray step), lookups (8 floats per
       ray step), 3 workgroups' partials, the control words; each region rounded up to 256 B */
    int64_t nb = 0;
    expect("raymarch_bwd scratch size", avr_raymarch_bwd_scratch_bytes(33, 10, 4096, &nb), AVR_OK);
    check("raymarch_bwd scratch layout", nb == 32768 + 84480 + 10752 + 13312 + 256);
    expect("raymarch_bwd scratch bad", avr_raymarch_bwd_scratch_bytes(-1, 10, 4096, &nb), AVR_E_INVALID);
  }

  /* measurement */
  expect("copy odd size", avr_stream_copy(buf, buf + 8, 15, NULL), AVR_E_INVALID);
  expect("copy null", avr_stream_copy(NULL, buf, 16, NULL), AVR_E_INVALID);
  expect("copy empty", avr_stream_copy(NULL, NULL, 0, NULL), AVR_OK);
  expect("fill odd size", avr_stream_fill(buf, 15, 0u, NULL), AVR_E_INVALID);
  expect("fill null", avr_stream_fill(NULL, 16, 0u, NULL), AVR_E_INVALID);
  expect("fill empty", avr_stream_fill(NULL, 0, 0u, NULL), AVR_OK);

  printf("abi_check: %d failure(s)\n", failures);
  return failures;
}
