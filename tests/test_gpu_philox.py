"""The benchmarked noise path pinned to the oracle.

bench.py renders with `VolumeRenderer.seed` set: the ray / sampling kernels
draw their noise in-kernel (Philox4x32-10 keyed by (seed, offset + frame ray
id, sample block, stream)) instead of reading torch.rand tensors. These tests
restate those draws on the CPU (oracle/philox.py, pinned to the Random123
known-answer vectors by tests/test_philox_cpu.py), feed them to the numpy
oracle and compare:
  * the sampling kernels alone in Philox mode, over seeds / offsets / 64-bit
    counters / frame ray ids / ragged and > 64 sample counts: coarse z, fine
    bins and fine z bit-exact, depth samples through the clamp;
  * BASELINE config 3 exactly as bench.py runs it (the bench's synthetic
    scene, seed 1234, x_pix from generator 100, orbit pose 0.7, 65 536 rays x
    (128 + 64)) through the drop-in VolumeRenderer, checked on 4 096 rays with
    the renderers.py:133-277 protocol of tests/test_gpu_scale.py: coarse z
    bit-exact, fine bins / fine z / merge bit-exact given the HIP weights,
    every ray's rgb / depth <= 1e-4 against the oracle's fine pass on the
    same samples, and end to end every outlier a bin flip (fp32 noise in the
    coarse weights moving a fine sample across a cdf step, quirk Q3).
"""
import functools

import numpy as np
import pytest
import torch

from helpers import oracle_field_from_net, to_np
from oracle import avr_oracle as O
from oracle import philox as P
from oracle import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None

R3, NC, NF = 65536, 128, 64
SUB = slice(0, R3, 16)           # 4 096 rays spread over the batch
SEED = 1234                      # bench.py: rend.seed = 1234 + rank


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


@pytest.mark.parametrize("seed,offset,n,ids", [(1234, 0, 128, False), (7, 5, 30, False), ((1 << 40) + 3, (1 << 33) + 11, 64, True),
                                               (0, 0, 1, False), (99, 12, 100, True)])
def test_sample_coarse_philox_bit_exact(seed, offset, n, ids):
    from avr import ops
    R = 777
    ray_ids = np.random.default_rng(seed % 1000).permutation(5 * R)[:R].astype(np.int64) if ids else None
    z = ops.sample_coarse(0.8, 1.8, R, n, DEV, seed=seed, offset=offset,
                          ray_ids=None if ray_ids is None else T(ray_ids))
    u = P.coarse_noise(seed, P.ray_keys(R, offset, ray_ids), n)
    want = O.sample_coarse(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), n, u[None])[0]
    np.testing.assert_array_equal(to_np(z), want)


@pytest.mark.parametrize("n", [128, 64, 30])
def test_rays_sample_coarse_philox_bit_exact(n):
    """The fused ray + stratified-z kernel the renderer launches (rays_coarse_kernel)."""
    from avr import ops
    R = 1000
    x_pix = np.random.default_rng(1).random((1, R, 2), dtype=np.float32)
    c2w = synth.orbit_cam2world(0.7)
    ro, rd, z, _, _ = ops.rays_sample_coarse(T(x_pix), T(synth.default_intrinsics())[None],
                                             T(c2w).reshape(1, 1, 4, 4).expand(1, R, 4, 4), 0.8, 1.8, n, seed=SEED,
                                             offset=3)
    u = P.coarse_noise(SEED, P.ray_keys(R, 3), n)
    want = O.sample_coarse(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), n, u[None])[0]
    np.testing.assert_array_equal(to_np(z), want)


@pytest.mark.parametrize("nc,nf,nd,std", [(128, 64, 0, 0.01), (64, 16, 16, 0.01), (32, 100, 0, 0.01),
                                          (64, 32, 8, 1.5)])
def test_sample_fine_philox_bit_exact(nc, nf, nd, std):
    """Bins and fine z bit-exact against the oracle fed the restated (u, u2);
    the merged list equals the oracle's sort of [z_c | z_f | clamp(randn*std)]
    (depth draws compared through the clamp: exactly `near` at std 0.01,
    quirk Q6; within 1e-5 where std 1.5 lands some inside [near, far])."""
    from avr import ops
    R, seed, offset = 1500, 4321, 77
    rng = np.random.default_rng(nc + nf)
    w = rng.random((R, nc), dtype=np.float32) ** 4
    w[::7] = 0.0                                    # all-zero rows: uniform pdf
    zc = P.coarse_noise(5, P.ray_keys(R), nc)
    zc = O.sample_coarse(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), nc, zc[None])[0]
    zs, idx, zf = ops.sample_fine(T(w), T(zc), 0.8, 1.8, nf, nd, std, seed=seed, offset=offset, want_idx=True,
                                  want_fine=True)
    keys = P.ray_keys(R, offset)
    u, u2 = P.fine_noise(seed, keys, nf)
    zf_o, idx_o = O.sample_fine(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), nf,
                                w[None, ..., None], u[None], u2[None], return_idx=True)
    np.testing.assert_array_equal(to_np(idx), idx_o[0])
    np.testing.assert_array_equal(to_np(zf), zf_o[0])
    zd = np.clip(P.depth_normal(seed, keys, nd) * np.float32(std), np.float32(0.8), np.float32(1.8)).astype(np.float32)
    want = np.sort(np.concatenate([zc, zf_o[0], zd], -1), -1)
    if std <= 0.01:
        assert (zd == np.float32(0.8)).all()
        np.testing.assert_array_equal(to_np(zs), want)
    else:
        assert ((zd > 0.8) & (zd < 1.8)).any()
        np.testing.assert_allclose(to_np(zs), want, atol=1e-5, rtol=0)


# ---------------------------------------------------------------- BASELINE config 3, as bench.py runs it
@functools.lru_cache(maxsize=1)
def _bench_scene():
    from avr.scene import synthetic_scene
    net = synthetic_scene(DEV)                                   # bench.py build_scene(device)
    g = torch.Generator(device="cpu").manual_seed(100)           # bench.py x_pix, rank 0
    x_pix = torch.rand(1, R3, 2, generator=g)
    return net, x_pix.numpy()


@functools.lru_cache(maxsize=1)
def _c3_philox_oracle():
    """O.render on the SUB rays with the restated Philox draws of those rays."""
    net, x_pix = _bench_scene()
    field = oracle_field_from_net(net)
    from bench import orbit_c2w
    c2w1 = orbit_c2w(0.7).numpy()
    K = synth.default_intrinsics()[None]
    ids = np.arange(R3)[SUB]
    draws = P.renderer_draws(SEED, R3, NC, NF, 0)                # frame ray ids 0..R-1, offset 0 (first call)
    xs = x_pix[:, SUB]
    ns = {k: v[:, SUB] for k, v in draws.items()}
    assert ns["coarse"].shape[1] == ids.size
    parts = []
    for a in range(0, ids.size, 512):
        b = min(ids.size, a + 512)
        parts.append(O.render(np.broadcast_to(c2w1, (1, b - a, 4, 4)), K, xs[:, a:b], field, 0.8, 1.8, NC, NF, 0,
                              0.01, True, ns["coarse"][:, a:b], ns["u"][:, a:b], ns["u2"][:, a:b],
                              ns["depth"][:, a:b], return_aux=True))
    cat = lambda i: np.concatenate([p[i] for p in parts], 1)  # noqa: E731
    aux = {k: np.concatenate([p[4][k] for p in parts], 1) for k in parts[0][4]}
    return cat(0), cat(1), cat(2), aux, ns


def _record(entry):
    """Append one JSON line to $AVR_TEST_REPORT (default gpurun_out/philox_c3_flip_rates.jsonl): the measured
    flip rates of the benchmarked path, kept under profiles/ per round."""
    import json
    import os
    path = os.environ.get("AVR_TEST_REPORT", os.path.join("gpurun_out", "philox_c3_flip_rates.jsonl"))
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(entry) + "\n")


@pytest.mark.parametrize("precision", ["x3", "fp32"])
def test_c3_philox_bench_path_vs_oracle(precision):
    """BASELINE config 3 exactly as bench.py runs it, at both field precisions: the bin-flip rate of the fog
    scene against the oracle is written to $AVR_TEST_REPORT for profiles/."""
    net, x_pix_np = _bench_scene()
    net.field_precision = precision
    try:
        _c3_philox_check(net, x_pix_np, precision)
    finally:
        net.field_precision = "x3"


def _c3_philox_check(net, x_pix_np, precision):
    from avr import ops
    from avr.renderers import VolumeRenderer
    from bench import orbit_c2w
    x_pix = T(x_pix_np)
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]], device=DEV)
    c2w = orbit_c2w(0.7).to(DEV).reshape(1, 1, 4, 4).expand(1, R3, 4, 4)
    rend = VolumeRenderer(0.8, 1.8, NC, NF, 0, 0.01, True)       # bench.py main()
    rend.seed = SEED                                             # bench.py main(): 1234 + rank
    with torch.no_grad():
        r_c, r_f, r_d, _ = rend(c2w, K, x_pix, net)
        # the same chain stage by stage (offset 0 = the renderer's first call)
        fused = net.fused()
        ro, rd, zc, _, info = ops.rays_sample_coarse(x_pix, K, c2w, 0.8, 1.8, NC, seed=SEED, offset=0)
        fc = fused.forward_rays(ro[0], rd[0], zc, True).reshape(R3, NC, 4)
        rgb_c, _, w_c = ops.composite(zc, fc)
        zs, idx, zf = ops.sample_fine(w_c, zc, 0.8, 1.8, NF, 0, 0.01, seed=SEED, offset=0, want_idx=True,
                                      want_fine=True)
        ff = fused.forward_rays(ro[0], rd[0], zs, False).reshape(R3, NC + NF, 4)
        rgb_f, dist_f, _ = ops.composite(zs, ff, want_weights=False)
        depth = ops.depth_from_world(ro, rd, dist_f.reshape(1, R3), info)
    torch.cuda.synchronize()
    assert rend.last_path == "fused"
    np.testing.assert_array_equal(to_np(r_c[0]), to_np(rgb_c))
    np.testing.assert_array_equal(to_np(r_f[0]), to_np(rgb_f))
    np.testing.assert_allclose(to_np(r_d), to_np(depth), atol=1e-6, rtol=0)   # epilogue vs depth kernel
    o_c, o_f, o_d, aux, ns = _c3_philox_oracle()
    S = SUB
    np.testing.assert_array_equal(to_np(ro[0, S]), aux["ro"][0])
    np.testing.assert_allclose(to_np(rd[0, S]), aux["rd"][0], atol=2e-7, rtol=0)
    np.testing.assert_array_equal(to_np(zc[S]), aux["z_coarse"][0])            # in-kernel draws = restated draws
    np.testing.assert_allclose(to_np(fc[S]), aux["field_coarse"][0], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(to_np(rgb_c[S]), o_c[0], atol=1e-4, rtol=0)
    w_h = to_np(w_c[S])[None, ..., None]
    n = w_h.shape[1]
    zf_o, idx_o = O.sample_fine(np.full((1, n), 0.8, np.float32), np.full((1, n), 1.8, np.float32), NF, w_h,
                                ns["u"], ns["u2"], return_idx=True)
    np.testing.assert_array_equal(to_np(idx[S]), idx_o[0])
    np.testing.assert_array_equal(to_np(zf[S]), zf_o[0])
    np.testing.assert_array_equal(to_np(zs[S]), np.sort(np.concatenate([to_np(zc[S]), zf_o[0]], -1), -1))
    same = (to_np(idx[S]) == aux["idx"][0]).all(-1)
    # the bench scene's random-init fog puts ~0.2 % of rays within fp32 noise of a cdf step (quirk Q3): those
    # rays take other fine bins than the oracle's own weights give; the oracle's fine pass on the HIP-chosen
    # samples (bins bit-exact above) must then match them like every other ray
    flips = np.flatnonzero(~same)
    sample_same = float((to_np(idx[S]) == aux["idx"][0]).mean())
    print(f"philox C3 {precision}: rays with the oracle's bins {same.mean():.5f} ({flips.size} bin flips)")
    assert same.mean() >= 0.985, same.mean()   # r04b: 0.9915 (x3) / 0.9917 (fp32) of rays keep all 64 bins
    np.testing.assert_allclose(to_np(ff[S])[same], aux["field_fine"][0][same], atol=5e-5, rtol=1e-4)
    rgb_ref, depth_ref = o_f[0].copy(), o_d[0].copy()
    if flips.size:
        field = oracle_field_from_net(net)
        c2w1 = orbit_c2w(0.7).numpy()
        zs_h = to_np(zs[S])[flips][None]
        ro_o, rd_o = aux["ro"][:, flips], aux["rd"][:, flips]
        pts = ro_o[..., None, :] + rd_o[..., None, :] * zs_h[..., None]
        vd = np.broadcast_to(rd_o[..., None, :], pts.shape)
        ff_o = field(pts.reshape(1, -1, 3), vd.reshape(1, -1, 3), coarse=False).reshape(1, flips.size, -1, 4)
        rgb_o, dist_o, _ = O.volume_integral(zs_h, ff_o[..., 3:4], ff_o[..., :3], True)
        rgb_ref[flips] = rgb_o[0]
        depth_ref[flips] = O.depth_from_world(ro_o + rd_o * dist_o, np.broadcast_to(c2w1, (1, flips.size, 4, 4)))[0]
    # staged: every ray within 1e-4 of the oracle's fine pass on the same samples
    staged = (np.abs(to_np(r_f[0, S]) - rgb_ref).max(-1) <= 1e-4) & (np.abs(to_np(r_d[0, S]) - depth_ref) <= 1e-4)
    assert staged.all(), staged.mean()
    # end to end against the pure oracle: an outlier only where the bins flipped
    ok = (np.abs(to_np(r_f[0, S]) - o_f[0]).max(-1) <= 1e-4) & (np.abs(to_np(r_d[0, S]) - o_d[0]) <= 1e-4)
    print(f"philox C3 {precision}: end-to-end within 1e-4 on {ok.mean():.5f} of rays")
    # the coarse field's accuracy against float64 (oracle/field64.py) next to the reference-order fp32 oracle's:
    # this random-init fog is ill-conditioned in fp32 (the fp32 lookup projection alone moves sigma by ~8e-5,
    # profiles/r05c_field_error_attribution.txt), so the HIP-vs-oracle distance is two fp32 errors, not a bias
    from oracle.field64 import field64
    n64 = 256
    sd = {k: v.detach().double().cpu().numpy() for k, v in net.mlp_coarse.state_dict().items()}
    ro_o, rd_o, zc_o = aux["ro"][0, :n64], aux["rd"][0, :n64], aux["z_coarse"][0, :n64]
    pts = (ro_o[:, None, :] + rd_o[:, None, :] * zc_o[..., None]).astype(np.float32).reshape(-1, 3)
    vdir = np.broadcast_to(rd_o[:, None, :], (n64, NC, 3)).reshape(-1, 3)
    f64 = field64(sd, to_np(net.encoder.latent[0]), to_np(net.poses[0]), to_np(net.focal[0]), to_np(net.c[0]),
                  to_np(net.image_shape), to_np(net.encoder.latent_scaling), pts, vdir,
                  n_blocks=net.mlp_coarse.n_blocks, combine_layer=net.mlp_coarse.combine_layer)
    e_hip = float(np.abs(to_np(fc[S])[:n64].reshape(-1, 4).astype(np.float64) - f64).max())
    e_ora = float(np.abs(aux["field_coarse"][0][:n64].reshape(-1, 4).astype(np.float64) - f64).max())
    print(f"philox C3 {precision}: coarse field vs float64: HIP {e_hip:.2e}, reference-order oracle {e_ora:.2e}")
    assert e_hip <= 1.5 * e_ora, (e_hip, e_ora)
    _record({"test": "test_c3_philox_bench_path_vs_oracle", "precision": precision, "rays": int(same.size),
             "coarse_field_err_vs_float64": e_hip, "oracle_coarse_field_err_vs_float64": e_ora,
             "rays_with_oracle_bins": float(same.mean()), "bin_flip_rays": int(flips.size),
             "fine_samples_with_oracle_bin": sample_same, "end_to_end_within_1e-4": float(ok.mean()),
             "outliers": int((~ok).sum()), "outliers_not_bin_flips": int((~ok & same).sum()),
             "max_coarse_field_err": float(np.abs(to_np(fc[S]) - aux["field_coarse"][0]).max()),
             "max_coarse_rgb_err": float(np.abs(to_np(rgb_c[S]) - o_c[0]).max())})
    # bar: the survey's >= 99.9 % is out of reach for ANY fp32 field on this random-init fog scene -- the strict
    # fp32 kernel flips as many rays as x3 (r04b: fp32 34 / 4096 bin-flip rays, 6 outliers = 0.99854; x3 35 and 8
    # = 0.99805; profiles/r04b_philox_c3_flip_rates.jsonl): the flips are fp32 noise of the coarse weights against
    # the numpy oracle's own fp32 field at cdf steps (quirk Q3), not a cost of the split-fp16 products. Both
    # precisions are held to 0.997 with every outlier a bin flip.
    assert ok.mean() >= 0.997, ok.mean()
    assert not (~ok & same).any(), "a ray with the oracle's bins must match it"
    assert np.abs(to_np(r_c[0, S]) - o_c[0]).max() <= 1e-4
