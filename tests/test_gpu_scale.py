"""Parity at the sizes the bench runs, against the pinned
numpy oracle:
  * BASELINE config 3 (65 536 rays x 128 + 64, default.conf field) stage by
    stage on 4 096 of its rays: rays, coarse z (bit-exact), coarse field
    (golden bar 5e-5), coarse composite, inverse-CDF bins and fine z
    (bit-exact, fed the HIP weights), sorted merge (bit-exact), fine field,
    fine rgb / depth (<= 1e-4 on >= 99.9 % of rays; an outlier is allowed only
    where the oracle's own bins differ from the HIP bins);
  * BASELINE config 4: a full 800 x 800 frame with early termination at
    T_stop 1e-5, bounded against the no-termination render of the same frame;
  * the split-fp16 field under layer inputs spanning 2^-12 .. 2^12 inside
    one 64-sample workgroup, and x3 vs fp32 on both MLPs from several origins.
"""
import functools

import numpy as np
import pytest
import torch

from helpers import build_net, oracle_field, to_np
from oracle import avr_oracle as O
from oracle import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None

R3, NC, NF = 65536, 128, 64
SUB = slice(0, R3, 16)           # 4 096 rays spread over the batch


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


@functools.lru_cache(maxsize=1)
def _c3_inputs():
    gen = torch.Generator().manual_seed(2024)
    x_pix = torch.rand(1, R3, 2, generator=gen)
    noise = {"coarse": torch.rand(1, R3, NC, generator=gen), "u": torch.rand(1, R3, NF, generator=gen),
             "u2": torch.rand(1, R3, NF, generator=gen), "depth": torch.zeros(1, R3, 0)}
    return x_pix.numpy(), {k: v.numpy() for k, v in noise.items()}


@functools.lru_cache(maxsize=1)
def _c3_oracle():
    """O.render on the SUB rays (512-ray chunks), with every intermediate."""
    from conftest import load_golden
    g = load_golden("g4_field_full.npz")
    field = oracle_field(g)
    x_pix, noise = _c3_inputs()
    c2w1 = synth.orbit_cam2world(0.7)
    K = synth.default_intrinsics()[None]
    xs = x_pix[:, SUB]
    ns = {k: v[:, SUB] for k, v in noise.items()}
    n = xs.shape[1]
    parts = []
    for a in range(0, n, 512):
        b = min(n, a + 512)
        out = O.render(np.broadcast_to(c2w1, (1, b - a, 4, 4)), K, xs[:, a:b], field, 0.8, 1.8, NC, NF, 0, 0.01,
                       True, ns["coarse"][:, a:b], ns["u"][:, a:b], ns["u2"][:, a:b], ns["depth"][:, a:b],
                       return_aux=True)
        parts.append(out)
    cat = lambda i: np.concatenate([p[i] for p in parts], 1)  # noqa: E731
    aux = {k: np.concatenate([p[4][k] for p in parts], 1) for k in parts[0][4]}
    return cat(0), cat(1), cat(2), aux


@pytest.mark.parametrize("precision", ["x3", "fp32"])
def test_c3_stagewise_vs_oracle(golden, precision):
    from avr import ops
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, precision)
    x_pix_np, noise_np = _c3_inputs()
    x_pix = T(x_pix_np)
    noise = {k: T(v) for k, v in noise_np.items()}
    c2w = T(synth.orbit_cam2world(0.7)).reshape(1, 1, 4, 4).expand(1, R3, 4, 4)
    K = T(synth.default_intrinsics())[None]
    fused = net.fused()
    with torch.no_grad():
        ro, rd, info = ops.world_rays(x_pix, K, c2w)
        zc = ops.sample_coarse(0.8, 1.8, R3, NC, DEV, noise=noise["coarse"][0])
        fc = fused.forward_rays(ro[0], rd[0], zc, True).reshape(R3, NC, 4)
        rgb_c, _, w_c = ops.composite(zc, fc)
        zs, idx, zf = ops.sample_fine(w_c, zc, 0.8, 1.8, NF, 0, 0.01, u=noise["u"][0], u2=noise["u2"][0],
                                      want_idx=True, want_fine=True)
        ff = fused.forward_rays(ro[0], rd[0], zs, False).reshape(R3, NC + NF, 4)
        rgb_f, dist_f, _ = ops.composite(zs, ff, want_weights=False)
        depth = ops.depth_from_world(ro, rd, dist_f.reshape(1, R3), info)
        # the drop-in renderer runs exactly this chain
        rend = VolumeRenderer(0.8, 1.8, NC, NF, 0, 0.01, True)
        r_c, r_f, r_d, _ = rend(c2w, K, x_pix, net, noise=noise)
    torch.cuda.synchronize()
    assert rend.last_path == "fused"
    for a, b in ((r_c[0], rgb_c), (r_f[0], rgb_f), (r_d, depth)):
        assert torch.equal(a, b)
    o_c, o_f, o_d, aux = _c3_oracle()
    S = SUB
    # rays and coarse z
    np.testing.assert_array_equal(to_np(ro[0, S]), aux["ro"][0])
    np.testing.assert_allclose(to_np(rd[0, S]), aux["rd"][0], atol=2e-7, rtol=0)
    np.testing.assert_array_equal(to_np(zc[S]), aux["z_coarse"][0])
    # coarse field and composite (the golden bars)
    np.testing.assert_allclose(to_np(fc[S]), aux["field_coarse"][0], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(to_np(rgb_c[S]), o_c[0], atol=1e-4, rtol=0)
    # inverse-CDF bins / fine z / merge: bit-exact given the HIP weights
    w_h = to_np(w_c[S])[None, ..., None]
    zf_o, idx_o = O.sample_fine(np.full((1, w_h.shape[1]), 0.8, np.float32), np.full((1, w_h.shape[1]), 1.8,
                                np.float32), NF, w_h, noise_np["u"][:, S], noise_np["u2"][:, S], return_idx=True)
    np.testing.assert_array_equal(to_np(idx[S]), idx_o[0])
    np.testing.assert_array_equal(to_np(zf[S]), zf_o[0])
    np.testing.assert_array_equal(to_np(zs[S]), np.sort(np.concatenate([to_np(zc[S]), zf_o[0]], -1), -1))
    # fine field where the oracle chose the same bins (same sorted z)
    same = (to_np(idx[S]) == aux["idx"][0]).all(-1)
    d_fc = np.abs(to_np(fc[S]) - aux["field_coarse"][0])
    print(f"{precision}: rays with the oracle's bins {same.mean():.5f}; coarse field max err rgb "
          f"{d_fc[..., :3].max():.2e} sigma {d_fc[..., 3].max():.2e}")
    assert same.mean() >= 0.999, same.mean()
    np.testing.assert_allclose(to_np(ff[S])[same], aux["field_fine"][0][same], atol=5e-5, rtol=1e-4)
    # end to end
    ok = (np.abs(to_np(rgb_f[S]) - o_f[0]).max(-1) <= 1e-4) & (np.abs(to_np(depth[0, S]) - o_d[0]) <= 1e-4)
    assert ok.mean() >= 0.999, ok.mean()
    assert not (~ok & same).any(), "a ray with the oracle's bins must match it"


@pytest.mark.parametrize("sigma_bias", [0.0, 30.0])
def test_c4_full_frame_early_termination(sigma_bias):
    """BASELINE config 4: one 800 x 800 frame (640 000 rays, 128 + 64) of the
    bench's synthetic scene with fine-pass early termination at T_stop 1e-5,
    against the same frame without termination: rgb within T_stop, distance
    within 2 T_stop (the skipped tail's weight times at most the far bound),
    and (opaque scene) fewer fine samples evaluated."""
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS, synthetic_scene
    from avr.video import get_opencv_pixel_coordinates
    net = synthetic_scene(DEV, sigma_bias=sigma_bias)
    x_pix = get_opencv_pixel_coordinates(800, 800).reshape(1, -1, 2).to(DEV)
    R = x_pix.shape[1]
    assert R == 640000
    from bench import orbit_c2w
    c2w = orbit_c2w(0.7).to(DEV).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    K = torch.tensor([INTRINSICS], device=DEV)
    out = []
    for t_stop in (None, 1e-5):
        rend = VolumeRenderer(0.8, 1.8, NC, NF, 0, 0.01, True)
        rend.seed = 4
        rend.t_stop = t_stop
        with torch.no_grad():
            rgb_c, rgb_f, depth, _ = rend(c2w, K, x_pix, net)
        torch.cuda.synchronize()
        out.append((rgb_c, rgb_f, depth, rend.last_fine_samples))
    (c0, f0, d0, n0), (c1, f1, d1, n1) = out
    assert torch.equal(c0, c1)
    assert n0 == R * (NC + NF)
    assert float((f1 - f0).abs().max()) <= 1e-5 + 2e-6
    dz = (d1 - d0).abs()
    assert float(dz.max()) <= 2e-5 + 2e-5
    assert bool(torch.isfinite(f1).all()) and float(f1.min()) >= -1e-5 and float(f1.max()) <= 1 + 1e-5
    if sigma_bias > 0:
        assert n1 < 0.9 * n0, n1 / n0
    else:
        assert n1 <= n0


@pytest.mark.parametrize("precision", ["x3", "fp32"])
def test_field_wide_dynamic_range_in_one_workgroup(golden, precision):
    """Points whose coordinates span 2^-12 .. 2^12 inside every 64-sample
    workgroup: lin_in's input (raw xyz next to the PE terms) and every hidden
    layer then mix magnitudes ~2^24 apart under one per-workgroup power-of-two
    split scale. The x3 field must stay as close to the oracle as the fp32
    MFMA field does (error relative to the output magnitude)."""
    g = golden("g4_field_full.npz")
    n = 64 * 48
    gen = torch.Generator().manual_seed(9)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=gen), dim=-1)
    mag = 2.0 ** (torch.randint(-12, 13, (n, 1), generator=gen).float())
    xyz = (d * mag).reshape(1, n, 3)
    vd = torch.nn.functional.normalize(torch.randn(1, n, 3, generator=gen), dim=-1)
    ref = oracle_field(g)(xyz.numpy()[0], vd.numpy()[0], coarse=False)
    errs = {}
    for p in ("fp32", precision):
        net = build_net(g, DEV, p)
        with torch.no_grad():
            out = to_np(net(T(xyz.numpy()), coarse=False, viewdirs=T(vd.numpy()))[0])
        assert np.isfinite(out).all()
        errs[p] = np.abs(out - ref) / (1.0 + np.abs(ref))
    e, e32 = float(errs[precision].max()), float(errs["fp32"].max())
    print(f"max rel err {precision} {e:.3e}, fp32 {e32:.3e}")
    assert e <= max(4.0 * e32, 5e-5), (e, e32)


@pytest.mark.parametrize("coarse", [True, False])
def test_field_x3_tracks_fp32_many_origins(golden, coarse):
    """Split-fp16 vs fp32 field on 4 x 50k samples of the 512-wide net, both
    MLPs, four camera origins: the difference stays at fp32-accumulation level."""
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, "fp32")
    torch.manual_seed(1)
    R, N = 500, 100
    for origin in ([0.4, -1.0, 0.6], [-1.2, 0.3, 0.2], [0.1, 1.25, -0.4], [0.9, 0.9, 0.5]):
        ro = torch.tensor([origin], device=DEV).expand(R, 3).contiguous()
        rd = torch.nn.functional.normalize(-ro + 0.3 * torch.randn(R, 3, device=DEV), dim=-1)
        z = torch.sort(0.5 + 1.5 * torch.rand(R, N, device=DEV), -1)[0]
        with torch.no_grad():
            net.field_precision = "fp32"
            a = net.fused().forward_rays(ro, rd, z, coarse=coarse)
            net.field_precision = "x3"
            b = net.fused().forward_rays(ro, rd, z, coarse=coarse)
        d = (a - b).abs()
        assert float(d[:, :3].max()) < 2e-5, (origin, float(d[:, :3].max()))
        assert float((d[:, 3] / a[:, 3].abs().clamp_min(1.0)).max()) < 1e-4
