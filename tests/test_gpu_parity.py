"""HIP kernels (through the C ABI) against the oracle and the reference's golden
vectors. Needs an MI355X: every test is marked gpu.

Tolerances (north_star): RGB / depth <= 1e-4 abs fp32; sample indices bit-exact.
"""
import numpy as np
import pytest
import torch

from helpers import build_net, oracle_field, to_np
from oracle import avr_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import avr
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    avr.load_library()


def T(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


# ----------------------------------------------------------------- composite
@pytest.mark.parametrize("N", [64, 128, 192])
@pytest.mark.parametrize("wb", [0, 1])
def test_composite_fwd_golden(golden, N, wb):
    from avr import ops
    g = golden("g1_volume_integral.npz")
    k = f"N{N}_wb{wb}"
    z, sig, rad = g[f"{k}_z"][0], g[f"{k}_sigma"][0], g[f"{k}_rad"][0]
    field = T(np.concatenate([rad, sig], -1))
    rgb, dist, w = ops.composite_fwd(T(z), field, bool(wb))
    np.testing.assert_allclose(to_np(w), g[f"{k}_weights"][0, ..., 0], atol=1e-6, rtol=0)
    np.testing.assert_allclose(to_np(rgb), g[f"{k}_rgb"][0], atol=2e-6, rtol=0)
    np.testing.assert_allclose(to_np(dist), g[f"{k}_depth"][0, :, 0], atol=2e-6, rtol=0)
    # and against the oracle
    orgb, odep, ow = O.volume_integral(z, sig, rad, bool(wb))
    np.testing.assert_allclose(to_np(rgb), orgb, atol=2e-6, rtol=0)


@pytest.mark.parametrize("N", [64, 128, 192])
@pytest.mark.parametrize("wb", [0, 1])
def test_composite_bwd_golden(golden, N, wb):
    """HIP backward vs the reference's own autograd (golden dsigma / drad)."""
    from avr.renderers import volume_integral
    g = golden("g1_volume_integral.npz")
    k = f"N{N}_wb{wb}"
    sig = T(g[f"{k}_sigma"]).requires_grad_(True)
    rad = T(g[f"{k}_rad"]).requires_grad_(True)
    rgb, dmap, _ = volume_integral(T(g[f"{k}_z"]), sig, rad, white_back=bool(wb))
    ((rgb * T(g[f"{k}_grad_rgb"])).sum() + (dmap * T(g[f"{k}_grad_depth"])).sum()).backward()
    np.testing.assert_allclose(to_np(rad.grad), g[f"{k}_drad"], atol=2e-6, rtol=0)
    ref = g[f"{k}_dsigma"]
    got = to_np(sig.grad)
    # the last interval is 1e10 long (renderers.py:80): d/dsigma there is ~1e10 * exp(-1e10 sigma)
    scale = np.maximum(np.abs(ref), 1.0)
    # dL/dalpha = g_w T - S / t cancels; the reference's own fp32 autograd carries ~1e-5 relative error here
    np.testing.assert_allclose(got / scale, ref / scale, atol=1e-4, rtol=0)


@pytest.mark.parametrize("N", [1, 5, 63, 65, 100, 333, 1024])
def test_composite_fwd_lane_segments(N):
    """Every lane-segment width K = ceil(N/64) (1..16), ragged last lanes,
    weights stored or not, against the oracle."""
    from avr import ops
    R = 97
    rng = np.random.default_rng(N)
    z = np.sort(rng.uniform(0.8, 1.8, (R, N)).astype(np.float32), -1)
    sig = np.maximum(rng.normal(0, 30, (R, N, 1)), 0).astype(np.float32)
    sig[::5] = 0.0
    rad = rng.random((R, N, 3), dtype=np.float32)
    field = T(np.concatenate([rad, sig], -1))
    orgb, odep, ow = O.volume_integral(z[None], sig[None], rad[None], True)
    rgb, dist, w = ops.composite_fwd(T(z), field, True)
    np.testing.assert_allclose(to_np(w), ow[0, ..., 0], atol=1e-6, rtol=0)
    np.testing.assert_allclose(to_np(rgb), orgb[0], atol=2e-6, rtol=0)
    np.testing.assert_allclose(to_np(dist), odep[0, :, 0], atol=2e-6, rtol=0)
    rgb2, dist2, w2 = ops.composite_fwd(T(z), field, True, want_weights=False)
    assert w2 is None and torch.equal(rgb2, rgb) and torch.equal(dist2, dist)


def test_composite_edge_cases():
    from avr import ops
    # one sample per ray, a ray of all zeros, a huge sigma
    z = T(np.array([[1.0], [1.2], [0.9]], np.float32))
    f = T(np.array([[[0.2, 0.4, 0.6, 0.0]], [[0.1, 0.1, 0.1, 5.0]], [[1, 1, 1, 1e30]]], np.float32))
    rgb, dist, w = ops.composite_fwd(z, f, True)
    o_rgb, o_d, o_w = O.volume_integral(to_np(z)[None], to_np(f)[None, ..., 3:], to_np(f)[None, ..., :3], True)
    np.testing.assert_allclose(to_np(rgb), o_rgb[0], atol=1e-6)
    np.testing.assert_allclose(to_np(dist), o_d[0, :, 0], atol=1e-6)
    # zero rays: no launch, no error
    e_rgb, e_d, e_w = ops.composite_fwd(torch.zeros(0, 8, device=DEV), torch.zeros(0, 8, 4, device=DEV))
    assert e_rgb.shape == (0, 3)


# ----------------------------------------------------------------- sampling
@pytest.mark.parametrize("case", ["vi", "zero", "exact", "spiky"])
def test_sample_fine_bit_exact(golden, case):
    from avr import ops
    g = golden("g2_sample_fine.npz")
    w = g[f"{case}_weights"][0, ..., 0]
    R, Nc = w.shape
    Nf = int(g["Nf"])
    zc = np.sort(np.random.default_rng(0).uniform(0.8, 1.8, (R, Nc)).astype(np.float32), -1)
    zs, idx, zf = ops.sample_fine(T(w), T(zc), float(g["near"]), float(g["far"]), Nf, 0, 0.0,
                                  u=T(g[f"{case}_u"]), u2=T(g[f"{case}_u2"]), want_idx=True, want_fine=True)
    np.testing.assert_array_equal(to_np(idx).astype(np.int32), g[f"{case}_idx"][0])
    np.testing.assert_array_equal(to_np(zf), g[f"{case}_z"][0])
    np.testing.assert_array_equal(to_np(zs), np.sort(np.concatenate([zc, g[f"{case}_z"][0]], -1), -1))


@pytest.mark.parametrize("Nc,Nf,Nd", [(64, 32, 16), (128, 64, 0), (32, 16, 8), (256, 128, 64), (200, 37, 5),
                                      (64, 64, 0), (192, 17, 0), (256, 64, 0), (96, 33, 0), (100, 1, 0)])
def test_sample_fine_vs_oracle(Nc, Nf, Nd):
    """Indices bit-exact vs the oracle on weights produced by a volume integral,
    odd sizes included; the sorted merge equals numpy's sort."""
    from avr import ops
    R = 1000
    rng = np.random.default_rng(Nc + Nf)
    zc = O.sample_coarse(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), Nc,
                         rng.random((1, R, Nc), dtype=np.float32))[0]
    sig = np.maximum(rng.normal(0, 3, (1, R, Nc, 1)), 0).astype(np.float32)
    sig[:, ::7] = 0.0
    _, _, w = O.volume_integral(zc[None], sig, rng.random((1, R, Nc, 3), dtype=np.float32))
    w = w[0, ..., 0]
    u = rng.random((R, Nf), dtype=np.float32)
    u2 = rng.random((R, Nf), dtype=np.float32)
    nd = rng.normal(0, 1, (R, Nd)).astype(np.float32)
    zs, idx, zf = ops.sample_fine(T(w), T(zc), 0.8, 1.8, Nf, Nd, 0.01, u=T(u), u2=T(u2), noise_depth=T(nd),
                                  want_idx=True, want_fine=True)
    oz, oidx = O.sample_fine(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), Nf, w[None, ..., None],
                             u[None], u2[None], return_idx=True)
    np.testing.assert_array_equal(to_np(idx), oidx[0])
    np.testing.assert_array_equal(to_np(zf), oz[0])
    od = np.clip(O.sample_depth(np.zeros((1, R, 1), np.float32), Nd, 0.01, nd[None]), np.float32(0.8),
                 np.float32(1.8))[0]
    np.testing.assert_array_equal(to_np(zs), np.sort(np.concatenate([zc, oz[0], od], -1), -1))


def test_sample_coarse_bit_exact():
    from avr import ops
    R, N = 777, 128
    noise = np.random.default_rng(3).random((R, N), dtype=np.float32)
    z = ops.sample_coarse(0.8, 1.8, R, N, DEV, noise=T(noise))
    ref = O.sample_coarse(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), N, noise[None])[0]
    np.testing.assert_array_equal(to_np(z), ref)


@pytest.mark.parametrize("N", [1, 6, 37, 64])
def test_sample_coarse_ragged_bit_exact(N):
    """N not a multiple of the kernel's 4-sample blocks: explicit noise bit-exact;
    in-kernel noise equal to the one-uniform-at-a-time draw (block k of ray r holds
    samples 4k..4k+3), i.e. a prefix of the N=64 draw."""
    from avr import ops
    R = 301
    noise = np.random.default_rng(N).random((R, N), dtype=np.float32)
    z = ops.sample_coarse(0.8, 1.8, R, N, DEV, noise=T(noise))
    ref = O.sample_coarse(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), N, noise[None])[0]
    np.testing.assert_array_equal(to_np(z), ref)
    zp = ops.sample_coarse(0.8, 1.8, R, N, DEV, seed=11, offset=5)
    z64 = ops.sample_coarse(0.8, 1.8, R, 64, DEV, seed=11, offset=5)
    u_n = (zp - (0.8 + torch.arange(N, device=DEV) / N)) * N
    u_64 = (z64 - (0.8 + torch.arange(64, device=DEV) / 64)) * 64
    torch.testing.assert_close(u_n, u_64[:, :N], atol=2e-5, rtol=0)


@pytest.mark.parametrize("R", [1, 3, 1001])
@pytest.mark.parametrize("Nc,Nf,Nd", [(128, 64, 0), (64, 32, 16)])
def test_sample_fine_partial_workgroup(R, Nc, Nf, Nd):
    """Ray counts that leave the last workgroup (4 rays) partly empty, for the
    compile-time-size path (128 -> 64) and the runtime one: indices, fine z and
    the merge bit-exact against the oracle."""
    from avr import ops
    rng = np.random.default_rng(R + Nc)
    zc = np.sort(rng.uniform(0.8, 1.8, (R, Nc)).astype(np.float32), -1)
    w = rng.random((R, Nc), dtype=np.float32)
    u, u2 = rng.random((R, Nf), dtype=np.float32), rng.random((R, Nf), dtype=np.float32)
    nd = rng.normal(0, 1, (R, Nd)).astype(np.float32)
    zs, idx, zf = ops.sample_fine(T(w), T(zc), 0.8, 1.8, Nf, Nd, 0.01, u=T(u), u2=T(u2), noise_depth=T(nd),
                                  want_idx=True, want_fine=True)
    oz, oidx = O.sample_fine(np.full((1, R), 0.8, np.float32), np.full((1, R), 1.8, np.float32), Nf, w[None, ..., None],
                             u[None], u2[None], return_idx=True)
    np.testing.assert_array_equal(to_np(idx), oidx[0])
    np.testing.assert_array_equal(to_np(zf), oz[0])
    od = np.clip(O.sample_depth(np.zeros((1, R, 1), np.float32), Nd, 0.01, nd[None]), np.float32(0.8),
                 np.float32(1.8))[0]
    np.testing.assert_array_equal(to_np(zs), np.sort(np.concatenate([zc, oz[0], od], -1), -1))


def test_sample_fine_merge_ties():
    """Coarse values equal to fine values (n_depth 0: the two-list slot merge):
    every slot filled once, the output equals numpy's sort."""
    from avr import ops
    R, Nc, Nf = 500, 128, 64
    rng = np.random.default_rng(9)
    zc = np.sort(rng.uniform(0.8, 1.8, (R, Nc)).astype(np.float32), -1)
    w = rng.random((R, Nc), dtype=np.float32)
    u, u2 = rng.random((R, Nf), dtype=np.float32), rng.random((R, Nf), dtype=np.float32)
    _, _, zf = ops.sample_fine(T(w), T(zc), 0.8, 1.8, Nf, 0, 0.0, u=T(u), u2=T(u2), want_fine=True)
    zf = to_np(zf)
    zc2 = np.sort(np.concatenate([zc[:, : Nc - 16], zf[:, :16]], -1), -1)      # 16 exact ties per ray
    zs, _, zf2 = ops.sample_fine(T(w), T(zc2), 0.8, 1.8, Nf, 0, 0.0, u=T(u), u2=T(u2), want_fine=True)
    np.testing.assert_array_equal(to_np(zf2), zf)
    np.testing.assert_array_equal(to_np(zs), np.sort(np.concatenate([zc2, zf], -1), -1))


def test_sample_fine_unsorted_coarse_fallback():
    """z_coarse given out of order (the reference sorts cat(z_c, z_f) whatever
    z_c holds): the wave-local bitonic path must equal numpy's sort."""
    from avr import ops
    R, Nc, Nf, Nd = 300, 64, 32, 8
    rng = np.random.default_rng(5)
    zc = rng.uniform(0.8, 1.8, (R, Nc)).astype(np.float32)
    zc[: R // 2] = np.sort(zc[: R // 2], -1)          # half sorted (fast path), half not (fallback)
    zc[::7, 3] = zc[::7, 4]                            # ties
    w = rng.random((R, Nc), dtype=np.float32)
    u, u2 = rng.random((R, Nf), dtype=np.float32), rng.random((R, Nf), dtype=np.float32)
    nd = rng.normal(0, 1, (R, Nd)).astype(np.float32)
    zs, idx, zf = ops.sample_fine(T(w), T(zc), 0.8, 1.8, Nf, Nd, 0.01, u=T(u), u2=T(u2), noise_depth=T(nd),
                                  want_idx=True, want_fine=True)
    od = np.clip(O.sample_depth(np.zeros((1, R, 1), np.float32), Nd, 0.01, nd[None]), np.float32(0.8),
                 np.float32(1.8))[0]
    np.testing.assert_array_equal(to_np(zs), np.sort(np.concatenate([zc, to_np(zf), od], -1), -1))


def test_philox_noise_properties():
    """In-kernel Philox noise: deterministic per (seed, offset), U[0,1) moments,
    stratified samples stay in their bins."""
    from avr import ops
    R, N = 65536, 128
    z1 = ops.sample_coarse(0.8, 1.8, R, N, DEV, seed=7, offset=0)
    z2 = ops.sample_coarse(0.8, 1.8, R, N, DEV, seed=7, offset=0)
    z3 = ops.sample_coarse(0.8, 1.8, R, N, DEV, seed=8, offset=0)
    assert torch.equal(z1, z2) and not torch.equal(z1, z3)
    u = (z1 - (0.8 + torch.arange(N, device=DEV) / N)) * N  # ~ U[0,1)
    assert float(u.min()) > -1e-4 and float(u.max()) < 1.0 + 1e-4
    assert abs(float(u.mean()) - 0.5) < 2e-3 and abs(float(u.var()) - 1 / 12) < 2e-3
    assert bool((z1[:, 1:] >= z1[:, :-1]).all())


# ----------------------------------------------------------------- geometry
def test_world_rays_and_depth_golden(golden):
    from avr import ops
    g = golden("g3_geometry.npz")
    ro, rd, info = ops.world_rays(T(g["x_pix"]), T(g["K"]), T(g["c2w"]))
    np.testing.assert_array_equal(to_np(ro), g["ro"])
    np.testing.assert_allclose(to_np(rd), g["rd"], atol=2e-7, rtol=0)
    depth = ops.depth_from_world(ro, rd, T(g["dist"][..., 0]), info)
    np.testing.assert_allclose(to_np(depth), g["depth"], atol=1e-6, rtol=0)
    # stride-0 (expanded) pose, un-normalised K
    R = g["x_pix2"].shape[1]
    c2w = T(g["c2w_one"]).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    ro2, rd2, _ = ops.world_rays(T(g["x_pix2"]), T(g["K2"]), c2w)
    np.testing.assert_allclose(to_np(rd2), g["rd2"], atol=2e-7, rtol=0)
    np.testing.assert_array_equal(to_np(ro2), g["ro2"])


# ----------------------------------------------------------------- field
PRECISIONS = ["fp32", "x3"]


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("tag", ["small", "small_mv", "full", "mv512", "d256"])
def test_field_points_golden(golden, tag, precision):
    _field_points_golden(golden, tag, precision)


@pytest.mark.parametrize("waves", ["8", "4"])
@pytest.mark.parametrize("tag", ["bn_small", "bn512", "bn_mv512"])
def test_field_points_golden_batchnorm(golden, tag, waves, monkeypatch):
    """train.py --bn nets (eval-mode BatchNorm: bn_0 in front of both relus of
    every block, models.py:456-461) on the fused x3 kernel, against the
    reference's own forward (g4 bn fixtures), both 512-wide layouts."""
    monkeypatch.setenv("AVR_X3_WAVES", waves)
    if waves == "4" and not tag.endswith("512"):
        pytest.skip("one layout below 512 wide")
    _field_points_golden(golden, tag, "x3")


@pytest.mark.parametrize("tag", ["spade_small", "spade512", "sp_small", "sp512", "spade_sp_mv"])
def test_field_points_golden_spade_softplus(golden, tag):
    """ResnetFC options on the fused x3 kernel against the reference's own forward (g4):
    use_spade (scale_z[b](z) * x + lin_z[b](z), models.py:528-534, 585-587) and Softplus(beta)
    in place of every ReLU (models.py:442-445, 536-537), alone and together."""
    g = golden(f"g4_field_{tag}.npz")
    net = build_net(g, DEV, "x3")
    with torch.no_grad():
        assert net.can_fuse(T(g["xyz"]))
    _field_points_golden(golden, tag, "x3")


@pytest.mark.parametrize("tag", ["spade_small", "spade512", "sp512", "spade_sp_mv"])
def test_field_spade_softplus_many_texels_and_rays(golden, tag):
    """Random points (a workgroup's 256 bilinear corners touch more distinct texels than one
    LDS stage holds: the multi-pass staging of both spade tables) and the rays mode, against the
    module's PyTorch graph of the same net; two scenes in one launch equal two launches."""
    g = golden(f"g4_field_{tag}.npz")
    net = build_net(g, DEV, "x3")
    gen = torch.Generator(device="cpu").manual_seed(7)
    xyz = (torch.rand(1, 6000, 3, generator=gen) - 0.5).to(DEV)
    vd = torch.nn.functional.normalize(torch.randn(1, 6000, 3, generator=gen), dim=-1).to(DEV)
    with torch.no_grad():
        a = net(xyz, coarse=False, viewdirs=vd)
        b = net.forward_torch(xyz, coarse=False, viewdirs=vd)
    np.testing.assert_allclose(to_np(a), to_np(b), atol=5e-5, rtol=1e-4)
    R, N = 200, 19
    ro = torch.tensor([[0.3, -1.1, 0.5]], device=DEV).expand(R, 3).contiguous()
    rd = torch.nn.functional.normalize(-ro + 0.2 * torch.randn(R, 3, device=DEV, generator=None), dim=-1)
    z = torch.sort(0.8 + torch.rand(R, N, device=DEV), -1)[0]
    with torch.no_grad():
        fr = net.fused().forward_rays(ro, rd, z, coarse=True)
        pts = ro[:, None, :] + rd[:, None, :] * z[..., None]
        fp = net(pts.reshape(1, -1, 3), coarse=True, viewdirs=rd[:, None, :].expand(R, N, 3).reshape(1, -1, 3))
    np.testing.assert_array_equal(to_np(fr), to_np(fp[0]))
    # two scenes (same latent) in one batched launch = one launch per scene
    with torch.no_grad():
        two = net.fused().forward_points(xyz[:, :3000].expand(2, 3000, 3).contiguous(),
                                         vd[:, :3000].expand(2, 3000, 3).contiguous(), False)
    np.testing.assert_array_equal(to_np(two[0]), to_np(two[1]))
    np.testing.assert_array_equal(to_np(two[0]), to_np(a[0, :3000]))


@pytest.mark.parametrize("tag", ["ns2_small", "ns2max_small", "ns3_mv512"])
def test_field_multiview_golden(golden, tag):
    """NS > 1 source views (models.py:749-853; ResnetFC combines the views at combine_layer,
    :566-579): the fused x3 field in two launches around the combine (avr_field_fwd_points_split)
    against the reference's own forward; the module's PyTorch graph agrees too."""
    g = golden(f"g4_field_{tag}.npz")
    net = build_net(g, DEV, "x3")
    xyz, vd = T(g["xyz"]), T(g["viewdirs"])
    assert net.num_views_per_obj == int(g["ns"]) > 1
    with torch.no_grad():
        assert not net.can_fuse(xyz) and net.can_fuse_multiview(xyz)
        oc = net(xyz, coarse=True, viewdirs=vd)
        of = net(xyz, coarse=False, viewdirs=vd)
        tc = net.forward_torch(xyz, coarse=True, viewdirs=vd)
    np.testing.assert_allclose(to_np(oc), g["out_coarse"], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(to_np(of), g["out_fine"], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(to_np(tc), g["out_coarse"], atol=5e-5, rtol=1e-4)


def test_field_multiview_combine_layer0_module_path(golden):
    """combine_layer 0 (the views combined right after lin_in) is a valid ResnetFC config the split
    launches do not run: the net routes it to the module path (no AVRError), and a direct FusedField call
    raises instead of serving it at x3; at fp32 precision the NS > 1 redirect raises as well."""
    from avr import _lib
    g = golden("g4_field_ns2_small.npz")
    net = build_net(g, DEV, "x3")
    xyz, vd = T(g["xyz"]), T(g["viewdirs"])
    with torch.no_grad():
        ref = net.forward_torch(xyz, coarse=True, viewdirs=vd)
        for mlp in (net.mlp_coarse, net.mlp_fine):
            mlp.combine_layer = 0
        assert not net.can_fuse(xyz) and not net.can_fuse_multiview(xyz)
        out = net(xyz, coarse=True, viewdirs=vd)
        np.testing.assert_array_equal(to_np(out), to_np(net.forward_torch(xyz, coarse=True, viewdirs=vd)))
        assert not np.array_equal(to_np(out), to_np(ref))      # the combine really moved
        with pytest.raises(_lib.AVRError):
            net.fused().forward_points(xyz, vd, True)
        for mlp in (net.mlp_coarse, net.mlp_fine):
            mlp.combine_layer = int(g["combine_layer"])
        net.field_precision = "fp32"
        with pytest.raises(_lib.AVRError):
            net.fused().forward_points(xyz, vd, True)


def test_field_multiview_objects_and_renderer(golden):
    """SB = 2 objects x NS = 2 views (more scenes than points per object would need: 4
    (object, view) pairs in the first launch, 2 objects in the second), equal to each object
    alone; a VolumeRenderer over an NS = 2 net routes its field calls to the split path."""
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS
    g = golden("g4_field_ns2_small.npz")
    net = build_net(g, DEV, "x3")
    lat, poses = net.encoder.latent, net.poses
    net.encoder.latent = torch.cat([lat, lat.flip(-1)], 0)           # (SB * NS, L, H, W)
    net.poses = torch.cat([poses, poses.flip(0)], 0)
    gen = torch.Generator(device="cpu").manual_seed(3)
    xyz = (torch.rand(2, 700, 3, generator=gen) - 0.5).to(DEV)
    vd = torch.nn.functional.normalize(torch.randn(2, 700, 3, generator=gen), dim=-1).to(DEV)
    with torch.no_grad():
        both = net(xyz, coarse=False, viewdirs=vd)
        ref = net.forward_torch(xyz, coarse=False, viewdirs=vd)
    np.testing.assert_allclose(to_np(both), to_np(ref), atol=5e-5, rtol=1e-4)
    for s in range(2):
        net.encoder.latent = torch.cat([lat, lat.flip(-1)], 0)[2 * s:2 * s + 2]
        net.poses = torch.cat([poses, poses.flip(0)], 0)[2 * s:2 * s + 2]
        with torch.no_grad():
            one = net(xyz[s:s + 1], coarse=False, viewdirs=vd[s:s + 1])
        np.testing.assert_array_equal(to_np(one[0]), to_np(both[s]))
    net.encoder.latent, net.poses = lat, poses
    R = 128
    x_pix = torch.rand(1, R, 2, generator=gen).to(DEV)
    c2w = torch.eye(4, device=DEV).reshape(1, 1, 4, 4).expand(1, R, 4, 4).clone()
    c2w[..., 2, 3] = -1.3
    rend = VolumeRenderer(0.8, 1.8, 16, 8, 0, 0.01, True)
    rend.seed = 5
    with torch.no_grad():
        rgb_c, rgb_f, depth, _ = rend(c2w, torch.tensor([INTRINSICS], device=DEV), x_pix, net)
    assert rend.last_path == "module" and torch.isfinite(rgb_f).all() and torch.isfinite(depth).all()


def test_field_spade_softplus_routes(golden):
    """use_spade / Softplus nets: fused on the x3 path for inference; precision fp32 and
    autograd run the module's PyTorch graph (which matches the reference's forward too)."""
    g = golden("g4_field_spade_sp_mv.npz")
    net = build_net(g, DEV, "fp32")
    xyz, vd = T(g["xyz"]), T(g["viewdirs"])
    with torch.no_grad():
        assert not net.can_fuse(xyz)
        np.testing.assert_allclose(to_np(net(xyz, coarse=True, viewdirs=vd)), g["out_coarse"], atol=5e-5, rtol=1e-4)
        net.field_precision = "x3"
        assert net.can_fuse(xyz)
    for p in net.parameters():
        p.requires_grad_(True)
    assert not net.can_train_fused(xyz, vd)


def test_field_batchnorm_routes(golden):
    """BatchNorm nets: fused only on the x3 path in eval mode. precision fp32,
    train-mode BN (batch statistics) and autograd run the module's PyTorch
    graph, which matches the reference's eval forward too."""
    g = golden("g4_field_bn512.npz")
    net = build_net(g, DEV, "fp32")
    xyz, vd = T(g["xyz"]), T(g["viewdirs"])
    with torch.no_grad():
        assert not net.can_fuse(xyz)
        np.testing.assert_allclose(to_np(net(xyz, coarse=True, viewdirs=vd)), g["out_coarse"], atol=5e-5, rtol=1e-4)
        net.field_precision = "x3"
        assert net.can_fuse(xyz)
        net.mlp_coarse.train()
        assert not net.can_fuse(xyz)
        net.mlp_coarse.eval()
    for p in net.parameters():
        p.requires_grad_(True)
    assert not net.can_train_fused(xyz, vd)


def _field_points_golden(golden, tag, precision):
    g = golden(f"g4_field_{tag}.npz")
    net = build_net(g, DEV, precision)
    with torch.no_grad():
        assert net.can_fuse(T(g["xyz"]))
        oc = net(T(g["xyz"]), coarse=True, viewdirs=T(g["viewdirs"]))
        of = net(T(g["xyz"]), coarse=False, viewdirs=T(g["viewdirs"]))
    np.testing.assert_allclose(to_np(oc), g["out_coarse"], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(to_np(of), g["out_fine"], atol=5e-5, rtol=1e-4)


def test_field_precision_switch_on_one_net(golden):
    """net.field_precision switched back and forth on one net: each precision gets its own
    packed blob and tables (an x3 blob holds only the x3 fragments, avr_field_pack), and every
    pass matches the reference's forward (g4 mv512)."""
    g = golden("g4_field_mv512.npz")
    net = build_net(g, DEV, "x3")
    xyz, vd = T(g["xyz"]), T(g["viewdirs"])
    with torch.no_grad():
        for precision in ("x3", "fp32", "x3", "fp32"):
            net.field_precision = precision
            assert net.can_fuse(xyz)
            np.testing.assert_allclose(to_np(net(xyz, coarse=True, viewdirs=vd)), g["out_coarse"], atol=5e-5,
                                       rtol=1e-4)
            np.testing.assert_allclose(to_np(net(xyz, coarse=False, viewdirs=vd)), g["out_fine"], atol=5e-5,
                                       rtol=1e-4)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("tag", ["small", "small_mv", "full", "mv512", "d256"])
def test_field_fused_matches_torch_path(golden, tag, precision):
    """The fused kernel and the module's PyTorch graph (same device, same
    weights) agree: the lin_z-per-texel factorisation and (x3) the split-fp16
    products change rounding only."""
    g = golden(f"g4_field_{tag}.npz")
    net = build_net(g, DEV, precision)
    xyz = torch.rand(1, 5000, 3, device=DEV) - 0.5
    vd = torch.nn.functional.normalize(torch.randn(1, 5000, 3, device=DEV), dim=-1)
    with torch.no_grad():
        a = net(xyz, coarse=False, viewdirs=vd)
        b = net.forward_torch(xyz, coarse=False, viewdirs=vd)
    np.testing.assert_allclose(to_np(a), to_np(b), atol=5e-5, rtol=1e-4)


@pytest.mark.parametrize("precision", PRECISIONS)
def test_field_rays_mode_matches_points_mode(golden, precision):
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, precision)
    R, N = 300, 17
    ro = torch.tensor([[0.3, -1.1, 0.5]], device=DEV).expand(R, 3).contiguous()
    rd = torch.nn.functional.normalize(-ro + 0.2 * torch.randn(R, 3, device=DEV), dim=-1)
    z = torch.sort(0.8 + torch.rand(R, N, device=DEV), -1)[0]
    with torch.no_grad():
        a = net.fused().forward_rays(ro, rd, z, coarse=True)
        pts = ro[:, None, :] + rd[:, None, :] * z[..., None]
        b = net(pts.reshape(1, -1, 3), coarse=True, viewdirs=rd[:, None, :].expand(R, N, 3).reshape(1, -1, 3))
    np.testing.assert_array_equal(to_np(a), to_np(b[0]))


# ----------------------------------------------------------------- end to end
@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("tag", ["c64f32d16", "c128f64d0"])
def test_volume_renderer_golden(golden, tag, precision):
    """Full VolumeRenderer.forward with the reference's captured noise: coarse
    rgb <= 1e-4; the inverse-CDF bins of the HIP chain equal the reference's
    own searchsorted result (g5 `idx`) on every ray, and fine rgb / depth are
    within 1e-4 on every ray."""
    from avr.renderers import VolumeRenderer
    g = golden(f"g5_forward_{tag}.npz")
    net = build_net(g, DEV, precision)
    R = g["x_pix"].shape[1]
    rend = VolumeRenderer(float(g["near"]), float(g["far"]), int(g["Nc"]), int(g["Nf"]), int(g["Nd"]),
                          float(g["depth_std"]), True)
    c2w = T(g["c2w_one"]).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    noise = {"coarse": T(g["noise_coarse"]), "u": T(g["u"]), "u2": T(g["u2"]), "depth": T(g["noise_depth"])}
    with torch.no_grad():
        rgb_c, rgb_f, depth, depth2 = rend(c2w, T(g["K"]), T(g["x_pix"]), net, noise=noise)
    assert rend.last_path == "fused"
    assert depth2 is depth
    np.testing.assert_allclose(to_np(rgb_c), g["rgb_coarse"], atol=1e-4)
    # the bins the renderer's sample_fine launch chose (same kernels, same inputs)
    from avr import ops
    with torch.no_grad():
        ro, rd, _ = ops.world_rays(T(g["x_pix"]), T(g["K"]), c2w)
        zc = ops.sample_coarse(float(g["near"]), float(g["far"]), R, int(g["Nc"]), DEV, noise=noise["coarse"][0])
        fc = net.fused().forward_rays(ro[0], rd[0], zc, True)
        _, _, w_c = ops.composite(zc, fc)
        nf = int(g["Nf"]) - int(g["Nd"])
        _, idx, _ = ops.sample_fine(w_c, zc, float(g["near"]), float(g["far"]), nf, int(g["Nd"]),
                                    float(g["depth_std"]), u=noise["u"][0], u2=noise["u2"][0],
                                    noise_depth=noise["depth"][0], want_idx=True)
    same = (to_np(idx) == g["idx"][0]).all(-1)
    ok = (np.abs(to_np(rgb_f) - g["rgb_fine"]).max(-1) <= 1e-4) & (np.abs(to_np(depth) - g["depth"]) <= 1e-4)
    print(f"{tag} {precision}: bins equal {(to_np(idx) == g['idx'][0]).mean():.4f}, rays with the reference's "
          f"bins {same.mean():.4f}, rays within 1e-4 {ok.mean():.4f}")
    # every ray takes the reference's own bins and lands within 1e-4 (both precisions, both configs: measured
    # 64 / 64). The bar is strict on purpose: a bin flip here would come from a ULP-level change of the coarse
    # weights, which the C3 test (test_gpu_scale.py) bounds statistically on 4 096 rays.
    assert same.all(), np.nonzero(~same)
    assert ok[0][same].all(), np.nonzero(~ok[0] & same)
    assert ok.all(), ok.mean()


@pytest.mark.parametrize("precision", PRECISIONS)
def test_volume_renderer_c3_shape_properties(golden, precision):
    """BASELINE config 3 size (65536 rays, 128 + 64, Nd = 0) with Philox noise:
    finite outputs, rgb in [0, 1] (white background), depth within the
    near/far shell, and the first 128 rays equal the oracle fed the same
    per-stage inputs."""
    from avr import ops
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, precision)
    R = 65536
    rend = VolumeRenderer(0.8, 1.8, 128, 64, 0, 0.01, True)
    rend.seed = 1234
    x_pix = torch.rand(1, R, 2, device=DEV)
    from oracle import synth
    c2w = T(synth.orbit_cam2world(0.7)).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    K = T(synth.default_intrinsics())[None]
    with torch.no_grad():
        rgb_c, rgb_f, depth, _ = rend(c2w, K, x_pix, net)
    torch.cuda.synchronize()
    for t in (rgb_c, rgb_f, depth):
        assert bool(torch.isfinite(t).all())
    assert float(rgb_f.min()) >= -1e-5 and float(rgb_f.max()) <= 1.0 + 1e-5
    # staged check of the coarse pass on a slice against the oracle
    with torch.no_grad():
        ro, rd, _ = ops.world_rays(x_pix[:, :128], K, c2w[:, :128])
        zc = ops.sample_coarse(0.8, 1.8, 128, 128, DEV, seed=1234, offset=0)
        fc = net.fused().forward_rays(ro[0], rd[0], zc, True)
    of = oracle_field(g)
    pts = to_np(ro[0])[:, None, :] + to_np(rd[0])[:, None, :] * to_np(zc)[..., None]
    ref = of(pts.reshape(1, -1, 3), np.broadcast_to(to_np(rd[0])[:, None, :], pts.shape).reshape(1, -1, 3))
    np.testing.assert_allclose(to_np(fc), ref[0], atol=5e-4, rtol=1e-3)
    rgb_o, _, _ = O.volume_integral(to_np(zc)[None], ref[..., 3:].reshape(1, 128, 128, 1),
                                    ref[..., :3].reshape(1, 128, 128, 3))
    np.testing.assert_allclose(to_np(rgb_c[0, :128]), rgb_o[0], atol=1e-4)


def test_volume_renderer_module_path_and_backward(golden):
    """With autograd on, the renderer calls the module (PyTorch field) and the
    HIP composite backward; gradients reach the MLP weights and match a
    pure-torch fp32 composite (torch reference of the floating-point kernel)."""
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_small.npz")
    net = build_net(g, DEV)
    for p in net.parameters():
        p.requires_grad_(True)
    R = 256
    rend = VolumeRenderer(0.8, 1.8, 32, 16, 8, 0.01, True)
    from oracle import synth
    c2w = T(synth.orbit_cam2world(1.1)).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    K = T(synth.default_intrinsics())[None]
    x_pix = torch.rand(1, R, 2, device=DEV)
    torch.manual_seed(0)
    noise = {"coarse": torch.rand(1, R, 32, device=DEV), "u": torch.rand(1, R, 8, device=DEV),
             "u2": torch.rand(1, R, 8, device=DEV), "depth": torch.randn(1, R, 8, device=DEV)}
    rgb_c, rgb_f, depth, _ = rend(c2w, K, x_pix, net, noise=noise)
    assert rend.last_path == "module"
    loss = rgb_c.square().mean() + rgb_f.square().mean() + depth.mean()
    loss.backward()
    gw = net.mlp_fine.lin_out.weight.grad.clone()
    assert torch.isfinite(gw).all() and float(gw.abs().max()) > 0
    # same loss through a torch-only volume integral
    net.zero_grad()

    def vi_torch(z, sig, rad):
        d = torch.cat([z[..., 1:] - z[..., :-1], torch.full_like(z[..., :1], 1e10)], -1)
        a = 1.0 - torch.exp(-sig[..., 0] * d)
        t = torch.cumprod(torch.cat([torch.ones_like(a[..., :1]), 1.0 - a + 1e-10], -1), -1)[..., :-1]
        w = a * t
        rgb = (w[..., None] * rad).sum(-2) + (1.0 - w.sum(-1, keepdim=True))
        zz = torch.cat([z[..., 1:], torch.full_like(z[..., :1], 1.8)], -1)
        return rgb, (w * zz).sum(-1, keepdim=True), w

    import avr.ops as ops
    orig = ops.composite

    def torch_composite(z, field, white_back=True, infinity=1.8, want_weights=True):
        rgb, dist, w = vi_torch(z, field[..., 3:], field[..., :3])
        return rgb, dist[..., 0], w

    ops.composite = torch_composite
    try:
        rgb_c2, rgb_f2, depth2, _ = rend(c2w, K, x_pix, net, noise=noise)
    finally:
        ops.composite = orig
    (rgb_c2.square().mean() + rgb_f2.square().mean() + depth2.mean()).backward()
    np.testing.assert_allclose(to_np(rgb_f), to_np(rgb_f2), atol=1e-5)
    np.testing.assert_allclose(to_np(gw), to_np(net.mlp_fine.lin_out.weight.grad), atol=1e-4, rtol=1e-3)


# ----------------------------------------------------------------- errors
def test_errors_are_loud():
    from avr import _lib, ops
    with pytest.raises(_lib.AVRError):
        ops.composite_fwd(torch.zeros(4, 8), torch.zeros(4, 8, 4))  # host tensors: no CPU path
    with pytest.raises(_lib.AVRError):
        ops.sample_fine(torch.zeros(2, 300, device=DEV), torch.zeros(2, 300, device=DEV), 0.8, 1.8, 8, 0, 0.0)


def test_fp32_kernel_rejects_x3_only_blob(golden):
    """an AVR_FIELD_X3 blob has no fp32 lin_in / fc_0 / fc_1 fragments; the fp32 field entry points
    refuse it instead of multiplying uninitialised memory, and accept the same net packed for AVR_FIELD_FP32."""
    import ctypes
    from avr import _lib
    from avr.field import FusedField
    g = golden("g4_field_small.npz")
    net = build_net(g, DEV, "x3")
    f = FusedField(net, "x3")
    entry = f.packed(True)
    xyz, vd = T(g["xyz"]), T(g["viewdirs"])
    p, v = xyz[0].contiguous(), vd.reshape(xyz.shape)[0].contiguous()
    out = torch.empty(p.shape[0], 4, device=DEV)
    table = f.table(True)
    dims = _lib.FieldDims.from_buffer_copy(entry.dims)
    dims.precision = _lib.FIELD_FP32
    with pytest.raises(_lib.AVRError, match="packed for AVR_FIELD_X3"):
        _lib.call("avr_field_fwd_points", ctypes.byref(dims), ctypes.byref(f.view(0)), _lib.ptr(entry.packed),
                  _lib.ptr(table), _lib.ptr(p), _lib.ptr(v), p.shape[0], _lib.ptr(out), _lib.stream_of(p))
    f32 = FusedField(net, "fp32")
    e32 = f32.packed(True)
    _lib.call("avr_field_fwd_points", ctypes.byref(e32.dims), ctypes.byref(f32.view(0)), _lib.ptr(e32.packed),
              _lib.ptr(f32.table(True)), _lib.ptr(p), _lib.ptr(v), p.shape[0], _lib.ptr(out), _lib.stream_of(p))
    torch.cuda.synchronize()
    assert bool(torch.isfinite(out).all())


def test_field_x3_tracks_fp32_at_scale(golden):
    """Split-fp16 field vs fp32 field on 200k random samples of the 512-wide net:
    the difference stays at fp32-accumulation level."""
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, "fp32")
    R, N = 2000, 100
    ro = torch.tensor([[0.4, -1.0, 0.6]], device=DEV).expand(R, 3).contiguous()
    rd = torch.nn.functional.normalize(-ro + 0.3 * torch.randn(R, 3, device=DEV), dim=-1)
    z = torch.sort(0.8 + torch.rand(R, N, device=DEV), -1)[0]
    with torch.no_grad():
        a = net.fused().forward_rays(ro, rd, z, coarse=True)
        net.field_precision = "x3"
        b = net.fused().forward_rays(ro, rd, z, coarse=True)
    d = (a - b).abs()
    assert float(d[:, :3].max()) < 2e-5, float(d[:, :3].max())
    assert float((d[:, 3] / a[:, 3].abs().clamp_min(1.0)).max()) < 1e-4


# ----------------------------------------------------------------- fused stage kernels
@pytest.mark.parametrize("n,noise,per_ray", [(128, False, False), (37, True, True), (192, False, True)])
def test_rays_sample_coarse_equals_separate_kernels(n, noise, per_ray):
    """avr_rays_sample_coarse (ray generation + stratified z + depth rows in one
    launch) equals avr_world_rays + avr_sample_coarse bit for bit, and the
    composite epilogue's depth equals avr_depth_from_world bit for bit."""
    from avr import ops
    from oracle import synth
    SB, R = 2, 777
    g = torch.Generator().manual_seed(n)
    x_pix = torch.rand(SB, R, 2, generator=g).to(DEV)
    K = T(np.stack([synth.default_intrinsics(), synth.default_intrinsics() * 1.1]).astype(np.float32))
    K[1, 2, 2] = 1.0
    if per_ray:
        c2w = T(np.stack([synth.orbit_cam2world(0.1 + 0.01 * i) for i in range(SB * R)]).astype(np.float32))
        c2w = c2w.reshape(SB, R, 4, 4)
    else:
        c2w = T(synth.orbit_cam2world(0.7)).reshape(1, 1, 4, 4).expand(SB, R, 4, 4)
    nz = torch.rand(SB, R, n, generator=g).to(DEV) if noise else None
    ids = torch.randperm(10 * SB * R, generator=g)[:SB * R].to(DEV)
    with torch.no_grad():
        ro, rd, info = ops.world_rays(x_pix, K, c2w)
        z = ops.sample_coarse(0.8, 1.8, SB * R, n, DEV, noise=nz, seed=5, offset=3, ray_ids=ids)
        ro2, rd2, z2, drow, _ = ops.rays_sample_coarse(x_pix, K, c2w, 0.8, 1.8, n, noise=nz, seed=5, offset=3,
                                                       ray_ids=ids, want_depth_row=True)
        assert torch.equal(ro, ro2) and torch.equal(rd, rd2) and torch.equal(z, z2)
        field = torch.cat([torch.rand(SB * R, n, 3, device=DEV), 3 * torch.rand(SB * R, n, 1, device=DEV)], -1)
        rgb, dist, w = ops.composite_fwd(z, field, True)
        depth = ops.depth_from_world(ro, rd, dist.reshape(SB, R), info)
        rgb2, dist2, w2, depth2 = ops.composite_depth(z, field, ro, rd, drow, True, want_weights=True)
    assert torch.equal(rgb, rgb2) and torch.equal(dist, dist2) and torch.equal(w, w2)
    assert torch.equal(depth.reshape(-1), depth2)


def test_sample_fine_philox_pairs():
    """In-kernel Philox for the fine pass (one block per fine sample: u, u2):
    deterministic per (seed, ray id), uniform, independent of the batch
    layout, and the merged output is the sorted union (numpy sort)."""
    from avr import ops
    R, Nc, Nf = 4096, 128, 64
    w = torch.rand(R, Nc, device=DEV) ** 4
    zc = ops.sample_coarse(0.8, 1.8, R, Nc, DEV, seed=1)
    zs, idx, zf = ops.sample_fine(w, zc, 0.8, 1.8, Nf, 0, 0.0, seed=9, want_idx=True, want_fine=True)
    zs2, idx2, zf2 = ops.sample_fine(w, zc, 0.8, 1.8, Nf, 0, 0.0, seed=9, want_idx=True, want_fine=True)
    assert torch.equal(zs, zs2) and torch.equal(idx, idx2)
    _, _, zf3 = ops.sample_fine(w, zc, 0.8, 1.8, Nf, 0, 0.0, seed=10, want_fine=True)
    assert not torch.equal(zf, zf3)
    # rays 100..199 alone, keyed by their ids, draw the same samples
    ids = torch.arange(100, 200, device=DEV)
    _, _, zf4 = ops.sample_fine(w[100:200].contiguous(), zc[100:200].contiguous(), 0.8, 1.8, Nf, 0, 0.0, seed=9,
                                want_fine=True, ray_ids=ids)
    assert torch.equal(zf4, zf[100:200])
    ref = np.sort(np.concatenate([to_np(zc), to_np(zf)], -1), -1)
    np.testing.assert_array_equal(to_np(zs), ref)
    # u2 ~ U[0,1): the position of z_fine inside its coarse bin
    frac = to_np(zf - 0.8) * Nc - to_np(idx).astype(np.float32)
    assert frac.min() > -1e-3 and frac.max() < 1 + 1e-3 and abs(frac.mean() - 0.5) < 5e-3


@pytest.mark.parametrize("SB", [3, 17])
def test_multi_scene_field_launch_equals_per_scene(SB):
    """avr_field_fwd_rays_batch / _points_batch (up to 16 scenes per launch, each
    with its own latent, pose and tables) equal one launch per scene bit for
    bit; the renderer's SB > 1 fused path uses them."""
    from avr.scene import synthetic_scene
    net = synthetic_scene(DEV)
    g = torch.Generator().manual_seed(SB)
    lat = torch.randn(SB, net.d_latent, 64, 64, generator=g).to(DEV)
    net.encoder.set_latent(lat)
    net.num_objs = SB
    poses = net.poses.repeat(SB, 1, 1)
    poses[:, 0, 3] += 0.03 * torch.arange(SB, device=DEV, dtype=torch.float32)
    net.poses = poses
    net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
    R, N = 100, 37
    ro = (torch.rand(SB, R, 3, generator=g) * 0.2 + torch.tensor([0.3, -1.1, 0.5])).to(DEV)
    rd = torch.nn.functional.normalize(-ro + 0.3 * torch.randn(SB, R, 3, generator=g).to(DEV), dim=-1)
    z = torch.sort(0.8 + torch.rand(SB * R, N, generator=g), -1)[0].to(DEV)
    f = net.fused()
    with torch.no_grad():
        batch = f.forward_rays_batch(ro, rd, z, False)
        loop = torch.cat([f.forward_rays(ro[b], rd[b], z[b * R:(b + 1) * R], False, sb=b) for b in range(SB)])
        assert torch.equal(batch, loop)
        xyz = ro[..., None, :] + rd[..., None, :] * z.reshape(SB, R, N, 1)
        vd = rd[..., None, :].expand(SB, R, N, 3)
        pts = net(xyz.reshape(SB, -1, 3), coarse=False, viewdirs=vd.reshape(SB, -1, 3))
    torch.testing.assert_close(pts.reshape(-1, 4), batch, atol=0, rtol=0)
