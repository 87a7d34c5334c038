"""Training through the HIP field (train.py:108-114's
loss.backward() through NewPixelNeRFNet, models.py:739-863): the x3 training
forward + HIP backward chain + sample-GEMM weight gradients against PyTorch
fp32 autograd of the same module (forward_torch), parameter by parameter,
including the latent map's gradient and a VolumeRenderer training step."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _net(d_hidden, n_blocks=3, d_latent=64, hw=(8, 8), combine_layer=1000, sb=1, seed=0, beta=0.0, spade=False,
         combine_type="average"):
    from avr.conf import Conf, default_conf
    from avr.scene import synthetic_scene
    conf = default_conf()["model"]
    d = dict(conf)
    mlp = {"type": "resnet", "n_blocks": n_blocks, "d_hidden": d_hidden, "combine_layer": combine_layer,
           "beta": beta, "use_spade": spade, "combine_type": combine_type}
    d["mlp_coarse"], d["mlp_fine"] = dict(mlp), dict(mlp)
    d["encoder"] = {"backbone": "resnet34", "pretrained": False,
                    "num_layers": {64: 1, 128: 2, 256: 3, 512: 4}[d_latent]}
    net = synthetic_scene(DEV, seed, Conf(d), latent_hw=hw)
    if sb > 1:   # independent source views per scene (train.py encodes SB scenes)
        g = torch.Generator(device="cpu").manual_seed(seed + 7)
        lat = torch.randn(sb, d_latent, hw[0], hw[1], generator=g).to(DEV)
        net.encoder.set_latent(lat)
        net.num_objs = sb
        poses = net.poses.repeat(sb, 1, 1)
        poses[1:, 0, 3] += 0.1 * torch.arange(1, sb, device=DEV, dtype=torch.float32)
        net.poses = poses
        net.focal = net.focal.repeat(sb, 1)
        net.c = net.c.repeat(sb, 1)
    for p in net.parameters():
        p.requires_grad_(True)
    return net


def _points(sb, n, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    xyz = (torch.rand(sb, n, 3, generator=g) - 0.5) * 0.8
    vd = torch.nn.functional.normalize(torch.randn(sb, n, 3, generator=g), dim=-1)
    w = torch.randn(sb, n, 4, generator=g)
    return xyz.to(DEV), vd.to(DEV), w.to(DEV)


def _grads(net, xyz, vd, w, coarse, hip, latent_grad=False):
    net.hip_backward = hip
    net.zero_grad(set_to_none=True)
    lat = net.encoder.latent
    if latent_grad:
        lat = lat.detach().clone().requires_grad_(True)
        net.encoder.latent = lat
    out = net(xyz, coarse=coarse, viewdirs=vd)
    (out * w).sum().backward()
    mlp = net.mlp_coarse if coarse else net.mlp_fine
    gr = {n: p.grad.detach().clone() for n, p in mlp.named_parameters() if p.grad is not None}
    return out.detach(), gr, (lat.grad.detach().clone() if latent_grad else None)


def _compare(ga, gb, rtol):
    assert set(ga) == set(gb), (sorted(ga), sorted(gb))
    for k in ga:
        a, b = ga[k].float().cpu().numpy(), gb[k].float().cpu().numpy()
        scale = float(np.abs(b).max())
        err = float(np.abs(a - b).max())
        assert err <= rtol * scale + 1e-7, f"{k}: max err {err:.3e} vs max |grad| {scale:.3e}"


def _fp64(net, fn):
    """fn() with the net in float64 on the module path (PyTorch autograd): the
    exact reference both fp32 implementations are measured against. The net is
    converted back afterwards (float32 -> float64 -> float32 is exact)."""
    use_fused = net.use_fused
    net.double()
    net.use_fused = False
    try:
        return fn()
    finally:
        net.float()
        net.use_fused = use_fused


def _compare64(g_hip, g_t32, g_64, floor=3e-5):
    """fp32-equivalence of the HIP gradients: against the float64 reference,
    every parameter's max error (relative to its max |grad|) is within twice
    PyTorch fp32 autograd's own error, or within `floor`. Where a relu sits at
    ~1e-7 of zero, fp32 rounding can flip its mask (PyTorch's too): that error
    is the fp32 one, not the kernel's."""
    assert set(g_hip) == set(g_t32) == set(g_64), (sorted(g_hip), sorted(g_64))
    worst = 0.0
    for k in g_64:
        ref = g_64[k].double()
        s = float(ref.abs().max()) or 1.0
        eh = float((g_hip[k].double() - ref).abs().max()) / s
        et = float((g_t32[k].double() - ref).abs().max()) / s
        worst = max(worst, eh)
        assert eh <= 2.0 * et + floor, f"{k}: HIP err {eh:.2e} vs fp32 autograd err {et:.2e} (of max |grad| {s:.2e})"
    return worst


@pytest.mark.parametrize("d_hidden,n_blocks,combine_layer", [(64, 3, 1000), (128, 5, 3), (512, 3, 1000),
                                                          (512, 5, 3)])   # (512, 5, 3): conf/default_mv.conf
def test_field_train_grads_match_torch_autograd(d_hidden, n_blocks, combine_layer):
    from avr.field import _FieldTrain  # noqa: F401  (the path under test)
    d_latent = 512 if d_hidden == 512 else 64
    net = _net(d_hidden, n_blocks, d_latent, (16, 16) if d_hidden == 512 else (8, 8), combine_layer)
    xyz, vd, w = _points(1, 1000)
    out_h, g_h, _ = _grads(net, xyz, vd, w, True, hip=True)
    out_t, g_t, _ = _grads(net, xyz, vd, w, True, hip=False)
    np.testing.assert_allclose(out_h.cpu().numpy(), out_t.cpu().numpy(), atol=1e-4)
    expect = {"lin_in.weight", "lin_in.bias", "lin_out.weight", "lin_out.bias"}
    expect |= {f"blocks.{b}.fc_{i}.{t}" for b in range(n_blocks) for i in (0, 1) for t in ("weight", "bias")}
    expect |= {f"lin_z.{b}.{t}" for b in range(min(combine_layer, n_blocks)) for t in ("weight", "bias")}
    assert set(g_h) == expect
    _, g_d, _ = _fp64(net, lambda: _grads(net, xyz.double(), vd.double(), w.double(), True, hip=False))
    worst = _compare64(g_h, g_t, g_d)
    print(f"d_hidden {d_hidden}: worst HIP gradient error vs float64 {worst:.2e} of max |grad|")


@pytest.mark.parametrize("d_hidden,n_blocks,combine_layer,beta", [(64, 3, 1000, 1.0), (128, 5, 3, 2.0),
                                                                 (512, 5, 3, 1.5)])
def test_field_train_softplus_grads_match_fp64(d_hidden, n_blocks, combine_layer, beta):
    """ResnetFC(beta > 0): Softplus(beta) everywhere the ReLU would be (models.py:442-445, 536-537), trained on
    the fused kernels (ABI 11): the training forward's SAVE instantiation with the Softplus epilogues, the
    backward chain taking the activation's slope from the saved activations (1 - exp(-beta y))."""
    from avr.field import softplus_beta
    d_latent = 512 if d_hidden == 512 else 64
    net = _net(d_hidden, n_blocks, d_latent, (16, 16) if d_hidden == 512 else (8, 8), combine_layer, beta=beta)
    assert softplus_beta(net.mlp_coarse) == beta
    xyz, vd, w = _points(1, 900, seed=5)
    assert net.can_train_fused(xyz, vd)
    out_h, g_h, _ = _grads(net, xyz, vd, w, True, hip=True)
    out_t, g_t, _ = _grads(net, xyz, vd, w, True, hip=False)
    np.testing.assert_allclose(out_h.cpu().numpy(), out_t.cpu().numpy(), atol=1e-4)
    _, g_d, _ = _fp64(net, lambda: _grads(net, xyz.double(), vd.double(), w.double(), True, hip=False))
    worst = _compare64(g_h, g_t, g_d)
    print(f"softplus({beta}) d_hidden {d_hidden}: worst HIP gradient error vs float64 {worst:.2e} of max |grad|")


def test_field_train_multi_scene_fine_mlp_and_latent_grad():
    """SB = 2 scenes with their own latents and poses, the fine MLP, and the
    latent map's gradient (encoder training, stop_encoder_grad False)."""
    net = _net(128, 3, 64, (8, 8), sb=2)
    xyz, vd, w = _points(2, 700, seed=3)
    _, g_h, l_h = _grads(net, xyz, vd, w, False, hip=True, latent_grad=True)
    _, g_t, l_t = _grads(net, xyz, vd, w, False, hip=False, latent_grad=True)
    _, g_d, l_d = _fp64(net, lambda: _grads(net, xyz.double(), vd.double(), w.double(), False, hip=False,
                                             latent_grad=True))
    _compare64(dict(g_h, latent=l_h), dict(g_t, latent=l_t), dict(g_d, latent=l_d))


def test_field_train_ragged_and_empty():
    """Sample counts that are not multiples of the 64-sample workgroup, and zero."""
    net = _net(64, 2, 64)
    for n in (1, 63, 65, 130):
        xyz, vd, w = _points(1, n, seed=n)
        _, g_h, _ = _grads(net, xyz, vd, w, True, hip=True)
        _, g_t, _ = _grads(net, xyz, vd, w, True, hip=False)
        _, g_d, _ = _fp64(net, lambda: _grads(net, xyz.double(), vd.double(), w.double(), True, hip=False))
        _compare64(g_h, g_t, g_d)
    xyz, vd, w = _points(1, 0)
    net.hip_backward = True
    out = net(xyz, coarse=True, viewdirs=vd)
    (out * w).sum().backward()
    assert out.shape == (1, 0, 4)


def test_volume_renderer_training_step_hip_vs_torch():
    """One train.py step (renderers.VolumeRenderer module path, MSE on rgb
    coarse + fine) with the HIP field backward vs the PyTorch graph, every
    parameter within 1e-4 of its max |grad|."""
    from avr import ops
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS
    net = _net(128, 3, 64, (8, 8))
    R = 300
    g = torch.Generator(device="cpu").manual_seed(5)
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4).reshape(1, 1, 4, 4).expand(1, R, 4, 4).clone()
    c2w[..., 2, 3] = -1.3
    c2w = c2w.to(DEV)
    K = torch.tensor([INTRINSICS], device=DEV)
    gt = torch.rand(1, R, 3, generator=g).to(DEV)
    res = {}
    for hip in (True, False):
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        rend = VolumeRenderer(0.8, 1.8, 32, 16, 0, 0.01, True)
        rend.seed = 11
        rgb_c, rgb_f, depth, _ = rend(c2w, K, x_pix, net)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
        loss.backward()
        res[hip] = (float(loss.detach()), {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None})
    assert abs(res[True][0] - res[False][0]) < 1e-5
    # measured worst 3.6e-6 of max |grad| (no bin flipped); the bar leaves room for one flipped fine bin
    _compare(res[True][1], res[False][1], 1e-4)
    del ops


def test_volume_renderer_coarse_loss_hip_vs_torch():
    """The renderer-level step with the loss on the coarse rgb only (no fine-pass bin choice in
    the gradient path) on train.py's default_mv net: the HIP field backward and the PyTorch graph
    agree to fp32 accuracy, 5e-4 of max |grad| for every coarse-MLP parameter (measured 1.1e-4:
    PyTorch fp32 autograd's own error on this 512-wide net is of that order, the float64 comparisons
    above bound the HIP side), and the fine MLP gets no gradient on either path."""
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS
    net = _net(512, 5, 64, (8, 8), combine_layer=3)
    R = 300
    g = torch.Generator(device="cpu").manual_seed(6)
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4).reshape(1, 1, 4, 4).expand(1, R, 4, 4).clone()
    c2w[..., 2, 3] = -1.3
    c2w = c2w.to(DEV)
    K = torch.tensor([INTRINSICS], device=DEV)
    gt = torch.rand(1, R, 3, generator=g).to(DEV)
    res = {}
    for hip in (True, False):
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        rend = VolumeRenderer(0.8, 1.8, 64, 32, 0, 0.01, True)
        rend.seed = 12
        rgb_c, _, _, _ = rend(c2w, K, x_pix, net)
        ((rgb_c - gt) ** 2).mean().backward()
        res[hip] = {n: p.grad.clone() for n, p in net.named_parameters()
                    if p.grad is not None and float(p.grad.abs().max()) > 0}
    assert all(n.startswith("mlp_coarse.") for n in res[True]), sorted(res[True])
    _compare(res[True], res[False], 5e-4)


@pytest.mark.parametrize("waves,pipe", [(8, 0), (8, 1), (4, 0)])
@pytest.mark.parametrize("M,O,I,ld", [(1000, 512, 512, 512), (77, 64, 44, 48), (4096, 4, 512, 512), (0, 128, 64, 64),
                                      (5000, 512, 64, 64)])
def test_weight_grads_kernel_vs_fp64(M, O, I, ld, waves, pipe, monkeypatch):
    """avr_weight_grads (split-K x3 MFMA, transposed LDS reads) against an fp64
    G^T X, with ragged row counts, narrow layers and row strides wider than the
    layer, in a batch of two layers; every workgroup layout (8 waves with the
    split pipelined into the MFMAs or after them, 4 waves: AVR_WGRAD_PIPE /
    AVR_WGRAD_WAVES)."""
    from avr import ops
    monkeypatch.setenv("AVR_WGRAD_WAVES", str(waves))
    monkeypatch.setenv("AVR_WGRAD_PIPE", str(pipe))
    g = torch.Generator(device="cpu").manual_seed(M + O + I)
    G = (torch.randn(M, O, generator=g) * 1e-3 * (torch.rand(M, 1, generator=g) < 0.7)).to(DEV)
    Xb = torch.relu(torch.randn(M, ld, generator=g)).to(DEV)
    X = Xb[:, :I]
    G2 = (torch.randn(M, O, generator=g) * 5.0).to(DEV)
    mb = ops._max_bits if M else (lambda t: torch.zeros(1, dtype=torch.int32, device=DEV))
    lay = [(G, X, mb(G), mb(X), True), (G2, X, mb(G2), mb(X), False)]
    # the library's own K-split, and an explicit 5-way split (avr_weight_grads_reduce sums the partials)
    for res in (ops.weight_grads(lay, M), ops.weight_grads(lay, M, n_split=5 if M >= 5 else 1)):
        for (dW, db), GG in zip(res, (G, G2)):
            ref = (GG.double().t() @ X.double()).float().cpu().numpy()
            got = dW.cpu().numpy()
            scale = max(float(np.abs(ref).max()), 1e-30)
            assert float(np.abs(got - ref).max()) <= 2e-6 * scale + 1e-30, float(np.abs(got - ref).max()) / scale
        bref = G.double().sum(0).float().cpu().numpy()
        np.testing.assert_allclose(res[0][1].cpu().numpy(), bref, rtol=0,
                                   atol=2e-6 * float(np.abs(bref).max(initial=0)) + 1e-30)
        assert res[1][1] is None


@pytest.mark.parametrize("M,O,I,ld", [(1000, 512, 512, 512), (333, 64, 128, 136), (4096, 4, 512, 512)])
def test_weight_grads_bn_transform_vs_fp64(M, O, I, ld):
    """avr_weight_grads with the BatchNorm-relu input transform (ABI 12: X = relu((x - mu) * scale + shift) per
    column, the training-mode BN path's operand rebuilt from its pre-BN rows in the staging) against an fp64
    G^T X of the same fp32 operand -- built with the kernels' own expression (one fma per value) -- in a batch
    with an untransformed layer, ragged rows and a row stride wider than the layer."""
    from avr import ops
    g = torch.Generator(device="cpu").manual_seed(M + O + I)
    pre = (torch.randn(M, ld, generator=g) * 3.0 + 0.5).to(DEV)
    mu = (torch.randn(I, generator=g) * 0.3 + 0.5).to(DEV)
    scale = (torch.rand(I, generator=g) + 0.2).to(DEV)
    shift = (torch.randn(I, generator=g) * 0.2).to(DEV)
    X = torch.relu(torch.addcmul(shift, pre[:, :I] - mu, scale))       # fma((x - mu), scale, shift), then relu
    G = (torch.randn(M, O, generator=g) * 1e-3).to(DEV)
    G2 = torch.randn(M, O, generator=g).to(DEV)
    Xp = torch.relu(torch.randn(M, I, generator=g)).to(DEV)
    mb = ops._max_bits
    lay = [(G, pre[:, :I], mb(G), mb(X), True, (mu, scale, shift)), (G2, Xp, mb(G2), mb(Xp), True)]
    res = ops.weight_grads(lay, M)
    for (dW, db), GG, XX in zip(res, (G, G2), (X, Xp)):
        ref = (GG.double().t() @ XX.double()).float().cpu().numpy()
        got = dW.cpu().numpy()
        scale_r = max(float(np.abs(ref).max()), 1e-30)
        assert float(np.abs(got - ref).max()) <= 2e-6 * scale_r, float(np.abs(got - ref).max()) / scale_r
        bref = GG.double().sum(0).float().cpu().numpy()
        np.testing.assert_allclose(db.cpu().numpy(), bref, rtol=0, atol=2e-6 * float(np.abs(bref).max()))
    with pytest.raises(Exception, match="BatchNorm transform"):
        ops.weight_grads([(G, pre[:, :I], mb(G), mb(X), True, (mu, scale, shift[:-4]))], M)
    # ABI 14: the relu-only transform (input_relu) beside the BatchNorm one and an untransformed layer
    R = torch.relu(pre[:, :I])
    lay = [(G2, pre[:, :I], mb(G2), mb(R), False, "relu")] + lay
    res = ops.weight_grads(lay, M)
    for (dW, _), GG, XX in zip(res, (G2, G, G2), (R, X, Xp)):
        ref = (GG.double().t() @ XX.double()).float().cpu().numpy()
        scale_r = max(float(np.abs(ref).max()), 1e-30)
        assert float(np.abs(dW.cpu().numpy() - ref).max()) <= 2e-6 * scale_r
    assert res[0][1] is None


def test_latent_features_kernel_vs_grid_sample():
    """avr_latent_features (row-major pixel-aligned lookup) against the module's
    SpatialEncoder.index (torch grid_sample), two scenes, points inside and
    outside the source image (border padding)."""
    from avr import ops
    net = _net(64, 2, 64, (8, 8), sb=2)
    xyz, vd, _ = _points(2, 333, seed=9)
    xyz = xyz * 3.0   # some points project outside the source view
    ref, _ = net.mlp_inputs(xyz, vd)
    fused = net.fused()
    for sb in range(2):
        got = ops.latent_features(fused.view(sb), net.encoder.latent[sb], xyz[sb])
        np.testing.assert_allclose(got.cpu().numpy(), ref[sb * 333:(sb + 1) * 333].cpu().numpy(), atol=2e-6, rtol=1e-5)


def test_latent_features_grad_points_vs_autograd():
    """avr_latent_features_grad_points (ABI 12: d loss / d xyz through the pixel-aligned lookup) against autograd
    of the module's SpatialEncoder.index (torch grid_sample) in float64: two scenes, 512 channels, points inside
    and outside the source image (border padding: a clipped coordinate passes no gradient), random feature
    gradients; the fp32 autograd of the same lookup as the yardstick (2x its error + 1e-6 of max)."""
    from avr import _lib
    from avr._lib import ViewDesc
    net = _net(128, 2, 512, (16, 16), sb=2)
    xyz, vd, _ = _points(2, 700, seed=21)
    xyz = xyz * torch.where(torch.arange(700, device=DEV) % 3 == 0, 3.0, 1.0).reshape(1, 700, 1)
    g = torch.Generator().manual_seed(5)
    gfeat = torch.randn(2 * 700, 512, generator=g).to(DEV)
    fused = net.fused()
    hwc = fused.latent_hwc_all(net.encoder.latent)
    views = (ViewDesc * 2)(*[fused.view(sb) for sb in range(2)])
    got = torch.empty(2 * 700, 3, device=DEV)
    _lib.call("avr_latent_features_grad_points", views, 2, _lib.ptr(hwc), 512, _lib.ptr(xyz.contiguous()), 700,
              _lib.ptr(gfeat), _lib.ptr(got), _lib.stream_of(got))

    def autograd(dtype):
        x = xyz.to(dtype).clone().requires_grad_(True)
        feat, _ = net.mlp_inputs(x, vd.to(dtype))
        return torch.autograd.grad(feat, x, gfeat.to(dtype))[0].reshape(-1, 3)

    ref32 = autograd(torch.float32)
    with torch.no_grad():
        net.double()
    try:
        ref64 = autograd(torch.float64)
    finally:
        net.float()
    s = float(ref64.abs().max())
    eh = float((got.double() - ref64).abs().max())
    et = float((ref32.double() - ref64).abs().max())
    assert eh <= 2.0 * et + 1e-6 * s, (eh, et, s)
    print(f"grad points: HIP err {eh / s:.2e}, torch fp32 err {et / s:.2e} of max {s:.3e}")


@pytest.mark.parametrize("n_tables", [1, 3])
def test_latent_tables_grad_points_vs_fp64(n_tables):
    """avr_latent_tables_grad_points (ABI 15): the lookup's position gradient from the per-texel lin_z tables, sum_b
    Gz[b] . interp(W_z[b] latent, p), against float64 autograd of the module's lookup with the feature gradient
    sum_b Gz[b] W_z[b] (the same quantity: both maps are linear); two scenes, points in and outside the image,
    gradient rows with a leading dimension past d_hidden. The fp32 autograd of the feature path is the yardstick."""
    from avr import _lib
    from avr._lib import ViewDesc
    H, C, M = 256, 512, 700
    net = _net(128, 2, C, (16, 16), sb=2)
    xyz, vd, _ = _points(2, M, seed=23)
    xyz = xyz * torch.where(torch.arange(M, device=DEV) % 3 == 0, 3.0, 1.0).reshape(1, M, 1)
    g = torch.Generator().manual_seed(6)
    Wz = [torch.randn(H, C, generator=g).to(DEV) * 0.05 for _ in range(n_tables)]
    ld = H + 8
    Gbuf = [torch.randn(2 * M, ld, generator=g).to(DEV) for _ in range(n_tables)]
    Gz = [b[:, :H] for b in Gbuf]
    lat = net.encoder.latent                                    # (2, C, h, w)
    tabs = torch.stack([torch.stack([(Wz[b] @ lat[s].reshape(C, -1)).t() for b in range(n_tables)])
                        for s in range(2)]).contiguous()        # (2, n_tables, h*w, H)
    fused = net.fused()
    views = (ViewDesc * 2)(*[fused.view(sb) for sb in range(2)])
    got = torch.empty(2 * M, 3, device=DEV)
    grads = (ctypes.c_void_p * n_tables)(*[t.data_ptr() for t in Gz])
    _lib.call("avr_latent_tables_grad_points", views, 2, _lib.ptr(tabs), tabs.stride(0), tabs.stride(1), n_tables, H,
              _lib.ptr(xyz.contiguous()), M, grads, ld, _lib.ptr(got), _lib.stream_of(got))

    def autograd(dtype):
        x = xyz.to(dtype).clone().requires_grad_(True)
        feat, _ = net.mlp_inputs(x, vd.to(dtype))
        gfeat = sum(Gz[b].to(dtype) @ Wz[b].to(dtype) for b in range(n_tables))
        return torch.autograd.grad(feat, x, gfeat)[0].reshape(-1, 3)

    ref32 = autograd(torch.float32)
    with torch.no_grad():
        net.double()
    try:
        ref64 = autograd(torch.float64)
    finally:
        net.float()
    s = float(ref64.abs().max())
    eh = float((got.double() - ref64).abs().max())
    et = float((ref32.double() - ref64).abs().max())
    assert eh <= 2.0 * et + 1e-6 * s, (eh, et, s)
    print(f"tables grad points ({n_tables}): HIP err {eh / s:.2e}, torch fp32 err {et / s:.2e} of max {s:.3e}")


@pytest.mark.parametrize("accumulate", [0, 1])
def test_zfeature_grad_points_vs_fp64(accumulate):
    """avr_zfeature_grad_points (ABI 16): the points' gradient through z_feature (rotation, positional encoding
    with include_input; models.py:753-794, :41-87) given d loss / d z_feature's encoded columns, against float64
    autograd of the module's z_features; two scenes with different poses, points far outside the unit cube (large
    f_k z), rows with a leading dimension past 3 + 6F; accumulate=1 adds to what grad_xyz holds."""
    from avr import _lib
    from avr._lib import ViewDesc
    net = _net(64, 2, 64, (8, 8), sb=2)
    M = 600
    xyz, vd, _ = _points(2, M, seed=29)
    xyz = xyz * torch.where(torch.arange(M, device=DEV) % 4 == 0, 5.0, 1.0).reshape(1, M, 1)
    F = net.code.num_freqs
    n_pe = 3 + 6 * F
    g = torch.Generator().manual_seed(8)
    ld = net.d_in + 5
    gbuf = torch.randn(2 * M, ld, generator=g).to(DEV)
    gzf = gbuf[:, :net.d_in]                                     # the viewdir columns carry no position gradient
    base = torch.randn(2 * M, 3, generator=g).to(DEV)
    got = base.clone()
    fused = net.fused()
    views = (ViewDesc * 2)(*[fused.view(sb) for sb in range(2)])
    _lib.call("avr_zfeature_grad_points", views, 2, _lib.ptr(xyz.contiguous()), M, _lib.ptr(gbuf), ld, F,
              fused.dims(net.mlp_coarse).freq_factor, accumulate, _lib.ptr(got), _lib.stream_of(got))
    if accumulate:
        got = got - base

    def autograd(dtype):
        x = xyz.to(dtype).clone().requires_grad_(True)
        zf = net.z_features(x, vd.to(dtype))
        return torch.autograd.grad(zf, x, gzf.to(dtype))[0].reshape(-1, 3)

    ref32 = autograd(torch.float32)
    with torch.no_grad():
        net.double()
    try:
        ref64 = autograd(torch.float64)
    finally:
        net.float()
    s = float(ref64.abs().max())
    eh = float((got.double() - ref64).abs().max())
    et = float((ref32.double() - ref64).abs().max())
    assert n_pe + 3 == net.d_in and eh <= 2.0 * et + 1e-6 * s, (eh, et, s)
    print(f"z_feature grad points: HIP err {eh / s:.2e}, torch fp32 err {et / s:.2e} of max {s:.3e}")


@pytest.mark.parametrize("via", ["tables", "features", "zf_autograd"])
def test_field_train_point_gradient_paths(via, monkeypatch):
    """The band points' lookup gradient on the fused training path both ways (ABI 15's tables path, the default,
    and the feature-gradient path it replaced, AVR_POINT_GRAD_VIA_FEATURES=1), and z_feature's part both ways (ABI
    16's avr_zfeature_grad_points, the default, and torch autograd, AVR_POINT_ZF_VIA_AUTOGRAD=1), against float64
    autograd."""
    monkeypatch.setenv("AVR_POINT_GRAD_VIA_FEATURES", "1" if via == "features" else "0")
    monkeypatch.setenv("AVR_POINT_ZF_VIA_AUTOGRAD", "1" if via == "zf_autograd" else "0")
    net = _net(512, 5, 512, (16, 16), 3)
    xyz0, vd, w = _points(1, 700, seed=19)
    res = {}
    for hip in (True, False, "fp64"):
        def run(hip=hip):
            xyz = (xyz0.double() if hip == "fp64" else xyz0.clone()).requires_grad_(True)
            v, ww = (vd.double(), w.double()) if hip == "fp64" else (vd, w)
            _, g, _ = _grads(net, xyz, v, ww, True, hip=hip is True)
            return dict(g, xyz=xyz.grad.detach().clone())
        res[hip] = _fp64(net, run) if hip == "fp64" else run()
    _compare64(res[True], res[False], res["fp64"])


def test_latent_features_grad_points_on_source_camera_plane():
    """A point on the source camera's plane (camera z = 0: the projection is infinite, the lookup clipped to the
    border) gets exactly the clip's zero position gradient from the lookup, not 0 * inf = NaN. The r04q adaptive
    train.py bench run failed on one such band point (world z = -1.3f with the source camera at z = -1.3;
    profiles/r05d_adaptive_nan_probe.log); torch's autograd of the reference lookup gives NaN there."""
    from avr import _lib
    from avr._lib import ViewDesc
    net = _net(64, 2, 64, (8, 8), sb=2)
    xyz, vd, _ = _points(2, 256, seed=23)
    plane = torch.arange(256, device=DEV) % 2 == 0                       # every other point on the plane
    tz = net.poses[:, 2, 3].reshape(2, 1)                                # R = I: camera z = world z + t_z
    xyz[..., 2] = torch.where(plane, -tz, xyz[..., 2])
    assert bool((xyz[..., 2][:, plane] + tz == 0).all())
    gfeat = torch.randn(2 * 256, 64, generator=torch.Generator().manual_seed(6)).to(DEV)
    fused = net.fused()
    hwc = fused.latent_hwc_all(net.encoder.latent)
    views = (ViewDesc * 2)(*[fused.view(sb) for sb in range(2)])
    got = torch.empty(2 * 256, 3, device=DEV)
    _lib.call("avr_latent_features_grad_points", views, 2, _lib.ptr(hwc), 64, _lib.ptr(xyz.contiguous()), 256,
              _lib.ptr(gfeat), _lib.ptr(got), _lib.stream_of(got))
    got = got.reshape(2, 256, 3)
    assert bool(torch.isfinite(got).all())
    assert bool((got[:, plane] == 0).all())
    x = xyz.clone().requires_grad_(True)
    feat, _ = net.mlp_inputs(x, vd)
    ref = torch.autograd.grad(feat, x, gfeat)[0]
    assert not bool(torch.isfinite(ref[:, plane]).all())                 # the reference's autograd: 0 * inf
    np.testing.assert_allclose(got[:, ~plane].cpu().numpy(), ref[:, ~plane].cpu().numpy(), rtol=1e-4,
                               atol=1e-5 * float(ref[:, ~plane].abs().max()))


@pytest.mark.parametrize("d_hidden,latent_grad,stop", [(64, False, False), (512, False, False), (512, True, False),
                                                    (64, False, True), (512, False, True)])
def test_field_train_point_gradient(d_hidden, latent_grad, stop):
    """Points that carry a gradient (the adaptive renderer's band samples,
    renderers.py:492-508): d loss / d xyz through PE, rotation, projection and
    the bilinear latent lookup, with the parameter gradients, vs PyTorch autograd.
    stop: train.py --stop_encoder_grad (train.py:279): the looked-up latent is detached
    (models.py:810-811), so the points get z_feature's gradient only."""
    d_latent = 512 if d_hidden == 512 else 64
    net = _net(d_hidden, 3, d_latent, (16, 16) if d_hidden == 512 else (8, 8))
    net.stop_encoder_grad = stop
    xyz0, vd, w = _points(1, 500, seed=17)
    res = {}
    for hip in (True, False, "fp64"):
        def run(hip=hip):
            xyz = (xyz0.double() if hip == "fp64" else xyz0.clone()).requires_grad_(True)
            v, ww = (vd.double(), w.double()) if hip == "fp64" else (vd, w)
            _, g, l = _grads(net, xyz, v, ww, True, hip=hip is True, latent_grad=latent_grad)
            out = dict(g, xyz=xyz.grad.detach().clone())
            if latent_grad:
                out["latent"] = l
            return out
        res[hip] = _fp64(net, run) if hip == "fp64" else run()
    _compare64(res[True], res[False], res["fp64"])
    if stop:   # the lookup's position gradient is really cut: it is not the stop_encoder_grad=False gradient
        net.stop_encoder_grad = False
        xyz = xyz0.clone().requires_grad_(True)
        _grads(net, xyz, vd, w, True, hip=True)
        assert float((xyz.grad - res[True]["xyz"]).abs().max()) > 1e-3 * float(xyz.grad.abs().max())


def test_encoder_training_step_hip_vs_torch():
    """train.py:68 + :108-114 end to end with the real encoder: net.encode on
    the source image, a VolumeRenderer step, loss.backward(): the gradient
    reaches the ResNet34 (through the HIP field's latent gradient) and equals
    PyTorch autograd of the same module; inference after encode() runs the
    fused field on the encoder's latent."""
    from avr.conf import Conf, default_conf
    from avr.models import NewPixelNeRFNet
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS
    d = dict(default_conf()["model"])
    mlp = {"type": "resnet", "n_blocks": 3, "d_hidden": 128}
    d["mlp_coarse"], d["mlp_fine"] = dict(mlp), dict(mlp)
    d["encoder"] = {"backbone": "resnet34", "pretrained": False, "num_layers": 2}
    torch.manual_seed(0)
    net = NewPixelNeRFNet(Conf(d)).to(DEV)
    g = torch.Generator(device="cpu").manual_seed(2)
    img = (torch.rand(1, 1, 3, 64, 64, generator=g) * 2 - 1).to(DEV)
    pose = torch.eye(4).reshape(1, 1, 4, 4).clone()
    pose[..., 2, 3] = -1.3
    pose = pose.to(DEV)
    R = 256
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    c2w = pose[0].expand(1, R, 4, 4)
    K = torch.tensor([INTRINSICS], device=DEV)
    gt = torch.rand(1, R, 3, generator=g).to(DEV)
    res = {}
    for hip in (True, False):
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        net.encode(img, pose, torch.tensor(64.0, device=DEV), c=torch.tensor(32.0, device=DEV))
        assert net.encoder.latent.shape == (1, 128, 32, 32) and net.encoder.latent.requires_grad
        rend = VolumeRenderer(0.8, 1.8, 32, 16, 0, 0.01, True)
        rend.seed = 3
        rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
        loss.backward()
        res[hip] = {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None}
    assert "encoder.model.conv1.weight" in res[True]
    _compare(res[True], res[False], 5e-4)   # measured 4.5e-5 of max |grad|
    with torch.no_grad():
        net.encode(img, pose, torch.tensor(64.0, device=DEV), c=torch.tensor(32.0, device=DEV))
        xyz = (torch.rand(1, 3000, 3, generator=g) - 0.5).to(DEV)
        vd = torch.nn.functional.normalize(torch.randn(1, 3000, 3, generator=g), dim=-1).to(DEV)
        assert net.can_fuse(xyz)
        a = net(xyz, coarse=True, viewdirs=vd)
        b = net.forward_torch(xyz, coarse=True, viewdirs=vd)
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=5e-5, rtol=1e-4)


@pytest.mark.parametrize("d_hidden,d_latent,hw,combine", [(512, 512, (16, 20), 3), (128, 64, (7, 9), 1000),
                                                          (64, 256, (5, 13), 2)])
def test_latent_tables_vs_fp64(d_hidden, d_latent, hw, combine):
    """The per-texel lin_z tables (table[t][texel] = lin_z[t].weight . latent[:, texel], the
    bias folded into the layer before): the x3 field's tables (table_x3_kernel, split-fp16
    GEMM) and the fp32 field's (exact fp32 MFMA products) against float64, ragged texel
    counts (HW not a multiple of the 64-texel tile)."""
    from avr.field import FusedField
    net = _net(d_hidden, n_blocks=3, d_latent=d_latent, hw=hw, combine_layer=combine)
    lat = net.encoder.latent[0].detach().double().reshape(d_latent, -1)
    for coarse in (True, False):
        mlp = net.mlp_coarse if coarse else net.mlp_fine
        ref = torch.stack([(l.weight.detach().double() @ lat).t() for l in mlp.lin_z]).cpu().numpy()
        for precision in ("x3", "fp32"):
            f = FusedField(net, precision)
            # the training path's tables (split-fp16 GEMM) and inference's (exact fp32 products)
            for got, bar in ((f.tables_batch(coarse, 1, fast=True)[0], 1e-5), (f.table(coarse, 0), 2e-6)):
                got = got[:len(mlp.lin_z)].double().cpu().numpy()
                assert got.shape == ref.shape
                err = float(np.abs(got - ref).max()) / float(np.abs(ref).max())
                assert err <= bar, (precision, bar, err)


def test_batched_latent_features_and_tables_match_per_scene():
    """avr_latent_features_batch and avr_field_latent_table_batch (every scene of a
    training batch in one launch) give the per-scene launches' results bit for bit."""
    from avr import _lib, ops
    from avr._lib import call, ptr, stream_of
    from avr.field import FusedField
    net = _net(512, 5, 64, (9, 11), combine_layer=3, sb=3)
    xyz, _, _ = _points(3, 777, seed=4)
    f = FusedField(net, "x3")
    lat = net.encoder.latent.detach()
    SB, C = lat.shape[:2]
    per = torch.cat([ops.latent_features(f.view(s), lat[s], xyz[s]) for s in range(SB)])
    got = torch.empty_like(per)
    views = (_lib.ViewDesc * SB)(*[f.view(s) for s in range(SB)])
    hwc = f.latent_hwc_all(lat)
    call("avr_latent_features_batch", views, SB, ptr(hwc), C, ptr(xyz.contiguous()), xyz.shape[1], ptr(got),
         stream_of(got))
    assert torch.equal(per, got)
    for coarse in (True, False):
        batch = f.tables_batch(coarse, SB)
        for s in range(SB):
            assert torch.equal(batch[s], f.table(coarse, s)), (coarse, s)
        # the split-fp16 tables: one launch over the scenes = one launch per scene
        fast = f.tables_batch(coarse, SB, fast=True)
        entry = f.packed(coarse)
        saved = entry.dims.precision
        entry.dims.precision = _lib.FIELD_X3
        try:
            for s in range(SB):
                one = torch.empty_like(fast[s])
                H, W = lat.shape[2:]
                call("avr_field_latent_table", ctypes.byref(entry.dims), ptr(entry.packed), ptr(lat[s].contiguous()),
                     H, W, ptr(one), stream_of(one))
                assert torch.equal(fast[s], one), (coarse, s)
        finally:
            entry.dims.precision = saved


def test_training_forward_stores_z_feature():
    """avr_field_fwd_points_train's z_feature rows (ABI 9: lin_in's weight-gradient operand, so the backward
    does not recompute the positional encoding) against the module's z_features (PE / rotation in torch),
    two scenes, a ragged point count, the padding columns zero, and their max |.|."""
    from avr import _lib
    from avr._lib import ViewDesc, call, ptr, stream_of
    from avr.field import FusedField
    net = _net(128, 3, 64, (8, 8), sb=2)
    xyz, vd, _ = _points(2, 333, seed=8)
    f = FusedField(net, "x3")
    entry = f.packed(True)
    dims = entry.dims
    SB, B = 2, 333
    H, nb = dims.d_hidden, dims.n_blocks
    act_n, mask_n = ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.check(_lib.load().avr_field_train_sizes(ctypes.byref(dims), SB, B, ctypes.byref(act_n),
                                                 ctypes.byref(mask_n)), "avr_field_train_sizes")
    out = torch.empty(SB * B, 4, device=DEV)
    act = torch.empty(act_n.value, device=DEV)
    mask = torch.empty(max(mask_n.value, 1), device=DEV, dtype=torch.int32)
    act_max = torch.zeros(2 * nb + 2, device=DEV, dtype=torch.int32)
    zs = dims.d_in + (-dims.d_in) % 4 + 4                        # two more padding columns than needed
    zf = torch.full((SB * B, zs), float("nan"), device=DEV)
    views = (ViewDesc * SB)(*[f.view(s) for s in range(SB)])
    tables = f.tables_batch(True, SB, fast=True)
    saved = dims.precision
    dims.precision = _lib.FIELD_X3
    try:
        call("avr_field_fwd_points_train", ctypes.byref(dims), views, SB, ptr(entry.packed), ptr(tables),
             ptr(xyz.contiguous()), ptr(vd.contiguous()), B, ptr(out), ptr(act), SB * B, ptr(mask), ptr(act_max),
             ptr(zf), zs, ctypes.c_void_p(act_max.data_ptr() + 4 * (2 * nb + 1)), stream_of(out))
    finally:
        dims.precision = saved
    with torch.no_grad():
        ref = net.z_features(xyz, vd).float()
    d_in = dims.d_in
    assert ref.shape == (SB * B, d_in)
    np.testing.assert_allclose(zf[:, :d_in].cpu().numpy(), ref.cpu().numpy(), atol=2e-6, rtol=1e-6)
    assert bool((zf[:, d_in:] == 0).all())
    zmax = act_max[2 * nb + 1:].view(torch.float32)
    assert float(zmax) == float(zf[:, :d_in].abs().max())


def test_fused_optimizer_step_reaches_the_field():
    """A fused optimizer (torch.optim.Adam(fused=True)) updates the parameters in one kernel without advancing
    their version counters: the packed blobs and tables must still be rebuilt after its step (the optimizer-step
    generation in FusedField's cache keys), on the training path and the inference path alike -- checked against
    PyTorch's forward of the same module after two large steps."""
    net = _net(64, 3, 64, (8, 8))
    xyz, vd, w = _points(1, 300, seed=29)
    opt = torch.optim.Adam(net.mlp_coarse.parameters(), lr=5e-2, fused=True)
    for _ in range(3):
        opt.zero_grad()
        out = net(xyz, coarse=True, viewdirs=vd)
        with torch.no_grad():
            ref = net.forward_torch(xyz, True, vd)
        np.testing.assert_allclose(out.detach().cpu().numpy(), ref.cpu().numpy(), atol=1e-4)
        (out * w).sum().backward()
        opt.step()
    with torch.no_grad():
        assert net.can_fuse(xyz)
        a = net(xyz, coarse=True, viewdirs=vd)
        b = net.forward_torch(xyz, True, vd)
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=1e-4)


def test_weight_grads_specs_bit_equal_to_tensor_api():
    """ops.weight_grads_specs (the layers as offsets into caller-owned buffers: _FieldTrain.backward's route) and
    ops.weight_grads (tensor views, checked) are one launch sequence: bit-equal dW / db on layers cut from one
    (layers, M, H) buffer, a narrow layer and one without bias."""
    from avr import ops
    M, H, nl = 777, 128, 3
    g = torch.Generator(device="cpu").manual_seed(5)
    G = (torch.randn(nl, M, H, generator=g) * 1e-3).to(DEV)
    A = torch.relu(torch.randn(nl, M, H, generator=g)).to(DEV)
    Z = torch.randn(M, 44, generator=g).to(DEV)
    gm = torch.stack([ops._max_bits(G[k])[0] for k in range(nl)])
    am = torch.stack([ops._max_bits(A[k])[0] for k in range(nl)] + [ops._max_bits(Z)[0]])
    lay = [(G[k], A[k], gm[k:k + 1], am[k:k + 1], True) for k in range(nl)]
    lay.append((G[0], Z, gm[0:1], am[nl:nl + 1], False))
    ref = ops.weight_grads(lay, M)
    sz, Gp, Ap = M * H * 4, G.data_ptr(), A.data_ptr()
    specs = [(Gp + k * sz, H, Ap + k * sz, H, H, H, gm.data_ptr() + 4 * k, am.data_ptr() + 4 * k, True, None,
              None, None, 0) for k in range(nl)]
    specs.append((Gp, H, Z.data_ptr(), 44, H, 44, gm.data_ptr(), am.data_ptr() + 4 * nl, False, None, None, None,
                  0))
    got = ops.weight_grads_specs(specs, M, DEV, ops.stream_of(G))
    for (dw0, db0), (dw1, db1) in zip(ref, got):
        assert torch.equal(dw0, dw1)
        assert (db0 is None) == (db1 is None) and (db0 is None or torch.equal(db0, db1))


def test_repack_after_in_place_update_matches_fresh_pack():
    """FusedField.packed() reuses the last build's weight pointers when an optimizer step updated the parameters in
    place (only the pack launch reruns): the field it evaluates must equal, bit for bit, that of a FusedField
    packing from scratch (the blobs' unwritten padding is not compared), and a replaced parameter tensor must be
    seen."""
    from avr.field import FusedField
    net = _net(64, 3, 64, (8, 8))
    fused = net.fused()
    opt = torch.optim.Adam(net.mlp_coarse.parameters(), lr=1e-2)
    xyz, vd, w = _points(1, 200, seed=31)
    for _ in range(3):
        opt.zero_grad()
        (net(xyz, coarse=True, viewdirs=vd) * w).sum().backward()
        opt.step()

    def both():
        with torch.no_grad():
            return (fused.forward_points(xyz, vd, True),
                    FusedField(net, fused.precision).forward_points(xyz, vd, True))
    a, b = both()
    assert torch.equal(a, b)
    with torch.no_grad():   # a new tensor object for one parameter: new pointers, a full rebuild
        net.mlp_coarse.lin_out.weight = torch.nn.Parameter(net.mlp_coarse.lin_out.weight * 2.0)
    a2, b2 = both()
    assert torch.equal(a2, b2) and not torch.equal(a2, a)
