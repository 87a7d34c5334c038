"""Autograd of the LSTM march on HIP (avr.renderers._MarchTrain: avr_raymarch_train / avr_raymarch_bwd) --
train.py's AdaptiveVolumeRenderer / Raymarcher step (renderers.py:413-432, :320-343; train.py:268-273)
against PyTorch autograd of the reference loop (LSTMCell on grid_sample'd features, the clamp hook on every
h gradient): the march alone (world points, every LSTM / out_layer / W_ih gradient, the latent's gradient)
against a float64 run of the same loop, and a whole AdaptiveVolumeRenderer training step."""
import numpy as np
import pytest
import torch

from test_gpu_train import _net

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _march_inputs(sb, R, seed=0, along_x=False):
    """along_x: cameras looking down the world x axis (|rd_x| ~ 1). AdaptiveVolumeRenderer's band centre is
    (x - ro)_x / rd_x (renderers.py:490, quirk kept): with rd_x near 0 (cameras looking down z, as below by
    default) its gradient is amplified by 1 / rd_x and a whole-step comparison of two fp32 paths measures
    that amplification of rounding noise, not the kernels."""
    from avr import ops
    from avr.scene import INTRINSICS
    g = torch.Generator().manual_seed(seed)
    x_pix = torch.rand(sb, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4).reshape(1, 1, 4, 4).repeat(sb, R, 1, 1)
    if along_x:   # rotation about y by 90 degrees: the camera's -z axis is the world's -x axis
        c2w[..., :3, :3] = torch.tensor([[0.0, 0.0, 1.0], [0.0, 1.0, 0.0], [-1.0, 0.0, 0.0]])
        c2w[..., 0, 3] = 1.3 + 0.1 * torch.arange(sb).reshape(sb, 1)
        c2w[..., 2, 3] = 0.05 * torch.randn(sb, R, generator=g)
    else:
        c2w[..., 2, 3] = -1.3 - 0.1 * torch.arange(sb).reshape(sb, 1)
        c2w[..., 0, 3] = 0.05 * torch.randn(sb, R, generator=g)
    K = torch.tensor([INTRINSICS] * sb, device=DEV)
    ros, rds, _ = ops.world_rays(x_pix, K, c2w.to(DEV))
    init = (0.8 + 0.05 * torch.randn(sb, R, 1, generator=g)).to(DEV)
    return ros, rds, init, x_pix, c2w.to(DEV), K


def _renderer(C, steps=10, cls="adaptive", seed=3):
    from avr.renderers import AdaptiveVolumeRenderer, Raymarcher
    torch.manual_seed(seed)
    r = AdaptiveVolumeRenderer(C, steps, 0.15, 20, True) if cls == "adaptive" else Raymarcher(C, steps)
    return r.to(DEV)


def _march_grads(rend, net, ros, rds, init, w, hip, latent_grad=True):
    net.hip_backward = hip
    rend.zero_grad(set_to_none=True)
    lat = net.encoder.latent.detach().clone().requires_grad_(latent_grad)
    net.encoder.latent = lat
    world = rend.march(ros, rds, init, net)
    (world * w).sum().backward()
    g = {n: p.grad.detach().clone() for n, p in rend.named_parameters()}
    if latent_grad:
        g["latent"] = lat.grad.detach().clone()
    return world.detach(), g, rend.last_path


@pytest.mark.parametrize("sb,R,steps", [(1, 300, 10), (3, 257, 10), (2, 64, 1)])
def test_march_autograd_matches_fp64(sb, R, steps):
    net = _net(64, 2, 64, (8, 8), sb=sb)
    rend = _renderer(64, steps)
    ros, rds, init, *_ = _march_inputs(sb, R, seed=sb)
    # loss weights large enough that some h gradients exceed 10: the reference's clamp hook engages
    w = 300.0 * torch.randn(sb, R, 3, generator=torch.Generator().manual_seed(7)).to(DEV)
    wh, gh, path = _march_grads(rend, net, ros, rds, init, w, hip=True)
    assert path == "hip_train"
    wt, gt, path_t = _march_grads(rend, net, ros, rds, init, w, hip=False)
    assert path_t == "module"
    np.testing.assert_allclose(wh.cpu().numpy(), wt.cpu().numpy(), atol=1e-3)   # sanity; the bar is the fp64 one
    # float64 reference of the reference loop
    net.double()
    rend.double()
    net.use_fused = False
    try:
        wd, gd, _ = _march_grads(rend, net, ros.double(), rds.double(), init.double(), w.double(), hip=False)
    finally:
        net.float()
        rend.float()
        net.use_fused = True
    ew = float((wh.double() - wd).abs().max())
    et_w = float((wt.double() - wd).abs().max())
    assert ew <= 2.0 * et_w + 1e-5, (ew, et_w)
    assert set(gh) == set(gt) == set(gd)
    worst = 0.0
    for k in gd:
        ref = gd[k].double()
        s = float(ref.abs().max()) or 1.0
        eh = float((gh[k].double() - ref).abs().max()) / s
        et = float((gt[k].double() - ref).abs().max()) / s
        worst = max(worst, eh)
        assert eh <= 2.0 * et + 1e-4, f"{k}: HIP err {eh:.2e} vs fp32 autograd err {et:.2e} of max |grad| {s:.2e}"
    print(f"march sb={sb} R={R} steps={steps}: worst HIP gradient error vs float64 {worst:.2e}")


@pytest.mark.parametrize("sb,R", [(1, 300), (2, 129)])
def test_march_autograd_stop_encoder_grad_matches_fp64(sb, R):
    """train.py --stop_encoder_grad (train.py:279): phi(return_features=True) returns a detached latent
    (models.py:810-811), so no gradient reaches the points through the lookup; W_ih, the LSTM and out_layer still
    get theirs. The HIP march (avr_raymarch_bwd with the position gradient off) against a float64 run of the
    reference loop, and against the march with the flag off (the lookup term must be gone)."""
    net = _net(64, 2, 64, (8, 8), sb=sb)
    net.stop_encoder_grad = True
    rend = _renderer(64, 10)
    ros, rds, init, *_ = _march_inputs(sb, R, seed=5 + sb)
    w = 300.0 * torch.randn(sb, R, 3, generator=torch.Generator().manual_seed(9)).to(DEV)
    wh, gh, path = _march_grads(rend, net, ros, rds, init, w, hip=True, latent_grad=False)
    assert path == "hip_train"
    wt, gt, _ = _march_grads(rend, net, ros, rds, init, w, hip=False, latent_grad=False)
    net.double()
    rend.double()
    net.use_fused = False
    try:
        _, gd, _ = _march_grads(rend, net, ros.double(), rds.double(), init.double(), w.double(), hip=False,
                                latent_grad=False)
    finally:
        net.float()
        rend.float()
        net.use_fused = True
    assert set(gh) == set(gt) == set(gd)
    for k in gd:
        ref = gd[k].double()
        s = float(ref.abs().max()) or 1.0
        eh = float((gh[k].double() - ref).abs().max()) / s
        et = float((gt[k].double() - ref).abs().max()) / s
        assert eh <= 2.0 * et + 1e-4, f"{k}: HIP err {eh:.2e} vs fp32 autograd err {et:.2e} of max |grad| {s:.2e}"
    net.stop_encoder_grad = False
    _, gon, _ = _march_grads(rend, net, ros, rds, init, w, hip=True, latent_grad=False)
    k = "lstm.weight_hh"
    assert float((gon[k] - gh[k]).abs().max()) > 1e-3 * float(gd[k].abs().max()), "lookup gradient not cut"


def test_march_backward_on_source_camera_plane_is_finite():
    """Rays that run inside the source camera's plane (every march point at camera z = 0: the lookup is clipped,
    1 / z infinite) get finite gradients: the clipped lookup passes exactly zero (avr_raymarch_bwd's lookup_grad),
    as avr_latent_features_grad_points does (test_gpu_train.py); a NaN would reach out_layer and the LSTM."""
    sb, R = 1, 64
    net = _net(64, 2, 64, (8, 8), sb=sb)
    rend = _renderer(64, 4)
    tz = float(net.poses[0, 2, 3])
    g = torch.Generator().manual_seed(3)
    ros = torch.zeros(sb, R, 3)
    ros[..., 0] = torch.rand(sb, R, generator=g) - 0.5
    ros[..., 1] = torch.rand(sb, R, generator=g) - 0.5
    ros[..., 2] = -tz                                                    # world z = -t_z: camera z = 0 (R = I)
    ang = torch.rand(sb, R, generator=g) * 6.28
    rds = torch.stack([torch.cos(ang), torch.sin(ang), torch.zeros_like(ang)], -1)   # inside the plane
    init = 0.8 + 0.05 * torch.randn(sb, R, 1, generator=g)
    w = torch.randn(sb, R, 3, generator=g).to(DEV)
    world, grads, path = _march_grads(rend, net, ros.to(DEV), rds.to(DEV), init.to(DEV), w, hip=True)
    assert path == "hip_train"
    assert bool(torch.isfinite(world).all())
    bad = [k for k, v in grads.items() if not bool(torch.isfinite(v).all())]
    assert not bad, bad


def test_adaptive_renderer_training_step_hip_vs_torch():
    """AdaptiveVolumeRenderer (conf adaptive_renderer: 10 steps, band of 20, epsilon 0.15) training step on
    the default_mv-shaped net (combine_layer 3): loss and every gradient (net, LSTM, out_layer) of the HIP
    march + HIP field against PyTorch autograd of the same modules."""
    sb, R = 2, 256
    net = _net(128, 5, 64, (8, 8), combine_layer=3, sb=sb)
    rend = _renderer(64)
    _, _, _, x_pix, c2w, K = _march_inputs(sb, R, seed=11, along_x=True)
    g = torch.Generator().manual_seed(12)
    noise = {"initial_distance": (0.8 + 0.05 * torch.randn(sb, R, 1, generator=g)).to(DEV),
             "band": torch.rand(sb, R, 20, generator=g).to(DEV)}
    gt = torch.rand(sb, R, 3, generator=g).to(DEV)

    def step(hip, eps=0.0):
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        rend.zero_grad(set_to_none=True)
        nz = dict(noise, initial_distance=noise["initial_distance"] * (1.0 + eps))
        rgb_c, rgb, _, _ = rend(c2w, K, x_pix, net, noise=nz)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb - gt) ** 2).mean()
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in list(net.named_parameters()) + list(rend.named_parameters())
                 if p.grad is not None}
        return float(loss.detach()), grads, rend.last_path

    lh, gh, ph = step(True)
    lt, gt_, pt = step(False)
    _, gp, _ = step(False, eps=1e-6)
    assert ph == "hip_train" and pt == "module"
    assert abs(lh - lt) <= 1e-5 * max(1.0, abs(lt))
    assert set(gh) == set(gt_) == set(gp)
    # An integration check, fp32 against fp32 (the renderer's ray kernels are fp32-only, so no float64 run of
    # the whole step): each piece is held to float64 elsewhere -- the march above, the field's parameter and
    # point gradients in test_gpu_train.py (2x PyTorch fp32's own error) -- and two fp32 implementations of a
    # 5-block ResnetFC legitimately differ by up to ~1e-2 of a weight gradient's max (both sit at that distance
    # from float64 where a relu mask flips). The bar: the march's sensitivity to fp32-sized noise (PyTorch's own
    # gradients when every start distance moves by 1e-6 relative, ~8 ulp) x 3, plus 2e-2 of the max |grad|.
    worst = 0.0
    for k in gt_:
        s = float(gt_[k].abs().max()) or 1.0
        err = float((gh[k] - gt_[k]).abs().max())
        noise_k = float((gp[k] - gt_[k]).abs().max())
        worst = max(worst, err / s)
        assert err <= 3.0 * noise_k + 2e-2 * s + 1e-7, f"{k}: {err:.3e} (torch's own spread {noise_k:.3e}) of {s:.3e}"
    print(f"adaptive step: worst HIP gradient difference {worst:.2e} of max |grad|")


def test_march_table_gradient_order_independent():
    """ABI 15: the gate-table gradient is summed as int64 fixed-point values (no floating-point atomics), so it
    does not depend on the order its contributions arrive in. Permuting the rays inside each scene changes the
    workgroups every contribution comes from and the order of the atomic adds: the latent's and W_ih's gradients
    (both computed from the table gradient alone) must come out bit for bit the same, the world points permuted
    with the rays; and a second identical backward gives every gradient bit for bit."""
    sb, R = 2, 300
    net = _net(64, 2, 64, (8, 8), sb=sb)
    rend = _renderer(64, 10)
    ros, rds, init, *_ = _march_inputs(sb, R, seed=21)
    w = 300.0 * torch.randn(sb, R, 3, generator=torch.Generator().manual_seed(22)).to(DEV)
    wa, ga, path = _march_grads(rend, net, ros, rds, init, w, hip=True)
    assert path == "hip_train"
    wb, gb, _ = _march_grads(rend, net, ros, rds, init, w, hip=True)
    assert torch.equal(wa, wb)
    for k in ga:
        assert torch.equal(ga[k], gb[k]), f"{k} differs between two identical backward passes"
    perm = torch.randperm(R, generator=torch.Generator().manual_seed(23)).to(DEV)
    wp, gp, _ = _march_grads(rend, net, ros[:, perm], rds[:, perm], init[:, perm], w[:, perm], hip=True)
    assert torch.equal(wp, wa[:, perm])
    for k in ("latent", "lstm.weight_ih"):
        assert torch.equal(gp[k], ga[k]), (k, float((gp[k] - ga[k]).abs().max()))
    assert float(ga["latent"].abs().max()) > 0 and float(ga["lstm.weight_ih"].abs().max()) > 0
    for k in gp:   # the parameter sums follow the ray order (fixed-order float sums): equal to rounding only
        s = float(ga[k].abs().max()) or 1.0
        assert float((gp[k] - ga[k]).abs().max()) <= 1e-5 * s, k
