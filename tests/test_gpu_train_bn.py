"""train.py --bn on the HIP path (avr.bn_train; train.py:210, :265; ResnetBlockFC(bn=True), models.py:430-432,
454-461): training-mode BatchNorm with batch statistics, layer by layer on the x3 GEMMs. Against PyTorch
autograd of the same module: the forward, the running-statistics update of both bn_0 applications, and
every parameter gradient (bn_0's weight / bias included) within twice PyTorch fp32's own error against a
float64 reference -- at (512, 3) and (512, 5, 3) (conf/default.conf and train.py's conf/default_mv.conf)."""
import numpy as np
import pytest
import torch

from test_gpu_train import _fp64, _points

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _compare64(g_hip, g_t32, g_64, floor=1e-4):
    """test_gpu_train._compare64 with one change: each parameter's error is measured against
    max(its max |grad|, 1e-4 of the largest gradient of the net). Under batch statistics fc_0's bias has an
    exactly zero gradient (the batch mean subtracts it, models.py:456-461): its float64 reference is ~1e-16 and
    its fp32 values are rounding noise, for PyTorch and HIP alike."""
    assert set(g_hip) == set(g_t32) == set(g_64), (sorted(g_hip), sorted(g_64))
    glob = max(float(v.double().abs().max()) for v in g_64.values())
    worst = 0.0
    for k in g_64:
        ref = g_64[k].double()
        s = max(float(ref.abs().max()), 1e-4 * glob) or 1.0
        eh = float((g_hip[k].double() - ref).abs().max()) / s
        et = float((g_t32[k].double() - ref).abs().max()) / s
        worst = max(worst, eh)
        assert eh <= 2.0 * et + floor, f"{k}: HIP err {eh:.2e} vs fp32 autograd err {et:.2e} (of {s:.2e})"
    return worst


def _bn_net(d_hidden, n_blocks, combine_layer=1000, d_latent=None, hw=(16, 16), sb=1, seed=0):
    from avr.conf import Conf, default_conf
    from avr.models import NewPixelNeRFNet
    d_latent = d_latent or (512 if d_hidden == 512 else 64)
    d = dict(default_conf()["model"])
    mlp = {"type": "resnet", "n_blocks": n_blocks, "d_hidden": d_hidden, "combine_layer": combine_layer}
    d["mlp_coarse"], d["mlp_fine"] = dict(mlp), dict(mlp)
    d["encoder"] = {"backbone": "resnet34", "pretrained": False,
                    "num_layers": {64: 1, 128: 2, 256: 3, 512: 4}[d_latent]}
    torch.manual_seed(seed)
    net = NewPixelNeRFNet(Conf(d), bn=True)
    with torch.no_grad():
        for m in (net.mlp_coarse, net.mlp_fine):
            for blk in m.blocks:
                blk.fc_1.weight.normal_(0.0, 0.02)          # not the reference's zero init (identity blocks)
                blk.bn_0.weight.uniform_(0.5, 1.5)          # and non-trivial affine parameters
                blk.bn_0.bias.uniform_(-0.2, 0.2)
    net = net.to(DEV).train()
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    net.encoder.set_latent(torch.randn(sb, d_latent, hw[0], hw[1], generator=g).to(DEV))
    poses = torch.zeros(sb, 3, 4)
    poses[:, :3, :3] = torch.eye(3)
    poses[:, 2, 3] = 1.3 + 0.1 * torch.arange(sb)
    net.poses = poses.to(DEV)
    net.num_objs = sb
    net.focal = torch.tensor([[131.25, -131.25]] * sb, device=DEV)
    net.c = torch.tensor([[64.0, 64.0]] * sb, device=DEV)
    net.image_shape = torch.tensor([128.0, 128.0], device=DEV)
    for p in net.parameters():
        p.requires_grad_(True)
    return net


def _running(net):
    """The running statistics of the MLPs' bn_0 (bn_1 is never applied; the encoder is not run here)."""
    return {n: b.detach().clone() for n, b in net.named_buffers()
            if n.startswith("mlp_") and ".bn_0." in n and ("running" in n or "num_batches" in n)}


def _set_running(net, state):
    with torch.no_grad():
        for n, b in net.named_buffers():
            if n in state:
                b.copy_(state[n].to(b.dtype))


def _grads_bn(net, xyz, vd, w, coarse, hip, latent_grad=False):
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


@pytest.mark.parametrize("d_hidden,n_blocks,combine_layer,sb,n", [(64, 3, 1000, 1, 1000), (128, 5, 3, 2, 700),
                                                                  (256, 3, 2, 2, 333), (512, 3, 1000, 1, 512),
                                                                  (512, 5, 3, 1, 1536)])
def test_bn_training_grads_match_fp64(d_hidden, n_blocks, combine_layer, sb, n):
    from avr.bn_train import bn_train_eligible
    net = _bn_net(d_hidden, n_blocks, combine_layer, sb=sb)
    assert bn_train_eligible(net) and net.can_train_bn(torch.zeros(sb, n, 3, device=DEV), torch.zeros(1, device=DEV))
    xyz, vd, w = _points(sb, n, seed=d_hidden + n_blocks)
    start = _running(net)
    out_h, g_h, _ = _grads_bn(net, xyz, vd, w, True, hip=True)
    run_h = _running(net)
    _set_running(net, start)
    out_t, g_t, _ = _grads_bn(net, xyz, vd, w, True, hip=False)
    run_t = _running(net)
    np.testing.assert_allclose(out_h.cpu().numpy(), out_t.cpu().numpy(), atol=2e-4)
    # both bn_0 applications of every block updated the running statistics as torch does
    for k in run_t:
        a, b = run_h[k].double(), run_t[k].double()
        if "num_batches" in k:   # bn_0 is applied twice per forward of its MLP (models.py:456-461)
            want = int(start[k]) + (2 if k.startswith("mlp_coarse") else 0)
            assert int(a) == int(b) == want, (k, int(a), int(b), want)
        else:
            assert float((a - b).abs().max()) <= 1e-4 * max(1.0, float(b.abs().max())), k
    expect = {"lin_in.weight", "lin_in.bias", "lin_out.weight", "lin_out.bias"}
    expect |= {f"blocks.{b}.fc_{i}.{t}" for b in range(n_blocks) for i in (0, 1) for t in ("weight", "bias")}
    expect |= {f"blocks.{b}.bn_0.{t}" for b in range(n_blocks) for t in ("weight", "bias")}
    expect |= {f"lin_z.{b}.{t}" for b in range(min(combine_layer, n_blocks)) for t in ("weight", "bias")}
    assert set(g_h) == expect, sorted(set(g_h) ^ expect)
    _set_running(net, start)
    _, g_d, _ = _fp64(net, lambda: _grads_bn(net, xyz.double(), vd.double(), w.double(), True, hip=False))
    worst = _compare64(g_h, g_t, g_d, floor=1e-4)
    print(f"bn ({d_hidden}, {n_blocks}, {combine_layer}): worst HIP gradient error vs float64 {worst:.2e} of max |grad|")


def test_bn_training_fine_mlp_latent_grad_and_ragged():
    """The fine MLP, the latent map's gradient, two scenes and a row count that is not a multiple of 64."""
    net = _bn_net(128, 3, sb=2)
    xyz, vd, w = _points(2, 333, seed=9)
    start = _running(net)
    _, g_h, l_h = _grads_bn(net, xyz, vd, w, False, hip=True, latent_grad=True)
    _set_running(net, start)
    _, g_t, l_t = _grads_bn(net, xyz, vd, w, False, hip=False, latent_grad=True)
    _set_running(net, start)
    _, g_d, l_d = _fp64(net, lambda: _grads_bn(net, xyz.double(), vd.double(), w.double(), False, hip=False,
                                                latent_grad=True))
    _compare64(dict(g_h, latent=l_h), dict(g_t, latent=l_t), dict(g_d, latent=l_d), floor=1e-4)


def test_bn_training_no_grad_and_eval_routes():
    """Training mode under no_grad still normalises with batch statistics (torch semantics) on the HIP path;
    eval mode runs the fused inference kernel with the running statistics folded in."""
    net = _bn_net(64, 2)
    xyz, vd, _ = _points(1, 300, seed=4)
    start = _running(net)
    with torch.no_grad():
        a = net(xyz, coarse=True, viewdirs=vd)
        _set_running(net, start)
        b = net.forward_torch(xyz, coarse=True, viewdirs=vd)
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=2e-4)
    net.eval()
    with torch.no_grad():
        assert net.can_fuse(xyz) and not net.can_train_bn(xyz, vd)
        c = net(xyz, coarse=True, viewdirs=vd)
        d = net.forward_torch(xyz, coarse=True, viewdirs=vd)
    np.testing.assert_allclose(c.cpu().numpy(), d.cpu().numpy(), atol=1e-4)


def test_bn_training_renderer_step():
    """A VolumeRenderer training step (train.py:108-114) of a --bn net: loss and every gradient of the HIP
    path against PyTorch autograd of the same module."""
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS
    net = _bn_net(128, 3, hw=(8, 8))
    R = 256
    g = torch.Generator().manual_seed(2)
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4, device=DEV).reshape(1, 1, 4, 4).expand(1, R, 4, 4).clone()
    c2w[..., 2, 3] = -1.3
    K = torch.tensor([INTRINSICS], device=DEV)
    gt = torch.rand(1, R, 3, generator=g).to(DEV)
    noise = {"coarse": torch.rand(1, R, 32, generator=g).to(DEV), "u": torch.rand(1, R, 16, generator=g).to(DEV),
             "u2": torch.rand(1, R, 16, generator=g).to(DEV), "depth": torch.zeros(1, R, 0, device=DEV)}
    start = _running(net)

    def step(hip):
        _set_running(net, start)
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        rend = VolumeRenderer(0.8, 1.8, 32, 16, 0, 0.01, True)
        rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net, noise=noise)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
        loss.backward()
        return float(loss), {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}

    lh, gh = step(True)
    lt, gt_ = step(False)
    assert abs(lh - lt) <= 1e-5 * max(1.0, abs(lt))
    assert set(gh) == set(gt_)
    glob = max(float(v.abs().max()) for v in gt_.values())
    for k in gt_:   # fc_0's bias has an exactly zero gradient under batch statistics (see _compare64)
        s = max(float(gt_[k].abs().max()), 1e-4 * glob)
        assert float((gh[k] - gt_[k]).abs().max()) <= 2e-3 * s, k


def test_bn_training_stop_encoder_grad_point_gradient():
    """stop_encoder_grad with points that need a gradient (the detached lookup, models.py:810-811, has
    no grad_fn, so the backward must not ask autograd for it): the points get z_feature's gradient alone, and every
    parameter and point gradient is within twice PyTorch fp32's own error against float64."""
    net = _bn_net(128, 3, combine_layer=2, hw=(8, 8))
    net.stop_encoder_grad = True
    xyz, vd, w = _points(1, 512, seed=21)
    start = _running(net)

    def grads(x0, v0, w0, hip):
        _set_running(net, start)
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        out = net(x, coarse=True, viewdirs=v0)
        (out * w0).sum().backward()
        gr = {n: p.grad.detach().clone() for n, p in net.mlp_coarse.named_parameters() if p.grad is not None}
        gr["xyz"] = x.grad.detach().clone()
        return gr

    assert net.can_train_bn(xyz, vd)
    g_h = grads(xyz, vd, w, True)
    g_t = grads(xyz, vd, w, False)
    g_d = _fp64(net, lambda: grads(xyz.double(), vd.double(), w.double(), False))
    assert float(g_h["xyz"].abs().max()) > 0
    _compare64(g_h, g_t, g_d, floor=1e-4)


def test_bn_training_512_two_scenes_ragged_lin_z():
    """d_hidden 512 (the width whose forward layers run bn_layer_kernel<4, 8, FWD, 512>): two scenes, in-kernel lin_z
    rows (combine_layer 3) and a row count that is not a multiple of 64 -- the forward and every gradient within
    twice PyTorch fp32's own error against float64. (Round 6 ran the rejected two-half kernels through this case,
    profiles/r06v_bn_h2_ab.txt.)"""
    net = _bn_net(512, 3, combine_layer=3, sb=2, hw=(8, 8))
    xyz, vd, w = _points(2, 333, seed=31)
    start = _running(net)
    out_h, g_h, _ = _grads_bn(net, xyz, vd, w, True, hip=True)
    _set_running(net, start)
    out_t, g_t, _ = _grads_bn(net, xyz, vd, w, True, hip=False)
    _set_running(net, start)
    _, g_d, _ = _fp64(net, lambda: _grads_bn(net, xyz.double(), vd.double(), w.double(), True, hip=False))
    np.testing.assert_allclose(out_h.cpu().numpy(), out_t.cpu().numpy(), atol=2e-4)
    _compare64(g_h, g_t, g_d, floor=1e-4)
