"""HIP training of use_spade and NS > 1 source-view nets (VERDICT r04 missing 2; avr.layer_train): the
layer-by-layer x3 GEMMs (avr_bn_layer_run with identity statistics), the spade product rule
(models.py:528-534, 585-587) and the views' combine adjoint (models.py:566-579, utils.py:71-81) against a
float64 autograd reference of the same module: every parameter gradient (scale_z's included), the latent-map
and point gradients within twice PyTorch fp32 autograd's own error (or 3e-5 of max |grad|), as the fused
training path is held (tests/test_gpu_train.py)."""
import numpy as np
import pytest
import torch

from test_gpu_train import _compare64, _fp64, _net

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _views_net(d_hidden, n_blocks, d_latent, hw, combine_layer, SB, NS, spade, combine_type="average", seed=0):
    """SB objects seen from NS source views each (train.py would encode SB x NS images): latent maps and poses per
    (object, view), focal / principal point per object."""
    net = _net(d_hidden, n_blocks, d_latent, hw, combine_layer, sb=1, seed=seed, spade=spade,
               combine_type=combine_type)
    K = SB * NS
    g = torch.Generator().manual_seed(seed + 11)
    net.encoder.set_latent(torch.randn(K, d_latent, hw[0], hw[1], generator=g).to(DEV))
    poses = net.poses.repeat(K, 1, 1)
    poses[:, 0, 3] += 0.07 * torch.arange(K, device=DEV, dtype=torch.float32)
    poses[:, 1, 3] -= 0.05 * torch.arange(K, device=DEV, dtype=torch.float32)
    net.poses = poses
    net.focal = net.focal.repeat(SB, 1)
    net.c = net.c.repeat(SB, 1)
    net.num_views_per_obj = NS
    net.num_objs = SB
    return net


def _grads(net, xyz, vd, w, coarse, hip, latent_grad):
    net.hip_backward = hip
    net.zero_grad(set_to_none=True)
    lat = net.encoder.latent.detach().clone().requires_grad_(latent_grad)
    net.encoder.latent = lat
    x = xyz.clone().requires_grad_(True)
    out = net(x, coarse=coarse, viewdirs=vd)
    (out * w).sum().backward()
    mlp = net.mlp_coarse if coarse else net.mlp_fine
    gr = {n: p.grad.detach().clone() for n, p in mlp.named_parameters() if p.grad is not None}
    gr["xyz"] = x.grad.detach().clone()
    if latent_grad:
        gr["latent"] = lat.grad.detach().clone()
    return out.detach(), gr


def _capture_forward(layer_train, store):
    """Wrap _FieldTrainLayers.forward so each call appends what the HIP forward decided: its stored fp32 rows
    (Xpre[b]: block b's residual stream before lin_z / spade / combine, Xin[b]: block b's input, N[b]: fc_0's
    output) and its output. The relu masks and the max-combine's winning views of the HIP run are read from these
    exactly as its backward reads them (layer_train.py:205-242). Returns the original forward."""
    orig = layer_train._FieldTrainLayers.forward

    def forward(ctx, fused, coarse, *rest):
        out = orig(ctx, fused, coarse, *rest)
        Xpre, Xin, N = ctx.keep[:3]
        store.append(([t.clone() for t in Xpre], [t.clone() for t in Xin], [t.clone() for t in N], out.clone()))
        return out

    layer_train._FieldTrainLayers.forward = staticmethod(forward)
    return orig


def _hip_masks(cap, mlp, SB, NS, B):
    """The branch of the piecewise-linear MLP the HIP forward took: relu masks [rows > 0] of every fc_0 / fc_1 /
    lin_out operand and of sigma (the backward's masks, layer_train.py:205-233), and with the max combine the view
    torch.max(dim) picks on the HIP rows (the one its adjoint, layer_train.py:238-242, sends the gradient to)."""
    Xpre, Xin, N, out = cap
    nb = mlp.n_blocks
    m = {"x": [x > 0 for x in Xin], "n": [n > 0 for n in N], "out": Xpre[nb] > 0,
         "sigma": out.reshape(-1, 4)[:, 3:] > 0}
    cl = mlp.combine_layer
    if NS > 1 and cl < nb and mlp.combine_type == "max":
        idx = Xpre[cl].reshape(SB, NS, B, -1).max(1).indices
        m["win"] = torch.nn.functional.one_hot(idx, NS).permute(0, 3, 1, 2)       # (SB, NS, B, H)
    return m


def _masked_forward(net, mlp, prm, xyz, vd, lat, m):
    """NewPixelNeRFNet.forward (models.py:739-863; ResnetFC models.py:541-592 with ResnetBlockFC models.py:454-470,
    spade models.py:585-587, the views' combine utils.py:71-81) with every relu replaced by its input times the HIP
    run's mask and the max combine by the HIP run's winning view: the same function as the reference's on the
    branch the HIP forward took, so its float64 gradient needs no excluded points."""
    F = torch.nn.functional
    SB, B, _ = xyz.shape
    NS = net.num_views_per_obj
    feat, zft = net.mlp_inputs(xyz, vd, latent=lat)
    dt = zft.dtype

    def lin(v, n):
        return F.linear(v, prm[n + ".weight"], prm[n + ".bias"])

    x = lin(zft, "lin_in")
    for b in range(mlp.n_blocks):
        if b == mlp.combine_layer and NS > 1:
            v = x.reshape(SB, NS, B, -1)
            x = ((v * m["win"].to(dt)).sum(1) if "win" in m else v.mean(1)).reshape(SB * B, -1)
        if b < mlp.combine_layer:
            tz = lin(feat, f"lin_z.{b}")
            x = lin(feat, f"scale_z.{b}") * x + tz if mlp.use_spade else x + tz
        h = lin(x * m["x"][b].to(dt), f"blocks.{b}.fc_0")
        x = x + lin(h * m["n"][b].to(dt), f"blocks.{b}.fc_1")
    raw = lin(x * m["out"].to(dt), "lin_out")
    return torch.cat([torch.sigmoid(raw[:, :3]), raw[:, 3:] * m["sigma"].to(dt)], -1).reshape(SB, B, 4)


def _masked_grads(net, xyz, vd, w, coarse, m, latent_grad):
    """Every parameter, point and (unless stop_encoder_grad) latent-map gradient of _masked_forward, in the
    net's current dtype (fp32, or float64 inside _fp64)."""
    mlp = net.mlp_coarse if coarse else net.mlp_fine
    prm = {n: p.detach().clone().requires_grad_(True) for n, p in mlp.named_parameters()}
    lat = net.encoder.latent.detach().clone().requires_grad_(latent_grad)
    x = xyz.clone().requires_grad_(True)
    out = _masked_forward(net, mlp, prm, x, vd, lat, m)
    (out * w).sum().backward()
    gr = {n: p.grad.detach().clone() for n, p in prm.items() if p.grad is not None}
    gr["xyz"] = x.grad.detach().clone()
    if latent_grad:
        gr["latent"] = lat.grad.detach().clone()
    return out.detach(), gr


CASES = [  # d_hidden, n_blocks, d_latent, combine_layer, SB, NS, spade, combine_type
    (64, 3, 64, 1000, 2, 1, True, "average"),
    (128, 5, 64, 3, 1, 1, True, "average"),
    (64, 3, 64, 2, 2, 2, False, "average"),
    (128, 4, 128, 2, 1, 3, False, "max"),
    (64, 3, 64, 2, 2, 2, True, "average"),
    (64, 3, 64, 2, 2, 2, True, "max"),
    (256, 3, 64, 2, 2, 2, True, "max"),
    (512, 5, 512, 3, 1, 2, True, "average"),
]


def _check_case(case, stop=False):
    from avr import layer_train
    d_hidden, n_blocks, d_latent, cl, SB, NS, spade, ctype = case
    hw = (16, 16) if d_hidden == 512 else (8, 8)
    net = _views_net(d_hidden, n_blocks, d_latent, hw, cl, SB, NS, spade, ctype)
    net.stop_encoder_grad = stop
    latent_grad = not stop        # a detached lookup (models.py:810-811) leaves the map without a gradient
    g = torch.Generator().manual_seed(17)
    B = 333
    xyz = ((torch.rand(SB, B, 3, generator=g) - 0.5) * 0.8).to(DEV)
    vd = torch.nn.functional.normalize(torch.randn(SB, B, 3, generator=g), dim=-1).to(DEV)
    w = torch.randn(SB, B, 4, generator=g).to(DEV)
    assert net.can_train_layers(xyz, vd) and not net.can_train_fused(xyz, vd)
    calls, caps = [], []
    orig = layer_train._FieldTrainLayers.apply
    orig_fwd = _capture_forward(layer_train, caps)
    layer_train._FieldTrainLayers.apply = lambda *a: calls.append(1) or orig(*a)
    try:
        for coarse in (True, False):
            mlp = net.mlp_coarse if coarse else net.mlp_fine
            caps.clear()
            out_h, g_h = _grads(net, xyz, vd, w, coarse, hip=True, latent_grad=latent_grad)
            n_hip = len(calls)
            out_t, g_t = _grads(net, xyz, vd, w, coarse, hip=False, latent_grad=latent_grad)
            assert n_hip >= 1 and len(calls) == n_hip and len(caps) == 1, \
                "the HIP run must take the layer path (once), torch's must not"
            np.testing.assert_allclose(out_h.cpu().numpy(), out_t.cpu().numpy(), atol=2e-4)
            if spade:
                assert any(k.startswith("scale_z.") for k in g_h)
            # the reference gradient on the branch the HIP forward took: every point carries its loss
            m = _hip_masks(caps[0], mlp, SB, NS, B)
            out_m, g_tm = _masked_grads(net, xyz, vd, w, coarse, m, latent_grad)
            np.testing.assert_allclose(out_m.cpu().numpy(), out_h.cpu().numpy(), atol=2e-4)
            _, g_dm = _fp64(net, lambda: _masked_grads(net, xyz.double(), vd.double(), w.double(), coarse,
                                                       m, latent_grad))
            # the unconditioned float64 reference, printed for the record (the relu / max flips of either fp32 run)
            _, g_d = _fp64(net, lambda: _grads(net, xyz.double(), vd.double(), w.double(), coarse, hip=False,
                                               latent_grad=latent_grad))
            assert set(g_h) == set(g_tm) == set(g_dm) == set(g_d), sorted(set(g_h) ^ set(g_dm))
            for k in g_dm:   # every key's errors first (the assertion below names only the first failing one)
                ref, ref_u = g_dm[k].double(), g_d[k].double()
                sc = float(ref.abs().max()) or 1.0
                print(f"   {k}: HIP {float((g_h[k].double() - ref).abs().max()) / sc:.2e} "
                      f"torch32 {float((g_tm[k].double() - ref).abs().max()) / sc:.2e} under the HIP masks; "
                      f"unconditioned: HIP {float((g_h[k].double() - ref_u).abs().max()) / sc:.2e} "
                      f"torch32 {float((g_t[k].double() - ref_u).abs().max()) / sc:.2e}")
            worst = _compare64(g_h, g_tm, g_dm)
            print(f"{case} stop={stop} coarse={coarse}: 0 points excluded; worst HIP gradient error vs float64 "
                  f"under the HIP masks {worst:.2e} of max |grad|")
    finally:
        layer_train._FieldTrainLayers.apply = orig
        layer_train._FieldTrainLayers.forward = staticmethod(orig_fwd)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"h{c[0]}-nb{c[1]}-cl{c[3]}-sb{c[4]}-ns{c[5]}"
                                                     f"{'-spade' if c[6] else ''}-{c[7]}")
def test_layer_train_grads_match_fp64(case):
    """Every parameter, point and latent-map gradient of every point (none excluded) within twice fp32's own
    error of the float64 gradient on the HIP forward's branch."""
    _check_case(case)


@pytest.mark.parametrize("case", [(64, 3, 64, 2, 2, 2, True, "average"), (128, 4, 128, 2, 1, 3, False, "max")],
                         ids=["spade-ns2", "ns3-max"])
def test_layer_train_stop_encoder_grad_point_gradient(case):
    """stop_encoder_grad with points that need a gradient (the detached lookup has no grad_fn): the
    points get z_feature's gradient alone, as torch's autograd of the module gives."""
    _check_case(case, stop=True)


@pytest.mark.parametrize("H,n,pad", [(64, 1, 0), (192, 5, 4), (512, 1003, 0), (512, 40000, 8)])
def test_lin_out_rows_vs_fp64(H, n, pad):
    """avr_lin_out_fwd_rows / avr_lin_out_bwd_rows (the layer-by-layer paths' output layer; and
    avr_lin_out_act_bwd_rows, the activations' backward alone) against float64 torch:
    out and g within 1e-5 of their scale, d_raw bit-equal to torch's own activation backward kernels
    (aten sigmoid_backward / threshold_backward), g exactly 0 where pre <= 0, both maxima exact; rows with a leading dimension past d_hidden."""
    from avr import ops
    g = torch.Generator().manual_seed(H + n)
    xw = torch.randn(n, H + pad, generator=g).to(DEV)
    x = xw[:, :H]
    W = (torch.randn(4, H, generator=g) * 0.05).to(DEV)
    b = torch.randn(4, generator=g).to(DEV)
    out, xmax = ops.lin_out_rows(x, W, b)
    raw = torch.relu(x.double()) @ W.double().t() + b.double()
    ref = torch.cat([torch.sigmoid(raw[:, :3]), torch.relu(raw[:, 3:])], -1)
    assert float((out.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))
    assert int(xmax) == int(torch.relu(x).max().reshape(1).view(torch.int32))
    go = torch.randn(n, 4, generator=g).to(DEV)
    d4, gr, dmax = ops.lin_out_rows_bwd(go, out, W, x)
    # torch's own activation backward kernels (SigmoidBackward0 / ReluBackward0), bit for bit
    d4_ref = torch.cat([torch.ops.aten.sigmoid_backward(go[:, :3], out[:, :3]),
                        torch.ops.aten.threshold_backward(go[:, 3:], out[:, 3:], 0.0)], -1)
    assert torch.equal(d4, d4_ref)
    assert int(dmax) == int(d4_ref.abs().max().reshape(1).view(torch.int32))
    g_ref = (d4.double() @ W.double()) * (x > 0)
    assert float((gr.double() - g_ref).abs().max()) <= 1e-5 * max(float(g_ref.abs().max()), 1e-30)
    assert bool((gr[x <= 0] == 0).all())
    # the activations' backward alone (ABI 16, the fused training path's d4): the same d_raw and max
    d4b, dmaxb = ops.lin_out_act_bwd(go, out)
    assert torch.equal(d4b, d4_ref) and int(dmaxb) == int(dmax)


@pytest.mark.parametrize("H,nb,cl,M", [(64, 3, 2, 333), (256, 3, 3, 64), (512, 5, 3, 1000)])
def test_lin_z_transposed_layers_vs_fp64(H, nb, cl, M):
    """The looked-up features' gradient sum_b Gz[b] . W_z[b] on avr_bn_layer_run's lin_z[b]^T layers (ABI 14: the
    backward blob's transposed lin_z fragments, no mask, each layer adding the previous sum) against float64, and
    the library fallback where the layers do not apply (d_latent != d_hidden)."""
    from avr.field import _feat_grad
    net = _net(H, nb, H, (8, 8), cl)
    fused = net.fused()
    mlp = net.mlp_coarse
    entry = fused.packed(True)
    bwd = fused.packed_bwd(True, entry)
    nz = entry.dims.n_lin_z
    assert nz == min(cl, nb)
    g = torch.Generator().manual_seed(H + M)
    Gz = [(torch.randn(M, H, generator=g) * 10.0 ** (-b)).to(DEV) for b in range(nz)]
    P = {f"lin_z.{b}.weight": mlp.lin_z[b].weight for b in range(nz)}
    got = _feat_grad(fused, entry, bwd, Gz, P, M)
    ref = sum(Gz[b].double() @ P[f"lin_z.{b}.weight"].detach().double() for b in range(nz))
    err = float((got.double() - ref).abs().max() / ref.abs().max())
    assert err <= 2e-6, err
    # d_latent 64 != d_hidden 128: the fallback's fp32 GEMMs
    net2 = _net(128, 3, 64, (8, 8), 2)
    f2 = net2.fused()
    e2 = f2.packed(True)
    Gz2 = [torch.randn(M, 128, generator=g).to(DEV) for _ in range(2)]
    P2 = {f"lin_z.{b}.weight": net2.mlp_coarse.lin_z[b].weight for b in range(2)}
    got2 = _feat_grad(f2, e2, f2.packed_bwd(True, e2), Gz2, P2, M)
    ref2 = sum(Gz2[b].double() @ P2[f"lin_z.{b}.weight"].detach().double() for b in range(2))
    assert float((got2.double() - ref2).abs().max() / ref2.abs().max()) <= 2e-6


@pytest.mark.parametrize("n", [4, 1000, 512 * 4097])
def test_spade_bwd_rows_bit_exact(n):
    """avr_spade_bwd_rows (the spade product rule's backward, ABI 14): g * x and s * g equal torch's products bit
    for bit, max |g * x| exact."""
    from avr import ops
    g0 = torch.Generator().manual_seed(n)
    g, x, s = (torch.randn(n // 4, 4, generator=g0).to(DEV) for _ in range(3))
    gs, go, gmax = ops.spade_bwd_rows(g, x, s)
    assert torch.equal(gs, g * x) and torch.equal(go, s * g)
    assert int(gmax) == int((g * x).abs().max().reshape(1).view(torch.int32))
