"""avr.layer_train's host logic on the CPU (no GPU): the forward / backward orchestration of the layer-by-layer
use_spade / NS > 1 training path -- the spade product rule, the views' combine and its adjoint, the bias folding,
which rows each layer runs over, the weight-gradient layer lists and their unpacking -- with every library call
replaced by a torch statement of its C-ABI contract (include/avr.h: avr_bn_layer_run FWD / BWD with identity
statistics, avr_weight_grads, the per-texel tables and their bilinear gather). Against torch autograd of the same
module (models.py:541-592, 739-863). The kernels themselves are held to float64 on the MI355X
(tests/test_gpu_layer_train.py)."""
import pytest
import torch

from avr import _lib, bn_train, field, layer_train, ops


def _net(d_hidden, n_blocks, d_latent, cl, SB, NS, spade, ctype, hw=(6, 7), seed=0):
    from avr.conf import Conf, default_conf
    from avr.scene import synthetic_scene
    d = dict(default_conf()["model"])
    mlp = {"type": "resnet", "n_blocks": n_blocks, "d_hidden": d_hidden, "combine_layer": cl, "beta": 0.0,
           "use_spade": spade, "combine_type": ctype}
    d["mlp_coarse"], d["mlp_fine"] = dict(mlp), dict(mlp)
    d["encoder"] = {"backbone": "resnet34", "pretrained": False, "num_layers": {64: 1, 128: 2}[d_latent]}
    net = synthetic_scene(torch.device("cpu"), seed, Conf(d), latent_hw=hw)
    K = SB * NS
    g = torch.Generator().manual_seed(seed + 3)
    net.encoder.set_latent(torch.randn(K, d_latent, hw[0], hw[1], generator=g))
    poses = net.poses.repeat(K, 1, 1)
    poses[:, 0, 3] += 0.07 * torch.arange(K, dtype=torch.float32)
    net.poses = poses
    net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
    net.num_views_per_obj, net.num_objs = NS, SB
    for p in net.parameters():
        p.requires_grad_(True)
    return net


class _Entry:
    def __init__(self, mlp, dims):
        self.dims, self.packed, self.mlp = dims, mlp, mlp


def _install(monkeypatch, net):
    """The library calls of avr.layer_train as torch statements of their contracts."""
    fused = net.fused()
    cur = {}

    def mlp_of(coarse):
        return net.mlp_coarse if (coarse or net.mlp_fine is None) else net.mlp_fine

    def packed(coarse, bn_fold=True):
        mlp = mlp_of(coarse)
        cur["mlp"] = mlp
        return _Entry(mlp, fused.dims(mlp))

    def tables_batch(coarse, K, fast=False, bn_fold=True):
        """(K, n_tables, H*W, d_hidden): lin_z[t] (then scale_z) of every texel; biases only with use_spade."""
        mlp, lat = mlp_of(coarse), net.encoder.latent.detach()
        rows = lat[:K].reshape(K, lat.shape[1], -1).transpose(1, 2)
        lins = list(mlp.lin_z) + (list(mlp.scale_z) if mlp.use_spade else [])
        return torch.stack([rows @ m.weight.detach().t() + (m.bias.detach() if mlp.use_spade else 0) for m in lins], 1)

    def gather(fused_, tab, K, NS, p, B, C):
        """tab (K, H*W, C) blended at the points like the latent (SpatialEncoder.index on a C-channel map)."""
        hold, hold_c = net.encoder.latent, net.latent_size
        hh, ww = hold.shape[-2:]
        try:
            net.encoder.latent = tab.transpose(1, 2).reshape(K, C, hh, ww)
            net.latent_size = C
            xyz = p.reshape(-1, NS, B, 3)[:, 0]
            feat, _ = net.mlp_inputs(xyz, torch.zeros_like(xyz))
        finally:
            net.encoder.latent, net.latent_size = hold, hold_c
        return feat.reshape(K * B, C).contiguous()

    def weight_of(layer, bwd):
        mlp = cur["mlp"]
        if layer >= _lib.BN_LAYER_LIN_Z_T:       # the backward blob's lin_z[b]^T (ABI 14)
            return mlp.lin_z[layer - _lib.BN_LAYER_LIN_Z_T].weight.detach()
        if layer == 0:
            return mlp.lin_in.weight.detach()
        blk = mlp.blocks[(layer - 2) // 2]
        return (blk.fc_0 if layer % 2 == 0 else blk.fc_1).weight.detach()

    def run(dims, kw, stream):
        W = weight_of(kw["layer"], kw["mode"] == _lib.BN_BWD)
        src = kw["src"][:, :kw["in_valid"]]
        if kw["mode"] == _lib.BN_FWD:
            op = src if kw["prologue"] == _lib.BN_PLAIN else \
                torch.relu((src - kw["in_mu"]) * kw["in_scale"] + kw["in_shift"])
            out = op @ W.t() + kw["bias"]
            for k in ("add1", "add2"):
                if kw.get(k) is not None:
                    out = out + kw[k]
            if kw.get("lin_z_table") is not None:    # the T rows gathered in the epilogue (scene-major rows)
                tz = kw["lin_z_table"]
                tab = tz.as_strided((kw["n_views"],) + tuple(tz.shape), (kw["lin_z_scene_stride"],) + tz.stride())
                out = out + gather(fused, tab, kw["n_views"], net.num_views_per_obj, kw["xyz"],
                                   kw["rows_per_scene"], tz.shape[1])
        else:
            assert kw["prologue"] == _lib.BN_PLAIN
            op = src
            if kw.get("pre_rows") is None:           # lin_z^T: no mask
                out = src @ W
            else:
                mask = torch.relu((kw["pre_rows"] - kw["out_mu"]) * kw["out_scale"] + kw["out_shift"]) > 0
                out = (src @ W) * mask
            if kw.get("add1") is not None:           # the residual gradient (ABI 14)
                out = out + kw["add1"]
        if kw.get("out_max") is not None:         # backward: max |out| of the stored rows (ABI 14)
            m = torch.maximum(out.abs().max().reshape(1), kw["out_max"][:1].view(torch.float32))
            kw["out_max"][:1].copy_(m.view(torch.int32))
        if kw.get("operand_max") is not None:     # publish max |operand| (float bits, max with what is there)
            m = torch.maximum(op.abs().max().reshape(1), kw["operand_max"][:1].view(torch.float32))
            kw["operand_max"][:1].copy_(m.view(torch.int32))
        kw["out"].copy_(out)

    def weight_grads(layers, n_rows, n_split=None):
        res = []
        for g, x, gmax, xmax, want_bias, *bn in layers:
            assert g.shape[0] == x.shape[0] == n_rows
            # the scales' inputs: max |G| exactly (the operand maxima the layer kernels publish, or a reduction)
            assert float(gmax.view(torch.float32)[0]) == float(g.abs().max()), "wrong max |G|"
            if bn and bn[0] == "relu":
                x = torch.relu(x)
            elif bn:
                mu, sc, sh = bn[0]
                x = torch.relu((x - mu) * sc + sh)
            res.append((g.t() @ x, g.sum(0) if want_bias else None))
        return res

    def bits(t):
        return t.abs().max().reshape(1).view(torch.int32)

    def lin_out_rows(x, weight, bias):
        """avr_lin_out_fwd_rows' contract."""
        raw = torch.relu(x) @ weight.t() + bias
        return torch.cat([torch.sigmoid(raw[:, :3]), torch.relu(raw[:, 3:])], -1), bits(torch.relu(x))

    def lin_out_rows_bwd(grad_out, out, weight, pre, g=None):
        """avr_lin_out_bwd_rows' contract."""
        d4 = torch.cat([torch.ops.aten.sigmoid_backward(grad_out[:, :3], out[:, :3]),
                        torch.ops.aten.threshold_backward(grad_out[:, 3:], out[:, 3:], 0.0)], -1)
        gr = torch.ops.aten.threshold_backward(d4 @ weight, pre, 0.0)
        if g is not None:
            g.copy_(gr)
            gr = g
        return d4, gr, bits(d4)

    def spade_bwd_rows(g, x, s):
        """avr_spade_bwd_rows' contract."""
        gs = g * x
        return gs, s * g, bits(gs)

    monkeypatch.setattr(ops, "spade_bwd_rows", spade_bwd_rows)
    monkeypatch.setattr(ops, "lin_out_rows", lin_out_rows)
    monkeypatch.setattr(ops, "lin_out_rows_bwd", lin_out_rows_bwd)
    monkeypatch.setattr(fused, "packed", packed)
    monkeypatch.setattr(fused, "packed_bwd", lambda coarse, entry=None: None)
    monkeypatch.setattr(fused, "tables_batch", tables_batch)
    monkeypatch.setattr(layer_train, "_gather", gather)
    monkeypatch.setattr(layer_train, "stream_of", lambda t: None)
    monkeypatch.setattr(field, "stream_of", lambda t: None)
    monkeypatch.setattr(bn_train, "_layer", lambda **kw: kw)
    monkeypatch.setattr(bn_train, "_run", run)
    monkeypatch.setattr(bn_train, "_partial", lambda M, H, dev: torch.empty(1))
    monkeypatch.setattr(ops, "weight_grads", weight_grads)
    return fused


@pytest.mark.parametrize("case", [
    (16, 3, 64, 1000, 2, 1, True, "average"),
    (16, 3, 64, 2, 2, 2, False, "average"),
    (16, 3, 64, 2, 2, 2, True, "average"),
    (32, 4, 64, 1, 1, 3, True, "max"),
    (16, 2, 128, 1, 2, 2, False, "max"),
    (64, 3, 64, 2, 2, 2, False, "average"),     # d_latent == d_hidden: the feature gradient on lin_z^T layers
], ids=lambda c: f"h{c[0]}-nb{c[1]}-cl{c[3]}-sb{c[4]}-ns{c[5]}{'-spade' if c[6] else ''}-{c[7]}")
@pytest.mark.parametrize("coarse", [True, False])
def test_layer_train_logic_matches_autograd(monkeypatch, case, coarse):
    _check(monkeypatch, case, coarse)


def test_layer_train_gathered_lin_z_rows(monkeypatch):
    """More scenes than one layer launch takes: the T rows gathered and added in torch (not in the epilogue)."""
    monkeypatch.setattr(_lib, "AVR_MAX_SCENES", 3)
    _check(monkeypatch, (16, 3, 64, 2, 2, 2, False, "average"), True)


def _check(monkeypatch, case, coarse):
    d_hidden, n_blocks, d_latent, cl, SB, NS, spade, ctype = case
    net = _net(d_hidden, n_blocks, d_latent, cl, SB, NS, spade, ctype)
    fused = _install(monkeypatch, net)
    g = torch.Generator().manual_seed(4)
    B = 37
    xyz = (torch.rand(SB, B, 3, generator=g) - 0.5) * 0.8
    vd = torch.nn.functional.normalize(torch.randn(SB, B, 3, generator=g), dim=-1)
    w = torch.randn(SB, B, 4, generator=g)
    lat = net.encoder.latent.clone().requires_grad_(True)

    def grads(fn):
        net.zero_grad(set_to_none=True)
        lat.grad = None
        net.encoder.latent = lat
        x = xyz.clone().requires_grad_(True)
        (fn(x) * w).sum().backward()
        mlp = net.mlp_coarse if coarse else net.mlp_fine
        out = {n: p.grad.clone() for n, p in mlp.named_parameters() if p.grad is not None}
        out.update(xyz=x.grad.clone(), latent=lat.grad.clone())
        return out

    got = grads(lambda x: layer_train.forward_train_layers(fused, x, vd, coarse))
    ref = grads(lambda x: net.forward_torch(x, coarse, vd))
    assert set(got) == set(ref)
    if spade:
        assert any(k.startswith("scale_z") for k in got)
    for k in ref:
        s = float(ref[k].abs().max()) or 1.0
        err = float((got[k] - ref[k]).abs().max())
        assert err <= 1e-4 * s, f"{k}: {err:.3e} of max |grad| {s:.3e}"


def test_fused_field_parameter_slots_follow_replacements():
    """FusedField._state (the cached per-module slots behind packed() / forward_train's parameter lists): the same
    tensors as named_parameters() in the same order, a parameter replaced in place and a submodule replaced after
    the first call both seen, and no rebuild while nothing is registered."""
    import torch.nn as nn
    from avr import field as fld
    net = _net(16, 3, 64, 2, 1, 1, False, "average")
    fused = net.fused()
    mlp = net.mlp_coarse
    named, ps, bs = fused._state(mlp)
    ref = dict(mlp.named_parameters())
    assert list(named) == list(ref) and all(named[k] is ref[k] for k in ref)
    assert [id(t) for t in ps] == [id(t) for t in mlp.parameters()]
    assert [id(b) for b in bs] == [id(b) for b in mlp.buffers() if b.is_floating_point()]
    slots = fused._slots[mlp]
    fused._state(mlp)
    assert fused._slots[mlp] is slots                          # cached
    # modules built elsewhere (with submodules) register children, but not under this MLP: no rebuild
    nn.Sequential(nn.Linear(3, 3), nn.ReLU())
    fused._state(mlp)
    assert fused._slots[mlp][0] is slots[0] and fld._MODULE_GEN[0] == fused._slots[mlp][2]
    mlp.lin_out.weight = nn.Parameter(torch.zeros_like(mlp.lin_out.weight))
    assert fused._state(mlp)[0]["lin_out.weight"] is mlp.lin_out.weight
    old = mlp.lin_in
    mlp.lin_in = nn.Linear(old.in_features, old.out_features)
    named = fused._state(mlp)[0]
    assert named["lin_in.weight"] is mlp.lin_in.weight and named["lin_in.weight"] is not old.weight
    assert fused._slots[mlp][0] is not slots[0] and fld._MODULE_GEN[0] == fused._slots[mlp][2]
    # the slots hold the MLP weakly: a dropped module's entry goes with it
    import gc
    tmp = nn.Sequential(nn.Linear(2, 2))
    fused._state(tmp)
    n = len(fused._slots)
    del tmp
    gc.collect()
    assert len(fused._slots) == n - 1


def test_fused_field_view_arrays_follow_the_sources():
    """FusedField.views (the cached ViewDesc array of a multi-scene launch, round 6): one array object while the
    source-view tensors are unchanged, holding view(i, ns) of each index; a new one after an in-place pose update, a
    replaced focal tensor or invalidate(); invalidate(views=False) (GraphedTrainStep before a capture) keeps it."""
    net = _net(16, 3, 64, 2, 1, 1, False, "average")
    net.poses = net.poses.repeat(3, 1, 1).clone()
    net.poses[:, 0, 3] += torch.tensor([0.0, 0.1, 0.2])
    net.focal, net.c = net.focal.repeat(3, 1).clone(), net.c.repeat(3, 1).clone()
    fused = net.fused()
    a = fused.views(range(3))
    assert fused.views(range(3)) is a and len(a) == 3
    assert [round(a[i].poses[3], 5) for i in range(3)] == [round(float(net.poses[i, 0, 3]), 5) for i in range(3)]
    b = fused.views(range(0, 3, 2))
    assert b is not a and [round(b[i].poses[3], 5) for i in range(2)] == [round(a[0].poses[3], 5),
                                                                          round(a[2].poses[3], 5)]
    with torch.no_grad():
        net.poses[1, 0, 3] += 1.0
    a2 = fused.views(range(3))
    assert a2 is not a and abs(a2[1].poses[3] - float(net.poses[1, 0, 3])) < 1e-6
    net.focal = net.focal * 2.0
    a3 = fused.views(range(3))
    assert a3 is not a2 and abs(a3[0].focal[0] - float(net.focal[0, 0])) < 1e-4
    fused.invalidate(views=False)
    assert fused.views(range(3)) is a3
    fused.invalidate()
    assert fused.views(range(3)) is not a3
