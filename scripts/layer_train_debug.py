"""Diagnostic: every avr_bn_layer_run call of avr.layer_train's training step compared with a torch statement of
its contract (the kernel's output vs torch on the same inputs), for one net configuration. Not part of the product.
usage: python scripts/layer_train_debug.py [d_hidden n_blocks d_latent combine_layer SB NS spade(0/1) type]"""
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in (REPO, os.path.join(REPO, "adaptive-volume-rendering_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)


def main():
    from avr import _lib, bn_train, layer_train
    from test_gpu_layer_train import _views_net
    a = sys.argv[1:] or ["64", "3", "64", "2", "2", "2", "1", "average"]
    d_hidden, n_blocks, d_latent, cl, SB, NS, spade = (int(x) for x in a[:7])
    net = _views_net(d_hidden, n_blocks, d_latent, (8, 8), cl, SB, NS, bool(spade), a[7])
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(17)
    B = 333
    xyz = ((torch.rand(SB, B, 3, generator=g) - 0.5) * 0.8).to(dev)
    vd = torch.nn.functional.normalize(torch.randn(SB, B, 3, generator=g), dim=-1).to(dev)
    w = torch.randn(SB, B, 4, generator=g).to(dev)
    cur = {"mlp": net.mlp_coarse}
    orig_layer, orig_run = bn_train._layer, bn_train._run
    calls = []
    snaps = {}

    def layer(**kw):
        lay = orig_layer(**kw)
        lay._kw = kw
        return lay

    def run(dims, lay, stream):
        orig_run(dims, lay, stream)
        kw = lay._kw
        mlp = cur["mlp"]
        L = kw["layer"]
        W = (mlp.lin_in.weight if L == 0 else
             (mlp.blocks[(L - 2) // 2].fc_0 if L % 2 == 0 else mlp.blocks[(L - 2) // 2].fc_1).weight).detach()
        src = kw["src"][:, :kw["in_valid"]]
        if kw["mode"] == _lib.BN_FWD:
            op = src if kw["prologue"] == _lib.BN_PLAIN else torch.relu(src)
            ref = op @ W.t() + kw["bias"] + (kw["add1"] if kw.get("add1") is not None else 0)
        else:
            ref = (src @ W) * (kw["pre_rows"] > 0)
        torch.cuda.synchronize()
        out = kw["out"]
        err = float((out - ref).abs().max()) / (float(ref.abs().max()) or 1.0)
        bad_rows = int(((out - ref).abs().amax(-1) > 1e-4 * float(ref.abs().max())).sum())
        calls.append(err)
        if kw["mode"] == _lib.BN_BWD:
            snaps[L] = (kw["out"], kw["out"].clone(), kw["src"], kw["src"].clone(), kw["pre_rows"].clone())
        print(f"{'FWD' if kw['mode'] == _lib.BN_FWD else 'BWD'} layer {L} rows {kw['n_rows']}: rel err {err:.2e}, "
              f"rows off by > 1e-4 of max: {bad_rows} of {out.shape[0]}", flush=True)

    def grads(hip, latent_grad):
        net.hip_backward = hip
        net.zero_grad(set_to_none=True)
        lat = net.encoder.latent.detach().clone().requires_grad_(latent_grad)
        net.encoder.latent = lat
        x = xyz.clone().requires_grad_(True)
        out = net(x, coarse=True, viewdirs=vd)
        (out * w).sum().backward()
        r = {n: p.grad.detach().clone() for n, p in net.mlp_coarse.named_parameters() if p.grad is not None}
        r["xyz"] = x.grad.detach().clone()
        if latent_grad:
            r["latent"] = lat.grad.detach().clone()
        return r

    orig_gather = layer_train._gather
    gathered = []

    def gather(fused, tab, K, NS, p, B, C):
        out = orig_gather(fused, tab, K, NS, p, B, C)
        gathered.append(out.clone())
        return out

    from avr import ops
    orig_wg = ops.weight_grads
    wg_calls = []

    def wg(layers, n_rows, n_split=None):
        wg_calls.append([l[0].clone() for l in layers])
        return orig_wg(layers, n_rows, n_split)

    bn_train._layer, bn_train._run = layer, run
    layer_train._gather = gather
    ops.weight_grads = wg
    try:
        gh = grads(True, False)
    finally:
        bn_train._layer, bn_train._run = orig_layer, orig_run
        layer_train._gather = orig_gather
        ops.weight_grads = orig_wg
    # torch reference of the gradients at every block input (after the spade product), by hand
    mlp = net.mlp_coarse
    from avr.models import combine_interleaved
    with torch.enable_grad():
        feat, zft = net.mlp_inputs(xyz, vd)
        x = mlp.lin_in(zft)
        xins = []
        for b in range(mlp.n_blocks):
            if b == mlp.combine_layer:
                x = combine_interleaved(x, (NS, B), mlp.combine_type)
            if b < mlp.combine_layer:
                x = mlp.scale_z[b](feat) * x + mlp.lin_z[b](feat) if mlp.use_spade else x + mlp.lin_z[b](feat)
            x.retain_grad()
            xins.append(x)
            x = mlp.blocks[b](x)
        o = mlp.lin_out(torch.relu(x)).reshape(-1, B, 4)
        o = torch.cat([torch.sigmoid(o[..., :3]), torch.relu(o[..., 3:4])], -1).reshape(SB, B, 4)
        (o * w).sum().backward()
    names = ["gp2_0", "g_0", "gp2_1", "g_1", "Gz0", "Gz1", "Gs0", "Gs1", "g_in0"]
    for nm, G in zip(names, wg_calls[0]):
        if nm in ("Gz0", "Gz1"):
            ref = xins[int(nm[-1])].grad.reshape(G.shape)
            print(f"{nm}: rel err vs torch {float((G - ref).abs().max()) / float(ref.abs().max()):.2e}", flush=True)
    print("wg calls", [len(c) for c in wg_calls])
    for L, (t, t0, src, src0, _) in sorted(snaps.items()):
        print(f"BWD layer {L}: out changed after the call by {float((t - t0).abs().max()):.2e}, src changed by "
              f"{float((src - src0).abs().max()):.2e}")
    gp1_0, g0, gp2_0, xin0 = snaps[2][1], snaps[3][3], snaps[2][3], snaps[2][4]
    W0 = mlp.blocks[0].fc_0.weight.detach()
    xr = xins[0].detach().reshape(xin0.shape)
    print(f"Xin0 vs torch: {float((xin0 - xr).abs().max()) / float(xr.abs().max()):.2e}; masks differ at "
          f"{int(((xin0 > 0) != (xr > 0)).sum())} entries")
    gp1_ref = (gp2_0 @ W0) * (xr > 0)
    print(f"gp1_0 vs torch-mask recompute: {float((gp1_0 - gp1_ref).abs().max()) / float(gp1_ref.abs().max()):.2e}")
    ref1 = xins[1].grad.reshape(g0.shape)
    print(f"g0 vs torch dL/dXpre1: {float((g0 - ref1 * 0).abs().max()):.2e} (|g0| max)")
    ref = xins[0].grad.reshape(gp1_0.shape)
    print(f"(g0 + gp1_0) vs torch: {float((g0 + gp1_0 - ref).abs().max()) / float(ref.abs().max()):.2e}; "
          f"Gz0 vs (g0 + gp1_0): {float((wg_calls[0][4] - (g0 + gp1_0)).abs().max()):.2e}")
    mlp = net.mlp_coarse
    with torch.no_grad():
        feat, _ = net.mlp_inputs(xyz, vd)
        nz = len(mlp.lin_z)
        refs = [mlp.lin_z[b](feat) - (0 if mlp.use_spade else mlp.lin_z[b].bias) for b in range(nz)]
        refs += [mlp.scale_z[b](feat) for b in range(nz)] if mlp.use_spade else []
        refs += [feat]
    for i, (got, ref) in enumerate(zip(gathered, refs)):
        d = (got - ref).abs()
        print(f"gather {i}: rel err {float(d.max()) / float(ref.abs().max()):.2e}, rows off by > 1e-4: "
              f"{int((d.amax(-1) > 1e-4 * float(ref.abs().max())).sum())} of {ref.shape[0]}; first bad rows "
              f"{torch.nonzero(d.amax(-1) > 1e-4 * float(ref.abs().max())).reshape(-1)[:8].tolist()}", flush=True)
    print(f"{len(calls)} layer calls, worst rel err {max(calls):.2e}")
    gh2 = grads(True, True)
    gt = grads(False, True)
    for k in gt:
        s_ = float(gt[k].abs().max()) or 1.0
        e1 = float((gh[k] - gt[k]).abs().max()) / s_ if k in gh else -1
        e2 = float((gh2[k] - gt[k]).abs().max()) / s_
        print(f"   {k}: HIP (no latent grad) vs torch {e1:.2e}, HIP (latent grad) vs torch {e2:.2e}")
    _ = layer_train


if __name__ == "__main__":
    main()
