"""Layer-by-layer HIP training of the ResnetFC options the fused training kernels do not carry: use_spade
(models.py:528-534, 585-587: before block b < combine_layer, x = scale_z[b](z) * x + lin_z[b](z)) and NS > 1
source views (models.py:566-579: block combine_layer starts from combine_interleaved, the mean or max over the
views, utils.py:71-81), alone or together, ReLU, no BatchNorm.

Both put an elementwise step between the fused kernels' 64-sample GEMM chains: the spade product needs the
interpolated scale rows, the combine mixes rows of different views (workgroups), so this path runs the MLP one
layer at a time on avr_bn_layer_run (the BatchNorm path's x3 layer GEMM over row-major fp32 rows, with identity
statistics: the operand is relu(x), the backward's mask [pre > 0]) with the elementwise steps between:
  forward   X[0] = lin_in(z_feature); per block b: (b < combine_layer) X'[b] = S_b * X[b] + T_b with T_b / S_b the
            bilinear blends of the per-texel lin_z / scale_z tables (avr_latent_features on the x3 tables: both
            carry their biases with use_spade, the product in torch; without it T_b has none, lin_z's bias is
            folded into the producing layer's bias and T_b is gathered in that layer's epilogue, avr_bn_layer's
            lin_z_table); (b == combine_layer, NS > 1) X'[b] = combine(X[b]) (torch); N[b] = fc_0(relu(X'[b]));
            X[b+1] = fc_1(relu(N[b])) + X'[b]; out = lin_out(relu(X[nb])), sigmoid / relu (avr_lin_out_fwd_rows).
  backward  lin_out and its activations (avr_lin_out_bwd_rows); the transposed layers on avr_bn_layer_run
            (W^T . g masked by [pre > 0]; fc_0^T adds the residual's g in its epilogue and publishes the max of
            what it stores), the spade product rule (d X = S * g, d S = g * X: avr_spade_bwd_rows; d T = g) and
            the combine's adjoint (the mean's in closed form, torch's for the max) between them; every weight
            gradient on avr_weight_grads (split-K x3; relu(X) rebuilt from the pre-activation rows in the
            staging), scale_z's against (g * X) rows; the latent / point gradients through the input functions
            as in avr.field._FieldTrain (the features' gradient on the lin_z^T layers where they apply).
"""
import ctypes

import torch

from . import _lib
from ._lib import call, ptr, stream_of

F32 = torch.float32


def layer_train_eligible(net):
    """A NewPixelNeRFNet this path trains: what the fused field runs for inference (avr.field.fused_eligible, with
    NS > 1 its multiview form), ReLU, no BatchNorm, and use_spade or NS > 1 source views (the other nets train on
    the fused kernels, avr.field._FieldTrain), d_latent a multiple of 64 up to 512 (x3 tables)."""
    from .field import fused_eligible, softplus_beta, uses_bn
    try:
        mlps = [net.mlp_coarse] + ([net.mlp_fine] if net.mlp_fine is not None else [])
        ns = net.num_views_per_obj
        if any(uses_bn(m) or softplus_beta(m) != 0.0 for m in mlps):
            return False
        if not (ns > 1 or any(getattr(m, "use_spade", False) for m in mlps)):
            return False
        if not (net.d_latent % 64 == 0 and net.d_latent <= 512 and getattr(net, "field_precision", "x3") == "x3"):
            return False
        return fused_eligible(net, multiview=ns > 1)
    except AttributeError:
        return False


def train_param_names_layers(mlp):
    from .field import train_param_names
    names = train_param_names(mlp)
    if getattr(mlp, "use_spade", False):
        for b in range(min(mlp.combine_layer, mlp.n_blocks)):
            names += [f"scale_z.{b}.weight", f"scale_z.{b}.bias"]
    return names


def forward_train_layers(fused, xyz, viewdirs, coarse):
    """The rf(xyz, viewdirs, coarse) protocol on this path (autograd when enabled)."""
    mlp = fused._mlp(coarse)
    names = train_param_names_layers(mlp)
    named, _, _ = fused._state(mlp)
    return _FieldTrainLayers.apply(fused, coarse, names, xyz, viewdirs, fused.net.encoder.latent,
                                   *[named[n] for n in names])


def _gather(fused, tab, K, NS, p, B, C):
    """Bilinear blends (avr_latent_features' lookup and order) of the (K, H*W, C) per-texel rows `tab` at the
    points p (K, B, 3), scene k seen from source view k (object k // NS) -> (K * B, C)."""
    out = torch.empty(K * B, C, device=p.device, dtype=F32)
    for g0 in range(0, K, _lib.AVR_MAX_SCENES):
        n = min(_lib.AVR_MAX_SCENES, K - g0)
        views = fused.views(range(g0, g0 + n), NS)
        call("avr_latent_features_batch", views, n, ptr(tab[g0]), C, ptr(p[g0]), B, ptr(out[g0 * B]),
             stream_of(out))
    return out


class _Ident:
    """Identity statistics: the BatchNorm layer kernels then compute relu(x) operands and [pre > 0] masks."""

    def __init__(self, H, dev):
        self.zero = torch.zeros(H, device=dev, dtype=F32)
        self.one = torch.ones(H, device=dev, dtype=F32)


class _FieldTrainLayers(torch.autograd.Function):
    """Autograd of NewPixelNeRFNet.forward (models.py:739-863) for use_spade / NS > 1 nets, layer by layer (see the
    module docstring), for train.py's loss.backward() (train.py:108-114)."""

    @staticmethod
    def forward(ctx, fused, coarse, names, xyz, viewdirs, latent, *params):
        from .bn_train import _layer, _partial, _run
        from .models import combine_interleaved
        from .ops import lin_out_rows
        net = fused.net
        mlp = fused._mlp(coarse)
        P = dict(zip(names, params))
        entry = fused.packed(coarse)
        dims = entry.dims
        H, nb, nz = dims.d_hidden, dims.n_blocks, dims.n_lin_z
        spade = bool(dims.spade)
        NS = net.num_views_per_obj
        cl = mlp.combine_layer if NS > 1 else nb
        SB, B, _ = xyz.shape
        K = SB * NS
        M1, M2 = K * B, SB * B
        dev = xyz.device
        stream = stream_of(xyz)
        with torch.no_grad():
            p = xyz.detach().to(F32).repeat_interleave(NS, 0).contiguous()      # (object, view) rows
            zf = net.z_features(xyz.detach(), viewdirs.detach()).to(F32)          # (M1, d_in)
            d_in = zf.shape[1]
            zs = d_in + (-d_in) % 4
            zfp = torch.zeros(M1, zs, device=dev, dtype=F32)
            zfp[:, :d_in] = zf
            tables = fused.tables_batch(coarse, K, fast=True)                     # (K, n_tables, HW, H)
            # without use_spade, X'[b] = X[b] + T_b: the T rows gathered in the epilogue of the layer producing X[b]
            # (avr_bn_layer's lin_z_table, as avr.bn_train; nz <= combine_layer, so X[b] is X'[b] and no T row is
            # stored); use_spade's product, or more scenes than one launch takes, gathers them here
            zk = not spade and 0 < nz and K <= _lib.AVR_MAX_SCENES
            views = fused.views(range(K), NS) if zk else None

            def lin_z(b):
                if not zk or b >= nz:
                    return {}
                return dict(lin_z_table=tables[0, b], lin_z_scene_stride=tables.stride(0), xyz=p,
                            views=ctypes.addressof(views), n_views=K, rows_per_scene=B)
            T = [] if zk else [_gather(fused, tables[:, b].contiguous(), K, NS, p, B, H) for b in range(nz)]
            S = [_gather(fused, tables[:, nz + b].contiguous(), K, NS, p, B, H) for b in range(nz)] if spade else []
            lz_b = [P[f"lin_z.{b}.bias"].detach().to(F32) for b in range(nz)]
            fold = (lambda b: 0) if spade else (lambda b: lz_b[b] if b < nz else 0)   # biases in the tables?
            b_in = (P["lin_in.bias"].detach().to(F32) + fold(0)).contiguous()
            b0 = [P[f"blocks.{b}.fc_0.bias"].detach().to(F32).contiguous() for b in range(nb)]
            b1 = [(P[f"blocks.{b}.fc_1.bias"].detach().to(F32) + fold(b + 1)).contiguous() for b in range(nb)]
            idt = _Ident(H, dev)
            part = _partial(M1, H, dev)
            amax = torch.zeros(2 * nb, device=dev, dtype=torch.int32)
            blob = entry.packed
            rows = lambda b: M1 if b < cl else M2   # noqa: E731  (rows of block b)
            Xpre = [torch.empty(M1, H, device=dev, dtype=F32)]
            _run(dims, _layer(n_rows=M1, mode=_lib.BN_FWD, prologue=_lib.BN_PLAIN, in_dim=64, in_valid=d_in, src=zfp,
                              ld_src=zs, blob=blob, layer=0, bias=b_in, out=Xpre[0], partial=part, **lin_z(0)),
                 stream)
            Xin, N = [], []
            for b in range(nb):
                x = Xpre[b]
                if b < nz and not zk:                                       # models.py:583-588
                    x = torch.addcmul(T[b], S[b], x) if spade else x + T[b]
                if b == cl and NS > 1:
                    x = combine_interleaved(x, (NS, B), mlp.combine_type).reshape(M2, H)
                x = x.contiguous()
                Xin.append(x)
                m = rows(b)
                N.append(torch.empty(m, H, device=dev, dtype=F32))
                _run(dims, _layer(n_rows=m, mode=_lib.BN_FWD, prologue=_lib.BN_RELU, in_dim=H, in_valid=H, src=x,
                                  ld_src=H, in_mu=idt.zero, in_scale=idt.one, in_shift=idt.zero,
                                  operand_max=amax[2 * b:], blob=blob, layer=2 + 2 * b, bias=b0[b], out=N[b],
                                  partial=part), stream)
                Xpre.append(torch.empty(m, H, device=dev, dtype=F32))
                _run(dims, _layer(n_rows=m, mode=_lib.BN_FWD, prologue=_lib.BN_RELU, in_dim=H, in_valid=H, src=N[b],
                                  ld_src=H, in_mu=idt.zero, in_scale=idt.one, in_shift=idt.zero,
                                  operand_max=amax[2 * b + 1:], blob=blob, layer=3 + 2 * b, bias=b1[b], add1=x,
                                  out=Xpre[b + 1], partial=part, **lin_z(b + 1)), stream)
            # lin_out + sigmoid / relu in one pass (max relu(x) for its weight gradient; relu(x) not stored)
            out, a_max = lin_out_rows(Xpre[nb], P["lin_out.weight"].detach(), P["lin_out.bias"].detach())
            out = out.reshape(SB, B, 4)
        ctx.fused, ctx.coarse, ctx.names, ctx.entry = fused, coarse, names, entry
        ctx.keep = (Xpre, Xin, N, S, amax, zfp, a_max, idt, p, cl)
        ctx.save_for_backward(xyz, viewdirs, latent, out, *params)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from .bn_train import _layer, _partial, _run
        from .models import combine_interleaved
        from .field import _feat_grad
        from .ops import _max_bits, lin_out_rows_bwd, spade_bwd_rows, sum_of_products, weight_grads
        xyz, viewdirs, latent, out, *params = ctx.saved_tensors
        Xpre, Xin, N, S, amax, zfp, a_max, idt, p, cl = ctx.keep
        ctx.keep = None
        fused, entry, names = ctx.fused, ctx.entry, ctx.names
        net = fused.net
        mlp = fused._mlp(ctx.coarse)
        P = dict(zip(names, params))
        dims = entry.dims
        H, nb, nz = dims.d_hidden, dims.n_blocks, dims.n_lin_z
        spade = bool(dims.spade)
        NS = net.num_views_per_obj
        SB, B, _ = xyz.shape
        K = SB * NS
        M1, M2 = K * B, SB * B
        dev = xyz.device
        stream = stream_of(xyz)
        want_latent = ctx.needs_input_grad[5] and not net.stop_encoder_grad
        want_xyz = ctx.needs_input_grad[3]
        with torch.no_grad():
            bwd = fused.packed_bwd(ctx.coarse, entry)
            part = _partial(M1, H, dev)
            # the activations' backward (d4), lin_out^T and its relu's backward in one pass
            d4, g, d4_max = lin_out_rows_bwd(grad_out.reshape(M2, 4), out.reshape(M2, 4),
                                             P["lin_out.weight"].detach(), Xpre[nb])
            wl1, wl2 = [], []           # weight-gradient layers over M1 / M2 rows
            Gz, Gs, Gz_max, Gs_max = [None] * nz, [None] * nz, [None] * nz, [None] * nz
            blk = [None] * nb
            # max |operand| of every backward layer call, published by the layer kernels (the weight gradients'
            # scales for gp2 and g without a reduction pass over the rows): [2b] fc_0^T's, [2b + 1] fc_1^T's
            omax = torch.zeros(2 * nb, device=dev, dtype=torch.int32)
            relu_x = "relu"                                # X = relu(rows), rebuilt in the staging
            # max |stored rows| of each block's fc_0^T launch (ABI 14 out_max): Gz[b] for b < n_lin_z (<= the
            # combine layer, so no combine adjoint follows them), and g_in0 (lin_in's output gradient) unless
            # spade's product or the views' combine follows block 0's launch
            fc0t_max = torch.zeros(max(nb, 1), device=dev, dtype=torch.int32)
            in0_direct = nb > 0 and not spade and not (cl == 0 and NS > 1)
            for b in range(nb - 1, -1, -1):
                m = M1 if b < cl else M2
                # fc_1^T: gradient at N[b]; fc_0^T: the fc_0 path's gradient at X'[b]
                gp2 = torch.empty(m, H, device=dev, dtype=F32)
                _run(dims, _layer(n_rows=m, mode=_lib.BN_BWD, prologue=_lib.BN_PLAIN, in_dim=H, in_valid=H, src=g,
                                  ld_src=H, operand_max=omax[2 * b + 1:], blob=bwd, layer=3 + 2 * b, out=gp2,
                                  pre_rows=N[b], out_mu=idt.zero, out_invstd=idt.one, out_scale=idt.one,
                                  out_shift=idt.zero, partial=part), stream)
                # fc_0^T, the residual's g added in its epilogue: d loss / d X'[b] (residual + fc_0 path)
                gin = torch.empty(m, H, device=dev, dtype=F32)
                _run(dims, _layer(n_rows=m, mode=_lib.BN_BWD, prologue=_lib.BN_PLAIN, in_dim=H, in_valid=H, src=gp2,
                                  ld_src=H, operand_max=omax[2 * b:], blob=bwd, layer=2 + 2 * b, out=gin,
                                  pre_rows=Xin[b], out_mu=idt.zero, out_invstd=idt.one, out_scale=idt.one,
                                  out_shift=idt.zero, add1=g, out_max=fc0t_max[b:b + 1], partial=part), stream)
                blk[b] = [(gp2, Xin[b], omax[2 * b:2 * b + 1], amax[2 * b:2 * b + 1], True, relu_x),
                          (g, N[b], omax[2 * b + 1:2 * b + 2], amax[2 * b + 1:2 * b + 2], True, relu_x)]
                if b == cl and NS > 1 and mlp.combine_type == "average":
                    # the mean's adjoint (torch's MeanBackward: the gradient expanded over the views, / NS)
                    gin = (gin.reshape(SB, 1, B, H).expand(SB, NS, B, H) / NS).reshape(M1, H)   # one pass
                elif b == cl and NS > 1:                       # torch's adjoint of the views' combine
                    with torch.enable_grad():
                        xr = Xpre[b].detach().requires_grad_(True)
                        yc = combine_interleaved(xr, (NS, B), mlp.combine_type).reshape(M2, H)
                        gin, = torch.autograd.grad(yc, xr, gin)
                if b < nz:
                    Gz[b] = gin.contiguous()
                    Gz_max[b] = fc0t_max[b:b + 1]
                    if spade:                                  # X' = S * X + T (models.py:585-587)
                        # dS = g * X (+ its max for scale_z's weight gradient), dX = S * g: one pass
                        Gs[b], gin, Gs_max[b] = spade_bwd_rows(Gz[b], Xpre[b].contiguous(), S[b])
                g = gin.contiguous()
            g_in0 = g                                          # d loss / d lin_in output
            for b in range(nb):
                (wl1 if b < cl else wl2).extend(blk[b])
            g_in0_max = fc0t_max[0:1] if in0_direct else _max_bits(g_in0)
            lat_feat = None
            if nz > 0:
                hwc = fused.latent_hwc_all(latent)
                if hwc.shape[0] != K:    # one map shared by the scenes (or more maps than scenes)
                    hwc = hwc[torch.clamp(torch.arange(K, device=dev), max=hwc.shape[0] - 1)].contiguous()
                lat_feat = _gather(fused, hwc, K, NS, p, B, net.d_latent)
                lat_max = fused.latent_max_bits(latent)
                for b in range(nz):
                    zmax = Gz_max[b]
                    wl1.append((Gz[b], lat_feat, zmax, lat_max, True))
                for b in range(nz if spade else 0):
                    wl1.append((Gs[b], lat_feat, Gs_max[b], lat_max, True))
            wl1.append((g_in0, zfp, g_in0_max, _max_bits(zfp), True))
            wl2.append((d4, Xpre[nb], d4_max, a_max, True, relu_x))
            if M1 == M2:     # one source view: every layer over the same rows, one launch
                r = weight_grads(wl1 + wl2, M1)
                r1, r2 = r[:len(wl1)], r[len(wl1):]
            else:
                r1, r2 = weight_grads(wl1, M1), weight_grads(wl2, M2)
            grads = {"lin_out.weight": r2[-1][0], "lin_out.bias": r2[-1][1]}
            i1, i2 = 0, 0
            for b in range(nb):
                if b < cl:
                    (w0, c0), (w1, c1) = r1[i1], r1[i1 + 1]
                    i1 += 2
                else:
                    (w0, c0), (w1, c1) = r2[i2], r2[i2 + 1]
                    i2 += 2
                grads[f"blocks.{b}.fc_0.weight"], grads[f"blocks.{b}.fc_0.bias"] = w0, c0
                grads[f"blocks.{b}.fc_1.weight"], grads[f"blocks.{b}.fc_1.bias"] = w1, c1
            for b in range(nz):
                grads[f"lin_z.{b}.weight"], grads[f"lin_z.{b}.bias"] = r1[i1]
                i1 += 1
            for b in range(nz if spade else 0):
                grads[f"scale_z.{b}.weight"], grads[f"scale_z.{b}.bias"] = r1[i1]
                i1 += 1
            w_in, c_in = r1[i1]
            grads["lin_in.weight"], grads["lin_in.bias"] = w_in[:, :net.d_in].contiguous(), c_in
        d_latent = d_xyz = None
        if want_latent or want_xyz:
            with torch.enable_grad():
                lat = latent.detach().requires_grad_(want_latent)
                x = xyz.detach().requires_grad_(want_xyz)
                feat, zft = net.mlp_inputs(x, viewdirs.detach(), latent=lat)
                outs, grads_out = [], []
                # with stop_encoder_grad the looked-up latent is detached (models.py:810-811): no gradient reaches
                # the points through the lookup, z_feature's part alone (as avr.field._FieldTrain)
                if nz > 0 and not net.stop_encoder_grad:
                    outs.append(feat)
                    if spade:
                        pairs = [(Gz[b], P[f"lin_z.{b}.weight"].detach()) for b in range(nz)]
                        pairs += [(Gs[b], P[f"scale_z.{b}.weight"].detach()) for b in range(nz)]
                        grads_out.append(sum_of_products(pairs))
                    else:   # the lin_z^T layers on the x3 layer GEMM where they apply (avr.field._feat_grad)
                        grads_out.append(_feat_grad(fused, entry, bwd, Gz, P, M1))
                if want_xyz:
                    outs.append(zft)
                    grads_out.append(g_in0 @ P["lin_in.weight"].detach())
                wrt = ([lat] if want_latent else []) + ([x] if want_xyz else [])
                res_in = torch.autograd.grad(outs, wrt, grads_out, allow_unused=True)
            if want_latent:
                d_latent = res_in[0] if res_in[0] is not None else torch.zeros_like(latent)
            if want_xyz:
                d_xyz = res_in[-1] if res_in[-1] is not None else torch.zeros_like(xyz)
        return (None, None, None, d_xyz, None, d_latent) + tuple(
            grads[n] if ctx.needs_input_grad[6 + i] else None for i, n in enumerate(names))
