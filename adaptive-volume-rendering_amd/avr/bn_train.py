"""Training-mode BatchNorm nets on the HIP path: train.py --bn (train.py:210, :265).

ResnetBlockFC(bn=True) (models.py:430-432, 454-461) computes relu(bn_0(x)) -> fc_0 -> relu(bn_0(net)) ->
fc_1, + x, with bn_0 applied twice per block and, in training mode, batch statistics over every row of the
field call (bn_1 is unused). Those statistics are a reduction over all rows between two GEMMs, which the
fused 64-sample field kernels cannot do, so this path runs the ResnetFC layer by layer on the C ABI's
avr_bn_layer_run: each hidden GEMM on the split-fp16 MFMA of the fused kernels over row-major fp32 rows, with
the normalisation + relu of its input in the prologue and its output's per-workgroup column statistics in
the epilogue; avr_bn_stats between launches turns them into the batch mean / invstd (fp64 combine) and
updates the running statistics as torch does. The backward runs the same GEMMs on the transposed weights,
with torch's batch_norm backward, (g - mean g - xhat mean(g xhat)) * gamma * invstd, built into the next
GEMM's prologue (avr_bn_grad_stats reduces the two means, dgamma and dbeta); the weight gradients are the
existing split-K x3 kernel (avr_weight_grads). The relu'd operands relu(bn_0(.)) are never stored: the
backward's relu masks and the weight gradients' staging rebuild them from the pre-BN rows (ABI 12).

lin_out's 4 outputs with sigmoid / relu and their backward run as one pass over the rows each
(avr_lin_out_fwd_rows / avr_lin_out_bwd_rows). The thin ends stay in torch: the z_feature input (positional
encoding, models.py:763-789) and the input gradients (grid_sample adjoint), as in avr.field._FieldTrain.
"""
import ctypes

import torch

from . import _lib
from ._lib import BnLayer, call, ptr, stream_of

F32 = torch.float32


def _bn_blocks(mlp):
    return [blk.bn_0 for blk in mlp.blocks]


def bn_train_eligible(net):
    """A NewPixelNeRFNet the BatchNorm training path runs: the fused field's configuration (avr.field.
    fused_eligible, one source view) except that every ResnetFC uses bn=True with its BatchNorm in training
    mode (batch statistics), ReLU, no use_spade, d_latent a multiple of 64 up to 512 (x3 lin_z tables)."""
    from .field import fused_eligible, uses_bn, softplus_beta
    try:
        mlps = [net.mlp_coarse] + ([net.mlp_fine] if net.mlp_fine is not None else [])
        if not all(uses_bn(m) and all(blk.bn for blk in m.blocks) for m in mlps):
            return False
        if not all(m.training and all(b.training and b.affine for b in _bn_blocks(m)) for m in mlps):
            return False
        if any(getattr(m, "use_spade", False) or softplus_beta(m) != 0.0 for m in mlps):
            return False
        if not (net.d_latent % 64 == 0 and net.d_latent <= 512):
            return False
        # the rest of the fused configuration (inputs, encoder, widths, one view); its BN check wants eval mode,
        # so it is asked about a stand-in state
        saved = [(b, b.training) for m in mlps for b in _bn_blocks(m)] + [(m, m.training) for m in mlps]
        saved += [(blk, blk.training) for m in mlps for blk in m.blocks]
        try:
            for mod, _ in saved:
                mod.training = False
            return fused_eligible(net)
        finally:
            for mod, t in saved:
                mod.training = t
    except AttributeError:
        return False


class _Stats:
    """Batch statistics of one BatchNorm application: mu, invstd, scale = gamma * invstd (d_hidden each)."""

    def __init__(self, H, dev):
        buf = torch.empty(3, H, device=dev, dtype=F32)
        self.mu, self.invstd, self.scale = buf[0], buf[1], buf[2]


def _layer(**kw):
    """An avr_bn_layer from keyword fields (tensors become their device addresses)."""
    l = BnLayer()
    for k, v in kw.items():
        setattr(l, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
    return l


def _run(dims, layer, stream):
    call("avr_bn_layer_run", ctypes.byref(dims), ctypes.byref(layer), stream)


def _partial(M, H, dev):
    """The per-workgroup column partials of avr_bn_layer_run plus the fold scratch of avr_bn_stats."""
    n = ctypes.c_int64(0)
    call("avr_bn_partial_floats", M, H, ctypes.byref(n))
    return torch.empty(n.value, device=dev, dtype=F32)


def _momentum(bn):
    """torch's BatchNorm momentum, None = cumulative average (1 / num_batches_tracked after the increment)."""
    if bn.momentum is None:
        return 1.0 / float(bn.num_batches_tracked.item())
    return float(bn.momentum)


def _bn_stats(bn, part, M, H, stats, stream):
    """avr_bn_stats for one training-mode application of `bn` (the running statistics updated as torch's
    batch_norm does: num_batches_tracked += 1, momentum, unbiased variance)."""
    track = bn.track_running_stats and bn.running_mean is not None
    if track:
        bn.num_batches_tracked.add_(1)
    call("avr_bn_stats", ptr(part), M, H, ptr(bn.weight), ctypes.c_float(bn.eps),
         ctypes.c_float(_momentum(bn) if track else 0.0), ptr(bn.running_mean) if track else None,
         ptr(bn.running_var) if track else None, ptr(stats.mu), ptr(stats.invstd), ptr(stats.scale), stream)
    if track:
        # the kernel wrote them through raw pointers: advance their versions as torch's in-place update does,
        # so every (data_ptr, _version)-keyed cache (FusedField.packed's eval blob with the running statistics
        # folded in, GraphedRenderer's capture check) sees the new statistics
        torch.autograd.graph.increment_version(bn.running_mean)
        torch.autograd.graph.increment_version(bn.running_var)


def train_param_names_bn(mlp):
    from .field import train_param_names
    names = train_param_names(mlp)
    for b in range(mlp.n_blocks):
        names += [f"blocks.{b}.bn_0.weight", f"blocks.{b}.bn_0.bias"]
    return names


def forward_train_bn(fused, xyz, viewdirs, coarse):
    """The rf(xyz, viewdirs, coarse) protocol for a training-mode BatchNorm net (autograd when enabled)."""
    mlp = fused._mlp(coarse)
    names = train_param_names_bn(mlp)
    named, _, _ = fused._state(mlp)
    params = [named[n] for n in names]
    return _FieldTrainBN.apply(fused, coarse, names, xyz, viewdirs, fused.net.encoder.latent, *params)


class _FieldTrainBN(torch.autograd.Function):
    """Autograd of NewPixelNeRFNet.forward (models.py:739-863) with ResnetFC(bn=True) in training mode
    (train.py --bn), for train.py's loss.backward() (train.py:108-114). See the module docstring."""

    @staticmethod
    def forward(ctx, fused, coarse, names, xyz, viewdirs, latent, *params):
        from .ops import lin_out_rows
        net = fused.net
        mlp = fused._mlp(coarse)
        P = dict(zip(names, params))
        entry = fused.packed(coarse, bn_fold=False)
        dims = entry.dims
        H, nb, nz = dims.d_hidden, dims.n_blocks, dims.n_lin_z
        SB, B, _ = xyz.shape
        M = SB * B
        dev = xyz.device
        stream = stream_of(xyz)
        if M < 2:
            raise ValueError("Expected more than 1 value per channel when training (BatchNorm, "
                             f"got {M} rows)")
        with torch.no_grad():
            # lin_in's input: z_feature rows padded to 16 B (the fused kernels' zf layout)
            zf = net.z_features(xyz.detach(), viewdirs.detach()).to(F32)
            d_in = zf.shape[1]
            zs = d_in + (-d_in) % 4
            zfp = torch.zeros(M, zs, device=dev, dtype=F32)
            zfp[:, :d_in] = zf
            # lin_z[b](latent features) rows: gathered from the per-texel tables in the layer epilogues
            tables = fused.tables_batch(coarse, SB, fast=True, bn_fold=False)
            views = fused.views(range(SB))
            p = xyz.detach().to(F32).contiguous()

            def lin_z(b):
                """avr_bn_layer fields adding lin_z[b](latent features) rows (none past the last lin_z)."""
                if b >= nz:
                    return {}
                return dict(lin_z_table=tables[0, b], lin_z_scene_stride=tables.stride(0), xyz=p,
                            views=ctypes.addressof(views), n_views=SB, rows_per_scene=B)
            # biases with the lin_z biases folded where the tables (no bias) are added
            lz_b = [P[f"lin_z.{b}.bias"].detach() for b in range(nz)]
            b_in = P["lin_in.bias"].detach() + (lz_b[0] if nz > 0 else 0)
            b0 = [P[f"blocks.{b}.fc_0.bias"].detach().contiguous() for b in range(nb)]
            b1 = [P[f"blocks.{b}.fc_1.bias"].detach() + (lz_b[b + 1] if b + 1 < nz else 0) for b in range(nb)]
            b_in, b1 = b_in.to(F32).contiguous(), [t.to(F32).contiguous() for t in b1]
            betas = [P[f"blocks.{b}.bn_0.bias"].detach().to(F32).contiguous() for b in range(nb)]
            X = torch.empty(nb + 1, M, H, device=dev, dtype=F32)        # block inputs (pre-BN) + the last output
            N = torch.empty(max(nb, 1), M, H, device=dev, dtype=F32)    # fc_0 outputs (pre-BN)
            # max |relu(bn_0(.))| of each hidden GEMM's operand (the operands themselves are not stored: the
            # backward's relu masks and the weight gradients rebuild them from X / N and the statistics)
            amax = torch.zeros(2 * nb + 2, device=dev, dtype=torch.int32)
            part = _partial(M, H, dev)
            st1 = [_Stats(H, dev) for _ in range(nb)]
            st2 = [_Stats(H, dev) for _ in range(nb)]
            bns = _bn_blocks(mlp)
            blob = entry.packed
            _run(dims, _layer(n_rows=M, mode=_lib.BN_FWD, prologue=_lib.BN_PLAIN, in_dim=64, in_valid=d_in,
                              src=zfp, ld_src=zs, blob=blob, layer=0, bias=b_in, out=X[0], partial=part,
                              **lin_z(0)), stream)
            for b in range(nb):
                bn = bns[b]
                _bn_stats(bn, part, M, H, st1[b], stream)
                _run(dims, _layer(n_rows=M, mode=_lib.BN_FWD, prologue=_lib.BN_RELU, in_dim=H, in_valid=H,
                                  src=X[b], ld_src=H, in_mu=st1[b].mu, in_scale=st1[b].scale, in_shift=betas[b],
                                  operand_max=amax[2 * b:], blob=blob, layer=2 + 2 * b,
                                  bias=b0[b], out=N[b], partial=part), stream)
                _bn_stats(bn, part, M, H, st2[b], stream)
                _run(dims, _layer(n_rows=M, mode=_lib.BN_FWD, prologue=_lib.BN_RELU, in_dim=H, in_valid=H,
                                  src=N[b], ld_src=H, in_mu=st2[b].mu, in_scale=st2[b].scale, in_shift=betas[b],
                                  operand_max=amax[2 * b + 1:], blob=blob,
                                  layer=3 + 2 * b, bias=b1[b], add1=X[b], out=X[b + 1], partial=part,
                                  **lin_z(b + 1)), stream)
            # lin_out on relu(x) (4 outputs; models.py:592), sigmoid rgb / relu sigma (models.py:856-862), and
            # max relu(x) for its weight gradient's scale (relu(x) itself is not stored)
            out, a_max = lin_out_rows(X[nb], P["lin_out.weight"].detach(), P["lin_out.bias"].detach())
            out = out.reshape(SB, B, 4)
        ctx.fused, ctx.coarse, ctx.names, ctx.entry = fused, coarse, names, entry
        ctx.keep = (X, N, amax, a_max, zfp, st1, st2, betas)
        ctx.save_for_backward(xyz, viewdirs, latent, out, *params)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from .ops import _max_bits, lin_out_rows_bwd, sum_of_products, weight_grads
        xyz, viewdirs, latent, out, *params = ctx.saved_tensors
        fused, entry, names = ctx.fused, ctx.entry, ctx.names
        X, N, amax, a_max, zfp, st1, st2, betas = ctx.keep
        ctx.keep = None
        net = fused.net
        P = dict(zip(names, params))
        dims = entry.dims
        H, nb, nz = dims.d_hidden, dims.n_blocks, dims.n_lin_z
        SB, B, _ = xyz.shape
        M = SB * B
        dev = xyz.device
        stream = stream_of(xyz)
        mlp = fused._mlp(ctx.coarse)
        bns = _bn_blocks(mlp)
        want_latent = ctx.needs_input_grad[5] and not net.stop_encoder_grad
        want_xyz = ctx.needs_input_grad[3]
        with torch.no_grad():
            bwd = fused.packed_bwd(ctx.coarse, entry)
            Gx = torch.empty(nb + 1, M, H, device=dev, dtype=F32)      # d loss / d X[k]
            # the activations' backward (d4), lin_out^T and its relu's backward (g where X > 0, else 0) in one pass
            d4, _, d4_max = lin_out_rows_bwd(grad_out.reshape(M, 4), out.reshape(M, 4), P["lin_out.weight"].detach(),
                                             X[nb], g=Gx[nb])
            # Gx[k] maxima (k = 0..nb): Gx[nb]'s published by fc_1[nb-1]^T's operand pass, the others by the GRAD
            # prologues that build them and avr_bn_grad_rows
            gmax = torch.zeros(2 * nb + 2, device=dev, dtype=torch.int32)
            if nb == 0:
                gmax[0:1] = _max_bits(Gx[0])
            DN = torch.empty(max(nb, 1), M, H, device=dev, dtype=F32)  # d loss / d fc_0 output (pre-BN)
            dn_max = torch.zeros(max(nb, 1), device=dev, dtype=torch.int32)
            gp2 = torch.empty(M, H, device=dev, dtype=F32)
            gp1 = torch.empty(max(nb, 1), M, H, device=dev, dtype=F32)
            part = _partial(M, H, dev)
            dgam = torch.zeros(nb, H, device=dev, dtype=F32)
            dbet = torch.zeros(nb, H, device=dev, dtype=F32)
            gs1 = [torch.empty(3, H, device=dev, dtype=F32) for _ in range(nb)]   # coef, m1, m2 of point 1
            gs2 = torch.empty(3, H, device=dev, dtype=F32)
            gammas = [bns[b].weight.detach().to(F32).contiguous() for b in range(nb)]
            for b in range(nb - 1, -1, -1):
                # fc_1[b]^T: operand = Gx[b+1] (for b < nb-1 built in the prologue from block b+1's BN backward)
                if b == nb - 1:
                    pro = dict(prologue=_lib.BN_PLAIN, src=Gx[nb], ld_src=H, operand_max=gmax[nb:])
                else:
                    c = gs1[b + 1]
                    pro = dict(prologue=_lib.BN_GRAD, src=gp1[b + 1], ld_src=H, src_pre=X[b + 1], src_res=Gx[b + 2],
                               in_mu=st1[b + 1].mu, in_invstd=st1[b + 1].invstd, in_scale=c[0], in_m1=c[1],
                               in_m2=c[2], operand_out=Gx[b + 1], operand_max=gmax[b + 1:])
                _run(dims, _layer(n_rows=M, mode=_lib.BN_BWD, in_dim=H, in_valid=H, blob=bwd, layer=3 + 2 * b,
                                  out=gp2, pre_rows=N[b], out_mu=st2[b].mu, out_invstd=st2[b].invstd,
                                  out_scale=st2[b].scale, out_shift=betas[b], partial=part, **pro), stream)
                call("avr_bn_grad_stats", ptr(part), M, H, ptr(gammas[b]), ptr(st2[b].invstd), ptr(gs2[0]),
                     ptr(gs2[1]), ptr(gs2[2]), ptr(dgam[b]), ptr(dbet[b]), stream)
                # fc_0[b]^T: operand = d loss / d fc_0 output = BN backward of gp2 (stored as DN[b])
                _run(dims, _layer(n_rows=M, mode=_lib.BN_BWD, prologue=_lib.BN_GRAD, in_dim=H, in_valid=H,
                                  src=gp2, ld_src=H, src_pre=N[b], in_mu=st2[b].mu, in_invstd=st2[b].invstd,
                                  in_scale=gs2[0], in_m1=gs2[1], in_m2=gs2[2], operand_out=DN[b],
                                  operand_max=dn_max[b:], blob=bwd, layer=2 + 2 * b, out=gp1[b], pre_rows=X[b],
                                  out_mu=st1[b].mu, out_invstd=st1[b].invstd, out_scale=st1[b].scale,
                                  out_shift=betas[b], partial=part), stream)
                c = gs1[b]
                call("avr_bn_grad_stats", ptr(part), M, H, ptr(gammas[b]), ptr(st1[b].invstd), ptr(c[0]), ptr(c[1]),
                     ptr(c[2]), ptr(dgam[b]), ptr(dbet[b]), stream)
            if nb > 0:   # Gx[0] = Gx[1] + block 0's first BN backward (no GEMM follows it)
                c = gs1[0]
                call("avr_bn_grad_rows", M, H, ptr(gp1[0]), ptr(X[0]), ptr(Gx[1]), ptr(c[0]), ptr(c[1]), ptr(c[2]),
                     ptr(st1[0].mu), ptr(st1[0].invstd), ptr(Gx[0]), ptr(gmax[0:1]), stream)
            # weight gradients: fc_0 (DN, relu(bn_0(X[b]))), fc_1 (Gx[b+1], relu(bn_0(N[b]))) -- both operands
            # rebuilt from the pre-BN rows in the kernel's staging --, lin_z (Gx[b], latent features),
            # lin_in (Gx[0], z_feature), lin_out (d4, relu(X[nb]))
            lat_feat = torch.empty(M, net.d_latent, device=dev, dtype=F32)
            if nz > 0:
                hwc = fused.latent_hwc_all(latent) if SB <= latent.shape[0] else None
                p = xyz.detach().to(F32).contiguous()
                for s in range(SB):
                    li = min(s, latent.shape[0] - 1)
                    lh = hwc[li] if hwc is not None else fused.latent_hwc(latent, li)
                    call("avr_latent_features", ctypes.byref(fused.view(s)), ptr(lh), net.d_latent, ptr(p[s]), B,
                         ptr(lat_feat[s * B:(s + 1) * B]), stream)
            lat_max = fused.latent_max_bits(latent)
            layers = []
            for b in range(nb):
                layers.append((DN[b], X[b], dn_max[b:b + 1], amax[2 * b:2 * b + 1], True,
                               (st1[b].mu, st1[b].scale, betas[b])))
                layers.append((Gx[b + 1], N[b], gmax[b + 1:b + 2], amax[2 * b + 1:2 * b + 2], True,
                               (st2[b].mu, st2[b].scale, betas[b])))
            for b in range(nz):
                layers.append((Gx[b], lat_feat, gmax[b:b + 1], lat_max, True))
            zf_max = _max_bits(zfp)
            layers.append((Gx[0], zfp, gmax[0:1], zf_max, True))
            layers.append((d4, X[nb], d4_max, a_max, True, "relu"))   # relu(X[nb]) rebuilt in the staging
            res = weight_grads(layers, M)
            grads = {"lin_out.weight": res[-1][0], "lin_out.bias": res[-1][1]}
            w_in, b_in = res[-2]
            grads["lin_in.weight"], grads["lin_in.bias"] = w_in[:, :net.d_in].contiguous(), b_in
            for b in range(nb):
                grads[f"blocks.{b}.fc_0.weight"], grads[f"blocks.{b}.fc_0.bias"] = res[2 * b]
                grads[f"blocks.{b}.fc_1.weight"], grads[f"blocks.{b}.fc_1.bias"] = res[2 * b + 1]
                grads[f"blocks.{b}.bn_0.weight"] = dgam[b]
                grads[f"blocks.{b}.bn_0.bias"] = dbet[b]
            for b in range(nz):
                grads[f"lin_z.{b}.weight"], grads[f"lin_z.{b}.bias"] = res[2 * nb + b]
        d_latent = d_xyz = None
        if want_latent or want_xyz:
            with torch.enable_grad():
                lat = latent.detach().requires_grad_(want_latent)
                x = xyz.detach().requires_grad_(want_xyz)
                feat, zft = net.mlp_inputs(x, viewdirs.detach(), latent=lat)
                outs, grads_out = [], []
                if nz > 0 and not net.stop_encoder_grad:   # a detached lookup (models.py:810-811) carries none
                    outs.append(feat)
                    grads_out.append(sum_of_products([(Gx[b], P[f"lin_z.{b}.weight"].detach()) for b in range(nz)]))
                if want_xyz:
                    outs.append(zft)
                    grads_out.append(Gx[0] @ P["lin_in.weight"].detach())
                wrt = ([lat] if want_latent else []) + ([x] if want_xyz else [])
                res_in = torch.autograd.grad(outs, wrt, grads_out, allow_unused=True)
            if want_latent:
                d_latent = res_in[0] if res_in[0] is not None else torch.zeros_like(latent)
            if want_xyz:
                d_xyz = res_in[-1] if res_in[-1] is not None else torch.zeros_like(xyz)
        return (None, None, None, d_xyz, None, d_latent) + tuple(
            grads[n] if ctx.needs_input_grad[6 + i] else None for i, n in enumerate(names))
