"""The PixelNeRF radiance field the renderer drives (models.py:41-87, 407-606,
609-863 of the reference), with the same module tree and state_dict keys so
reference checkpoints load (`strict=False`: the per-scene ResNet34 encoder is
out of scope and replaced by a latent holder).

`NewPixelNeRFNet.forward(xyz, coarse, viewdirs)` keeps the reference protocol:
(SB, B, 3) points -> (SB, B, 4) = (sigmoid rgb, relu sigma). Under no_grad on
a HIP device it runs the fused fp32-MFMA kernel (avr.field); with autograd it
runs the module's PyTorch graph so train.py can back-propagate through it.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .conf import Conf
from .encoder import make_encoder


def repeat_interleave(x, repeats, dim=0):
    """utils.py:62-69: repeat each entry `repeats` times along dim 0."""
    out = x.unsqueeze(1).expand(-1, repeats, *x.shape[1:])
    return out.reshape(-1, *x.shape[1:])


def combine_interleaved(t, inner_dims=(1,), agg_type="average"):
    """utils.py:71-81: mean/max over the NS interleaved source views."""
    if len(inner_dims) == 1 and inner_dims[0] == 1:
        return t
    t = t.reshape(-1, *inner_dims, *t.shape[1:])
    if agg_type == "average":
        return torch.mean(t, dim=1)
    if agg_type == "max":
        return torch.max(t, dim=1)[0]
    raise NotImplementedError("Unsupported combine type " + agg_type)


class PositionalEncoding(nn.Module):
    """models.py:41-87: [x, sin(f_k x), sin(f_k x + pi/2), ...], f_k = freq_factor * 2^k."""

    def __init__(self, num_freqs=6, d_in=3, freq_factor=np.pi, include_input=True):
        super().__init__()
        self.num_freqs, self.d_in, self.include_input = num_freqs, d_in, include_input
        self.freq_factor = float(freq_factor)
        self.freqs = freq_factor * 2.0 ** torch.arange(0, num_freqs)
        self.d_out = num_freqs * 2 * d_in + (d_in if include_input else 0)
        self.register_buffer("_freqs", torch.repeat_interleave(self.freqs, 2).view(1, -1, 1))
        ph = torch.zeros(2 * num_freqs)
        ph[1::2] = np.pi * 0.5
        self.register_buffer("_phases", ph.view(1, -1, 1))

    def forward(self, x):
        emb = torch.addcmul(self._phases, x.unsqueeze(1).repeat(1, self.num_freqs * 2, 1), self._freqs)
        emb = torch.sin(emb).view(x.shape[0], -1)
        return torch.cat((x, emb), dim=-1) if self.include_input else emb

    @classmethod
    def from_conf(cls, conf, d_in=3):
        return cls(conf.get_int("num_freqs", 6), d_in, conf.get_float("freq_factor", np.pi),
                   conf.get_bool("include_input", True))


class ResnetBlockFC(nn.Module):
    """models.py:407-470 (fc_1 zero-initialised as in the reference)."""

    def __init__(self, size_in, size_out=None, size_h=None, bn=False, beta=0.0):
        super().__init__()
        size_out = size_in if size_out is None else size_out
        size_h = min(size_in, size_out) if size_h is None else size_h
        self.bn, self.size_in, self.size_h, self.size_out = bn, size_in, size_h, size_out
        self.bn_0 = nn.BatchNorm1d(size_in)
        self.fc_0 = nn.Linear(size_in, size_h)
        self.bn_1 = nn.BatchNorm1d(size_h)
        self.fc_1 = nn.Linear(size_h, size_out)
        nn.init.constant_(self.fc_0.bias, 0.0)
        nn.init.kaiming_normal_(self.fc_0.weight, a=0, mode="fan_in")
        nn.init.constant_(self.fc_1.bias, 0.0)
        nn.init.zeros_(self.fc_1.weight)
        self.activation = nn.Softplus(beta=beta) if beta > 0 else nn.ReLU()
        self.shortcut = None if size_in == size_out else nn.Linear(size_in, size_out, bias=False)

    def forward(self, x):
        if self.bn:
            net = self.fc_0(self.activation(self.bn_0(x.reshape(-1, self.size_in)).reshape(x.shape)))
            dx = self.fc_1(self.activation(self.bn_0(net.reshape(-1, self.size_h)).reshape(net.shape)))
        else:
            dx = self.fc_1(self.activation(self.fc_0(self.activation(x))))
        xs = x if self.shortcut is None else self.shortcut(x)
        return xs + dx


class ResnetFC(nn.Module):
    """models.py:473-606."""

    def __init__(self, d_in, d_out=4, n_blocks=5, d_latent=0, d_hidden=128, bn=False, beta=0.0,
                 combine_layer=1000, combine_type="average", use_spade=False):
        super().__init__()
        if d_in > 0:
            self.lin_in = nn.Linear(d_in, d_hidden)
            nn.init.constant_(self.lin_in.bias, 0.0)
            nn.init.kaiming_normal_(self.lin_in.weight, a=0, mode="fan_in")
        self.lin_out = nn.Linear(d_hidden, d_out)
        nn.init.constant_(self.lin_out.bias, 0.0)
        nn.init.kaiming_normal_(self.lin_out.weight, a=0, mode="fan_in")
        self.n_blocks, self.d_latent, self.d_in, self.d_out, self.d_hidden = n_blocks, d_latent, d_in, d_out, d_hidden
        self.combine_layer, self.combine_type, self.use_spade, self.beta, self.bn = (
            combine_layer, combine_type, use_spade, beta, bn)
        self.blocks = nn.ModuleList([ResnetBlockFC(d_hidden, bn=bn, beta=beta) for _ in range(n_blocks)])
        if d_latent != 0:
            n_lin_z = min(combine_layer, n_blocks)
            self.lin_z = nn.ModuleList([nn.Linear(d_latent, d_hidden) for _ in range(n_lin_z)])
            for lz in self.lin_z:
                nn.init.constant_(lz.bias, 0.0)
                nn.init.kaiming_normal_(lz.weight, a=0, mode="fan_in")
            if use_spade:
                self.scale_z = nn.ModuleList([nn.Linear(d_latent, d_hidden) for _ in range(n_lin_z)])
                for sz in self.scale_z:
                    nn.init.constant_(sz.bias, 0.0)
                    nn.init.kaiming_normal_(sz.weight, a=0, mode="fan_in")
        self.activation = nn.Softplus(beta=beta) if beta > 0 else nn.ReLU()

    def forward(self, zx, combine_inner_dims=(1,), combine_index=None, dim_size=None):
        assert zx.size(-1) == self.d_latent + self.d_in
        if self.d_latent > 0:
            z, x = zx[..., :self.d_latent], zx[..., self.d_latent:]
        else:
            z, x = None, zx
        x = self.lin_in(x) if self.d_in > 0 else torch.zeros(self.d_hidden, device=zx.device)
        for b in range(self.n_blocks):
            if b == self.combine_layer:
                x = combine_interleaved(x, combine_inner_dims, self.combine_type)
            if self.d_latent > 0 and b < self.combine_layer:
                tz = self.lin_z[b](z)
                x = self.scale_z[b](z) * x + tz if self.use_spade else x + tz
            x = self.blocks[b](x)
        return self.lin_out(self.activation(x))

    @classmethod
    def from_conf(cls, conf, d_in, **kwargs):
        return cls(d_in, n_blocks=conf.get_int("n_blocks", 5), d_hidden=conf.get_int("d_hidden", 128),
                   beta=conf.get_float("beta", 0.0), combine_layer=conf.get_int("combine_layer", 1000),
                   combine_type=conf.get_string("combine_type", "average"),
                   use_spade=conf.get_bool("use_spade", False), **kwargs)


def make_mlp(conf, d_in, d_latent=0, allow_empty=False, bn=False, **kwargs):
    """models.py:18-28 (the resnet type; 'mlp' ImplicitNet is not part of this path)."""
    mlp_type = conf.get_string("type", "mlp")
    if mlp_type == "resnet":
        return ResnetFC.from_conf(conf, d_in, d_latent=d_latent, bn=bn, **kwargs)
    if mlp_type == "empty" and allow_empty:
        return None
    raise NotImplementedError(f"Unsupported MLP type {mlp_type!r} (only 'resnet' is on the hot path)")


class NewPixelNeRFNet(nn.Module):
    """models.py:609-863. The encoder is avr.encoder.SpatialEncoder (ResNet34
    feature pyramid, torchvision module names); encode() runs it on the source
    images, encode_latent() installs a precomputed feature map instead."""

    def __init__(self, conf, stop_encoder_grad=False, bn=False):
        super().__init__()
        conf = conf if hasattr(conf, "get_bool") else Conf(conf)
        enc = conf["encoder"] if "encoder" in conf else Conf({})
        self.encoder = make_encoder(enc if hasattr(enc, "get_bool") else Conf(enc))
        self.use_encoder = conf.get_bool("use_encoder", True)
        self.use_xyz = conf.get_bool("use_xyz", False)
        assert self.use_encoder or self.use_xyz
        self.normalize_z = conf.get_bool("normalize_z", True)
        self.stop_encoder_grad = stop_encoder_grad
        self.use_code = conf.get_bool("use_code", False)
        self.use_code_viewdirs = conf.get_bool("use_code_viewdirs", True)
        self.use_viewdirs = conf.get_bool("use_viewdirs", False)
        self.use_global_encoder = conf.get_bool("use_global_encoder", False)
        if self.use_global_encoder:
            raise NotImplementedError("global image encoder is out of scope")
        d_latent = self.encoder.latent_size if self.use_encoder else 0
        d_in = 3 if self.use_xyz else 1
        if self.use_viewdirs and self.use_code_viewdirs:
            d_in += 3
        if self.use_code and d_in > 0:
            self.code = PositionalEncoding.from_conf(conf["code"], d_in=d_in)
            d_in = self.code.d_out
        if self.use_viewdirs and not self.use_code_viewdirs:
            d_in += 3
        self.latent_size = self.encoder.latent_size
        self.mlp_coarse = make_mlp(conf["mlp_coarse"], d_in, d_latent, d_out=4, bn=bn)
        self.mlp_fine = make_mlp(conf["mlp_fine"], d_in, d_latent, d_out=4, allow_empty=True, bn=bn)
        self.register_buffer("poses", torch.empty(1, 3, 4), persistent=False)
        self.register_buffer("image_shape", torch.empty(2), persistent=False)
        self.register_buffer("focal", torch.empty(1, 2), persistent=False)
        self.register_buffer("c", torch.empty(1, 2), persistent=False)
        self.d_in, self.d_out, self.d_latent = d_in, 4, d_latent
        self.num_objs, self.num_views_per_obj = 0, 1
        self.use_fused = True           # HIP field under no_grad (avr.field)
        self.field_precision = "x3"     # "x3" split-fp16 MFMA | "fp32" MFMA
        self.hip_backward = True        # autograd through the HIP field (avr.field._FieldTrain)
        self._fused = None

    def encode(self, images, poses, focal, z_bounds=None, c=None):
        """models.py:682-737: run the encoder on the source views and keep
        their world->camera poses, focal (fy negated) and principal point.
        images (NS, 3, H, W) or (SB, NS, 3, H, W); poses (NS, 4, 4) or
        (SB, NS, 4, 4) camera->world."""
        self.num_objs = images.size(0)
        if len(images.shape) == 5:
            assert len(poses.shape) == 4
            assert poses.size(1) == images.size(1)   # NS input views
            self.num_views_per_obj = images.size(1)
            images = images.reshape(-1, *images.shape[2:])
            poses = poses.reshape(-1, 4, 4)
        else:
            self.num_views_per_obj = 1
        self.encoder(images)
        self._set_view(poses, focal, c, (images.shape[-1], images.shape[-2]), images.device)

    def encode_latent(self, latent, poses, focal, c=None, image_shape=None):
        """encode() for a precomputed feature map (NS, L, H, W) (e.g. cached
        per scene): the same pose / focal / principal-point bookkeeping;
        image_shape (W, H) of the source images, by default 2x the map (the
        ResNet's stride-2 conv1)."""
        self.num_objs = latent.size(0)
        self.num_views_per_obj = 1
        self.encoder.set_latent(latent)
        if image_shape is None:
            image_shape = (latent.shape[-1] * 2, latent.shape[-2] * 2)
        self._set_view(poses, focal, c, image_shape, latent.device)

    def _set_view(self, poses, focal, c, image_shape, device):
        """models.py:705-734."""
        rot = poses[:, :3, :3].transpose(1, 2)
        trans = -torch.bmm(rot, poses[:, :3, 3:])
        self.poses = torch.cat((rot, trans), dim=-1)
        self.image_shape = torch.tensor([float(image_shape[0]), float(image_shape[1])], device=device)
        focal = torch.as_tensor(focal, dtype=torch.float32, device=device)
        if focal.dim() == 0:
            focal = focal[None, None].repeat((1, 2))
        elif focal.dim() == 1:
            focal = focal.unsqueeze(-1).repeat((1, 2))
        else:
            focal = focal.clone()
        self.focal = focal.float()
        self.focal[..., 1] *= -1.0
        if c is None:
            c = (self.image_shape * 0.5).unsqueeze(0)
        else:
            c = torch.as_tensor(c, dtype=torch.float32, device=device)
            if c.dim() == 0:
                c = c[None, None].repeat((1, 2))
            elif c.dim() == 1:
                c = c.unsqueeze(-1).repeat((1, 2))
        self.c = c

    # ------------------------------------------------------------------ forward
    def fused(self):
        from .field import FusedField
        if self._fused is None:
            self._fused = FusedField(self, self.field_precision)
        self._fused.precision = self.field_precision
        return self._fused

    def can_fuse(self, xyz):
        from .field import fused_eligible
        return (self.use_fused and xyz.is_cuda
                and not (torch.is_grad_enabled() and (self._needs_grad() or xyz.requires_grad))
                and fused_eligible(self))

    def _needs_grad(self):
        return any(p.requires_grad for p in self.parameters()) or self.encoder.latent.requires_grad

    def can_train_fused(self, xyz, viewdirs):
        """Autograd on the HIP path (avr.field._FieldTrain): parameters, the
        latent or the points need gradients (VolumeRenderer training; the
        adaptive renderer's band points); view directions must not."""
        from .field import fused_eligible, inference_only
        return (self.use_fused and self.hip_backward and xyz.is_cuda and torch.is_grad_enabled()
                and viewdirs is not None and not viewdirs.requires_grad and fused_eligible(self)
                and not any(inference_only(m) for m in (self.mlp_coarse, self.mlp_fine) if m is not None))

    def can_fuse_multiview(self, xyz):
        """NS > 1 source views, inference: the fused x3 field in two launches around the
        views' combine (FusedField.forward_points_multiview)."""
        from .field import fused_eligible
        return (self.use_fused and xyz.is_cuda and self.num_views_per_obj > 1
                and not (torch.is_grad_enabled() and (self._needs_grad() or xyz.requires_grad))
                and fused_eligible(self, multiview=True))

    def forward(self, xyz, coarse=True, viewdirs=None, far=False, return_features=False):
        if not return_features and self.can_fuse(xyz):
            return self.fused().forward_points(xyz, viewdirs, coarse)
        if not return_features and self.can_fuse_multiview(xyz):
            return self.fused().forward_points_multiview(xyz, viewdirs, coarse)
        if not return_features and self.can_train_fused(xyz, viewdirs):
            return self.fused().forward_train(xyz, viewdirs, coarse)
        if not return_features and self.can_train_bn(xyz, viewdirs):
            from .bn_train import forward_train_bn
            return forward_train_bn(self.fused(), xyz, viewdirs, coarse)
        if not return_features and self.can_train_layers(xyz, viewdirs):
            from .layer_train import forward_train_layers
            return forward_train_layers(self.fused(), xyz, viewdirs, coarse)
        return self.forward_torch(xyz, coarse, viewdirs, far, return_features)

    def can_train_layers(self, xyz, viewdirs):
        """use_spade and / or NS > 1 source views with autograd: the layer-by-layer HIP path (avr.layer_train);
        view directions must not need gradients."""
        from .layer_train import layer_train_eligible
        return (self.use_fused and self.hip_backward and xyz.is_cuda and torch.is_grad_enabled()
                and viewdirs is not None and not viewdirs.requires_grad and layer_train_eligible(self))

    def can_train_bn(self, xyz, viewdirs):
        """train.py --bn in training mode (batch statistics): the layer-by-layer HIP path (avr.bn_train), with
        or without autograd, up to AVR_MAX_SCENES scenes per call (its layer epilogues gather the lin_z rows of
        every scene); points must not need gradients through it (view directions never)."""
        from . import _lib
        from .bn_train import bn_train_eligible
        return (self.use_fused and self.hip_backward and xyz.is_cuda and viewdirs is not None
                and not viewdirs.requires_grad and xyz.shape[0] * xyz.shape[1] >= 2
                and xyz.shape[0] <= _lib.AVR_MAX_SCENES and bn_train_eligible(self))

    def mlp_inputs(self, xyz, viewdirs, latent=None):
        """(latent features (SB*B, d_latent), z_feature (SB*B, d_in)) at the
        points: the MLP input halves of models.py:753-823 (forward_torch's code;
        `latent` overrides the encoder's map, for its gradient)."""
        return self._inputs(xyz, viewdirs, latent, batched_rot=True)[:2]

    def z_features(self, xyz, viewdirs):
        """z_feature (SB*B, d_in) alone: the positional-encoded MLP input half."""
        return self._inputs(xyz, viewdirs, batched_rot=True, want_latent=False)[1]

    def _inputs(self, xyz, viewdirs, latent_map=None, batched_rot=False, want_latent=True):
        SB, B, _ = xyz.shape
        NS = self.num_views_per_obj
        xyz = repeat_interleave(xyz, NS)
        rot = self.poses[:, :3, :3]

        def rotate(v):   # R v per point: the reference's per-point (3x3)(3x1) matmul, or one bmm per scene
            if batched_rot and rot.shape[0] == v.shape[0] and v.dim() == 3:
                return torch.bmm(v, rot.transpose(1, 2))
            return torch.matmul(rot[:, None], v.unsqueeze(-1))[..., 0]

        xyz_rot = rotate(xyz)
        xyz = xyz_rot + self.poses[:, None, :3, 3]
        z_feature = latent = None
        if self.d_in > 0:
            if self.use_xyz:
                z_feature = (xyz_rot if self.normalize_z else xyz).reshape(-1, 3)
            else:
                z_feature = -(xyz_rot if self.normalize_z else xyz)[..., 2].reshape(-1, 1)
            if self.use_code and not self.use_code_viewdirs:
                z_feature = self.code(z_feature)
            if self.use_viewdirs:
                vd = repeat_interleave(viewdirs.reshape(SB, B, 3), NS)
                vd = rotate(vd).reshape(-1, 3)
                z_feature = torch.cat((z_feature, vd), dim=1)
            if self.use_code and self.use_code_viewdirs:
                z_feature = self.code(z_feature)
        if self.use_encoder and want_latent:
            uv = -xyz[:, :, :2] / xyz[:, :, 2:]
            uv = uv * repeat_interleave(self.focal.unsqueeze(1), NS if self.focal.shape[0] > 1 else 1)
            uv = uv + repeat_interleave(self.c.unsqueeze(1), NS if self.c.shape[0] > 1 else 1)
            if latent_map is None:
                latent = self.encoder.index(uv, None, self.image_shape)
            else:
                held = self.encoder.latent
                try:
                    self.encoder.latent = latent_map
                    latent = self.encoder.index(uv, None, self.image_shape)
                finally:
                    self.encoder.latent = held
            if self.stop_encoder_grad:
                latent = latent.detach()
            latent = latent.transpose(1, 2).reshape(-1, self.latent_size)
        return latent, z_feature, B

    def forward_torch(self, xyz, coarse=True, viewdirs=None, far=False, return_features=False):
        """models.py:739-863 as PyTorch ops (the autograd path)."""
        SB = xyz.shape[0]
        latent, z_feature, B = self._inputs(xyz, viewdirs)
        if self.d_in > 0:
            mlp_input = z_feature
        if self.use_encoder:
            mlp_input = latent if self.d_in == 0 else torch.cat((latent, z_feature), dim=-1)
        if return_features:
            return latent
        mlp = self.mlp_coarse if (coarse or self.mlp_fine is None) else self.mlp_fine
        out = mlp(mlp_input, combine_inner_dims=(self.num_views_per_obj, B)).reshape(-1, B, self.d_out)
        out = torch.cat([torch.sigmoid(out[..., :3]), torch.relu(out[..., 3:4])], dim=-1)
        return out.reshape(SB, B, -1)

    def load_weights(self, model_path, opt_init=False, strict=True, device=None):
        import os
        import warnings
        if os.path.exists(model_path):
            self.load_state_dict(torch.load(model_path, map_location=device, weights_only=True), strict=strict)
        elif not opt_init:
            warnings.warn(f"WARNING: {model_path} does not exist, not loaded!! Model will be re-initialized.")
        return self

    def save_weights(self, model_path, opt_init=False):
        torch.save(self.state_dict(), model_path)
        return self


def make_new_model(conf, *args, **kwargs):
    """models.py:9-16."""
    model_type = conf.get_string("type", "pixelnerf") if hasattr(conf, "get_string") else "pixelnerf"
    if model_type != "pixelnerf":
        raise NotImplementedError("Unsupported model type", model_type)
    return NewPixelNeRFNet(conf, *args, **kwargs)


class RadFieldAndRenderer(nn.Module):
    """models.py:913-960."""

    def __init__(self, rf, renderer):
        super().__init__()
        self.rf = rf
        self.renderer = renderer

    def forward(self, model_input):
        return self.renderer(model_input["cam2world"], model_input["intrinsics"], model_input["x_pix"], self.rf)

    def load_weights(self, model_path, opt_init=False, strict=True, device=None):
        import os
        import warnings
        if os.path.exists(model_path):
            self.load_state_dict(torch.load(model_path, map_location=device, weights_only=True), strict=strict)
        elif not opt_init:
            warnings.warn(f"WARNING: {model_path} does not exist, not loaded!! Model will be re-initialized.")
        return self

    def save_weights(self, model_path, opt_init=False):
        torch.save(self.state_dict(), model_path)
        return self
