"""Per-scene image encoder of NewPixelNeRFNet: SpatialEncoder (models.py:178-342)
on a ResNet-18/34 backbone (the torchvision architecture the reference
instantiates with `getattr(torchvision.models, backbone)(pretrained=...,
norm_layer=...)`, models.py:224-229).

torchvision is not part of this stack, so the backbone is written out here with
torchvision's module names (conv1, bn1, relu, maxpool, layer1..layer4, each
block conv1/bn1/relu/conv2/bn2/downsample), so `encoder.model.*` state_dict keys
of a reference checkpoint load unchanged. Pretrained ImageNet weights cannot be
downloaded offline: `pretrained=True` keeps torchvision's random init (warns)
and expects the weights from a checkpoint. Convolutions run on PyTorch-ROCm
(MIOpen); the encoder runs once per scene per training step, off the per-ray
hot path.
"""
import functools
import warnings

import torch
import torch.nn.functional as F
from torch import nn


def get_norm_layer(norm_type="instance", group_norm_groups=32):
    """utils.py:136-157."""
    if norm_type == "batch":
        return functools.partial(nn.BatchNorm2d, affine=True, track_running_stats=True)
    if norm_type == "instance":
        return functools.partial(nn.InstanceNorm2d, affine=False, track_running_stats=False)
    if norm_type == "group":
        return functools.partial(nn.GroupNorm, group_norm_groups)
    if norm_type == "none":
        return None
    raise NotImplementedError(f"normalization layer [{norm_type}] is not found")


def _conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    """torchvision's ResNet basic block: 3x3 -> norm -> relu -> 3x3 -> norm, + shortcut."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, norm_layer=nn.BatchNorm2d):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


class ResNet(nn.Module):
    """torchvision.models.ResNet with BasicBlock (resnet18: 2-2-2-2, resnet34:
    3-4-6-3), same attribute names and init (kaiming fan_out for convolutions,
    norm weight 1 / bias 0)."""

    def __init__(self, layers, num_classes=1000, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self._norm_layer = norm_layer
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes, kernel_size=1, stride=stride, bias=False),
                                       norm_layer(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, downsample, norm_layer)]
        self.inplanes = planes
        layers += [BasicBlock(planes, planes, norm_layer=norm_layer) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def _resnet(layers, pretrained=False, norm_layer=None, **kwargs):
    if pretrained:
        warnings.warn("pretrained ImageNet weights are not available offline: random init; load the "
                      "encoder weights from a checkpoint")
    return ResNet(layers, norm_layer=norm_layer, **kwargs)


def resnet18(pretrained=False, norm_layer=None, **kwargs):
    return _resnet([2, 2, 2, 2], pretrained, norm_layer, **kwargs)


def resnet34(pretrained=False, norm_layer=None, **kwargs):
    return _resnet([3, 4, 6, 3], pretrained, norm_layer, **kwargs)


BACKBONES = {"resnet18": resnet18, "resnet34": resnet34}


class SpatialEncoder(nn.Module):
    """models.py:178-342: ResNet feature pyramid (conv1 .. layer{num_layers-1}),
    every level bilinearly upsampled to conv1's resolution and concatenated
    into `latent` (B, latent_size, H/2, W/2); `index` samples it at image
    points (grid_sample, align_corners=True). `set_latent` installs a
    precomputed feature map instead (inference from cached latents)."""

    def __init__(self, backbone="resnet34", pretrained=True, num_layers=4, index_interp="bilinear",
                 index_padding="border", upsample_interp="bilinear", feature_scale=1.0, use_first_pool=True,
                 norm_type="batch"):
        super().__init__()
        if norm_type != "batch":
            assert not pretrained
        if backbone not in BACKBONES:
            raise NotImplementedError(f"backbone {backbone!r}: resnet18 / resnet34 (the custom ConvEncoder is "
                                      "experimental in the reference and not provided)")
        self.use_custom_resnet = False
        self.feature_scale = feature_scale
        self.use_first_pool = use_first_pool
        self.model = BACKBONES[backbone](pretrained=pretrained, norm_layer=get_norm_layer(norm_type))
        # models.py:230-232: no classifier head
        self.model.fc = nn.Sequential()
        self.model.avgpool = nn.Sequential()
        self.latent_size = [0, 64, 128, 256, 512, 1024][num_layers]
        self.num_layers = num_layers
        self.index_interp = index_interp
        self.index_padding = index_padding
        self.upsample_interp = upsample_interp
        self.register_buffer("latent", torch.empty(1, 1, 1, 1), persistent=False)
        self.register_buffer("latent_scaling", torch.empty(2, dtype=torch.float32), persistent=False)

    def index(self, uv, cam_z=None, image_size=(), z_bounds=None):
        """models.py:245-274: uv (B, N, 2) image points -> (B, L, N)."""
        if uv.shape[0] == 1 and self.latent.shape[0] > 1:
            uv = uv.expand(self.latent.shape[0], -1, -1)
        if len(image_size) > 0:
            if len(image_size) == 1:
                image_size = (image_size, image_size)
            uv = uv * (self.latent_scaling / image_size) - 1.0
        samples = F.grid_sample(self.latent, uv.unsqueeze(2), align_corners=True, mode=self.index_interp,
                                padding_mode=self.index_padding)
        return samples[:, :, :, 0]

    def _set_scaling(self):
        # models.py:326-328: (W, H) / (W - 1, H - 1) * 2
        ls = torch.tensor([self.latent.shape[-1], self.latent.shape[-2]], dtype=torch.float32,
                          device=self.latent.device)
        self.latent_scaling = ls / (ls - 1) * 2.0

    def set_latent(self, latent):
        """Install a precomputed feature map (B, latent_size, H, W)."""
        self.latent = latent
        self._set_scaling()
        return self.latent

    def forward(self, x):
        """models.py:276-329: image (B, 3, H, W) -> latent (B, latent_size, H/2, W/2)."""
        if self.feature_scale != 1.0:
            x = F.interpolate(x, scale_factor=self.feature_scale,
                              mode="bilinear" if self.feature_scale > 1.0 else "area",
                              align_corners=True if self.feature_scale > 1.0 else None, recompute_scale_factor=True)
        x = x.to(device=self.latent.device)
        m = self.model
        x = m.relu(m.bn1(m.conv1(x)))
        latents = [x]
        if self.num_layers > 1:
            if self.use_first_pool:
                x = m.maxpool(x)
            x = m.layer1(x)
            latents.append(x)
        for k, layer in ((2, m.layer2), (3, m.layer3), (4, m.layer4)):
            if self.num_layers > k:
                x = layer(x)
                latents.append(x)
        align_corners = None if self.index_interp == "nearest " else True   # (sic, models.py:316)
        size = latents[0].shape[-2:]
        latents = [F.interpolate(t, size, mode=self.upsample_interp, align_corners=align_corners) for t in latents]
        # the reference interpolates its list in place (models.py:315-324): encoder.latents holds the upsampled maps
        self.latents = latents
        self.latent = torch.cat(latents, dim=1)
        self._set_scaling()
        return self.latent

    @classmethod
    def from_conf(cls, conf):
        """models.py:331-342."""
        return cls(conf.get_string("backbone", "resnet34"), pretrained=conf.get_bool("pretrained", True),
                   num_layers=conf.get_int("num_layers", 4),
                   index_interp=conf.get_string("index_interp", "bilinear"),
                   index_padding=conf.get_string("index_padding", "border"),
                   upsample_interp=conf.get_string("upsample_interp", "bilinear"),
                   feature_scale=conf.get_float("feature_scale", 1.0),
                   use_first_pool=conf.get_bool("use_first_pool", True))


def make_encoder(conf, **kwargs):
    """models.py:31-39 (the spatial type; the global ImageEncoder is not used by the shipped configs)."""
    enc_type = conf.get_string("type", "spatial")
    if enc_type == "spatial":
        return SpatialEncoder.from_conf(conf, **kwargs)
    raise NotImplementedError(f"encoder type {enc_type!r}: only 'spatial' (conf/default*.conf)")
