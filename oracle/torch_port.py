"""torch-CPU restatement of the reference's coarse/fine render path — the timed
CPU baseline ("kind": "port") of bench.py.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg,
never by the product. It restates, with the same torch operators the
reference calls on the CPU, VolumeRenderer.forward (renderers.py:133-277:
sample_coarse :4-24, volume_integral :69-119, sample_fine :27-54, sort
:257-258, depth_from_world utils.py:358-361) over NewPixelNeRFNet.forward
(models.py:739-863: PositionalEncoding :41-87, SpatialEncoder.index :245-274,
ResnetFC :541-592 with the per-sample lin_z of every block). It is what the
reference's CPU path costs per ray, not a faster algorithm: no lin_z
factorisation, no fusion. Its outputs are checked against the numpy oracle
(tests/test_oracle_golden.py::test_torch_port_matches_oracle).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


class TorchField:
    """NewPixelNeRFNet.forward for the default.conf family (NS = 1), torch on the CPU."""

    def __init__(self, params_coarse, params_fine, latent, poses, focal, c, image_shape, latent_scaling,
                 n_blocks=3, combine_layer=1000, num_freqs=6, freq_factor=1.5):
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32))  # noqa: E731
        self.pc = {k: T(v) for k, v in params_coarse.items()}
        self.pf = {k: T(v) for k, v in params_fine.items()}
        lat = T(latent)
        self.latent = lat.reshape((1,) + tuple(lat.shape[-3:]))                      # (1, L, H, W)
        self.poses = T(poses).reshape(1, 3, 4)
        self.focal, self.c = T(focal).reshape(1, 2), T(c).reshape(1, 2)
        self.image_shape, self.latent_scaling = T(image_shape), T(latent_scaling)
        self.n_blocks, self.combine_layer = n_blocks, combine_layer
        freqs = freq_factor * 2.0 ** torch.arange(0, num_freqs)
        self._freqs = torch.repeat_interleave(freqs, 2).view(1, -1, 1)                 # models.py:56-58
        ph = torch.zeros(2 * num_freqs)
        ph[1::2] = math.pi * 0.5
        self._phases = ph.view(1, -1, 1)
        self.d_latent = self.latent.shape[1]

    def _code(self, x):                                                                # models.py:65-87
        embed = x.unsqueeze(1).repeat(1, self._freqs.shape[1], 1)
        embed = torch.sin(torch.addcmul(self._phases, embed, self._freqs))
        return torch.cat((x, embed.view(x.shape[0], -1)), dim=-1)

    def _mlp(self, zx, p):                                                             # models.py:541-592
        z, x = zx[:, :self.d_latent], zx[:, self.d_latent:]
        x = F.linear(x, p["lin_in.weight"], p["lin_in.bias"])
        for b in range(self.n_blocks):
            if b < self.combine_layer:
                x = x + F.linear(z, p[f"lin_z.{b}.weight"], p[f"lin_z.{b}.bias"])
            net = F.linear(F.relu(x), p[f"blocks.{b}.fc_0.weight"], p[f"blocks.{b}.fc_0.bias"])
            x = x + F.linear(F.relu(net), p[f"blocks.{b}.fc_1.weight"], p[f"blocks.{b}.fc_1.bias"])
        return F.linear(F.relu(x), p["lin_out.weight"], p["lin_out.bias"])

    def __call__(self, xyz, viewdirs, coarse=True):
        SB, B, _ = xyz.shape
        xyz_rot = torch.matmul(self.poses[:, None, :3, :3], xyz.unsqueeze(-1))[..., 0]
        xyz_c = xyz_rot + self.poses[:, None, :3, 3]
        zf = self._code(xyz_rot.reshape(-1, 3))
        vd = torch.matmul(self.poses[:, None, :3, :3], viewdirs.reshape(SB, B, 3, 1)).reshape(-1, 3)
        zf = torch.cat((zf, vd), dim=1)
        uv = -xyz_c[:, :, :2] / xyz_c[:, :, 2:]
        uv = uv * self.focal.unsqueeze(1) + self.c.unsqueeze(1)
        scale = self.latent_scaling / self.image_shape                                 # models.py:245-274
        grid = (uv * scale - 1.0).unsqueeze(2)
        lat = F.grid_sample(self.latent, grid, align_corners=True, mode="bilinear", padding_mode="border")
        lat = lat[..., 0].transpose(1, 2).reshape(-1, self.d_latent)
        out = self._mlp(torch.cat((lat, zf), dim=-1), self.pc if coarse else self.pf).reshape(-1, B, 4)
        return torch.cat([torch.sigmoid(out[..., :3]), torch.relu(out[..., 3:4])], -1).reshape(SB, B, 4)


def world_rays(x_pix, K, c2w):
    """utils.py:315-336 (unproject, normalise, rotate by cam2world)."""
    hom = torch.cat([x_pix, torch.ones_like(x_pix[..., :1])], -1)
    cam = torch.einsum("bij,bkj->bki", torch.inverse(K), hom)
    cam = torch.stack([-cam[..., 0], cam[..., 1], cam[..., 2]], -1) * -1.0
    d = cam / cam.norm(dim=-1, keepdim=True)
    rd = torch.einsum("bkij,bkj->bki", c2w[..., :3, :3], d)
    return c2w[..., :3, 3], rd


def volume_integral(z, sigma, rad, white_back=True, infinity=1.8):                     # renderers.py:69-119
    dists = torch.cat([z[..., 1:] - z[..., :-1], torch.full_like(z[..., :1], 1e10)], -1)
    alpha = 1.0 - torch.exp(-sigma[..., 0] * dists)
    T = torch.cumprod(1.0 - alpha + 1e-10, -1)
    T = torch.cat([torch.ones_like(T[..., :1]), T[..., :-1]], -1)
    w = alpha * T
    rgb = torch.einsum("bri,bric->brc", w, rad)
    zz = torch.cat([z[..., 1:], torch.full_like(z[..., :1], infinity)], -1)
    depth = torch.einsum("bri,bri->br", w, zz)[..., None]
    if white_back:
        rgb = rgb + (1.0 - w.sum(-1, keepdim=True))
    return rgb, depth, w[..., None]


def render(c2w, K, x_pix, field, near, far, n_coarse, n_fine, white_back, gen, coarse_only=False):
    """VolumeRenderer.forward (renderers.py:133-277) with n_fine_depth = 0;
    draws from the torch.Generator `gen` in the reference's order."""
    SB, R, _ = x_pix.shape
    ro, rd = world_rays(x_pix, K, c2w)
    nearv, farv = torch.full((SB, R), near), torch.full((SB, R), far)
    steps = torch.arange(n_coarse, dtype=torch.float32) / n_coarse                       # renderers.py:12-14
    zc = nearv.unsqueeze(-1) + torch.einsum("bs,j->bsj", farv - nearv, steps)
    zc = zc + torch.einsum("bsi,bs->bsi", torch.rand(zc.shape, generator=gen), farv - nearv) / n_coarse
    pts = ro.unsqueeze(-2) + rd.unsqueeze(-2) * zc.unsqueeze(-1)
    vd = rd.unsqueeze(-2).expand(pts.shape)
    fc = field(pts.reshape(SB, -1, 3), vd.reshape(SB, -1, 3), coarse=True).reshape(SB, R, n_coarse, 4)
    rgb_c, _, w = volume_integral(zc, fc[..., 3:], fc[..., :3], white_back)
    if coarse_only:
        return rgb_c
    w = w[..., 0] + 1e-5                                                                 # renderers.py:36-46
    cdf = torch.cumsum(w / torch.sum(w, -1, keepdim=True), -1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    u = torch.rand(SB, R, n_fine, generator=gen)
    inds = torch.clamp_min(torch.searchsorted(cdf, u, right=True).float() - 1.0, 0.0)
    zf = nearv.unsqueeze(-1) + torch.einsum("bs,bsj->bsj", farv - nearv,
                                            (inds + torch.rand(inds.shape, generator=gen)) / n_coarse)
    zs, _ = torch.sort(torch.cat([zc, zf], -1), -1)
    pts = ro.unsqueeze(-2) + rd.unsqueeze(-2) * zs.unsqueeze(-1)
    vd = rd.unsqueeze(-2).expand(pts.shape)
    ff = field(pts.reshape(SB, -1, 3), vd.reshape(SB, -1, 3), coarse=False).reshape(SB, R, zs.shape[-1], 4)
    rgb_f, dist, _ = volume_integral(zs, ff[..., 3:], ff[..., :3], white_back)
    world = ro + rd * dist
    hom = torch.cat([world, torch.ones_like(world[..., :1])], -1)                        # utils.py:358-361
    depth = -torch.einsum("bri,bri->br", torch.inverse(c2w)[..., 2, :], hom)
    return rgb_c, rgb_f, depth
