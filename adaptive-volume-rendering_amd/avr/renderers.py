"""Drop-in for the reference's renderers.py hot path (VolumeRenderer and the
four sampling/compositing functions it calls), on HIP kernels.

    from avr.renderers import VolumeRenderer          # instead of `from renderers import *`
    renderer = VolumeRenderer.from_conf(conf["normal_renderer"]).to(device)
    rgb_coarse, rgb_fine, depth, depth = renderer(cam2world, intrinsics, x_pix, radiance_field)

Signatures, argument meaning, draw order of the noise and return values follow
renderers.py:4-289. Tensors must live on a ROCm/HIP device: there is no CPU
path, and every stage raises if libavr_hip.so is missing.

Two evaluation modes for the radiance field:
  * fused  — `radiance_field` is an eligible NewPixelNeRFNet and no gradient
    is needed: sigma/RGB come from the split-fp16 ("x3", fp32-equivalent)
    MFMA field kernel straight from
    (ro, rd, z), with no points / viewdirs / mlp_input tensors materialised;
  * module — anything else (any nn.Module honouring rf(xyz, viewdirs=, coarse=)),
    or training: the module is called on the sample points, and compositing
    runs on the HIP kernel with its HIP backward.
"""
import ctypes
from typing import Tuple

import torch
from torch import nn

from . import _lib, ops
from .field import param_generation


def _noise(shape, like, kind):
    if kind == "rand":
        return torch.rand(shape, dtype=torch.float32, device=like.device)
    return torch.randn(shape, dtype=torch.float32, device=like.device)


# ---------------------------------------------------------------- functions
def sample_coarse(near_depth, far_depth, num_samples: int, device: torch.device, infinity=-1, noise=None):
    """renderers.py:4-24. near/far (SB, R) -> z (SB, R, num_samples).
    Draws rand_like(z) like the reference unless `noise` is given."""
    SB, R = near_depth.shape
    if noise is None:
        noise = _noise((SB, R, num_samples), near_depth, "rand")
    if torch.is_grad_enabled() and (near_depth.requires_grad or far_depth.requires_grad):
        # differentiable in near/far (AdaptiveVolumeRenderer's band): the same fp32 ops as renderers.py:10-14
        span = far_depth - near_depth
        steps = torch.arange(num_samples, dtype=torch.float32, device=near_depth.device) / num_samples
        z = (near_depth[..., None] + span[..., None] * steps) + (noise * span[..., None]) / num_samples
    else:
        z = ops.sample_coarse_rays(near_depth.expand(SB, R), far_depth.expand(SB, R), num_samples,
                                   noise=noise).reshape(SB, R, num_samples)
    if infinity != -1:
        z = torch.cat([z[..., 1:], torch.full_like(z[..., :1], float(infinity))], -1)
    return z


def sample_fine(near_depth, far_depth, num_samples: int, weights, device: torch.device, u=None, u2=None,
                return_idx=False):
    """renderers.py:27-54. weights (SB, R, Nc, 1) -> z (SB, R, num_samples),
    unsorted, with the reference's rand / rand_like draws (or the given u, u2)."""
    SB, R, Nc, _ = weights.shape
    if (u is None) != (u2 is None):
        raise ValueError("sample_fine: u and u2 must be given together")
    if u is None:
        u = _noise((SB, R, num_samples), weights, "rand")
        u2 = _noise((SB, R, num_samples), weights, "rand")
    near_t = torch.as_tensor(near_depth, dtype=torch.float32, device=weights.device)
    far_t = torch.as_tensor(far_depth, dtype=torch.float32, device=weights.device)
    uniform = bool((near_t == near_t.reshape(-1)[0]).all()) and bool((far_t == far_t.reshape(-1)[0]).all())
    near, far = float(near_t.reshape(-1)[0]), float(far_t.reshape(-1)[0])
    # the z_coarse input only feeds the merge; any (R, Nc) tensor works here
    zc = torch.zeros(SB * R, Nc, device=weights.device, dtype=torch.float32)
    _, idx, zf = ops.sample_fine(weights.detach().reshape(SB * R, Nc), zc, near, far, num_samples, 0, 0.0, u=u,
                                 u2=u2, want_idx=True, want_fine=True)
    idx = idx.reshape(SB, R, num_samples)
    if uniform:
        zf = zf.reshape(SB, R, num_samples)
    else:
        # per-ray bounds: the kernel's bins with renderers.py:45-46's fp32 ops on (SB, R) near/far
        z_steps = (idx.float() + u2.reshape(SB, R, num_samples)) / Nc
        near_t, far_t = near_t.expand(SB, R), far_t.expand(SB, R)
        zf = near_t.unsqueeze(-1) + (far_t - near_t).unsqueeze(-1) * z_steps
    return (zf, idx) if return_idx else zf


def sample_depth(depth, num_samples: int, depth_std, noise=None):
    """renderers.py:56-66 — returns randn * depth_std (the reference ignores `depth`: quirk Q6)."""
    SB, R, _ = depth.shape
    if noise is None:
        noise = _noise((SB, R, num_samples), depth, "randn")
    return noise * depth_std


def volume_integral(z_vals, sigmas, radiances, white_back=True, infinity=1.8) -> Tuple[torch.Tensor, ...]:
    """renderers.py:69-119. z (SB,R,N), sigmas (SB,R,N,1), radiances (SB,R,N,3)
    -> rgb (SB,R,3), depth_map (SB,R,1), weights (SB,R,N,1). Differentiable
    w.r.t. sigmas and radiances (HIP backward kernel)."""
    SB, R, N = z_vals.shape
    field = torch.cat([radiances, sigmas], -1).reshape(SB * R, N, 4)
    rgb, dist, w = ops.composite(z_vals.reshape(SB * R, N), field, white_back, infinity)
    return rgb.reshape(SB, R, 3), dist.reshape(SB, R, 1), w.reshape(SB, R, N, 1)


def volume_integral_packed(z_vals, field, white_back=True, infinity=1.8):
    """volume_integral(z_vals, field[..., 3:], field[..., :3]) for a field output (SB,R,N,4) in its own [r, g, b,
    sigma] layout -- the layout volume_integral's cat builds -- so the same composite on the same values, without
    the cat in the forward and the two slices' zero-padded adjoints and their sum in the backward."""
    SB, R, N = z_vals.shape
    rgb, dist, w = ops.composite(z_vals.reshape(SB * R, N), field.reshape(SB * R, N, 4), white_back, infinity)
    return rgb.reshape(SB, R, 3), dist.reshape(SB, R, 1), w.reshape(SB, R, N, 1)


# ---------------------------------------------------------------- renderer
class VolumeRenderer(nn.Module):
    """renderers.py:121-289: coarse stratified pass -> inverse-CDF fine pass
    (+ n_fine_depth 'depth' samples) -> sort -> fine pass -> depth."""

    def __init__(self, near, far, n_coarse, n_fine, n_fine_depth, depth_std, white_back=True):
        super().__init__()
        self.near = torch.tensor([near], dtype=torch.float32)
        self.far = torch.tensor([far], dtype=torch.float32)
        self.n_coarse, self.n_fine, self.n_fine_depth = int(n_coarse), int(n_fine), int(n_fine_depth)
        self.depth_std = float(depth_std)
        self.white_back = bool(white_back)
        self.seed = None          # None: torch RNG draws (reference order); int: in-kernel Philox
        self._offset = 0
        self.last_path = None     # "fused" | "module" (for tests / introspection)
        # Early ray termination of the fine pass (BASELINE config 4, not in the
        # reference): None = evaluate every sample (reference behaviour); a
        # float T_stop stops a ray once its transmittance drops below it
        # (inference only; rgb changes by <= T_stop).
        self.t_stop = None
        self.last_fine_samples = 0

    @classmethod
    def from_conf(cls, conf, white_back=True):
        return cls(near=conf.get_float("near", 0.8), far=conf.get_float("far", 1.8),
                   n_coarse=conf.get_int("n_coarse", 32), n_fine=conf.get_int("n_fine", 16),
                   n_fine_depth=conf.get_int("n_fine_depth", 8), depth_std=conf.get_float("depth_std", 0.01),
                   white_back=conf.get_float("white_back", white_back))

    def _fine_early_termination(self, ro, rd, z_sorted, radiance_field, fuse, SB, R):
        """Fine pass with early ray termination at transmittance < self.t_stop
        (BASELINE config 4, inference only; ops.march_fine)."""
        Nt = z_sorted.shape[-1]
        zs = z_sorted.reshape(SB, R, Nt)
        rgbs, dists, self.last_fine_samples = [], [], 0
        for b in range(SB):
            def fn(ro_c, rd_c, z_c, b=b):
                if fuse:
                    return radiance_field.fused().forward_rays(ro_c, rd_c, z_c, False, sb=b)
                pts, vd = ops.points(ro_c, rd_c, z_c)
                xyz = torch.zeros(SB, pts.shape[0], 3, device=pts.device, dtype=pts.dtype)
                vds = torch.zeros_like(xyz)
                xyz[b], vds[b] = pts, vd
                return radiance_field(xyz, viewdirs=vds, coarse=False)[b]
            rgb_b, dist_b, n = ops.march_fine(ro[b], rd[b], zs[b], fn, self.t_stop, self.white_back)
            rgbs.append(rgb_b)
            dists.append(dist_b)
            self.last_fine_samples += n
        return torch.cat(rgbs, 0), torch.cat(dists, 0)

    def _draws(self, SB, R, dev, noise):
        """The reference's RNG draws in its order (renderers.py:14, :41, :45, :63)."""
        if noise is not None:
            return noise
        if self.seed is not None:
            return None
        nf = self.n_fine - self.n_fine_depth
        return {
            "coarse": torch.rand(SB, R, self.n_coarse, device=dev),
            "u": torch.rand(SB, R, nf, device=dev),
            "u2": torch.rand(SB, R, nf, device=dev),
            "depth": torch.randn(SB, R, self.n_fine_depth, device=dev),
        }

    def forward(self, cam2world, intrinsics, x_pix, radiance_field: nn.Module, noise=None, ray_ids=None,
                n_rays_total=None):
        """ray_ids (R,) / n_rays_total: these R rays are rays ray_ids of an
        n_rays_total-ray frame (a rank's share, avr.parallel.render_sharded):
        the in-kernel Philox draws are keyed by the frame-wide ray index, so
        a sharded render equals the single-GPU render of the same seed."""
        SB, R, _ = x_pix.shape
        dev = x_pix.device
        near, far = float(self.near[0]), float(self.far[0])
        nf = self.n_fine - self.n_fine_depth
        Nc, Nt = self.n_coarse, self.n_coarse + self.n_fine
        draws = self._draws(SB, R, dev, noise)
        seed, off = (self.seed or 0), self._offset
        ids = None
        if ray_ids is not None:
            Rt = int(n_rays_total)
            ids = (torch.arange(SB, device=dev, dtype=torch.int64)[:, None] * Rt
                   + ray_ids.to(dev, torch.int64).reshape(1, R)).reshape(-1)
        if self.seed is not None:
            self._offset += SB * (R if ray_ids is None else int(n_rays_total))

        # without autograd or termination, depth comes from the fine composite's epilogue (fp64 depth rows)
        fast_depth = not torch.is_grad_enabled() and self.t_stop is None
        ro, rd, zc, depth_row, c2w_info = ops.rays_sample_coarse(
            x_pix, intrinsics, cam2world, near, far, Nc, noise=None if draws is None else draws["coarse"], seed=seed,
            offset=off, ray_ids=ids, want_depth_row=fast_depth)

        fuse = hasattr(radiance_field, "can_fuse") and radiance_field.can_fuse(x_pix)
        self.last_path = "fused" if fuse else "module"

        def field(z, coarse):
            n = z.shape[-1]
            if fuse:
                fusedf = radiance_field.fused()
                if SB == 1:
                    return fusedf.forward_rays(ro[0], rd[0], z, coarse).reshape(SB * R, n, 4)
                return fusedf.forward_rays_batch(ro, rd, z, coarse).reshape(SB * R, n, 4)   # one launch per 16 scenes
            pts, vd = ops.points(ro.reshape(SB * R, 3), rd.reshape(SB * R, 3), z)
            out = radiance_field(pts.reshape(SB, -1, 3), viewdirs=vd.reshape(SB, -1, 3), coarse=coarse)
            return out.reshape(SB * R, n, 4)

        fc = field(zc, True)
        rgb_c, dist_c, w_c = ops.composite(zc, fc, self.white_back)
        z_sorted, _, _ = ops.sample_fine(
            w_c.detach(), zc, near, far, nf, self.n_fine_depth, self.depth_std,
            u=None if draws is None else draws["u"], u2=None if draws is None else draws["u2"],
            noise_depth=None if draws is None else draws["depth"], seed=seed, offset=off, ray_ids=ids)
        if self.t_stop is not None and not torch.is_grad_enabled():
            rgb_f, dist_f = self._fine_early_termination(ro, rd, z_sorted, radiance_field, fuse, SB, R)
        else:
            ff = field(z_sorted, False)
            self.last_fine_samples = z_sorted.numel()
            if fast_depth:
                # the fine weights are not returned (renderers.py:264-277): no store without autograd
                rgb_f, dist_f, _, depth = ops.composite_depth(z_sorted, ff, ro, rd, depth_row, self.white_back)
                depth = depth.reshape(SB, R)
                return rgb_c.reshape(SB, R, 3), rgb_f.reshape(SB, R, 3), depth, depth
            rgb_f, dist_f, _ = ops.composite(z_sorted, ff, self.white_back, want_weights=False)
        depth = ops.depth_from_world(ro, rd, dist_f.reshape(SB, R), c2w_info)
        assert z_sorted.shape[-1] == Nt
        return rgb_c.reshape(SB, R, 3), rgb_f.reshape(SB, R, 3), depth, depth


# ---------------------------------------------------------------- adaptive renderers
def init_recurrent_weights(self):
    """utils.py:109-118 (only matches nn.GRU/LSTM/RNN: a no-op on the LSTMCell
    the renderers use, which keeps torch's default init, as in the reference)."""
    for m in self.modules():
        if type(m) in [nn.GRU, nn.LSTM, nn.RNN]:
            for name, param in m.named_parameters():
                if "weight_ih" in name:
                    nn.init.kaiming_normal_(param.data)
                elif "weight_hh" in name:
                    nn.init.orthogonal_(param.data)
                elif "bias" in name:
                    param.data.fill_(0)


def lstm_forget_gate_init(lstm_layer):
    """utils.py:121-126: forget-gate biases (second quarter) = 1."""
    for name, parameter in lstm_layer.named_parameters():
        if "bias" not in name:
            continue
        n = parameter.size(0)
        parameter.data[n // 4:n // 2].fill_(1.0)


class _LSTMMarch(nn.Module):
    """The march shared by Raymarcher and AdaptiveVolumeRenderer
    (renderers.py:320-343 and :413-432): LSTMCell(num_feature_channels -> 16)
    on the field's latent features, Linear(16 -> 1) signed distance, x += rd * sd.

    fused: a fusable NewPixelNeRFNet and no gradient -> one HIP kernel for all
    steps (avr_raymarch) on a per-texel projection of the latent through the
    LSTM input weights; module: the reference's loop on phi(return_features=True)."""

    def __init__(self, num_feature_channels, raymarch_steps):
        super().__init__()
        self.n_feature_channels = num_feature_channels
        self.steps = raymarch_steps
        hidden_size = 16
        self.lstm = nn.LSTMCell(input_size=self.n_feature_channels, hidden_size=hidden_size)
        self.lstm.apply(init_recurrent_weights)
        lstm_forget_gate_init(self.lstm)
        self.out_layer = nn.Linear(hidden_size, 1)
        self.counter = 0
        self._gate_cache = None
        self.last_path = None
        self._graph_init = None   # start distances read by a captured training step (stage_host_draws)

    def _initial_distance(self, SB, num_rays, device, noise):
        if noise is not None and "initial_distance" in noise:
            return noise["initial_distance"].reshape(SB, num_rays, 1).to(device)
        if torch.device(device).type == "cuda" and torch.cuda.is_current_stream_capturing():
            # inside a HIP-graph capture (avr.graphs.GraphedTrainStep): a static device buffer that
            # stage_host_draws() refills before every replay with the same CPU draw an eager step makes
            buf = self._graph_init
            if buf is None or buf.shape != (SB, num_rays, 1) or buf.device != torch.device(device):
                buf = self._graph_init = torch.empty((SB, num_rays, 1), device=device)
            return buf
        # renderers.py:322 / :402: drawn on the CPU generator, then moved -- through pinned memory, asynchronously:
        # a pageable host-to-device copy waits for the stream to drain, a bubble in every training step
        d = torch.zeros((SB, num_rays, 1)).normal_(mean=0.8, std=5e-2)
        if torch.device(device).type != "cuda":
            return d.to(device)
        return d.pin_memory().to(device, non_blocking=True)

    def stage_host_draws(self):
        """Before a replay of a captured training step (avr.graphs.GraphedTrainStep): the start distances an eager
        step draws on the CPU generator (renderers.py:322 / :402, same call, same values), copied into the buffer
        the captured march reads, on the current stream. Two pinned slots alternate; a slot is refilled only after
        the copy that last read it has run."""
        buf = self._graph_init
        if buf is None:
            return
        ring = getattr(self, "_graph_ring", None)
        if ring is None or ring[0][0].shape != buf.shape:
            ring = self._graph_ring = [[torch.empty(buf.shape).pin_memory(), None] for _ in range(2)]
            self._graph_slot = 0
        slot = ring[self._graph_slot]
        self._graph_slot ^= 1
        if slot[1] is not None:
            slot[1].synchronize()
        slot[0].normal_(mean=0.8, std=5e-2)
        buf.copy_(slot[0], non_blocking=True)
        slot[1] = torch.cuda.Event()
        slot[1].record(torch.cuda.current_stream(buf.device))

    def _side_stream(self, phi, world):
        """A second stream of world's device for the marched point's field pass (AdaptiveVolumeRenderer training on
        the HIP path; None otherwise: CPU, inference, the module path, or AVR_ADAPTIVE_SIDE_STREAM=0)."""
        import os
        if not (world.is_cuda and torch.is_grad_enabled() and getattr(phi, "use_fused", False)
                and getattr(phi, "hip_backward", False)) or os.environ.get("AVR_ADAPTIVE_SIDE_STREAM") == "0":
            return None
        if torch.cuda.is_current_stream_capturing() and os.environ.get("AVR_ADAPTIVE_SIDE_STREAM_IN_GRAPH") == "0":
            return None
        key = world.device
        if getattr(self, "_side", None) is None or self._side[0] != key:
            self._side = (key, torch.cuda.Stream(device=key))
        return self._side[1]

    def _gate_table(self, phi):
        lat = phi.encoder.latent
        w = self.lstm.weight_ih
        key = (param_generation(), lat.data_ptr(), lat._version, tuple(lat.shape), w.data_ptr(), w._version)
        if self._gate_cache is not None and self._gate_cache[0] == key:
            return self._gate_cache[1]
        C = lat.shape[1]
        # (H*W, C) @ (C, 64): the LSTM input projection of every latent texel (a plain library GEMM)
        table = torch.matmul(lat[0].detach().reshape(C, -1).t().float(), w.detach().t().float()).contiguous()
        self._gate_cache = (key, table, lat, w)
        return table

    def can_fuse(self, phi, ros):
        return (ros.shape[0] == 1 and not torch.is_grad_enabled() and hasattr(phi, "can_fuse")
                and phi.can_fuse(ros) and phi.encoder.latent.shape[1] == self.n_feature_channels)

    def can_train_fused(self, phi, ros, rds, init_dist):
        """Autograd through the march on HIP (avr_raymarch_train / _bwd): the net's latent lookup is the fused
        field's (bilinear / border, one source view per scene), the LSTM has its biases, and only the LSTM /
        out_layer parameters and the latent may need gradients (cameras and start distances do not)."""
        from .bn_train import bn_train_eligible
        from .field import fused_eligible
        if not (torch.is_grad_enabled() and ros.is_cuda and getattr(phi, "use_fused", False)
                and getattr(phi, "hip_backward", False) and hasattr(phi, "fused")):
            return False
        if ros.requires_grad or rds.requires_grad or init_dist.requires_grad:
            return False
        lat = phi.encoder.latent
        SB = ros.shape[0]
        if not (1 <= SB <= _lib.AVR_MAX_SCENES and lat.shape[1] == self.n_feature_channels
                and lat.shape[0] in (1, SB) and self.lstm.bias and self.lstm.hidden_size == 16):
            return False
        return fused_eligible(phi) or bn_train_eligible(phi)

    def march(self, ros, rds, init_dist, phi):
        """-> final world coordinates (SB, R, 3)."""
        SB, num_rays, _ = ros.shape
        if self.can_train_fused(phi, ros, rds, init_dist):
            self.last_path = "hip_train"
            lstm, out = self.lstm, self.out_layer
            return _MarchTrain.apply(self.steps, phi, ros, rds, init_dist, phi.encoder.latent, lstm.weight_ih,
                                     lstm.weight_hh, lstm.bias_ih, lstm.bias_hh, out.weight, out.bias)
        if self.can_fuse(phi, ros):
            self.last_path = "fused"
            world, _ = ops.raymarch(phi.fused().view(0), self._gate_table(phi), self.lstm, self.out_layer,
                                    ros[0], rds[0], init_dist[0, :, 0], self.steps)
            return world.reshape(SB, num_rays, 3)
        self.last_path = "module"
        world_coords = [ros + rds * init_dist]
        states = [None]
        for _ in range(self.steps):
            v = phi(world_coords[-1].reshape(SB, -1, 3), viewdirs=rds.reshape(SB, -1, 3), return_features=True)
            state = self.lstm(v.reshape(-1, self.n_feature_channels), states[-1])
            if state[0].requires_grad:
                state[0].register_hook(lambda x: x.clamp(min=-10, max=10))
            signed_distance = self.out_layer(state[0]).view(SB, num_rays, 1)
            world_coords.append(world_coords[-1] + rds * signed_distance)
            states.append(state)
        return world_coords[-1]


class _Band(torch.autograd.Function):
    """AdaptiveVolumeRenderer's band in training on HIP (renderers.py:490-508): from the marched points, z =
    sample_coarse(d - eps, d + eps) per ray (d = (world - ro)_x / rd_x, quirk kept) sorted, and the band points ro +
    rd z, in one launch (avr_band_fwd, bit-identical to the torch operations it replaces); backward avr_band_bwd
    (dz / dd = 1 per sample: d loss / d world_x = sum (gz + gpts . rd) / rd_x). ros / rds must not need gradients."""

    @staticmethod
    def forward(ctx, world, ros, rds, noise, eps, n):
        SB, R, _ = world.shape
        with torch.no_grad():
            w, ro, rd = (t.detach().float().reshape(SB * R, 3).contiguous() for t in (world, ros, rds))
            u = noise.detach().float().reshape(SB * R, n).contiguous()
            z = torch.empty(SB, R, n, device=w.device, dtype=torch.float32)
            pts = torch.empty(SB * R * n, 3, device=w.device, dtype=torch.float32)
            _lib.call("avr_band_fwd", SB * R, n, _lib.ptr(w), _lib.ptr(ro), _lib.ptr(rd), _lib.ptr(u), float(eps),
                      _lib.ptr(z), _lib.ptr(pts), _lib.stream_of(w))
        ctx.n, ctx.shape, ctx.rd = n, (SB, R), rd
        return z, pts

    @staticmethod
    def backward(ctx, grad_z, grad_pts):
        SB, R = ctx.shape
        rd, ctx.rd = ctx.rd, None
        gz = None if grad_z is None else grad_z.float().contiguous()
        gp = None if grad_pts is None else grad_pts.float().contiguous()
        gw = torch.empty(SB, R, 3, device=rd.device, dtype=torch.float32)
        _lib.call("avr_band_bwd", SB * R, ctx.n, _lib.ptr(rd), _lib.ptr(gz), _lib.ptr(gp), _lib.ptr(gw),
                  _lib.stream_of(rd))
        return gw, None, None, None, None, None


def _band_on_hip(phi, world, ros, rds, n):
    """The training band on HIP: with the net's HIP backward on (its torch reference keeps the torch ops)."""
    return (getattr(phi, "hip_backward", False) and torch.is_grad_enabled() and world.requires_grad and world.is_cuda
            and world.dtype == torch.float32 and not ros.requires_grad and not rds.requires_grad and 1 <= n <= 64)


class _MarchTrain(torch.autograd.Function):
    """Autograd of the LSTM march (renderers.py:413-432 / :320-343) on HIP: forward avr_raymarch_train on the
    per-texel gate tables (latent^T W_ih^T, one library GEMM per scene), backward avr_raymarch_bwd (reverse
    steps per ray: out_layer, the clamp hook, LSTMCell, the lookup's table and position gradients), then W_ih's
    and the latent's gradients from the table gradient (two more GEMMs)."""

    @staticmethod
    def forward(ctx, steps, phi, ros, rds, init_dist, latent, w_ih, w_hh, b_ih, b_hh, w_out, b_out):
        SB, R, _ = ros.shape
        dev = ros.device
        fused = phi.fused()
        with torch.no_grad():
            lat = latent.detach().float()
            L, C, H, W = lat.shape
            lat_t = lat.reshape(L, C, H * W)
            tables = torch.matmul(lat_t.transpose(1, 2), w_ih.detach().float().t())        # (L, H*W, 64)
            if L != SB:
                tables = tables.expand(SB, -1, -1)
            tables = tables.contiguous()
            n = SB * R
            world = torch.empty(n, 3, device=dev, dtype=torch.float32)
            trace = torch.empty(steps + 1, n, 3, device=dev, dtype=torch.float32)
            state = torch.empty(max(steps, 1), n, 96, device=dev, dtype=torch.float32)
            views = fused.views(range(SB))
            P = [t.detach().float().contiguous() for t in (w_hh, b_ih, b_hh, w_out, b_out)]
            ro = ros.detach().float().reshape(n, 3).contiguous()
            rd = rds.detach().float().reshape(n, 3).contiguous()
            d0 = init_dist.detach().float().reshape(n).contiguous()
            _lib.call("avr_raymarch_train", views, SB, _lib.ptr(tables), *[_lib.ptr(t) for t in P], _lib.ptr(ro),
                      _lib.ptr(rd), _lib.ptr(d0), R, steps, _lib.ptr(world), _lib.ptr(trace), _lib.ptr(state),
                      _lib.stream_of(world))
        ctx.steps, ctx.phi, ctx.views, ctx.L = steps, phi, views, L
        ctx.keep = (tables, trace, state, rd, P, lat_t)
        ctx.save_for_backward(latent, w_ih)
        return world.reshape(SB, R, 3)

    @staticmethod
    def backward(ctx, grad_world):
        latent, w_ih = ctx.saved_tensors
        tables, trace, state, rd, P, lat_t = ctx.keep
        ctx.keep = None
        SB = tables.shape[0]
        n = rd.shape[0]
        R = n // SB
        with torch.no_grad():
            # bit-deterministic backward (ABI 15): the table gradient as int64 fixed-point sums, the parameter sums
            # in a fixed order; no floating-point atomics
            d_tab = torch.empty(tables.shape, device=rd.device, dtype=torch.float32)
            d_grads = torch.empty(64 * 16 + 64 + 16 + 1, device=rd.device, dtype=torch.float32)
            nb = ctypes.c_int64(0)
            _lib.check(_lib.load().avr_raymarch_bwd_scratch_bytes(n, ctx.steps, tables.numel(), ctypes.byref(nb)),
                       "avr_raymarch_bwd_scratch_bytes")
            scratch = torch.empty(max(nb.value, 1), device=rd.device, dtype=torch.uint8)
            gw = grad_world.float().reshape(n, 3).contiguous()
            stop = bool(getattr(ctx.phi, "stop_encoder_grad", False))   # detached lookup: no position gradient
            _lib.call("avr_raymarch_bwd", ctx.views, SB, _lib.ptr(tables), _lib.ptr(P[0]), _lib.ptr(P[3]),
                      _lib.ptr(rd), _lib.ptr(trace), _lib.ptr(state), _lib.ptr(gw), R, ctx.steps, 0 if stop else 1,
                      _lib.ptr(d_tab), _lib.ptr(d_grads), _lib.ptr(scratch), scratch.numel(), _lib.stream_of(gw))
            d_whh = d_grads[:1024].reshape(64, 16)
            d_b = d_grads[1024:1088]
            d_wout = d_grads[1088:1104].reshape(1, 16)
            d_bout = d_grads[1104:1105]
            # per-scene products summed after (the einsum's single K = SB * H*W product ran on a handful of
            # workgroups: 183 vs 41 us, scripts/march_gemm_bench.py)
            if ctx.L == SB:
                d_wih = torch.bmm(d_tab.transpose(1, 2), lat_t.transpose(1, 2)).sum(0)          # (64, C)
            else:
                d_wih = torch.mm(d_tab.sum(0).t(), lat_t[0].t())
            d_lat = None
            if ctx.needs_input_grad[5] and not getattr(ctx.phi, "stop_encoder_grad", False):
                # W_ih^T d_tab^T: written in the latent's own (C, H*W) layout, no transpose pass (71 vs 24 us)
                dl = torch.matmul(w_ih.detach().float().t(), d_tab.transpose(1, 2))             # (SB, C, H*W)
                if ctx.L != SB:
                    dl = dl.sum(0, keepdim=True)
                d_lat = dl.reshape(latent.shape).to(latent.dtype)
        return (None, None, None, None, None, d_lat, d_wih.to(w_ih.dtype), d_whh, d_b.clone(), d_b.clone(), d_wout,
                d_bout)


class Raymarcher(_LSTMMarch):
    """renderers.py:290-358: LSTM march, then the coarse field at the final
    point -> (rgb, None, depth, depth)."""

    def __init__(self, num_feature_channels, raymarch_steps):
        super().__init__(num_feature_channels, raymarch_steps)

    def forward(self, cam2world, intrinsics, xy_pix, phi, noise=None):
        SB, num_rays, _ = xy_pix.shape
        ros, rds, c2w_info = ops.world_rays(xy_pix, intrinsics, cam2world)
        init = self._initial_distance(SB, num_rays, xy_pix.device, noise)
        world = self.march(ros, rds, init, phi)
        self.counter += 1
        output = phi(world.reshape(SB, -1, 3), viewdirs=rds.reshape(SB, -1, 3), coarse=True, return_features=False)
        rgb = output[..., :3].reshape(SB, num_rays, 3)
        final_depth = ops.depth_of_points(world, c2w_info).reshape(SB, num_rays, -1)
        return rgb, None, final_depth, final_depth

    @classmethod
    def from_conf(cls, conf, raymarch_steps):
        return cls(num_feature_channels=conf.get_int("num_feature_channels", 512), raymarch_steps=raymarch_steps)


class AdaptiveVolumeRenderer(_LSTMMarch):
    """renderers.py:360-557: LSTM march to a surface estimate, the coarse field
    at it, then n_coarse stratified samples in [d - epsilon, d + epsilon]
    (d = (x - ro)_x / rd_x, quirk kept), the fine field on them, volume
    integral and depth -> (rgb_coarse, rgb, depth_coarse, depth_map)."""

    def __init__(self, num_feature_channels, raymarch_steps, epsilon, n_coarse, white_back):
        super().__init__(num_feature_channels, raymarch_steps)
        self.epsilon = epsilon
        self.n_coarse = n_coarse
        self.white_back = white_back

    def forward(self, cam2world, intrinsics, xy_pix, phi, debug=False, noise=None):
        SB, num_rays, _ = xy_pix.shape
        dev = xy_pix.device
        ros, rds, c2w_info = ops.world_rays(xy_pix, intrinsics, cam2world)
        init = self._initial_distance(SB, num_rays, dev, noise)
        world = self.march(ros, rds, init, phi)
        # coarse image at the marched point. In training on the HIP path it runs on a side stream, beside the band
        # pass: its field launches cover 64 samples per workgroup, so SB x R points fill a tenth of the chip. It is
        # issued after the band pass, so autograd (which runs each backward on its forward's stream, later nodes
        # first) starts its backward first, on the side stream, and the band's backward fills the rest of the chip.
        # The kernels and their results are the same (no random draws in it); only their order on the device changes.
        def coarse_pass():
            out = phi(world.reshape(SB, -1, 3), viewdirs=rds.reshape(SB, -1, 3), coarse=True, return_features=False)
            return out, ops.depth_of_points(world, c2w_info).reshape(SB, num_rays, -1)

        side = self._side_stream(phi, world)
        if side is None:
            output_coarse, depth_coarse = coarse_pass()
        else:   # the march's outputs are ready at this point of the caller's stream
            main = torch.cuda.current_stream(dev)
            marched = torch.cuda.Event()
            marched.record(main)
        # band around the marched distance (renderers.py:490-496); the sort rarely changes stratified z (only
        # rounding can swap neighbours)
        u = None if noise is None else noise.get("band")
        band = None
        if _band_on_hip(phi, world, ros, rds, self.n_coarse):   # training: sampling, sort and band points in one launch
            if u is None:
                u = _noise((SB, num_rays, self.n_coarse), world, "rand")   # sample_coarse's draw
            z_vals_sorted, band = _Band.apply(world, ros, rds, u, self.epsilon, self.n_coarse)
        else:
            final_distance = (world[..., 0] - ros[..., 0]) / rds[..., 0]
            z_vals = sample_coarse(final_distance - self.epsilon, final_distance + self.epsilon, self.n_coarse, dev,
                                   noise=u)
            z_vals_sorted, _ = torch.sort(z_vals, dim=-1)
        fuse = (SB == 1 and not torch.is_grad_enabled() and hasattr(phi, "can_fuse") and phi.can_fuse(xy_pix))
        if band is not None:
            vd = rds.reshape(SB * num_rays, 1, 3).expand(SB * num_rays, self.n_coarse, 3)
            field = phi(band.reshape(SB, -1, 3), coarse=False, viewdirs=vd.reshape(SB, -1, 3),
                        return_features=False).reshape(SB, num_rays, self.n_coarse, 4)
        elif fuse:
            field = phi.fused().forward_rays(ros[0], rds[0], z_vals_sorted[0], False).reshape(SB, num_rays,
                                                                                               self.n_coarse, 4)
        else:
            pts, vd = ops.points(ros.reshape(-1, 3), rds.reshape(-1, 3), z_vals_sorted.reshape(-1, self.n_coarse))
            if z_vals_sorted.requires_grad:   # gradient to the band through the sample points
                pts = ros.unsqueeze(-2) + rds.unsqueeze(-2) * z_vals_sorted.unsqueeze(-1)
            field = phi(pts.reshape(SB, -1, 3), coarse=False, viewdirs=vd.reshape(SB, -1, 3),
                        return_features=False).reshape(SB, num_rays, self.n_coarse, 4)
        if side is not None:   # fork (issued after the band's field launch, waiting only for the march)
            side.wait_event(marched)
            for t in (world, rds) + tuple(x for x in c2w_info if torch.is_tensor(x)):
                t.record_stream(side)
            with torch.cuda.stream(side):
                output_coarse, depth_coarse = coarse_pass()
        # renderers.py:503: volume_integral(z, sigma, rad) with sigma = field[..., 3:], rad = field[..., :3]
        rgb, distance_map, _ = volume_integral_packed(z_vals_sorted, field, white_back=self.white_back)
        depth_map = ops.depth_from_world(ros, rds, distance_map.reshape(SB, num_rays), c2w_info)
        if side is not None:   # join: the coarse outputs are read on the caller's stream from here on
            main.wait_stream(side)
            for t in (output_coarse, depth_coarse):
                t.record_stream(main)
        rgb_coarse = output_coarse[..., :3].reshape(SB, num_rays, 3)
        return rgb_coarse, rgb, depth_coarse, depth_map

    @classmethod
    def from_conf(cls, conf, white_back=False):
        return cls(num_feature_channels=conf.get_int("num_feature_channels", 512),
                   raymarch_steps=conf.get_int("raymarch_steps", 10), epsilon=conf.get_float("epsilon", 0.05),
                   n_coarse=conf.get_int("n_coarse", 20), white_back=conf.get_float("white_back", white_back))
