"""Fused HIP evaluation of a NewPixelNeRFNet (models.py:739-863).

FusedField repacks each ResnetFC into MFMA fragment order (avr_field_pack),
projects the latent map through lin_z once per texel (avr_field_latent_table)
and evaluates sigma/RGB with one kernel launch per pass (avr_field_fwd_rays /
avr_field_fwd_points). Packed weights and tables are cached and rebuilt when a
parameter or the latent changes (tensor version counters), so an inference
loop over many frames of one scene pays for them once, as the reference pays
for encode() once.
"""
import ctypes

import torch

from . import _lib
from ._lib import FieldDims, ResnetFCWeights, ViewDesc, call, ptr, require_device, stream_of

F32 = torch.float32


def _resnetfc_ok(mlp, d_in, d_latent):
    return (mlp is not None and type(mlp).__name__ == "ResnetFC" and getattr(mlp, "d_in", -1) == d_in
            and mlp.d_latent == d_latent and mlp.d_out == 4 and mlp.d_hidden in (64, 128, 256, 512)
            and not getattr(mlp, "use_spade", False) and isinstance(mlp.activation, torch.nn.ReLU)
            and 1 <= mlp.n_blocks <= _lib.AVR_MAX_BLOCKS
            and all(not blk.bn and blk.shortcut is None and isinstance(blk.activation, torch.nn.ReLU)
                    for blk in mlp.blocks))


def fused_eligible(net):
    """True when `net` is a NewPixelNeRFNet configured like conf/default*.conf:
    local encoder, xyz + PE(xyz) + raw viewdirs, normalize_z, bilinear/border
    latent lookup, ResNet MLPs, one source view."""
    try:
        code = getattr(net, "code", None)
        enc = net.encoder
        ok = (net.use_encoder and net.use_xyz and net.normalize_z and net.use_code and net.use_viewdirs
              and not net.use_code_viewdirs and not getattr(net, "use_global_encoder", False)
              and net.num_views_per_obj == 1 and code is not None and code.include_input and code.d_in == 3
              and getattr(enc, "index_interp", "bilinear") == "bilinear"
              and getattr(enc, "index_padding", "border") == "border"
              and enc.latent.dim() == 4 and enc.latent.shape[1] % 16 == 0 and enc.latent.shape[1] <= 1024
              and net.d_in == 6 * code.num_freqs + 6)
        if not ok:
            return False
        mlps = [net.mlp_coarse] + ([net.mlp_fine] if net.mlp_fine is not None else [])
        return all(_resnetfc_ok(m, net.d_in, net.d_latent) for m in mlps)
    except AttributeError:
        return False


def _freq_factor(code):
    ff = getattr(code, "freq_factor", None)
    if ff is None:
        ff = float(code.freqs[0])
    return float(ff)


def _version_key(tensors):
    return tuple((t.data_ptr(), t._version) for t in tensors)


class _Packed:
    def __init__(self, dims, packed, table_keys):
        self.dims = dims
        self.packed = packed
        self.tables = {}


PRECISIONS = {"fp32": _lib.FIELD_FP32, "x3": _lib.FIELD_X3}


class FusedField:
    """precision: "x3" (default) = split-fp16 MFMA (3 products per fp32 product,
    fp32 accumulation, within fp32 noise of the fp32 path); "fp32" = fp32 MFMA."""

    def __init__(self, net, precision="x3"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self.precision = precision
        self.net = net
        self._packed = {}     # coarse(bool) -> (key, _Packed)
        self._view_cache = {}

    # ----------------------------------------------------------- parameters
    def _mlp(self, coarse):
        net = self.net
        return net.mlp_coarse if (coarse or net.mlp_fine is None) else net.mlp_fine

    def dims(self, mlp):
        code = self.net.code
        return FieldDims(self.net.d_in, self.net.d_latent, mlp.d_hidden, mlp.n_blocks,
                         min(mlp.combine_layer, mlp.n_blocks), code.num_freqs, _freq_factor(code),
                         PRECISIONS[self.precision])

    def packed(self, coarse):
        mlp = self._mlp(coarse)
        params = [p.detach() for p in mlp.parameters()]
        key = (id(mlp), _version_key(params))
        hit = self._packed.get(coarse)
        if hit is not None and hit[0] == key:
            return hit[1]
        dims = self.dims(mlp)
        n = ctypes.c_int64(0)
        _lib.check(_lib.load().avr_field_packed_floats(ctypes.byref(dims), ctypes.byref(n)), "avr_field_packed_floats")
        dev = params[0].device
        packed = torch.empty(n.value, device=dev, dtype=F32)
        w = ResnetFCWeights()
        keep = []

        def P(t):
            t = t.detach().to(F32).contiguous()
            keep.append(t)
            return t.data_ptr()

        w.lin_in_w, w.lin_in_b = P(mlp.lin_in.weight), P(mlp.lin_in.bias)
        w.lin_out_w, w.lin_out_b = P(mlp.lin_out.weight), P(mlp.lin_out.bias)
        for b, blk in enumerate(mlp.blocks):
            w.fc0_w[b], w.fc0_b[b] = P(blk.fc_0.weight), P(blk.fc_0.bias)
            w.fc1_w[b], w.fc1_b[b] = P(blk.fc_1.weight), P(blk.fc_1.bias)
        for b in range(dims.n_lin_z):
            w.lin_z_w[b], w.lin_z_b[b] = P(mlp.lin_z[b].weight), P(mlp.lin_z[b].bias)
        require_device(*keep)
        call("avr_field_pack", ctypes.byref(dims), ctypes.byref(w), ptr(packed), stream_of(packed))
        entry = _Packed(dims, packed, None)
        entry._keep = keep
        self._packed[coarse] = (key, entry)
        return entry

    def table(self, coarse, sb=0):
        entry = self.packed(coarse)
        lat = self.net.encoder.latent
        key = (sb, lat.data_ptr(), lat._version, tuple(lat.shape))
        hit = entry.tables.get(sb)
        if hit is not None and hit[0] == key:
            return hit[1]
        dims = entry.dims
        L, H, W = lat.shape[1:]
        latent = lat[sb].detach().to(F32).contiguous()
        require_device(latent)
        table = torch.empty(max(dims.n_lin_z, 1), H * W, dims.d_hidden, device=latent.device, dtype=F32)
        call("avr_field_latent_table", ctypes.byref(dims), ptr(entry.packed), ptr(latent), H, W, ptr(table),
             stream_of(table))
        entry.tables[sb] = (key, table, lat)  # holding `lat` keeps its address from being reused
        return table

    def view(self, sb=0):
        net = self.net
        srcs = [net.poses, net.focal, net.c, net.image_shape, net.encoder.latent_scaling]
        key = (sb, _version_key(srcs), tuple(net.encoder.latent.shape))
        hit = self._view_cache.get(sb)
        if hit is not None and hit[0] == key:
            return hit[1]
        pick = lambda t: t[min(sb, t.shape[0] - 1)] if t.dim() > 1 else t  # noqa: E731
        v = ViewDesc()
        v.poses[:] = [float(x) for x in pick(net.poses).reshape(-1)[:12].tolist()]
        v.focal[:] = [float(x) for x in pick(net.focal).reshape(-1)[:2].tolist()]
        v.c[:] = [float(x) for x in pick(net.c).reshape(-1)[:2].tolist()]
        v.image_shape[:] = [float(x) for x in net.image_shape.reshape(-1)[:2].tolist()]
        v.latent_scaling[:] = [float(x) for x in net.encoder.latent_scaling.reshape(-1)[:2].tolist()]
        v.latent_h, v.latent_w = int(net.encoder.latent.shape[-2]), int(net.encoder.latent.shape[-1])
        self._view_cache[sb] = (key, v, srcs)  # holding the sources keeps (ptr, version) keys sound
        return v

    # ----------------------------------------------------------- evaluation
    def forward_rays(self, ro, rd, z, coarse, sb=0):
        """sigma/RGB at ro[r] + rd[r]*z[r,s] with viewdir rd[r]: (R*N, 4)."""
        R, N = z.shape
        ro = ro.reshape(R, 3).to(F32).contiguous()
        rd = rd.reshape(R, 3).to(F32).contiguous()
        z = z.to(F32).contiguous()
        require_device(ro, rd, z)
        entry = self.packed(coarse)
        table = self.table(coarse, sb)
        out = torch.empty(R * N, 4, device=z.device, dtype=F32)
        entry.dims.precision = PRECISIONS[self.precision]
        call("avr_field_fwd_rays", ctypes.byref(entry.dims), ctypes.byref(self.view(sb)), ptr(entry.packed),
             ptr(table), ptr(ro), ptr(rd), ptr(z), R, N, ptr(out), stream_of(z))
        return out

    def forward_points(self, xyz, viewdirs, coarse):
        """The rf(xyz (SB,B,3), viewdirs, coarse) protocol -> (SB, B, 4)."""
        SB, B, _ = xyz.shape
        out = torch.empty(SB, B, 4, device=xyz.device, dtype=F32)
        entry = self.packed(coarse)
        for sb in range(SB):
            p = xyz[sb].to(F32).contiguous()
            v = viewdirs.reshape(SB, B, 3)[sb].to(F32).contiguous()
            require_device(p, v)
            table = self.table(coarse, sb)
            entry.dims.precision = PRECISIONS[self.precision]
            call("avr_field_fwd_points", ctypes.byref(entry.dims), ctypes.byref(self.view(sb)), ptr(entry.packed),
                 ptr(table), ptr(p), ptr(v), B, ptr(out[sb]), stream_of(p))
        return out
