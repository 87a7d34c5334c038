"""Torch-tensor wrappers over the C ABI (one function per kernel entry point).

All tensors are device tensors owned by PyTorch; every launch is enqueued on
torch's current HIP stream. No function here has a host/CPU implementation.
"""
import ctypes
import functools

import torch

from . import _lib
from ._lib import call, ptr, require_device, stream_of

F32 = torch.float32


def _f32c(t):
    return t if (t.dtype == F32 and t.is_contiguous()) else t.to(F32).contiguous()


def world_rays(x_pix, intrinsics, cam2world):
    """get_world_rays (utils.py:315-336). x_pix (SB,R,2), intrinsics (SB,3,3),
    cam2world (SB,R,4,4) -- may be a stride-0 expand of one pose per batch."""
    SB, R, _ = x_pix.shape
    x_pix = _f32c(x_pix)
    K = _f32c(intrinsics.reshape(SB, 3, 3))
    c2w = cam2world.to(F32)
    if c2w.dim() == 3:
        c2w = c2w.unsqueeze(1)
    if c2w.stride(-1) != 1 or c2w.stride(-2) != 4:
        c2w = c2w.contiguous()
    sb_stride = c2w.stride(0) if c2w.shape[0] > 1 else 0
    ray_stride = c2w.stride(1) if c2w.shape[1] > 1 else 0
    require_device(x_pix, K)
    ro = torch.empty(SB, R, 3, device=x_pix.device, dtype=F32)
    rd = torch.empty_like(ro)
    call("avr_world_rays", ptr(x_pix), ptr(K), ptr(c2w), sb_stride, ray_stride, SB, R, ptr(ro), ptr(rd),
         stream_of(x_pix))
    return ro, rd, (c2w, sb_stride, ray_stride)


def _c2w_view(cam2world):
    c2w = cam2world.to(F32)
    if c2w.dim() == 3:
        c2w = c2w.unsqueeze(1)
    if c2w.stride(-1) != 1 or c2w.stride(-2) != 4:
        c2w = c2w.contiguous()
    sb_stride = c2w.stride(0) if c2w.shape[0] > 1 else 0
    ray_stride = c2w.stride(1) if c2w.shape[1] > 1 else 0
    return c2w, sb_stride, ray_stride


def rays_sample_coarse(x_pix, intrinsics, cam2world, near, far, n_samples, noise=None, seed=0, offset=0,
                       ray_ids=None, want_depth_row=False):
    """get_world_rays + sample_coarse in one launch (avr_rays_sample_coarse):
    -> ro, rd (SB, R, 3), z (SB*R, n_samples), depth_row (SB*R, 4) fp64 or None,
    c2w_info. Bit-identical to world_rays followed by sample_coarse."""
    SB, R, _ = x_pix.shape
    x_pix = _f32c(x_pix)
    K = _f32c(intrinsics.reshape(SB, 3, 3))
    c2w, sb_stride, ray_stride = _c2w_view(cam2world)
    require_device(x_pix, K)
    dev = x_pix.device
    ro = torch.empty(SB, R, 3, device=dev, dtype=F32)
    rd = torch.empty_like(ro)
    z = torch.empty(SB * R, n_samples, device=dev, dtype=F32)
    drow = torch.empty(SB * R, 4, device=dev, dtype=torch.float64) if want_depth_row else None
    if noise is not None:
        noise = _f32c(noise.reshape(SB * R, n_samples))
        require_device(noise)
    ray_ids = _ray_ids(ray_ids, SB * R)
    call("avr_rays_sample_coarse", ptr(x_pix), ptr(K), ptr(c2w), sb_stride, ray_stride, SB, R, float(near), float(far),
         n_samples, ptr(noise), seed, offset, ptr(ray_ids), ptr(ro), ptr(rd), ptr(drow), ptr(z), stream_of(x_pix))
    return ro, rd, z, drow, (c2w, sb_stride, ray_stride)


def composite_depth(z, field, ro, rd, depth_row, white_back=True, infinity=1.8, want_weights=False):
    """volume_integral + depth_from_world of the expected distance in one launch
    (avr_composite_fwd_depth; no autograd) -> rgb (R,3), dist (R,), weights or
    None, depth (R,)."""
    R, N = z.shape
    z = _f32c(z)
    field = _f32c(field.reshape(R, N, 4))
    ro, rd = _f32c(ro.reshape(R, 3)), _f32c(rd.reshape(R, 3))
    require_device(z, field, ro, rd, depth_row)
    rgb = torch.empty(R, 3, device=z.device, dtype=F32)
    dist = torch.empty(R, device=z.device, dtype=F32)
    depth = torch.empty(R, device=z.device, dtype=F32)
    w = torch.empty(R, N, device=z.device, dtype=F32) if want_weights else None
    call("avr_composite_fwd_depth", ptr(z), ptr(field), R, N, int(bool(white_back)), float(infinity), ptr(ro),
         ptr(rd), ptr(depth_row), ptr(rgb), ptr(dist), ptr(w), ptr(depth), stream_of(z))
    return rgb, dist, w, depth


def depth_from_world_fwd(ro, rd, dist, c2w_info, want_grad=False):
    c2w, sb_stride, ray_stride = c2w_info
    SB, R, _ = ro.shape
    dist = _f32c(dist.detach().reshape(SB, R))
    depth = torch.empty(SB, R, device=ro.device, dtype=F32)
    dd = torch.empty(SB, R, device=ro.device, dtype=F32) if want_grad else None
    call("avr_depth_from_world", ptr(ro), ptr(rd), ptr(dist), ptr(c2w), sb_stride, ray_stride, SB, R, ptr(depth),
         ptr(dd), stream_of(ro))
    return depth, dd


class _Depth(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dist, ro, rd, c2w_info):
        depth, dd = depth_from_world_fwd(ro, rd, dist, c2w_info, want_grad=True)
        ctx.save_for_backward(dd)
        ctx.dist_shape = dist.shape
        return depth

    @staticmethod
    def backward(ctx, g):
        (dd,) = ctx.saved_tensors
        return (g * dd).reshape(ctx.dist_shape), None, None, None


def depth_from_world(ro, rd, dist, c2w_info):
    """depth_from_world(ro + rd*dist, c2w) (renderers.py:274-275, utils.py:358-361);
    differentiable w.r.t. dist."""
    if torch.is_grad_enabled() and dist.requires_grad:
        return _Depth.apply(dist, ro, rd, c2w_info)
    return depth_from_world_fwd(ro, rd, dist, c2w_info)[0]


def _ray_ids(ray_ids, n_rays):
    if ray_ids is None:
        return None
    ray_ids = ray_ids.reshape(-1).to(torch.int64).contiguous()
    if ray_ids.numel() != n_rays:
        raise _lib.AVRError(f"ray_ids has {ray_ids.numel()} entries for {n_rays} rays")
    require_device(ray_ids)
    return ray_ids


def sample_coarse(near, far, n_rays, n_samples, device, noise=None, seed=0, offset=0, ray_ids=None):
    """sample_coarse (renderers.py:4-24) -> z (n_rays, n_samples). `noise` is the
    rand_like draw (n_rays, n_samples) or None for in-kernel Philox keyed on
    offset + ray (or offset + ray_ids[ray]: global ray ids of a sharded frame)."""
    z = torch.empty(n_rays, n_samples, device=device, dtype=F32)
    if noise is not None:
        noise = _f32c(noise.reshape(n_rays, n_samples))
        require_device(noise)
    ray_ids = _ray_ids(ray_ids, n_rays)
    call("avr_sample_coarse", float(near), float(far), n_rays, n_samples, ptr(noise), seed, offset, ptr(ray_ids),
         ptr(z), stream_of(z))
    return z


def sample_fine(weights, z_coarse, near, far, n_importance, n_depth, depth_std, u=None, u2=None, noise_depth=None,
                seed=0, offset=0, want_idx=False, want_fine=False, ray_ids=None):
    """sample_fine + sample_depth + clamp + sort (renderers.py:27-66, :252-258).
    weights, z_coarse (R, Nc) -> z_sorted (R, Nc+Nf+Nd) [, idx (R,Nf) int32, z_fine (R,Nf)]."""
    R, Nc = z_coarse.shape
    weights = _f32c(weights.reshape(R, Nc))
    z_coarse = _f32c(z_coarse)
    dev = z_coarse.device
    if (u is None) != (u2 is None):
        raise _lib.AVRError("sample_fine: u and u2 must be given together")
    if u is not None:
        u = _f32c(u.reshape(R, n_importance))
        u2 = _f32c(u2.reshape(R, n_importance))
        noise_depth = _f32c(noise_depth.reshape(R, n_depth)) if n_depth > 0 else None
    require_device(weights, z_coarse, u, u2, noise_depth)
    ray_ids = _ray_ids(ray_ids, R)
    z_sorted = torch.empty(R, Nc + n_importance + n_depth, device=dev, dtype=F32)
    idx = torch.empty(R, n_importance, device=dev, dtype=torch.int32) if want_idx else None
    z_fine = torch.empty(R, n_importance, device=dev, dtype=F32) if want_fine else None
    call("avr_sample_fine", ptr(weights), ptr(z_coarse), float(near), float(far), R, Nc, n_importance, n_depth,
         float(depth_std), ptr(u), ptr(u2), ptr(noise_depth), seed, offset, ptr(ray_ids), ptr(z_sorted), ptr(idx),
         ptr(z_fine),
         stream_of(z_coarse))
    return z_sorted, idx, z_fine


def composite_fwd(z, field, white_back=True, infinity=1.8, want_weights=True):
    """volume_integral (renderers.py:69-119). z (R,N), field (R,N,4) ->
    rgb (R,3), dist (R,), weights (R,N)."""
    R, N = z.shape
    z = _f32c(z)
    field = _f32c(field.reshape(R, N, 4))
    require_device(z, field)
    rgb = torch.empty(R, 3, device=z.device, dtype=F32)
    dist = torch.empty(R, device=z.device, dtype=F32)
    w = torch.empty(R, N, device=z.device, dtype=F32) if want_weights else None
    call("avr_composite_fwd", ptr(z), ptr(field), R, N, int(bool(white_back)), float(infinity), ptr(rgb),
         ptr(dist), ptr(w), stream_of(z))
    return rgb, dist, w


def composite_bwd(z, field, grad_rgb, grad_dist, grad_w, white_back=True, infinity=1.8, want_grad_z=False):
    """Gradients of volume_integral: d/d field (R,N,4) and, if want_grad_z, d/dz (R,N)."""
    R, N = z.shape
    grad_rgb = _f32c(grad_rgb.reshape(R, 3))
    grad_dist = None if grad_dist is None else _f32c(grad_dist.reshape(R))
    grad_w = None if grad_w is None else _f32c(grad_w.reshape(R, N))
    require_device(grad_rgb, grad_dist, grad_w)
    gfield = torch.empty(R, N, 4, device=z.device, dtype=F32)
    gz = torch.empty(R, N, device=z.device, dtype=F32) if want_grad_z else None
    call("avr_composite_bwd", ptr(z), ptr(field), R, N, int(bool(white_back)), float(infinity), ptr(grad_rgb),
         ptr(grad_dist), ptr(grad_w), ptr(gfield), ptr(gz), stream_of(z))
    return (gfield, gz) if want_grad_z else gfield


class _Composite(torch.autograd.Function):
    """Autograd node for volume_integral: gradients flow to (rgb, sigma) of the
    field output and, when z requires grad (AdaptiveVolumeRenderer's band), to z."""

    @staticmethod
    def forward(ctx, z, field, white_back, infinity):
        zd = _f32c(z.detach())
        field = _f32c(field.detach())
        rgb, dist, w = composite_fwd(zd, field, white_back, infinity, want_weights=True)
        ctx.save_for_backward(zd, field)
        ctx.white_back, ctx.infinity = white_back, infinity
        return rgb, dist, w

    @staticmethod
    def backward(ctx, g_rgb, g_dist, g_w):
        z, field = ctx.saved_tensors
        if g_rgb is None:
            g_rgb = torch.zeros(z.shape[0], 3, device=z.device, dtype=F32)
        want_z = ctx.needs_input_grad[0]
        out = composite_bwd(z, field, g_rgb, g_dist, g_w, ctx.white_back, ctx.infinity, want_grad_z=want_z)
        gfield, gz = out if want_z else (out, None)
        return gz, gfield if ctx.needs_input_grad[1] else None, None, None


def composite(z, field, white_back=True, infinity=1.8, want_weights=True):
    """Differentiable volume_integral on (R,N) z and (R,N,4) field. Without
    autograd, want_weights=False skips the (R,N) weights store (returns None)."""
    if torch.is_grad_enabled() and (field.requires_grad or z.requires_grad):
        return _Composite.apply(z, field, white_back, infinity)
    return composite_fwd(z, field, white_back, infinity, want_weights=want_weights)


def points(ro, rd, z):
    """pts = ro + rd * z, viewdirs = rd per sample (renderers.py:171, :174) as
    (R*N, 3) tensors for a generic radiance field."""
    R, N = z.shape
    pts = torch.addcmul(ro.reshape(R, 1, 3), rd.reshape(R, 1, 3), z.reshape(R, N, 1))
    vd = rd.reshape(R, 1, 3).expand(R, N, 3)
    return pts.reshape(R * N, 3), vd.reshape(R * N, 3)


def march_fine(ro, rd, z, field_fn, t_stop, white_back=True, infinity=1.8, chunk=64):
    """Fine pass with early ray termination (BASELINE config 4; not in the
    reference): the samples z (R, N) are evaluated front to back in chunks of
    `chunk`, and a ray leaves the active set once its transmittance drops
    below `t_stop` (its skipped tail changes rgb by <= t_stop).
    field_fn(ro_c, rd_c, z_c) -> (n_act * C, 4) evaluates the field on a chunk.
    Returns rgb (R, 3), dist (R,), and the number of field samples evaluated."""
    R, N = z.shape
    ro, rd, z = _f32c(ro.reshape(R, 3)), _f32c(rd.reshape(R, 3)), _f32c(z)
    require_device(ro, rd, z)
    dev, s = z.device, stream_of(z)
    nbytes = ctypes.c_int64()
    call("avr_march_state_bytes", R, ctypes.byref(nbytes))
    state = torch.empty(max(nbytes.value, 8), device=dev, dtype=torch.uint8)
    active = torch.empty(max(R, 1), device=dev, dtype=torch.int32)
    spare = torch.empty_like(active)
    count = torch.zeros(1, device=dev, dtype=torch.int32)
    call("avr_march_init", R, ptr(state), ptr(active), s)
    n_act, evaluated = R, 0
    for c0 in range(0, N, chunk):
        if n_act == 0:
            break
        C = min(chunk, N - c0)
        ro_c = torch.empty(n_act, 3, device=dev, dtype=F32)
        rd_c = torch.empty_like(ro_c)
        z_c = torch.empty(n_act, C, device=dev, dtype=F32)
        call("avr_march_gather", ptr(ro), ptr(rd), ptr(z), ptr(active), n_act, N, c0, C, ptr(ro_c), ptr(rd_c),
             ptr(z_c), s)
        f_c = _f32c(field_fn(ro_c, rd_c, z_c).reshape(n_act, C, 4))
        evaluated += n_act * C
        count.zero_()
        call("avr_march_composite", ptr(z), ptr(f_c), ptr(active), n_act, N, c0, C, float(infinity), float(t_stop),
             ptr(state), ptr(spare), ptr(count), s)
        active, spare = spare, active
        n_act = int(count.item()) if c0 + C < N else 0
    rgb = torch.empty(R, 3, device=dev, dtype=F32)
    dist = torch.empty(R, device=dev, dtype=F32)
    call("avr_march_finish", ptr(state), R, 1 if white_back else 0, ptr(rgb), ptr(dist), s)
    return rgb, dist, evaluated


def sample_coarse_rays(near, far, n_samples, noise=None, seed=0, offset=0):
    """sample_coarse with per-ray bounds near/far (R,) -> z (R, n_samples)
    (renderers.py:4-24 called with tensors, as AdaptiveVolumeRenderer does)."""
    near, far = _f32c(near.reshape(-1)), _f32c(far.reshape(-1))
    R = near.shape[0]
    require_device(near, far)
    z = torch.empty(R, n_samples, device=near.device, dtype=F32)
    if noise is not None:
        noise = _f32c(noise.reshape(R, n_samples))
    call("avr_sample_coarse_rays", ptr(near), ptr(far), R, n_samples, ptr(noise), int(seed), int(offset), ptr(z),
         stream_of(z))
    return z


def depth_of_points_fwd(world, c2w_info):
    c2w, sb_stride, ray_stride = c2w_info
    SB, R, _ = world.shape
    world = _f32c(world.detach())
    depth = torch.empty(SB, R, device=world.device, dtype=F32)
    call("avr_depth_from_world", ptr(world), None, None, ptr(c2w), sb_stride, ray_stride, SB, R, ptr(depth), None,
         stream_of(world))
    return depth


class _DepthOfPoints(torch.autograd.Function):
    """depth = -(inv(c2w)[2, :3] . x + inv(c2w)[2, 3]): d depth / d x = -inv(c2w)[2, :3]
    (utils.py:358-361 is differentiable in the world points: the raymarchers' depth
    loss reaches the LSTM through them, renderers.py:349, :486)."""

    @staticmethod
    def forward(ctx, world, c2w_info):
        ctx.c2w_info = c2w_info
        ctx.shape = world.shape
        return depth_of_points_fwd(world, c2w_info)

    @staticmethod
    def backward(ctx, g):
        c2w, sb_stride, ray_stride = ctx.c2w_info
        SB, R, _ = ctx.shape
        if ray_stride == 0:
            # one pose per batch (the stride-0 expand the callers pass): invert it once, not per ray
            c2w = c2w[:, :1]
        if sb_stride == 0:
            c2w = c2w[:1]
        row = -torch.linalg.inv(c2w.double())[..., 2, :3].to(F32)       # (SB or 1, R or 1, 3)
        return g.reshape(SB, R, 1) * row.expand(SB, R, 3), None


def depth_of_points(world, c2w_info):
    """depth_from_world(world, cam2world) for explicit world points (SB, R, 3) -> (SB, R);
    differentiable w.r.t. world."""
    if torch.is_grad_enabled() and world.requires_grad:
        return _DepthOfPoints.apply(world, c2w_info)
    return depth_of_points_fwd(world, c2w_info)


def raymarch(view, gate_table, lstm, out_layer, ro, rd, init_dist, steps, trace=False):
    """LSTM ray march (renderers.py:329-343): ro, rd, init_dist (R,) ->
    world (R, 3), final_dist (R,) [, trace (steps+1, R, 3)]. gate_table
    (H*W, 64) = per-texel W_ih projection of the latent."""
    R = ro.shape[0]
    ro, rd, d0 = _f32c(ro.reshape(R, 3)), _f32c(rd.reshape(R, 3)), _f32c(init_dist.reshape(R))
    ps = [_f32c(t.detach()) for t in (gate_table, lstm.weight_hh, lstm.bias_ih, lstm.bias_hh,
                                      out_layer.weight.reshape(-1), out_layer.bias.reshape(-1))]
    require_device(ro, rd, d0, *ps)
    world = torch.empty(R, 3, device=ro.device, dtype=F32)
    fd = torch.empty(R, device=ro.device, dtype=F32)
    tr = torch.empty(steps + 1, R, 3, device=ro.device, dtype=F32) if trace else None
    call("avr_raymarch", ctypes.byref(view), *[ptr(t) for t in ps], ptr(ro), ptr(rd), ptr(d0), R, int(steps),
         ptr(world), ptr(fd), ptr(tr), stream_of(ro))
    return (world, fd, tr) if trace else (world, fd)


def sum_of_products(pairs):
    """sum_i A_i @ B_i with the accumulation inside the GEMMs (addmm_, beta = 1): no separate add passes over the
    (rows, cols) partial products."""
    (a0, b0), *rest = pairs
    out = a0 @ b0
    for a, b in rest:
        out.addmm_(a, b)
    return out


def _max_bits(t):
    """max |t| as a one-element int32 device tensor of float bits (avr_weight_grads' scale input): one
    min / max pass over t, no |t| copy (max |t| = max(|max t|, |min t|) exactly)."""
    t = t.detach()
    if t.numel() == 0:
        return torch.zeros(1, device=t.device, dtype=torch.int32)
    mn, mx = torch.aminmax(t)
    return torch.maximum(mx.abs(), mn.abs()).reshape(1).to(torch.float32).view(torch.int32)


def lin_out_rows(x, weight, bias):
    """lin_out of the layer-by-layer training paths over (n, d_hidden) rows x: (out (n, 4) = [sigmoid rgb,
    relu sigma] of relu(x) . weight^T + bias (models.py:592, 856-862), max relu(x) as int32 float bits)
    (avr_lin_out_fwd_rows, one pass over x)."""
    n, H = x.shape
    out = torch.empty(n, 4, device=x.device, dtype=F32)
    xmax = torch.zeros(1, device=x.device, dtype=torch.int32)
    call("avr_lin_out_fwd_rows", n, H, ptr(x), x.stride(0), ptr(_f32c(weight)), ptr(_f32c(bias)), ptr(out),
         ptr(xmax), stream_of(x))
    return out, xmax


def lin_out_rows_bwd(grad_out, out, weight, pre, g=None):
    """The backward of lin_out_rows: (d_raw (n, 4), g (n, d_hidden) = d_raw . weight where pre > 0, max |d_raw|
    as int32 float bits) (avr_lin_out_bwd_rows; torch's sigmoid / relu / threshold backward in one pass); g may
    be given (contiguous rows)."""
    n, H = pre.shape
    d_raw = torch.empty(n, 4, device=pre.device, dtype=F32)
    if g is None:
        g = torch.empty(n, H, device=pre.device, dtype=F32)
    assert g.shape == (n, H) and g.is_contiguous() and g.dtype == F32
    dmax = torch.zeros(1, device=pre.device, dtype=torch.int32)
    call("avr_lin_out_bwd_rows", n, H, ptr(_f32c(grad_out)), ptr(_f32c(out)), ptr(_f32c(weight)), ptr(pre),
         pre.stride(0), ptr(d_raw), ptr(g), ptr(dmax), stream_of(pre))
    return d_raw, g, dmax


def lin_out_act_bwd(grad_out, out):
    """The activations' backward of lin_out's outputs alone: (d_raw (n, 4) = [sigmoid_backward rgb,
    threshold_backward sigma], max |d_raw| as int32 float bits) (avr_lin_out_act_bwd_rows; torch's
    sigmoid_backward / threshold_backward bit for bit), over contiguous (..., 4) fp32 grad_out / out."""
    go, y = _f32c(grad_out.reshape(-1, 4)), _f32c(out.reshape(-1, 4))
    n = go.shape[0]
    d_raw = torch.empty(n, 4, device=go.device, dtype=F32)
    dmax = torch.zeros(1, device=go.device, dtype=torch.int32)
    call("avr_lin_out_act_bwd_rows", n, ptr(go), ptr(y), ptr(d_raw), ptr(dmax), stream_of(go))
    return d_raw, dmax


def spade_bwd_rows(g, x, s):
    """The spade product rule's backward (avr_spade_bwd_rows): (g * x, s * g, max |g * x| as int32 float bits) in
    one pass over contiguous fp32 tensors of one shape, bit-identical to torch's two products."""
    for t in (g, x, s):
        if t.dtype != F32 or not t.is_contiguous() or t.shape != g.shape or t.data_ptr() % 16:
            raise _lib.AVRError("spade_bwd_rows: contiguous 16-B aligned fp32 tensors of one shape")
    gs, g_out = torch.empty_like(g), torch.empty_like(g)
    gmax = torch.zeros(1, device=g.device, dtype=torch.int32)
    call("avr_spade_bwd_rows", g.numel(), ptr(g), ptr(x), ptr(s), ptr(gs), ptr(g_out), ptr(gmax), stream_of(g))
    return gs, g_out, gmax


_DW_TILE = 256        # avr_weight_grads output tile (weight_grad.hip kDwTile), one workgroup per CU


def _wgrad_splits(tiles, n_rows, dev):
    """K-split of avr_weight_grads: the grid (tiles x splits workgroups, one per
    CU) should end in full rounds, with K-ranges of at least 2048 rows."""
    return _wgrad_splits_cu(tiles, n_rows, torch.cuda.get_device_properties(dev).multi_processor_count)


@functools.lru_cache(maxsize=256)
def _wgrad_splits_cu(tiles, n_rows, slots):
    best, best_eff = 1, 0.0
    for n in range(1, 65):
        if n > 1 and n_rows < 2048 * n:
            break
        w = n * tiles
        eff = w / (-(-w // slots) * slots) * min(1.0, w / slots)
        if eff >= 0.95:
            return n      # the fewest splits (partials) that fill the rounds
        if eff > best_eff + 1e-3:
            best, best_eff = n, eff
    return best


def weight_grads(layers, n_rows, n_split=None):
    """dW = G^T X and db = colsum(G) for each (grad, input, grad_max, input_max, want_bias[, bn])
    of `layers` (avr_weight_grads: split-K x3 MFMA). grad (n_rows, out) / input
    (n_rows, in) fp32 row-major (row strides may exceed the widths); *_max: int32
    (1,) float bits of max |.|; bn = (mu, scale, shift) (in,) each: X = relu((input - mu) * scale + shift)
    per column, a training-mode BatchNorm's operand rebuilt from its pre-BN rows (input_max then of X), or
    bn = "relu": X = relu(input).
    Returns [(dW (out, in), db (out,) or None)]."""
    if not layers:
        return []
    dev = layers[0][0].device
    if n_rows == 0:
        return [(torch.zeros(l[0].shape[1], l[1].shape[1], device=dev), torch.zeros(l[0].shape[1], device=dev) if l[4] else None)
                for l in layers]
    specs = []
    for g, x, gmax, xmax, want_bias, *bn in layers:
        O, I = g.shape[1], x.shape[1]
        bn = bn[0] if bn else None
        relu = isinstance(bn, str)
        if relu and bn != "relu":
            raise _lib.AVRError(f"weight_grads: unknown input transform {bn!r}")
        bn = None if relu else bn
        for t in (g, x):
            if t.dtype != torch.float32 or t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
                raise _lib.AVRError("weight_grads: operands must be fp32 rows, 16-B aligned, unit column stride")
        if bn is not None and any(t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != I
                                  or t.data_ptr() % 16 for t in bn):
            raise _lib.AVRError("weight_grads: the BatchNorm transform takes (in,) fp32 mu / scale / shift")
        specs.append((g.data_ptr(), g.stride(0), x.data_ptr(), x.stride(0), O, I, gmax.data_ptr(), xmax.data_ptr(),
                      bool(want_bias), *([t.data_ptr() for t in bn] if bn is not None else [None] * 3), int(relu)))
    return weight_grads_specs(specs, n_rows, dev, stream_of(layers[0][0]), n_split)


def weight_grads_specs(specs, n_rows, dev, stream, n_split=None):
    """weight_grads on layers given as plain integers -- (grad ptr, grad row stride, input ptr, input row stride,
    out, in, grad_max ptr, input_max ptr, want_bias, mu ptr, scale ptr, shift ptr, input relu) -- for callers
    that own the row buffers and address their layers by offset (the fused field's training backward: no
    per-layer views, checks or tensor calls). Same launches and results as weight_grads."""
    if n_rows == 0:
        return [(torch.zeros(s[4], s[5], device=dev), torch.zeros(s[4], device=dev) if s[8] else None)
                for s in specs]
    if n_split is None:
        n_split = _wgrad_splits(sum(-(-s[4] // _DW_TILE) * -(-s[5] // _DW_TILE) for s in specs), n_rows, dev)
    out = []
    for base in range(0, len(specs), _lib.AVR_WGRAD_MAX_LAYERS):
        chunk = specs[base:base + _lib.AVR_WGRAD_MAX_LAYERS]
        arr = (_lib.WGradLayer * len(chunk))()
        # the partials of the whole chunk in one buffer (every piece a multiple of 16 B: O, I multiples of 4)
        sizes = [n_split * s[4] * (s[5] + (1 if s[8] else 0)) for s in chunk]
        flat = torch.empty(sum(sizes), device=dev, dtype=torch.float32)
        dw_ptrs, db_ptrs = (ctypes.c_void_p * len(chunk))(), (ctypes.c_void_p * len(chunk))()
        # every dW / db of the chunk as views of one allocation, cut by one split (two allocations per layer, then
        # two slices per layer, were host time); the partials are addressed by offset, no view of them is needed
        pieces = []
        for s in chunk:
            pieces += [s[4] * s[5], s[4]] if s[8] else [s[4] * s[5]]
        outs = torch.empty(sum(pieces), device=dev, dtype=torch.float32).split(pieces)
        flat_p = flat.data_ptr()
        res, off, vi = [], 0, 0
        for k, (gp, ldg, xp, ldx, O, I, gmp, xmp, want_bias, mu, sc, sh, relu) in enumerate(chunk):
            part_p = flat_p + 4 * off
            off += sizes[k]
            arr[k] = _lib.WGradLayer(gp, ldg, xp, ldx, O, I, gmp, xmp, part_p,
                                     part_p + 4 * n_split * O * I if want_bias else 0, mu, sc, sh, relu)
            dw = outs[vi].view(O, I)
            db = outs[vi + 1] if want_bias else None
            vi += 2 if want_bias else 1
            dw_ptrs[k], db_ptrs[k] = dw.data_ptr(), (db.data_ptr() if want_bias else None)
            res.append((dw, db))
        call("avr_weight_grads", arr, len(chunk), n_rows, n_split, stream)
        # sum over the splits, every layer in one launch (avr_weight_grads_reduce)
        call("avr_weight_grads_reduce", arr, len(chunk), n_split, dw_ptrs, db_ptrs, stream)
        out += res
    return out


def latent_hwc(latent_chw):
    """(C, H, W) -> the (H*W, C) channels-last fp32 copy avr_latent_features reads."""
    C, H, W = latent_chw.shape
    return latent_chw.detach().to(F32).reshape(C, H * W).t().contiguous()


def latent_features(view, latent_chw, xyz, out=None, hwc=None):
    """SpatialEncoder.index at world points (models.py:245-274, 753-810):
    latent (C, H, W) of one source view (avr.field.FusedField.view gives the
    ViewDesc), xyz (N, 3) -> (N, C) row-major (avr_latent_features). hwc: the
    latent_hwc copy of latent_chw when the caller already has it."""
    C, H, W = latent_chw.shape
    lat = latent_hwc(latent_chw) if hwc is None else hwc
    xyz = _f32c(xyz.reshape(-1, 3))
    n = xyz.shape[0]
    if out is None:
        out = torch.empty(n, C, device=xyz.device, dtype=F32)
    require_device(lat, xyz, out)
    call("avr_latent_features", ctypes.byref(view), ptr(lat), C, ptr(xyz), n, ptr(out), stream_of(xyz))
    return out


def stream_copy(src, dst):
    """dst <- src (same byte size, 16-B aligned): the streaming copy kernel
    bench.py uses as its achievable-HBM yardstick (avr_stream_copy)."""
    require_device(src, dst)
    nb = src.numel() * src.element_size()
    if nb != dst.numel() * dst.element_size():
        raise _lib.AVRError("stream_copy: size mismatch")
    call("avr_stream_copy", ptr(src), ptr(dst), nb, stream_of(src))
    return dst


def stream_fill(dst, word):
    """Every 32-bit word of dst <- word (16-B aligned): the write-only yardstick
    bench.py reports store-dominated kernels against (avr_stream_fill)."""
    require_device(dst)
    call("avr_stream_fill", ptr(dst), dst.numel() * dst.element_size(), int(word) & 0xFFFFFFFF, stream_of(dst))
    return dst
