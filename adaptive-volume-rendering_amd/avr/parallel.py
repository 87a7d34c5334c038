"""Multi-GPU ray sharding (BASELINE config 5): one process per GPU, rays of a
frame dealt to ranks in interleaved 64-ray tiles (early-terminating or
background-heavy image regions then spread evenly), every rank renders its
tiles with the single-GPU path, and one collective assembles the frame:
all_gather of (rgb_coarse, rgb_fine, depth) = 28 B per ray over RCCL/xGMI.

The reference is single-process (train.py:238-242 pins cuda:0); there is no
other exchange on the path: rays are independent and the field weights and
latent are read-only, so each rank builds them locally (or receives them once
through `broadcast_scene`).
"""
import inspect

import torch
import torch.distributed as dist


def ray_tiles(n_rays, rank, world, tile=64, device=None):
    """Indices of the rays owned by `rank`: tiles t with t % world == rank."""
    n_tiles = (n_rays + tile - 1) // tile
    if rank >= n_tiles:
        return torch.zeros(0, dtype=torch.long, device=device)
    mine = torch.arange(rank, n_tiles, world, device=device)
    idx = (mine[:, None] * tile + torch.arange(tile, device=device)[None, :]).reshape(-1)
    return idx[idx < n_rays]


def max_local_rays(n_rays, world, tile=64):
    n_tiles = (n_rays + tile - 1) // tile
    return ((n_tiles + world - 1) // world) * tile


def broadcast_scene(net, src=0, group=None):
    """Send the field weights and the latent map from `src` to every rank (once per scene)."""
    for t in list(net.parameters()) + [net.encoder.latent, net.poses, net.focal, net.c, net.image_shape,
                                       net.encoder.latent_scaling]:
        dist.broadcast(t.data, src, group=group)


def _takes_ray_ids(fn):
    """True when fn names both `ray_ids` and `n_rays_total` as parameters (a
    bare **kwargs does not count: it may forward to something that does not
    take them)."""
    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        return False
    return "ray_ids" in params and "n_rays_total" in params


def render_sharded(render_fn, cam2world, intrinsics, x_pix, tile=64, group=None, pass_ray_ids=None):
    """render_fn(cam2world, intrinsics, x_pix[, ray_ids=, n_rays_total=]) ->
    (rgb_c, rgb_f, depth, depth) on this rank's tiles; returns the full-frame
    outputs on every rank. The frame-wide index of each of the rank's rays is
    passed as `ray_ids` (with `n_rays_total`) when pass_ray_ids is True, or,
    by default (None), when render_fn declares both parameters (a
    VolumeRenderer call: its Philox draws then match the single-GPU frame).
    cam2world (SB,R,4,4) may be a stride-0 expand; x_pix (SB,R,2)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    SB, R, _ = x_pix.shape
    dev = x_pix.device
    idx = ray_tiles(R, rank, world, tile, device=dev)
    c2w_local = cam2world if cam2world.shape[1] == 1 else cam2world[:, idx]
    if c2w_local.shape[1] == 1 and idx.numel() != 1:
        c2w_local = c2w_local.expand(SB, idx.numel(), 4, 4)
    if pass_ray_ids if pass_ray_ids is not None else _takes_ray_ids(render_fn):
        # frame-wide ray indices: the renderer's Philox draws then match the single-GPU render of the frame
        rgb_c, rgb_f, depth, _ = render_fn(c2w_local, intrinsics, x_pix[:, idx].contiguous(), ray_ids=idx,
                                           n_rays_total=R)
    else:
        rgb_c, rgb_f, depth, _ = render_fn(c2w_local, intrinsics, x_pix[:, idx].contiguous())
    n_loc = idx.numel()
    cap = max_local_rays(R, world, tile)
    packed = torch.zeros(SB, cap, 7, device=dev, dtype=torch.float32)
    packed[:, :n_loc, 0:3] = rgb_c
    packed[:, :n_loc, 3:6] = rgb_f
    packed[:, :n_loc, 6] = depth
    out = torch.empty(world * SB, cap, 7, device=dev, dtype=torch.float32)
    dist.all_gather_into_tensor(out, packed, group=group)
    out = out.view(world, SB, cap, 7)
    full = torch.empty(SB, R, 7, device=dev, dtype=torch.float32)
    for r in range(world):
        ridx = ray_tiles(R, r, world, tile, device=dev)
        full[:, ridx] = out[r, :, :ridx.numel()]
    depth_full = full[..., 6].contiguous()
    return full[..., 0:3].contiguous(), full[..., 3:6].contiguous(), depth_full, depth_full
