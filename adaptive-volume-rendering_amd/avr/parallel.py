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
import time

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


_DTYPES = [torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.uint8,
           torch.bool]
_MAX_DIMS = 6


def _scene_tensors(net):
    """(owner module, attribute name, tensor, qualified name) of every parameter and buffer of `net`, in
    module order (the same on every rank for one architecture)."""
    out = []
    for mname, mod in net.named_modules():
        for name, t in list(mod.named_parameters(recurse=False)) + list(mod.named_buffers(recurse=False)):
            if t is not None:
                out.append((mod, name, t, f"{mname}.{name}" if mname else name))
    return out


def broadcast_scene(net, src=0, group=None):
    """Make every rank's `net` equal to rank `src`'s: all parameters and buffers -- the field weights, the
    latent map (encoder.latent, latent_scaling) and the source view (poses, focal, c, image_shape) -- in one
    collective per dtype (once per scene, ~27 MB at default.conf; the reference is single-process,
    train.py:238-240, so this replaces nothing there).

    Receiving ranks copy the values in with in-place `copy_` under no_grad, so every tensor's version counter
    advances: the caches keyed by (data_ptr, _version) -- FusedField's packed weights, lin_z tables and view
    descriptors, GraphedRenderer's capture check -- rebuild on the next render instead of serving the weights
    the rank had before (a c10d collective writing into the tensors does not advance it). A buffer whose shape
    differs from src's (another latent resolution, more source views) is replaced by a tensor of src's shape;
    a parameter shape mismatch (another architecture) raises on every rank. The net's FusedField, if any, is
    also invalidated explicitly. Returns the number of bytes broadcast."""
    is_src = dist.get_rank() == src            # src is a global rank, as in dist.broadcast
    entries = _scene_tensors(net)
    dev = entries[0][2].device
    comm_dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else dev

    def any_rank(flag):      # every rank takes the same branch (no rank left waiting in a collective)
        f = torch.tensor([int(flag)], dtype=torch.int64, device=comm_dev)
        dist.all_reduce(f, group=group)
        return bool(f.item())

    # header: per tensor [dtype, ndim, shape...]: the receivers check the architecture and resize buffers
    head = torch.zeros(len(entries), 2 + _MAX_DIMS, dtype=torch.int64)
    for i, (_, _, t, full) in enumerate(entries):
        if t.dim() > _MAX_DIMS or t.dtype not in _DTYPES:
            raise ValueError(f"broadcast_scene: unsupported tensor {full} {t.dtype} {tuple(t.shape)}")
        head[i, 0], head[i, 1] = _DTYPES.index(t.dtype), t.dim()
        head[i, 2:2 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
    n = torch.tensor([len(entries)], dtype=torch.int64, device=comm_dev)
    dist.broadcast(n, src, group=group)
    if any_rank(int(n.item()) != len(entries)):
        raise ValueError("broadcast_scene: the ranks' nets hold different numbers of parameters / buffers")
    src_head = head.to(comm_dev)
    dist.broadcast(src_head, src, group=group)
    src_head = src_head.cpu()
    mismatch = any(not torch.equal(src_head[i], head[i]) and (isinstance(t, torch.nn.Parameter)
                                                             or int(src_head[i, 0]) != int(head[i, 0]))
                   for i, (_, _, t, _) in enumerate(entries))
    if any_rank(mismatch):
        raise ValueError("broadcast_scene: the ranks' nets differ in architecture (a parameter's shape or a dtype)")
    if not is_src:
        for i, (mod, name, t, full) in enumerate(entries):
            shape = tuple(int(s) for s in src_head[i, 2:2 + int(src_head[i, 1])])
            if tuple(t.shape) != shape:     # a buffer of another shape: replaced by one of src's
                t = torch.empty(shape, dtype=t.dtype, device=dev)
                setattr(mod, name, t)
                entries[i] = (mod, name, t, full)
    total = 0
    with torch.no_grad():
        for dtype in _DTYPES:
            group_ts = [t for _, _, t, _ in entries if t.dtype == dtype]
            if not group_ts:
                continue
            flat = torch.cat([t.detach().reshape(-1) for t in group_ts]).to(comm_dev) if is_src else \
                torch.empty(sum(t.numel() for t in group_ts), dtype=dtype, device=comm_dev)
            dist.broadcast(flat, src, group=group)
            total += flat.numel() * flat.element_size()
            if not is_src:
                off = 0
                for t in group_ts:
                    t.copy_(flat[off:off + t.numel()].view(t.shape))   # in place: advances t._version
                    off += t.numel()
    fused = getattr(net, "_fused", None)
    if fused is not None and not is_src:
        fused.invalidate()
    return total


def _takes_ray_ids(fn):
    """True when fn names both `ray_ids` and `n_rays_total` as parameters (a
    bare **kwargs does not count: it may forward to something that does not
    take them)."""
    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        return False
    return "ray_ids" in params and "n_rays_total" in params


class ShardTimer:
    """Per-phase time of render_sharded calls on this rank, summed over the calls since reset(): `render` (the
    rank's renderer call on its tiles, including the tile gather of its inputs), `all_gather` (the collective,
    including the wait for the slowest rank) and `reassembly` (packing the local outputs plus scattering every
    rank's tiles into the frame). HIP events on the current stream on a GPU (no synchronisation inside the
    step), wall clock on the CPU (gloo is synchronous). bench.py reports them per step, min / max over ranks,
    so a 1 -> N shortfall can be attributed."""
    PHASES = ("render", "all_gather", "reassembly")

    def __init__(self):
        self.calls = []
        self._dev = None

    def reset(self):
        self.calls = []

    def _mark(self):
        if self._dev.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def begin(self, dev):
        self._dev = dev
        self._last = self._mark()
        self.calls.append({p: [] for p in self.PHASES})

    def lap(self, phase):
        m = self._mark()
        self.calls[-1][phase].append((self._last, m))
        self._last = m

    def totals_ms(self):
        """{phase: ms summed over the calls} (synchronises the device)."""
        out = {p: 0.0 for p in self.PHASES}
        if self._dev is not None and self._dev.type == "cuda":
            torch.cuda.synchronize(self._dev)
        for call in self.calls:
            for p, pairs in call.items():
                for a, b in pairs:
                    out[p] += a.elapsed_time(b) if isinstance(a, torch.cuda.Event) else (b - a) * 1e3
        return out


def render_sharded(render_fn, cam2world, intrinsics, x_pix, tile=64, group=None, pass_ray_ids=None, timer=None):
    """render_fn(cam2world, intrinsics, x_pix[, ray_ids=, n_rays_total=]) ->
    (rgb_c, rgb_f, depth, depth) on this rank's tiles; returns the full-frame
    outputs on every rank. The frame-wide index of each of the rank's rays is
    passed as `ray_ids` (with `n_rays_total`) when pass_ray_ids is True, or,
    by default (None), when render_fn declares both parameters (a
    VolumeRenderer call: its Philox draws then match the single-GPU frame).
    cam2world (SB,R,4,4) may be a stride-0 expand; x_pix (SB,R,2).
    timer: a ShardTimer that records the call's render / all_gather / reassembly phases."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    SB, R, _ = x_pix.shape
    dev = x_pix.device
    if timer is not None:
        timer.begin(dev)
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
    if timer is not None:
        timer.lap("render")
    n_loc = idx.numel()
    cap = max_local_rays(R, world, tile)
    packed = torch.zeros(SB, cap, 7, device=dev, dtype=torch.float32)
    packed[:, :n_loc, 0:3] = rgb_c
    packed[:, :n_loc, 3:6] = rgb_f
    packed[:, :n_loc, 6] = depth
    out = torch.empty(world * SB, cap, 7, device=dev, dtype=torch.float32)
    if timer is not None:
        timer.lap("reassembly")
    if dist.get_backend(group) == "gloo" and dev.type != "cpu":   # gloo moves host memory (one-GPU rehearsals)
        out_h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(out_h, packed.cpu(), group=group)
        out.copy_(out_h)
    else:
        dist.all_gather_into_tensor(out, packed, group=group)
    if timer is not None:
        timer.lap("all_gather")
    out = out.view(world, SB, cap, 7)
    full = torch.empty(SB, R, 7, device=dev, dtype=torch.float32)
    for r in range(world):
        ridx = ray_tiles(R, r, world, tile, device=dev)
        full[:, ridx] = out[r, :, :ridx.numel()]
    depth_full = full[..., 6].contiguous()
    res = full[..., 0:3].contiguous(), full[..., 3:6].contiguous(), depth_full, depth_full
    if timer is not None:
        timer.lap("reassembly")
    return res


def gather_bytes(n_rays, world, sb=1, tile=64):
    """Bytes one render_sharded all_gather moves into each rank: world x SB x (max tiles per rank x tile) x 28."""
    return world * sb * max_local_rays(n_rays, world, tile) * 7 * 4


def phase_spread(timer, steps, device, group=None):
    """Every rank's ShardTimer totals per step -> {phase: {"min": ms, "max": ms, "per_rank": [...]}} on every
    rank (one small all_gather; on the CPU tensor for gloo)."""
    tot = timer.totals_ms()
    comm = torch.device("cpu") if dist.get_backend(group) == "gloo" else device
    mine = torch.tensor([tot[p] / max(steps, 1) for p in ShardTimer.PHASES], dtype=torch.float64, device=comm)
    world = dist.get_world_size(group)
    allr = torch.empty(world * mine.numel(), dtype=torch.float64, device=comm)
    dist.all_gather_into_tensor(allr, mine, group=group)
    allr = allr.cpu().reshape(world, mine.numel())
    return {p: {"min": round(float(allr[:, i].min()), 3), "max": round(float(allr[:, i].max()), 3),
                "per_rank": [round(float(v), 3) for v in allr[:, i]]} for i, p in enumerate(ShardTimer.PHASES)}
