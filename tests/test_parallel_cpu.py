"""World-size-2 (and 3) gloo tests of the ray-sharding + gather path on CPU.
The per-rank renderer is a deterministic stand-in (the HIP renderer needs a
GPU); what is tested is tile ownership, the collective and frame assembly."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_render(c2w, K, x_pix):
    # per-ray function of its own inputs only (rays are independent)
    rgb_c = torch.stack([x_pix[..., 0], x_pix[..., 1], x_pix.sum(-1)], -1)
    rgb_f = rgb_c * 2 + c2w[..., 0, 3:4]
    depth = x_pix[..., 0] * 10 + K[:, 0, 0, None]
    return rgb_c, rgb_f, depth, depth


def _worker(rank, world, port, R, tile, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from avr.parallel import render_sharded
        g = torch.Generator().manual_seed(0)
        x_pix = torch.rand(2, R, 2, generator=g)
        K = torch.eye(3).expand(2, 3, 3).clone()
        c2w = torch.eye(4).reshape(1, 1, 4, 4).expand(2, R, 4, 4)
        rgb_c, rgb_f, depth, depth2 = render_sharded(fake_render, c2w, K, x_pix, tile=tile)
        ref = fake_render(c2w, K, x_pix)
        ok = torch.equal(rgb_c, ref[0]) and torch.equal(rgb_f, ref[1]) and torch.equal(depth, ref[2])
        q.put((rank, ok, ""))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- report instead of hanging the peer
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("world,R,tile", [(2, 1000, 64), (3, 777, 64), (2, 50, 64)])
def test_render_sharded_gloo(world, R, tile):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, R, tile, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=90) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert all(ok for _, ok, _ in res), res


def test_ray_tiles_partition():
    from avr.parallel import max_local_rays, ray_tiles
    for R, world in ((1000, 2), (777, 3), (65536, 8), (10, 4)):
        parts = [ray_tiles(R, r, world) for r in range(world)]
        allidx = torch.cat(parts).sort()[0]
        assert torch.equal(allidx, torch.arange(R))
        assert max(p.numel() for p in parts) <= max_local_rays(R, world)
