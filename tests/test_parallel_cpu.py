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


def _bcast_worker(rank, world, port, q, mismatch):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from avr.conf import default_conf
        from avr.parallel import broadcast_scene
        from avr.scene import synthetic_scene
        cpu = torch.device("cpu")
        if mismatch and rank == 1:    # another architecture (default_mv: 5 blocks) must raise on every rank
            net = synthetic_scene(cpu, 7, default_conf(multiview=True)["model"])
        else:
            # rank 1: other weights, another latent (other resolution) and another source pose than rank 0
            net = synthetic_scene(cpu, 0 if rank == 0 else 7, latent_hw=(64, 64) if rank == 0 else (32, 48))
            if rank == 1:
                net.poses[0, 2, 3] = 2.0
        fused = net.fused()
        view_before = fused.view(0)            # rank 1 caches its own scene's view descriptor first
        params = list(net.mlp_coarse.parameters())
        key_before = [(p.data_ptr(), p._version) for p in params]
        fused._packed[True] = (("stale",), None)   # stands in for a packed blob of rank 1's weights
        try:
            nbytes = broadcast_scene(net, src=0)
        except ValueError as e:
            q.put((rank, mismatch and "architecture" in str(e) or "numbers" in str(e), repr(e)))
            dist.destroy_process_group()
            return
        key_after = [(p.data_ptr(), p._version) for p in params]
        checks = {"bytes": nbytes > 27e6}
        if rank == 1:
            checks["versions_advanced"] = all(a[1] > b[1] for a, b in zip(key_after, key_before))
            checks["caches_dropped"] = not fused._packed and fused.view(0) is not view_before
        else:
            checks["src_untouched"] = key_after == key_before and bool(fused._packed)
        checks["latent_shape"] = tuple(net.encoder.latent.shape) == (1, 512, 64, 64)
        checks["pose"] = abs(float(fused.view(0).poses[11]) - 1.3) < 1e-6
        # the field itself (module path on the CPU) gives rank 0's outputs on every rank
        g = torch.Generator().manual_seed(3)
        xyz = torch.rand(1, 64, 3, generator=g) * 0.6 - 0.3
        vd = torch.nn.functional.normalize(torch.rand(1, 64, 3, generator=g) - 0.5, dim=-1)
        with torch.no_grad():
            out = torch.cat([net(xyz, coarse=c, viewdirs=vd).reshape(-1) for c in (True, False)])
        outs = [torch.empty_like(out) for _ in range(world)]
        dist.all_gather(outs, out)
        checks["same_field"] = all(torch.equal(o, outs[0]) for o in outs)
        q.put((rank, all(checks.values()), str(checks)))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- report instead of hanging the peer
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("mismatch", [False, True])
def test_broadcast_scene_gloo(mismatch):
    """rank 1 starts from another scene (weights, latent of another size, source pose) and has
    cached its view descriptor and a packed blob; after broadcast_scene every tensor's version advanced, the
    caches are gone, and the field gives rank 0's outputs bit for bit. Another architecture raises on both."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q, mismatch)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert all(ok for _, ok, _ in res), res
