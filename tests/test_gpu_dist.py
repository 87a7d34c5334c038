"""The multi-GPU code path on the MI355X itself, at world size 1 (SURVEY
§8e; the driver runs the N = 1..8 curve): an RCCL ("nccl") process group
bound to the device, avr.parallel.render_sharded dealing the frame's 64-ray
tiles and all_gather_into_tensor assembling (rgb_coarse, rgb_fine, depth) --
equal bit for bit to the non-distributed render of the same frame; and
bench.py's N > 1 step (config 5 through render_sharded) at one rank."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def nccl_world1():
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_render_sharded_over_rccl_equals_single_render(nccl_world1):
    from avr.parallel import render_sharded
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS, synthetic_scene
    from bench import frame_views
    dist = nccl_world1
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    net = synthetic_scene(DEV)
    x_pix, c2w = frame_views(4, 100, DEV)           # config 5's layout: 4 orbit views, a per-ray pose
    R = x_pix.shape[1]
    K = torch.tensor([INTRINSICS], device=DEV)

    def renderer():
        r = VolumeRenderer(0.8, 1.8, 128, 64, 0, 0.01, True)
        r.seed = 1234
        return r

    rend_a, rend_b = renderer(), renderer()
    with torch.no_grad():
        full = rend_a(c2w, K, x_pix, net)
        shard = render_sharded(lambda c, k, x, ray_ids=None, n_rays_total=None:
                               rend_b(c, k, x, net, ray_ids=ray_ids, n_rays_total=n_rays_total), c2w, K, x_pix)
    torch.cuda.synchronize()
    assert rend_b.last_path == "fused"
    for k in range(3):
        assert shard[k].shape == full[k].shape
        torch.testing.assert_close(shard[k], full[k], atol=0, rtol=0)
    # a raw all_gather of the packed 28 B/ray record, as bench.py's config-3 N > 1 step does
    local = torch.cat([full[0].reshape(-1), full[1].reshape(-1), full[2].reshape(-1)])
    out = torch.empty_like(local)
    dist.all_gather_into_tensor(out, local)
    torch.cuda.synchronize()
    assert torch.equal(out, local) and local.numel() == 7 * R


def test_bench_dist_path_at_one_rank():
    """bench.py --dist: init_process_group("nccl", device_id=...), render_sharded and the all_gather inside the
    timed step -- the exact N > 1 code -- on one GPU, launched by torch.distributed.run."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "1", "--dist",
           "--config", "5", "--frame", "160", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-pmc"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["scaling"] == "strong"
    assert "RCCL gather" in line["config"]["parallelism"]
    assert line["config"]["rays_per_gpu"] == 4 * 160 * 160 and line["value"] > 0
    # the N > 1 attribution every config-5 line with a process group carries: per-rank
    # shard phases, the scene broadcast, and every rank's field time (min / max over ranks)
    assert {"render_ms_per_step", "all_gather_ms_per_step", "reassembly_ms_per_step"} <= set(line["shard_phases"])
    assert "scene_broadcast" in line
    fr = line["field_ms_per_rank"]
    assert 0 < fr["min"] <= fr["max"] and fr["steps"] == 2 and fr["launches_per_rank"] > 0


def test_broadcast_scene_over_rccl_world1(nccl_world1):
    """broadcast_scene on the RCCL group (device tensors, one collective per dtype): at src the net is left
    as it was (no version bump, caches kept) and the render after it equals the render before it."""
    from avr.parallel import broadcast_scene
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS, synthetic_scene
    net = synthetic_scene(DEV)
    R = 512
    g = torch.Generator().manual_seed(5)
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    from bench import orbit_c2w
    c2w = orbit_c2w(0.3).to(DEV).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    K = torch.tensor([INTRINSICS], device=DEV)
    rend = VolumeRenderer(0.8, 1.8, 64, 32, 0, 0.01, True)
    with torch.no_grad():
        rend.seed, rend._offset = 9, 0
        before = rend(c2w, K, x_pix, net)
        key = net.fused()._packed[True][0]
        nbytes = broadcast_scene(net, src=0)
        rend.seed, rend._offset = 9, 0
        after = rend(c2w, K, x_pix, net)
    torch.cuda.synchronize()
    assert nbytes > 27e6 and rend.last_path == "fused"
    assert net.fused()._packed[True][0] == key        # src: nothing rewritten, nothing repacked
    for a, b in zip(before[:3], after[:3]):
        assert torch.equal(a, b)


def _bcast_gpu_worker(rank, port, q):
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-volume-rendering_amd")]
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        # two ranks on the one GPU of the box: RCCL needs one GPU per rank, so the group is gloo (broadcast_scene
        # stages the device tensors through the host) -- what is tested is the receivers' cache invalidation
        dist.init_process_group("gloo", rank=rank, world_size=2)
        import avr
        from avr.parallel import broadcast_scene
        from avr.renderers import VolumeRenderer
        from avr.scene import INTRINSICS, synthetic_scene
        from bench import orbit_c2w
        avr.load_library()
        net = synthetic_scene(dev, 0 if rank == 0 else 7, latent_hw=(64, 64) if rank == 0 else (32, 32))
        R = 640
        g = torch.Generator().manual_seed(5)
        x_pix = torch.rand(1, R, 2, generator=g).to(dev)
        c2w = orbit_c2w(0.3).to(dev).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
        K = torch.tensor([INTRINSICS], device=dev)
        rend = VolumeRenderer(0.8, 1.8, 64, 32, 0, 0.01, True)
        with torch.no_grad():
            rend.seed, rend._offset = 9, 0
            own = rend(c2w, K, x_pix, net)          # rank 1 renders its own scene first: caches built
            fused = net.fused()
            key0 = fused._packed[True][0]
            broadcast_scene(net, src=0)
            rend.seed, rend._offset = 9, 0
            shared = rend(c2w, K, x_pix, net)
            key1 = fused._packed[True][0]
        torch.cuda.synchronize()
        res = torch.cat([t.reshape(-1) for t in shared[:3]]).cpu()
        outs = [torch.empty_like(res) for _ in range(2)]
        dist.all_gather(outs, res)
        own_flat = torch.cat([t.reshape(-1) for t in own[:3]]).cpu()
        checks = {"fused": rend.last_path == "fused", "equal_to_rank0": torch.equal(outs[0], outs[1]),
                  "repacked": (key1 != key0) if rank == 1 else (key1 == key0),
                  "changed": (not torch.equal(own_flat, res)) if rank == 1 else torch.equal(own_flat, res)}
        q.put((rank, all(checks.values()), str(checks)))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- report instead of hanging the peer
        q.put((rank, False, repr(e)))


def test_broadcast_scene_two_ranks_repack():
    """SURVEY §8e on the GPU: rank 1 renders its own scene (other weights, a 32x32 latent), receives rank 0's
    with broadcast_scene, repacks its weights / rebuilds its tables on the next render, and renders rank 0's
    frame bit for bit; rank 0 keeps its caches."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_gpu_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert all(ok for _, ok, _ in res), res
