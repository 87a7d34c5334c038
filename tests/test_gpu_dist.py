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
