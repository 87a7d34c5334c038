"""Eager renderer call vs HIP-graph replay (avr.graphs.GraphedRenderer) for small ray batches: ms per frame
(median of REPS), the bench's synthetic scene, 128 coarse + 64 fine samples, Philox noise."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from avr.graphs import GraphedRenderer  # noqa: E402
from avr.renderers import VolumeRenderer  # noqa: E402

dev = torch.device("cuda:0")
net = bench.build_scene(dev)
K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]], device=dev)
reps = int(os.environ.get("REPS", "30"))


def timed(fn):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


for R in (256, 1024, 4096, 16384):
    rend = VolumeRenderer(0.8, 1.8, 128, 64, 0, 0.01, True)
    rend.seed = 5
    x_pix = torch.rand(1, R, 2, device=dev)
    c2w = bench.orbit_c2w(0.7).to(dev).reshape(1, 1, 4, 4).expand(1, R, 4, 4).contiguous()
    with torch.no_grad():
        eager = timed(lambda: rend(c2w, K, x_pix, net))
    gr = GraphedRenderer(rend, net, c2w, K, x_pix)
    graph = timed(lambda: gr(c2w, K, x_pix))
    print(f"R={R:6d}: eager {eager:7.3f} ms, graph replay {graph:7.3f} ms ({eager / graph:.2f}x)", flush=True)
