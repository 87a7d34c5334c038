"""Diagnostic: STEPS train.py steps of bench.py's --mode train workload on the HIP path, printing the step
time and the allocator's memory every 50 steps (caches must not grow; the loss must stay finite)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from avr.conf import default_conf  # noqa: E402
from avr.renderers import VolumeRenderer  # noqa: E402

dev = torch.device("cuda:0")
SB, R = 4, 512
net = bench.build_scene(dev, conf=os.environ.get("CONF", "default_mv"))
g = torch.Generator(device="cpu").manual_seed(7)
net.encoder.set_latent(torch.randn(SB, net.d_latent, 64, 64, generator=g).to(dev))
net.num_objs = SB
net.poses = net.poses.repeat(SB, 1, 1)
net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
net.train()
for p in net.parameters():
    p.requires_grad_(True)
rend = VolumeRenderer.from_conf(default_conf()["normal_renderer"]).to(dev)
rend.seed = 99
K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]] * SB, device=dev)
opt = torch.optim.Adam(net.parameters(), lr=1e-4)
net.hip_backward = True
steps = int(os.environ.get("STEPS", "400"))
t0 = time.perf_counter()
for i in range(1, steps + 1):
    x_pix = torch.rand(SB, R, 2, generator=g).to(dev)            # fresh rays every step, as train.py
    c2w = torch.stack([bench.orbit_c2w(0.3 + 0.9 * b + 0.01 * i) for b in range(SB)]).to(dev)
    c2w = c2w.reshape(SB, 1, 4, 4).expand(SB, R, 4, 4)
    gt = torch.rand(SB, R, 3, generator=g).to(dev)
    rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
    loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
    opt.zero_grad()
    loss.backward()
    opt.step()
    if i % 50 == 0:
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 50
        t0 = time.perf_counter()
        print(f"step {i}: loss {float(loss):.5f}  {dt * 1e3:.2f} ms/step (incl. host ray setup)  allocated "
              f"{torch.cuda.memory_allocated() / 2**20:.0f} MiB  reserved {torch.cuda.memory_reserved() / 2**20:.0f} MiB",
              flush=True)
        assert torch.isfinite(loss)
