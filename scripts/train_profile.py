"""Diagnostic: torch.profiler over bench.py's --mode train step (HIP path), the aten ops by CUDA time with
their input shapes and the Python call sites of the copies / cats / fills (what the kernel list calls
direct_copy, CatArrayBatchedCopy, FillFunctor). Not part of the product or the bench.

env: CONF (default_mv | default), STEPS, BN (1: train.py --bn), RENDERER (volume | adaptive: AdaptiveVolumeRenderer, train.py:268-273),
CPUSORT=1 (also the ops by host time)
"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from avr.conf import default_conf  # noqa: E402
from avr.renderers import AdaptiveVolumeRenderer, VolumeRenderer  # noqa: E402

dev = torch.device("cuda:0")
SB, R = 4, 512
net = bench.build_scene(dev, conf=os.environ.get("CONF", "default_mv"), bn=os.environ.get("BN", "0") == "1")
g = torch.Generator(device="cpu").manual_seed(7)
net.encoder.set_latent(torch.randn(SB, net.d_latent, 64, 64, generator=g).to(dev))
net.num_objs = SB
net.poses = net.poses.repeat(SB, 1, 1)
net.poses[:, 0, 3] += 0.05 * torch.arange(SB, device=dev, dtype=torch.float32)
net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
net.train()
for p in net.parameters():
    p.requires_grad_(True)
params = list(net.parameters())
if os.environ.get("RENDERER", "volume") == "adaptive":
    torch.manual_seed(11)
    rend = AdaptiveVolumeRenderer.from_conf(default_conf()["adaptive_renderer"]).to(dev)
    params += list(rend.parameters())
else:
    rend = VolumeRenderer.from_conf(default_conf()["normal_renderer"]).to(dev)
    rend.seed = 99
x_pix = torch.rand(SB, R, 2, generator=g).to(dev)
c2w = torch.stack([bench.orbit_c2w(0.3 + 0.9 * b) for b in range(SB)]).to(dev).reshape(SB, 1, 4, 4).expand(SB, R, 4, 4)
K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]] * SB, device=dev)
gt = torch.rand(SB, R, 3, generator=g).to(dev)
opt = torch.optim.Adam(params, lr=1e-4)
net.hip_backward = True


def step():
    rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
    loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
    opt.zero_grad()
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
steps = int(os.environ.get("STEPS", "3"))
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=45,
                                                         max_name_column_width=40, max_shapes_column_width=70))
if os.environ.get("CPUSORT") == "1":   # host time: what keeps the GPU waiting between launches
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40, max_name_column_width=60))
    print(prof.key_averages(group_by_stack_n=4).table(sort_by="cpu_time_total", row_limit=30,
                                                      max_name_column_width=40, max_src_column_width=120))
for name in ("aten::copy_", "aten::cat", "aten::fill_", "aten::zero_", "aten::abs", "aten::amax", "aten::max"):
    print(f"==== {name} by stack")
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_device_time_total", row_limit=8,
                                                      max_name_column_width=30, max_src_column_width=160)
          if False else "")
    rows = [e for e in prof.key_averages(group_by_stack_n=6) if e.key == name]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:8]:
        print(f"  {e.self_device_time_total / steps:9.1f} us/step  calls {e.count / steps:5.1f}")
        for fr in e.stack[:6]:
            print(f"      {fr}")
