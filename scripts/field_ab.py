"""Diagnostic: field launch time on the bench's C3 fine pass (65 536 rays x 192
sorted samples), for A/B runs of kernel variants on one box. Not part of the
product or the bench.

env: AVR_LIB_PATH  library to load (default: the in-tree build)
     AVR_DEBUG     diagnostic flags for -DAVR_STAMPS builds (avr_debug_set_flags)
     REPS          timed launches (default 12)
prints one line: tag, median / min ms per launch, TF/s fp32-equivalent
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
sys.path.insert(0, REPO)
import avr._lib as L  # noqa: E402

lib = L.load()
if os.environ.get("AVR_DEBUG"):
    lib.avr_debug_set_flags.argtypes = [ctypes.c_int]
    lib.avr_debug_set_flags(int(os.environ["AVR_DEBUG"]))
import bench  # noqa: E402
from avr import ops  # noqa: E402

dev = torch.device("cuda:0")
net = bench.build_scene(dev)
net.field_precision = os.environ.get("PREC", "x3")
f = net.fused()
R, N = 65536, 192
K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]], device=dev)
c2w = bench.orbit_c2w(0.7).to(dev).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
x_pix = torch.rand(1, R, 2, generator=torch.Generator().manual_seed(100)).to(dev)
ro, rd, _ = ops.world_rays(x_pix, K, c2w)
ro, rd = ro[0].contiguous(), rd[0].contiguous()
z = torch.sort(0.8 + torch.rand(R, N, device=dev, generator=torch.Generator(device=dev).manual_seed(3)), -1)[0]
reps = int(os.environ.get("REPS", "12"))
times = []
with torch.no_grad():
    out = f.forward_rays(ro, rd, z, False)
    torch.cuda.synchronize()
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f.forward_rays(ro, rd, z, False)
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
times.sort()
med = times[len(times) // 2]
tf = R * N * bench.field_flops_per_sample() / (med * 1e-3) / 1e12
tag = os.environ.get("TAG", os.path.basename(os.environ.get("AVR_LIB_PATH", "default")))
print(f"[{tag}] debug={os.environ.get('AVR_DEBUG', '-')} median {med:.3f} ms min {times[0]:.3f} ms  {tf:.1f} TF/s "
      f"checksum {float(out.double().sum()):.6e}", flush=True)
