"""Diagnostic: per-phase clock breakdown of field_x3_kernel (wave 0 of every
workgroup) from the -DAVR_STAMPS build. Not part of the product or the bench."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
sys.path.insert(0, REPO)
import avr._lib as L  # noqa: E402

L.LIB_PATH = os.environ.get("STAMPS_LIB") or os.path.join(REPO, "adaptive-volume-rendering_amd", "build", "libavr_hip_stamps.so")
lib = L.load(L.LIB_PATH)
lib.avr_debug_set_stamps.argtypes = [ctypes.c_void_p]
lib.avr_debug_set_flags.argtypes = [ctypes.c_int]
lib.avr_debug_set_flags(int(os.environ.get('AVR_DEBUG', '0')))
import bench  # noqa: E402

dev = torch.device("cuda:0")
net = bench.build_scene(dev)
net.field_precision = os.environ.get("PREC", "x3")
f = net.fused()
R, N = 65536, 192
# the bench's rays (config 3: orbit pose 0.7, normalized intrinsics, x_pix ~ U[0,1)^2)
from avr import ops  # noqa: E402
K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]], device=dev)
c2w = bench.orbit_c2w(0.7).to(dev).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
x_pix = torch.rand(1, R, 2, generator=torch.Generator().manual_seed(100)).to(dev)
ro, rd, _ = ops.world_rays(x_pix, K, c2w)
ro, rd = ro[0].contiguous(), rd[0].contiguous()
z = torch.sort(0.8 + torch.rand(R, N, device=dev), -1)[0]
blocks = (R * N + 63) // 64
stamps = torch.zeros(blocks * 64, dtype=torch.int64, device=dev)
with torch.no_grad():
    f.forward_rays(ro, rd, z, False)
    torch.cuda.synchronize()
    lib.avr_debug_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
    t0.record(); f.forward_rays(ro, rd, z, False); t1.record()
    torch.cuda.synchronize()
    lib.avr_debug_set_stamps(None)
st_all = stamps.view(blocks, 2, 32).cpu().numpy().astype(np.int64)
st = st_all[:, 0]
w4 = st_all[:, 1]
have4 = (w4[:, 0] != 0).mean() > 0.99
names = {0: "start", 27: "sample_geom", 28: "dedup texels", 1: "PE sines", 2: "publish X0", 3: "lin_in init",
         4: "lin_in gemm"}
for b in range(4):
    if b == 3:
        continue
    names.update({5 + 5 * b: f"b{b} lin_z interp", 6 + 5 * b: f"b{b} prep+publish h", 7 + 5 * b: f"b{b} fc0 gemm",
                  8 + 5 * b: f"b{b} prep+publish t", 9 + 5 * b: f"b{b} fc1 init+gemm"})
names.update({25: "lin_out prep+publish", 26: "lin_out gemm", 29: "b2 stage issue", 30: "b2 stage wait",
              20: "b1 t max pass", 21: "b1 bias/prefetch issue"})
used = [k for k in names if (st[:, k] != 0).mean() > 0.99]
used.sort(key=lambda k: np.median(st[:, k] - st[:, 0]))
print(f"kernel {t0.elapsed_time(t1):.2f} ms for {R * N} samples, {blocks} blocks")
tot = np.median(st[:, used[-1]] - st[:, 0])
prev = used[0]
print(f"{'phase':28s} {'wave0':>10s}        {'end(w0)':>9s} {'end(w4)':>9s}")
for k in used[1:]:
    d = np.median(st[:, k] - st[:, prev])
    e0 = np.median(st[:, k] - st[:, 0])
    e4 = np.median(w4[:, k] - st[:, 0]) if have4 else float("nan")
    print(f"{names[k]:28s} {d:10.0f} cyc  {100 * d / tot:5.1f} % {e0:9.0f} {e4:9.0f}")
    prev = k
print(f"{'total (median per block)':28s} {tot:10.0f} cyc")
span = (st[:, used[-1]].max() - st[:, 0].min())
print("blocks per CU (approx)", blocks / 256, "span cycles", span)
dd = st_all[:, 0, 31]
if (dd > 0).mean() > 0.99:
    q = np.percentile(dd, [0, 10, 50, 90, 99, 100])
    print("distinct texels per workgroup D: min/p10/p50/p90/p99/max " + " ".join(f"{x:.0f}" for x in q)
          + f"; D > 64: {100 * (dd > 64).mean():.2f} % of workgroups")
