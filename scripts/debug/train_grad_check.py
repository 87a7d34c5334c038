"""Diagnostic: per-parameter gradient error of the HIP training path and of
PyTorch fp32 autograd against a float64 autograd reference (test_gpu_train's
512-wide case)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-volume-rendering_amd"), os.path.join(REPO, "tests")]
import test_gpu_train as T  # noqa: E402

net = T._net(512, 3, 512, (16, 16), 1000)
xyz, vd, w = T._points(1, 1000)
_, g_h, _ = T._grads(net, xyz, vd, w, True, hip=True)
_, g_t, _ = T._grads(net, xyz, vd, w, True, hip=False)
net64 = net.double()
net64.encoder.latent = net64.encoder.latent.double()
net64.poses, net64.focal, net64.c = net64.poses.double(), net64.focal.double(), net64.c.double()
net64.image_shape = net64.image_shape.double()
net64.encoder.latent_scaling = net64.encoder.latent_scaling.double()
net64.use_fused = False
_, g_d, _ = T._grads(net64, xyz.double(), vd.double(), w.double(), True, hip=False)
for k in sorted(g_d):
    ref = g_d[k]
    s = float(ref.abs().max())
    eh = float((g_h[k].double() - ref).abs().max())
    et = float((g_t[k].double() - ref).abs().max())
    print(f"{k:28s} max|g| {s:9.3e}  hip err {eh / s:9.2e}  torch32 err {et / s:9.2e}")
