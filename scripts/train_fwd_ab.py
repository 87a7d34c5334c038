"""Diagnostic: the training forward (field_x3_kernel SAVE) against the inference
forward on the same points, at train.py's fine-pass shape (4 scenes x 512 rays x
96 samples) on the default_mv.conf field. Not part of the product or the bench.

env: AVR_LIB_PATH (library to load), CONF (default_mv | default), B (points per scene),
     REPS (timed launches per variant), VARIANTS (comma list of the tags to run)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402

dev = torch.device("cuda:0")
conf = os.environ.get("CONF", "default_mv")
net = bench.build_scene(dev, conf=conf)
SB, B = 4, int(os.environ.get("B", str(512 * 96)))
g = torch.Generator(device="cpu").manual_seed(1)
xyz = ((torch.rand(SB, B, 3, generator=g) - 0.5) * 0.8).to(dev)
vd = torch.nn.functional.normalize(torch.randn(SB, B, 3, generator=g), dim=-1).to(dev)
f = net.fused()
reps = int(os.environ.get("REPS", "10"))
m = net.mlp_fine
flops = SB * B * bench.field_flops_per_sample(d_hidden=m.d_hidden, n_blocks=m.n_blocks,
                                              n_lin_z=min(m.combine_layer, m.n_blocks))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def infer():
    with torch.no_grad():
        return f.forward_points(xyz, vd, False)


def train():
    with torch.no_grad():
        return f.forward_train(xyz, vd, False)


w = torch.randn(SB, B, 4, generator=g).to(dev)
for p_ in f._mlp(False).parameters():
    p_.requires_grad_(True)


def train_bwd():
    out = f.forward_train(xyz, vd, False)
    (out * w).sum().backward()


variants = [("infer8", infer, "8"), ("infer4", infer, "4"), ("train", train, "8"), ("train+bwd", train_bwd, "8")]
want = os.environ.get("VARIANTS")
for tag, fn, waves in variants:
    if want and tag not in want.split(","):
        continue
    os.environ["AVR_X3_WAVES"] = waves
    ms = timed(fn)
    print(f"[{tag}] {conf} SB={SB} B={B}: {ms:.3f} ms  {flops / (ms * 1e-3) / 1e12:.1f} TF/s", flush=True)
