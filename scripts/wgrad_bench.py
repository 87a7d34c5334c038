"""Isolated timing of avr_weight_grads on a training step's layer list: WG_CONF=default (the fine pass of
conf/default.conf: 9 hidden 512 x 512 layers) or default_mv (train.py's conf/default_mv.conf: 13), plus lin_in
(512 x 44) and lin_out (4 x 512), M = 4 scenes x 512 rays x 96 samples. WG_SPLITS="a,b,..." times explicit K-splits
beside the library's own choice; WG_THIN=0 leaves out lin_in / lin_out; WG_XF=ident|bn|relu adds the staging's
BatchNorm-relu (or relu-only) transform to the hidden layers. Prints ms per call and TFLOP/s (fp32-equivalent). Diagnostic only."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adaptive-volume-rendering_amd"))


def main():
    from avr import ops
    dev = torch.device("cuda:0")
    M = int(os.environ.get("WG_M", 196608))
    reps = int(os.environ.get("WG_REPS", 5))
    n_hidden = {"default": 9, "default_mv": 13}[os.environ.get("WG_CONF", "default")]
    g = torch.Generator(device="cpu").manual_seed(0)
    Gs = [torch.randn(M, 512, generator=g).to(dev) * 1e-3 for _ in range(7)]
    Xs = [torch.relu(torch.randn(M, 512, generator=g)).to(dev) for _ in range(8)]
    zf = torch.randn(M, 44, generator=g).to(dev)
    d4 = torch.randn(M, 4, generator=g).to(dev)
    mb = ops._max_bits
    # WG_XF=ident / bn: the hidden layers' X rebuilt in the staging as relu((x - mu) * scale + shift) (identity
    # statistics as avr.layer_train passes them, or BatchNorm-like ones as avr.bn_train)
    xf = os.environ.get("WG_XF", "none")
    if xf == "ident":
        tf = (torch.zeros(512, device=dev), torch.ones(512, device=dev), torch.zeros(512, device=dev))
    elif xf == "relu":
        tf = "relu"
    elif xf == "bn":
        tf = ((torch.rand(512, generator=g) * 0.2).to(dev), (torch.rand(512, generator=g) + 0.5).to(dev),
              (torch.randn(512, generator=g) * 0.1).to(dev))
    layers = [(Gs[i % 7], Xs[i % 8], mb(Gs[i % 7]), mb(Xs[i % 8]), i < 6) + ((tf,) if xf != "none" else ())
              for i in range(n_hidden)]
    thin = os.environ.get("WG_THIN", "1") == "1"   # WG_THIN=0: without lin_in / lin_out (their tiles' cost)
    if thin:
        layers += [(Gs[6], zf, mb(Gs[6]), mb(zf), True), (d4, Xs[7], mb(d4), mb(Xs[7]), True)]
    flops = 2.0 * M * (n_hidden * 512 * 512 + (512 * 44 + 4 * 512 if thin else 0))
    splits = [None] + [int(x) for x in os.environ.get("WG_SPLITS", "").split(",") if x]
    for n in splits:
        ops.weight_grads(layers, M, n_split=n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ops.weight_grads(layers, M, n_split=n)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"M={M} hidden={n_hidden} thin={int(thin)} xf={xf} n_split={n or 'auto'} weight_grads {dt * 1e3:.3f} ms/call (incl. partial sums) "
              f"{flops / dt / 1e12:.1f} TFLOP/s fp32-eq", flush=True)


if __name__ == "__main__":
    main()
