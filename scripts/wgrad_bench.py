"""Isolated timing of avr_weight_grads on the training step's fine-pass layer
list (M = 4 scenes x 512 rays x 96 samples): 9 hidden 512 x 512 layers,
lin_in (512 x 44) and lin_out (4 x 512). Prints ms per call and TFLOP/s
(fp32-equivalent). Diagnostic only."""
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
    g = torch.Generator(device="cpu").manual_seed(0)
    Gs = [torch.randn(M, 512, generator=g).to(dev) * 1e-3 for _ in range(7)]
    Xs = [torch.relu(torch.randn(M, 512, generator=g)).to(dev) for _ in range(8)]
    zf = torch.randn(M, 44, generator=g).to(dev)
    d4 = torch.randn(M, 4, generator=g).to(dev)
    mb = ops._max_bits
    layers = [(Gs[i % 7], Xs[i % 8], mb(Gs[i % 7]), mb(Xs[i % 8]), i < 6) for i in range(9)]
    layers += [(Gs[6], zf, mb(Gs[6]), mb(zf), True), (d4, Xs[7], mb(d4), mb(Xs[7]), True)]
    flops = 2.0 * M * (9 * 512 * 512 + 512 * 44 + 4 * 512)
    ops.weight_grads(layers, M)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ops.weight_grads(layers, M)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"M={M} weight_grads {dt * 1e3:.3f} ms/call (incl. partial sums) {flops / dt / 1e12:.1f} TFLOP/s fp32-eq",
          flush=True)


if __name__ == "__main__":
    main()
