"""Isolated timing of avr_sample_fine at the C3 shape (65536 rays, 128 coarse
-> 64 importance, sorted 192): synthetic composite weights (peaked, like a
surface) and stratified coarse z. Prints us per call and the algorithmic
HBM rate. Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adaptive-volume-rendering_amd"))


def main():
    from avr import ops
    dev = torch.device("cuda:0")
    R, Nc, Nf = int(os.environ.get("FINE_R", 65536)), 128, 64
    reps = int(os.environ.get("FINE_REPS", 50))
    g = torch.Generator(device="cpu").manual_seed(0)
    near, far = 0.8, 1.8
    zc = near + (far - near) * (torch.arange(Nc) + torch.rand(R, Nc, generator=g)) / Nc
    centre = torch.rand(R, 1, generator=g) * Nc
    w = torch.exp(-0.5 * ((torch.arange(Nc) - centre) / 3.0) ** 2) * torch.rand(R, 1, generator=g)
    zc, w = zc.to(dev), w.to(dev)
    ops.sample_fine(w, zc, near, far, Nf, 0, 0.0, seed=1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        ops.sample_fine(w, zc, near, far, Nf, 0, 0.0, seed=1 + i)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = R * (2 * Nc + (Nc + Nf)) * 4
    print(f"R={R} sample_fine {us:.2f} us/call, {nbytes / us / 1e3:.1f} GB/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
