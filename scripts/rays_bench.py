"""Isolated timing of avr_rays_sample_coarse at the C3 shape (65536 rays x 128,
one pose expanded per ray as in the bench): with and without the fp64 depth
rows, and avr_sample_coarse alone (z only), and a plain fill of the z bytes (the store floor). Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adaptive-volume-rendering_amd"))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from avr import ops
    dev = torch.device("cuda:0")
    R, N, reps = 65536, 128, int(os.environ.get("RAYS_REPS", 50))
    x_pix = torch.rand(1, R, 2, device=dev) * 64
    K = torch.tensor([[[60.0, 0, 32], [0, 60.0, 32], [0, 0, 1]]], device=dev)
    c2w = torch.eye(4, device=dev)
    c2w[2, 3] = 1.3
    c2w = c2w.reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    for drow in (True, False):
        us = timed(lambda: ops.rays_sample_coarse(x_pix, K, c2w, 0.8, 1.8, N, seed=3, want_depth_row=drow), reps)
        print(f"rays_sample_coarse depth_row={drow}: {us:.2f} us", flush=True)
    us = timed(lambda: ops.sample_coarse(0.8, 1.8, R, N, dev, seed=3), reps)
    print(f"sample_coarse (z only): {us:.2f} us", flush=True)
    zbuf = torch.empty(R * N, device=dev)
    us = timed(lambda: ops.stream_fill(zbuf, 0), reps)
    print(f"stream_fill of the z bytes: {us:.2f} us", flush=True)


if __name__ == "__main__":
    main()
