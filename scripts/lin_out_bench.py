"""Diagnostic: avr_lin_out_fwd_rows / avr_lin_out_bwd_rows timed alone at the layer paths' row counts (d_hidden
512), one vs two rows per lane group per pass (AVR_LIN_OUT_RR, read per call): us per call and the algorithmic
bytes' rate (forward: the rows read; backward: rows read + gradient rows written). usage: python scripts/lin_out_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adaptive-volume-rendering_amd"))


def timed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(n):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / n * 1e3


def main():
    from avr import ops
    dev = torch.device("cuda:0")
    H = 512
    g = torch.Generator().manual_seed(0)
    W = (torch.randn(4, H, generator=g) * 0.05).to(dev)
    b = torch.randn(4, generator=g).to(dev)
    for M in (131072, 98304):
        x = torch.randn(M, H, generator=g).to(dev)
        go = torch.randn(M, 4, generator=g).to(dev)
        out, _ = ops.lin_out_rows(x, W, b)
        for rr in ("1", "2"):
            os.environ["AVR_LIN_OUT_RR"] = rr
            f = timed(lambda: ops.lin_out_rows(x, W, b))
            bw = timed(lambda: ops.lin_out_rows_bwd(go, out, W, x))
            nb = M * H * 4
            print(f"M={M} RR={rr}: fwd {f:7.1f} us ({nb / f / 1e3:6.0f} GB/s)  bwd {bw:7.1f} us "
                  f"({2 * nb / bw / 1e3:6.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
