"""Diagnostic: the adaptive renderer's three library GEMMs around the LSTM march (renderers.py _MarchTrain: the
per-texel gate tables latent^T W_ih^T, W_ih's gradient d_tab^T latent, the latent's gradient d_tab W_ih) at
train.py's shapes (4 scenes, 512 x 64 x 64 latent, 64 gates), each timed as written and in alternative forms
(channels-last latent rows, the transposed product written in the latent's own layout, the x3 weight-gradient
kernel). Prints us per call. usage: python scripts/march_gemm_bench.py"""
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
    SB, C, H, W, G = 4, 512, 64, 64, 64
    T = H * W
    g = torch.Generator(device="cpu").manual_seed(0)
    lat = torch.randn(SB, C, H, W, generator=g).to(dev)
    w_ih = (torch.randn(G, C, generator=g) * 0.05).to(dev)
    d_tab = (torch.randn(SB, T, G, generator=g) * 1e-3).to(dev)
    lat_t = lat.reshape(SB, C, T)
    hwc = lat_t.transpose(1, 2).contiguous()                      # (SB, T, C) channels-last rows
    cases = {
        "tables: matmul(lat_t^T, w^T) [current]": lambda: torch.matmul(lat_t.transpose(1, 2), w_ih.t()).contiguous(),
        "tables: hwc rows @ w^T": lambda: torch.matmul(hwc.reshape(SB * T, C), w_ih.t()),
        "hwc: transpose copy of the latent": lambda: lat_t.transpose(1, 2).contiguous(),
        "d_wih: einsum sth,sct->hc [current]": lambda: torch.einsum("sth,sct->hc", d_tab, lat_t),
        "d_wih: mm(d_tab^T, hwc rows)": lambda: torch.mm(d_tab.reshape(SB * T, G).t(), hwc.reshape(SB * T, C)),
        "d_wih: bmm per scene + sum": lambda: torch.bmm(d_tab.transpose(1, 2), lat_t.transpose(1, 2)).sum(0),
        "d_wih: avr_weight_grads on hwc rows": lambda: ops.weight_grads(
            [(d_tab.reshape(SB * T, G), hwc.reshape(SB * T, C), ops._max_bits(d_tab), ops._max_bits(hwc), False)],
            SB * T),
        "d_lat: matmul(d_tab, w) + transpose [current]": lambda: torch.matmul(d_tab, w_ih).transpose(1, 2).contiguous(),
        "d_lat: matmul(w^T, d_tab^T)": lambda: torch.matmul(w_ih.t(), d_tab.transpose(1, 2)),
    }
    ref_w = torch.einsum("sth,sct->hc", d_tab.double(), lat_t.double())
    for name, fn in cases.items():
        us = timed(fn)
        extra = ""
        if name.startswith("d_wih"):
            r = fn()
            r = r[0][0] if isinstance(r, list) else r
            extra = f"  max err / max {float((r.double() - ref_w).abs().max() / ref_w.abs().max()):.2e}"
        print(f"{name:48s} {us:8.1f} us{extra}", flush=True)


if __name__ == "__main__":
    main()
