"""Diagnostic: the adaptive step's point-gradient product g_feat = sum_b Gz[b] @ W_z[b] (avr.field
_FieldTrain.backward, three lin_z layers) at the band's row count, as three chained addmm (avr.ops.sum_of_products)
against one GEMM over the concatenated K. Prints us per call. usage: python scripts/gfeat_bench.py [rows]"""
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
    from avr.ops import sum_of_products
    dev = torch.device("cuda:0")
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    g = torch.Generator(device="cpu").manual_seed(0)
    G = torch.randn(7, M, 512, generator=g).to(dev)
    Gz = [G[6], G[1], G[3]]
    Wz = [(torch.randn(512, 512, generator=g) * 0.05).to(dev) for _ in range(3)]
    Wcat = torch.cat(Wz, 0)
    ref = sum(a.double() @ b.double() for a, b in zip(Gz, Wz))
    cases = {
        "sum_of_products (3 addmm) [current]": lambda: sum_of_products(list(zip(Gz, Wz))),
        "cat(Gz) @ cat(W) (copy + 1 GEMM)": lambda: torch.cat(Gz, 1) @ Wcat,
        "bmm(stack) + sum": lambda: torch.bmm(torch.stack(Gz), torch.stack(Wz)).sum(0),
    }
    for name, fn in cases.items():
        us = timed(fn)
        err = float((fn().double() - ref).abs().max() / ref.abs().max())
        print(f"M={M} {name:40s} {us:8.1f} us  err {err:.1e}  {2 * 3 * M * 512 * 512 / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
