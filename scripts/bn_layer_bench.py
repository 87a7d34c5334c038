"""Diagnostic: one avr_bn_layer_run launch (the BatchNorm / layer-by-layer training GEMM) timed alone at the --bn
step's row count, per d_hidden and layer kind: us per launch, HBM bytes per launch (the rows each reads and writes) and the x3 MFMA work, as fractions of 8 TB/s and 833 TF.
usage: python scripts/bn_layer_bench.py [rows]"""
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))


def main():
    from avr import _lib
    from avr.bn_train import _layer, _partial, _run
    from avr.conf import Conf, default_conf
    from avr.scene import synthetic_scene
    dev = torch.device("cuda:0")
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 163840
    for H in (256, 512):
        d = dict(default_conf()["model"])
        mlp = {"type": "resnet", "n_blocks": 3, "d_hidden": H, "combine_layer": 3}
        d["mlp_coarse"], d["mlp_fine"] = dict(mlp), dict(mlp)
        net = synthetic_scene(dev, 0, Conf(d))
        fused = net.fused()
        entry = fused.packed(True)
        bwd = fused.packed_bwd(True, entry)
        g = torch.Generator(device="cpu").manual_seed(0)
        src = torch.randn(M, H, generator=g).to(dev)
        res = torch.randn(M, H, generator=g).to(dev)
        out = torch.empty(M, H, device=dev)
        zero, one = torch.zeros(H, device=dev), torch.ones(H, device=dev)
        bias = torch.zeros(H, device=dev)
        part = _partial(M, H, dev)
        stream = _lib.stream_of(src)
        fwd = _layer(n_rows=M, mode=_lib.BN_FWD, prologue=_lib.BN_RELU, in_dim=H, in_valid=H, src=src, ld_src=H,
                     in_mu=zero, in_scale=one, in_shift=zero, blob=entry.packed, layer=3, bias=bias, add1=res, out=out,
                     partial=part)
        bwl = _layer(n_rows=M, mode=_lib.BN_BWD, prologue=_lib.BN_PLAIN, in_dim=H, in_valid=H, src=src, ld_src=H,
                     blob=bwd, layer=3, out=out, pre_rows=res, out_mu=zero, out_invstd=one, out_scale=one,
                     out_shift=zero, partial=part)
        zin = torch.randn(M, 64, generator=g).to(dev)
        lin = _layer(n_rows=M, mode=_lib.BN_FWD, prologue=_lib.BN_PLAIN, in_dim=64, in_valid=39, src=zin, ld_src=64,
                     blob=entry.packed, layer=0, bias=bias, out=out, partial=part)
        pre2 = torch.randn(M, H, generator=g).to(dev)
        bwg = _layer(n_rows=M, mode=_lib.BN_BWD, prologue=_lib.BN_GRAD, in_dim=H, in_valid=H, src=src, ld_src=H,
                     src_pre=pre2, src_res=res, in_mu=zero, in_invstd=one, in_m1=zero, in_m2=zero, in_scale=one,
                     blob=bwd, layer=2, out=out, pre_rows=res, out_mu=zero, out_invstd=one, out_scale=one,
                     out_shift=zero, partial=part)
        cases = (("fwd fc_1 (relu operand + residual)", fwd, 3), ("bwd fc_1^T (mask from pre rows)", bwl, 3),
                 ("fwd lin_in (39 of 64 columns)", lin, None), ("bwd fc_0^T (BN-grad prologue + residual)", bwg, 5))
        for name, lay, nrows in cases:
            for _ in range(3):
                _run(entry.dims, lay, stream)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            t0.record()
            for _ in range(n):
                _run(entry.dims, lay, stream)
            t1.record()
            torch.cuda.synchronize()
            us = t0.elapsed_time(t1) / n * 1e3
            nbytes = (nrows * M * H if nrows else M * (64 + H)) * 4
            flops = 2.0 * M * H * (H if nrows else 64)
            print(f"H {H:3d} {name:42s}: {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s ({nbytes / us / 1e3 / 8000:.3f} of "
                  f"8 TB/s)  {flops / us / 1e6:6.1f} TF/s fp32-eq ({flops / us / 1e6 / 833.3:.3f} of the x3 peak)",
                  flush=True)


if __name__ == "__main__":
    main()
