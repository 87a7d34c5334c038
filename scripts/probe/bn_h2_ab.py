"""Diagnostic: the d_hidden-512 fc_1 forward layer (bn_layer_bench.py's case) launched 10 times with each of the
two-half kernels (bn_layer_h2_fwd_kernel<RG>, AVR_BN_H2=2 / 1: 128 / 64 rows per workgroup) and 10 times with the
one-workgroup kernel (AVR_BN_H2=0), for rocprofv3 kernel traces and counter passes that see every name in one process. Needs scripts/ab/bn_h2_fwd_two_halves.patch
applied to csrc/bn_train.hip (rejected: profiles/r06v_bn_h2_ab.txt); without it all three runs are the product kernel."""
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))


def main():
    from avr import _lib
    from avr.bn_train import _layer, _partial, _run
    from avr.conf import Conf, default_conf
    from avr.scene import synthetic_scene
    dev = torch.device("cuda:0")
    M, H = int(sys.argv[1]) if len(sys.argv) > 1 else 163840, 512
    d = dict(default_conf()["model"])
    mlp = {"type": "resnet", "n_blocks": 3, "d_hidden": H, "combine_layer": 3}
    d["mlp_coarse"], d["mlp_fine"] = dict(mlp), dict(mlp)
    net = synthetic_scene(dev, 0, Conf(d))
    entry = net.fused().packed(True)
    g = torch.Generator(device="cpu").manual_seed(0)
    src, res = torch.randn(M, H, generator=g).to(dev), torch.randn(M, H, generator=g).to(dev)
    out = torch.empty(M, H, device=dev)
    zero, one = torch.zeros(H, device=dev), torch.ones(H, device=dev)
    part = _partial(M, H, dev)
    stream = _lib.stream_of(src)
    fwd = _layer(n_rows=M, mode=_lib.BN_FWD, prologue=_lib.BN_RELU, in_dim=H, in_valid=H, src=src, ld_src=H,
                 in_mu=zero, in_scale=one, in_shift=zero, blob=entry.packed, layer=3, bias=zero, add1=res, out=out,
                 partial=part)
    outs = {}
    for h2 in ("2", "1", "0"):
        os.environ["AVR_BN_H2"] = h2
        for _ in range(10):
            _run(entry.dims, fwd, stream)
        torch.cuda.synchronize()
        outs[h2] = out.clone()
    for h2 in ("2", "1"):
        print(f"AVR_BN_H2={h2}: max |out - one-workgroup out| =", float((outs[h2] - outs["0"]).abs().max()), "of",
              float(outs["0"].abs().max()))


if __name__ == "__main__":
    main()
