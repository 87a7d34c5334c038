"""Diagnostic: after in-place optimizer steps, FusedField.packed()'s pointer-reusing repack vs a pack from scratch:
which blob floats differ (not part of the product or the tests). Measured (round 6): the first 41 472 floats of the
default 64-wide x3 blob differ -- a region the x3 pack does not write (allocator garbage in both); the fields the two
blobs evaluate are bit-equal (test_repack_after_in_place_update_matches_fresh_pack) and no kernel reads unwritten
memory (tests/test_gpu_poison.py)."""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "adaptive-volume-rendering_amd"); sys.path.insert(0, ".")
import test_gpu_train as T  # noqa: E402
from avr.field import FusedField  # noqa: E402
net = T._net(64, 3, 64, (8, 8))
fused = net.fused()
opt = torch.optim.Adam(net.mlp_coarse.parameters(), lr=1e-2)
xyz, vd, w = T._points(1, 200, seed=31)
for _ in range(3):
    opt.zero_grad()
    (net(xyz, coarse=True, viewdirs=vd) * w).sum().backward()
    opt.step()
e1 = fused.packed(True)
e2 = FusedField(net, "x3").packed(True)
b1, b2 = e1.packed, e2.packed
d = (b1 != b2)
idx = d.nonzero().flatten()
print("numel", b1.numel(), "differing", idx.numel(), "dims", bytes(e1.dims) == bytes(e2.dims), e1.dims.precision, e2.dims.precision)
if idx.numel():
    print("first", idx[:8].tolist(), "last", idx[-8:].tolist())
    print("b1", b1[idx[:8]].tolist()); print("b2", b2[idx[:8]].tolist())
    print("as int b1", b1[idx[:4]].view(torch.int32).tolist(), "b2", b2[idx[:4]].view(torch.int32).tolist())
