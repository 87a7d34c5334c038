"""avr.anomaly on the GPU: a NaN fed to a HIP kernel is caught at that kernel's launch under torch's anomaly
mode (train.py:106's switch) and under avr's own flag, passes through silently with both off, and clean
renders / backward passes raise nothing with checking on (no false positives)."""
import numpy as np
import pytest
import torch

from helpers import build_net
from oracle import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _composite_inputs(nan):
    g = torch.Generator(device=DEV).manual_seed(5)
    z = torch.sort(0.8 + torch.rand(32, 64, device=DEV, generator=g), -1)[0]
    field = torch.rand(32, 64, 4, device=DEV, generator=g)
    if nan:
        field[7, 11, 3] = float("nan")
    return z, field


def test_nan_caught_at_the_launch():
    from avr import anomaly, ops
    z, field = _composite_inputs(True)
    rgb, _, _ = ops.composite_fwd(z, field)          # off: NaN propagates like the reference's kernels
    assert torch.isnan(rgb[7]).any()
    with torch.autograd.set_detect_anomaly(True):
        with pytest.raises(FloatingPointError, match="ops.composite_fwd"):
            ops.composite_fwd(z, field)
    anomaly.set_detect_anomaly(True)
    try:
        with pytest.raises(FloatingPointError, match="ops.composite_fwd"):
            ops.composite_fwd(z, field)
    finally:
        anomaly.set_detect_anomaly(False)


def test_clean_render_and_backward_under_anomaly(golden):
    from avr import ops
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, "x3")
    R = 200
    rend = VolumeRenderer(0.8, 1.8, 128, 64, 0, 0.01, True)
    rend.seed = 3
    c2w = torch.as_tensor(np.ascontiguousarray(synth.orbit_cam2world(0.7)), device=DEV).reshape(1, 1, 4, 4)
    K = torch.as_tensor(np.ascontiguousarray(synth.default_intrinsics()[None]), device=DEV)
    x = torch.rand(1, R, 2, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    with torch.autograd.set_detect_anomaly(True):
        with torch.no_grad():
            out = rend(c2w.expand(1, R, 4, 4), K, x, net)
        assert rend.last_path == "fused" and torch.isfinite(out[1]).all()
        z, field = _composite_inputs(False)
        field.requires_grad_(True)
        rgb, dist, _ = ops.composite(z, field)
        (rgb.sum() + dist.sum()).backward()
    assert torch.isfinite(field.grad).all()
