"""avr.anomaly on the CPU: the hooks are installed on every op / field forward / HIP Function backward, and
the check fires under either switch (avr's own flag, torch's anomaly mode as train.py:106 sets it) and only
then. No kernel is launched: the wrapped callable here is a stand-in."""
import pytest
import torch

from avr import anomaly, field, ops


def test_every_hook_installed():
    for n in anomaly.OPS:
        assert getattr(getattr(ops, n), "__avr_checked__", False), n
    for n in anomaly.FIELD_METHODS:
        assert getattr(getattr(field.FusedField, n), "__avr_checked__", False), n
    for m, c in anomaly.FUNCTIONS:
        assert getattr(getattr({"ops": ops, "field": field}[m], c).backward, "__avr_checked__", False), c
    anomaly.install()   # idempotent: no double wrapping
    assert not getattr(ops.world_rays.__wrapped__, "__avr_checked__", False)


def test_switches():
    bad = anomaly._checked("standin", lambda: (torch.zeros(2), None, torch.tensor([0.0, float("inf")])))
    good = anomaly._checked("standin", lambda: (torch.ones(3), torch.arange(3)))
    assert not anomaly.is_enabled()
    bad()                                   # off: passes NaN / Inf through like the kernels do
    anomaly.set_detect_anomaly(True)
    try:
        with pytest.raises(FloatingPointError, match=r"standin returned 1 non-finite values \(0 NaN\) in output\[2\]"):
            bad()
        good()
    finally:
        anomaly.set_detect_anomaly(False)
    with torch.autograd.set_detect_anomaly(True):
        with pytest.raises(FloatingPointError):
            bad()
    bad()
