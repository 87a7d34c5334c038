"""avr.anomaly on the CPU: the hooks are installed on every op / field forward / HIP Function backward, and
the check fires under either switch (avr's own flag, torch's anomaly mode as train.py:106 sets it) and only
then. No kernel is launched: the wrapped callable here is a stand-in."""
import pytest
import torch

from avr import anomaly, bn_train, field, ops, renderers


def test_every_hook_installed():
    for n in anomaly.OPS:
        assert getattr(getattr(ops, n), "__avr_checked__", False), n
    for n in anomaly.FIELD_METHODS:
        assert getattr(getattr(field.FusedField, n), "__avr_checked__", False), n
    for m, c in anomaly.FUNCTIONS:
        assert getattr(getattr({"ops": ops, "field": field, "bn_train": bn_train,
                                                "renderers": renderers}[m], c).backward, "__avr_checked__", False), c
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


def test_poison_allocations_fills_and_restores():
    """avr.anomaly.poison_allocations: floating-point buffers from torch.empty / empty_like / new_empty start as
    the poison value while active (integer buffers untouched), and the originals come back afterwards."""
    import math

    import torch
    from avr.anomaly import poison_allocations
    before = (torch.empty, torch.empty_like, torch.Tensor.new_empty)
    with poison_allocations(float("nan"), device_types=("cpu",)):
        a = torch.empty(5, 3)
        b = torch.empty_like(torch.zeros(4, dtype=torch.float64))
        c = torch.zeros(2).new_empty(7)
        i = torch.empty(6, dtype=torch.int32)
        assert all(math.isnan(float(x)) for t in (a, b, c) for x in t.reshape(-1))
        assert i.dtype == torch.int32
    with poison_allocations(0.0, device_types=("cpu",)):
        assert float(torch.empty(9).abs().sum()) == 0.0
    assert (torch.empty, torch.empty_like, torch.Tensor.new_empty) == before
