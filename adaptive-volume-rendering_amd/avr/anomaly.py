"""Non-finite checks on every HIP op's outputs: the HIP-side counterpart of the reference's
`--anomaly_detection` flag (train.py:106,208: `torch.autograd.set_detect_anomaly(flag)`).

torch's anomaly mode checks the gradients autograd Functions return, but it cannot see the forward outputs of
kernels it did not write. With checking on, every public op of `avr.ops` (rays, sampling, compositing, depth,
march, raymarch, latent features, weight gradients), every `FusedField` forward and every HIP autograd
Function's backward synchronises and raises `FloatingPointError` naming the op, the output and the count of
NaN / Inf values, so a NaN is caught at the launch that produced it instead of in the loss.

Checking is on when any of these holds:
  * `torch.autograd.set_detect_anomaly(True)` / `torch.autograd.detect_anomaly()` is active (so train.py's own
    flag covers the HIP path unchanged);
  * `avr.anomaly.set_detect_anomaly(True)` was called;
  * the environment has AVR_DETECT_ANOMALY=1 at import.
Off (the default), an op pays one flag test. Ops inside a HIP-graph capture are never checked (a capture cannot
synchronise); integer outputs (bins, indices) are not checked.
"""
import functools
import os

import torch

__all__ = ["set_detect_anomaly", "is_enabled", "check_outputs", "poison_allocations"]

_flag = os.environ.get("AVR_DETECT_ANOMALY", "0") not in ("", "0")
_installed = False


def set_detect_anomaly(mode: bool):
    """Turn the per-op non-finite checks on or off (independently of torch's anomaly mode)."""
    global _flag
    _flag = bool(mode)


def is_enabled():
    return _flag or torch.is_anomaly_enabled()


def _tensors(out, path="output"):
    if isinstance(out, torch.Tensor):
        yield path, out
    elif isinstance(out, (tuple, list)):
        for i, o in enumerate(out):
            yield from _tensors(o, f"{path}[{i}]")


def check_outputs(name, out):
    """Raise FloatingPointError if a floating-point tensor in `out` holds a NaN or an Inf."""
    for path, t in _tensors(out):
        if not t.is_floating_point() or t.numel() == 0:
            continue
        if t.is_cuda and torch.cuda.is_current_stream_capturing():
            return
        bad = ~torch.isfinite(t.detach())
        if bool(bad.any()):
            n_nan = int(torch.isnan(t.detach()).sum())
            raise FloatingPointError(f"avr anomaly: {name} returned {int(bad.sum())} non-finite values "
                                     f"({n_nan} NaN) in {path} of shape {tuple(t.shape)}")
    return out


def _checked(name, fn):
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        out = fn(*args, **kwargs)
        if _flag or torch.is_anomaly_enabled():
            check_outputs(name, out)
        return out
    wrapper.__avr_checked__ = True
    return wrapper


OPS = ("world_rays", "rays_sample_coarse", "composite_depth", "depth_from_world_fwd", "sample_coarse", "sample_fine",
       "composite_fwd", "composite_bwd", "march_fine", "sample_coarse_rays", "depth_of_points_fwd", "raymarch",
       "weight_grads", "weight_grads_specs", "latent_features")
FIELD_METHODS = ("forward_rays", "forward_rays_batch", "forward_points_multiview", "forward_points", "forward_train")
FUNCTIONS = (("ops", "_Depth"), ("ops", "_Composite"), ("ops", "_DepthOfPoints"), ("field", "_FieldTrain"),
             ("bn_train", "_FieldTrainBN"), ("renderers", "_MarchTrain"),
             ("renderers", "_Band"))


def install():
    """Wrap the ops, the FusedField forwards and the HIP autograd Functions' backward (idempotent)."""
    global _installed
    if _installed:
        return
    from . import bn_train, field, ops, renderers
    mods = {"ops": ops, "field": field, "bn_train": bn_train, "renderers": renderers}
    for n in OPS:
        f = getattr(ops, n)
        if not getattr(f, "__avr_checked__", False):
            setattr(ops, n, _checked(f"ops.{n}", f))
    for n in FIELD_METHODS:
        f = getattr(field.FusedField, n)
        if not getattr(f, "__avr_checked__", False):
            setattr(field.FusedField, n, _checked(f"FusedField.{n}", f))
    for m, c in FUNCTIONS:
        cls = getattr(mods[m], c)
        f = cls.backward
        if not getattr(f, "__avr_checked__", False):
            cls.backward = staticmethod(_checked(f"{c}.backward", f))
    _installed = True


class poison_allocations:
    """Debug allocation hook: while active, every floating-point device tensor made by torch.empty /
    torch.empty_like / Tensor.new_empty (the buffers the HIP kernels write their outputs into) starts filled with
    `value` (default NaN) instead of whatever the caching allocator or a fresh hipMalloc left there. A kernel
    that reads an output element it did not write -- a padding row, a tail past M, a table column -- then yields
    NaN (or, with value=0.0, a reproducible zero), so two runs under different fills differ exactly where memory
    is read before it is written. Integer buffers are left alone (garbage indices would fault the GPU).

        with avr.anomaly.poison_allocations(float("nan")):
            loss = step(); loss.backward()
    """

    def __init__(self, value=float("nan"), device_types=("cuda",)):
        self.value = float(value)
        self.device_types = tuple(device_types)
        self._saved = None

    def _fill(self, t):
        if (isinstance(t, torch.Tensor) and t.device.type in self.device_types and t.is_floating_point()
                and t.numel() > 0):
            with torch.no_grad():
                t.fill_(self.value)
        return t

    def __enter__(self):
        self._saved = (torch.empty, torch.empty_like, torch.Tensor.new_empty)
        real_empty, real_like, real_new = self._saved
        fill = self._fill
        torch.empty = functools.wraps(real_empty)(lambda *a, **k: fill(real_empty(*a, **k)))
        torch.empty_like = functools.wraps(real_like)(lambda *a, **k: fill(real_like(*a, **k)))
        torch.Tensor.new_empty = lambda self_, *a, **k: fill(real_new(self_, *a, **k))
        return self

    def __exit__(self, *exc):
        torch.empty, torch.empty_like, torch.Tensor.new_empty = self._saved
        return False
