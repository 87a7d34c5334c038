"""avr — MI355X-native (gfx950 HIP) coarse/fine volume renderer with the
interface of yankeesong/adaptive-volume-rendering's renderers.py.

    from avr.renderers import VolumeRenderer, volume_integral, sample_coarse, sample_fine, sample_depth
    from avr.models import NewPixelNeRFNet, RadFieldAndRenderer
"""
from . import _lib  # noqa: F401
from . import anomaly
from .renderers import VolumeRenderer, sample_coarse, sample_depth, sample_fine, volume_integral  # noqa: F401

anomaly.install()   # per-op non-finite checks, off unless anomaly mode is on (avr/anomaly.py)

__all__ = ["VolumeRenderer", "sample_coarse", "sample_fine", "sample_depth", "volume_integral"]


def load_library():
    """Load libavr_hip.so (raises if it is not built)."""
    return _lib.load()
