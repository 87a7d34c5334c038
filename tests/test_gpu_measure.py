"""The bench's HBM yardsticks (avr_stream_copy / avr_stream_fill): exact results, argument checks."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from avr import ops
    return ops


def test_stream_copy_and_fill_exact(ops):
    dev = torch.device("cuda:0")
    for n in (4, 1000, 1 << 20, (1 << 20) + 12):   # partial last workgroup included
        src = torch.randn(n, device=dev)
        dst = torch.zeros(n, device=dev)
        ops.stream_copy(src, dst)
        assert torch.equal(src, dst)
        ops.stream_fill(dst, 0x3F800000)
        assert bool((dst == 1.0).all())
        ops.stream_fill(dst, 0xFFFFFFFF)
        assert bool((dst.view(torch.int32) == -1).all())


def test_stream_fill_rejects_ragged(ops):
    from avr._lib import AVRError
    x = torch.zeros(3, device="cuda:0")
    with pytest.raises(AVRError):
        ops.stream_fill(x, 0)
