"""The CPU restatement of the kernels' in-kernel noise (oracle/philox.py):
pinned to the published Philox4x32-10 known-answer vectors of the Random123
reference implementation, and the per-stream layout the renderer's kernels
use (csrc/sampling.hip, csrc/avr_common.h)."""
import numpy as np
import pytest

from oracle import philox as P

# Random123 kat_vectors, philox4x32 with 10 rounds: counter (4 words), key (2 words) -> 4 words
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox4x32_10_known_answers(ctr, key, want):
    got = P.philox4x32_10(np.array(ctr, np.uint32), np.array(key, np.uint32))
    assert [int(v) for v in got] == list(want)


def test_philox_vectorised_equals_scalar():
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2 ** 32, (257, 4), dtype=np.uint64).astype(np.uint32)
    key = rng.integers(0, 2 ** 32, 2, dtype=np.uint64).astype(np.uint32)
    batch = P.philox4x32_10(ctr, key)
    for i in (0, 1, 100, 256):
        np.testing.assert_array_equal(batch[i], P.philox4x32_10(ctr[i], key))


def test_uniform_grid_and_counter_layout():
    seed, keys = (1 << 40) + 1234, P.ray_keys(5, offset=(1 << 33) + 7)
    u = P.uniform4(seed, keys, np.arange(3), P.STREAM_COARSE)
    assert u.dtype == np.float32 and u.shape == (5, 3, 4)
    assert float(u.min()) >= 0.0 and float(u.max()) < 1.0
    # every value is k * 2^-24 for an integer k < 2^24
    k = u.astype(np.float64) * 2.0 ** 24
    np.testing.assert_array_equal(k, np.round(k))
    # counter = (ray lo, ray hi, block, stream), key = (seed lo, seed hi)
    r, b = 3, 2
    ray = int(keys[r])
    bits = P.philox4x32_10(np.array([ray & 0xFFFFFFFF, ray >> 32, b, P.STREAM_COARSE], np.uint32),
                           np.array([seed & 0xFFFFFFFF, seed >> 32], np.uint32))
    np.testing.assert_array_equal(u[r, b], ((bits >> 8).astype(np.float64) * 2.0 ** -24).astype(np.float32))


def test_stream_layout():
    """coarse sample s = word s & 3 of block s >> 2 (ragged counts truncate);
    fine sample f = (word 0, word 1) of block f; streams are distinct."""
    keys = P.ray_keys(4, offset=10, ray_ids=np.array([5, 0, 99, 3]))
    np.testing.assert_array_equal(keys, np.array([15, 10, 109, 13], np.uint64))
    c30 = P.coarse_noise(7, keys, 30)
    c32 = P.coarse_noise(7, keys, 32)
    assert c30.shape == (4, 30)
    np.testing.assert_array_equal(c30, c32[:, :30])
    blk = P.uniform4(7, keys, np.arange(8), P.STREAM_COARSE)
    np.testing.assert_array_equal(c32, blk.reshape(4, 32))
    u, u2 = P.fine_noise(7, keys, 9)
    fb = P.uniform4(7, keys, np.arange(9), P.STREAM_FINE)
    np.testing.assert_array_equal(u, fb[..., 0])
    np.testing.assert_array_equal(u2, fb[..., 1])
    assert not np.array_equal(u[:, :8], c32[:, :8])
    d = P.renderer_draws(7, 4, 30, 9, 5, offset=10, ray_ids=np.array([5, 0, 99, 3]))
    assert d["coarse"].shape == (1, 4, 30) and d["u"].shape == (1, 4, 9) and d["depth"].shape == (1, 4, 5)
    np.testing.assert_array_equal(d["coarse"][0], c30)


def test_uniform_moments():
    """A million draws: mean 1/2, variance 1/12, no correlation between u and u2."""
    u, u2 = P.fine_noise(3, P.ray_keys(16384), 64)
    assert abs(u.mean() - 0.5) < 2e-3 and abs(u.var() - 1 / 12) < 1e-3
    assert abs(np.corrcoef(u.ravel(), u2.ravel())[0, 1]) < 3e-3
    n = P.depth_normal(3, P.ray_keys(16384), 16)
    assert abs(n.mean()) < 1e-2 and abs(n.std() - 1.0) < 1e-2
