"""CPU restatement of the in-kernel noise of the HIP renderer (TEST
INFRASTRUCTURE ONLY: imported by tests/, smoke() and bench.py's cpu_baseline
leg, never by the product path).

The reference draws its noise from torch's global RNG (renderers.py:14
`rand_like`, :41 `rand`, :45 `rand_like`, :63 `randn_like`). With
`VolumeRenderer.seed` set (the benchmarked configuration, bench.py) the HIP
kernels draw the same quantities themselves from a counter-based generator,
so no noise bytes are read from HBM. This module restates that generator so
the oracle can be fed exactly the draws the kernels made:

  * Philox4x32-10 (Salmon, Moraes, Dror, Shaw: "Parallel random numbers: as
    easy as 1, 2, 3", SC'11; the Random123 reference algorithm): 10 rounds of
        (hi0, lo0) = M0 * c0,  (hi1, lo1) = M1 * c2       (32x32 -> 64 bit)
        c = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0)
    with M0 = 0xD2511F53, M1 = 0xCD9E8D57 and the Weyl key bump
    k += (0x9E3779B9, 0xBB67AE85) after each round. Pinned by the published
    Random123 known-answer vectors (tests/test_philox_cpu.py).
  * counter = (ray_lo, ray_hi, block, stream), key = (seed_lo, seed_hi), where
    ray = offset + frame-wide ray id (csrc/avr_common.h philox_uniform4);
  * uniform = (x >> 8) * 2^-24 for each of the 4 output words;
  * streams (csrc/sampling.hip): coarse 0x1001 -- sample s of a ray is word
    s & 3 of block s >> 2; fine 0x2002 -- importance sample f takes u = word 0
    and u2 = word 1 of block f; depth 0x4004 -- Box-Muller on words 0, 1 of
    block d (quirk Q6: after clamp(near, far) every depth sample is `near` for
    any draw below near / depth_std standard deviations, so the depth draw is
    restated in float64 and compared through the clamp only).
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
STREAM_COARSE, STREAM_FINE, STREAM_DEPTH = 0x1001, 0x2002, 0x4004
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr (..., 4) uint32, key (..., 2) uint32 (broadcast) -> (..., 4) uint32."""
    c = [np.asarray(ctr[..., i], dtype=np.uint32) for i in range(4)]
    k0 = np.asarray(key[..., 0], dtype=np.uint32).copy()
    k1 = np.asarray(key[..., 1], dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c[0].astype(np.uint64)
            p1 = M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK32).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = k0 + W0
            k1 = k1 + W1
    return np.stack(np.broadcast_arrays(*c), -1)


def uniform4(seed, rays, blocks, stream):
    """philox_uniform4 (csrc/avr_common.h): rays (R,) uint64 counters (offset
    already added), blocks (B,) -> (R, B, 4) float32 uniforms on the 2^-24 grid."""
    rays = np.asarray(rays, dtype=np.uint64)[:, None]
    blocks = np.asarray(blocks, dtype=np.uint32)[None, :]
    R, B = rays.shape[0], blocks.shape[1]
    ctr = np.empty((R, B, 4), np.uint32)
    ctr[..., 0] = (rays & _MASK32).astype(np.uint32)
    ctr[..., 1] = (rays >> np.uint64(32)).astype(np.uint32)
    ctr[..., 2] = blocks
    ctr[..., 3] = np.uint32(stream)
    s = np.uint64(seed)
    key = np.array([np.uint32(s & _MASK32), np.uint32(s >> np.uint64(32))], np.uint32)
    bits = philox4x32_10(ctr, key)
    return ((bits >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)


def ray_keys(n_rays, offset=0, ray_ids=None):
    """The per-ray Philox counter: offset + (ray_ids[r] if given else r)."""
    ids = np.arange(n_rays, dtype=np.uint64) if ray_ids is None else np.asarray(ray_ids, dtype=np.uint64)
    return np.uint64(offset) + ids


def coarse_noise(seed, keys, n_samples):
    """The rand_like draw of sample_coarse (renderers.py:14): (R, n_samples)."""
    nq = (n_samples + 3) // 4
    v = uniform4(seed, keys, np.arange(nq), STREAM_COARSE)
    return np.ascontiguousarray(v.reshape(len(keys), nq * 4)[:, :n_samples])


def fine_noise(seed, keys, n_fine):
    """sample_fine's rand / rand_like pair (renderers.py:41, :45): u, u2 (R, n_fine)."""
    v = uniform4(seed, keys, np.arange(n_fine), STREAM_FINE)
    return np.ascontiguousarray(v[..., 0]), np.ascontiguousarray(v[..., 1])


def depth_normal(seed, keys, n_depth):
    """sample_depth's randn_like (renderers.py:63), Box-Muller in float64
    (the kernel's logf / cospif are not restated bit for bit; see the header)."""
    v = uniform4(seed, keys, np.arange(n_depth), STREAM_DEPTH).astype(np.float64)
    u1 = np.maximum(v[..., 0], 1e-7)
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * v[..., 1])).astype(np.float32)


def renderer_draws(seed, n_rays, n_coarse, n_fine, n_depth, offset=0, ray_ids=None):
    """Every draw VolumeRenderer.forward makes with `seed` set, keyed as the
    kernels key them, in the reference's noise-dict layout (1, R, n)."""
    keys = ray_keys(n_rays, offset, ray_ids)
    u, u2 = fine_noise(seed, keys, n_fine)
    return {"coarse": coarse_noise(seed, keys, n_coarse)[None], "u": u[None], "u2": u2[None],
            "depth": depth_normal(seed, keys, n_depth)[None]}
