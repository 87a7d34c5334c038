"""Deterministic synthetic data for golden vectors and parity tests.

TEST INFRASTRUCTURE ONLY: imported by tests/, tests/golden/make_golden.py,
__graft_entry__.smoke() and bench.py's cpu_baseline leg. Never by the product.

Values come from an integer hash (splitmix64) of (seed, flat index), mapped to
24-bit fractions, so every value is an exact float32 and identical on any host,
numpy version or CPU (no libm, no PRNG stream-compatibility assumptions). This
lets fixtures store only a seed for large tensors (e.g. the 512-wide MLP
weights) instead of megabytes of data.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def hashed_bits(shape, seed):
    n = int(np.prod(shape)) if len(shape) else 1
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) * np.uint64(0x100000001B3)) & _M64
        h = _splitmix64(idx ^ key)
        h = _splitmix64(h + np.uint64(seed))
    return h.reshape(shape)


def hashed_uniform(shape, seed, lo=0.0, hi=1.0):
    """Exact-float32 values in [lo, hi) on a 2^-24 grid (lo/hi should be dyadic)."""
    h = hashed_bits(shape, seed)
    frac = (h >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)  # [0,1), 24 bits
    return (lo + (hi - lo) * frac).astype(np.float32)


def hashed_centered(shape, seed, scale):
    """Uniform in [-scale/2, scale/2), exact in fp32 when scale is a power of two."""
    return hashed_uniform(shape, seed, -0.5 * scale, 0.5 * scale)


def hashed_normalish(shape, seed, scale):
    """Sum of 4 hashed uniforms (Irwin-Hall), centred: a bell-shaped value with
    std ~= 0.577*scale. Exact in fp32 for power-of-two scales."""
    acc = np.zeros(shape, np.float64)
    for k in range(4):
        acc += hashed_uniform(shape, seed * 4 + k + 1).astype(np.float64)
    return ((acc - 2.0) * scale).astype(np.float32)


def pow2_scale(fan_in):
    """Power-of-two width for a centred uniform whose std ~ kaiming sqrt(2/fan_in)."""
    target = np.sqrt(2.0 / fan_in) / np.sqrt(1.0 / 12.0)
    return float(2.0 ** np.round(np.log2(target)))


def resnetfc_params(d_in, d_latent, d_hidden, n_blocks, combine_layer, seed, d_out=4, spade=False):
    """Hash-generated parameters for a reference ResnetFC (models.py:473-606),
    keyed by the reference's state_dict names. fc_1 weights are NON-zero on
    purpose (the reference zero-inits them at models.py:440, which would make
    every block an identity and hide bugs). spade: also scale_z[b]
    (models.py:528-534), with biases around 1 so scale_z(z) * x keeps x's size."""
    p = {}
    s = seed * 1000
    p["lin_in.weight"] = hashed_centered((d_hidden, d_in), s + 1, pow2_scale(d_in))
    p["lin_in.bias"] = hashed_centered((d_hidden,), s + 2, 0.125)
    p["lin_out.weight"] = hashed_centered((d_out, d_hidden), s + 3, pow2_scale(d_hidden))
    p["lin_out.bias"] = hashed_centered((d_out,), s + 4, 0.125)
    for b in range(n_blocks):
        p[f"blocks.{b}.fc_0.weight"] = hashed_centered((d_hidden, d_hidden), s + 10 + 4 * b, pow2_scale(d_hidden))
        p[f"blocks.{b}.fc_0.bias"] = hashed_centered((d_hidden,), s + 11 + 4 * b, 0.0625)
        p[f"blocks.{b}.fc_1.weight"] = hashed_centered((d_hidden, d_hidden), s + 12 + 4 * b, 0.125)
        p[f"blocks.{b}.fc_1.bias"] = hashed_centered((d_hidden,), s + 13 + 4 * b, 0.0625)
    if d_latent > 0:
        for b in range(min(combine_layer, n_blocks)):
            p[f"lin_z.{b}.weight"] = hashed_centered((d_hidden, d_latent), s + 100 + 2 * b, pow2_scale(d_latent))
            p[f"lin_z.{b}.bias"] = hashed_centered((d_hidden,), s + 101 + 2 * b, 0.0625)
            if spade:
                p[f"scale_z.{b}.weight"] = hashed_centered((d_hidden, d_latent), s + 200 + 2 * b,
                                                           0.5 * pow2_scale(d_latent))
                p[f"scale_z.{b}.bias"] = (1.0 + hashed_centered((d_hidden,), s + 201 + 2 * b, 0.25)).astype(np.float32)
    return p


def orbit_cam2world(angle, radius=1.3, z_height=0.4):
    """Orbit camera pose as built by the reference's generate_video
    (utils.py:497-513 with get_R utils.py:464-479), restated in float64 and
    rounded to float32 once."""
    rr = np.sqrt(radius * radius - z_height * z_height)
    t = np.array([rr * np.sin(angle), rr * np.cos(angle), z_height])
    zax = -t / max(np.linalg.norm(t), 1e-5)
    up = np.array([0.0, 0.0, -1.0])
    xax = np.cross(up, zax)
    xax /= max(np.linalg.norm(xax), 1e-5)
    yax = np.cross(zax, xax)
    yax /= max(np.linalg.norm(yax), 1e-5)
    R = np.stack([xax, yax, zax], 0).T
    c2w = np.eye(4)
    c2w[:3, :3] = R
    c2w[:3, 3] = t
    c2w = c2w @ np.diag([1.0, -1.0, -1.0, 1.0])
    return c2w.astype(np.float32)


def default_intrinsics():
    """Normalised SRN-cars intrinsics (focal/W, cx/W) as used by the survey configs."""
    return np.array([[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]], np.float32)


def source_view(latent_hw=(64, 64), image_hw=(128, 128)):
    """Source-view buffers the reference's NewPixelNeRFNet.encode would set
    (models.py:705-734): world->cam pose (1,3,4), focal (1,2) with fy negated,
    principal point (1,2), image_shape (W,H), and latent_scaling
    (SpatialEncoder.forward, models.py:326-328)."""
    H, W = image_hw
    poses = np.zeros((1, 3, 4), np.float32)
    poses[0, :3, :3] = np.eye(3)
    poses[0, 2, 3] = 1.3
    focal = np.array([[131.25, -131.25]], np.float32)
    c = np.array([[W * 0.5, H * 0.5]], np.float32)
    image_shape = np.array([W, H], np.float32)
    hl, wl = latent_hw
    ls = np.array([wl, hl], np.float32)
    latent_scaling = (ls / (ls - np.float32(1.0)) * np.float32(2.0)).astype(np.float32)
    return poses, focal, c, image_shape, latent_scaling


def field_from_meta(g):
    """Rebuild (params_coarse, params_fine, latent (1,L,H,W)) for a golden
    fixture written by tests/golden/make_golden.py.build_field."""
    d_hidden, n_blocks, combine = int(g["d_hidden"]), int(g["n_blocks"]), int(g["combine_layer"])
    L, d_in = int(g["d_latent"]), int(g["d_in"])
    hw = tuple(int(v) for v in g["latent_hw"])
    if "coarse.lin_in.weight" in g:
        pc = {k[len("coarse."):]: g[k] for k in g if k.startswith("coarse.")}
        pf = {k[len("fine."):]: g[k] for k in g if k.startswith("fine.")}
        latent = g["latent"]
    else:
        spade = bool(int(g["spade"])) if "spade" in g else False
        pc = resnetfc_params(d_in, L, d_hidden, n_blocks, combine, int(g["weight_seed_coarse"]), spade=spade)
        pf = resnetfc_params(d_in, L, d_hidden, n_blocks, combine, int(g["weight_seed_fine"]), spade=spade)
        ns = int(g["ns"]) if "ns" in g else 1
        latent = hashed_normalish((ns, L) + hw, int(g["latent_seed"]), 1.0)
    # eval-mode BatchNorm statistics / affine of bn=True nets (stored explicitly in the fixture)
    for tag, p in (("coarse", pc), ("fine", pf)):
        pre = f"bn_{tag}."
        p.update({k[len(pre):]: g[k] for k in g if k.startswith(pre)})
    return pc, pf, latent


def bn_params(d_hidden, n_blocks, seed):
    """Non-trivial eval BatchNorm1d state for every block's bn_0 / bn_1 (the
    reference creates both; only bn_0 is applied, models.py:456-461): weights
    of both signs, shifts, running means and variances."""
    p = {}
    for b in range(n_blocks):
        for m in ("bn_0", "bn_1"):
            s = seed * 100 + 10 * b + (0 if m == "bn_0" else 5)
            w = hashed_uniform((d_hidden,), s + 1, 0.5, 1.5)
            sign = np.where(hashed_uniform((d_hidden,), s + 2) < 0.1, -1.0, 1.0).astype(np.float32)
            p[f"blocks.{b}.{m}.weight"] = (w * sign).astype(np.float32)
            p[f"blocks.{b}.{m}.bias"] = hashed_uniform((d_hidden,), s + 3, -0.2, 0.2)
            p[f"blocks.{b}.{m}.running_mean"] = hashed_uniform((d_hidden,), s + 4, -0.3, 0.3)
            p[f"blocks.{b}.{m}.running_var"] = hashed_uniform((d_hidden,), s + 5, 0.3, 2.0)
    return p
