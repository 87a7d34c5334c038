"""CPU oracle: a numpy restatement of the reference's coarse/fine volume-rendering
hot path (yankeesong/adaptive-volume-rendering, renderers.py / models.py / utils.py).

TEST INFRASTRUCTURE ONLY — the checker for the HIP path and the timed CPU
baseline ("kind": "port") in bench.py. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it. The product never does.

Parity pinning: every function below is checked against golden vectors that
tests/golden/make_golden.py produced by importing the reference itself in the
build container (torch 2.10.0 CPU, AVX512). See tests/test_oracle_golden.py.

Numerics contract restated here:
  * torch-CPU fp32 `sum` over a row = fixed 8-lane x ILP-4 cascade (cascade_sum).
  * torch-CPU fp32 `cumsum` / `cumprod` accumulate sequentially in fp64 and round
    each prefix to fp32 (cumsum_f64 / cumprod_f64).
  * everything else is plain fp32 elementwise arithmetic in the reference's
    operation order; contractions (einsum/bmm/addmm) are matched to tolerance.
"""
import numpy as np

F32 = np.float32


# ----------------------------------------------------------------------------- reductions
def cascade_sum(x):
    """torch.sum(x, -1) for fp32 on the CPU (used at renderers.py:37 and :111).

    Row split into 8-wide vectors v_k = x[8k:8k+8]; four accumulators take
    v_{4i+j} (j = 0..3) in order over full groups of four; leftover vectors go to
    acc0; acc = ((acc0+acc1)+acc2)+acc3; then the tail elements (N mod 8) are
    summed sequentially, followed by the 8 lanes of acc in order.
    Pinned bit-exact for N >= 8 (g0_reductions.npz); N < 8 is not pinned."""
    x = np.asarray(x, F32)
    lead, N = x.shape[:-1], x.shape[-1]
    x2 = x.reshape(-1, N)
    R = x2.shape[0]
    nvec = N // 8
    acc = np.zeros((4, R, 8), F32)
    nfull = (nvec // 4) * 4
    for i in range(0, nfull, 4):
        for j in range(4):
            acc[j] = acc[j] + x2[:, 8 * (i + j):8 * (i + j) + 8]
    for i in range(nfull, nvec):
        acc[0] = acc[0] + x2[:, 8 * i:8 * i + 8]
    a = ((acc[0] + acc[1]) + acc[2]) + acc[3]
    s = np.zeros(R, F32)
    for k in range(nvec * 8, N):
        s = s + x2[:, k]
    for lane in range(8):
        s = s + a[:, lane]
    return s.reshape(lead)


def cumsum_f64(x):
    """torch.cumsum(fp32, -1) on CPU: fp64 running sum, each prefix rounded to fp32."""
    return np.cumsum(np.asarray(x, F32).astype(np.float64), axis=-1).astype(F32)


def cumprod_f64(x):
    """torch.cumprod(fp32, -1) on CPU: fp64 running product, each prefix rounded to fp32."""
    return np.cumprod(np.asarray(x, F32).astype(np.float64), axis=-1).astype(F32)


def _dot_f64(a, b, axis):
    """Contraction to tolerance (einsum/bmm order is not part of the contract)."""
    return np.sum(a.astype(np.float64) * b.astype(np.float64), axis=axis).astype(F32)


# ----------------------------------------------------------------------------- geometry
def get_world_rays(x_pix, K, c2w):
    """utils.py:315-336 (+ unproject :246-267, get_normalized_cam_ray_directions
    :309-312, homogenize_* :220-243, transform_rigid :297-307).
    x_pix (SB,R,2), K (SB,3,3), c2w (SB,R,4,4) -> ro, rd (SB,R,3)."""
    x_pix = np.asarray(x_pix, F32)
    K = np.asarray(K, F32)
    c2w = np.broadcast_to(np.asarray(c2w, F32), x_pix.shape[:-1] + (4, 4))
    Kinv = np.linalg.inv(K.astype(np.float64)).astype(F32)           # (SB,3,3)
    hom = np.concatenate([x_pix, np.ones_like(x_pix[..., :1])], -1)   # (SB,R,3)
    cam = np.einsum("bij,bkj->bki", Kinv.astype(np.float64), hom.astype(np.float64)).astype(F32)
    cam[..., 0] = -cam[..., 0]
    cam = cam * F32(-1.0)
    nrm = np.sqrt(np.sum(cam.astype(np.float64) ** 2, -1)).astype(F32)
    d = cam / nrm[..., None]
    rd = _dot_f64(c2w[..., :3, :3], d[..., None, :], axis=-1)         # R_c2w . d (+ 0 * t)
    ro = np.ascontiguousarray(c2w[..., :3, 3])
    return ro, rd


def depth_from_world(world, c2w):
    """utils.py:358-361 via transform_world2cam :270-281 (torch.inverse per ray)."""
    world = np.asarray(world, F32)
    c2w = np.broadcast_to(np.asarray(c2w, F32), world.shape[:-1] + (4, 4))
    w2c = np.linalg.inv(c2w.astype(np.float64))
    hom = np.concatenate([world, np.ones_like(world[..., :1])], -1).astype(np.float64)
    cam_z = np.sum(w2c[..., 2, :] * hom, -1)
    return (-cam_z).astype(F32)


def opencv_pixel_coordinates(y_res, x_res):
    """utils.py:339-356 (quirk Q8: x_resolution spacing on both axes, top-left corners)."""
    xs = np.linspace(0, 1 - 1 / x_res, x_res).astype(F32)
    ys = np.linspace(0, 1 - 1 / x_res, y_res).astype(F32)
    i, j = np.meshgrid(xs, ys, indexing="ij")
    return np.stack([i, j], -1).transpose(1, 0, 2)


# ----------------------------------------------------------------------------- sampling
def sample_coarse(near, far, num_samples, noise):
    """renderers.py:4-24 (infinity == -1 branch). near/far (SB,R), noise (SB,R,N) U[0,1)."""
    near = np.asarray(near, F32)
    far = np.asarray(far, F32)
    steps = np.arange(num_samples, dtype=F32) / F32(num_samples)
    span = far - near
    z = near[..., None] + span[..., None] * steps
    z = z + (np.asarray(noise, F32) * span[..., None]) / F32(num_samples)
    return z.astype(F32)


def sample_fine(near, far, num_samples, weights, u, u2, return_idx=False):
    """renderers.py:27-54. weights (SB,R,Nc,1); u, u2 (SB,R,Nf) the two rand draws.
    idx = searchsorted(cdf, u, right=True) - 1, clamped >= 0 (may equal Nc: quirk Q5)."""
    w = np.asarray(weights, F32)[..., 0] + F32(1e-5)
    n_coarse = w.shape[-1]
    pdf = w / cascade_sum(w)[..., None]
    cdf = np.concatenate([np.zeros_like(pdf[..., :1]), cumsum_f64(pdf)], -1)
    u = np.asarray(u, F32)
    cnt = np.sum(cdf[..., None, :] <= u[..., :, None], axis=-1)
    idx = np.maximum(cnt.astype(F32) - F32(1.0), F32(0.0))
    steps = (idx + np.asarray(u2, F32)) / F32(n_coarse)
    near = np.asarray(near, F32)
    far = np.asarray(far, F32)
    z = near[..., None] + (far - near)[..., None] * steps
    z = z.astype(F32)
    return (z, idx.astype(np.int32)) if return_idx else z


def sample_depth(depth, num_samples, depth_std, noise):
    """renderers.py:56-66 — returns randn * std (quirk Q6: not depth + noise)."""
    d = np.asarray(depth, F32)
    return (np.asarray(noise, F32).reshape(d.shape[:-1] + (num_samples,)) * F32(depth_std)).astype(F32)


def volume_integral(z, sigma, rad, white_back=True, infinity=1.8):
    """renderers.py:69-119. z (SB,R,N), sigma (SB,R,N,1), rad (SB,R,N,3)
    -> rgb (SB,R,3), depth (SB,R,1), weights (SB,R,N,1)."""
    z = np.asarray(z, F32)
    s = np.asarray(sigma, F32)[..., 0]
    rad = np.asarray(rad, F32)
    dists = np.concatenate([z[..., 1:] - z[..., :-1], np.full_like(z[..., :1], 1e10)], -1)
    alpha = F32(1.0) - np.exp(-(s * dists))
    t = (F32(1.0) - alpha) + F32(1e-10)
    T = np.concatenate([np.ones_like(t[..., :1]), cumprod_f64(t)[..., :-1]], -1)
    w = alpha * T
    rgb = _dot_f64(w[..., None], rad, axis=-2)
    zz = np.concatenate([z[..., 1:], np.full_like(z[..., :1], infinity)], -1)
    depth = _dot_f64(w, zz, axis=-1)[..., None]
    if white_back:
        rgb = rgb + (F32(1.0) - cascade_sum(w))[..., None]
    return rgb.astype(F32), depth.astype(F32), w[..., None].astype(F32)


# ----------------------------------------------------------------------------- field
def positional_encoding(x, num_freqs=6, freq_factor=1.5, include_input=True):
    """models.py:41-87: [x, sin(f_k x + 0), sin(f_k x + pi/2), ...] with the
    (freq-pair, dim) flattening order of embed.view(B, -1)."""
    x = np.asarray(x, F32)
    freqs = (F32(freq_factor) * (F32(2.0) ** np.arange(num_freqs).astype(F32))).astype(F32)
    fr = np.repeat(freqs, 2)                                            # f0 f0 f1 f1 ...
    ph = np.zeros(2 * num_freqs, F32)
    ph[1::2] = F32(np.pi * 0.5)
    emb = np.sin(ph[None, :, None] + x[:, None, :] * fr[None, :, None]).astype(F32)
    emb = emb.reshape(x.shape[0], -1)
    return np.concatenate([x, emb], -1) if include_input else emb


def grid_sample_bilinear_border(latent, uv, latent_scaling, image_shape, rows=None):
    """SpatialEncoder.index (models.py:245-274): uv*scale - 1, then
    F.grid_sample(bilinear, padding=border, align_corners=True).
    latent (L,H,W), uv (B,2) -> (B,L). `rows` is the same latent as (H*W, L)
    texel rows (a layout cache: the gathers then read contiguous rows)."""
    latent = np.asarray(latent, F32)
    L, H, W = latent.shape
    if rows is None:
        rows = np.ascontiguousarray(latent.reshape(L, H * W).T)
    scale = (np.asarray(latent_scaling, F32) / np.asarray(image_shape, F32)).astype(F32)
    g = (np.asarray(uv, F32) * scale - F32(1.0)).astype(F32)
    ix = ((g[:, 0] + F32(1)) / F32(2)) * F32(W - 1)
    iy = ((g[:, 1] + F32(1)) / F32(2)) * F32(H - 1)
    ix = np.clip(ix, F32(0), F32(W - 1))
    iy = np.clip(iy, F32(0), F32(H - 1))
    x0 = np.floor(ix)
    y0 = np.floor(iy)
    x1, y1 = x0 + F32(1), y0 + F32(1)
    wx1, wy1 = ix - x0, iy - y0
    wx0, wy0 = x1 - ix, y1 - iy
    out = np.zeros((uv.shape[0], L), np.float64)
    for xx, yy, ww in ((x0, y0, wx0 * wy0), (x1, y0, wx1 * wy0), (x0, y1, wx0 * wy1), (x1, y1, wx1 * wy1)):
        ok = (xx <= W - 1) & (yy <= H - 1)
        xi = np.minimum(xx, W - 1).astype(np.int64)
        yi = np.minimum(yy, H - 1).astype(np.int64)
        out += np.where(ok, ww, 0).astype(np.float64)[:, None] * rows[yi * W + xi]   # fp64 accumulate
    return out.astype(F32)


def _linear(x, W, b):
    y = np.asarray(x, F32) @ np.asarray(W, F32).T
    return np.add(y, np.asarray(b, F32), out=y)


def batch_norm_eval(x, p, prefix, eps=1e-5):
    """nn.BatchNorm1d in eval mode on (B, C) as ATen's CPU kernel evaluates it:
    alpha = weight / sqrt(running_var + eps), beta = bias - running_mean * alpha,
    y = x * alpha + beta (fp32)."""
    invstd = (F32(1) / np.sqrt(np.asarray(p[prefix + ".running_var"], F32) + F32(eps))).astype(F32)
    alpha = (invstd * np.asarray(p[prefix + ".weight"], F32)).astype(F32)
    beta = (np.asarray(p[prefix + ".bias"], F32) - np.asarray(p[prefix + ".running_mean"], F32) * alpha).astype(F32)
    return (np.asarray(x, F32) * alpha + beta).astype(F32)


def softplus(v, beta):
    """nn.Softplus(beta) (threshold 20) as ATen evaluates it in fp32:
    x where x * beta > 20, else log1p(exp(x * beta)) / beta."""
    v = np.asarray(v, F32)
    bx = (v * F32(beta)).astype(F32)
    with np.errstate(over="ignore"):
        sp = (np.log1p(np.exp(bx)) / F32(beta)).astype(F32)
    return np.where(bx > F32(20), v, sp).astype(F32)


def combine_interleaved(x, ns, agg_type="average"):
    """utils.py:71-81 for one object: rows (ns, B) -> (B): mean or max over the source views
    (fp32; the views are summed in order, then divided, as ATen's CPU mean does for small ns)."""
    x = np.asarray(x, F32).reshape(ns, -1, x.shape[-1])
    if agg_type == "average":
        acc = x[0].copy()
        for v in range(1, ns):
            acc = (acc + x[v]).astype(F32)
        return (acc / F32(ns)).astype(F32)
    if agg_type == "max":
        return x.max(axis=0)
    raise NotImplementedError(agg_type)


def resnetfc_forward(zx, p, d_latent, n_blocks, combine_layer, beta=0.0, ns=1, combine_type="average"):
    """ResnetFC.forward (models.py:541-592) with ResnetBlockFC (:454-470),
    NS=1 (combine_interleaved is the identity). beta > 0: every ReLU is
    Softplus(beta) (models.py:442-445, 536-537). With scale_z parameters in `p`
    (use_spade, :528-534) block b < combine_layer starts from
    scale_z[b](z) * x + lin_z[b](z) (:585-587). With bn parameters in `p`
    (train.py --bn, eval mode) every block applies bn_0 in front of BOTH relus,
    as the reference does (models.py:456-461: bn_1 unused). ns > 1: rows are
    (source view, point) of one object; block combine_layer starts from the
    views' combine (models.py:566-579)."""
    z = zx[:, :d_latent]
    x = _linear(zx[:, d_latent:], p["lin_in.weight"], p["lin_in.bias"])
    if beta > 0:
        relu = lambda v: softplus(v, beta)  # noqa: E731
    else:
        relu = lambda v: np.maximum(v, F32(0))  # noqa: E731
    for b in range(n_blocks):
        if b == combine_layer and ns > 1:
            x = combine_interleaved(x, ns, combine_type)
        if d_latent > 0 and b < combine_layer:
            tz = _linear(z, p[f"lin_z.{b}.weight"], p[f"lin_z.{b}.bias"])
            if f"scale_z.{b}.weight" in p:
                x = (_linear(z, p[f"scale_z.{b}.weight"], p[f"scale_z.{b}.bias"]) * x).astype(F32) + tz
            else:
                x = x + tz
        bn = f"blocks.{b}.bn_0"
        if bn + ".running_mean" in p:
            net = _linear(relu(batch_norm_eval(x, p, bn)), p[f"blocks.{b}.fc_0.weight"], p[f"blocks.{b}.fc_0.bias"])
            dx = _linear(relu(batch_norm_eval(net, p, bn)), p[f"blocks.{b}.fc_1.weight"], p[f"blocks.{b}.fc_1.bias"])
        else:
            net = _linear(relu(x), p[f"blocks.{b}.fc_0.weight"], p[f"blocks.{b}.fc_0.bias"])
            dx = _linear(relu(net), p[f"blocks.{b}.fc_1.weight"], p[f"blocks.{b}.fc_1.bias"])
        x = x + dx
    return _linear(relu(x), p["lin_out.weight"], p["lin_out.bias"])


class PixelNeRFField:
    """NewPixelNeRFNet.forward (models.py:739-863) for default.conf-style
    configs: use_encoder, use_xyz, normalize_z, use_code (PE on xyz only),
    use_viewdirs without PE, no global encoder, NS = 1."""

    def __init__(self, params_coarse, params_fine, latent, poses, focal, c, image_shape, latent_scaling,
                 n_blocks=3, combine_layer=1000, num_freqs=6, freq_factor=1.5, beta=0.0):
        self.pc, self.pf = params_coarse, params_fine
        self.latent = np.asarray(latent, F32).reshape(np.asarray(latent).shape[-3:])
        L_, H_, W_ = self.latent.shape
        self.latent_rows = np.ascontiguousarray(self.latent.reshape(L_, H_ * W_).T)   # (H*W, L) texel rows
        self.poses = np.asarray(poses, F32).reshape(3, 4)
        self.focal = np.asarray(focal, F32).reshape(2)
        self.c = np.asarray(c, F32).reshape(2)
        self.image_shape = np.asarray(image_shape, F32)
        self.latent_scaling = np.asarray(latent_scaling, F32)
        self.n_blocks, self.combine_layer = n_blocks, combine_layer
        self.num_freqs, self.freq_factor = num_freqs, freq_factor
        self.beta = beta
        self.d_latent = self.latent.shape[0]

    def features(self, xyz, viewdirs):
        """Everything before the MLP: returns (latent (B,L), z_feature (B,42))."""
        xyz = np.asarray(xyz, F32).reshape(-1, 3)
        Rm, t = self.poses[:, :3], self.poses[:, 3]
        xyz_rot = _dot_f64(Rm[None], xyz[:, None, :], axis=-1)
        xyz_c = xyz_rot + t
        zf = positional_encoding(xyz_rot, self.num_freqs, self.freq_factor)
        vd = _dot_f64(Rm[None], np.asarray(viewdirs, F32).reshape(-1, 3)[:, None, :], axis=-1)
        zf = np.concatenate([zf, vd], -1)
        uv = -xyz_c[:, :2] / xyz_c[:, 2:]
        uv = uv * self.focal + self.c
        lat = grid_sample_bilinear_border(self.latent, uv, self.latent_scaling, self.image_shape, self.latent_rows)
        return lat, zf

    def __call__(self, xyz, viewdirs, coarse=True):
        shp = np.asarray(xyz).shape
        lat, zf = self.features(xyz, viewdirs)
        p = self.pc if coarse else self.pf
        out = resnetfc_forward(np.concatenate([lat, zf], -1), p, self.d_latent, self.n_blocks, self.combine_layer,
                               self.beta)
        res = np.concatenate([1.0 / (1.0 + np.exp(-out[:, :3].astype(np.float64))), np.maximum(out[:, 3:4], 0)], -1)
        return res.astype(F32).reshape(shp[:-1] + (4,))


class MultiViewField:
    """NewPixelNeRFNet.forward with NS > 1 source views of one object (models.py:749-853):
    every point is transformed into each view (pose v, the object's focal / principal point,
    view v's latent map), the MLP runs on the (view, point) rows and combines the views at
    combine_layer."""

    def __init__(self, params_coarse, params_fine, latents, poses, focal, c, image_shape, latent_scaling,
                 n_blocks=3, combine_layer=1000, combine_type="average", num_freqs=6, freq_factor=1.5, beta=0.0):
        latents = np.asarray(latents, F32)
        self.views = [PixelNeRFField(params_coarse, params_fine, latents[v], np.asarray(poses, F32)[v], focal, c,
                                     image_shape, latent_scaling, n_blocks, combine_layer, num_freqs, freq_factor,
                                     beta) for v in range(latents.shape[0])]
        self.pc, self.pf = params_coarse, params_fine
        self.n_blocks, self.combine_layer, self.combine_type, self.beta = n_blocks, combine_layer, combine_type, beta
        self.d_latent = latents.shape[1]

    def __call__(self, xyz, viewdirs, coarse=True):
        shp = np.asarray(xyz).shape
        rows = [np.concatenate(f.features(xyz, viewdirs), -1) for f in self.views]
        p = self.pc if coarse else self.pf
        out = resnetfc_forward(np.concatenate(rows, 0), p, self.d_latent, self.n_blocks, self.combine_layer, self.beta,
                               ns=len(self.views), combine_type=self.combine_type)
        res = np.concatenate([1.0 / (1.0 + np.exp(-out[:, :3].astype(np.float64))), np.maximum(out[:, 3:4], 0)], -1)
        return res.astype(F32).reshape(shp[:-1] + (4,))


# ----------------------------------------------------------------------------- renderer
def render(cam2world, intrinsics, x_pix, field, near, far, n_coarse, n_fine, n_fine_depth, depth_std,
           white_back, noise_coarse, u, u2, noise_depth, return_aux=False):
    """VolumeRenderer.forward (renderers.py:133-277) with explicit noise tensors
    (draw order: rand_like coarse, rand u, rand_like u2, randn_like depth).
    Returns (rgb_coarse (SB,R,3), rgb_fine (SB,R,3), depth (SB,R), depth)."""
    x_pix = np.asarray(x_pix, F32)
    SB, R, _ = x_pix.shape
    ro, rd = get_world_rays(x_pix, intrinsics, cam2world)
    nearv = np.full((SB, R), near, F32)
    farv = np.full((SB, R), far, F32)
    zc = sample_coarse(nearv, farv, n_coarse, noise_coarse)
    pts = ro[..., None, :] + rd[..., None, :] * zc[..., None]
    vd = np.broadcast_to(rd[..., None, :], pts.shape)
    fc = field(pts.reshape(SB, -1, 3), vd.reshape(SB, -1, 3), coarse=True).reshape(SB, R, n_coarse, 4)
    rgb_c, dist_c, w_c = volume_integral(zc, fc[..., 3:4], fc[..., :3], white_back)
    zf, idx = sample_fine(nearv, farv, n_fine - n_fine_depth, w_c, u, u2, return_idx=True)
    zd = sample_depth(dist_c, n_fine_depth, depth_std, noise_depth)
    zd = np.minimum(np.maximum(zd, F32(near)), F32(far))
    zs = np.sort(np.concatenate([zc, zf, zd], -1), -1)
    N = zs.shape[-1]
    pts = ro[..., None, :] + rd[..., None, :] * zs[..., None]
    vd = np.broadcast_to(rd[..., None, :], pts.shape)
    ff = field(pts.reshape(SB, -1, 3), vd.reshape(SB, -1, 3), coarse=False).reshape(SB, R, N, 4)
    rgb_f, dist_f, _ = volume_integral(zs, ff[..., 3:4], ff[..., :3], white_back)
    world = ro + rd * dist_f
    depth = depth_from_world(world, cam2world)
    if return_aux:
        aux = dict(z_coarse=zc, field_coarse=fc, weights_coarse=w_c, dist_coarse=dist_c, idx=idx, z_fine=zf,
                   z_sorted=zs, field_fine=ff, dist_fine=dist_f, ro=ro, rd=rd)
        return rgb_c, rgb_f, depth, depth, aux
    return rgb_c, rgb_f, depth, depth


# ----------------------------------------------------------------------------- adaptive renderer
def _sigmoid(x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(F32)


def lstm_cell(x, h, c, w_ih, w_hh, b_ih, b_hh):
    """torch.nn.LSTMCell: gates = x W_ih^T + b_ih + h W_hh^T + b_hh, order i f g o."""
    x = np.asarray(x, F32)
    gates = ((x @ np.asarray(w_ih, F32).T).astype(F32) + b_ih) + ((h @ np.asarray(w_hh, F32).T).astype(F32) + b_hh)
    H = h.shape[-1]
    i, f, g, o = (gates[:, k * H:(k + 1) * H] for k in range(4))
    i, f, o = _sigmoid(i), _sigmoid(f), _sigmoid(o)
    g = np.tanh(g.astype(np.float64)).astype(F32)
    c2 = (f * c + i * g).astype(F32)
    h2 = (o * np.tanh(c2.astype(np.float64)).astype(F32)).astype(F32)
    return h2, c2


def raymarch(ro, rd, init_dist, field, lstm, out_w, out_b, steps):
    """The LSTM march of Raymarcher / AdaptiveVolumeRenderer (renderers.py:320-343,
    :404-432): x = ro + rd d0; steps x {v = latent at x (return_features=True,
    models.py:822-823); (h, c) = LSTMCell(v); sd = out_layer(h); x += rd sd}.
    ro, rd (R,3), init_dist (R,1); lstm = (w_ih, w_hh, b_ih, b_hh).
    Returns the list of x per step (steps + 1 entries)."""
    R = ro.shape[0]
    x = (ro + rd * init_dist).astype(F32)
    h = np.zeros((R, 16), F32)
    c = np.zeros((R, 16), F32)
    trace = [x]
    for _ in range(steps):
        v, _ = field.features(x, rd)
        h, c = lstm_cell(v, h, c, *lstm)
        sd = ((h @ np.asarray(out_w, F32).reshape(1, 16).T).astype(F32) + np.asarray(out_b, F32)).astype(F32)
        x = (x + rd * sd).astype(F32)
        trace.append(x)
    return trace


def adaptive_render(cam2world, intrinsics, x_pix, field, lstm, out_w, out_b, steps, epsilon, n_coarse, white_back,
                    init_dist, band_noise):
    """AdaptiveVolumeRenderer.forward (renderers.py:380-547) with explicit noise:
    init_dist (SB,R,1) ~ N(0.8, 0.05) and the band's rand_like (SB,R,n_coarse).
    Returns (rgb_coarse, rgb, depth_coarse (SB,R,1), depth_map (SB,R), trace)."""
    x_pix = np.asarray(x_pix, F32)
    SB, R, _ = x_pix.shape
    assert SB == 1
    ro, rd = get_world_rays(x_pix, intrinsics, cam2world)
    trace = raymarch(ro[0], rd[0], np.asarray(init_dist, F32)[0], field, lstm, out_w, out_b, steps)
    world = trace[-1][None]
    out_c = field(world, rd, coarse=True)
    rgb_coarse = out_c[..., :3]
    depth_coarse = depth_from_world(world, cam2world)[..., None]
    fd = ((world[..., 0] - ro[..., 0]) / rd[..., 0]).astype(F32)
    z = sample_coarse((fd - F32(epsilon)).astype(F32), (fd + F32(epsilon)).astype(F32), n_coarse, band_noise)
    z = np.sort(z, -1)
    pts = ro[..., None, :] + rd[..., None, :] * z[..., None]
    vd = np.broadcast_to(rd[..., None, :], pts.shape)
    f = field(pts.reshape(SB, -1, 3), vd.reshape(SB, -1, 3), coarse=False).reshape(SB, R, n_coarse, 4)
    rgb, dist, _ = volume_integral(z, f[..., 3:4], f[..., :3], white_back)
    depth_map = depth_from_world(ro + rd * dist, cam2world)
    return rgb_coarse, rgb, depth_coarse, depth_map, trace
