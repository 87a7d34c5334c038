"""Float64 restatement of NewPixelNeRFNet.forward (models.py:739-863) for default.conf-style nets (ReLU
ResnetFC, NS = 1, no BatchNorm / use_spade): the exact result both fp32 implementations -- the HIP field and
the reference-order numpy oracle (avr_oracle.PixelNeRFField) -- are measured against.

TEST INFRASTRUCTURE ONLY (tests/, scripts/ diagnostics): the product never imports it.

Follows the reference's operation order, every step in float64:
  camera point  xyz_rot = R xyz, xyz_c = xyz_rot + t                         models.py:753-758
  z_feature     [xyz_rot, sin(f_k xyz_rot + phase)..., R viewdir]           models.py:41-87, 761-789
  latent        uv = -xyz_c[:2] / xyz_c[2] * focal + c, grid = uv * latent_scaling / image_shape - 1,
                grid_sample bilinear / border / align_corners=True            models.py:796-806, :260-273
  ResnetFC      lin_in, blocks (x += lin_z[b](latent) for b < combine_layer; x += fc_1(relu(fc_0(relu(x))))),
                lin_out(relu(x))                                              models.py:541-592, :454-470
  output        sigmoid(rgb), relu(sigma)                                     models.py:856-862
"""
import numpy as np

F64 = np.float64


def field64(sd, latent_chw, pose, focal, c, image_shape, latent_scaling, xyz, viewdirs, n_blocks=3,
            combine_layer=3, num_freqs=6, freq_factor=1.5):
    """sd: the ResnetFC state dict (numpy); latent_chw (L, H, W); pose (3, 4) world -> camera; xyz, viewdirs
    (N, 3) -> (N, 4) float64."""
    R, t = np.asarray(pose, F64)[:, :3], np.asarray(pose, F64)[:, 3]
    x = np.asarray(xyz, F64).reshape(-1, 3)
    xr = x @ R.T
    xc = xr + t
    fr = np.repeat(freq_factor * 2.0 ** np.arange(num_freqs), 2)
    ph = np.zeros(2 * num_freqs)
    ph[1::2] = np.pi / 2
    emb = np.sin(xr[:, None, :] * fr[None, :, None] + ph[None, :, None]).reshape(len(x), -1)
    zf = np.concatenate([xr, emb, np.asarray(viewdirs, F64).reshape(-1, 3) @ R.T], -1)
    lat = np.asarray(latent_chw, F64)
    L, H, W = lat.shape
    uv = -xc[:, :2] / xc[:, 2:] * np.asarray(focal, F64).reshape(2) + np.asarray(c, F64).reshape(2)
    g = uv * (np.asarray(latent_scaling, F64) / np.asarray(image_shape, F64)) - 1.0
    ix = np.clip((g[:, 0] + 1) / 2 * (W - 1), 0, W - 1)
    iy = np.clip((g[:, 1] + 1) / 2 * (H - 1), 0, H - 1)
    x0, y0 = np.floor(ix), np.floor(iy)
    wx1, wy1 = ix - x0, iy - y0
    wx0, wy0 = 1 - wx1, 1 - wy1
    x0i, y0i = x0.astype(np.int64), y0.astype(np.int64)
    x1i, y1i = np.minimum(x0i + 1, W - 1), np.minimum(y0i + 1, H - 1)
    rows = lat.reshape(L, H * W).T
    z = (rows[y0i * W + x0i] * (wx0 * wy0)[:, None] + rows[y0i * W + x1i] * (wx1 * wy0)[:, None]
         + rows[y1i * W + x0i] * (wx0 * wy1)[:, None] + rows[y1i * W + x1i] * (wx1 * wy1)[:, None])

    def lin(v, name):
        return v @ np.asarray(sd[name + ".weight"], F64).T + np.asarray(sd[name + ".bias"], F64)

    h = lin(zf, "lin_in")
    for b in range(n_blocks):
        if b < combine_layer:
            h = h + lin(z, f"lin_z.{b}")
        net = lin(np.maximum(h, 0), f"blocks.{b}.fc_0")
        h = h + lin(np.maximum(net, 0), f"blocks.{b}.fc_1")
    out = lin(np.maximum(h, 0), "lin_out")
    return np.concatenate([1 / (1 + np.exp(-out[:, :3])), np.maximum(out[:, 3:4], 0)], -1)
