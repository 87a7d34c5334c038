#!/usr/bin/env python
"""Generate the golden vectors in tests/golden/*.npz by importing the reference.

Runs ONLY in the build container, where the read-only reference lives at
/root/reference (it never travels to the GPU box). The reference's module-scope
imports that the hot path never calls (torchvision, lpips, gdown, h5py,
imageio, skimage, dotmap, pyhocon) are absent here, so they are replaced by
empty stub modules before `import utils, renderers, models`.

Every torch RNG draw the reference makes (torch.rand / rand_like / randn_like)
and every torch.searchsorted result is captured by thin wrappers so the
fixtures hold the exact noise and the exact integer sample indices.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("AVR_REFERENCE", "/root/reference")
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
from oracle import synth  # noqa: E402


# --------------------------------------------------------------------------- stubs
def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _FakeResnet(torch.nn.Module):
    """Stands in for torchvision.models.resnet34: the encoder is per-scene and
    out of scope; the latent map is injected directly."""

    def __init__(self, *a, **k):
        super().__init__()
        self.fc = torch.nn.Sequential()
        self.avgpool = torch.nn.Sequential()


def install_stubs():
    tv = _stub("torchvision")
    tv.datasets = _stub("torchvision.datasets")
    tv.transforms = _stub("torchvision.transforms")
    tv.models = _stub("torchvision.models", resnet34=_FakeResnet, resnet18=_FakeResnet)
    _stub("lpips")
    _stub("gdown")
    _stub("h5py")
    _stub("imageio")
    sk = _stub("skimage")
    sk.transform = _stub("skimage.transform", resize=lambda *a, **k: None)
    sk.metrics = _stub("skimage.metrics")
    _stub("dotmap", DotMap=dict)
    _stub("pyhocon", ConfigFactory=None)


class Conf(dict):
    """Minimal pyhocon ConfigTree stand-in (get_int/get_float/get_bool/get_string)."""

    def _g(self, k, d):
        cur = self
        for part in k.split("."):
            if not isinstance(cur, dict) or part not in cur:
                return d
            cur = cur[part]
        return cur

    def get_int(self, k, d=None):
        return int(self._g(k, d))

    def get_float(self, k, d=None):
        return float(self._g(k, d))

    def get_bool(self, k, d=None):
        return bool(self._g(k, d))

    def get_string(self, k, d=None):
        return str(self._g(k, d))

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        return Conf(v) if isinstance(v, dict) and not isinstance(v, Conf) else v


def model_conf(d_hidden, n_blocks, combine_layer, num_layers, spade=False, beta=0.0):
    mlp = {"type": "resnet", "n_blocks": n_blocks, "d_hidden": d_hidden, "combine_layer": combine_layer}
    if spade:
        mlp["use_spade"] = True
    if beta > 0:
        mlp["beta"] = beta
    return Conf({
        "use_encoder": True, "use_global_encoder": False, "use_xyz": True, "canon_xyz": False,
        "use_code": True, "code": {"num_freqs": 6, "freq_factor": 1.5, "include_input": True},
        "use_viewdirs": True, "use_code_viewdirs": False,
        "mlp_coarse": dict(mlp), "mlp_fine": dict(mlp),
        "encoder": {"backbone": "resnet34", "pretrained": False, "num_layers": num_layers},
    })


# --------------------------------------------------------------------------- capture
class Capture:
    def __init__(self):
        self.log = []
        self._orig = {}
        self.inject = {}

    def __enter__(self):
        for name in ("rand", "rand_like", "randn_like", "searchsorted"):
            orig = getattr(torch, name)
            self._orig[name] = orig

            def wrap(*a, _orig=orig, _name=name, **k):
                if _name in self.inject and self.inject[_name]:
                    out = self.inject[_name].pop(0).clone()
                else:
                    out = _orig(*a, **k)
                self.log.append((_name, out.detach().clone()))
                return out

            setattr(torch, name, wrap)
        return self

    def __exit__(self, *exc):
        for name, orig in self._orig.items():
            setattr(torch, name, orig)

    def get(self, name):
        return [t for n, t in self.log if n == name]


def import_reference():
    install_stubs()
    sys.path.insert(0, REF)
    import utils as ref_utils  # noqa
    import renderers as ref_renderers  # noqa
    import models as ref_models  # noqa
    return ref_utils, ref_renderers, ref_models


def build_field(ref_models, d_hidden, n_blocks, combine_layer, num_layers, latent_hw, seed, store_weights, bn=False,
                spade=False, beta=0.0):
    net = ref_models.NewPixelNeRFNet(model_conf(d_hidden, n_blocks, combine_layer, num_layers, spade, beta), bn=bn)
    L = net.latent_size
    d_in = net.d_in
    params = {}
    for tag, mlp, s in (("coarse", net.mlp_coarse, seed), ("fine", net.mlp_fine, seed + 17)):
        p = synth.resnetfc_params(d_in, L, d_hidden, n_blocks, combine_layer, s, spade=spade)
        bnp = synth.bn_params(d_hidden, n_blocks, s) if bn else {}
        sd = mlp.state_dict()
        for k, v in list(p.items()) + list(bnp.items()):
            assert k in sd, k
            sd[k] = torch.from_numpy(v)
        assert all(k in p or ".bn_" in k for k in sd), [k for k in sd if k not in p]
        mlp.load_state_dict(sd)
        if store_weights:
            for k, v in p.items():
                params[f"{tag}.{k}"] = v
        for k, v in bnp.items():    # eval BatchNorm state: always stored (not hash-regenerated by the tests)
            params[f"bn_{tag}.{k}"] = v
    poses, focal, c, image_shape, latent_scaling = synth.source_view(latent_hw)
    latent = synth.hashed_normalish((1, L) + tuple(latent_hw), seed + 5, 1.0)
    net.encoder.latent = torch.from_numpy(latent)
    net.encoder.latent_scaling = torch.from_numpy(latent_scaling)
    net.poses = torch.from_numpy(poses)
    net.focal = torch.from_numpy(focal)
    net.c = torch.from_numpy(c)
    net.image_shape = torch.from_numpy(image_shape)
    net.num_views_per_obj = 1
    meta = dict(d_hidden=d_hidden, n_blocks=n_blocks, combine_layer=combine_layer, d_latent=L, d_in=d_in, bn=int(bn),
                latent_hw=np.array(latent_hw), weight_seed_coarse=seed, weight_seed_fine=seed + 17,
                latent_seed=seed + 5, poses=poses, focal=focal, c=c, image_shape=image_shape,
                latent_scaling=latent_scaling)
    if store_weights:
        meta["latent"] = latent
    if spade or beta > 0:   # (absent from the older fixtures: ReLU, no spade)
        meta["spade"] = int(spade)
        meta["beta"] = np.float32(beta)
    return net.eval(), meta, params


def provenance():
    return dict(torch_version=np.array(torch.__version__),
                cpu_capability=np.array(torch.backends.cpu.get_cpu_capability()))


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()}, **provenance())
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


# --------------------------------------------------------------------------- fixtures
def g0_reductions():
    """torch CPU sum / cumsum / cumprod on fp32 rows: pins the summation-order
    emulation."""
    out = {}
    for N in (7, 8, 20, 33, 56, 64, 120, 128, 192, 200):
        x = synth.hashed_uniform((32, N), 900 + N) * synth.hashed_uniform((32, 1), 950 + N, 0.0, 4.0)
        t = torch.from_numpy(x)
        out[f"x_{N}"] = x
        out[f"sum_{N}"] = torch.sum(t, -1).numpy()
        out[f"cumsum_{N}"] = torch.cumsum(t, -1).numpy()
        out[f"cumprod_{N}"] = torch.cumprod(t * 0.5 + 0.5, -1).numpy()
        out[f"sum4d_{N}"] = t.reshape(1, 32, N, 1).sum(dim=-2).reshape(32).numpy()
    save("g0_reductions.npz", **out)


def g1_volume_integral(R):
    out = {}
    for N in (64, 128, 192):
        for wb in (True, False):
            key = f"N{N}_wb{int(wb)}"
            seed = 10 * N + wb
            u = synth.hashed_uniform((1, R, N), seed)
            steps = (np.arange(N, dtype=np.float32) / np.float32(N)).astype(np.float32)
            z = (np.float32(0.8) + np.float32(1.0) * steps + u * np.float32(1.0 / N)).astype(np.float32)
            if N == 192:  # merged coarse+fine rays are sorted but irregular
                z = np.sort(np.concatenate([z[..., :128], synth.hashed_uniform((1, R, 64), seed + 1, 0.8, 1.8)], -1), -1)
            sig = synth.hashed_normalish((1, R, N, 1), seed + 2, 6.0)
            sig = np.maximum(sig, 0.0).astype(np.float32)
            sig[0, 0] = 0.0                        # all-zero sigma ray
            sig[0, 1, -1] = 0.0                    # last sample exactly 0
            sig[0, 2, -1] = 1e-30                  # last sample tiny (quirk Q2)
            sig[0, 3, :] = 0.0
            sig[0, 3, N // 2] = 1e4                # opaque spike
            rad = synth.hashed_uniform((1, R, N, 3), seed + 3)
            ts, tr = torch.from_numpy(sig).requires_grad_(True), torch.from_numpy(rad).requires_grad_(True)
            rgb, dmap, w = REF_R.volume_integral(torch.from_numpy(z), ts, tr, white_back=wb)
            g_rgb = synth.hashed_centered((1, R, 3), seed + 4, 2.0)
            g_dep = synth.hashed_centered((1, R, 1), seed + 5, 2.0)
            ((rgb * torch.from_numpy(g_rgb)).sum() + (dmap * torch.from_numpy(g_dep)).sum()).backward()
            out[f"{key}_z"], out[f"{key}_sigma"], out[f"{key}_rad"] = z, sig, rad
            out[f"{key}_rgb"], out[f"{key}_depth"] = rgb.detach().numpy(), dmap.detach().numpy()
            out[f"{key}_weights"] = w.detach().numpy()
            out[f"{key}_grad_rgb"], out[f"{key}_grad_depth"] = g_rgb, g_dep
            out[f"{key}_dsigma"], out[f"{key}_drad"] = ts.grad.numpy(), tr.grad.numpy()
    save("g1_volume_integral.npz", **out)


def g2_sample_fine(R):
    out = {}
    cases = []
    Nc, Nf = 64, 32
    # (a) weights from a volume integral of random sigma
    z = synth.hashed_uniform((1, R, Nc), 21, 0.8, 1.8)
    z = np.sort(z, -1)
    sig = np.maximum(synth.hashed_normalish((1, R, Nc, 1), 22, 6.0), 0).astype(np.float32)
    rad = synth.hashed_uniform((1, R, Nc, 3), 23)
    _, _, w = REF_R.volume_integral(torch.from_numpy(z), torch.from_numpy(sig), torch.from_numpy(rad))
    cases.append(("vi", w.numpy(), None))
    # (b) all-zero weights (uniform pdf)
    cases.append(("zero", np.zeros((1, R, Nc, 1), np.float32), None))
    # (c) arbitrary [0,1) weights (sum >> 1) and u landing exactly on cdf entries
    wc = synth.hashed_uniform((1, R, Nc, 1), 24)
    wt = torch.from_numpy(wc).squeeze(-1) + 1e-5
    cdf = torch.cumsum(wt / torch.sum(wt, -1, keepdim=True), -1)
    u = synth.hashed_uniform((1, R, Nf), 25)
    for r in range(R):
        for j in range(0, Nf, 3):
            k = int((r * 7 + j * 5) % Nc)
            if cdf[0, r, k] < 1.0:
                u[0, r, j] = cdf[0, r, k].item()
    cases.append(("exact", wc, u))
    # (d) sparse spiky weights: cdf[-1] may be < 1, u near 1 (quirk Q5)
    wd = np.zeros((1, R, Nc, 1), np.float32)
    wd[0, :, 5] = 0.7
    wd[0, :, 40, 0] = synth.hashed_uniform((R,), 26, 0.0, 0.3)
    ud = synth.hashed_uniform((1, R, Nf), 27, 0.999, 1.0)
    cases.append(("spiky", wd, ud))
    for i, (name, w, uu) in enumerate(cases):
        torch.manual_seed(2000 + i)        # the un-injected draws are reproducible from this recipe
        cap = Capture()
        if uu is not None:
            cap.inject["rand"] = [torch.from_numpy(uu)]
        with cap:
            zf = REF_R.sample_fine(torch.full((1, R), 0.8), torch.full((1, R), 1.8), Nf, torch.from_numpy(w),
                                   device=torch.device("cpu"))
        (u_,) = cap.get("rand")
        (u2,) = cap.get("rand_like")
        (ss,) = cap.get("searchsorted")
        out[f"{name}_weights"] = w
        out[f"{name}_u"] = u_.numpy()
        out[f"{name}_u2"] = u2.numpy()
        out[f"{name}_idx"] = np.maximum(ss.numpy().astype(np.int64) - 1, 0).astype(np.int32)
        out[f"{name}_z"] = zf.numpy()
    out["Nc"], out["Nf"], out["near"], out["far"] = Nc, Nf, np.float32(0.8), np.float32(1.8)
    save("g2_sample_fine.npz", **out)


def g3_geometry(R):
    x_pix = synth.hashed_uniform((1, R, 2), 31)
    K = synth.default_intrinsics()[None]
    c2w = np.stack([synth.orbit_cam2world(0.1 + 0.37 * i) for i in range(R)], 0)[None]
    ro, rd = REF_U.get_world_rays(torch.from_numpy(x_pix), torch.from_numpy(K), torch.from_numpy(c2w))
    dist = synth.hashed_uniform((1, R, 1), 32, 0.8, 1.8)
    world = ro + rd * torch.from_numpy(dist)
    depth = REF_U.depth_from_world(world, torch.from_numpy(c2w))
    # an un-normalised K (pixels) and a shared (stride-0) pose too
    K2 = np.array([[[131.25, 0, 64.0], [0, 131.25, 64.0], [0, 0, 1]]], np.float32)
    x2 = synth.hashed_uniform((1, R, 2), 33, 0.0, 128.0)
    c2w_one = synth.orbit_cam2world(2.0)
    c2w2 = torch.from_numpy(c2w_one).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    ro2, rd2 = REF_U.get_world_rays(torch.from_numpy(x2), torch.from_numpy(K2), c2w2)
    pix = REF_U.get_opencv_pixel_coordinates(8, 8)
    save("g3_geometry.npz", x_pix=x_pix, K=K, c2w=c2w, ro=ro.numpy(), rd=rd.numpy(), dist=dist,
         depth=depth.numpy(), x_pix2=x2, K2=K2, c2w_one=c2w_one, ro2=ro2.numpy(), rd2=rd2.numpy(),
         opencv_pix_8=pix.numpy())


def g4_field():
    B = 384
    for tag, (d_hidden, n_blocks, combine, num_layers, lhw, store) in {
        "small": (64, 3, 1000, 1, (8, 8), True),
        "small_mv": (64, 5, 3, 1, (8, 8), True),
        "full": (512, 3, 1000, 4, (64, 64), False),
        # conf/default_mv.conf:4-21 (5 x 512, combine_layer 3): train.py:262's config
        "mv512": (512, 5, 3, 4, (64, 64), False),
        "d256": (256, 3, 1000, 4, (64, 64), False),
        # train.py --bn (train.py:210, :265): eval-mode BatchNorm blocks, default.conf and default_mv.conf nets
        "bn_small": (64, 3, 1000, 1, (8, 8), True),
        "bn512": (512, 3, 1000, 4, (64, 64), False),
        "bn_mv512": (512, 5, 3, 4, (64, 64), False),
        # ResnetFC options no shipped conf sets (models.py:442-445 Softplus(beta), :528-534 use_spade)
        "spade_small": (64, 3, 1000, 1, (8, 8), True),
        "spade512": (512, 3, 1000, 4, (64, 64), False),
        "sp_small": (64, 3, 1000, 1, (8, 8), True),
        "sp512": (512, 3, 1000, 4, (64, 64), False),
        "spade_sp_mv": (64, 5, 3, 1, (8, 8), True),
    }.items():
        beta = {"sp_small": 3.0, "sp512": 100.0, "spade_sp_mv": 1.0}.get(tag, 0.0)
        net, meta, params = build_field(REF_M, d_hidden, n_blocks, combine, num_layers, lhw, 40, store,
                                        bn=tag.startswith("bn"), spade=tag.startswith("spade"), beta=beta)
        xyz = synth.hashed_uniform((1, B, 3), 41, -0.5, 0.5)
        vd = synth.hashed_uniform((1, B, 3), 42, -1.0, 1.0)
        vd /= np.linalg.norm(vd, axis=-1, keepdims=True).astype(np.float32)
        vd = vd.astype(np.float32)
        with torch.no_grad():
            oc = net(torch.from_numpy(xyz), coarse=True, viewdirs=torch.from_numpy(vd))
            of = net(torch.from_numpy(xyz), coarse=False, viewdirs=torch.from_numpy(vd))
            lat = net(torch.from_numpy(xyz), coarse=True, viewdirs=torch.from_numpy(vd), return_features=True)
        save(f"g4_field_{tag}.npz", xyz=xyz, viewdirs=vd, out_coarse=oc.numpy(), out_fine=of.numpy(),
             latent_at_points=lat.numpy()[:64], **meta, **params)


def g4_field_multiview():
    """NewPixelNeRFNet.forward with NS > 1 source views of one object (models.py:749-853): per-view
    poses rotated about the y axis, one latent map per view, the views combined at combine_layer."""
    B = 256
    for tag, (d_hidden, n_blocks, combine, num_layers, lhw, store, ns, ctype) in {
        "ns2_small": (64, 5, 3, 1, (8, 8), True, 2, "average"),
        "ns2max_small": (64, 4, 2, 1, (8, 8), True, 2, "max"),
        "ns3_mv512": (512, 5, 3, 4, (64, 64), False, 3, "average"),
    }.items():
        net, meta, params = build_field(REF_M, d_hidden, n_blocks, combine, num_layers, lhw, 40, store)
        for mlp in (net.mlp_coarse, net.mlp_fine):
            mlp.combine_type = ctype
        L = meta["d_latent"]
        latent = synth.hashed_normalish((ns, L) + tuple(lhw), 45, 1.0)
        poses = np.zeros((ns, 3, 4), np.float32)
        for v in range(ns):
            a = 0.35 * v
            poses[v, :3, :3] = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]], np.float32)
            poses[v, 2, 3] = 1.3
        net.encoder.latent = torch.from_numpy(latent)
        net.poses = torch.from_numpy(poses)
        net.num_views_per_obj = ns
        meta.update(ns=ns, combine_type=ctype, poses=poses, latent_seed=45)
        if store:
            meta["latent"] = latent
        xyz = synth.hashed_uniform((1, B, 3), 46, -0.5, 0.5)
        vd = synth.hashed_uniform((1, B, 3), 47, -1.0, 1.0)
        vd = (vd / np.linalg.norm(vd, axis=-1, keepdims=True)).astype(np.float32)
        with torch.no_grad():
            oc = net(torch.from_numpy(xyz), coarse=True, viewdirs=torch.from_numpy(vd))
            of = net(torch.from_numpy(xyz), coarse=False, viewdirs=torch.from_numpy(vd))
        assert oc.shape == (1, B, 4)
        save(f"g4_field_{tag}.npz", xyz=xyz, viewdirs=vd, out_coarse=oc.numpy(), out_fine=of.numpy(), **meta, **params)


def g5_forward(R):
    for tag, (Nc, Nf, Nd) in {"c64f32d16": (64, 32, 16), "c128f64d0": (128, 64, 0)}.items():
        net, meta, _ = build_field(REF_M, 512, 3, 1000, 4, (64, 64), 40, False)
        renderer = REF_R.VolumeRenderer(0.8, 1.8, Nc, Nf, Nd, 0.01, white_back=True)
        x_pix = synth.hashed_uniform((1, R, 2), 51)
        K = synth.default_intrinsics()[None]
        c2w = torch.from_numpy(synth.orbit_cam2world(0.7)).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
        field_log = []

        def rf(xyz, viewdirs=None, coarse=True, return_features=False):
            o = net(xyz, coarse=coarse, viewdirs=viewdirs)
            field_log.append(o.detach().clone())
            return o

        torch.manual_seed(1234)
        with Capture() as cap, torch.no_grad():
            rgb_c, rgb_f, depth, depth2 = renderer(c2w, torch.from_numpy(K), torch.from_numpy(x_pix), rf)
        noise_c = cap.get("rand_like")[0]
        u = cap.get("rand")[0]
        u2 = cap.get("rand_like")[1]
        nd = cap.get("randn_like")[0]
        (ss,) = cap.get("searchsorted")
        save(f"g5_forward_{tag}.npz", Nc=Nc, Nf=Nf, Nd=Nd, near=np.float32(0.8), far=np.float32(1.8),
             depth_std=np.float32(0.01), x_pix=x_pix, K=K, c2w_one=c2w[0, 0].numpy(),
             noise_coarse=noise_c.numpy(), u=u.numpy(), u2=u2.numpy(), noise_depth=nd.numpy(),
             idx=np.maximum(ss.numpy().astype(np.int64) - 1, 0).astype(np.int32),
             field_coarse=field_log[0].numpy(), field_fine=field_log[1].numpy(),
             rgb_coarse=rgb_c.numpy(), rgb_fine=rgb_f.numpy(), depth=depth.numpy(), **meta)
        assert depth2 is depth


def g6_adaptive(R):
    """AdaptiveVolumeRenderer.forward (renderers.py:380-547) on the small field
    (d_latent 64 -> num_feature_channels 64): LSTM parameters, the N(0.8, 0.05)
    initial distances, the band's rand_like, every point the LSTM queried, and
    the four outputs."""
    net, meta, params = build_field(REF_M, 64, 3, 1000, 1, (8, 8), 40, True)
    torch.manual_seed(77)
    avr = REF_R.AdaptiveVolumeRenderer(num_feature_channels=64, raymarch_steps=10, epsilon=0.05, n_coarse=20,
                                       white_back=True)
    x_pix = synth.hashed_uniform((1, R, 2), 61, 0.2, 0.8)
    K = synth.default_intrinsics()[None]
    c2w = torch.from_numpy(synth.orbit_cam2world(0.9)).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    queries = []

    def rf(xyz, viewdirs=None, coarse=True, return_features=False):
        queries.append((xyz.detach().clone(), return_features, coarse))
        return net(xyz, coarse=coarse, viewdirs=viewdirs, return_features=return_features)

    torch.manual_seed(1234)
    init = torch.zeros((1, R, 1)).normal_(mean=0.8, std=5e-2)
    torch.manual_seed(1234)
    with Capture() as cap, torch.no_grad():
        rgb_c, rgb, depth_c, depth = avr(c2w, torch.from_numpy(K), torch.from_numpy(x_pix), rf)
    band = cap.get("rand_like")[0]
    trace = np.stack([q[0].numpy()[0] for q in queries if q[1]] + [queries[10][0].numpy()[0]], 0)
    assert len(queries) == 12 and not queries[10][1] and queries[10][2] and not queries[11][2]
    lstm = {f"lstm_{k}": v.detach().numpy() for k, v in avr.lstm.state_dict().items()}
    save("g6_adaptive.npz", x_pix=x_pix, K=K, c2w_one=c2w[0, 0].numpy(), init_dist=init.numpy(),
         band_noise=band.numpy(), trace=trace, out_w=avr.out_layer.weight.detach().numpy(),
         out_b=avr.out_layer.bias.detach().numpy(), steps=10, epsilon=np.float32(0.05), n_coarse=20,
         rgb_coarse=rgb_c.numpy(), rgb=rgb.numpy(), depth_coarse=depth_c.numpy(), depth=depth.numpy(),
         **lstm, **meta, **params)


def g7_encoder():
    """NewPixelNeRFNet.encode (models.py:682-737) + SpatialEncoder.forward
    (:276-329), the reference's own code, on the avr ResNet34 backbone
    (torchvision is absent: the stub module hands the reference
    avr.encoder.resnet34, so this pins the pyramid / upsample / concat,
    latent_scaling and the pose / focal / c bookkeeping, not torchvision's
    numerics). Eval mode (BatchNorm on running statistics)."""
    tv = sys.modules["torchvision.models"]
    from avr import encoder as avr_encoder
    tv.resnet34, tv.resnet18 = avr_encoder.resnet34, avr_encoder.resnet18
    out = {}
    for tag, num_layers, shape in (("nl4", 4, (1, 1, 3, 64, 64)), ("nl3", 3, (2, 3, 48, 40))):
        torch.manual_seed(700 + num_layers)
        conf = model_conf(64, 3, 1000, num_layers)
        conf["encoder"] = {"backbone": "resnet34", "pretrained": False, "num_layers": num_layers}
        net = REF_M.NewPixelNeRFNet(conf).eval()
        images = synth.hashed_uniform(shape, 71 + num_layers, -1.0, 1.0)
        n = int(np.prod(shape[:-3]))
        poses = np.stack([synth.orbit_cam2world(0.3 + 0.5 * i) for i in range(n)]).astype(np.float32)
        poses = poses.reshape(shape[:-3] + (4, 4))
        focal = np.float32(70.0)
        c = np.array([31.5, 30.0], np.float32)
        with torch.no_grad():
            net.encode(torch.from_numpy(images), torch.from_numpy(poses), torch.tensor(focal), c=torch.from_numpy(c))
        lat = net.encoder.latent.numpy()
        out[f"{tag}_images"], out[f"{tag}_poses"], out[f"{tag}_focal"], out[f"{tag}_c"] = images, poses, focal, c
        out[f"{tag}_latent_sub"] = lat[:, :, ::3, ::3]
        out[f"{tag}_latent_shape"] = np.array(lat.shape)
        out[f"{tag}_latent_sum"] = np.float64(lat.astype(np.float64).sum())
        out[f"{tag}_latent_scaling"] = net.encoder.latent_scaling.numpy()
        out[f"{tag}_w2c"] = net.poses.numpy()
        out[f"{tag}_focal_out"] = net.focal.numpy()
        out[f"{tag}_c_out"] = net.c.numpy()
        out[f"{tag}_image_shape"] = net.image_shape.numpy()
        out[f"{tag}_num_views_per_obj"] = np.int64(net.num_views_per_obj)
        out[f"{tag}_seed"] = np.int64(700 + num_layers)
        keys = sorted(k for k in net.state_dict() if k.startswith("encoder."))
        out[f"{tag}_encoder_keys"] = np.array(keys)
    save("g7_encoder.npz", **out)


def g8_batching():
    """train.py:53-83's ray batching with the reference's utils (batched_index_select_nd,
    bbox_sample) and its draw order, on a small synthetic collated batch."""
    SB, NV, sl = 2, 3, 8
    sl2 = sl * sl
    images = torch.from_numpy(synth.hashed_uniform((SB, NV, sl2, 3), 81, -1.0, 1.0))
    cam2world = torch.from_numpy(synth.hashed_uniform((SB, NV, 4, 4), 82))
    intr = torch.from_numpy(synth.hashed_uniform((SB, NV, 3, 3), 83))
    focal = torch.from_numpy(synth.hashed_uniform((SB, NV), 84, 50.0, 60.0))
    c = torch.from_numpy(synth.hashed_uniform((SB, NV, 2), 85, 30.0, 34.0))
    x_pix = torch.from_numpy(synth.hashed_uniform((SB, NV, sl2, 2), 86))
    bbox = torch.tensor([[[1, 2, 5, 6], [0, 0, 7, 7], [3, 1, 4, 2]], [[2, 2, 2, 2], [0, 3, 6, 7], [1, 1, 6, 5]]],
                        dtype=torch.float32)
    out = dict(images=images.numpy(), cam2world=cam2world.numpy(), intrinsics=intr.numpy(), focal=focal.numpy(),
               c=c.numpy(), x_pix=x_pix.numpy(), bbox=bbox.numpy())
    for with_bbox in (False, True):
        torch.manual_seed(880 + int(with_bbox))
        R = 16
        src_idx = torch.randint(0, NV, (SB, 1))
        src_images = REF_U.batched_index_select_nd(images, src_idx).reshape(SB, 1, sl, sl, 3).permute(0, 1, 4, 2, 3)
        poses = REF_U.batched_index_select_nd(cam2world, src_idx)
        f = REF_U.batched_index_select_nd(focal, src_idx)[0, 0]
        cc = REF_U.batched_index_select_nd(c, src_idx)[0, 0, :]
        if with_bbox:
            rays_idx = torch.stack([(lambda p: p[..., 0] * sl2 + p[..., 1] * sl + p[..., 2])(
                REF_U.bbox_sample(bbox[sb], R)) for sb in range(SB)])
        else:
            rays_idx = torch.randint(0, NV * sl2, (SB, R))
        xp = REF_U.batched_index_select_nd(x_pix.reshape(SB, -1, 2), rays_idx)
        cw = REF_U.batched_index_select_nd(cam2world.unsqueeze(2).expand(SB, NV, sl2, 4, 4).reshape(SB, -1, 4, 4),
                                           rays_idx)
        gt = 0.5 * REF_U.batched_index_select_nd(images.reshape(SB, -1, 3), rays_idx) + 0.5
        k = f"bbox{int(with_bbox)}"
        out.update({f"{k}_seed": np.int64(880 + int(with_bbox)), f"{k}_src_images": src_images.numpy(),
                    f"{k}_poses": poses.numpy(), f"{k}_focal": f.numpy(), f"{k}_c": cc.numpy(),
                    f"{k}_x_pix": xp.numpy(), f"{k}_cam2world": cw.numpy(), f"{k}_gt": gt.numpy()})
    save("g8_batching.npz", **out)


if __name__ == "__main__":
    REF_U, REF_R, REF_M = import_reference()
    sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))
    torch.set_num_threads(8)
    g0_reductions()
    g1_volume_integral(48)
    g2_sample_fine(48)
    g3_geometry(64)
    g4_field()
    g4_field_multiview()
    g5_forward(64)
    g6_adaptive(48)
    g7_encoder()
    g8_batching()
