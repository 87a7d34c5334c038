"""Edge ray counts of the whole VolumeRenderer.forward on the HIP path
(/root/reference/renderers.py:133-277), against the pinned numpy oracle fed the
same explicit noise: 1, 3, 65 and 127 rays (every workgroup partly empty, a
64-sample field tile spanning two rays, a single ray) and two scenes with a
ragged per-scene count, plus R = 0, which the reference itself cannot render
(models.py:74 views a 0-row PE as (0, -1) and raises): the HIP path must end
cleanly -- empty outputs or a Python error -- and leave the device usable.

Bars as in test_gpu_parity.py's g5 test: coarse rgb <= 1e-4 on every ray; fine
rgb / depth <= 1e-4 on every ray whose inverse-CDF bins equal the oracle's (a
bin flip is an fp32 tie at a cdf step), and at least the
rays with equal bins must be all of them at these sizes (measured).
"""
import numpy as np
import pytest
import torch

from helpers import build_net, oracle_field, to_np
from oracle import avr_oracle as O
from oracle import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
NC, NF = 128, 64


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def _inputs(R, seed):
    rng = np.random.default_rng(seed)
    x_pix = rng.random((1, R, 2), dtype=np.float32)
    noise = {"coarse": rng.random((1, R, NC), dtype=np.float32), "u": rng.random((1, R, NF), dtype=np.float32),
             "u2": rng.random((1, R, NF), dtype=np.float32), "depth": np.zeros((1, R, 0), np.float32)}
    return x_pix, noise


@pytest.mark.parametrize("precision", ["x3", "fp32"])
@pytest.mark.parametrize("R", [1, 3, 65, 127])
def test_renderer_edge_ray_counts_vs_oracle(golden, precision, R):
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, precision)
    x_pix, noise = _inputs(R, 100 + R)
    c2w1 = synth.orbit_cam2world(0.7)
    K = synth.default_intrinsics()[None]
    rend = VolumeRenderer(0.8, 1.8, NC, NF, 0, 0.01, True)
    c2w = T(c2w1).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    with torch.no_grad():
        rgb_c, rgb_f, depth, _ = rend(c2w, T(K), T(x_pix), net, noise={k: T(v) for k, v in noise.items()})
    assert rend.last_path == "fused"
    assert tuple(rgb_c.shape) == (1, R, 3) and tuple(rgb_f.shape) == (1, R, 3) and depth.numel() == R
    oc, of, od, _, aux = O.render(np.broadcast_to(c2w1, (1, R, 4, 4)), K, x_pix, oracle_field(g), 0.8, 1.8, NC, NF,
                                  0, 0.01, True, noise["coarse"], noise["u"], noise["u2"], noise["depth"],
                                  return_aux=True)
    np.testing.assert_allclose(to_np(rgb_c), oc, atol=1e-4)
    from avr import ops
    with torch.no_grad():
        ro, rd, _ = ops.world_rays(T(x_pix), T(K), c2w)
        zc = ops.sample_coarse(0.8, 1.8, R, NC, DEV, noise=T(noise["coarse"][0]))
        _, _, w_c = ops.composite(zc, net.fused().forward_rays(ro[0], rd[0], zc, True))
        _, idx, _ = ops.sample_fine(w_c, zc, 0.8, 1.8, NF, 0, 0.01, u=T(noise["u"][0]), u2=T(noise["u2"][0]),
                                    want_idx=True)
    same = (to_np(idx) == aux["idx"][0]).all(-1)
    ok = (np.abs(to_np(rgb_f) - of).max(-1) <= 1e-4) & (np.abs(to_np(depth).reshape(od.shape) - od) <= 1e-4)
    assert ok[0][same].all(), np.nonzero(~ok[0] & same)
    assert same.all(), np.nonzero(~same)


def test_renderer_two_scenes_ragged(golden):
    """SB = 2 scenes in one call (the batched field launch), 67 rays each, both
    scenes the fixture's source view: each scene equals the one-scene render of
    its own rays bit for bit."""
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, "x3")
    one_scene = (net.encoder.latent, net.poses, net.focal, net.c)
    net.encoder.latent = net.encoder.latent.expand(2, *net.encoder.latent.shape[1:]).contiguous()
    net.poses = net.poses.expand(2, *net.poses.shape[1:]).contiguous()
    if net.focal.dim() > 1:
        net.focal = net.focal.expand(2, *net.focal.shape[1:]).contiguous()
    if net.c.dim() > 1:
        net.c = net.c.expand(2, *net.c.shape[1:]).contiguous()
    R = 67
    xs, ns = zip(*[_inputs(R, 7 + s) for s in range(2)])
    x_pix = np.concatenate(xs, 0)
    noise = {k: np.concatenate([n[k] for n in ns], 0) for k in ns[0]}
    c2w = torch.stack([T(synth.orbit_cam2world(a)) for a in (0.7, 2.1)]).reshape(2, 1, 4, 4).expand(2, R, 4, 4)
    K = T(synth.default_intrinsics()[None]).expand(2, 3, 3)
    rend = VolumeRenderer(0.8, 1.8, NC, NF, 0, 0.01, True)
    with torch.no_grad():
        both = rend(c2w, K, T(x_pix), net, noise={k: T(v) for k, v in noise.items()})
        assert rend.last_path == "fused"
        net.encoder.latent, net.poses, net.focal, net.c = one_scene
        for s in range(2):
            one = rend(c2w[s:s + 1], K[s:s + 1], T(x_pix[s:s + 1]), net,
                       noise={k: T(v[s:s + 1]) for k, v in noise.items()})
            for a, b in zip(both[:3], one[:3]):
                assert torch.equal(a[s:s + 1], b), (s, float((a[s:s + 1] - b).abs().max()))


def test_renderer_zero_rays_ends_cleanly(golden):
    """R = 0: the reference raises (PE view of a 0-row tensor); the HIP path
    either returns empty outputs or raises a Python error -- no launch of an
    empty grid, no fault -- and the device still renders afterwards."""
    from avr.renderers import VolumeRenderer
    g = golden("g4_field_full.npz")
    net = build_net(g, DEV, "x3")
    rend = VolumeRenderer(0.8, 1.8, NC, NF, 0, 0.01, True)
    K = T(synth.default_intrinsics()[None])
    c2w = T(synth.orbit_cam2world(0.7)).reshape(1, 1, 4, 4)
    with torch.no_grad():
        try:
            out = rend(c2w.expand(1, 0, 4, 4), K, torch.zeros(1, 0, 2, device=DEV), net)
        except (RuntimeError, ValueError) as e:
            print("R = 0 raised:", type(e).__name__, str(e)[:200])
        else:
            assert tuple(out[0].shape) == (1, 0, 3) and tuple(out[1].shape) == (1, 0, 3)
            assert out[2].numel() == 0
        torch.cuda.synchronize()
        rgb_c, rgb_f, depth, _ = rend(c2w.expand(1, 5, 4, 4), K, torch.rand(1, 5, 2, device=DEV), net)
        torch.cuda.synchronize()
    assert torch.isfinite(rgb_f).all() and torch.isfinite(depth).all()
