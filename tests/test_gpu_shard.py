"""Ray sharding on one GPU: the shares avr.parallel.ray_tiles deals to W ranks,
each rendered with its frame-wide ray ids (VolumeRenderer(ray_ids=...)), put
back together equal the single render of the whole frame under the same
in-kernel Philox seed — the draws do not depend on how the frame was dealt."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


@pytest.mark.parametrize("world,R", [(2, 1000), (3, 777)])
def test_sharded_philox_matches_single_render(world, R):
    from avr.parallel import ray_tiles
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS, synthetic_scene
    net = synthetic_scene(DEV)
    g = torch.Generator().manual_seed(5)
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4, device=DEV)
    c2w[2, 3] = 1.3
    c2w = c2w.reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    K = torch.tensor([INTRINSICS], device=DEV)

    def renderer():
        r = VolumeRenderer(0.8, 1.8, 64, 32, 0, 0.01, True)
        r.seed = 77
        return r

    with torch.no_grad():
        full = renderer()(c2w, K, x_pix, net)
        parts = [torch.empty_like(full[k]) for k in range(3)]
        for rank in range(world):
            idx = ray_tiles(R, rank, world, device=DEV)
            rc, rf, d, _ = renderer()(c2w[:, idx], K, x_pix[:, idx].contiguous(), net, ray_ids=idx, n_rays_total=R)
            for k, t in enumerate((rc, rf, d)):
                parts[k][:, idx] = t
        torch.cuda.synchronize()
    for k in range(3):
        torch.testing.assert_close(parts[k], full[k], atol=0, rtol=0)
    # and without ray ids the shares would draw different noise (the defect this guards against)
    with torch.no_grad():
        idx = ray_tiles(R, 1, world, device=DEV)
        _, rf_local, _, _ = renderer()(c2w[:, idx], K, x_pix[:, idx].contiguous(), net)
    assert not torch.equal(rf_local, full[1][:, idx])


def test_sample_fine_per_ray_bounds():
    """renderers.sample_fine with per-ray (SB, R) near/far: renderers.py:45-46 per ray."""
    from avr.renderers import sample_fine
    torch.manual_seed(0)
    SB, R, Nc, Nf = 2, 100, 32, 16
    w = torch.rand(SB, R, Nc, 1, device=DEV)
    near = 0.5 + torch.rand(SB, R, device=DEV)
    far = near + 0.2 + torch.rand(SB, R, device=DEV)
    u = torch.rand(SB, R, Nf, device=DEV)
    u2 = torch.rand(SB, R, Nf, device=DEV)
    z, idx = sample_fine(near, far, Nf, w, DEV, u=u, u2=u2, return_idx=True)
    ww = w[..., 0] + 1e-5
    cdf = torch.cumsum((ww / ww.sum(-1, keepdim=True)).double(), -1).float()
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    inds = torch.clamp_min(torch.searchsorted(cdf, u, right=True).float() - 1.0, 0.0)
    assert (idx.float() != inds).float().mean() < 1e-3     # ties of the fp64-vs-fp32 cdf aside
    z_ref = near.unsqueeze(-1) + (far - near).unsqueeze(-1) * ((idx.float() + u2) / Nc)
    torch.testing.assert_close(z, z_ref, atol=0, rtol=0)
    with pytest.raises(ValueError):
        sample_fine(near, far, Nf, w, DEV, u=u)
