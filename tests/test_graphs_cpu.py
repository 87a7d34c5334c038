"""GraphedRenderer's state check (host logic, no GPU): in-place parameter updates and a new latent / source
view mark the captured graph stale; an unchanged net does not."""
import warnings

import torch


def _graphed_state():
    from avr.conf import default_conf
    from avr.field import param_generation
    from avr.graphs import GraphedRenderer
    from avr.models import NewPixelNeRFNet
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")   # random-init encoder (no pretrained weights offline)
        net = NewPixelNeRFNet(default_conf()["model"]).eval()
    net.encoder.set_latent(torch.randn(1, net.d_latent, 8, 8))
    net.poses, net.focal = torch.zeros(1, 3, 4), torch.ones(1, 2)
    net.c, net.image_shape = torch.ones(1, 2), torch.ones(2)
    g = GraphedRenderer.__new__(GraphedRenderer)   # the check alone: no capture
    g.net = net

    def hold():
        views = g._views()
        g._held_views = views
        g._held = [(t, t._version) for t in g._params() + views if isinstance(t, torch.Tensor)]
        g._held_precision = net.field_precision
        g._held_gen = param_generation()
    hold()
    return g, net, hold


def test_state_check_sees_updates():
    g, net, hold = _graphed_state()
    assert not g._stale()
    with torch.no_grad():
        net.mlp_fine.lin_out.bias.add_(1.0)        # optimizer-style in-place step
    assert g._stale()
    hold()
    net.load_state_dict(net.state_dict())           # copies in place
    assert g._stale()
    hold()
    net.encoder.set_latent(net.encoder.latent * 2)  # net.encode() of new images
    assert g._stale()
    hold()
    net.poses = net.poses.clone()
    assert g._stale()
    hold()
    assert not g._stale()
    net.field_precision = "fp32"                    # the captured kernels are the x3 ones
    assert g._stale()
    hold()
    assert not g._stale()
    p = net.mlp_coarse.lin_out.bias                 # a fused optimizer: no version bump, a generation step
    p.grad = torch.ones_like(p)
    torch.optim.Adam([p], lr=1e-3, fused=True).step()
    assert g._stale()
    hold()
    assert not g._stale()


def test_optimizer_steps_advance_the_param_generation():
    """Every torch.optim step (fused ones too, which leave the parameters' version counters alone) advances the
    generation FusedField's cache keys carry; GraphedTrainStep advances it per replay."""
    import torch
    from avr.field import bump_param_generation, param_generation
    p = torch.nn.Parameter(torch.randn(8))
    for opt in (torch.optim.Adam([p], lr=1e-2, fused=True), torch.optim.SGD([p], lr=1e-2)):
        p.grad = torch.randn(8)
        g0, v0 = param_generation(), p._version
        opt.step()
        assert param_generation() == g0 + 1
    assert p._version >= v0
    g0 = param_generation()
    bump_param_generation()
    assert param_generation() == g0 + 1
