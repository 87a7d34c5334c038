"""The per-scene encoder: avr.encoder.SpatialEncoder on the
ResNet34 backbone and NewPixelNeRFNet.encode, against tests/golden/g7_encoder.npz
— the reference's own SpatialEncoder.forward / encode() (models.py:276-329,
682-737) run by make_golden.py on the same backbone and weights (torchvision
is absent, so the backbone's agreement with torchvision is by architecture and
state_dict keys only: parity of the ResNet numerics is unpinned)."""
import numpy as np
import pytest
import torch

from helpers import model_conf


def _net(tag, g):
    from avr.models import NewPixelNeRFNet
    num_layers = 4 if tag == "nl4" else 3
    torch.manual_seed(int(g[f"{tag}_seed"]))
    conf = model_conf(64, 3, 1000, 512)
    conf["encoder"] = {"backbone": "resnet34", "pretrained": False, "num_layers": num_layers}
    return NewPixelNeRFNet(conf).eval()


@pytest.mark.parametrize("tag", ["nl4", "nl3"])
def test_encode_matches_reference(golden, tag):
    g = golden("g7_encoder.npz")
    net = _net(tag, g)
    keys = sorted(k for k in net.state_dict() if k.startswith("encoder."))
    assert keys == list(g[f"{tag}_encoder_keys"])
    with torch.no_grad():
        net.encode(torch.from_numpy(g[f"{tag}_images"]), torch.from_numpy(g[f"{tag}_poses"]),
                   torch.tensor(g[f"{tag}_focal"]), c=torch.from_numpy(g[f"{tag}_c"]))
    lat = net.encoder.latent.numpy()
    assert tuple(lat.shape) == tuple(g[f"{tag}_latent_shape"])
    np.testing.assert_allclose(lat[:, :, ::3, ::3], g[f"{tag}_latent_sub"], atol=2e-5, rtol=1e-5)
    assert abs(lat.astype(np.float64).sum() - float(g[f"{tag}_latent_sum"])) <= 1e-5 * abs(lat).sum()
    np.testing.assert_array_equal(net.encoder.latent_scaling.numpy(), g[f"{tag}_latent_scaling"])
    np.testing.assert_allclose(net.poses.numpy(), g[f"{tag}_w2c"], atol=1e-6)
    np.testing.assert_array_equal(net.focal.numpy(), g[f"{tag}_focal_out"])
    np.testing.assert_array_equal(net.c.numpy(), g[f"{tag}_c_out"])
    np.testing.assert_array_equal(net.image_shape.numpy(), g[f"{tag}_image_shape"])
    assert net.num_views_per_obj == int(g[f"{tag}_num_views_per_obj"])


def test_resnet34_architecture():
    """torchvision resnet34: 21 797 672 parameters with the classifier; the
    encoder drops fc / avgpool (models.py:230-232)."""
    from avr.encoder import SpatialEncoder, resnet34
    assert sum(p.numel() for p in resnet34().parameters()) == 21797672
    enc = SpatialEncoder(pretrained=False)
    assert sum(p.numel() for p in enc.parameters()) == 21797672 - 513000
    assert enc.latent_size == 512
    out = enc(torch.rand(2, 3, 64, 48))
    assert tuple(out.shape) == (2, 512, 32, 24)
    np.testing.assert_allclose(enc.latent_scaling.numpy(), [24 / 23 * 2, 32 / 31 * 2], rtol=1e-6)


def test_encoder_gradient_reaches_backbone():
    """train.py trains the encoder through the latent unless stop_encoder_grad."""
    from avr.encoder import SpatialEncoder
    torch.manual_seed(0)
    enc = SpatialEncoder(pretrained=False, num_layers=2)
    lat = enc(torch.rand(1, 3, 32, 32))
    uv = torch.rand(1, 10, 2) * 32
    enc.index(uv, image_size=torch.tensor([32.0, 32.0])).square().sum().backward()
    assert enc.model.conv1.weight.grad is not None and float(enc.model.conv1.weight.grad.abs().max()) > 0
    assert lat.shape[1] == 128
