"""The synthetic scene every measurement uses (SURVEY §8d "Synthetic
inputs"): the conf/default.conf PixelNeRF field with the reference's init
(kaiming; ResnetBlockFC.fc_1 ~ N(0, 0.02) instead of the reference's zero
init, which would make every block an identity), a seeded N(0, 1) latent map
of 512 x 64 x 64 standing in for the ResNet34 features of a 128^2 view, and
the source camera: identity rotation, t = (0, 0, 1.3), focal 131.25 px (fy
negated), c = (64, 64), image 128 x 128."""
import torch

# normalized intrinsics of the synthetic target camera
INTRINSICS = [[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]


def synthetic_scene(device, seed=0, conf=None, latent_hw=(64, 64), sigma_bias=0.0, bn=False):
    """NewPixelNeRFNet on `device` (eval, no grad) with the synthetic latent
    and source view. sigma_bias is added to both MLPs' density output bias
    (0 = the measured fog of a random-init field; > 0 makes rays saturate,
    as on a real scene, for early-termination runs)."""
    from .conf import default_conf
    from .models import NewPixelNeRFNet
    torch.manual_seed(seed)
    net = NewPixelNeRFNet(conf if conf is not None else default_conf()["model"], bn=bn)   # bn: train.py --bn
    with torch.no_grad():
        for mlp in (net.mlp_coarse, net.mlp_fine):
            for blk in mlp.blocks:
                blk.fc_1.weight.normal_(0.0, 0.02)
            mlp.lin_out.bias[3] += sigma_bias
    net = net.to(device).eval()
    for p in net.parameters():
        p.requires_grad_(False)
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    latent = torch.randn(1, net.d_latent, latent_hw[0], latent_hw[1], generator=g).to(device)
    net.encoder.set_latent(latent)
    poses = torch.zeros(1, 3, 4)
    poses[0, :3, :3] = torch.eye(3)
    poses[0, 2, 3] = 1.3
    net.poses = poses.to(device)
    net.focal = torch.tensor([[131.25, -131.25]], device=device)
    net.c = torch.tensor([[64.0, 64.0]], device=device)
    net.image_shape = torch.tensor([128.0, 128.0], device=device)
    return net
