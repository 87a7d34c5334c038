"""Shared test helpers: build the product's NewPixelNeRFNet from a golden
fixture, and the oracle field with the same parameters."""
import numpy as np
import torch

from oracle import avr_oracle as O
from oracle import synth


def model_conf(d_hidden, n_blocks, combine_layer, d_latent, spade=False, beta=0.0):
    from avr.conf import Conf
    num_layers = {64: 1, 128: 2, 256: 3, 512: 4, 1024: 5}[d_latent]
    mlp = {"type": "resnet", "n_blocks": n_blocks, "d_hidden": d_hidden, "combine_layer": combine_layer,
           "use_spade": bool(spade), "beta": float(beta)}
    return Conf({"use_encoder": True, "use_global_encoder": False, "use_xyz": True, "use_code": True,
                 "code": {"num_freqs": 6, "freq_factor": 1.5, "include_input": True}, "use_viewdirs": True,
                 "use_code_viewdirs": False, "mlp_coarse": dict(mlp), "mlp_fine": dict(mlp),
                 "encoder": {"backbone": "resnet34", "pretrained": False, "num_layers": num_layers}})


def build_net(g, device, precision="x3"):
    """avr.models.NewPixelNeRFNet carrying the fixture's weights and source view."""
    from avr.models import NewPixelNeRFNet
    pc, pf, latent = synth.field_from_meta(g)
    net = NewPixelNeRFNet(model_conf(int(g["d_hidden"]), int(g["n_blocks"]), int(g["combine_layer"]),
                                     int(g["d_latent"]), _spade(g), _beta(g)),
                          bn=bool(int(g["bn"])) if "bn" in g else False)
    for mlp, p in ((net.mlp_coarse, pc), (net.mlp_fine, pf)):
        sd = mlp.state_dict()
        for k, v in p.items():
            sd[k] = torch.from_numpy(np.ascontiguousarray(v))
        mlp.load_state_dict(sd)
    net = net.to(device).eval()
    net.encoder.latent = torch.from_numpy(latent).to(device)
    net.encoder.latent_scaling = torch.from_numpy(g["latent_scaling"]).to(device)
    net.poses = torch.from_numpy(g["poses"]).to(device)
    net.focal = torch.from_numpy(g["focal"]).to(device)
    net.c = torch.from_numpy(g["c"]).to(device)
    net.image_shape = torch.from_numpy(g["image_shape"]).to(device)
    net.num_views_per_obj = int(g["ns"]) if "ns" in g else 1
    if "combine_type" in g:
        for mlp in (net.mlp_coarse, net.mlp_fine):
            mlp.combine_type = str(g["combine_type"])
    net.field_precision = precision
    for p in net.parameters():
        p.requires_grad_(False)
    return net


def _spade(g):
    return bool(int(g["spade"])) if "spade" in g else False


def _beta(g):
    return float(g["beta"]) if "beta" in g else 0.0


def oracle_field(g):
    pc, pf, latent = synth.field_from_meta(g)
    if "ns" in g:
        return O.MultiViewField(pc, pf, latent, g["poses"], g["focal"], g["c"], g["image_shape"], g["latent_scaling"],
                                n_blocks=int(g["n_blocks"]), combine_layer=int(g["combine_layer"]),
                                combine_type=str(g["combine_type"]), beta=_beta(g))
    return O.PixelNeRFField(pc, pf, latent, g["poses"], g["focal"], g["c"], g["image_shape"], g["latent_scaling"],
                            n_blocks=int(g["n_blocks"]), combine_layer=int(g["combine_layer"]), beta=_beta(g))


def oracle_field_from_net(net):
    """The oracle field with the parameters, latent and source view of a
    product NewPixelNeRFNet (e.g. the bench's avr.scene.synthetic_scene)."""
    sd = lambda m: {k: v.detach().float().cpu().numpy() for k, v in m.state_dict().items()}  # noqa: E731
    mlp = net.mlp_coarse
    return O.PixelNeRFField(sd(net.mlp_coarse), sd(net.mlp_fine), net.encoder.latent.detach().float().cpu().numpy(),
                            to_np(net.poses), to_np(net.focal), to_np(net.c), to_np(net.image_shape),
                            to_np(net.encoder.latent_scaling), n_blocks=mlp.n_blocks,
                            combine_layer=mlp.combine_layer)


def to_np(t):
    return t.detach().float().cpu().numpy()
