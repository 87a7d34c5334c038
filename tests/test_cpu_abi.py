"""CPU-only checks: the C-ABI library loads and exports every symbol that
include/avr.h declares, the Python surface mirrors the reference's, and the
product refuses host tensors (no CPU fallback). No kernel is launched."""
import ctypes
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "avr.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(avr_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("avr_world_rays", "avr_sample_coarse", "avr_sample_fine", "avr_composite_fwd", "avr_composite_bwd",
              "avr_field_fwd_rays", "avr_field_fwd_points", "avr_depth_from_world", "avr_version"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from avr import _lib
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), f"libavr_hip.so does not export {s}"
    assert set(_lib.EXPORTED) == set(declared_symbols())
    assert lib.avr_version() == _lib.ABI_VERSION


def test_device_count_without_gpu_does_not_fail():
    from avr import _lib
    assert _lib.load().avr_device_count() >= 0


def test_invalid_arguments_return_codes():
    """Argument validation runs before any HIP call, so it is testable on CPU."""
    from avr import _lib
    lib = _lib.load()
    rc = lib.avr_composite_fwd(None, None, 4, 8, 1, ctypes.c_float(1.8), None, None, None, None)
    assert rc == 1001 and b"null" in lib.avr_last_error_string()
    dims = _lib.FieldDims(42, 512, 384, 3, 3, 6, 1.5)  # 384 hidden is unsupported
    n = ctypes.c_int64()
    assert lib.avr_field_packed_floats(ctypes.byref(dims), ctypes.byref(n)) == 1001
    dims = _lib.FieldDims(42, 512, 512, 3, 3, 6, 1.5)
    assert lib.avr_field_packed_floats(ctypes.byref(dims), ctypes.byref(n)) == 0
    # fp32 fragments: 3 blocks x 2 x 512^2 + lin_in (3 tiles) + lin_out + 3 lin_z x 512^2 (+ biases)
    fp32 = 3 * 2 * 512 * 512 + 3 * 16 * 512 + 512 * 16 + 3 * 512 * 512 + 512 * 7 + 16
    # split-fp16 fragments (hi+lo = 4 B per weight): header, lin_in (K 64), 6 x 512^2, lin_out (16 rows),
    # and the 3 lin_z (512 x 512, d_latent 512) for the x3 table kernel
    x3 = 64 + 64 * 512 + 6 * 512 * 512 + 16 * 512 + 3 * 512 * 512
    assert n.value == ((fp32 + 63) // 64) * 64 + x3


def test_lin_out_rows_argument_checks():
    """avr_lin_out_fwd_rows / avr_lin_out_bwd_rows (ABI 14): zero rows is a no-op, d_hidden outside 64..512 or not
    a multiple of 64 and null pointers are refused before any HIP call."""
    from avr import _lib
    lib = _lib.load()
    f, b = lib.avr_lin_out_fwd_rows, lib.avr_lin_out_bwd_rows
    assert f(0, 512, None, 512, None, None, None, None, None) == 0
    assert b(0, 512, None, None, None, None, 512, None, None, None, None) == 0
    for H in (0, 32, 100, 576):
        assert f(4, H, None, 512, None, None, None, None, None) == 1001
        assert b"d_hidden" in lib.avr_last_error_string()
    assert f(4, 512, None, 512, None, None, None, None, None) == 1001
    assert b"null" in lib.avr_last_error_string()
    assert b(4, 256, None, None, None, None, 256, None, None, None, None) == 1001


def test_round6_point_gradient_entry_points_argument_checks():
    """avr_lin_out_act_bwd_rows, avr_zfeature_grad_points and avr_band_fwd / _bwd (ABI 16): zero rows is a no-op; null pointers, a scene
    count outside 1..AVR_MAX_SCENES and gradient rows shorter than 3 + 6 num_freqs are refused before any HIP call."""
    import ctypes
    from avr import _lib
    lib = _lib.load()
    assert lib.avr_lin_out_act_bwd_rows(0, None, None, None, None, None) == 0
    assert lib.avr_lin_out_act_bwd_rows(4, None, None, None, None, None) == 1001
    assert b"null" in lib.avr_last_error_string()
    v = (_lib.ViewDesc * 1)()
    z = lib.avr_zfeature_grad_points
    assert z(v, 1, None, 0, None, 39, 6, ctypes.c_float(3.14159), 0, None, None) == 0
    assert z(v, 0, None, 3, None, 39, 6, ctypes.c_float(3.14159), 0, None, None) == 1001
    assert z(v, 1, None, 3, None, 38, 6, ctypes.c_float(3.14159), 0, None, None) == 1001
    assert b"bad sizes" in lib.avr_last_error_string()
    assert z(v, 1, None, 3, None, 39, 6, ctypes.c_float(3.14159), 0, None, None) == 1001
    assert b"null" in lib.avr_last_error_string()
    # the training band (avr_band_fwd / avr_band_bwd): 1..64 samples, null pointers refused, no rays a no-op
    assert lib.avr_band_fwd(0, 20, None, None, None, None, ctypes.c_float(0.05), None, None, None) == 0
    assert lib.avr_band_fwd(4, 65, None, None, None, None, ctypes.c_float(0.05), None, None, None) == 1001
    assert lib.avr_band_fwd(4, 20, None, None, None, None, ctypes.c_float(0.05), None, None, None) == 1001
    assert lib.avr_band_bwd(0, 20, None, None, None, None, None) == 0
    assert lib.avr_band_bwd(4, 0, None, None, None, None, None) == 1001
    assert lib.avr_band_bwd(4, 20, None, None, None, None, None) == 1001


def test_spade_bwd_rows_argument_checks():
    """avr_spade_bwd_rows (ABI 14): zero values is a no-op; a count not a multiple of 4 and null pointers are
    refused before any HIP call."""
    from avr import _lib
    lib = _lib.load()
    assert lib.avr_spade_bwd_rows(0, None, None, None, None, None, None, None) == 0
    assert lib.avr_spade_bwd_rows(6, None, None, None, None, None, None, None) == 1001
    assert b"multiple of 4" in lib.avr_last_error_string()
    assert lib.avr_spade_bwd_rows(8, None, None, None, None, None, None, None) == 1001
    assert b"null" in lib.avr_last_error_string()


def test_ops_refuse_host_tensors():
    from avr import _lib, ops
    with pytest.raises(_lib.AVRError):
        ops.composite_fwd(torch.zeros(4, 8), torch.zeros(4, 8, 4))
    with pytest.raises(_lib.AVRError):
        ops.world_rays(torch.zeros(1, 4, 2), torch.eye(3)[None], torch.eye(4).expand(1, 4, 4, 4))


def test_renderer_surface_matches_reference():
    import inspect
    from avr import renderers
    from avr.conf import Conf, default_conf
    sig = inspect.signature(renderers.VolumeRenderer.__init__)
    assert list(sig.parameters)[1:] == ["near", "far", "n_coarse", "n_fine", "n_fine_depth", "depth_std",
                                        "white_back"]
    r = renderers.VolumeRenderer.from_conf(default_conf()["normal_renderer"])
    assert (r.n_coarse, r.n_fine, r.n_fine_depth, r.white_back) == (64, 32, 16, True)
    r = renderers.VolumeRenderer.from_conf(Conf({}))
    assert (r.n_coarse, r.n_fine, r.n_fine_depth, r.depth_std) == (32, 16, 8, 0.01)  # renderers.py:279-289
    assert len(list(r.parameters())) == 0 and len(r.state_dict()) == 0  # contributes no state_dict keys
    for name in ("sample_coarse", "sample_fine", "sample_depth", "volume_integral"):
        assert callable(getattr(renderers, name))


def test_model_state_dict_keys_match_reference_layout():
    from avr.conf import default_conf
    from avr.models import NewPixelNeRFNet
    net = NewPixelNeRFNet(default_conf()["model"])
    keys = set(net.state_dict())
    for k in ("mlp_coarse.lin_in.weight", "mlp_coarse.lin_z.2.bias", "mlp_fine.blocks.2.fc_1.weight",
              "mlp_fine.blocks.0.bn_0.running_mean", "mlp_coarse.lin_out.bias", "code._freqs"):
        assert k in keys, k
    assert net.mlp_coarse.lin_in.weight.shape == (512, 42)
    assert net.d_latent == 512
    from avr.field import fused_eligible
    net.encoder.set_latent(torch.zeros(1, 512, 4, 4))
    assert fused_eligible(net)
    mv = NewPixelNeRFNet(default_conf(multiview=True)["model"])
    mv.encoder.set_latent(torch.zeros(1, 512, 4, 4))
    assert fused_eligible(mv) and len(mv.mlp_coarse.lin_z) == 3 and mv.mlp_coarse.n_blocks == 5
    # NS > 1 source views (the split launches): combine_layer must leave at least one block before the combine
    mv.num_views_per_obj = 2
    assert fused_eligible(mv, multiview=True) and not fused_eligible(mv)
    for mlp in (mv.mlp_coarse, mv.mlp_fine):
        mlp.combine_layer = 0
    assert not fused_eligible(mv, multiview=True)


def test_bn_training_route_eligibility():
    """train.py --bn nets in training mode take the layer-by-layer HIP path (avr.bn_train), in eval mode the
    fused kernel (running statistics folded); nets without BatchNorm neither."""
    from avr.bn_train import bn_train_eligible
    from avr.conf import default_conf
    from avr.field import fused_eligible
    from avr.models import NewPixelNeRFNet
    net = NewPixelNeRFNet(default_conf(multiview=True)["model"], bn=True)
    net.encoder.set_latent(torch.zeros(1, 512, 4, 4))
    assert bn_train_eligible(net.train()) and not fused_eligible(net)
    assert not bn_train_eligible(net.eval()) and fused_eligible(net)
    plain = NewPixelNeRFNet(default_conf()["model"])
    plain.encoder.set_latent(torch.zeros(1, 512, 4, 4))
    assert not bn_train_eligible(plain.train())
    net.train()
    for m in (net.mlp_coarse, net.mlp_fine):   # Softplus with BatchNorm: module path
        for blk in m.blocks:
            blk.activation = torch.nn.Softplus(beta=2.0)
        m.activation = torch.nn.Softplus(beta=2.0)
    assert not bn_train_eligible(net)


def test_graft_entry_build():
    """__graft_entry__.build(): make (no-op when built) + load + ABI check."""
    import importlib
    import sys
    sys.path.insert(0, REPO)
    ge = importlib.import_module("__graft_entry__")
    ge.build()
