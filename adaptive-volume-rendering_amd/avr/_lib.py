"""ctypes binding of libavr_hip.so (include/avr.h).

The library is built in-tree (`make -C adaptive-volume-rendering_amd`, or
__graft_entry__.build()) and loaded from this directory. There is no fallback:
if the library or a HIP device is missing, every op raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# AVR_LIB_PATH: another build of the same ABI (A/B diagnostics)
LIB_PATH = os.environ.get("AVR_LIB_PATH") or os.path.join(_HERE, "libavr_hip.so")
AVR_MAX_BLOCKS = 8
AVR_MAX_SCENES = 16
AVR_LOOKUP_GRAD_TERMS = 8
ABI_VERSION = 16

c_float_p = ctypes.POINTER(ctypes.c_float)
c_void_p = ctypes.c_void_p
i64 = ctypes.c_int64
u64 = ctypes.c_uint64
c_uint32 = ctypes.c_uint32
c_int = ctypes.c_int
c_float = ctypes.c_float


class FieldDims(ctypes.Structure):
    _fields_ = [("d_in", c_int), ("d_latent", c_int), ("d_hidden", c_int), ("n_blocks", c_int),
                ("n_lin_z", c_int), ("num_freqs", c_int), ("freq_factor", c_float), ("precision", c_int),
                ("bn", c_int), ("spade", c_int), ("beta", c_float)]


FIELD_FP32 = 0
FIELD_X3 = 1


class ResnetFCWeights(ctypes.Structure):
    _fields_ = [("lin_in_w", c_void_p), ("lin_in_b", c_void_p), ("lin_out_w", c_void_p), ("lin_out_b", c_void_p),
                ("fc0_w", c_void_p * AVR_MAX_BLOCKS), ("fc0_b", c_void_p * AVR_MAX_BLOCKS),
                ("fc1_w", c_void_p * AVR_MAX_BLOCKS), ("fc1_b", c_void_p * AVR_MAX_BLOCKS),
                ("lin_z_w", c_void_p * AVR_MAX_BLOCKS), ("lin_z_b", c_void_p * AVR_MAX_BLOCKS),
                ("bn_scale", c_void_p * AVR_MAX_BLOCKS), ("bn_shift", c_void_p * AVR_MAX_BLOCKS),
                ("scale_z_w", c_void_p * AVR_MAX_BLOCKS), ("scale_z_b", c_void_p * AVR_MAX_BLOCKS)]


class ViewDesc(ctypes.Structure):
    _fields_ = [("poses", c_float * 12), ("focal", c_float * 2), ("c", c_float * 2), ("image_shape", c_float * 2),
                ("latent_scaling", c_float * 2), ("latent_h", c_int), ("latent_w", c_int)]


AVR_WGRAD_MAX_LAYERS = 16


class WGradLayer(ctypes.Structure):
    _fields_ = [("grad", c_void_p), ("ld_grad", i64), ("input", c_void_p), ("ld_input", i64),
                ("out_dim", c_int), ("in_dim", c_int), ("grad_max", c_void_p), ("input_max", c_void_p),
                ("partial", c_void_p), ("bias_partial", c_void_p),
                ("in_mu", c_void_p), ("in_scale", c_void_p), ("in_shift", c_void_p), ("input_relu", c_int)]


BN_FWD, BN_BWD = 0, 1
BN_PLAIN, BN_RELU, BN_GRAD = 0, 1, 2
BN_LAYER_LIN_Z_T = 34     # avr.h AVR_BN_LAYER_LIN_Z_T: + b, lin_z[b]^T of the backward blob (ABI 14)


class BnLayer(ctypes.Structure):
    """avr_bn_layer (ABI 12): one layer GEMM of the training-mode BatchNorm path (see include/avr.h)."""
    _fields_ = [("n_rows", i64), ("mode", c_int), ("prologue", c_int), ("in_dim", c_int), ("in_valid", c_int),
                ("src", c_void_p), ("ld_src", i64), ("src_pre", c_void_p), ("src_res", c_void_p),
                ("in_mu", c_void_p), ("in_scale", c_void_p), ("in_shift", c_void_p),
                ("in_m1", c_void_p), ("in_m2", c_void_p), ("in_invstd", c_void_p),
                ("operand_out", c_void_p), ("operand_max", c_void_p),
                ("blob", c_void_p), ("layer", c_int),
                ("bias", c_void_p), ("add1", c_void_p), ("add2", c_void_p), ("out", c_void_p),
                ("pre_rows", c_void_p), ("out_mu", c_void_p), ("out_invstd", c_void_p), ("out_scale", c_void_p),
                ("out_shift", c_void_p),
                ("partial", c_void_p),
                ("lin_z_table", c_void_p), ("lin_z_scene_stride", i64), ("xyz", c_void_p), ("views", c_void_p),
                ("n_views", c_int), ("rows_per_scene", i64), ("out_max", c_void_p)]


# name -> argtypes (all return int status)
_SIGS = {
    "avr_world_rays": [c_void_p, c_void_p, c_void_p, i64, i64, i64, i64, c_void_p, c_void_p, c_void_p],
    "avr_depth_from_world": [c_void_p, c_void_p, c_void_p, c_void_p, i64, i64, i64, i64, c_void_p, c_void_p,
                             c_void_p],
    "avr_sample_coarse": [c_float, c_float, i64, c_int, c_void_p, u64, u64, c_void_p, c_void_p, c_void_p],
    "avr_sample_fine": [c_void_p, c_void_p, c_float, c_float, i64, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                        c_void_p, u64, u64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_composite_fwd": [c_void_p, c_void_p, i64, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_composite_fwd_depth": [c_void_p, c_void_p, i64, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_rays_sample_coarse": [c_void_p, c_void_p, c_void_p, i64, i64, i64, i64, c_float, c_float, c_int, c_void_p,
                               u64, u64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_composite_bwd": [c_void_p, c_void_p, i64, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_void_p],
    "avr_sample_coarse_rays": [c_void_p, c_void_p, i64, c_int, c_void_p, u64, u64, c_void_p, c_void_p],
    "avr_raymarch": [ctypes.POINTER(ViewDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_raymarch_train": [ctypes.POINTER(ViewDesc), c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p, i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_raymarch_bwd_scratch_bytes": [i64, c_int, i64, ctypes.POINTER(i64)],
    "avr_latent_tables_grad_points": [ctypes.POINTER(ViewDesc), c_int, c_void_p, i64, i64, c_int, c_int, c_void_p, i64,
                                      c_void_p, i64, c_void_p, c_void_p],
    "avr_band_fwd": [i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float, c_void_p, c_void_p, c_void_p],
    "avr_band_bwd": [i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_zfeature_grad_points": [ctypes.POINTER(ViewDesc), c_int, c_void_p, i64, c_void_p, i64, c_int, ctypes.c_float,
                                 c_int, c_void_p, c_void_p],
    "avr_raymarch_bwd": [ctypes.POINTER(ViewDesc), c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, i64, c_int, c_int, c_void_p, c_void_p, c_void_p, i64, c_void_p],
    "avr_march_state_bytes": [i64, ctypes.POINTER(i64)],
    "avr_march_init": [i64, c_void_p, c_void_p, c_void_p],
    "avr_march_gather": [c_void_p, c_void_p, c_void_p, c_void_p, i64, c_int, c_int, c_int, c_void_p, c_void_p,
                         c_void_p, c_void_p],
    "avr_march_composite": [c_void_p, c_void_p, c_void_p, i64, c_int, c_int, c_int, c_float, c_float, c_void_p,
                            c_void_p, c_void_p, c_void_p],
    "avr_march_finish": [c_void_p, i64, c_int, c_void_p, c_void_p, c_void_p],
    "avr_field_packed_floats": [ctypes.POINTER(FieldDims), ctypes.POINTER(i64)],
    "avr_field_pack": [ctypes.POINTER(FieldDims), ctypes.POINTER(ResnetFCWeights), c_void_p, c_void_p],
    "avr_field_latent_table": [ctypes.POINTER(FieldDims), c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "avr_field_latent_table_batch": [ctypes.POINTER(FieldDims), c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                     c_void_p],
    "avr_field_fwd_rays": [ctypes.POINTER(FieldDims), ctypes.POINTER(ViewDesc), c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, i64, c_int, c_void_p, c_void_p],
    "avr_field_fwd_points": [ctypes.POINTER(FieldDims), ctypes.POINTER(ViewDesc), c_void_p, c_void_p, c_void_p,
                             c_void_p, i64, c_void_p, c_void_p],
    "avr_field_fwd_rays_batch": [ctypes.POINTER(FieldDims), ctypes.POINTER(ViewDesc), c_int, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, i64, c_int, c_void_p, c_void_p],
    "avr_field_fwd_points_batch": [ctypes.POINTER(FieldDims), ctypes.POINTER(ViewDesc), c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, i64, c_void_p, c_void_p],
    "avr_field_fwd_points_split": [ctypes.POINTER(FieldDims), ctypes.POINTER(ViewDesc), c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, i64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_field_train_sizes": [ctypes.POINTER(FieldDims), c_int, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)],
    "avr_field_bwd_packed_floats": [ctypes.POINTER(FieldDims), ctypes.POINTER(i64)],
    "avr_field_pack_bwd": [ctypes.POINTER(FieldDims), ctypes.POINTER(ResnetFCWeights), c_void_p, c_void_p],
    "avr_field_fwd_points_train": [ctypes.POINTER(FieldDims), ctypes.POINTER(ViewDesc), c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, i64, c_void_p, c_void_p, i64, c_void_p, c_void_p, c_void_p,
                                   c_int, c_void_p, c_void_p],
    "avr_field_bwd": [ctypes.POINTER(FieldDims), c_void_p, c_void_p, c_int, i64, c_void_p, c_void_p, c_void_p,
                      c_void_p, i64, c_void_p, i64, c_void_p, c_void_p],
    "avr_weight_grads": [ctypes.POINTER(WGradLayer), c_int, i64, c_int, c_void_p],
    "avr_weight_grads_reduce": [ctypes.POINTER(WGradLayer), c_int, c_int, ctypes.POINTER(c_void_p),
                                ctypes.POINTER(c_void_p), c_void_p],
    "avr_latent_features": [ctypes.POINTER(ViewDesc), c_void_p, c_int, c_void_p, i64, c_void_p, c_void_p],
    "avr_latent_features_batch": [ctypes.POINTER(ViewDesc), c_int, c_void_p, c_int, c_void_p, i64, c_void_p, c_void_p],
    "avr_latent_features_grad_points": [ctypes.POINTER(ViewDesc), c_int, c_void_p, c_int, c_void_p, i64, c_void_p,
                                        c_void_p, c_void_p],
    "avr_bn_layer_run": [ctypes.POINTER(FieldDims), ctypes.POINTER(BnLayer), c_void_p],
    "avr_bn_partial_floats": [i64, c_int, ctypes.POINTER(i64)],
    "avr_bn_stats": [c_void_p, i64, c_int, c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p],
    "avr_bn_grad_stats": [c_void_p, i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p],
    "avr_bn_grad_rows": [i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p],
    "avr_lin_out_fwd_rows": [i64, c_int, c_void_p, i64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_lin_out_bwd_rows": [i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, i64, c_void_p, c_void_p, c_void_p,
                             c_void_p],
    "avr_lin_out_act_bwd_rows": [i64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_spade_bwd_rows": [i64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "avr_stream_copy": [c_void_p, c_void_p, i64, c_void_p],
    "avr_stream_fill": [c_void_p, i64, c_uint32, c_void_p],
}
EXPORTED = ("avr_version", "avr_last_error_string", "avr_device_count") + tuple(_SIGS)

_lib = None


class AVRError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load (once) and return the ctypes handle. Raises if the .so is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise AVRError(f"libavr_hip.so not built at {path}: run `make -C adaptive-volume-rendering_amd` "
                       "(or __graft_entry__.build()); there is no non-HIP fallback")
    torch.cuda.is_available()  # make torch's HIP runtime the one the library binds to
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    lib.avr_version.restype = c_int
    lib.avr_last_error_string.restype = ctypes.c_char_p
    lib.avr_device_count.restype = c_int
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = c_int
    if lib.avr_version() != ABI_VERSION:
        raise AVRError(f"libavr_hip.so ABI {lib.avr_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().avr_last_error_string().decode(errors="replace")
        raise AVRError(f"{what} failed (code {rc}): {msg}")


def call(name, *args):
    check(getattr(load(), name)(*args), name)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t):
    """hipStream_t of torch's current stream on t's device (the raw handle without building a torch Stream object:
    a few microseconds per launch of host time, dozens of launches per training step)."""
    if _raw_stream is not None and t.is_cuda:
        return c_void_p(_raw_stream(t.get_device()))
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def require_device(*tensors):
    """Every tensor must be a contiguous fp32 (or int32) tensor on a HIP device."""
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise AVRError("avr kernels need tensors on a ROCm/HIP device (got device %s); there is no CPU path"
                           % t.device)
        if not t.is_contiguous():
            raise AVRError("avr kernels need contiguous tensors")
