"""Fused HIP evaluation of a NewPixelNeRFNet (models.py:739-863).

FusedField repacks each ResnetFC into MFMA fragment order (avr_field_pack),
projects the latent map through lin_z once per texel (avr_field_latent_table)
and evaluates sigma/RGB with one kernel launch per pass (avr_field_fwd_rays /
avr_field_fwd_points). Packed weights and tables are cached and rebuilt when a
parameter or the latent changes (tensor version counters), so an inference
loop over many frames of one scene pays for them once, as the reference pays
for encode() once.
"""
import collections
import ctypes
import os
import weakref

import torch
from torch.optim.optimizer import register_optimizer_step_post_hook

from . import _lib
from ._lib import FieldDims, ResnetFCWeights, ViewDesc, call, ptr, require_device, stream_of

F32 = torch.float32


def uses_bn(mlp):
    """ResnetBlockFC(bn=True) blocks (train.py --bn, models.py:430-432, 456-461)."""
    return any(getattr(blk, "bn", False) for blk in getattr(mlp, "blocks", ()))


def softplus_beta(mlp):
    """beta of a ResnetFC(beta > 0) (models.py:442-445, 536-537: Softplus(beta) everywhere the
    ReLU would be), 0.0 for ReLU nets, None for anything else (torch's default threshold 20 only)."""
    acts = [mlp.activation] + [blk.activation for blk in mlp.blocks]
    if all(isinstance(a, torch.nn.ReLU) for a in acts):
        return 0.0
    if all(isinstance(a, torch.nn.Softplus) and a.threshold == 20 and a.beta > 0 for a in acts):
        betas = {float(a.beta) for a in acts}
        if len(betas) == 1:
            return betas.pop()
    return None


def inference_only(mlp):
    """ResnetFC options the fused x3 kernels run for inference only: BatchNorm (training mode trains layer by
    layer, avr.bn_train) and use_spade (module path). Softplus(beta) trains on the fused kernels (ABI 11)."""
    return uses_bn(mlp) or getattr(mlp, "use_spade", False)


def _bn_ok(blk):
    """Eval-mode BatchNorm with running statistics: a per-feature affine the
    x3 kernel applies (training-mode BN needs cross-sample statistics: module
    path)."""
    bn = blk.bn_0
    return (not blk.training and not bn.training and bn.track_running_stats and bn.running_mean is not None
            and bn.affine)


def _resnetfc_ok(mlp, d_in, d_latent, precision="x3"):
    if not (mlp is not None and type(mlp).__name__ == "ResnetFC" and getattr(mlp, "d_in", -1) == d_in
            and mlp.d_latent == d_latent and mlp.d_out == 4 and mlp.d_hidden in (64, 128, 256, 512)
            and 1 <= mlp.n_blocks <= _lib.AVR_MAX_BLOCKS and all(blk.shortcut is None for blk in mlp.blocks)):
        return False
    beta = softplus_beta(mlp)
    spade = getattr(mlp, "use_spade", False)
    bn = uses_bn(mlp)
    if beta is None or ((spade or beta > 0 or bn) and precision != "x3"):
        return False          # the fp32 kernel runs the default ReLU net only
    if bn and (spade or beta > 0):
        return False          # BatchNorm with use_spade / Softplus: module path
    return all(not blk.bn or _bn_ok(blk) for blk in mlp.blocks)


def fused_eligible(net, multiview=False):
    """True when `net` is a NewPixelNeRFNet configured like conf/default*.conf:
    local encoder, xyz + PE(xyz) + raw viewdirs, normalize_z, bilinear/border
    latent lookup, ResNet MLPs (eval-mode BatchNorm, use_spade and Softplus
    allowed on the x3 path), one source view. multiview: instead NS > 1 source
    views, x3, every MLP combining them (combine_layer < n_blocks, mean or max):
    FusedField.forward_points_multiview."""
    try:
        ns = net.num_views_per_obj
        if multiview:
            mlps = [net.mlp_coarse] + ([net.mlp_fine] if net.mlp_fine is not None else [])
            if not (ns > 1 and getattr(net, "field_precision", "x3") == "x3"
                    and all(1 <= m.combine_layer < m.n_blocks and m.combine_type in ("average", "max")
                            for m in mlps)):
                # combine_layer 0 (views combined right after lin_in, no lin_z): module path -- the split
                # launch's first half needs at least one block (avr_field_fwd_points_split, b_end > 0)
                return False
        elif ns != 1:
            return False
        code = getattr(net, "code", None)
        enc = net.encoder
        ok = (net.use_encoder and net.use_xyz and net.normalize_z and net.use_code and net.use_viewdirs
              and not net.use_code_viewdirs and not getattr(net, "use_global_encoder", False)
              and code is not None and code.include_input and code.d_in == 3
              and getattr(enc, "index_interp", "bilinear") == "bilinear"
              and getattr(enc, "index_padding", "border") == "border"
              and enc.latent.dim() == 4 and enc.latent.shape[1] % 16 == 0 and enc.latent.shape[1] <= 1024
              and net.d_in == 6 * code.num_freqs + 6)
        if not ok:
            return False
        mlps = [net.mlp_coarse] + ([net.mlp_fine] if net.mlp_fine is not None else [])
        precision = getattr(net, "field_precision", "x3")
        return all(_resnetfc_ok(m, net.d_in, net.d_latent, precision) for m in mlps)
    except AttributeError:
        return False


def _freq_factor(code):
    ff = getattr(code, "freq_factor", None)
    if ff is None:
        ff = float(code.freqs[0])
    return float(ff)


class _precision:
    """dims.precision set for one library call and restored after it."""

    def __init__(self, dims, value):
        self.dims, self.value = dims, value

    def __enter__(self):
        self.saved = self.dims.precision
        self.dims.precision = self.value

    def __exit__(self, *exc):
        self.dims.precision = self.saved
        return False


# Submodule (re)registrations anywhere in the process, numbered, with the id of the module that registered: a
# FusedField._state slot is rebuilt after a registration under its MLP, so a module replaced in an MLP
# (mlp.lin_in = nn.Linear(...)) is seen, and only then (modules built elsewhere, e.g. per training step, leave it
# alone); parameters and buffers replaced in place are read through their owners' dicts anyway.
_MODULE_GEN = [0]
_REG_LOG = collections.deque(maxlen=4096)   # (generation, id(parent module))


def _module_registered(module, name, submodule):
    _MODULE_GEN[0] += 1
    _REG_LOG.append((_MODULE_GEN[0], id(module)))


def _slot_current(gen, module_ids):
    """No registration since generation `gen` under a module of module_ids (the log must still cover them all;
    a reused id only costs a rebuild)."""
    if gen == _MODULE_GEN[0]:
        return True
    if not _REG_LOG or _REG_LOG[0][0] > gen + 1:
        return False
    return not any(pid in module_ids for g, pid in _REG_LOG if g > gen)


torch.nn.modules.module.register_module_module_registration_hook(_module_registered)


# Every optimizer step anywhere in the process, counted: a fused optimizer (torch.optim.Adam(fused=True)) updates
# the parameters in one multi-tensor kernel without advancing their version counters, so the (data_ptr, _version)
# keys of the caches below would not see it (the blob would keep the old weights). The count is part of every key;
# GraphedTrainStep advances it after each replay (a captured optimizer step runs no host hook).
_PARAM_GEN = [0]
_EXPLICIT_GEN = [0]   # bump_param_generation() calls alone: the key of latent maps no optimizer can hold


def _optimizer_stepped(optimizer, args, kwargs):
    _PARAM_GEN[0] += 1


register_optimizer_step_post_hook(_optimizer_stepped)


def bump_param_generation():
    """Invalidate every FusedField cache entry derived from parameters or the latent map (after an update the
    version counters do not record: a replayed optimizer step, a write through .data)."""
    _PARAM_GEN[0] += 1
    _EXPLICIT_GEN[0] += 1


def param_generation():
    return _PARAM_GEN[0]


def _version_key(tensors, gen=True):
    """(data_ptr, _version) of each tensor, with the optimizer-step generation for anything an optimizer may
    update (gen=False: the source views -- poses, focal, principal point -- which none does)."""
    return ((_PARAM_GEN[0],) if gen else ()) + tuple((t.data_ptr(), t._version) for t in tensors)


def _stamp(t):
    """(stream, event) marking the current stream's work that filled the cached device tensor t (None on the CPU
    or while a HIP graph is being captured: one stream then, nothing to join)."""
    if t is None or not t.is_cuda or torch.cuda.is_current_stream_capturing():
        return None
    s = torch.cuda.current_stream(t.device)
    ev = torch.cuda.Event()
    ev.record(s)
    return s, ev


def _join(stamp, *tensors):
    """A cached value read from another stream than the one that made it (the adaptive renderer's side stream,
    avr.renderers): that stream waits for the maker's work, and the tensors' memory is kept from reuse under the
    maker's later allocations until this stream's work on them is done."""
    if stamp is None:
        return
    s = torch.cuda.current_stream(stamp[0].device)
    if s == stamp[0]:
        return
    s.wait_event(stamp[1])
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(s)


class _Packed:
    def __init__(self, dims, packed, table_keys):
        self.dims = dims
        self.packed = packed
        self.tables = {}
        self.bwd = None
        self.bwd_stamp = None
        self.stamp = None


PRECISIONS = {"fp32": _lib.FIELD_FP32, "x3": _lib.FIELD_X3}


def n_tables(dims):
    """Per-texel tables of a packed net: lin_z[b], then scale_z[b] with use_spade."""
    return dims.n_lin_z * (2 if dims.spade else 1)


class FusedField:
    """precision: "x3" (default) = split-fp16 MFMA (3 products per fp32 product,
    fp32 accumulation, within fp32 noise of the fp32 path); "fp32" = fp32 MFMA."""

    def __init__(self, net, precision="x3"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self.precision = precision
        self.net = net
        self._packed = {}     # coarse(bool) -> (key, _Packed)
        self._pack_args = {}  # coarse(bool) -> (pointer key, blob floats, ResnetFCWeights, kept tensors)
        self._view_cache = {}
        self._views_cache = {}    # (range, ns) -> ViewDesc arrays (views())
        self._latent_cache = {}   # per latent version: channels-last copies, max |latent| (both MLPs share them)
        # mlp (weakly) -> ([(name, owner dict, key)] params, [...] float buffers, generation, ids of its modules)
        self._slots = weakref.WeakKeyDictionary()

    def invalidate(self, views=True):
        """Drop every cached blob, table and (views=True) view descriptor (avr.parallel.broadcast_scene calls it
        after writing a scene into the net; the (data_ptr, _version) keys would catch that too). views=False keeps
        the host-side view descriptors (avr.graphs.GraphedTrainStep before a capture: building one reads the poses
        back to the host, which a capture cannot do)."""
        self._packed.clear()
        self._pack_args.clear()
        if views:
            self._view_cache.clear()
            self._views_cache.clear()
        self._latent_cache.clear()

    def cache_tensors(self):
        """Every device buffer the caches hold (packed blobs, backward blobs, lin_z tables, batched tables):
        what a captured HIP graph reads (avr.graphs.GraphedRenderer keeps references to them, so an eager call
        that replaces a cache entry cannot free memory a replay still reads)."""
        out = []
        for _, entry in self._packed.values():
            if entry is None:
                continue
            out.append(entry.packed)
            if getattr(entry, "bwd", None) is not None:
                out.append(entry.bwd)
            out += [hit[1] for hit in entry.tables.values()]
            out += [hit[1] for hit in entry.__dict__.get("batch_tables", {}).values()]
        return out

    def _latent_cached(self, what, latent, make):
        # the optimizer-step count matters only for a latent an optimizer can hold (a leaf that requires grad): a
        # fixed or encoder-produced map keeps its copies across steps (its version counter sees in-place writes)
        gen = _PARAM_GEN[0] if (latent.is_leaf and latent.requires_grad) else (-1, _EXPLICIT_GEN[0])
        key = (gen, latent.data_ptr(), latent._version, tuple(latent.shape))
        hit = self._latent_cache.get(what)
        if hit is not None and hit[0] == key:
            _join(hit[3], hit[1])
            return hit[1]
        val = make()
        # holding `latent` keeps its address from being reused
        self._latent_cache[what] = (key, val, latent, _stamp(val))
        return val

    def latent_hwc(self, latent, s):
        """Scene s's latent map channels-last (avr_latent_features' operand), once per latent version."""
        from .ops import latent_hwc
        return self._latent_cached(("hwc", s), latent, lambda: latent_hwc(latent[s]))

    def latent_hwc_all(self, latent):
        """Every scene's latent map channels-last, (SB, H*W, C), once per latent version."""
        def make():
            SB, C, H, W = latent.shape
            return latent.detach().to(F32).reshape(SB, C, H * W).transpose(1, 2).contiguous()
        return self._latent_cached("hwc_all", latent, make)

    def latent_max_bits(self, latent):
        """max |latent| as int32 float bits (the lin_z weight gradients' X scale), once per latent version."""
        from .ops import _max_bits
        return self._latent_cached("max", latent, lambda: _max_bits(latent))

    # ----------------------------------------------------------- parameters
    def _state(self, mlp):
        """(named parameters, parameters, floating-point buffers) of mlp in named_parameters() / buffers() order,
        read through each owning module's dict: the module tree is walked once per mlp and again after any
        submodule registration (a walk per call was a large part of the adaptive step's host time), and a
        parameter or buffer replaced later is still seen."""
        hit = self._slots.get(mlp)
        if hit is not None and hit[2] != _MODULE_GEN[0]:
            hit = (hit[0], hit[1], _MODULE_GEN[0], hit[3]) if _slot_current(hit[2], hit[3]) else None
            if hit is not None:
                self._slots[mlp] = hit
        if hit is None:
            mods = list(mlp.named_modules())
            ps = [(f"{mn}.{n}" if mn else n, m._parameters, n) for mn, m in mods
                  for n, t in m._parameters.items() if t is not None]
            bs = [(f"{mn}.{n}" if mn else n, m._buffers, n) for mn, m in mods
                  for n, t in m._buffers.items() if t is not None and t.is_floating_point()]
            hit = (ps, bs, _MODULE_GEN[0], frozenset(id(m) for _, m in mods))
            self._slots[mlp] = hit
        named = {full: d[k] for full, d, k in hit[0]}
        return named, list(named.values()), [d[k] for _, d, k in hit[1]]

    def _mlp(self, coarse):
        net = self.net
        return net.mlp_coarse if (coarse or net.mlp_fine is None) else net.mlp_fine

    def dims(self, mlp):
        code = self.net.code
        return FieldDims(self.net.d_in, self.net.d_latent, mlp.d_hidden, mlp.n_blocks,
                         min(mlp.combine_layer, mlp.n_blocks), code.num_freqs, _freq_factor(code),
                         PRECISIONS[self.precision], int(uses_bn(mlp)), int(getattr(mlp, "use_spade", False)),
                         float(softplus_beta(mlp) or 0.0))

    def packed(self, coarse, bn_fold=True):
        """bn_fold=False: the training-mode BatchNorm path's blob (avr.bn_train): x3, raw fc_0 weights (no
        eval-BN folding, dims.bn = 0), cached beside the inference blob."""
        mlp = self._mlp(coarse)
        _, ps, bs = self._state(mlp)
        params = ps + bs
        # the precision is part of the key: an x3 blob holds only the fragments the x3 kernels read
        # (avr_field_pack), and net.fused() switches a FusedField's precision in place
        slot = coarse if bn_fold else (coarse, "bn_train")
        key = (id(mlp), self.precision if bn_fold else "x3", _version_key(params))
        hit = self._packed.get(slot)
        if hit is not None and hit[0] == key:
            _join(hit[1].stamp, hit[1].packed)
            return hit[1]
        dims = self.dims(mlp)
        if not bn_fold:
            dims.bn, dims.precision = 0, _lib.FIELD_X3
        # an optimizer step updates the parameters in place: the same tensors at the same addresses, so the last
        # build's weight pointers, blob size and kept tensors serve again and only the pack launch reruns (when
        # every pointer was a parameter or buffer read in place; derived tensors -- the eval-BN folds, dtype
        # conversions -- are rebuilt every time)
        args_key = (id(mlp), tuple(pv[0] for pv in key[2][1:]), bytes(dims))
        args = self._pack_args.get(slot)
        if args is not None and args[0] == args_key:
            _, n, w, keep = args
            packed = torch.empty(n, device=params[0].device, dtype=F32)
            call("avr_field_pack", ctypes.byref(dims), ctypes.byref(w), ptr(packed), stream_of(packed))
            return self._store_packed(slot, key, dims, packed, keep, w)
        n = ctypes.c_int64(0)
        _lib.check(_lib.load().avr_field_packed_floats(ctypes.byref(dims), ctypes.byref(n)), "avr_field_packed_floats")
        dev = params[0].device
        packed = torch.empty(n.value, device=dev, dtype=F32)
        w = ResnetFCWeights()
        keep = []
        derived = [False]

        def P(t):
            if not (t.dtype == F32 and t.is_contiguous()):   # (fp32 contiguous parameters: read in place)
                t = t.detach().to(F32).contiguous()
                derived[0] = True
            keep.append(t)
            return t.data_ptr()

        w.lin_in_w, w.lin_in_b = P(mlp.lin_in.weight), P(mlp.lin_in.bias)
        w.lin_out_w, w.lin_out_b = P(mlp.lin_out.weight), P(mlp.lin_out.bias)
        for b, blk in enumerate(mlp.blocks):
            if dims.bn:
                # eval BatchNorm1d as y = a x + c (torch's batch_norm: a = w / sqrt(var + eps), c = b - mean a);
                # bn_0 sits in front of both relus of the block (models.py:456-461): the first is applied by
                # the kernel, the second folds into fc_0's rows
                bn = blk.bn_0
                a = (bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps))
                c = bn.bias.detach().float() - bn.running_mean.detach().float() * a
                w.bn_scale[b], w.bn_shift[b] = P(a), P(c)
                w.fc0_w[b] = P(blk.fc_0.weight.detach().float() * a[:, None])
                w.fc0_b[b] = P(blk.fc_0.bias.detach().float() * a + c)
            else:
                w.fc0_w[b], w.fc0_b[b] = P(blk.fc_0.weight), P(blk.fc_0.bias)
            w.fc1_w[b], w.fc1_b[b] = P(blk.fc_1.weight), P(blk.fc_1.bias)
        for b in range(dims.n_lin_z):
            w.lin_z_w[b], w.lin_z_b[b] = P(mlp.lin_z[b].weight), P(mlp.lin_z[b].bias)
            if dims.spade:   # scale_z[b](z) * x + lin_z[b](z) (models.py:585-587): both as per-texel tables
                w.scale_z_w[b], w.scale_z_b[b] = P(mlp.scale_z[b].weight), P(mlp.scale_z[b].bias)
        require_device(*keep)
        call("avr_field_pack", ctypes.byref(dims), ctypes.byref(w), ptr(packed), stream_of(packed))
        if dims.bn or derived[0]:
            self._pack_args.pop(slot, None)
        else:
            self._pack_args[slot] = (args_key, n.value, w, keep)
        return self._store_packed(slot, key, dims, packed, keep, w)

    def _store_packed(self, slot, key, dims, packed, keep, w):
        entry = _Packed(dims, packed, None)
        entry._keep = keep
        entry.weights = w
        entry.stamp = _stamp(packed)
        self._packed[slot] = (key, entry)
        return entry

    def packed_bwd(self, coarse, entry=None):
        """Transposed fc_0 / fc_1 fragments for the backward kernel, cached with
        the forward blob (rebuilt whenever a parameter changes)."""
        entry = entry or self.packed(coarse)
        if getattr(entry, "bwd", None) is None:
            dims = entry.dims
            n = ctypes.c_int64(0)
            _lib.check(_lib.load().avr_field_bwd_packed_floats(ctypes.byref(dims), ctypes.byref(n)),
                       "avr_field_bwd_packed_floats")
            bwd = torch.empty(n.value, device=entry.packed.device, dtype=F32)
            call("avr_field_pack_bwd", ctypes.byref(dims), ctypes.byref(entry.weights), ptr(bwd), stream_of(bwd))
            entry.bwd, entry.bwd_stamp = bwd, _stamp(bwd)
        else:
            _join(entry.bwd_stamp, entry.bwd)
        return entry.bwd

    def table(self, coarse, sb=0):
        entry = self.packed(coarse)
        lat = self.net.encoder.latent
        key = (sb, _PARAM_GEN[0], lat.data_ptr(), lat._version, tuple(lat.shape))
        hit = entry.tables.get(sb)
        if hit is not None and hit[0] == key:
            _join(hit[3], hit[1])
            return hit[1]
        dims = entry.dims
        L, H, W = lat.shape[1:]
        latent = lat[sb].detach().to(F32).contiguous()
        require_device(latent)
        table = torch.empty(max(n_tables(dims), 1), H * W, dims.d_hidden, device=latent.device, dtype=F32)
        with _precision(dims, _lib.FIELD_FP32):   # inference: exact fp32 tables, computed once per latent map
            call("avr_field_latent_table", ctypes.byref(dims), ptr(entry.packed), ptr(latent), H, W, ptr(table),
                 stream_of(table))
        entry.tables[sb] = (key, table, lat, _stamp(table))  # holding `lat` keeps its address from being reused
        return table

    def tables_batch(self, coarse, n_scenes, fast=False, bn_fold=True, entry=None):
        """The lin_z tables of scenes 0 .. n_scenes-1 back to back, (n_scenes,
        max(n_tables, 1), H*W, d_hidden): one buffer for the multi-scene launches.
        fast (the training path, which recomputes them every step): on the split-fp16
        GEMM (table_x3_kernel); otherwise exact fp32 products. bn_fold: which blob's
        cache holds them (packed()); entry: that packed() result when the caller has it."""
        entry = entry or self.packed(coarse, bn_fold)
        lat = self.net.encoder.latent
        key = (n_scenes, bool(fast), _PARAM_GEN[0], lat.data_ptr(), lat._version, tuple(lat.shape))
        cache = entry.__dict__.setdefault("batch_tables", {})
        hit = cache.get(bool(fast))
        if hit is not None and hit[0] == key:
            _join(hit[3], hit[1])
            return hit[1]
        dims = entry.dims
        L, H, W = lat.shape[1:]
        out = torch.empty(n_scenes, max(n_tables(dims), 1), H * W, dims.d_hidden, device=lat.device, dtype=F32)
        with _precision(dims, _lib.FIELD_X3 if fast else _lib.FIELD_FP32):
            if n_scenes <= lat.shape[0]:   # every scene its own map: one launch
                latent = lat[:n_scenes].detach().to(F32).contiguous()
                call("avr_field_latent_table_batch", ctypes.byref(dims), ptr(entry.packed), ptr(latent), n_scenes,
                     H, W, ptr(out), stream_of(out))
            else:
                for sb in range(n_scenes):
                    latent = lat[min(sb, lat.shape[0] - 1)].detach().to(F32).contiguous()
                    call("avr_field_latent_table", ctypes.byref(dims), ptr(entry.packed), ptr(latent), H, W,
                         ptr(out[sb]), stream_of(out))
        cache[bool(fast)] = (key, out, lat, _stamp(out))
        return out

    def view(self, sb=0, ns=1):
        """Source view sb (pose sb; with ns > 1 views per object, focal / principal point of
        object sb // ns, as models.py:796-801 repeat_interleaves them)."""
        net = self.net
        srcs = [net.poses, net.focal, net.c, net.image_shape, net.encoder.latent_scaling]
        key = (sb, ns, _version_key(srcs, gen=False), tuple(net.encoder.latent.shape))
        hit = self._view_cache.get((sb, ns))
        if hit is not None and hit[0] == key:
            return hit[1]
        pick = lambda t, i=sb: t[min(i, t.shape[0] - 1)] if t.dim() > 1 else t  # noqa: E731
        v = ViewDesc()
        v.poses[:] = [float(x) for x in pick(net.poses).reshape(-1)[:12].tolist()]
        v.focal[:] = [float(x) for x in pick(net.focal, sb // ns).reshape(-1)[:2].tolist()]
        v.c[:] = [float(x) for x in pick(net.c, sb // ns).reshape(-1)[:2].tolist()]
        v.image_shape[:] = [float(x) for x in net.image_shape.reshape(-1)[:2].tolist()]
        v.latent_scaling[:] = [float(x) for x in net.encoder.latent_scaling.reshape(-1)[:2].tolist()]
        v.latent_h, v.latent_w = int(net.encoder.latent.shape[-2]), int(net.encoder.latent.shape[-1])
        self._view_cache[(sb, ns)] = (key, v, srcs)  # holding the sources keeps (ptr, version) keys sound
        return v

    def views(self, idx, ns=1):
        """The ViewDesc array of view(i, ns) for i in the range idx (the multi-scene launches' argument), cached
        under one source-version key (per-view keys for every scene of every launch were host time)."""
        net = self.net
        srcs = [net.poses, net.focal, net.c, net.image_shape, net.encoder.latent_scaling]
        slot = (idx.start, idx.stop, idx.step, ns)
        key = (_version_key(srcs, gen=False), tuple(net.encoder.latent.shape))
        hit = self._views_cache.get(slot)
        if hit is not None and hit[0] == key:
            return hit[1]
        arr = (ViewDesc * len(idx))(*[self.view(i, ns) for i in idx])
        self._views_cache[slot] = (key, arr, srcs)   # holding the sources keeps (ptr, version) keys sound
        return arr

    # ----------------------------------------------------------- evaluation
    def forward_rays(self, ro, rd, z, coarse, sb=0):
        """sigma/RGB at ro[r] + rd[r]*z[r,s] with viewdir rd[r]: (R*N, 4)."""
        R, N = z.shape
        ro = ro.reshape(R, 3).to(F32).contiguous()
        rd = rd.reshape(R, 3).to(F32).contiguous()
        z = z.to(F32).contiguous()
        require_device(ro, rd, z)
        entry = self.packed(coarse)
        table = self.table(coarse, sb)
        out = torch.empty(R * N, 4, device=z.device, dtype=F32)
        entry.dims.precision = PRECISIONS[self.precision]
        call("avr_field_fwd_rays", ctypes.byref(entry.dims), ctypes.byref(self.view(sb)), ptr(entry.packed),
             ptr(table), ptr(ro), ptr(rd), ptr(z), R, N, ptr(out), stream_of(z))
        return out

    def forward_rays_batch(self, ro, rd, z, coarse):
        """SB scenes at once: ro, rd (SB, R, 3), z (SB*R, N) -> (SB*R*N, 4); one x3
        launch per group of up to AVR_MAX_SCENES scenes (avr_field_fwd_rays_batch)."""
        SB, R, _ = ro.shape
        N = z.shape[-1]
        ro = ro.to(F32).contiguous()
        rd = rd.to(F32).contiguous()
        z = z.to(F32).reshape(SB * R, N).contiguous()
        require_device(ro, rd, z)
        out = torch.empty(SB * R * N, 4, device=z.device, dtype=F32)
        if self.precision != "x3":     # the fp32 kernel is single-scene
            for b in range(SB):
                out[b * R * N:(b + 1) * R * N] = self.forward_rays(ro[b], rd[b], z[b * R:(b + 1) * R], coarse, sb=b)
            return out
        entry = self.packed(coarse)
        tables = self.tables_batch(coarse, SB)
        entry.dims.precision = _lib.FIELD_X3
        for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
            n = min(_lib.AVR_MAX_SCENES, SB - g0)
            views = self.views(range(g0, g0 + n))
            call("avr_field_fwd_rays_batch", ctypes.byref(entry.dims), views, n, ptr(entry.packed), ptr(tables[g0]),
                 ptr(ro[g0]), ptr(rd[g0]), ptr(z[g0 * R]), R, N, ptr(out[g0 * R * N]), stream_of(z))
        return out

    def forward_points_multiview(self, xyz, viewdirs, coarse):
        """NS = net.num_views_per_obj > 1 source views per object (models.py:749-853): the MLP's
        first combine_layer blocks run on every (object, view) pair (avr_field_fwd_points_split,
        first launch), the residual streams are combined over the views exactly as ResnetFC does
        (combine_interleaved, models.py:566-579 / utils.py:71-81: mean or max over NS), and the
        remaining blocks + lin_out run once per object (second launch). (SB, B, 3) -> (SB, B, 4)."""
        from .models import combine_interleaved
        net = self.net
        NS = net.num_views_per_obj
        SB, B, _ = xyz.shape
        mlp = self._mlp(coarse)
        entry = self.packed(coarse)
        dims = entry.dims
        H, nb, cl = dims.d_hidden, dims.n_blocks, mlp.combine_layer
        dev = xyz.device
        p = xyz.to(F32).repeat_interleave(NS, 0).contiguous()              # (SB*NS, B, 3), views of an object adjacent
        v = viewdirs.reshape(SB, B, 3).to(F32).repeat_interleave(NS, 0).contiguous()
        require_device(p, v)
        K = SB * NS
        tables = self.tables_batch(coarse, K)
        h = torch.empty(K * B, H, device=dev, dtype=F32)
        out = torch.empty(SB, B, 4, device=dev, dtype=F32)
        with _precision(dims, _lib.FIELD_X3):
            for g0 in range(0, K, _lib.AVR_MAX_SCENES):
                n = min(_lib.AVR_MAX_SCENES, K - g0)
                views = self.views(range(g0, g0 + n), NS)
                call("avr_field_fwd_points_split", ctypes.byref(entry.dims), views, n, ptr(entry.packed),
                     ptr(tables[g0]), ptr(p[g0]), ptr(v[g0]), B, 0, cl, None, ptr(h[g0 * B]), None, stream_of(p))
            hc = combine_interleaved(h, (NS, B), mlp.combine_type).reshape(SB * B, H).contiguous()
            for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
                n = min(_lib.AVR_MAX_SCENES, SB - g0)
                views = self.views(range(g0 * NS, (g0 + n) * NS, NS), NS)
                call("avr_field_fwd_points_split", ctypes.byref(entry.dims), views, n, ptr(entry.packed),
                     ptr(tables[0]), None, None, B, cl, nb, ptr(hc[g0 * B]), None, ptr(out[g0]), stream_of(p))
        return out

    def forward_points(self, xyz, viewdirs, coarse):
        """The rf(xyz (SB,B,3), viewdirs, coarse) protocol -> (SB, B, 4)."""
        if getattr(self.net, "num_views_per_obj", 1) > 1:
            # NS > 1 runs on the x3 split launches only: another precision or an ineligible combine must not be
            # served silently at x3
            if self.precision != "x3" or not fused_eligible(self.net, multiview=True):
                raise _lib.AVRError("FusedField.forward_points: NS > 1 source views need precision 'x3' and an "
                                    "eligible combine (1 <= combine_layer < n_blocks); use the module path")
            return self.forward_points_multiview(xyz, viewdirs, coarse)
        SB, B, _ = xyz.shape
        out = torch.empty(SB, B, 4, device=xyz.device, dtype=F32)
        entry = self.packed(coarse)
        if SB > 1 and self.precision == "x3":   # one launch per group of scenes
            p = xyz.to(F32).contiguous()
            v = viewdirs.reshape(SB, B, 3).to(F32).contiguous()
            require_device(p, v)
            tables = self.tables_batch(coarse, SB)
            entry.dims.precision = _lib.FIELD_X3
            for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
                n = min(_lib.AVR_MAX_SCENES, SB - g0)
                views = self.views(range(g0, g0 + n))
                call("avr_field_fwd_points_batch", ctypes.byref(entry.dims), views, n, ptr(entry.packed),
                     ptr(tables[g0]), ptr(p[g0]), ptr(v[g0]), B, ptr(out[g0]), stream_of(p))
            return out
        for sb in range(SB):
            p = xyz[sb].to(F32).contiguous()
            v = viewdirs.reshape(SB, B, 3)[sb].to(F32).contiguous()
            require_device(p, v)
            table = self.table(coarse, sb)
            entry.dims.precision = PRECISIONS[self.precision]
            call("avr_field_fwd_points", ctypes.byref(entry.dims), ctypes.byref(self.view(sb)), ptr(entry.packed),
                 ptr(table), ptr(p), ptr(v), B, ptr(out[sb]), stream_of(p))
        return out

    # ----------------------------------------------------------- training
    def forward_train(self, xyz, viewdirs, coarse):
        """The rf(xyz, viewdirs, coarse) protocol with autograd: HIP forward that
        keeps every GEMM input, HIP backward through the ResnetFC, weight
        gradients as GEMMs over the samples (see _FieldTrain)."""
        mlp = self._mlp(coarse)
        names = train_param_names(mlp)
        named, _, _ = self._state(mlp)
        params = [named[n] for n in names]
        return _FieldTrain.apply(self, coarse, names, xyz, viewdirs, self.net.encoder.latent, *params)


def _feat_grad(fused, entry, bwd, Gz, P, Mt):
    """The looked-up latent features' gradient sum_b Gz[b] . W_z[b] (the point / latent gradients' input):
    avr_bn_layer_run's lin_z[b]^T layers from the backward blob (x3, ABI 14), one launch per layer adding the
    previous layers' sum in its epilogue, where they apply (d_latent == d_hidden, ReLU, 64..512 wide); else
    fp32 library GEMMs (avr.ops.sum_of_products)."""
    from .bn_train import _layer, _partial, _run
    from .ops import sum_of_products
    dims = entry.dims
    H, nz = dims.d_hidden, dims.n_lin_z
    if not (dims.d_latent == H and H in (64, 128, 256, 512) and not dims.spade and not dims.bn
            and not dims.beta > 0 and Mt > 0 and all(g.is_contiguous() for g in Gz)):
        return sum_of_products([(Gz[b], P[f"lin_z.{b}.weight"].detach()) for b in range(nz)])
    dev = Gz[0].device
    part = _partial(Mt, H, dev)
    stream = stream_of(Gz[0])
    prev = None
    saved, dims.precision = dims.precision, _lib.FIELD_X3
    try:
        for b in range(nz):
            out = torch.empty(Mt, H, device=dev, dtype=F32)
            _run(dims, _layer(n_rows=Mt, mode=_lib.BN_BWD, prologue=_lib.BN_PLAIN, in_dim=H, in_valid=H, src=Gz[b],
                              ld_src=H, blob=bwd, layer=_lib.BN_LAYER_LIN_Z_T + b, add1=prev, out=out, partial=part),
                 stream)
            prev = out
    finally:
        dims.precision = saved
    return prev


def train_param_names(mlp):
    """The ResnetFC parameters the training path differentiates, in a fixed order."""
    names = ["lin_in.weight", "lin_in.bias", "lin_out.weight", "lin_out.bias"]
    for b in range(mlp.n_blocks):
        names += [f"blocks.{b}.fc_0.weight", f"blocks.{b}.fc_0.bias", f"blocks.{b}.fc_1.weight", f"blocks.{b}.fc_1.bias"]
    for b in range(min(mlp.combine_layer, mlp.n_blocks)):
        names += [f"lin_z.{b}.weight", f"lin_z.{b}.bias"]
    return names


class _FieldTrain(torch.autograd.Function):
    """Autograd of NewPixelNeRFNet.forward (models.py:739-863) for train.py's
    loss.backward() (train.py:108-114).

    forward: avr_field_fwd_points_train per scene (x3 MFMA, the inference
    kernel plus a store of every hidden GEMM input, its relu mask and the
    layer's running max) into one (layers, SB * B, d_hidden) buffer.
    backward: avr_field_bwd runs the input-gradient chain per scene (lin_out^T,
    then fc_1^T / fc_0^T per block with the relu masks, x3 MFMA) and writes the
    gradient at every layer output; avr_weight_grads then forms every weight
    and bias gradient in one batched split-K x3 GEMM over all samples
    (fc_0 / fc_1 against the saved inputs, lin_z against the interpolated latent
    (grid_sample, models.py:266-273), lin_in against the positional-encoded
    input). The latent map gets the grid_sample adjoint of sum_b G_z[b] W_z[b]
    when it requires grad."""

    @staticmethod
    def forward(ctx, fused, coarse, names, xyz, viewdirs, latent, *params):
        SB, B, _ = xyz.shape
        entry = fused.packed(coarse)
        dims = entry.dims
        dims.precision = _lib.FIELD_X3
        H, nb = dims.d_hidden, dims.n_blocks
        n_l, Mt = 2 * nb + 1, SB * B
        dev = xyz.device
        out = torch.empty(SB, B, 4, device=dev, dtype=F32)
        act = torch.empty(n_l, Mt, H, device=dev, dtype=F32)
        act_max = torch.zeros(n_l + 1, device=dev, dtype=torch.int32)   # + max |z_feature|
        zs = dims.d_in + (-dims.d_in) % 4                                # z_feature rows padded to 16 B
        zf = torch.empty(Mt, zs, device=dev, dtype=F32)
        p = xyz.detach().to(F32).contiguous()
        v = viewdirs.reshape(SB, B, 3).detach().to(F32).contiguous()
        require_device(p, v)
        tables = fused.tables_batch(coarse, SB, fast=True, entry=entry)
        masks = []
        for g0 in range(0, SB, _lib.AVR_MAX_SCENES):     # one launch per group of scenes
            n = min(_lib.AVR_MAX_SCENES, SB - g0)
            act_n, mask_n = ctypes.c_int64(0), ctypes.c_int64(0)
            _lib.check(_lib.load().avr_field_train_sizes(ctypes.byref(dims), n, B, ctypes.byref(act_n),
                                                         ctypes.byref(mask_n)), "avr_field_train_sizes")
            views = fused.views(range(g0, g0 + n))
            mask = torch.empty(max(mask_n.value, 1), device=dev, dtype=torch.int32)
            call("avr_field_fwd_points_train", ctypes.byref(dims), views, n, ptr(entry.packed), ptr(tables[g0]),
                 ptr(p[g0]), ptr(v[g0]), B, ptr(out[g0]), ctypes.c_void_p(act.data_ptr() + g0 * B * H * 4), Mt,
                 ptr(mask), ptr(act_max), ctypes.c_void_p(zf.data_ptr() + g0 * B * zs * 4), zs,
                 ctypes.c_void_p(act_max.data_ptr() + 4 * n_l), stream_of(p))
            masks.append((g0, n, mask))
        entry.dims.precision = PRECISIONS[fused.precision]
        ctx.fused, ctx.coarse, ctx.names, ctx.entry = fused, coarse, names, entry
        ctx.act, ctx.act_max, ctx.masks, ctx.zf = act, act_max, masks, zf
        ctx.tables = tables
        ctx.save_for_backward(xyz, viewdirs, latent, out, *params)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from .ops import latent_features, lin_out_act_bwd, weight_grads_specs
        xyz, viewdirs, latent, out, *params = ctx.saved_tensors
        fused, entry, names = ctx.fused, ctx.entry, ctx.names
        net = fused.net
        P = dict(zip(names, params))
        dims = entry.dims
        H, nb, nz = dims.d_hidden, dims.n_blocks, dims.n_lin_z
        SB, B, _ = xyz.shape
        n_l, Mt = 2 * nb + 1, SB * B
        want_latent = ctx.needs_input_grad[5] and not net.stop_encoder_grad
        if B == 0:
            zeros = tuple(torch.zeros_like(p) if ctx.needs_input_grad[6 + i] else None for i, p in enumerate(params))
            return (None, None, None, torch.zeros_like(xyz) if ctx.needs_input_grad[3] else None, None,
                    torch.zeros_like(latent) if want_latent else None) + zeros
        dev = xyz.device
        dims.precision = _lib.FIELD_X3
        bwd = fused.packed_bwd(ctx.coarse, entry)
        grad_out = grad_out.to(F32).contiguous()
        G = torch.empty(n_l, Mt, H, device=dev, dtype=F32)
        g_max = torch.zeros(n_l, device=dev, dtype=torch.int32)
        act = ctx.act
        for g0, n, mask in ctx.masks:
            call("avr_field_bwd", ctypes.byref(dims), ptr(entry.packed), ptr(bwd), n, B, ptr(out[g0]),
                 ptr(grad_out[g0]), ptr(mask), ctypes.c_void_p(act.data_ptr() + g0 * B * H * 4), Mt,
                 ctypes.c_void_p(G.data_ptr() + g0 * B * H * 4), Mt, ptr(g_max), stream_of(G))
        entry.dims.precision = PRECISIONS[fused.precision]
        act_max, zf = ctx.act_max, ctx.zf
        ctx.act = ctx.act_max = ctx.masks = ctx.zf = None
        # MLP inputs the lin_z / lin_in gradients contract against: the latent
        # features (avr_latent_features, row-major) and z_feature (the training forward
        # stored it, padded to 16 B, with its max in act_max[n_l])
        d_in = dims.d_in
        p = xyz.detach().to(F32).contiguous()
        with torch.no_grad():
            lat_feat = torch.empty(Mt, net.d_latent, device=dev, dtype=F32)
            if SB <= latent.shape[0]:   # every scene its own map: one launch per AVR_MAX_SCENES scenes
                hwc = fused.latent_hwc_all(latent)
                for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
                    n = min(_lib.AVR_MAX_SCENES, SB - g0)
                    views = fused.views(range(g0, g0 + n))
                    call("avr_latent_features_batch", views, n, ptr(hwc[g0]), net.d_latent, ptr(p[g0]), B,
                         ptr(lat_feat[g0 * B]), stream_of(lat_feat))
            else:
                for sb in range(SB):
                    s = min(sb, latent.shape[0] - 1)
                    latent_features(fused.view(sb), latent[s], xyz[sb], out=lat_feat[sb * B:(sb + 1) * B],
                                    hwc=fused.latent_hwc(latent, s))
        lat_max = fused.latent_max_bits(latent)   # |interpolated latent| <= max |latent| (convex blend)
        zf_max = act_max[n_l:n_l + 1]
        Gz = [G[2 * b - 1] if b > 0 else G[2 * nb] for b in range(nz)]
        # lin_out (4 outputs): d out through sigmoid / relu (torch: g * (1 - y) * y, g * (y > 0)), with its max
        d4, d4_max = lin_out_act_bwd(grad_out, out)
        # the layers of the batched weight-gradient launch addressed by offset into the buffers this Function
        # allocated (row strides H, d_latent, zs, 4; 16-B aligned by construction): the fc layers (G_k, act_k),
        # lin_z[b] (the gradient at block b's input, the interpolated latent), lin_in (the gradient at the first
        # block's input, z_feature), lin_out (d4, the last block's output) -- no per-layer views or checks
        Gp, Ap, gmp, amp, lay = G.data_ptr(), act.data_ptr(), g_max.data_ptr(), act_max.data_ptr(), Mt * H * 4
        specs = [(Gp + k * lay, H, Ap + k * lay, H, H, H, gmp + 4 * k, amp + 4 * k, True, None, None, None, 0)
                 for k in range(2 * nb)]
        for b in range(nz):
            k = 2 * b - 1 if b > 0 else 2 * nb
            specs.append((Gp + k * lay, H, lat_feat.data_ptr(), net.d_latent, H, net.d_latent, gmp + 4 * k,
                          lat_max.data_ptr(), False, None, None, None, 0))
        specs.append((Gp + 2 * nb * lay, H, zf.data_ptr(), zf.shape[1], H, zf.shape[1], gmp + 8 * nb,
                      zf_max.data_ptr(), True, None, None, None, 0))
        specs.append((d4.data_ptr(), 4, Ap + 2 * nb * lay, H, 4, H, d4_max.data_ptr(), amp + 8 * nb, True, None, None,
                      None, 0))
        res = weight_grads_specs(specs, Mt, dev, stream_of(G))
        grads = {"lin_out.weight": res[-1][0], "lin_out.bias": res[-1][1]}
        res = res[:-1]
        for b in range(nb):
            grads[f"blocks.{b}.fc_0.weight"], grads[f"blocks.{b}.fc_0.bias"] = res[2 * b]
            grads[f"blocks.{b}.fc_1.weight"], grads[f"blocks.{b}.fc_1.bias"] = res[2 * b + 1]
        for b in range(nz):
            grads[f"lin_z.{b}.weight"] = res[2 * nb + b][0]
            # lin_z[b]'s output gradient is the gradient at block b's input
            grads[f"lin_z.{b}.bias"] = res[2 * b - 1][1] if b > 0 else res[-1][1]
        w_in, b_in = res[-1]
        grads["lin_in.weight"], grads["lin_in.bias"] = w_in[:, :d_in].contiguous(), b_in
        # the gradient at the MLP inputs, sent through the (cheap) torch input
        # functions: the latent map via the grid_sample adjoint, the points via
        # PE / rotation / projection (the adaptive renderer's band points)
        d_latent = d_xyz = None
        want_xyz = ctx.needs_input_grad[3]
        if want_xyz and not want_latent and (net.stop_encoder_grad or (nz > 0 and SB <= latent.shape[0])):
            # the points alone (the adaptive renderer's band, fixed latent): the lookup's adjoint on HIP
            # (avr_latent_tables_grad_points / avr_latent_features_grad_points), then z_feature's. With
            # stop_encoder_grad the looked-up latent is detached (models.py:810-811), so no gradient reaches the
            # points through the lookup: z_feature's part alone.
            d_look = None
            if not net.stop_encoder_grad:
                with torch.no_grad():
                    d_look = torch.empty(Mt, 3, device=dev, dtype=F32)
                    tabs = ctx.tables
                    via_tables = (not dims.spade and nz <= _lib.AVR_LOOKUP_GRAD_TERMS and tabs.shape[0] == SB
                                  and os.environ.get("AVR_POINT_GRAD_VIA_FEATURES") != "1")
                    if via_tables:
                        # sum_b Gz[b] . lin_z[b](interp(latent, p)) = sum_b Gz[b] . interp(table_b, p): the corner
                        # differences of the forward's per-texel tables against each Gz row (ABI 15), no
                        # d_hidden x d_latent product per point for the feature gradient
                        ld = Gz[0].stride(0)
                        assert all(g.stride(0) == ld and g.stride(1) == 1 for g in Gz)
                        gptr = [g.data_ptr() for g in Gz]
                        for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
                            n = min(_lib.AVR_MAX_SCENES, SB - g0)
                            views = fused.views(range(g0, g0 + n))
                            gr = (ctypes.c_void_p * nz)(*[g + g0 * B * ld * 4 for g in gptr])
                            call("avr_latent_tables_grad_points", views, n, ptr(tabs[g0]), tabs.stride(0),
                                 tabs.stride(1), nz, H, ptr(p[g0]), B, gr, ld, ptr(d_look[g0 * B]),
                                 stream_of(d_look))
                    else:
                        g_feat = _feat_grad(fused, entry, bwd, Gz, P, Mt)
                        hwc = fused.latent_hwc_all(latent)
                        for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
                            n = min(_lib.AVR_MAX_SCENES, SB - g0)
                            views = fused.views(range(g0, g0 + n))
                            call("avr_latent_features_grad_points", views, n, ptr(hwc[g0]), net.d_latent,
                                 ptr(p[g0]), B, ptr(g_feat[g0 * B]), ptr(d_look[g0 * B]), stream_of(d_look))
            # z_feature's part (ABI 16): d loss / d z_feature = G_in W_in (its positional-encoded columns only), then
            # the encoding's and the rotation's adjoint per point in one launch, added to the lookup's part
            # (AVR_POINT_ZF_VIA_AUTOGRAD=1: torch autograd of z_features instead, the round-5 path, for A/B)
            n_pe = 3 + 6 * dims.num_freqs
            if os.environ.get("AVR_POINT_ZF_VIA_AUTOGRAD") == "1":
                with torch.enable_grad():
                    x = xyz.detach().requires_grad_(True)
                    zft = net.z_features(x, viewdirs.detach())
                    d_z, = torch.autograd.grad(zft, x, G[2 * nb] @ P["lin_in.weight"].detach())
                d_xyz = (d_z if d_look is None else d_look.reshape(SB, B, 3) + d_z).to(xyz.dtype)
            else:
                with torch.no_grad():
                    d_zf = G[2 * nb] @ P["lin_in.weight"].detach()[:, :n_pe]
                    if d_look is None:
                        d_look = torch.empty(Mt, 3, device=dev, dtype=F32)
                    for g0 in range(0, SB, _lib.AVR_MAX_SCENES):
                        n = min(_lib.AVR_MAX_SCENES, SB - g0)
                        views = fused.views(range(g0, g0 + n))
                        call("avr_zfeature_grad_points", views, n, ptr(p[g0]), B, ptr(d_zf[g0 * B]), d_zf.stride(0),
                             dims.num_freqs, dims.freq_factor, int(not net.stop_encoder_grad), ptr(d_look[g0 * B]),
                             stream_of(d_look))
                d_xyz = d_look.reshape(SB, B, 3).to(xyz.dtype)
        elif want_latent or want_xyz:
            with torch.enable_grad():
                lat = latent.detach().requires_grad_(want_latent)
                x = xyz.detach().requires_grad_(want_xyz)
                feat, zft = net.mlp_inputs(x, viewdirs.detach(), latent=lat)
                outs, grads_out = [], []
                if nz > 0:
                    outs.append(feat)
                    grads_out.append(_feat_grad(fused, entry, bwd, Gz, P, Mt))
                if want_xyz:
                    outs.append(zft)
                    grads_out.append(G[2 * nb] @ P["lin_in.weight"].detach())
                wrt = ([lat] if want_latent else []) + ([x] if want_xyz else [])
                res_in = torch.autograd.grad(outs, wrt, grads_out, allow_unused=True)
            if want_latent:
                d_latent = res_in[0] if res_in[0] is not None else torch.zeros_like(latent)
            if want_xyz:
                d_xyz = res_in[-1] if res_in[-1] is not None else torch.zeros_like(xyz)
        return (None, None, None, d_xyz, None, d_latent) + tuple(
            grads[n] if ctx.needs_input_grad[6 + i] else None for i, n in enumerate(names))
