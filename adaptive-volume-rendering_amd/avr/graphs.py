"""HIP-graph replay of the inference renderer for fixed shapes (serving).

`VolumeRenderer.forward` on the fused path is a fixed chain of launches (rays + stratified z, coarse field,
composite, inverse-CDF sampling + merge, fine field, composite + depth) whose host side -- argument packing,
ctypes calls, tensor allocation -- costs tens of microseconds per launch. For small ray batches that host time
is a large part of a frame. `GraphedRenderer` captures the chain once into a HIP graph (torch.cuda.CUDAGraph,
hipGraph on ROCm) and replays it: new cameras / pixels are copied into the captured input buffers, the outputs
are the captured output buffers.

Noise: with `renderer.seed = None` the reference's draws (torch.rand / randn, renderers.py:14, :41, :45, :63)
are captured too and advance on every replay like eager calls. With an integer seed the in-kernel Philox draws
are keyed by the offset the renderer held at capture time, so every replay draws the same noise (eager calls
advance the offset per call).

State: the captured launches read the packed weights, lin_z tables and source-view descriptors the renderer
built from the net at capture time. Every call checks the tensors those come from for an in-place update (the
MLPs' parameters and buffers: an optimizer step, load_state_dict) or a new tensor (the encoder's latent, the
source poses / focal / principal point: net.encode() of new images) and captures the chain again when one
changed, so a replay never renders with stale weights or views (a few microseconds per call). A change of
net.field_precision captures again too. The packed weights and lin_z tables the captured launches read are
referenced by the GraphedRenderer, so an eager call that replaces those cache entries (another scene count or
precision) cannot free memory a replay reads. Replacing a Parameter object itself is not seen: call refresh()
after that. Warm-ups and re-captures leave the renderer's Philox offset where it was.
"""
import torch

from . import anomaly

__all__ = ["GraphedRenderer"]


class GraphedRenderer:
    """renderer(cam2world, intrinsics, x_pix, net) captured for the shapes of the example inputs.

    __call__(cam2world, intrinsics, x_pix) -> (rgb_coarse, rgb_fine, depth, depth), the captured buffers
    (overwritten by the next replay; clone to keep). Inference only (no autograd), fused field only.
    """

    def __init__(self, renderer, net, cam2world, intrinsics, x_pix, warmup=2):
        if renderer.t_stop is not None:
            raise ValueError("GraphedRenderer: early termination sizes its launches on the host (t_stop must be None)")
        self.renderer, self.net = renderer, net
        self.warmup = warmup
        self.c2w = cam2world.detach().clone().contiguous()
        self.K = intrinsics.detach().clone().contiguous()
        self.x_pix = x_pix.detach().clone().contiguous()
        self.captures = 0
        self._capture()

    def _params(self):
        """The MLPs' parameters and buffers: updated in place (optimizer steps, load_state_dict), so their
        versions are compared; the Parameter objects are collected once per capture."""
        ts = []
        for mlp in (getattr(self.net, "mlp_coarse", None), getattr(self.net, "mlp_fine", None)):
            if mlp is not None:
                ts += list(mlp.parameters()) + list(mlp.buffers())
        return ts

    def _views(self):
        """The source-view state net.encode() replaces: latent, latent scaling, poses, focal, principal point."""
        enc = getattr(self.net, "encoder", None)
        return [getattr(enc, "latent", None), getattr(enc, "latent_scaling", None)] + \
               [getattr(self.net, a, None) for a in ("poses", "focal", "c", "image_shape")]

    def _stale(self):
        # held references: no address is reused while compared
        return any(t._version != v for t, v in self._held) or \
            any(a is not b for a, b in zip(self._views(), self._held_views)) or \
            getattr(self.net, "field_precision", None) != self._held_precision

    def refresh(self):
        """Capture again (after replacing a Parameter object of the net, which the per-call check does not see)."""
        self._capture()

    def _capture(self):
        renderer, net = self.renderer, self.net
        warmup = self.warmup
        self.graph = self.out = None
        offset0 = renderer._offset    # warm-ups and re-captures leave the eager calls' Philox offset as it was
        stream = torch.cuda.Stream(device=self.x_pix.device)
        stream.wait_stream(torch.cuda.current_stream())
        with torch.no_grad(), torch.cuda.stream(stream):
            # warm-up outside the capture: packs the weights, builds the lin_z tables, caches the views, sets the
            # kernels' LDS attributes -- everything that touches the host or allocates outside the graph pool
            for _ in range(warmup):
                renderer(self.c2w, self.K, self.x_pix, net)
            if renderer.last_path != "fused":
                raise ValueError("GraphedRenderer: the net must take the fused field path (net.can_fuse)")
        torch.cuda.current_stream().wait_stream(stream)
        renderer._offset = self.offset = offset0
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = renderer(self.c2w, self.K, self.x_pix, net)
        renderer._offset = offset0   # the captured launches keep the offset they were recorded with
        # the packed weights, lin_z tables and batched tables the captured kernels read: referenced here, so an
        # eager call that replaces a cache entry (another scene count, another precision) cannot free them
        fused = getattr(net, "_fused", None)
        self._held_buffers = fused.cache_tensors() if fused is not None else []
        self._held_precision = getattr(net, "field_precision", None)
        views = self._views()
        self._held_views = views
        self._held = [(t, t._version) for t in self._params() + views if isinstance(t, torch.Tensor)]
        self.captures += 1

    def __call__(self, cam2world=None, intrinsics=None, x_pix=None):
        if cam2world is not None:
            self.c2w.copy_(cam2world)
        if intrinsics is not None:
            self.K.copy_(intrinsics)
        if x_pix is not None:
            self.x_pix.copy_(x_pix)
        if self._stale():
            self._capture()
        self.graph.replay()
        if anomaly.is_enabled():   # the captured launches were not checked at capture time (avr/anomaly.py)
            anomaly.check_outputs("GraphedRenderer replay", self.out)
        return self.out
