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
from .field import bump_param_generation, param_generation

__all__ = ["GraphedRenderer", "GraphedTrainStep"]


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
            getattr(self.net, "field_precision", None) != self._held_precision or \
            param_generation() != self._held_gen   # an optimizer step (fused ones leave versions alone)

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
        self._held_gen = param_generation()
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


class GraphedTrainStep:
    """One training step -- the renderer and net forward, the loss, loss.backward() and optimizer.step()
    (train.py:108-114) -- captured into one HIP graph for fixed shapes and replayed, for training loops whose step
    is bound by launch overhead (the AdaptiveVolumeRenderer step: ~190 launches of a few to a few hundred
    microseconds each).

    step_fn() runs one step on tensors the caller keeps at fixed addresses (refill them in place between calls)
    and returns what the caller reads after the step (e.g. the loss); it may call optimizer.zero_grad() (the
    default set_to_none: a host-only no-op once captured: the captured backward writes the gradients). The
    optimizer must be capturable: torch.optim.Adam(..., capturable=True, fused=True) (the fused form is one
    multi-tensor kernel; the capturable foreach form adds many small launches).

    Calls 1 .. warmup run step_fn eagerly (real steps, on a side stream, so the graph's memory pool starts clean);
    the next call captures it (the capture records launches without running them) and replays it once; later
    calls replay. Every call is one training step. The outputs returned are detached; drop any reference to an
    earlier step's autograd graph (a loss kept from an eager step) before the first call: it would keep the
    parameters' AccumulateGrad nodes, created on the streams of that step, alive into the capture.

    Host-side inputs: each marcher in `renderers` (Raymarcher / AdaptiveVolumeRenderer) draws its start distances
    on the CPU generator in an eager step (renderers.py:322 / :402); before every replay stage_host_draws() makes
    the same draw and copies it into the buffer the captured march reads, so the random stream matches eager steps.
    The band's torch.rand draws advance on device per replay as eager calls would (PyTorch's graph-safe generator).

    State: the captured kernels take the source-view descriptors (poses, focal, principal point, latent map
    shape) as launch arguments, and read the latent map through its address: like GraphedRenderer, every call
    checks the nets' view tensors (a new latent or pose tensor, or an in-place update of one) and the field
    precision; when one changed, that call runs eagerly (rebuilding the view descriptors on the host, which a
    capture cannot) and the next one captures again. Parameters are updated by the captured optimizer step
    itself. The nets' FusedField blob and table caches are dropped before a capture, so every blob and lin_z
    table the step reads is rebuilt inside the graph from the current parameters.
    """

    @staticmethod
    def _detach(out):
        """The caller's view of a step's outputs, without the autograd graph (kept alive it would hold the
        parameters' AccumulateGrad nodes, and their streams, into the next step)."""
        if isinstance(out, torch.Tensor):
            return out.detach()
        if isinstance(out, (list, tuple)):
            return type(out)(GraphedTrainStep._detach(o) for o in out)
        if isinstance(out, dict):
            return {k: GraphedTrainStep._detach(v) for k, v in out.items()}
        return out

    def __init__(self, step_fn, nets=(), renderers=(), warmup=3):
        self.step_fn = step_fn
        self.nets = [n for n in nets if n is not None]
        self.renderers = [r for r in renderers if r is not None]
        self.warmup = warmup
        self.calls = 0
        self.captures = 0
        self.graph = None
        self.out = None

    def _views(self):
        out = []
        for net in self.nets:
            enc = getattr(net, "encoder", None)
            out += [getattr(enc, "latent", None), getattr(enc, "latent_scaling", None)]
            out += [getattr(net, a, None) for a in ("poses", "focal", "c", "image_shape")]
        return [t for t in out if isinstance(t, torch.Tensor)]

    def _stale(self):
        views = self._views()
        return (len(views) != len(self._held) or any(a is not b or a._version != v
                                                       for a, (b, v) in zip(views, self._held))
                or [getattr(n, "field_precision", None) for n in self.nets] != self._held_precision)

    def _capture(self):
        self.graph = self.out = None
        for net in self.nets:
            fused = getattr(net, "_fused", None)
            if fused is not None:
                fused.invalidate(views=False)   # every blob / table the step reads is made inside the graph
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self.step_fn()
        self.graph, self.out = graph, self._detach(out)
        self._held = [(t, t._version) for t in self._views()]
        self._held_precision = [getattr(n, "field_precision", None) for n in self.nets]
        self.captures += 1

    def __call__(self):
        self.calls += 1
        if self.graph is not None and self._stale():
            # new views: this step runs eagerly (it rebuilds the host-side view descriptors, which a capture
            # cannot), the next one captures again
            self.graph = self.out = None
            self._eager_until = self.calls
        if self.calls <= max(self.warmup, getattr(self, "_eager_until", 0)):
            stream = torch.cuda.Stream()
            stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(stream):
                out = self._detach(self.step_fn())
            torch.cuda.current_stream().wait_stream(stream)
            return out
        if self.graph is None:
            self._capture()
        for r in self.renderers:
            r.stage_host_draws()
        self.graph.replay()
        bump_param_generation()   # the replayed optimizer step ran no host hook: eager calls must repack
        if anomaly.is_enabled():
            anomaly.check_outputs("GraphedTrainStep replay", self.out)
        return self.out
