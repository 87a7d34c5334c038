#!/usr/bin/env python
"""Benchmark: rays/s of the coarse/fine VolumeRenderer hot path on MI355X.

Workload (BASELINE.json configs[2], the metric's config): 65 536 rays per GPU
x (128 coarse + 64 importance samples, n_fine_depth = 0), one scene, the
conf/default.conf PixelNeRF field (PE(6) + ResnetFC 3 x 512 with lin_z on all
blocks, d_latent 512) with random-init weights and a random 512x64x64 latent
map (synthetic: no dataset or checkpoint is available offline).

One step = VolumeRenderer.forward over the batch: ray generation, stratified
sampling, coarse field, compositing, inverse-CDF sampling + merge, fine field,
compositing, depth -- plus, on N > 1 GPUs, the RCCL gather of every rank's
(rgb_coarse, rgb_fine, depth) to rank 0. The per-scene preparation (weight
repack and lin_z latent table) is redone inside every step, not cached.

python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3|4|5]; N > 1 via torch.distributed.run.
--config 5 (BASELINE configs[4]): a fixed 4 x 800 x 800 rays per step for the whole job, dealt to the ranks in
64-ray tiles by avr.parallel.render_sharded and gathered with one all_gather ("scaling": "strong").
Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

dist = None   # torch.distributed, imported when the job has more than one rank

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA (= fp32 vector), MI355X_MICROARCH.md
FP16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 MFMA
HBM_PEAK_GBS = 8000.0


def field_flops_per_sample(d_in=42, d_hidden=512, n_blocks=3, n_lin_z=3, d_out=4):
    """Algorithmic FLOPs of the fused field per sample (this design: lin_z is
    applied per texel, so per sample it is a 4-tap bilinear blend)."""
    macs = d_in * d_hidden + n_blocks * 2 * d_hidden * d_hidden + d_hidden * d_out
    return 2 * macs + n_lin_z * d_hidden * 8


def reference_flops_per_sample(d_in=42, d_latent=512, d_hidden=512, n_blocks=3, n_lin_z=3, d_out=4):
    """FLOPs the reference's unfactored ResnetFC spends per sample (4.766 M)."""
    return 2 * (d_in * d_hidden + n_lin_z * d_latent * d_hidden + n_blocks * 2 * d_hidden * d_hidden
                + d_hidden * d_out)


def build_scene(device, seed=0, sigma_bias=0.0, conf="default", bn=False, spade=False):
    """avr.scene.synthetic_scene: the default.conf field (or default_mv.conf's: 5 blocks, combine_layer 3)
    with fc_1 ~ N(0, 0.02), random 512x64x64 latent. spade: ResnetFC(use_spade=True) in both MLPs."""
    from avr.conf import default_conf
    from avr.scene import synthetic_scene
    model = default_conf(multiview=conf == "default_mv")["model"]
    if spade:
        model["mlp_coarse"] = dict(model["mlp_coarse"], use_spade=True)
        model["mlp_fine"] = dict(model["mlp_fine"], use_spade=True)
    return synthetic_scene(device, seed, model, sigma_bias=sigma_bias, bn=bn)


def orbit_c2w(angle, radius=1.3, z_height=0.4):
    """generate_video's orbit pose (utils.py:497-513)."""
    rr = np.sqrt(radius * radius - z_height * z_height)
    t = np.array([rr * np.sin(angle), rr * np.cos(angle), z_height])
    zax = -t / np.linalg.norm(t)
    xax = np.cross([0.0, 0.0, -1.0], zax)
    xax /= np.linalg.norm(xax)
    yax = np.cross(zax, xax)
    c2w = np.eye(4)
    c2w[:3, :3] = np.stack([xax, yax, zax], 1)
    c2w[:3, 3] = t
    return torch.from_numpy((c2w @ np.diag([1.0, -1.0, -1.0, 1.0])).astype(np.float32))


class FieldTimer:
    """HIP events around every field launch, recorded on the launch stream."""

    def __init__(self):
        self.events = []
        self.samples = 0

    def wrap(self, fused):
        orig = fused.forward_rays

        def timed(ro, rd, z, coarse, sb=0):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            fused.packed(coarse)
            fused.table(coarse, sb)
            s.record()
            out = orig(ro, rd, z, coarse, sb)
            e.record()
            self.events.append((s, e))
            self.samples += z.numel()
            return out

        fused.forward_rays = timed

    def reset(self):
        self.events, self.samples = [], 0

    def total_ms(self):
        return sum(s.elapsed_time(e) for s, e in self.events)


class HbmKernelTimer:
    """The renderer's HBM-bound launches (avr.ops wrappers; each enqueues one
    kernel on torch's current stream), measured in isolation: the arguments of
    their first call inside the timed steps are kept and every launch is then
    replayed `reps` times back to back between two HIP events, so the average
    is kernel time without host launch gaps (one HIP graph of `reps` launches).
    Bytes are ALGORITHMIC per launch
    (SURVEY §8d): compulsory reads + writes, fp32, Philox noise (no noise bytes)."""

    def __init__(self, ops):
        self.ops = ops
        self.calls = {}    # label -> (fn, args, kwargs, bytes)
        self.on = False

    def _wrap(self, name, kernel, nbytes):
        orig = getattr(self.ops, name)

        def timed(*a, **k):
            out = orig(*a, **k)
            if self.on:
                nb, nw, what = nbytes(a, k, out)
                label = f"{kernel} ({what})" if what else kernel
                self.calls.setdefault(label, (orig, a, k, (nb, nw)))
            return out

        setattr(self.ops, name, timed)

    def install(self):
        # each returns (bytes, of which written, label)
        def composite_bytes(a, k, out):
            R, N = a[0].shape
            ww = out[2] is not None
            return (R * (N * (4 + 16 + (4 if ww else 0)) + 16), R * ((4 * N if ww else 0) + 16),
                    f"N={N}, weights {'stored' if ww else 'not stored'}")

        def sample_fine_bytes(a, k, out):
            w, zc = a[0], a[1]
            nw = out[0].numel() * 4
            return w.numel() * 4 + zc.numel() * 4 + nw, nw, f"Nc={zc.shape[1]}, out {out[0].shape[1]}"

        def rays_coarse_bytes(a, k, out):
            R, N = out[2].shape
            nw = R * (24 + 4 * N + (32 if out[3] is not None else 0))
            return R * 8 + nw, nw, f"N={N}, depth rows"

        def composite_depth_bytes(a, k, out):
            R, N = a[0].shape
            return R * (N * (4 + 16) + 16 + 24 + 32 + 4), R * 20, f"N={N}, + depth"

        def per_point(read, write):
            return lambda a, k, out: (a[0].shape[0] * a[0].shape[1] * (read + write),
                                      a[0].shape[0] * a[0].shape[1] * write, "")

        self._wrap("rays_sample_coarse", "rays_coarse_kernel", rays_coarse_bytes)
        self._wrap("composite_depth", "composite_fwd_kernel", composite_depth_bytes)
        self._wrap("world_rays", "world_rays_kernel", per_point(8, 24))
        self._wrap("sample_coarse", "sample_coarse_kernel",
                   lambda a, k, out: (out.numel() * 4, out.numel() * 4, f"N={out.shape[1]}"))
        self._wrap("composite_fwd", "composite_fwd_kernel", composite_bytes)
        self._wrap("sample_fine", "sample_fine_kernel", sample_fine_bytes)
        self._wrap("depth_from_world_fwd", "depth_kernel", per_point(28, 4))

    @staticmethod
    def _input_sets(a, k, min_bytes, max_sets):
        """Copies of one launch's device inputs, enough sets that they span
        min_bytes together (more than the 256 MB Infinity Cache, so replayed
        launches read HBM, not MALL hits). Stride-0 views (a broadcast pose)
        are shared, not materialised."""
        def tensors(x):
            return [t for t in x if isinstance(t, torch.Tensor) and t.is_cuda]
        nb = sum(t.numel() * t.element_size() for t in tensors(list(a) + list(k.values())))
        n = max(1, min(max_sets, -(-min_bytes // max(nb, 1))))

        def clone(x):
            if isinstance(x, torch.Tensor) and x.is_cuda and 0 not in x.stride():
                return x.clone()
            return x
        sets = [(a, k)] + [(tuple(clone(x) for x in a), {kk: clone(v) for kk, v in k.items()}) for _ in range(n - 1)]
        return sets, nb

    @classmethod
    def _replay_us(cls, fn, a, k, reps, min_bytes):
        """Average launch duration: `reps` launches captured in one HIP graph
        (no host launch gaps between them) cycling over input copies that span
        min_bytes, every launch writing outputs of its own (kept alive during
        the capture); plain back-to-back launches if capture is refused."""
        sets, in_b = cls._input_sets(a, k, min_bytes, reps)
        n_sets = len(sets)
        keep = []

        def launch(i):
            aa, kk = sets[i % len(sets)]
            keep.append(fn(*aa, **kk))

        for i in range(len(sets)):
            launch(i)
        torch.cuda.synchronize()
        keep.clear()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        try:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    for i in range(reps):
                        launch(i)
            torch.cuda.current_stream().wait_stream(side)
            g.replay()
            torch.cuda.synchronize()
            s.record()
            g.replay()
            e.record()
        except Exception:  # noqa: BLE001 -- capture refused: time plain launches
            keep.clear()
            torch.cuda.synchronize()
            s.record()
            for i in range(reps):
                launch(i)
            e.record()
        e.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        keep.clear()
        del sets
        torch.cuda.empty_cache()
        return us, n_sets, in_b

    def report(self, reps=20, achievable=None, min_bytes=1 << 30):
        """achievable: (copy GB/s, fill GB/s) on this box. A kernel's achievable time is its read bytes at
        the copy's read rate plus its written bytes at the fill's write rate (the copy's time split by the
        fill's: a copy of N bytes takes N/read + N/write), frac_of_achievable = that time / measured."""
        res = []
        for label, (fn, a, k, (nb, nw)) in self.calls.items():
            us, n_sets, in_b = self._replay_us(fn, a, k, reps, min_bytes)
            gbs = nb / (us * 1e-6) / 1e9
            res.append({"kernel": label, "avg_us": round(us, 2), "bytes_per_launch": int(nb),
                        "written_bytes_per_launch": int(nw),
                        "achieved_GBs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
                        "input_sets": n_sets, "input_bytes_rotated": int(n_sets * in_b)})
            if achievable:
                copy_gbs, fill_gbs = achievable
                sec_per_read_byte = max(2.0 / copy_gbs - 1.0 / fill_gbs, 1.0 / HBM_PEAK_GBS) / 1e9
                floor_us = ((nb - nw) * sec_per_read_byte + nw / fill_gbs / 1e9) * 1e6
                res[-1]["achievable_us"] = round(floor_us, 2)
                res[-1]["frac_of_achievable"] = round(floor_us / us, 4)
        return res


def achievable_hbm_gbs(device, nbytes=1 << 31, reps=5):
    """the HBM bandwidth streaming kernels reach on this box, over
    2 GiB buffers (8x the Infinity Cache), best of `reps` launches timed one by
    one with HIP events: avr_stream_copy (16 B per lane, 4 loads in flight per
    lane; the kind of float4 copy MI355X_MICROARCH.md measures at 6.29 TB/s),
    read + write bytes / time, and avr_stream_fill (the same stores, no loads),
    written bytes / time -- the ceiling of store-dominated kernels.
    Returns (copy GB/s, fill GB/s)."""
    import avr
    src = torch.empty(nbytes // 4, device=device, dtype=torch.float32).fill_(1.0)
    dst = torch.empty_like(src)

    def best_ms(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e)
            best = ms if best is None else min(best, ms)
        return best

    copy_ms = best_ms(lambda: avr.ops.stream_copy(src, dst))
    assert bool((dst[:: 1 << 20] == 1.0).all())
    fill_ms = best_ms(lambda: avr.ops.stream_fill(dst, 0x40000000))   # 2.0f
    assert bool((dst[:: 1 << 20] == 2.0).all())
    del src, dst
    torch.cuda.empty_cache()
    return 2 * nbytes / (copy_ms * 1e-3) / 1e9, nbytes / (fill_ms * 1e-3) / 1e9


def cpu_share():
    """CPU threads this process may use on the host: the affinity mask, the
    cgroup CPU quota and OMP_NUM_THREADS (the GPU box pins these to the box's
    share of the host), plus the host's physical core count for the record."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    cores, model = set(), ""
    try:
        phys = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and not model:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                cores.add((phys, v))
    except OSError:
        pass
    return n, len(cores) or None, model


def _median_rate(fn, units, runs=3):
    """1 untimed warm-up call, then the median rate of `runs` timed calls."""
    fn(warm=True)
    rates = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        rates.append(units / (time.perf_counter() - t0))
    return float(np.median(rates)), rates


def cpu_baseline(c3_rays=384, c1_rays=4096):
    """The reference's CPU path on this host's cores, SURVEY §8d protocol:
    every thread this process may use, 1 warm-up, median of 3. Two ports are
    timed and the faster one is the baseline (which one wins depends on the
    host's BLAS / oneDNN): oracle/torch_port.py (the reference's own torch
    operators: per-sample lin_z, grid_sample, searchsorted, cumprod) and the
    numpy oracle (oracle/avr_oracle.py, row-layout latent gathers).
      * C3 sample: c3_rays rays of the 128 + 64 configuration (same field
        architecture, random-init weights, 512x64x64 latent) per run;
      * C1 (BASELINE configs[0], the reference's own CPU case: 64 coarse
        samples, coarse pass only): c1_rays of its 4096 rays per run, torch port."""
    sys.path.insert(0, REPO)
    from threadpoolctl import threadpool_limits
    from oracle import avr_oracle as O
    from oracle import synth
    from oracle import torch_port as TP
    threads, physical, model = cpu_share()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    pc = synth.resnetfc_params(42, 512, 512, 3, 1000, 40)
    pf = synth.resnetfc_params(42, 512, 512, 3, 1000, 57)
    poses, focal, c, image_shape, latent_scaling = synth.source_view((64, 64))
    latent = synth.hashed_normalish((1, 512, 64, 64), 45, 1.0)
    tfield = TP.TorchField(pc, pf, latent, poses, focal, c, image_shape, latent_scaling)
    nfield = O.PixelNeRFField(pc, pf, latent, poses, focal, c, image_shape, latent_scaling)
    gen = torch.Generator().manual_seed(0)
    rng = np.random.default_rng(0)
    K = synth.default_intrinsics()[None].astype(np.float32)
    c2w1 = synth.orbit_cam2world(0.7).astype(np.float32)
    Kt, c2wt = torch.from_numpy(K), torch.from_numpy(c2w1).reshape(1, 1, 4, 4)

    def c3_torch(warm=False, chunk=128):
        for _ in range(1 if warm else c3_rays // chunk):
            TP.render(c2wt.expand(1, chunk, 4, 4), Kt, torch.rand(1, chunk, 2, generator=gen), tfield, 0.8, 1.8, 128,
                      64, True, gen)

    def c3_numpy(warm=False, chunk=128):
        for _ in range(1 if warm else c3_rays // chunk):
            noise = [rng.random((1, chunk, n), dtype=np.float32) for n in (128, 64, 64)]
            O.render(np.broadcast_to(c2w1, (1, chunk, 4, 4)), K, rng.random((1, chunk, 2), dtype=np.float32),
                     nfield, 0.8, 1.8, 128, 64, 0, 0.01, True, noise[0], noise[1], noise[2],
                     np.zeros((1, chunk, 0), np.float32))

    def c1_torch(warm=False, chunk=512):
        for _ in range(1 if warm else c1_rays // chunk):
            TP.render(c2wt.expand(1, chunk, 4, 4), Kt, torch.rand(1, chunk, 2, generator=gen), tfield, 0.8, 1.8, 64,
                      0, True, gen, coarse_only=True)

    t0 = time.perf_counter()
    try:
        with torch.no_grad(), threadpool_limits(limits=threads):
            vt, rt = _median_rate(c3_torch, c3_rays)
            vn, rn = _median_rate(c3_numpy, c3_rays)
            v1, r1 = _median_rate(c1_torch, c1_rays)
    finally:
        torch.set_num_threads(prev_threads)
    best = "torch_port" if vt >= vn else "numpy_oracle"
    host = f"{model or 'host CPU'}, {os.cpu_count()} logical CPUs / {physical} physical cores on the host"
    return {"value": round(max(vt, vn), 2), "unit": "rays/s", "cores": int(threads), "kind": "port", "runs": 3,
            "stat": "median", "warmup": 1, "port": best,
            "sample": f"{c3_rays} rays x (128 coarse + 64 fine) per run, the faster of oracle/torch_port.render "
                      f"(the reference's torch CPU operators) and oracle/avr_oracle.render (numpy), fp32, on "
                      f"{threads} threads = this process's CPU share (affinity / cgroup quota / OMP_NUM_THREADS); "
                      f"{host}",
            "torch_port": {"value": round(vt, 2), "runs_rays_per_s": [round(x, 2) for x in rt]},
            "numpy_oracle": {"value": round(vn, 2), "runs_rays_per_s": [round(x, 2) for x in rn]},
            "config1": {"value": round(v1, 2), "unit": "rays/s", "runs": 3, "stat": "median",
                        "sample": f"BASELINE configs[0] (4096 rays x 64 coarse samples, coarse pass only: rays, "
                                  f"stratified z, coarse field, volume integral), {c1_rays} rays per run, torch port",
                        "runs_rays_per_s": [round(x, 2) for x in r1]},
            "wall_s": round(time.perf_counter() - t0, 1)}


def run_train(args, device, train_pmc=None):
    """--mode train: one train.py step (train.py:50-114) per step — SB = 4
    scenes x 512 rays (train.py defaults batch_size 4, ray_batch_size 512),
    the conf/default.conf renderer (64 coarse + 32 fine of which 16 depth
    samples) and field, MSE on rgb coarse + fine, backward, Adam (lr 1e-4).
    The latent maps are fixed inputs (the ResNet34 encoder is out of scope).
    --conf default_mv: the field train.py itself builds (train.py:262 parses
    conf/default_mv.conf: ResnetFC 5 x 512, combine_layer 3), same renderer.
    Timed twice: autograd through the HIP field (x3 training forward + HIP
    backward chain + the x3 weight-gradient kernel) and PyTorch autograd of
    the same module (forward_torch; the rest of the step is identical)."""
    from avr.conf import default_conf
    from avr.renderers import AdaptiveVolumeRenderer, VolumeRenderer
    SB, R = 4, 512
    NS = args.views                  # source views per object (train.py:56 fixes 1; models.py:566-579 combines them)
    net = build_scene(device, conf=args.conf, bn=args.bn, spade=args.spade)
    g = torch.Generator(device="cpu").manual_seed(7)
    net.encoder.set_latent(torch.randn(SB * NS, net.d_latent, 64, 64, generator=g).to(device))
    net.num_objs = SB
    net.num_views_per_obj = NS
    net.poses = net.poses.repeat(SB * NS, 1, 1)
    net.poses[:, 0, 3] += 0.05 * torch.arange(SB * NS, device=device, dtype=torch.float32)
    net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
    net.train()
    for p in net.parameters():
        p.requires_grad_(True)
    if args.renderer == "adaptive":
        # train.py:272-273 (any run name not starting with "VR" / naming "Raymarcher"):
        # AdaptiveVolumeRenderer.from_conf(conf["adaptive_renderer"]); its LSTM / out_layer train with the net
        # (rf_and_renderer.parameters(), train.py:300)
        torch.manual_seed(11)
        rend = AdaptiveVolumeRenderer.from_conf(default_conf()["adaptive_renderer"]).to(device)
        params = list(net.parameters()) + list(rend.parameters())
    else:
        rend = VolumeRenderer.from_conf(default_conf()["normal_renderer"]).to(device)
        rend.seed = 99
        params = list(net.parameters())
    x_pix = torch.rand(SB, R, 2, generator=g).to(device)
    c2w = torch.stack([orbit_c2w(0.3 + 0.9 * b) for b in range(SB)]).to(device)
    c2w = c2w.reshape(SB, 1, 4, 4).expand(SB, R, 4, 4)
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]] * SB, device=device)
    gt = torch.rand(SB, R, 3, generator=g).to(device)
    opt = torch.optim.Adam(params, lr=1e-4)

    def step():
        rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    res, nonfinite = {}, {}
    for mode in args.train_modes.split(","):
        net.hip_backward = mode in ("hip", "hip_graph")
        run = step
        if mode == "hip_graph":
            # the same step captured into one HIP graph (avr.graphs.GraphedTrainStep) with a capturable Adam; the
            # VolumeRenderer's in-kernel Philox draws would be keyed by the capture-time offset, so the adaptive
            # renderer only (its draws: the CPU start distances, staged per replay, and torch.rand on device)
            from avr.graphs import GraphedTrainStep
            if args.renderer != "adaptive":
                raise SystemExit("bench.py: --train-modes hip_graph needs --renderer adaptive")
            # the optimizer a captured step needs: capturable (its step counts on the device); fused (one
            # multi-tensor kernel: the capturable foreach form adds ~0.7 ms of small launches to this step,
            # profiles/r06l_adaptive_graph_fused_adam_ab.txt)
            opt_g = torch.optim.Adam(params, lr=1e-4, capturable=True, fused=True)

            def step_g():
                rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
                loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
                opt_g.zero_grad()
                loss.backward()
                opt_g.step()
                return loss
            run = GraphedTrainStep(step_g, nets=[net], renderers=[rend], warmup=3)
        for _ in range(max(args.warmup, 5 if mode == "hip_graph" else 0)):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = run()
        torch.cuda.synchronize()
        res[mode] = (time.perf_counter() - t0) / args.steps
        # no autograd graph of this mode outlives it (its AccumulateGrad nodes would carry their streams into the
        # next mode's steps, and into a capture)
        loss = loss.detach()
        if mode == "hip_graph":
            assert run.captures == 1 and bool(torch.isfinite(loss)), (run.captures, float(loss))
        if mode == "hip":
            assert bool(torch.isfinite(loss)), f"{mode}: non-finite loss {float(loss)} after the timed steps"
        elif not bool(torch.isfinite(loss)):
            # PyTorch autograd of the reference's own lookup divides by the camera z (models.py:799): a sample on
            # the source camera's plane gives 0 * inf = NaN there (DivBackward0; DESIGN.md "non-finite adaptive
            # step"). The yardstick leg records it instead of failing the line; the HIP leg above must be finite.
            nonfinite[mode] = float(loss)
    if args.renderer == "adaptive":
        spr = 1 + rend.n_coarse      # the marched point (coarse MLP) + the band (fine MLP); + steps latent lookups
        wl = (f"train.py defaults: {SB} scenes x {R} rays, AdaptiveVolumeRenderer (conf adaptive_renderer: "
              f"{rend.steps} LSTM march steps on 512-channel latent lookups, band of {rend.n_coarse} samples, "
              f"epsilon {rend.epsilon}), Adam lr 1e-4 over net + LSTM / out_layer")
    else:
        spr = rend.n_coarse + rend.n_coarse + rend.n_fine
        wl = (f"train.py defaults: {SB} scenes x {R} rays, {rend.n_coarse} coarse + {rend.n_fine} fine "
              f"({rend.n_fine_depth} depth) samples, Adam lr 1e-4")
    hip_t = res["hip"] if "hip" in res else res["hip_graph"]
    line = {
        "metric": "training rays/s (train.py step: forward + loss.backward() + Adam through "
                  + ("AdaptiveVolumeRenderer)" if args.renderer == "adaptive" else "VolumeRenderer)"),
        "value": round(SB * R / hip_t, 1), "unit": "rays/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(hip_t * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32 (field products as 3 fp16 MFMA terms)",
        "data": f"synthetic: random-init {args.conf}.conf field{' with --bn (training-mode BatchNorm)' if args.bn else ''}"
                f"{' with use_spade' if args.spade else ''}, {SB * NS} random 512x64x64 latents"
                f"{f' ({NS} source views per object)' if NS > 1 else ''}, random pixels/targets",
        "config": {"workload": wl + f", field of conf/{args.conf}.conf ({net.mlp_coarse.n_blocks} x "
                               f"{net.mlp_coarse.d_hidden} ResnetFC, combine_layer {net.mlp_coarse.combine_layer}"
                               + (", bn=True: training-mode BatchNorm, avr.bn_train)" if args.bn else
                                  ", layer by layer: avr.layer_train)" if (args.spade or NS > 1) else ")"),
                   "field_samples_per_step": SB * R * spr},
    }
    if "hip_graph" in res:
        line["hip_graph"] = {"value": round(SB * R / res["hip_graph"], 1), "ms_per_step": round(res["hip_graph"] * 1e3, 3),
                             "note": "the same step captured once into a HIP graph and replayed (avr.graphs."
                                     "GraphedTrainStep; Adam(capturable=True, fused=True) -- the eager legs use "
                                     "train.py's default Adam); the CPU start distances are drawn and staged per "
                                     "replay as an eager step draws them"}
    if "torch" in res:
        line["torch_autograd"] = {"value": round(SB * R / res["torch"], 1), "ms_per_step": round(res["torch"] * 1e3, 3)}
        if "torch" in nonfinite:
            line["torch_autograd"]["nonfinite_loss"] = nonfinite["torch"]
        line["speedup_vs_torch_autograd"] = round(res["torch"] / hip_t, 3)
    if train_pmc is not None:
        kern, note = train_pmc
        line["pmc"] = kern if kern is not None else {"note": note}
        line["pmc_source"] = ("rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE over a child bench.py "
                              "--pmc-child of this train step (1 warm-up + 1 step): mfma_busy = busy cycles / "
                              "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), clock = GRBM_GUI_ACTIVE / 8 / dispatch time")
    print(json.dumps(line), flush=True)


def _free_port():
    import socket
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        return sock.getsockname()[1]


def spawn_ranks(n):
    """`--gpus N` (N > 1) started without a torch.distributed launcher: run the
    N ranks as a child `torch.distributed.run` (one process per GPU, rendezvous
    on 127.0.0.1) and return its exit status. This process has not touched
    the GPU (nothing before this call initialises HIP), and it is never
    replaced by exec: the ranks are children."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def standin_render(c2w, K, x_pix, ray_ids=None, n_rays_total=None):
    """--device cpu: a deterministic per-ray function of the ray's own inputs
    (the HIP renderer needs a GPU). It exercises the launcher, the tile
    dealing and the gather of the config-5 path on gloo; it measures nothing."""
    rgb_c = torch.stack([x_pix[..., 0], x_pix[..., 1], x_pix.sum(-1)], -1)
    rgb_f = torch.sin(rgb_c * 3.0) + c2w[..., 0, 3:4]
    depth = x_pix[..., 0] * 10 + K[:, 0, 0, None]
    return rgb_c, rgb_f, depth, depth


def share_scene(net, device, use_dist):
    """N > 1: every rank renders rank 0's scene. avr.parallel.broadcast_scene sends its weights, latent map and
    source view (one collective per dtype) and invalidates the receivers' packed-weight / table / view caches;
    timed between barriers, max over ranks (once per scene, not per step)."""
    if not use_dist:
        return None
    from avr.parallel import broadcast_scene
    dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    nbytes = broadcast_scene(net, src=0)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                     device=device if dist.get_backend() != "gloo" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"ms": round(float(t[0]) * 1e3, 3), "bytes": int(nbytes), "src": 0,
            "what": "field weights + latent map + source view (avr.parallel.broadcast_scene), before the timed steps"}


def scene_checksum(net):
    """Sum of a few scene tensors in fp64: equal on every rank after share_scene."""
    ts = [net.mlp_coarse.lin_in.weight, net.mlp_fine.lin_out.weight, net.encoder.latent, net.poses]
    return round(float(sum(t.detach().double().sum().cpu() for t in ts)), 6)


def run_standin(args, config, world, rank):
    from avr.parallel import render_sharded
    from avr.video import get_opencv_pixel_coordinates
    n_views = 4 if config == 5 else 1
    x_pix = get_opencv_pixel_coordinates(args.frame, args.frame).reshape(1, -1, 2).repeat(1, n_views, 1)
    R = x_pix.shape[1]
    c2w = torch.stack([orbit_c2w(2 * np.pi * v / n_views) for v in range(n_views)])
    c2w = c2w.repeat_interleave(R // n_views, 0).reshape(1, R, 4, 4)
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]])
    # the scene distribution of the GPU path: ranks > 0 start from another scene and receive rank 0's
    net = build_scene(torch.device("cpu"), seed=0 if rank == 0 else 1000 + rank)
    shared = share_scene(net, torch.device("cpu"), world > 1)

    stimer = None
    if world > 1:
        from avr.parallel import ShardTimer
        stimer = ShardTimer()

    def step():
        if world > 1:
            return render_sharded(standin_render, c2w, K, x_pix, timer=stimer)
        return standin_render(c2w, K, x_pix)

    for _ in range(args.warmup):
        step()
    if world > 1:
        stimer.reset()
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    phases = shard_phases(stimer, args.steps, torch.device("cpu"), R) if world > 1 else None
    if rank == 0:
        line = {"metric": "rays/sec (128 coarse + 64 fine samples) + achieved HBM GB/s vs roofline",
                "value": round(R * args.steps / elapsed, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "strong" if config == 5 else "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "STAND-IN renderer on the CPU (--device cpu): launcher / sharding test, not a measurement",
                "config": {"workload": f"stand-in, {n_views} views x {args.frame}x{args.frame}", "rays_per_step": R,
                           "parallelism": f"ray-shard x{world} + gloo gather"},
                "checksum": [round(float(o.double().sum()), 6) for o in out[:3]],
                "scene_checksum": scene_checksum(net)}
        if shared is not None:
            line["scene_broadcast"] = shared
        if phases is not None:
            line["shard_phases"] = phases
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


FIELD_KERNEL_SOURCES = ("csrc/field_x3.hip", "csrc/x3_gemm.h", "csrc/field_common.h")


def field_kernel_hash():
    """sha256[:16] of the x3 field kernel's sources (what a PMC profile was taken of)."""
    import hashlib
    h = hashlib.sha256()
    for f in FIELD_KERNEL_SOURCES:
        with open(os.path.join(REPO, "adaptive-volume-rendering_amd", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _run_killable(cmd, timeout, env):
    """Run cmd in its own process group; on timeout kill the whole group."""
    import signal
    import subprocess
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True, cwd=REPO)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return None, "", f"timed out after {timeout} s"
    return p.returncode, out, err


def _short_kernel(name):
    import re
    return re.sub(r"\(.*", "", name).replace("void ", "").strip()


def pmc_passes(child_args, groups, match, timeout=240):
    """rocprofv3 --pmc passes over a child `bench.py --pmc-child <child_args>`, one pass per counter group (each
    group within one pass's limits, MI355X_MICROARCH.md), started BEFORE this process touches the GPU. Returns
    ({kernel: {counter: mean per dispatch, "dispatches": n, "mean_ns": mean dispatch time}} over the kernels
    whose name contains one of `match`, note)."""
    import csv
    import glob
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="avr_pmc_", dir=os.environ.get("TMPDIR") or "/tmp")
    env = dict(os.environ)
    env.setdefault("TMPDIR", "/tmp")
    vals, durs = {}, {}
    try:
        for counters in groups:
            d = os.path.join(tmp, counters[0])
            cmd = [prof, "--pmc", *counters, "-f", "csv", "-d", d, "-o", "pmc", "--", sys.executable,
                   os.path.abspath(__file__), "--pmc-child", *child_args]
            print(f"bench.py: rocprofv3 --pmc {' '.join(counters)} pass ...", file=sys.stderr, flush=True)
            rc, _, err = _run_killable(cmd, timeout, env)
            if rc != 0:
                return None, f"rocprofv3 --pmc {counters[0]} pass failed ({rc}): {err.strip()[-300:]}"
            for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(path) as fh:
                    for r in csv.DictReader(fh):
                        if not any(m in r["Kernel_Name"] for m in match):
                            continue
                        k = _short_kernel(r["Kernel_Name"])
                        key = (counters[0], r["Dispatch_Id"])
                        per = vals.setdefault(k, {}).setdefault(r["Counter_Name"], {})
                        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
                        if "End_Timestamp" in r:
                            durs.setdefault(k, {})[key] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    out = {}
    for k, cs in vals.items():
        e = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        dk = durs.get(k, {})
        e["mean_ns"] = sum(dk.values()) / max(len(dk), 1)
        # each counter's own dispatches' mean time (a clock is cycles of one pass over that pass's times)
        e["mean_ns_of"] = {c: sum(dk.get(key, 0.0) for key in v) / len(v) for c, v in cs.items()}
        out[k] = e
    return out, "ok"


def pmc_derived(e):
    """Clock and MFMA-busy of one kernel's pass averages: GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy =
    SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over the 1024 SIMDs) / (1024 x GRBM_GUI_ACTIVE / 8)."""
    d = {}
    g = e.get("GRBM_GUI_ACTIVE")
    if g:
        ns = e.get("mean_ns_of", {}).get("GRBM_GUI_ACTIVE") or e.get("mean_ns")
        if ns:
            d["clock_ghz"] = g / 8.0 / ns
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e:
            d["mfma_busy"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * g / 8.0)
    return d


def pmc_traffic(args, timeout=240):
    """The `roofline.traffic` and `roofline.mfma_busy` leg, measured in this run: two rocprofv3 --pmc passes
    (FETCH_SIZE + GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES; WRITE_SIZE + TCC_HIT/MISS) over a child
    `bench.py --pmc-child` (the same C3 workload: one warm-up + one timed step). Per field dispatch: L2->fabric
    bytes = 2 x FETCH_SIZE (gfx950 counts half of 16-B-per-lane reads) + WRITE_SIZE, Infinity-Cache hits
    included; the clock it ran at and its MFMA-busy fraction. Returns (dict or None, note)."""
    child = ["--precision", args.precision, "--rays", str(args.rays), "--n-coarse", str(args.n_coarse),
             "--n-fine", str(args.n_fine)]
    groups = (["FETCH_SIZE", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"],
              ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"])
    per, note = pmc_passes(child, groups, ("field_x3_kernel", "field_fwd_kernel"), timeout)
    if per is None:
        return None, note
    if len(per) != 1:
        return None, f"expected one field kernel instantiation, found {sorted(per)}"
    (kname, e), = per.items()
    for c in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
        if c not in e:
            return None, f"no {c} rows for the field kernel"
    hit, miss = e["TCC_HIT_sum"], e["TCC_MISS_sum"]
    der = pmc_derived(e)
    return {"kernel": kname, "bytes_per_launch": int((2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024),
            "fetch_size_kb_raw": e["FETCH_SIZE"], "write_size_kb": e["WRITE_SIZE"],
            "l2_hit_rate": hit / (hit + miss) if hit + miss > 0 else None, "dispatches": e["dispatches"],
            "clock_ghz": der.get("clock_ghz"), "mfma_busy": der.get("mfma_busy")}, "ok"


TRAIN_PMC_KERNELS = ("field_x3_kernel", "field_bwd_x3_kernel", "weight_grad_kernel", "bn_layer_kernel",
                     "lin_out_", "raymarch_")


def pmc_train(args, timeout=300):
    """--mode train --pmc-train: MFMA busy and clock per training kernel (the SAVE forward, the backward chain,
    the weight gradients, the layer-by-layer GEMMs) in one rocprofv3 --pmc pass over a child train step
    (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE). Returns ({kernel: {...}} or None, note)."""
    child = ["--mode", "train", "--train-modes", "hip", "--conf", args.conf, "--views", str(args.views),
             "--renderer", args.renderer] + (["--bn"] if args.bn else []) + (["--spade"] if args.spade else [])
    per, note = pmc_passes(child, (["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],), TRAIN_PMC_KERNELS, timeout)
    if per is None:
        return None, note
    res = {}
    for k, e in sorted(per.items(), key=lambda kv: -kv[1]["mean_ns"] * kv[1]["dispatches"]):
        der = pmc_derived(e)
        res[k] = {"dispatches": e["dispatches"], "mean_us": round(e["mean_ns"] / 1e3, 2),
                  "mfma_busy": None if der.get("mfma_busy") is None else round(der["mfma_busy"], 4),
                  "clock_ghz": None if der.get("clock_ghz") is None else round(der["clock_ghz"], 3)}
    return res, note


def _comm_device(device):
    """Where a cross-rank reduction's tensor lives: the GPU on RCCL, the host on gloo."""
    import torch.distributed as dist
    return torch.device("cpu") if dist.is_initialized() and dist.get_backend() == "gloo" else device


def time_steps(step, steps, warmup, world, device):
    """W untimed steps, then K timed steps between barrier + synchronize on
    both sides; the max over ranks. Returns (seconds, last output)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=_comm_device(device), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    return elapsed, out


def frame_views(n_views, frame, device):
    """BASELINE config 5's rays: n_views orbit views of a frame x frame
    get_opencv_pixel_coordinates grid, one ray batch with a per-ray pose."""
    from avr.video import get_opencv_pixel_coordinates
    x_pix = get_opencv_pixel_coordinates(frame, frame).reshape(1, -1, 2).repeat(1, n_views, 1).to(device)
    R = x_pix.shape[1]
    c2w = torch.stack([orbit_c2w(2 * np.pi * v / n_views) for v in range(n_views)]).to(device)
    c2w = c2w.repeat_interleave(R // n_views, 0).reshape(1, R, 4, 4)
    return x_pix, c2w


def config5_leg(args, net, fused, K, device):
    """BASELINE config 5's workload (4 orbit views x 800x800 per step) on this
    one GPU: the same renderer call each rank of `--gpus N` makes on its tiles,
    so the driver's 1 -> N ratio compares one workload."""
    from avr.renderers import VolumeRenderer
    x_pix, c2w = frame_views(4, args.frame, device)
    rend = VolumeRenderer(0.8, 1.8, args.n_coarse, args.n_fine, 0, 0.01, True)
    rend.seed = 1234
    sharded = dist is not None and dist.is_initialized()   # --dist: the per-rank path of --gpus N, gather included
    stimer = None
    if sharded:
        from avr.parallel import ShardTimer, render_sharded
        stimer = ShardTimer()

        def render_fn(c, k, x, ray_ids=None, n_rays_total=None):
            return rend(c, k, x, net, ray_ids=ray_ids, n_rays_total=n_rays_total)

    def step():
        fused._packed.clear()
        fused._pack_args.clear()
        with torch.no_grad():
            if sharded:
                return render_sharded(render_fn, c2w, K, x_pix, timer=stimer)[1]
            return rend(c2w, K, x_pix, net)[1]

    if sharded:
        step()
        stimer.reset()
    elapsed, out = time_steps(step, args.config5_steps, 0 if sharded else 1, dist.get_world_size() if sharded else 1,
                              device)
    assert rend.last_path == "fused" and bool(torch.isfinite(out).all())
    R = x_pix.shape[1]
    leg = {"value": round(R * args.config5_steps / elapsed, 1), "unit": "rays/s", "steps": args.config5_steps,
           "warmup": 1, "ms_per_step": round(elapsed / args.config5_steps * 1e3, 3), "rays_per_step": R,
           "scaling": "strong",
           "workload": f"BASELINE config 5 on 1 GPU: 4 orbit views x {args.frame}x{args.frame} ({R} rays) per step "
                       f"x ({args.n_coarse} coarse + {args.n_fine} fine), the per-rank renderer call of --gpus N"
                       + (" through avr.parallel.render_sharded (tiles, RCCL all_gather, reassembly)" if sharded else "")}
    if sharded:
        leg["shard_phases"] = shard_phases(stimer, args.config5_steps, device, R)
    return leg


def shard_phases(stimer, steps, device, n_rays):
    """The N > 1 attribution keys: per-step render / all_gather / reassembly ms of every rank (min / max over
    ranks; HIP events on each rank's stream), rays per rank and the gather's bytes per step."""
    from avr.parallel import gather_bytes, max_local_rays, phase_spread
    world = dist.get_world_size()
    ph = phase_spread(stimer, steps, device)
    return {"render_ms_per_step": ph["render"], "all_gather_ms_per_step": ph["all_gather"],
            "reassembly_ms_per_step": ph["reassembly"], "rays_per_rank_max": max_local_rays(n_rays, world),
            "gather_bytes_per_step": gather_bytes(n_rays, world),
            "note": "render: the rank's renderer call on its 64-ray tiles; all_gather: the RCCL collective "
                    "(includes waiting for the slowest rank); reassembly: packing + scattering the tiles into "
                    "the frame (avr.parallel.ShardTimer)"}


def config2_leg(args, net, fused, K, c2w, x_pix, device):
    """BASELINE configs[1]: the coarse pass alone on the headline rays (65536 x 128: rays, stratified z,
    field, composite), one launch chain per step."""
    import avr

    def step():
        fused._packed.clear()
        fused._pack_args.clear()
        with torch.no_grad():
            ro, rd, zc, _, _ = avr.ops.rays_sample_coarse(x_pix, K, c2w, 0.8, 1.8, args.n_coarse, seed=1234)
            rgb_c, _, _ = avr.ops.composite(zc, fused.forward_rays(ro[0], rd[0], zc, True), True, want_weights=False)
        return rgb_c

    steps = max(args.config5_steps, 3)
    elapsed, out = time_steps(step, steps, 1, 1, device)
    assert bool(torch.isfinite(out).all())
    R = x_pix.shape[1]
    return {"value": round(R * steps / elapsed, 1), "unit": "rays/s", "steps": steps, "warmup": 1,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "workload": f"BASELINE config 2: {R} rays x {args.n_coarse} coarse samples, coarse pass only"}


def config4_leg(args, net, K, device):
    """BASELINE configs[3]: one 800x800 frame per step with fine-pass early termination at T_stop 1e-5, on the
    bench's field (a fog that never reaches T < 1e-5 in [0.8, 1.8]: every sample is evaluated) and on the same
    field with its density biased by +30 (rays saturate as on an opaque scene: the tail is skipped)."""
    from avr.renderers import VolumeRenderer
    from avr.video import get_opencv_pixel_coordinates
    x_pix = get_opencv_pixel_coordinates(args.frame, args.frame).reshape(1, -1, 2).to(device)
    R = x_pix.shape[1]
    c2w = orbit_c2w(0.7).to(device).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
    res = {}
    for bias in (0.0, 30.0):
        n = net if bias == args.sigma_bias else build_scene(device, sigma_bias=bias)
        n.field_precision = args.precision
        rend = VolumeRenderer(0.8, 1.8, args.n_coarse, args.n_fine, 0, 0.01, True)
        rend.seed = 1234
        rend.t_stop = 1e-5
        evaluated = [0]

        def step():
            with torch.no_grad():
                out = rend(c2w, K, x_pix, n)[1]
            evaluated[0] += rend.last_fine_samples
            return out

        steps = args.config5_steps
        step()
        evaluated[0] = 0
        elapsed, out = time_steps(step, steps, 0, 1, device)
        assert rend.last_path == "fused" and bool(torch.isfinite(out).all())
        res[f"sigma_bias_{int(bias)}"] = {
            "value": round(R * steps / elapsed, 1), "unit": "rays/s", "steps": steps, "warmup": 1,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "fine_samples_evaluated_fraction": round(evaluated[0] / (steps * R * (args.n_coarse + args.n_fine)), 4)}
    out = dict(res["sigma_bias_0"])
    out["workload"] = (f"BASELINE config 4: one {args.frame}x{args.frame} frame ({R} rays) per step x "
                       f"({args.n_coarse} coarse + {args.n_fine} fine), fine-pass early termination T_stop 1e-5")
    out["sigma_bias_30"] = res["sigma_bias_30"]
    return out


def fp32_leg(args, net, fused, timer, K, c2w, x_pix, device):
    """The strict-fp32 field (v_mfma_f32_16x16x4_f32) on the headline workload,
    same box and process: a measured anchor for the x3 number."""
    from avr.renderers import VolumeRenderer
    rend = VolumeRenderer(0.8, 1.8, args.n_coarse, args.n_fine, 0, 0.01, True)
    rend.seed = 1234
    prev = net.field_precision
    net.field_precision = "fp32"

    def step():
        fused._packed.clear()
        fused._pack_args.clear()
        with torch.no_grad():
            return rend(c2w, K, x_pix, net)[1]

    try:
        step()
        timer.reset()
        elapsed, out = time_steps(step, args.fp32_steps, 0, 1, device)
        field_ms = timer.total_ms()
        ach = timer.samples * field_flops_per_sample() / (field_ms * 1e-3) / 1e12
    finally:
        net.field_precision = prev
    R = x_pix.shape[1]
    return {"value": round(R * args.fp32_steps / elapsed, 1), "unit": "rays/s", "steps": args.fp32_steps,
            "warmup": 1, "ms_per_step": round(elapsed / args.fp32_steps * 1e3, 3), "dtype": "fp32",
            "kernel": "field_fwd_kernel<32> (v_mfma_f32_16x16x4_f32)", "field_achieved_TFLOPs": round(ach, 2),
            "field_frac_of_fp32_peak": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
            "avg_launch_ms": round(field_ms / max(len(timer.events), 1), 3)}


def main():
    global dist
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without torch.distributed.run's environment, N > 1 starts the ranks "
                         "itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rays", type=int, default=65536, help="config 3: rays per GPU per step")
    ap.add_argument("--n-coarse", type=int, default=128)
    ap.add_argument("--n-fine", type=int, default=64)
    ap.add_argument("--precision", choices=["x3", "fp32"], default="x3",
                    help="field MFMA path: split-fp16 (3 products, fp32 accumulate) or fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc traffic leg")
    ap.add_argument("--no-legs", action="store_true", help="skip the config-2/4/5 and fp32 legs of the N=1 line")
    ap.add_argument("--config5-steps", type=int, default=2, help="N=1: timed steps of the config-4 / 5 legs")
    ap.add_argument("--fp32-steps", type=int, default=3, help="N=1: timed steps of the strict-fp32 leg")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-train", action="store_true",
                    help="--mode train: one rocprofv3 --pmc pass (MFMA busy + clock per training kernel) first")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the RCCL process group even at one rank (the N > 1 code path on one GPU)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=None,
                    help="BASELINE config (default: 3 on one GPU, 5 on more): 2 = the coarse pass only (65536 "
                         "rays x 128 samples: rays, stratified z, field, composite); 3 = 65536 random rays per GPU (weak "
                         "scaling); 5 = 4 orbit views of 800x800 per step for the whole job, dealt to the ranks in "
                         "64-ray tiles (strong scaling, avr.parallel.render_sharded); 4 = one 800x800 frame per "
                         "step with fine-pass early termination at T_stop 1e-5")
    ap.add_argument("--frame", type=int, default=800, help="configs 4/5: frame side in pixels")
    ap.add_argument("--sigma-bias", type=float, default=0.0,
                    help="density bias of the synthetic field (config 4: opacity of the scene)")
    ap.add_argument("--mode", choices=["render", "train"], default="render",
                    help="render: the headline inference metric; train: one train.py step per step (1 GPU)")
    ap.add_argument("--conf", choices=["default", "default_mv"], default="default",
                    help="--mode train: the field of conf/default.conf or conf/default_mv.conf (train.py:262)")
    ap.add_argument("--train-modes", default="hip,torch", help="--mode train: which autograd paths to time")
    ap.add_argument("--bn", action="store_true",
                    help="--mode train: train.py --bn (ResnetBlockFC(bn=True), training-mode BatchNorm: the "
                         "layer-by-layer HIP path avr.bn_train)")
    ap.add_argument("--spade", action="store_true", help="--mode train: ResnetFC(use_spade=True) (avr.layer_train)")
    ap.add_argument("--views", type=int, default=1,
                    help="--mode train: source views per object, NS (> 1: the views' combine, avr.layer_train)")
    ap.add_argument("--renderer", choices=["volume", "adaptive"], default="volume",
                    help="--mode train: VolumeRenderer (train.py 'VR*' runs) or AdaptiveVolumeRenderer (train.py's "
                         "default for other run names, train.py:268-273)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: stand-in renderer on gloo (tests the launcher and the config-5 sharding only)")
    args = ap.parse_args()
    if args.pmc_child:
        args.steps, args.warmup, args.no_cpu_baseline, args.no_pmc, args.no_legs = 1, 1, True, True, True
        args.pmc_train, args.train_modes = False, "hip"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    config = args.config if args.config is not None else (3 if world == 1 else 5)
    use_dist = world > 1 or args.dist
    if args.device == "cpu":
        if use_dist:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        return run_standin(args, config, world, rank)

    # the traffic leg runs first: its profiled children use the GPU before this process does
    pmc, pmc_note = None, "skipped"
    if (world == 1 and args.mode == "render" and config == 3 and not args.no_pmc):
        pmc, pmc_note = pmc_traffic(args)
    train_pmc = None
    if world == 1 and args.mode == "train" and args.pmc_train:
        train_pmc = pmc_train(args)

    if use_dist:
        import torch.distributed as dist
        if "RANK" not in os.environ:   # --dist at one rank without a launcher: a one-rank rendezvous on 127.0.0.1
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(_free_port()))
        if os.environ.get("AVR_BENCH_ONE_GPU_GLOO") == "1":
            # rehearsal of the N > 1 path on a one-GPU box: every rank on GPU 0, the group on gloo (RCCL needs one
            # GPU per rank); the timing means nothing, the code path is the multi-GPU one
            local_rank = 0
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    import avr
    from avr.renderers import VolumeRenderer
    avr.load_library()
    if args.mode == "train":
        return run_train(args, device, train_pmc)

    # N > 1: ranks > 0 build a scene of the same architecture and receive rank 0's (broadcast_scene)
    net = build_scene(device, seed=0 if rank == 0 else 1000 + rank, sigma_bias=args.sigma_bias)
    net.field_precision = args.precision
    fused = net.fused()
    shared = share_scene(net, device, use_dist)
    timer = FieldTimer()
    timer.wrap(fused)
    hbm = HbmKernelTimer(avr.ops)
    hbm.install()
    rend = VolumeRenderer(0.8, 1.8, args.n_coarse, args.n_fine, 0, 0.01, True)
    # config 5: one frame-wide Philox stream keyed by global ray ids (render_sharded); else a batch per rank
    rend.seed = 1234 if config == 5 else 1234 + rank
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]], device=device)
    if config == 4:
        # one full 800x800 frame per step (get_opencv_pixel_coordinates grid), fine pass with early
        # termination at T_stop = 1e-5; with N GPUs each rank renders its own frame
        from avr.video import get_opencv_pixel_coordinates
        x_pix = get_opencv_pixel_coordinates(args.frame, args.frame).reshape(1, -1, 2).to(device)
        R = x_pix.shape[1]
        rend.t_stop = 1e-5
    elif config == 5:
        # BASELINE config 5: 4 views x 800x800 per step for the whole job; every rank renders its 64-ray tiles
        # of all 4 views and one all_gather assembles the frames (avr.parallel.render_sharded)
        # (one scene: the 4 views are one ray batch of 4 x 640 000 rays with a per-ray pose)
        x_pix, c2w = frame_views(4, args.frame, device)
        R = x_pix.shape[1]
    else:
        R = args.rays
        g = torch.Generator(device="cpu").manual_seed(100 + rank)
        x_pix = torch.rand(1, R, 2, generator=g).to(device)
    gathered = None
    stimer = None
    if config == 5:
        from avr.parallel import ShardTimer, render_sharded
        stimer = ShardTimer()
    else:
        c2w = orbit_c2w(0.7 + 0.5 * rank).to(device).reshape(1, 1, 4, 4).expand(1, R, 4, 4)
        if use_dist:
            gathered = torch.empty(world * R * 7, device=device)

    def render_fn(c, k, x, ray_ids=None, n_rays_total=None):
        return rend(c, k, x, net, ray_ids=ray_ids, n_rays_total=n_rays_total)

    def step():
        fused._packed.clear()       # per-scene prep inside the step: repack weights (from scratch), rebuild lin_z tables
        fused._pack_args.clear()
        with torch.no_grad():
            if config == 5:
                if use_dist:
                    rgb_c, rgb_f, depth, _ = render_sharded(render_fn, c2w, K, x_pix, timer=stimer)
                else:
                    rgb_c, rgb_f, depth, _ = rend(c2w, K, x_pix, net)
                return rgb_f
            if config == 2:   # BASELINE configs[1]: the coarse pass alone
                ro, rd, zc, _, _ = avr.ops.rays_sample_coarse(x_pix, K, c2w, 0.8, 1.8, args.n_coarse, seed=rend.seed)
                rgb_c, _, _ = avr.ops.composite(zc, fused.forward_rays(ro[0], rd[0], zc, True), True,
                                                want_weights=False)
                rend.last_path, rend.last_fine_samples = "fused", 0
                return rgb_c
            rgb_c, rgb_f, depth, _ = rend(c2w, K, x_pix, net)
            if use_dist:
                local = torch.cat([rgb_c.reshape(-1), rgb_f.reshape(-1), depth.reshape(-1)])
                dist.all_gather_into_tensor(gathered, local)
        return rgb_f

    for _ in range(args.warmup):
        step()
    assert rend.last_path == "fused", "bench must run the fused HIP field"
    torch.cuda.synchronize()
    timer.reset()
    if stimer is not None:
        stimer.reset()
    hbm.on = True
    fine_evaluated = [0]

    def counted_step():
        out = step()
        fine_evaluated[0] += rend.last_fine_samples
        return out

    elapsed, out = time_steps(counted_step, args.steps, 0, world if use_dist else 1, device)
    hbm.on = False
    field_ms = timer.total_ms()
    field_launches = len(timer.events)
    field_spread = None
    if use_dist:
        t = torch.tensor([field_ms, -field_ms], device=_comm_device(device), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        field_spread = {"min": round(-float(t[1]), 3), "max": round(float(t[0]), 3)}
        field_ms = float(t[0])
    assert bool(torch.isfinite(out).all())
    if args.pmc_child:
        return

    # whole-job rays: config 5 renders a fixed 4 x 800 x 800 per step over all ranks (strong scaling)
    rays_total = (R if config == 5 else R * world) * args.steps
    value = rays_total / elapsed
    samples_per_ray = args.n_coarse if config == 2 else args.n_coarse + args.n_coarse + args.n_fine
    fps = field_flops_per_sample()
    achieved_tflops = timer.samples * fps / (field_ms * 1e-3) / 1e12
    # compulsory bytes of an average field launch: z in + (r, g, b, sigma) out per sample, ro / rd
    # per ray, the x3 weight blob (4 B per weight: fp16 hi + lo) and the three lin_z tables (fp32)
    rays_per_launch = -(-R // world) if (config == 5 and use_dist) else R
    alg_bytes = (timer.samples / max(field_launches, 1) * 20 + rays_per_launch * 24
                 + 4 * (42 * 512 + 6 * 512 * 512 + 512 * 4) + 3 * 64 * 64 * 512 * 4)
    if args.precision == "x3":
        # each fp32-equivalent MAC is 3 fp16 MFMA MACs: the attainable fp32-equivalent peak is fp16 / 3
        peak, kname = FP16_MFMA_PEAK_TFLOPS / 3.0, ("field_x3_kernel<4,8> (8 waves; fused PE + lin_z interpolation + ResnetFC on "
                                                    "split-fp16 v_mfma_f32_16x16x32_f16 x3, fp32 accumulate)")
    else:
        peak, kname = FP32_MFMA_PEAK_TFLOPS, ("field_fwd_kernel<32> (fused PE + latent lookup + ResnetFC on "
                                              "v_mfma_f32_16x16x4_f32)")
    line = {
        "metric": "rays/sec (128 coarse + 64 fine samples) + achieved HBM GB/s vs roofline",
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if config == 5 else "weak",
        "vs_baseline": None,
        "dtype": "fp32" if args.precision == "fp32" else "fp32 (field products as 3 fp16 MFMA terms)",
        "data": ("synthetic rays (x_pix ~ U[0,1)^2, orbit pose)" if config in (2, 3) else
                 "synthetic rays (get_opencv_pixel_coordinates 800x800 grid, orbit poses)")
                + ", random-init default.conf field, random 512x64x64 latent",
        "config": {"workload": (f"BASELINE config 3: {R} rays/GPU x ({args.n_coarse} coarse + {args.n_fine} fine, "
                                "n_fine_depth 0), conf/default.conf PixelNeRF field (3x512 ResnetFC, d_latent 512)")
                   if config == 3 else
                   (f"BASELINE config 2: {R} rays/GPU x {args.n_coarse} coarse samples, coarse pass only (rays, "
                    "stratified z, field, composite), conf/default.conf PixelNeRF field") if config == 2 else
                   (f"BASELINE config 4: 800x800 frame ({R} rays)/GPU x ({args.n_coarse} coarse + {args.n_fine} "
                    f"fine), fine-pass early termination T_stop 1e-5, sigma bias {args.sigma_bias}, "
                    "conf/default.conf PixelNeRF field") if config == 4 else
                   (f"BASELINE config 5: 4 orbit views x 800x800 ({R} rays) per step over {world} GPU(s) in "
                    f"64-ray tiles x ({args.n_coarse} coarse + {args.n_fine} fine), conf/default.conf PixelNeRF field"),
                   "rays_per_gpu": R if config != 5 else -(-R // world), "n_coarse": args.n_coarse, "n_fine": args.n_fine,
                   "field_samples_per_ray": samples_per_ray,
                   "parallelism": f"ray-shard x{world}" + (" + RCCL gather" if use_dist else " (no collective at N=1)")},
        "roofline": {
            "kernel": kname,
            "bound": "mfma",
            "achieved": round(achieved_tflops, 2),
            "peak": round(peak, 1),
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / peak, 4),
            "precision": args.precision,
            "traffic": None,
            "flops_per_sample": fps,
            "reference_flops_per_sample": reference_flops_per_sample(),
            "avg_launch_ms": round(field_ms / max(field_launches, 1), 3),
            "field_share_of_step": round(field_ms / (elapsed * 1e3), 4),
            "field_kernel_sha16": field_kernel_hash(),
            "algorithmic_bytes_per_launch": int(alg_bytes),
        },
    }
    if args.precision == "x3":
        # context, not the contract's peak: back-to-back 16x16x32 fp16 MFMAs with random operands are held by
        # the board's power limit to ~1.87 PFLOP/s (1.32 kW, 1.85-1.95 GHz; profiles/r02_mfma_power_probe.txt)
        pl = 1868.0 / 3.0
        line["roofline"]["power_limited_peak"] = {
            "value": round(pl, 1), "unit": "TFLOP/s", "frac": round(achieved_tflops / pl, 4),
            "source": "profiles/r02_mfma_power_probe.txt (scripts/probe/mfma_probe.hip, random fp16 operands) / 3"}
    if pmc is not None:
        line["roofline"]["traffic"] = pmc["bytes_per_launch"]
        line["roofline"]["traffic_source"] = (
            f"this run: rocprofv3 --pmc passes over a child bench.py --pmc-child (same workload), mean of "
            f"{pmc['dispatches']} field dispatches; 2 x FETCH_SIZE + WRITE_SIZE = L2->fabric bytes incl. "
            "Infinity-Cache hits")
        line["roofline"]["traffic_over_algorithmic"] = round(pmc["bytes_per_launch"] / alg_bytes, 1)
        line["roofline"]["l2_hit_rate"] = None if pmc["l2_hit_rate"] is None else round(pmc["l2_hit_rate"], 4)
        if pmc.get("mfma_busy") is not None:
            line["roofline"]["mfma_busy"] = round(pmc["mfma_busy"], 4)
            line["roofline"]["mfma_busy_source"] = (
                f"the --pmc pass of this run over {pmc['kernel']}: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x "
                "GRBM_GUI_ACTIVE / 8 XCDs), the fraction of the kernel's cycles the matrix cores were busy")
        if pmc.get("clock_ghz"):
            # the MFMA peak scales with the clock the board's power limit allows (2.4 GHz nominal)
            c = pmc["clock_ghz"]
            line["roofline"]["clock"] = {
                "ghz": round(c, 3), "peak_at_clock": round(peak * c / 2.4, 1),
                "frac_at_clock": round(achieved_tflops / (peak * c / 2.4), 4),
                "source": "the --pmc pass of this run: GRBM_GUI_ACTIVE / 8 XCDs / field dispatch time"}
    else:
        line["roofline"]["traffic_source"] = f"not measured in this run ({pmc_note})"
    # the renderer's HBM-bound kernels (the metric's "achieved HBM GB/s vs roofline"), HIP events per launch,
    # against the 8 TB/s peak and against what a streaming copy reaches on this box
    ach = achievable_hbm_gbs(device)
    line["hbm_achievable_GBs"] = round(ach[0], 1)
    line["hbm_write_achievable_GBs"] = round(ach[1], 1)
    line["hbm_kernels"] = hbm.report(achievable=ach)
    if shared is not None:
        line["scene_broadcast"] = shared
        line["scene_checksum"] = scene_checksum(net)
    if config == 5 and use_dist:
        line["shard_phases"] = shard_phases(stimer, args.steps, device, R)
    if field_spread is not None:
        # every rank's field kernel time over the timed steps (HIP events around its field launches): a slow
        # rank or an uneven tile split shows as max >> min
        line["field_ms_per_rank"] = dict(field_spread, steps=args.steps, launches_per_rank=field_launches)
    if config == 4:
        line["config"]["fine_samples_evaluated_fraction"] = round(
            fine_evaluated[0] / (args.steps * R * (args.n_coarse + args.n_fine)), 4)
    if world == 1 and config == 3 and not args.no_legs:
        line["config2"] = config2_leg(args, net, fused, K, c2w, x_pix, device)
        line["config4"] = config4_leg(args, net, K, device)
        line["config5"] = config5_leg(args, net, fused, K, device)
        if args.precision == "x3":
            line["fp32"] = fp32_leg(args, net, fused, timer, K, c2w, x_pix, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
