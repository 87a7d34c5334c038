"""Reads before writes on the training paths (one adaptive train.py bench run ended on a
non-finite loss, profiles/r04q_bench_train_adaptive_mv.log, and did not repeat; the bench is seeded, so a run
that differs between boxes points at memory read before it is written -- a fresh hipMalloc holds whatever the
box's last job left there).

Every floating-point device buffer the product allocates with torch.empty / empty_like / new_empty -- kernel
outputs, packed weight blobs, lin_z tables, the training forward's saved rows, the march's trace and state, the
weight-gradient partials -- starts as NaN in one run and as 0.0 in another (avr.anomaly.poison_allocations).
bench.py's own train.py step (run_train: 4 scenes x 512 rays, conf/default_mv.conf's field, Adam) runs twice from
the same seeds under each fill: every loss, output and gradient must be finite, and the two fills must agree.
An element read before it is written makes them differ (NaN against a reproducible value).

Match: /root/reference/renderers.py:413-432, :480-509 (AdaptiveVolumeRenderer), :121-289 (VolumeRenderer);
train.py:108-114."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _setup(renderer, bn):
    """bench.run_train's scene, renderer, pixels, targets and optimizer (train.py defaults)."""
    import bench
    from avr.conf import default_conf
    from avr.renderers import AdaptiveVolumeRenderer, VolumeRenderer
    SB, R = 4, 512
    net = bench.build_scene(DEV, conf="default_mv", bn=bn)
    g = torch.Generator(device="cpu").manual_seed(7)
    net.encoder.set_latent(torch.randn(SB, net.d_latent, 64, 64, generator=g).to(DEV))
    net.num_objs = SB
    net.poses = net.poses.repeat(SB, 1, 1)
    net.poses[:, 0, 3] += 0.05 * torch.arange(SB, device=DEV, dtype=torch.float32)
    net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
    net.train()
    for p in net.parameters():
        p.requires_grad_(True)
    torch.manual_seed(11)
    if renderer == "adaptive":
        rend = AdaptiveVolumeRenderer.from_conf(default_conf()["adaptive_renderer"]).to(DEV)
    else:
        rend = VolumeRenderer.from_conf(default_conf()["normal_renderer"]).to(DEV)
        rend.seed = 99
    named = [("net." + n, p) for n, p in net.named_parameters()] + [("rend." + n, p) for n, p in rend.named_parameters()]
    x_pix = torch.rand(SB, R, 2, generator=g).to(DEV)
    c2w = torch.stack([bench.orbit_c2w(0.3 + 0.9 * b) for b in range(SB)]).to(DEV)
    c2w = c2w.reshape(SB, 1, 4, 4).expand(SB, R, 4, 4)
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]] * SB, device=DEV)
    gt = torch.rand(SB, R, 3, generator=g).to(DEV)
    opt = torch.optim.Adam([p for _, p in named], lr=1e-4)
    return net, rend, named, (c2w, K, x_pix, gt), opt


def _run(fill, renderer, bn, steps=2):
    """`steps` train steps under one allocation fill -> per step: loss, outputs, every gradient."""
    from avr.anomaly import poison_allocations
    torch.manual_seed(1234)
    rec = []
    with poison_allocations(fill):
        net, rend, named, (c2w, K, x_pix, gt), opt = _setup(renderer, bn)
        for _ in range(steps):
            outs = rend(c2w, K, x_pix, net)
            rgb_c, rgb_f = outs[0], outs[1]
            loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
            opt.zero_grad()
            loss.backward()
            grads = {n: p.grad.detach().clone() for n, p in named if p.grad is not None}
            rec.append(dict(grads, loss=loss.detach().reshape(1), rgb_c=rgb_c.detach(), rgb_f=rgb_f.detach(),
                            depth=outs[2].detach()))
            opt.step()
    torch.cuda.synchronize()
    assert rend.last_path == ("hip_train" if renderer == "adaptive" else "module"), rend.last_path
    return rec


@pytest.mark.parametrize("renderer,bn", [("adaptive", False), ("volume", False), ("volume", True)])
def test_training_step_reads_no_unwritten_memory(renderer, bn):
    """Three runs: NaN fill, zero fill, zero fill again. The NaN run must be finite and equal to the zero run
    (within 4x the zero runs' own spread), and the two zero runs must agree bit for bit: every training path is
    deterministic since ABI 13. (Before, the march backward's float atomics made two identical adaptive steps
    differ in the LSTM gradients' last bits -- 7.6e-7 of max -- and one Adam step turned that into 0.74 of some
    gradient's max at the next step, profiles/r05a_pytest_poison.log.)"""
    nan_run = _run(float("nan"), renderer, bn)
    zero_run = _run(0.0, renderer, bn)
    zero2 = _run(0.0, renderer, bn)
    for step, (a, b, c) in enumerate(zip(nan_run, zero_run, zero2)):
        assert set(a) == set(b) == set(c)
        for name, run in (("NaN", a), ("zero", b)):
            bad = [k for k, t in run.items() if not bool(torch.isfinite(t).all())]
            assert not bad, f"step {step}: non-finite under the {name} fill: {bad}"
        worst, spread, nondet = 0.0, 0.0, []
        for k in a:
            s = float(b[k].abs().max()) or 1.0
            d = float((a[k] - b[k]).abs().max())
            dz = float((c[k] - b[k]).abs().max())
            if dz > 0:
                nondet.append(k)
            worst, spread = max(worst, d / s), max(spread, dz / s)
            assert d <= 4.0 * dz + 1e-7 * s, (f"step {step}: {k} differs between the NaN and zero fills by {d:.3e} "
                                              f"(zero vs zero {dz:.3e}) of {s:.3e}")
        print(f"{renderer}{' --bn' if bn else ''} step {step}: loss {float(a['loss']):.6f}, NaN vs zero fill "
              f"{worst:.2e} of max, zero vs zero {spread:.2e}; not bit-reproducible: {nondet}")
        assert not nondet, f"step {step}: two identical runs differ in {nondet}"
