"""Diagnostic: the bench's AdaptiveVolumeRenderer train step (bench.py run_train --renderer adaptive) run for
PROBE_STEPS steps per mode (PROBE_MODES, default "hip,torch", each from the same fresh scene, or with
PROBE_CONTINUE=1 one after the other on one scene as bench.py times them), checking every step
that the loss, the renderer outputs and every parameter gradient are finite; at the first non-finite value it
prints which, with the largest finite gradient magnitudes, and stops that mode. Not part of the product."""
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "adaptive-volume-rendering_amd"))


def setup():
    import bench
    from avr.conf import default_conf
    from avr.renderers import AdaptiveVolumeRenderer
    dev = torch.device("cuda:0")
    SB, R = 4, 512
    net = bench.build_scene(dev, conf="default_mv", bn=False)
    g = torch.Generator(device="cpu").manual_seed(7)
    net.encoder.set_latent(torch.randn(SB, net.d_latent, 64, 64, generator=g).to(dev))
    net.num_objs = SB
    net.poses = net.poses.repeat(SB, 1, 1)
    net.poses[:, 0, 3] += 0.05 * torch.arange(SB, device=dev, dtype=torch.float32)
    net.focal, net.c = net.focal.repeat(SB, 1), net.c.repeat(SB, 1)
    net.train()
    for p in net.parameters():
        p.requires_grad_(True)
    torch.manual_seed(11)
    rend = AdaptiveVolumeRenderer.from_conf(default_conf()["adaptive_renderer"]).to(dev)
    named = [("net." + n, p) for n, p in net.named_parameters()] + [("rend." + n, p) for n, p in rend.named_parameters()]
    x_pix = torch.rand(SB, R, 2, generator=g).to(dev)
    c2w = torch.stack([bench.orbit_c2w(0.3 + 0.9 * b) for b in range(SB)]).to(dev)
    c2w = c2w.reshape(SB, 1, 4, 4).expand(SB, R, 4, 4)
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]] * SB, device=dev)
    gt = torch.rand(SB, R, 3, generator=g).to(dev)
    opt = torch.optim.Adam([p for _, p in named], lr=1e-4)
    return net, rend, named, (c2w, K, x_pix, gt), opt


def diagnose(state):
    """Re-run the failing step (same parameters, same RNG state) with avr's per-op non-finite checks and torch's
    anomaly mode on, and with a hook on every tensor the march's backward receives: names the first op whose
    output or gradient is non-finite."""
    from avr import anomaly
    from avr import renderers as rmod
    net, rend, named, (c2w, K, x_pix, gt), opt = state
    seen = {}
    orig = rmod._MarchTrain.backward

    def spy(ctx, grad_world):
        g = grad_world.detach()
        seen["grad_world"] = (int((~torch.isfinite(g)).sum()), float(g[torch.isfinite(g)].abs().max()) if
                              bool(torch.isfinite(g).any()) else 0.0)
        tables, trace, st, rd, P, lat_t = ctx.keep
        seen["trace_finite"] = bool(torch.isfinite(trace).all())
        seen["min_abs_rd_x"] = float(rd[:, 0].abs().min())
        return orig(ctx, grad_world)

    from avr import field as fmod
    forig = fmod._FieldTrain.backward

    def fspy(ctx, grad_out):
        xyz = ctx.saved_tensors[0]
        res = getattr(forig, "__wrapped__", forig)(ctx, grad_out)   # the unchecked backward: print, then raise
        d_xyz = res[3]
        if d_xyz is not None and not bool(torch.isfinite(d_xyz).all()):
            bad = torch.nonzero(~torch.isfinite(d_xyz.reshape(-1, 3)).all(-1)).reshape(-1)
            pts = xyz.detach().reshape(-1, 3)[bad]
            poses = ctx.fused.net.poses
            for i, pt in zip(bad.tolist()[:4], pts.tolist()[:4]):
                sc = i // xyz.shape[1]
                Pm = poses[min(sc, poses.shape[0] - 1)].double()
                xc = (Pm[:3, :3] @ torch.tensor(pt, dtype=torch.float64, device=Pm.device) + Pm[:3, 3]).tolist()
                ptf = torch.tensor(pt, dtype=torch.float32, device=poses.device)
                xc32 = (poses[min(sc, poses.shape[0] - 1), :3, :3] @ ptf + poses[min(sc, poses.shape[0] - 1), :3, 3])
                print(f"diagnose: non-finite d_xyz at point {i} (scene {sc}) xyz {pt} camera point (fp64) {xc} "
                      f"(fp32 {xc32.tolist()}) d_xyz {d_xyz.reshape(-1, 3)[i].tolist()}", flush=True)
        anomaly.check_outputs("_FieldTrain.backward", res)
        return res

    fmod._FieldTrain.backward = staticmethod(fspy)
    rmod._MarchTrain.backward = staticmethod(spy)
    anomaly.set_detect_anomaly(True)
    try:
        with torch.autograd.set_detect_anomaly(True):
            rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
            loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
            opt.zero_grad()
            loss.backward()
        print("diagnose: no non-finite value raised", flush=True)
    except Exception as e:   # noqa: BLE001 -- the diagnosis is the message
        print(f"diagnose: {type(e).__name__}: {str(e)[:600]}", flush=True)
    finally:
        anomaly.set_detect_anomaly(False)
        rmod._MarchTrain.backward = staticmethod(orig)
        fmod._FieldTrain.backward = staticmethod(forig)
    print(f"diagnose: march backward input {seen}", flush=True)


def run(mode, steps, state):
    net, rend, named, (c2w, K, x_pix, gt), opt = state
    net.hip_backward = mode == "hip"
    for it in range(steps):
        rng = (torch.get_rng_state(), torch.cuda.get_rng_state())
        rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        bad = [n for n, p in named if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
        if (not bool(torch.isfinite(loss)) or bad) and os.environ.get("PROBE_DIAGNOSE", "1") == "1":
            torch.set_rng_state(rng[0])
            torch.cuda.set_rng_state(rng[1])
            diagnose(state)
        if not bool(torch.isfinite(loss)) or bad:
            print(f"{mode}: step {it}: loss {float(loss)} finite outputs "
                  f"{bool(torch.isfinite(rgb_c).all())}/{bool(torch.isfinite(rgb_f).all())}; non-finite grads {bad}",
                  flush=True)
            for n, p in named:
                if p.grad is not None:
                    fin = p.grad[torch.isfinite(p.grad)]
                    print(f"   {n}: max|finite grad| {float(fin.abs().max()) if fin.numel() else 0:.3e} "
                          f"non-finite {int((~torch.isfinite(p.grad)).sum())}", flush=True)
            return False
        opt.step()
        if it % 10 == 0:
            print(f"{mode}: step {it} loss {float(loss):.6f}", flush=True)
    print(f"{mode}: {steps} steps finite, last loss {float(loss):.6f}", flush=True)
    return True


if __name__ == "__main__":
    steps = int(os.environ.get("PROBE_STEPS", 60))
    # PROBE_CONTINUE=1: the modes in turn on one scene and optimizer state, as bench.py times them
    cont = os.environ.get("PROBE_CONTINUE", "0") == "1"
    state = setup() if cont else None
    for m in os.environ.get("PROBE_MODES", "hip,torch").split(","):
        if not run(m, steps, state if cont else setup()):
            break
