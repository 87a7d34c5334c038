"""A/B of the adaptive train.py step (bench.py --mode train --renderer adaptive, default_mv) inside one process:
blocks of STEPS steps alternate between arms (environment switches read per call), ROUNDS times, so box jitter
hits both arms alike; prints each arm's per-block ms and median.

usage: python scripts/adaptive_ab.py [ROUNDS] [STEPS] ARM_A ARM_B   (an arm: "NAME=VALUE,..." environment
switches, or "-"; a leading "graph:" runs that arm through avr.graphs.GraphedTrainStep with a capturable Adam,
"graphf:" with a capturable fused Adam)"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    arms = sys.argv[3:5] if len(sys.argv) > 4 else ["AVR_ADAPTIVE_SIDE_STREAM=1", "AVR_ADAPTIVE_SIDE_STREAM=0"]
    from avr.conf import default_conf
    from avr.renderers import AdaptiveVolumeRenderer
    import avr
    avr.load_library()
    dev = torch.device("cuda", 0)
    SB, R = 4, 512
    net = bench.build_scene(dev, conf="default_mv")
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
    params = list(net.parameters()) + list(rend.parameters())
    opt = torch.optim.Adam(params, lr=1e-4)
    opt_g = torch.optim.Adam(params, lr=1e-4, capturable=True)
    opt_gf = torch.optim.Adam(params, lr=1e-4, capturable=True, fused=True)
    x_pix = torch.rand(SB, R, 2, generator=g).to(dev)
    c2w = torch.stack([bench.orbit_c2w(0.3 + 0.9 * b) for b in range(SB)]).to(dev)
    c2w = c2w.reshape(SB, 1, 4, 4).expand(SB, R, 4, 4)
    K = torch.tensor([[[1.0254, 0.0, 0.5], [0.0, 1.0254, 0.5], [0.0, 0.0, 1.0]]] * SB, device=dev)
    gt = torch.rand(SB, R, 3, generator=g).to(dev)

    def make_step(o):
        def step():
            rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
            loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
            o.zero_grad()
            loss.backward()
            o.step()
            return loss.detach()
        return step

    from avr.graphs import GraphedTrainStep
    runners = {}
    for a in arms:
        if a.startswith("graph:") or a.startswith("graphf:"):
            o = opt_gf if a.startswith("graphf:") else opt_g
            runners[a] = GraphedTrainStep(make_step(o), nets=[net], renderers=[rend], warmup=2)
        else:
            runners[a] = make_step(opt)

    def setenv(arm):
        arm = arm.split(":", 1)[1] if arm.startswith(("graph:", "graphf:")) else arm
        if arm in ("-", ""):
            return
        for kv in arm.split(","):
            k, v = kv.split("=", 1)
            os.environ[k] = v

    res = {a: [] for a in arms}
    host = {}
    for a in arms:
        setenv(a)
        for _ in range(5):
            runners[a]()
    torch.cuda.synchronize()
    for r in range(rounds):
        for a in arms:
            setenv(a)
            step = runners[a]
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                loss = step()
            t_host = time.perf_counter() - t0          # the host's enqueue time (the GPU may still be running)
            torch.cuda.synchronize()
            res[a].append((time.perf_counter() - t0) / steps * 1e3)
            host.setdefault(a, []).append(t_host / steps * 1e3)
        print(f"round {r}: " + "  ".join(f"{a}: {res[a][-1]:.3f} ms (host {host[a][-1]:.3f})" for a in arms),
              flush=True)
    assert bool(torch.isfinite(loss))
    for a in arms:
        print(f"{a}: median {statistics.median(res[a]):.3f} ms per step over {rounds} blocks of {steps} "
              f"({', '.join(f'{x:.3f}' for x in res[a])})")


if __name__ == "__main__":
    main()
