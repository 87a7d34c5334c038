"""Which parameters of the adaptive train step differ between eager steps and a captured step (probe)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "adaptive-volume-rendering_amd"))
from test_gpu_poison import _setup  # noqa: E402
from avr.graphs import GraphedTrainStep  # noqa: E402

fused = os.environ.get("FUSED", "1") == "1"
res = []
for graphed in (False, True):
    net, rend, named, (c2w, K, x_pix, gt), _ = _setup("adaptive", False)
    opt = torch.optim.Adam([p for _, p in named], lr=1e-4, capturable=True, fused=fused)

    def step():
        rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
        loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss
    run = GraphedTrainStep(step, nets=[net], renderers=[rend], warmup=2) if graphed else step
    torch.manual_seed(123)
    losses = [float(run()) for _ in range(3)]
    grads = {n: (None if p.grad is None else p.grad.detach().clone()) for n, p in named}
    res.append((losses, {n: p.detach().clone() for n, p in named}, grads,
                {n: {k: v.clone() for k, v in opt.state[p].items()} for n, p in named if p in opt.state}))
(le, pe, ge, se), (lg, pg, gg, sg) = res
print("fused", fused, "losses", le, lg)
d = sorted(((float((pe[n] - pg[n]).abs().max()), n) for n in pe), reverse=True)
print("param diffs", d[:8])
print("grad None differ:", sorted(set(n for n in ge if ge[n] is None) ^ set(n for n in gg if gg[n] is None)))
gd = sorted(((float((ge[n] - gg[n]).abs().max()), n) for n in ge if ge[n] is not None and gg[n] is not None), reverse=True)
print("grad diffs", gd[:8])
for n in list(se)[:3] + [x[1] for x in d[:3]]:
    if n in se and n in sg:
        print(n, {k: (float((se[n][k].float() - sg[n][k].float()).abs().max()) if torch.is_tensor(se[n][k]) else None)
                  for k in se[n]}, "step", se[n].get("step"), sg[n].get("step"))
