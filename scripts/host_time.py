"""Host (Python) time of the eager adaptive train.py step by phase (diagnostic): the HIP autograd Functions'
forward and backward wrapped with wall-clock accumulators (the backward runs on the autograd engine's device
thread, which cProfile does not see), plus the step's forward, backward and optimizer calls as a whole. Not part of
the product or the bench.  env: STEPS (default 40)."""
import collections
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
os.environ.setdefault("RENDERER", "adaptive")
os.environ["STEPS"] = "0"
import train_profile as tp  # noqa: E402

from avr import bn_train, field, layer_train, ops, renderers  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.defaultdict(int)


import cProfile  # noqa: E402
import pstats  # noqa: E402

PROF = cProfile.Profile() if os.environ.get("PROFILE_FN") else None   # e.g. PROFILE_FN=FieldTrain.backward or step_forward


def wrap(cls, name):
    for meth in ("forward", "backward"):
        fn = getattr(cls, meth)

        def timed(*a, _fn=fn, _k=f"{name}.{meth}", **k):
            t0 = time.perf_counter()
            try:
                if PROF is not None and _k == os.environ.get("PROFILE_FN") and PROFILING[0]:
                    return PROF.runcall(_fn, *a, **k)
                return _fn(*a, **k)
            finally:
                acc[_k] += time.perf_counter() - t0
                cnt[_k] += 1
        setattr(cls, meth, staticmethod(timed))


PROFILING = [False]


for cls, name in [(field._FieldTrain, "FieldTrain"), (renderers._MarchTrain, "MarchTrain"),
                  (ops._Composite, "Composite"), (ops._Depth, "Depth"), (ops._DepthOfPoints, "DepthOfPoints"),
                  (bn_train._FieldTrainBN, "FieldTrainBN"), (layer_train._FieldTrainLayers, "FieldTrainLayers")]:
    wrap(cls, name)

steps = int(os.environ.get("STEPS_H", "40"))
for _ in range(5):
    tp.step()
torch.cuda.synchronize()
acc.clear()
cnt.clear()
PROFILING[0] = True
phase = collections.defaultdict(float)
t_all = time.perf_counter()
for _ in range(steps):
    t0 = time.perf_counter()
    if PROF is not None and os.environ.get("PROFILE_FN") == "step_forward":   # the main thread's forward + loss
        PROF.enable()
    rgb_c, rgb_f, _, _ = tp.rend(tp.c2w, tp.K, tp.x_pix, tp.net)
    loss = ((rgb_c - tp.gt) ** 2).mean() + ((rgb_f - tp.gt) ** 2).mean()
    if PROF is not None and os.environ.get("PROFILE_FN") == "step_forward":
        PROF.disable()
    t1 = time.perf_counter()
    tp.opt.zero_grad()
    loss.backward()
    t2 = time.perf_counter()
    tp.opt.step()
    t3 = time.perf_counter()
    phase["forward + loss"] += t1 - t0
    phase["zero_grad + backward"] += t2 - t1
    phase["optimizer"] += t3 - t2
host = time.perf_counter() - t_all
torch.cuda.synchronize()
total = time.perf_counter() - t_all
print(f"{steps} steps: host {host / steps * 1e3:.3f} ms / step, with the GPU drained {total / steps * 1e3:.3f} ms")
for k, v in phase.items():
    print(f"  {k:24s} {v / steps * 1e3:8.3f} ms / step")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v / steps * 1e3:8.3f} ms / step ({cnt[k] // steps} calls)")
if PROF is not None:
    pstats.Stats(PROF).sort_stats("tottime").print_stats(30)
    pstats.Stats(PROF).sort_stats("cumulative").print_stats(45)
