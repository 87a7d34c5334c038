"""Diagnostic: wall-clock host time per source line of the HIP training autograd Functions (avr.field._FieldTrain
forward / backward, avr.renderers._MarchTrain) over the eager adaptive train.py step of scripts/train_profile.py.
A line's time includes everything it calls; nested frames are not traced line by line. The backward runs on the
autograd engine's thread, so the tracer is installed inside the wrapped call. Not part of the product or the bench.
env: STEPS_H (default 40), TOP (default 25)."""
import collections
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "scripts"))
os.environ.setdefault("RENDERER", "adaptive")
os.environ["STEPS"] = "0"
import train_profile as tp  # noqa: E402

from avr import field, renderers  # noqa: E402

acc = collections.defaultdict(float)
hits = collections.defaultdict(int)
ON = [False]


def traced(outer):
    fn = getattr(outer, "__wrapped__", outer)   # avr.anomaly wraps the Functions' methods
    code = fn.__code__
    tag = f"{os.path.basename(code.co_filename)}:{code.co_name}"

    def local(frame, event, arg, state=[None, 0.0]):
        now = time.perf_counter()
        if state[0] is not None:
            acc[(tag, state[0])] += now - state[1]
            hits[(tag, state[0])] += 1
        state[0], state[1] = (frame.f_lineno, now) if event == "line" else (None, now)
        return local

    def glob(frame, event, arg):
        if event == "call" and frame.f_code is code:
            return local
        return None

    def wrapper(*a, **k):
        if not ON[0]:
            return outer(*a, **k)
        sys.settrace(glob)
        try:
            return outer(*a, **k)
        finally:
            sys.settrace(None)
    return staticmethod(wrapper)


for cls in (field._FieldTrain, renderers._MarchTrain):
    for meth in ("forward", "backward"):
        setattr(cls, meth, traced(getattr(cls, meth)))

for _ in range(5):
    tp.step()
torch.cuda.synchronize()
ON[0] = True
steps = int(os.environ.get("STEPS_H", "40"))
t0 = time.perf_counter()
for _ in range(steps):
    tp.step()
host = (time.perf_counter() - t0) / steps
ON[0] = False
print(f"{steps} steps (traced): host {host * 1e3:.3f} ms / step")
for (name, line), v in sorted(acc.items(), key=lambda kv: -kv[1])[:int(os.environ.get("TOP", "25"))]:
    print(f"  {v / steps * 1e6:8.1f} us/step  {hits[(name, line)] // steps:3d}x  {name}:{line}")
