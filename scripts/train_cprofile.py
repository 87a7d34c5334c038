"""Diagnostic: the host (Python) time of bench.py's --mode train step under cProfile, by own time -- for steps whose
GPU work is shorter than their launch path (the adaptive renderer's). Not part of the product or the bench.
env: RENDERER (adaptive | volume), CONF, CSTEPS, CALLERS (comma-separated function-name patterns whose callers to list)"""
import cProfile
import os
import pstats
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
os.environ.setdefault("RENDERER", "adaptive")
os.environ["STEPS"] = "0"
import train_profile as tp  # noqa: E402  (builds the scene, renderer and step; STEPS=0 profiles nothing there)

steps = int(os.environ.get("CSTEPS", "20"))
for _ in range(3):
    tp.step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    tp.step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(45)
for fn in os.environ.get("CALLERS", "").split(","):
    if fn:
        st.print_callers(fn)
