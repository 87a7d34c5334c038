"""Diagnostic: which operations of bench.py's --mode train step synchronise the host with the GPU
(torch.cuda.set_sync_debug_mode("warn") over two steps, each warning with the stack of the call that made it).
env: RENDERER (adaptive | volume), CONF. Not part of the product or the bench."""
import os
import sys
import traceback
import warnings

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
os.environ.setdefault("RENDERER", "adaptive")
os.environ["STEPS"] = "0"
import train_profile as tp  # noqa: E402

for _ in range(3):
    tp.step()
torch.cuda.synchronize()
seen = {}


def show(message, category, filename, lineno, file=None, line=None):
    stack = "".join(traceback.format_stack(limit=12)[:-2])
    key = stack
    seen[key] = seen.get(key, 0) + 1
    if seen[key] == 1:
        print(f"---- {message}\n{stack}", flush=True)


warnings.showwarning = show
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
for _ in range(2):
    tp.step()
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
print(f"{len(seen)} distinct synchronising call sites, {sum(seen.values())} calls in 2 steps")
