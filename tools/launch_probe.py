"""Fixed cost of one launch inside a hipGraph on MI355X: N back-to-back
cfsd_scale launches over 1 / 64k floats, captured once and replayed; reports
microseconds per launch (the floor every separate kernel of the step pays)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import ops  # noqa: E402


def run(n_launch, numel, reps=200):
    y = torch.ones(numel, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            ops.scale(y, 1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n_launch):
            ops.scale(y, 1.0)
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / n_launch


for numel in (1, 65536):
    for n in (1, 10, 40):
        print(f"numel {numel:6d} launches/graph {n:3d}: {run(n, numel):6.2f} us per launch", flush=True)
