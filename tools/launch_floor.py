"""Launch floor inside a hipGraph on this box: N back-to-back tiny libcfsd
launches (cfsd_elu_bwd on 256 floats, one 256-thread workgroup) captured in one
graph; per-launch device time = replay time / N (measurement only)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for n_el in (256, 65536, 1 << 20):
        a = torch.randn(n_el, device=dev)
        y = torch.randn(n_el, device=dev)
        for n in (1, 40):
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                ops.elu_bwd(a, y, out=a)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    ops.elu_bwd(a, y, out=a)
            for _ in range(20):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            reps = 200
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(f"elements {n_el:8d}: graph of {n:3d} launches {ms * 1e3:8.2f} us per replay, "
                  f"{ms * 1e3 / n:6.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
