"""Host gaps of the data-parallel step structure on ONE GPU (measurement only).

The data-parallel TrainStep (step.py) replays three hipGraphs per step with
the two gradient all-reduce buckets issued from the host between them.  This
runs that exact structure in one process with a loopback averager (world 2
semantics: the buckets are issued and joined, the gradient is scaled by 1/2,
Adam is a separate launch -- but no bytes move), so a kernel trace shows the
graph-replay / join gaps the data-parallel step adds on top of the kernels,
without a second process sharing the GPU.  RCCL's own time is not in it.
usage: rocprofv3 --kernel-trace --stats -d <dir> -o dp -- python3 tools/dp_gaps.py [steps]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from craniofacialsd_vae_amd import dist as cdist  # noqa: E402
from craniofacialsd_vae_amd.step import TrainStep  # noqa: E402


class LoopbackAverager(cdist.GradientAverager):
    """GradientAverager with world-N bookkeeping and no communication."""

    def bucket_ready(self, view):
        pass

    def finish(self, grad):
        self.scale(grad, 1.0 / self.world)
        return grad


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    r = bench.Runner(1, 0, dev, 256, True)
    ts = TrainStep(r.eng, r.data, LoopbackAverager(2))
    ts.capture()
    for _ in range(10):
        ts.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ts.step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    # the single-GPU structure on the same engine, for comparison
    ts1 = TrainStep(r.eng, r.data, None)
    ts1.capture()
    ts1.capture_pair()
    ts1.run(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ts1.run(steps)
    torch.cuda.synchronize()
    el1 = (time.perf_counter() - t0) / steps
    print(f"dp-structure (3 graphs + host bucket calls, loopback) {el * 1e6:.1f} us/step; "
          f"single-GPU graph {el1 * 1e6:.1f} us/step; difference {(el - el1) * 1e6:.1f} us")


if __name__ == "__main__":
    main()
