"""Data-parallel HIP training step, two ranks sharing the one GPU of the test
box over gloo (RCCL itself needs one GPU per rank and runs in
the driver's multi-GPU bench).

Each rank runs ``SDVAEEngine.train_step_on(..., grad_hook=GradientAverager)``
on its own swap group -- the same bucketed, overlapped all-reduce object the
N>1 bench replays (two contiguous buckets started from inside the backward).
Rank 0 also trains both groups separately on single-rank engines.  Checks:
the averaged device gradient equals the mean of the two single-rank device
gradients (bit-exact: a sum of two fp32 values and a 0.5 scale are exact),
and the parameters after Adam are bit-identical across ranks.  The
justification for DP is that every loss term is intra-swap-group
(model_manager.py:360-393).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = r'''
import json, os, sys
ROOT = sys.argv[1]
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch, torch.distributed as dist
import cfsd_loader, recipe
from oracle import cfsd_oracle as O
cfsd_loader.load()
from craniofacialsd_vae_amd import engine as E, dist as D, ops, topology
world, rank, _ = D.init_from_env(backend="gloo")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
T = topology.DeviceTopology.from_npz(recipe.load_topology(), device=dev)
w = {k: torch.from_numpy(v) for k, v in recipe.golden_weights().items()}
meshes = recipe.normalized_meshes(8)
feats = O.Topology(recipe.load_topology()).region_features

def group(r, step):
    key = recipe.train_key_index(step + 3 * r)
    eps = torch.from_numpy(recipe.train_eps(step + 3 * r)).to(dev)
    x = torch.from_numpy(O.swap_features(meshes[4 * r:4 * r + 4], feats, key)).to(dev)
    return x, key, eps

eng = E.SDVAEEngine(T, E.ModelSpec(), device=dev)
if rank == 1:
    eng.params.data.zero_()
eng.load_state_dict(w) if rank == 0 else None
D.broadcast_parameters(eng.params.data, 0)
avg = D.GradientAverager(world)
res = {}
for step in range(2):
    x, key, eps = group(rank, step)
    b = eng.set_batch(x, key_index=key, eps=eps)
    eng.train_step_on(b, grad_hook=avg)
    torch.cuda.synchronize()
    g = eng.params.grad.cpu()
    p = eng.params.data.cpu()
    gs = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gs, p.clone())
    res[f"params_equal_{step}"] = all(torch.equal(gs[0], t) for t in gs)
    if rank == 0 and step == 0:
        singles = []
        for r in range(world):
            e1 = E.SDVAEEngine(T, E.ModelSpec(), device=dev)
            e1.load_state_dict(w)
            xr, kr, er = group(r, 0)
            e1.train_step_on(e1.set_batch(xr, key_index=kr, eps=er))
            torch.cuda.synchronize()
            singles.append(e1.params.grad.cpu())
        mean = (singles[0] + singles[1]) * 0.5
        res["grad_equal_mean"] = bool(torch.equal(g, mean))
        res["grad_max_abs_diff"] = float((g - mean).abs().max())
        res["grad_norm"] = float(mean.norm())
        res["groups_differ"] = not torch.equal(singles[0], singles[1])
if rank == 0:
    with open(sys.argv[2], "w") as f:
        json.dump(res, f)
dist.destroy_process_group()
'''


def test_dp2_hip_step_matches_single_rank_mean(tmp_path):
    wfile = tmp_path / "dp_worker.py"
    wfile.write_text(WORKER)
    out = tmp_path / "res.json"
    env = dict(os.environ, CFSD_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(wfile), ROOT, str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["groups_differ"]
    assert res["grad_equal_mean"], res
    assert res["params_equal_0"] and res["params_equal_1"], res
