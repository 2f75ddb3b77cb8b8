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


def _run2(tmp_path, script, *args):
    wfile = tmp_path / "dp_worker.py"
    wfile.write_text(script)
    out = tmp_path / "res.json"
    # both ranks on the one test GPU (CFSD_SHARE_DEVICE: the engine then avoids the
    # spin-waiting one-launch bottleneck, whose forward progress needs the device to itself)
    env = dict(os.environ, CFSD_DIST_BACKEND="gloo", CFSD_SHARE_DEVICE="1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(wfile), ROOT, str(out),
           *args]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads(out.read_text())


def test_dp2_hip_step_matches_single_rank_mean(tmp_path):
    res = _run2(tmp_path, WORKER)
    assert res["groups_differ"]
    assert res["grad_equal_mean"], res
    assert res["params_equal_0"] and res["params_equal_1"], res


# The step bench.py times at N > 1 (configuration C3): step.TrainStep with a
# GradientAverager, captured as three hipGraphs replayed around the two
# all-reduce buckets, trained from a resident, device-shuffled data shard.
GRAPH_WORKER = r'''
import json, os, sys
ROOT, OUT, PREC = sys.argv[1], sys.argv[2], sys.argv[3]
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch, torch.distributed as dist
import cfsd_loader, recipe
cfsd_loader.load()
from craniofacialsd_vae_amd import engine as E, dist as D, topology
from craniofacialsd_vae_amd.step import TrainStep
world, rank, _ = D.init_from_env(backend="gloo")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
T = topology.DeviceTopology.from_npz(recipe.load_topology(), device=dev)
w = {k: torch.from_numpy(v) for k, v in recipe.golden_weights().items()}
nv = T.n_verts[0]
meshes = torch.randn(16, nv, 3, generator=torch.Generator().manual_seed(99)).to(dev)

def make(r, perturb=False):
    eng = E.SDVAEEngine(T, E.ModelSpec(), seed=1234 + r, device=dev, precision=PREC)
    eng.load_state_dict(w)
    if perturb:  # rank 1 starts elsewhere: the broadcast must fix it
        eng.params.data.mul_(0.5)
    lo, hi = D.shard_range(16, r, world)
    data = E.ResidentData(meshes, bs=4, rows=torch.arange(lo, hi), shuffle=True)
    return eng, data

def state(eng):
    P = eng.params
    out = [P.data, P.grad, P.exp_avg, P.exp_avg_sq, P.step, eng.counter]
    if P.shadow is not None:
        out.append(P.shadow)
    return [t.detach().cpu().clone() for t in out]

def gather_equal(t):
    gs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gs, t.contiguous())
    return all(torch.equal(gs[0], x) for x in gs)

eng_g, data_g = make(rank, perturb=rank == 1)
D.broadcast_parameters(eng_g.params.data, 0)
eng_g.sync_shadow()
ts = TrainStep(eng_g, data_g, D.GradientAverager(world))
eng_e, data_e = make(rank)
avg_e = D.GradientAverager(world)
b_e = eng_e.buffers(16)
res = {"steps": []}
ts.capture()                       # step 1 runs eagerly inside capture()
eng_e.resident_step(b_e, data_e, acc=eng_e.loss_acc, grad_hook=avg_e)
torch.cuda.synchronize()
g1 = eng_g.params.grad.detach().cpu().clone()
for step in range(1, 4):
    if step > 1:
        ts.step()                  # graph replays
        eng_e.resident_step(b_e, data_e, acc=eng_e.loss_acc, grad_hook=avg_e)
        torch.cuda.synchronize()
    sg, se = state(eng_g), state(eng_e)
    names = ["data", "grad", "exp_avg", "exp_avg_sq", "step", "counter", "shadow"]
    rec = {"graph_equals_eager": all(torch.equal(a, b) for a, b in zip(sg, se)),
           "differs": [(n, float((a.double() - b.double()).abs().max()), int((a != b).sum()))
                       for n, a, b in zip(names, sg, se) if not torch.equal(a, b)],
           "params_equal_ranks": gather_equal(eng_g.params.data.cpu()),
           "moments_equal_ranks": gather_equal(eng_g.params.exp_avg_sq.cpu()),
           "batch_idx": ts.b.batch_idx.cpu().tolist()}
    if eng_g.params.shadow is not None:
        rec["shadow_equal_ranks"] = gather_equal(eng_g.params.shadow.float().cpu())  # exact widening (gloo has no 16-bit types)
        rec["shadow_is_cast"] = bool(torch.equal(eng_g.params.shadow.cpu(),
                                                 eng_g.params.data.cpu().to(torch.bfloat16)))
    rec["losses_finite"] = bool(torch.isfinite(eng_g.loss_acc).all())
    res["steps"].append(rec)
rows = [torch.tensor(s["batch_idx"]) for s in res["steps"]]
res["rows_in_shard"] = all(((r >= D.shard_range(16, rank, world)[0]) &
                            (r < D.shard_range(16, rank, world)[1])).all().item() for r in rows)
if rank == 0:
    singles = []
    for r in range(world):
        e1, d1 = make(r)
        t1 = TrainStep(e1, d1)       # single GPU: Adam fused into the reduce
        t1.step()
        torch.cuda.synchronize()
        singles.append(e1.params.grad.cpu())
    mean = (singles[0] + singles[1]) * 0.5
    res["grad_equal_mean"] = bool(torch.equal(g1, mean))
    res["grad_max_abs_diff"] = float((g1 - mean).abs().max())
    res["groups_differ"] = not torch.equal(singles[0], singles[1])
    with open(OUT, "w") as f:
        json.dump(res, f)
dist.barrier()
dist.destroy_process_group()
'''


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_dp2_graph_trainstep(tmp_path, precision):
    """C3 path: 2 ranks x 16 meshes, graph-replayed TrainStep (the object the
    N > 1 bench replays) -- (1) the averaged gradient of the first step is
    bit-equal to the mean of the two single-GPU gradients of the same batches;
    (2) after every step parameters, Adam moments and the bf16 shadows are
    bit-identical across ranks; (3) every graph-replayed step is bit-identical
    to the eager ``resident_step(grad_hook=GradientAverager)`` step
    (train_step_on's overlapped buckets) -- parameters, gradient, moments,
    Adam t, device counter, shadow; (4) each rank only draws its shard."""
    res = _run2(tmp_path, GRAPH_WORKER, precision)
    assert res["groups_differ"]
    assert res["grad_equal_mean"], res
    assert res["rows_in_shard"], res
    for i, s in enumerate(res["steps"]):
        assert s["graph_equals_eager"], (i, s)
        assert s["params_equal_ranks"] and s["moments_equal_ranks"], (i, s)
        assert s["losses_finite"], (i, s)
        if precision == "bf16":
            assert s["shadow_equal_ranks"] and s["shadow_is_cast"], (i, s)


def test_bench_line_self_verifies_at_world2(tmp_path):
    """bench.py's N > 1 line carries its own evidence:
    the process group's world size and backend, every rank's PCI id, per-rank
    ms per step, and ``ranks_in_sync`` -- bit checksums of parameters,
    gradient, Adam moments and t equal on every rank after the timed steps.
    Rehearsed with 2 gloo ranks sharing the test GPU (the driver's 8-GPU run
    uses RCCL, one GPU per rank: ``distinct_devices`` then holds)."""
    env = dict(os.environ, CFSD_DIST_BACKEND="gloo", CFSD_SHARE_DEVICE="1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "2", "--dataset", "32", "--no-cpu", "--no-extras"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    out = json.loads(lines[0])
    dc = out["dist_check"]
    assert out["n_gpus"] == 2 and dc["world_size"] == 2 and dc["backend"] == "gloo"
    assert dc["shared_device_rehearsal"] and len(dc["pci_bus_ids"]) == 2
    assert dc["ranks_in_sync"], dc
    assert dc["checksums_rank0"]["adam_t"] == 1 + 2 + 4  # capture step + warmup + timed
    assert 0 < dc["ms_per_step_min"] <= dc["ms_per_step_max"] <= out["ms_per_step"] * 1.0001
