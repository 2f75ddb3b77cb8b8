"""BASELINE configurations C3 and C5 at their stated sizes, and RCCL itself.

* C5 (``configs[4]``): the training set is 50 000 spectral-interpolation
  meshes (``data_loading.py:292-374``, ``utils.py:238-267``), resident in HBM:
  50 000 x 17 039 x 3 = 2.56e9 fp32 elements, more than 2^31.  Three bf16
  steps over the whole set and three over the last eighth of it (the shard
  rank 7 of 8 trains: every picked mesh starts past element 2^31) -- each
  step's swapped batch must equal the host gather of the picked indices run
  through the oracle's swap (``swap_batch_transform.py:13-42``).
* C3 (``configs[2]``): 8 ranks x 16 meshes = 128 meshes per step in bf16,
  rehearsed as eight gloo ranks sharing the one test GPU, through
  ``TrainStep``'s data-parallel graphs.  Parameters, Adam moments and bf16
  shadows bit-identical on every rank after each step; the averaged gradient
  equal to the mean of the eight single-rank gradients within the bound of
  fp32 summation in any order (gloo's reduction order is its own).
* RCCL: a one-rank ``nccl`` process group forcing the data-parallel step
  (``GradientAverager(always=True)``): RCCL's all-reduce runs, captured INTO
  the step graph (and the multi-step graph), and every step is bit-equal to
  the single-process step (Adam fused into the reduce) and to the
  three-graph structure with host-issued all-reduces.
The per-rank step these stand for is ``model_manager.py:257-326``.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, script, nproc, *args, env_extra=None, timeout=600):
    wfile = tmp_path / "worker.py"
    wfile.write_text(script)
    out = tmp_path / "res.json"
    # (nproc > 1: every rank on the one test GPU -- the engine then avoids the
    # spin-waiting one-launch bottleneck, whose forward progress needs the device to itself)
    env = dict(os.environ, OMP_NUM_THREADS="1", **({"CFSD_SHARE_DEVICE": "1"} if nproc > 1 else {}),
               **(env_extra or {}))
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(wfile), ROOT, str(out), *args]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:  # the first error lines (a C++ exception's what() precedes its long trace)
        errs = [ln for ln in (r.stdout + r.stderr).splitlines()
                if any(k in ln for k in ("Error", "error", "what()", "Exception", "failed"))][:20]
        raise AssertionError("\n".join(errs) + "\n---\n" + r.stderr[-2000:])
    return json.loads(out.read_text())


# ----------------------------------------------------------------------- C5
def test_c5_50k_resident_set_bf16(otopo):
    """>= 3 bf16 TrainStep steps on a resident 50 000-mesh augmented set
    (> 2^31 fp32 elements); every picked batch equals the host gather."""
    import torch

    import bench
    from craniofacialsd_vae_amd import engine as E
    from craniofacialsd_vae_amd.step import TrainStep
    from oracle import cfsd_oracle as O
    dev = torch.device("cuda", 0)
    n = 50_000
    meshes, norm, info = bench.augmented_set(n, dev, seed=77)
    assert info["finite"] and meshes.shape == (n, 17039, 3)
    assert meshes.numel() > 2 ** 31
    topo = bench.load_topology("craniofacial", dev)
    eng = E.SDVAEEngine(topo, E.ModelSpec(latent_size=75), swap_bs=4, seed=5, device=dev, precision="bf16")
    eng.reset_parameters()
    data = E.ResidentData(meshes, bs=4, shuffle=True, norm=norm, inplace=True)
    del meshes
    assert data.meshes.numel() > 2 ** 31
    feats = otopo.region_features
    p0 = eng.params.data.clone()

    def check(ts, steps, run):
        picks = []
        for k in range(steps):
            run(ts, k)
            torch.cuda.synchronize()
            idx = ts.b.batch_idx.cpu().numpy().astype(np.int64)
            key = int(ts.b.key.item())
            host4 = np.stack([data.meshes[int(i)].cpu().numpy() for i in idx])  # torch's own copies
            want = O.swap_features(host4, feats, key)
            got = ts.b.x.cpu().numpy()
            assert np.array_equal(got, want), (k, idx.tolist(), key)
            assert torch.isfinite(eng.loss_acc).all()
            picks.append(idx.tolist())
        return picks

    ts = TrainStep(eng, data)
    ts.capture()                                  # step 1: eager, inside capture()
    picks = check(ts, 3, lambda t, k: t.step() if k else None)
    picks += check(ts, 1, lambda t, k: t.step())
    # the last eighth of the set (the shard rank 7 of 8 trains): every
    # element offset of every picked mesh is past 2^31
    lo = 7 * n // 8
    assert lo * 17039 * 3 > 2 ** 31
    tail = E.ResidentData(data.meshes, bs=4, rows=torch.arange(lo, n), shuffle=True)
    ts2 = TrainStep(eng, tail)
    ts2.capture()
    picks2 = check(ts2, 3, lambda t, k: t.step() if k else None)
    assert all(lo <= i < n for p in picks2 for i in p), picks2
    assert max(i for p in picks for i in p) < n
    assert int(eng.params.step.item()) == 7
    assert torch.isfinite(eng.params.data).all() and not torch.equal(eng.params.data, p0)
    assert torch.equal(eng.params.shadow, eng.params.data.to(torch.bfloat16))


# ----------------------------------------------------------------------- C3
C3_WORKER = r'''
import json, os, sys
ROOT, OUT = sys.argv[1], sys.argv[2]
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
nv = T.n_verts[0]
PER = 16
meshes = torch.randn(PER * world, nv, 3, generator=torch.Generator().manual_seed(7)).to(dev)

def make(r):
    eng = E.SDVAEEngine(T, E.ModelSpec(), seed=1234 + r, device=dev, precision="bf16")
    eng.reset_parameters()   # same init on every rank (seeded); broadcast below anyway
    lo, hi = D.shard_range(PER * world, r, world)
    return eng, E.ResidentData(meshes, bs=4, rows=torch.arange(lo, hi), shuffle=True)

def gather_equal(t):
    gs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gs, t.contiguous())
    return all(torch.equal(gs[0], x) for x in gs)

eng, data = make(rank)
if rank:
    eng.params.data.mul_(0.5)          # the broadcast must fix this
D.broadcast_parameters(eng.params.data, 0)
eng.sync_shadow()
p_init = eng.params.data.clone()
ts = TrainStep(eng, data, D.GradientAverager(world))
res = {"world": world, "backend": dist.get_backend(), "one_graph": ts.one_graph, "steps": []}
ts.capture()                           # step 1 runs eagerly inside capture()
torch.cuda.synchronize()
g1 = eng.params.grad.detach().cpu().clone()
for step in range(1, 4):
    if step > 1:
        ts.step()
        torch.cuda.synchronize()
    P = eng.params
    res["steps"].append({
        "params_equal_ranks": gather_equal(P.data.cpu()),
        "exp_avg_equal_ranks": gather_equal(P.exp_avg.cpu()),
        "exp_avg_sq_equal_ranks": gather_equal(P.exp_avg_sq.cpu()),
        "shadow_equal_ranks": gather_equal(P.shadow.float().cpu()),
        "shadow_is_cast": bool(torch.equal(P.shadow.cpu(), P.data.cpu().to(torch.bfloat16))),
        "finite": bool(torch.isfinite(eng.loss_acc).all() and torch.isfinite(P.data).all()),
        "batch_idx": ts.b.batch_idx.cpu().tolist()})
lo, hi = D.shard_range(PER * world, rank, world)
rows = [i for s in res["steps"] for i in s["batch_idx"]]
res["rows_in_shard"] = all(lo <= i < hi for i in rows)
res["all_rows_in_shard"] = [None] * world
dist.all_gather_object(res["all_rows_in_shard"], res["rows_in_shard"])
if rank == 0:
    singles = []
    for r in range(world):
        e1, d1 = make(r)
        e1.params.data.copy_(p_init)
        e1.sync_shadow()
        t1 = TrainStep(e1, d1)       # one GPU, Adam fused into the reduce
        t1.step()
        torch.cuda.synchronize()
        singles.append(e1.params.grad.cpu().double())
        del t1, e1, d1
    S = torch.stack(singles)
    mean = S.sum(0) / world
    # fp32 sum of `world` terms in any order: |err| <= (world - 1) u sum|g_r|,
    # the 1/world scale is exact (power of two)
    bound = (world - 1) * 2.0 ** -24 * S.abs().sum(0) / world
    err = (g1.double() - mean).abs()
    res["grad_within_sum_bound"] = bool((err <= bound).all())
    res["grad_max_abs_err"] = float(err.max())
    res["grad_max_rel_err"] = float((err / mean.abs().clamp_min(1e-30)).max())
    res["grad_bitequal_frac"] = float((g1.double() == mean).double().mean())
    res["groups_differ"] = not torch.equal(singles[0], singles[1])
    with open(OUT, "w") as f:
        json.dump(res, f)
dist.barrier()
dist.destroy_process_group()
'''


def test_c3_eight_ranks_bf16(tmp_path):
    """C3: 8 ranks x 16 meshes (128 per step), bf16, TrainStep's DP graphs."""
    res = _run(tmp_path, C3_WORKER, 8, env_extra={"CFSD_DIST_BACKEND": "gloo"})
    assert res["world"] == 8 and res["backend"] == "gloo" and not res["one_graph"]
    assert res["groups_differ"]
    assert res["grad_within_sum_bound"], res
    assert all(res["all_rows_in_shard"]), res
    for i, s in enumerate(res["steps"]):
        for k in ("params_equal_ranks", "exp_avg_equal_ranks", "exp_avg_sq_equal_ranks", "shadow_equal_ranks",
                  "shadow_is_cast", "finite"):
            assert s[k], (i, k, s)


# ----------------------------------------------------------------------- RCCL
RCCL_WORKER = r'''
import json, os, sys
ROOT, OUT, PREC = sys.argv[1], sys.argv[2], sys.argv[3]
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch, torch.distributed as dist
import cfsd_loader, recipe
cfsd_loader.load()
from craniofacialsd_vae_amd import engine as E, dist as D, topology
from craniofacialsd_vae_amd.step import TrainStep
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
T = topology.DeviceTopology.from_npz(recipe.load_topology(), device=dev)
nv = T.n_verts[0]
meshes = torch.randn(32, nv, 3, generator=torch.Generator().manual_seed(3)).to(dev)

P0 = []

def make():
    eng = E.SDVAEEngine(T, E.ModelSpec(), seed=99, device=dev, precision=PREC)
    eng.reset_parameters()
    if P0:
        eng.params.data.copy_(P0[0])
        eng.sync_shadow()
    else:
        P0.append(eng.params.data.clone())
    return eng, E.ResidentData(meshes, bs=4, shuffle=True)

def state(eng):
    P = eng.params
    out = [P.data, P.grad, P.exp_avg, P.exp_avg_sq, P.step, eng.counter]
    if P.shadow is not None:
        out.append(P.shadow)
    return [t.detach().cpu().clone() for t in out]

import craniofacialsd_vae_amd.step as S
real_graph = torch.cuda.graph

class RefusingGraph:  # a backend that refuses the first capture (the fallback path)
    calls = 0
    def __init__(self, *a, **k):
        self.inner = real_graph(*a, **k)
    def __enter__(self):
        RefusingGraph.calls += 1
        if RefusingGraph.calls == 1:
            raise RuntimeError("simulated: collective not capturable")
        return self.inner.__enter__()
    def __exit__(self, *exc):
        return self.inner.__exit__(*exc)

runs = {}
for mode in ("single", "rccl_one_graph", "rccl_three_graphs", "rccl_fallback"):
    eng, data = make()
    avg = None if mode == "single" else D.GradientAverager(1, always=True)
    ts = TrainStep(eng, data, avg)
    ts.steps_per_graph = 4
    if mode == "rccl_three_graphs":
        ts.one_graph = False
    S.torch.cuda.graph = RefusingGraph if mode == "rccl_fallback" else real_graph
    ts.capture()                     # step 1 (eager, RCCL communicator warm)
    S.torch.cuda.graph = real_graph
    ts.step()                        # step 2: one replay
    ts.run(8)                        # steps 3-10: multi-step graph (one-graph modes)
    torch.cuda.synchronize()
    runs[mode] = {"state": state(eng), "one_graph": ts.one_graph, "dp": ts.avg is not None,
                  "multi": ts.graph_multi is not None, "loss_acc": eng.loss_acc.cpu().clone(),
                  "fallback": ts.fallback}
names = ["data", "grad", "exp_avg", "exp_avg_sq", "step", "counter", "shadow"]
res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
try:
    res["nccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
except Exception as e:  # version query only
    res["nccl_version"] = repr(e)
with open("/proc/self/maps") as f:
    res["rccl_libs"] = sorted({ln.split()[-1] for ln in f if "rccl" in ln.split()[-1]})
for mode in ("rccl_one_graph", "rccl_three_graphs", "rccl_fallback"):
    a, s = runs[mode], runs["single"]
    res[mode] = {"one_graph": a["one_graph"], "dp": a["dp"], "multi": a["multi"], "fallback": a["fallback"],
                 "equal_single": all(torch.equal(x, y) for x, y in zip(a["state"], s["state"])),
                 "differs": [n for n, x, y in zip(names, a["state"], s["state"]) if not torch.equal(x, y)],
                 "loss_equal": bool(torch.equal(a["loss_acc"], s["loss_acc"]))}
res["adam_t"] = int(runs["single"]["state"][4].item())
with open(OUT, "w") as f:
    json.dump(res, f)
dist.destroy_process_group()
'''


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_rccl_world1_dp_step_bitequal(tmp_path, precision):
    """RCCL executes: a one-rank nccl group running TrainStep's data-parallel
    structure with the bucket all-reduces captured into the step graph and the
    16-step graph; bit-equal to the single-process step after 10 steps."""
    res = _run(tmp_path, RCCL_WORKER, 1, precision)
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["rccl_libs"], "librccl not mapped"
    assert res["adam_t"] == 10
    one, three = res["rccl_one_graph"], res["rccl_three_graphs"]
    assert one["dp"] and one["one_graph"] and one["multi"], one
    assert three["dp"] and not three["one_graph"], three
    assert one["equal_single"] and one["loss_equal"], one
    assert three["equal_single"] and three["loss_equal"], three
    fb = res["rccl_fallback"]  # a refused capture falls back to the three-graph structure
    assert fb["dp"] and not fb["one_graph"] and "simulated" in (fb["fallback"] or ""), fb
    assert fb["equal_single"] and fb["loss_equal"], fb
