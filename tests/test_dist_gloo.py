"""Data-parallel logic on CPU: world_size 2 over gloo (no GPU needed).

Each rank trains the ORACLE step on its own swap group; the gradient bucket is
averaged with craniofacialsd_vae_amd.dist.GradientAverager (the same object the
GPU path uses, with a CPU scale routine).  Checks: the averaged gradient equals
the single-process mean of the per-group gradients, and parameters stay
bit-identical across ranks after Adam.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat(grads, names):
    return torch.cat([grads[n].reshape(-1) for n in names])


def _worker(rank, world, port, out_dir):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    import cfsd_loader
    import recipe
    from oracle import cfsd_oracle as O
    cfsd_loader.load()
    from craniofacialsd_vae_amd import dist as D
    w, r, _ = D.init_from_env(backend="gloo")
    assert (w, r) == (world, rank)
    topo = O.Topology(recipe.load_topology())
    weights = recipe.golden_weights()
    names = list(weights)
    P = O.make_params(weights)
    flat = torch.cat([P[n].detach().reshape(-1) for n in names])
    if rank == 1:
        flat.zero_()  # broadcast must restore rank 0's parameters
    D.broadcast_parameters(flat, 0)
    off = 0
    with torch.no_grad():
        for n in names:
            k = P[n].numel()
            P[n].copy_(flat[off:off + k].view_as(P[n]))
            off += k
    avg = D.GradientAverager(world=world, scale=lambda t, a: t.mul_(a))
    opt = O.Adam(P)
    meshes = recipe.normalized_meshes(12)
    lo, hi = D.shard_range(8, rank, world)  # 8 meshes -> 2 groups of 4
    assert hi - lo == 4
    x4 = meshes[lo:hi]
    for p in P.values():
        p.grad = None
    out = O.losses(P, torch.from_numpy(O.swap_features(x4, topo.region_features, 2)), topo, 2,
                   torch.from_numpy(recipe.train_eps(rank)))
    out["tot"].backward()
    g = _flat({n: P[n].grad for n in names}, names)
    local = g.clone()
    avg(g)
    off = 0
    grads = {}
    for n in names:
        k = P[n].numel()
        grads[n] = g[off:off + k].view_as(P[n])
        off += k
    opt.step(P, grads)
    params = torch.cat([P[n].detach().reshape(-1) for n in names])
    torch.save({"local": local, "avg": g, "params": params}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.slow
def test_two_rank_gradient_average(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    mean = (r0["local"] + r1["local"]) / 2
    np.testing.assert_allclose(r0["avg"].numpy(), mean.numpy(), rtol=1e-6, atol=1e-9)
    assert torch.equal(r0["avg"], r1["avg"])
    assert torch.equal(r0["params"], r1["params"])
    assert not torch.equal(r0["local"], r1["local"])  # the two groups differ


def test_shard_range_covers_everything():
    import sys
    sys.path.insert(0, ROOT)
    import cfsd_loader
    cfsd_loader.load()
    from craniofacialsd_vae_amd.dist import shard_range
    for n in (0, 1, 7, 8, 50000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _epoch_worker(rank, world, port, n_items, bs, out_dir):
    """One data-parallel epoch's collective sequence: per step one gradient
    all-reduce (the step's bucket), then the end-of-epoch loss all-reduce of a
    DIFFERENT size (manager.run_epoch).  Every rank runs
    dist.steps_per_epoch steps over its own shard_range shard."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import cfsd_loader
    cfsd_loader.load()
    from craniofacialsd_vae_amd.dist import shard_range, steps_per_epoch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n_items, rank, world)
    steps = steps_per_epoch(n_items, world, bs)
    assert 1 <= steps <= (hi - lo) // bs
    grad = torch.full((1000,), float(rank))
    for _ in range(steps):
        dist.all_reduce(grad)
    acc = torch.tensor([float(steps), 1.0, 2.0, 3.0, 4.0, 5.0])
    dist.all_reduce(acc)
    torch.save({"steps": steps, "acc0": float(acc[0]), "grad0": float(grad[0])},
               os.path.join(out_dir, f"e{rank}.pt"))
    dist.destroy_process_group()


def test_unequal_shards_run_equal_steps(tmp_path):
    """31 train meshes over 2 ranks = shards of 16 and 15,
    i.e. 4 and 3 batches of 4.  Both ranks must run 3 steps, or rank 0's 4th
    gradient all-reduce pairs with rank 1's 6-float loss all-reduce (gloo
    errors, RCCL hangs).  Also: the count is the smallest shard's for every
    size / world / bs."""
    import sys
    sys.path.insert(0, ROOT)
    import cfsd_loader
    cfsd_loader.load()
    from craniofacialsd_vae_amd.dist import shard_range, steps_per_epoch
    for n in range(0, 200, 7):
        for world in (1, 2, 3, 8):
            for bs in (1, 4, 5):
                spans = [shard_range(n, r, world) for r in range(world)]
                assert steps_per_epoch(n, world, bs) == min((h - l) // bs for l, h in spans)
    mp.spawn(_epoch_worker, args=(2, _free_port(), 31, 4, str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"e{i}.pt", weights_only=True) for i in range(2)]
    assert r[0]["steps"] == r[1]["steps"] == 3
    assert r[0]["acc0"] == r[1]["acc0"] == 6.0
