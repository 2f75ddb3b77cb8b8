"""Benchmark: SD-VAE training throughput (meshes/s) on MI355X.

Workload (BASELINE.json config 2, ``configurations/craniofacial.yaml``): the
real craniofacial template hierarchy (17039/4260/1065/267/67 vertices,
spiral length 9, channels [32, 32, 32, 64], latent 75, VAE), batch_size 4
swapped to 16 meshes per GPU per step, fp32.  A step is the full reference
``_do_iteration``: device-side batch pick + swap key + VAE noise, feature
swap, forward, MSE + Laplacian + KL + latent-consistency losses, backward,
(RCCL all-reduce of the flat gradient when N > 1), Adam.  The dataset is
synthetic N(0, 1) meshes resident in HBM (no checkpoint/dataset egress).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(for N > 1 launch with torch.distributed.run, one rank per GPU).
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import engine as E  # noqa: E402
from craniofacialsd_vae_amd import ops, topology  # noqa: E402

METRIC = "train meshes/sec + per-vertex L1, craniofacial SD-VAE @1/2/4/8 MI355X"
TOPO_NPZ = os.path.join(ROOT, "tests", "golden", "topology_craniofacial.npz")
PROFILES = os.path.join(ROOT, "profiles")
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--dataset", type=int, default=256, help="resident synthetic meshes per rank")
    p.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample budget")
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


class Runner:
    def __init__(self, world, rank, device, n_meshes, use_graph):
        npz = dict(np.load(TOPO_NPZ))
        self.topo = topology.DeviceTopology.from_npz(npz, device=device)
        self.eng = E.SDVAEEngine(self.topo, E.ModelSpec(), lr=1e-4, swap_bs=4, seed=1234 + rank,
                                 device=device)
        g = torch.Generator(device="cpu").manual_seed(0)
        self.eng.reset_parameters()  # same init on every rank (broadcast below)
        self.world, self.rank = world, rank
        nv = self.topo.n_verts[0]
        gen = torch.Generator(device=device).manual_seed(1234 + rank)
        self.data = torch.randn(n_meshes, nv, 3, device=device, generator=gen)
        self.n_batches = n_meshes // 4
        perm = torch.randperm(n_meshes, generator=g)[: self.n_batches * 4]
        self.perm = perm.to(torch.int32).to(device)
        self.b = self.eng.buffers(16)
        if world > 1:
            dist.broadcast(self.eng.params.data, 0)
        self.use_graph = use_graph
        self.graph_fwdbwd = self.graph_adam = None

    # --- the step, split where the collective goes
    def part_a(self):
        eng, b, T = self.eng, self.b, self.topo
        ops.step_begin(eng._step_counter(b), eng.seed, eps=b.eps, key=b.key,
                       n_regions=T.n_regions, batch_idx=b.batch_idx, bs=4,
                       n_batches=self.n_batches, perm=self.perm, adam_step=eng.params.step)
        ops.swap_features(self.data, b.batch_idx, T.region_mask, b.key, 4, out=b.x)
        eng.forward(b, train=True, acc=eng.loss_acc, finalize=False)
        eng.backward(b)

    def part_b(self):
        self.eng.adam_step()

    def allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.eng.params.grad)
            ops.scale(self.eng.params.grad, 1.0 / self.world)

    def capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.part_a()
                self.allreduce()
                self.part_b()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self.world == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.part_a()
                self.part_b()
            self.graph_fwdbwd, self.graph_adam = g, None
        else:
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga):
                self.part_a()
            with torch.cuda.graph(gb):
                self.part_b()
            self.graph_fwdbwd, self.graph_adam = ga, gb

    def step(self):
        if self.graph_fwdbwd is not None:
            self.graph_fwdbwd.replay()
            if self.graph_adam is not None:
                self.allreduce()
                self.graph_adam.replay()
        else:
            self.part_a()
            self.allreduce()
            self.part_b()


def kernel_probe(runner, n_iter=20):
    """Per-kernel device time of the dominant kernels, HIP events on the
    launch stream (eager replays of the same step, same inputs)."""
    eng, b, T = runner.eng, runner.b, runner.topo
    st = torch.cuda.current_stream()
    res = {}

    def timed(name, fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(n_iter):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / n_iter * 1e-3  # seconds per launch

    dec = eng.spec.dec_layers()
    i3 = len(dec) - 1
    w3, bias3 = eng._dec_w(i3)
    timed("conv_fwd_D3", lambda: ops.spiral_conv_fwd(b.dec_up[i3], T.spiral[0], w3, bias3, 1,
                                                      out=b.dec_out[i3]))
    # the D3 backward kernels exactly as the step launches them (dx with the
    # previous Deblock's ELU folded in is the Pool transpose's input here;
    # dW deferred: slab kernel only, reduced by the batched reduce)
    timed("conv_dx_D3", lambda: ops.spiral_conv_bwd_data(b.dpre_dec[i3], T.spiral_inv[0], w3, T.n_verts[0],
                                                         out=b.g_dec_up[i3], workspace=b.ws))
    timed("conv_dw_D3", lambda: ops.spiral_conv_bwd_weight(b.dec_up[i3], T.spiral[0], b.dpre_dec[i3], None,
                                                           None, b.ws_dw[("dec", i3)]))
    g = torch.empty(16, T.n_verts[0], 9 * 32, device=b.x.device)
    timed("spiral_gather_L0", lambda: ops.spiral_gather(b.dec_up[i3], T.spiral[0], out=g))
    del g
    return res


def pmc_traffic(key="conv_fwd_d3"):
    """HBM bytes per launch of a D3 kernel from the newest committed PMC pass
    (tools/gpu_round.sh -> tools/pmc_traffic.py: FETCH_SIZE and WRITE_SIZE in
    separate rocprofv3 runs, gfx950 FETCH_SIZE x2 correction)."""
    import glob
    files = sorted(glob.glob(os.path.join(PROFILES, f"*_pmc_traffic_{key}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def c1_parity(device):
    """The metric's second half: per-vertex L1 of C1 (encode + decode of the
    first 8 demo meshes, eval mode, golden weights) through the HIP path
    against the reconstructions the reference's own model.py produced
    (tests/golden/golden_eval.npz, made by tests/golden/make_golden.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import recipe
    npz = dict(np.load(TOPO_NPZ))
    topo = topology.DeviceTopology.from_npz(npz, device=device)
    eng = E.SDVAEEngine(topo, E.ModelSpec(), device=device)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in recipe.golden_weights().items()})
    b = eng.set_batch(torch.from_numpy(recipe.normalized_meshes(8)).to(device))
    eng.forward(b, train=False)
    torch.cuda.synchronize()
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden_eval.npz"))
    # per-vertex L1 by the device kernel (cfsd_vertex_errors, l1 term)
    _, l1 = ops.vertex_errors(b.out.contiguous(), torch.from_numpy(g["recon"]).to(device),
                              want_l1=True)
    d = l1.cpu().numpy()
    return {"config": "C1: demo encode+decode, 8 meshes, eval (z = mu), golden weights",
            "reference": "tests/golden/golden_eval.npz (reference model.py run in the build container)",
            "l1_kernel": "cfsd_vertex_errors",
            "max_vertex_l1": float(d.max()), "mean_vertex_l1": float(d.mean()),
            "z_max_abs_diff": float(np.abs(b.z.cpu().numpy() - g["z"]).max()),
            "tolerance": 1e-4, "pass": bool(d.max() <= 1e-4)}


def cpu_baseline(budget_s):
    """Oracle (PyTorch-CPU restatement of the reference step) on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle import cfsd_oracle as O
    npz = dict(np.load(TOPO_NPZ))
    T = O.Topology(npz)
    import recipe
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    P = O.make_params(recipe.golden_weights())
    opt = O.Adam(P)
    rs = np.random.RandomState(0)
    x4 = rs.randn(4, T.n_verts[0], 3).astype(np.float32)
    eps = rs.randn(16, 75).astype(np.float32)
    O.train_step(P, opt, x4, T, 0, eps)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        O.train_step(P, opt, x4, T, n % 15, eps)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    return {"value": 16 * n / el, "unit": "meshes/s", "cores": threads, "kind": "port",
            "sample": f"{n} full train steps (16 swapped meshes each, fp32, oracle/cfsd_oracle.py "
                      f"torch-CPU restatement) in {el:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for the N>1 path on a one-GPU box (default off: RCCL,
    # one GPU per rank): CFSD_DIST_BACKEND=gloo CFSD_SHARE_DEVICE=1.
    backend = os.environ.get("CFSD_DIST_BACKEND", "nccl")
    if os.environ.get("CFSD_SHARE_DEVICE"):
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    runner = Runner(world, rank, device, args.dataset, not args.no_graph)
    if runner.use_graph:
        runner.capture()
    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    meshes = 16 * world * args.steps
    losses = runner.eng.loss_acc.cpu().numpy()
    finite = bool(np.isfinite(losses).all())
    probe = kernel_probe(runner)
    if rank == 0:
        nv = runner.topo.n_verts[0]
        # dominant kernel: fused gather+contraction of D3 (32 -> 32, 17039 rows x 16)
        flops = 2.0 * 16 * nv * 9 * 32 * 32
        gather_bytes = 16 * nv * (32 + 9 * 32) * 4 + nv * 9 * 4
        t_g = probe["spiral_gather_L0"]
        parity = c1_parity(device)
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline(args.cpu_seconds)  # N=1 only
        # the three D3 (decoder level 0, 32 -> 32) conv kernels, 5.02 GFLOP
        # each; `roofline` is the dominant one (longest launch)
        d3 = {}
        for name, key in (("conv_fwd_D3", "conv_fwd_d3"), ("conv_dx_D3", "conv_dx_d3"),
                          ("conv_dw_D3", "conv_dw_d3")):
            t = probe[name]
            traffic, traffic_src = pmc_traffic(key)
            d3[name] = {"us_per_launch": t * 1e6, "achieved": flops / t / 1e12,
                        "frac": flops / t / 1e12 / FP32_PEAK_TFLOPS, "traffic": traffic,
                        "traffic_source": traffic_src}
        dom = max(d3, key=lambda k: d3[k]["us_per_launch"])
        kern_names = {"conv_fwd_D3": "conv_fwd_mfma<32,32> (decoder level 0 forward)",
                      "conv_dx_D3": "conv_dx_mfma<32,32> (decoder level 0 data gradient)",
                      "conv_dw_D3": "conv_dw_mfma<32,32> (decoder level 0 weight gradient)"}
        out = {
            "metric": METRIC, "value": meshes / el, "unit": "meshes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic N(0,1) meshes resident in HBM, random-init weights",
            "config": {"workload": "craniofacial.yaml SD-VAE train step (swap bs 4->16, fwd, "
                                   "MSE+Laplacian+KL+latent-consistency, bwd, Adam)",
                       "template_vertices": nv, "levels": runner.topo.n_verts,
                       "global_batch": 16 * world, "per_gpu_batch": 16,
                       "parallelism": f"dp{world}", "graph": runner.use_graph,
                       "collective": None if world == 1 else ("rccl all_reduce" if backend == "nccl" else backend)},
            "roofline": {"kernel": "cfsd " + kern_names[dom], "bound": "mfma",
                         "achieved": d3[dom]["achieved"], "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": d3[dom]["frac"],
                         "traffic": d3[dom]["traffic"], "traffic_source": d3[dom]["traffic_source"],
                         "algorithmic_flop": flops, "us_per_launch": d3[dom]["us_per_launch"]},
            "d3_kernels": d3,
            "gather_roofline": {"kernel": "cfsd spiral_gather_k (level 0, 32 ch, 16 meshes)",
                                "bound": "hbm", "achieved": gather_bytes / t_g / 1e9,
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": gather_bytes / t_g / 1e9 / HBM_PEAK_GBS,
                                "us_per_launch": t_g * 1e6},
            "parity": parity,
            "cpu_baseline": cpu,
            "losses_mean": (losses[:5] / max(losses[5], 1)).tolist(), "losses_finite": finite,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
