"""Benchmark: SD-VAE training throughput (meshes/s) on MI355X.

Workload (BASELINE.json config 2, ``configurations/craniofacial.yaml``): the
real craniofacial template hierarchy (17039/4260/1065/267/67 vertices,
spiral length 9, channels [32, 32, 32, 64], latent 75, VAE), batch_size 4
swapped to 16 meshes per GPU per step, fp32.  A step is the full reference
``_do_iteration``: device-side epoch-shuffled batch pick + swap key + VAE
noise, feature swap, forward, MSE + Laplacian + KL + latent-consistency
losses, backward, (RCCL all-reduce of the flat gradient when N > 1, in two
buckets overlapped with the encoder backward), Adam.  The dataset is
synthetic N(0, 1) meshes resident in HBM (no checkpoint/dataset egress).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
                       [--topology craniofacial|synth5k]
(for N > 1 launch with torch.distributed.run, one rank per GPU).
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import _abi, ops, topology  # noqa: E402
from craniofacialsd_vae_amd import dist as cdist  # noqa: E402
from craniofacialsd_vae_amd import engine as E  # noqa: E402
from craniofacialsd_vae_amd.step import TrainStep  # noqa: E402

METRIC = "train meshes/sec + per-vertex L1, craniofacial SD-VAE @1/2/4/8 MI355X"
TOPO_NPZ = os.path.join(ROOT, "tests", "golden", "topology_craniofacial.npz")
PROFILES = os.path.join(ROOT, "profiles")
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--dataset", type=int, default=256, help="resident synthetic meshes per rank")
    p.add_argument("--topology", default="craniofacial", choices=["craniofacial", "synth5k"])
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                   help="fp32 (reference arithmetic) or bf16 (configs C3/C5: bf16 level-0/1 tensors on "
                        "bf16 MFMA, fp32 accumulation and master weights)")
    p.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    p.add_argument("--batch-major", action="store_true",
                   help="fp32: keep every tensor batch-major (the reference's [B, V, C]) instead of storing "
                        "the level-0/1 tensors vertex-major (A/B of the layouts)")
    p.add_argument("--augmented", type=int, default=0,
                   help="configuration C5: train on N spectral-interpolation meshes (k = 1000 eigenvectors of "
                        "the template, pairs of the demo meshes) generated on the device and resident in HBM, "
                        "N / world per rank, instead of N(0, 1) meshes")
    p.add_argument("--cpu-seconds", type=float, default=24.0, help="CPU-baseline sample budget")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the secondary measurements (synthetic ~5k line, kernel trace, bf16 block)")
    p.add_argument("--no-bf16", action="store_true",
                   help="skip the bf16 block (configs C3/C5's precision, timed in the same run)")
    return p.parse_args()


def augmented_set(n, device, seed):
    """C5's training set (BASELINE config 5): ``n`` meshes generated on the
    device by spectral interpolation (utils.py:256-267) of same-class pairs of
    the 12 demo meshes (data_loading.py:292-374), k = 1000 eigenvectors of
    the template Laplacian, normalised by their own per-vertex mean / std
    (data_loading.py:231-252).  Returns (meshes, norm, timing)."""
    from craniofacialsd_vae_amd import augment as A
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import recipe
    npz = np.load(TOPO_NPZ)
    faces, nv = npz["face_0"].astype(np.int64), int(npz["pos_0"].shape[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, u = A.laplacian_eigendecomposition(faces, nv, k=1000, device=device)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m = recipe.load_meshes()
    raw = torch.from_numpy(m["verts"]).to(device)
    aug, cls = A.synthesize(u, raw, [str(x)[0] for x in m["names"]], n, seed=seed)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    std = torch.std(aug, dim=0)
    norm = {"mean": torch.mean(aug, dim=0), "std": torch.where(std > 0, std, torch.full_like(std, 1e-8))}
    del u, raw
    return aug, norm, {"meshes": n, "classes": {c: cls.count(c) for c in sorted(set(cls))},
                       "eigendecomposition_s": t1 - t0, "generation_s": t2 - t1,
                       "k": 1000, "source": "12 demo meshes (tests/golden/demo_meshes.npz), same-class pairs",
                       "finite": bool(torch.isfinite(aug).all())}


def load_topology(name, device):
    if name == "craniofacial":
        return topology.DeviceTopology.from_npz(dict(np.load(TOPO_NPZ)), device=device)
    from craniofacialsd_vae_amd import precompute
    return precompute.synthetic_hierarchy(device=device)


class Runner:
    """The benchmarked step is :class:`step.TrainStep` -- the same object
    the data-parallel GPU tests (tests/test_gpu_dist.py) and the training
    driver (manager.ModelManager) run."""

    def __init__(self, world, rank, device, n_meshes, use_graph, topo_name="craniofacial",
                 precision="fp32", meshes=None, norm=None, vertex_major=True):
        self.topo = load_topology(topo_name, device)
        self.topo_name = topo_name
        self.precision = precision
        self.eng = E.SDVAEEngine(self.topo, E.ModelSpec(latent_size=75), lr=1e-4, swap_bs=4,
                                 seed=1234 + rank, device=device, precision=precision,
                                 vertex_major=vertex_major)
        self.eng.reset_parameters()  # same init on every rank (broadcast below)
        self.world, self.rank = world, rank
        nv = self.topo.n_verts[0]
        if meshes is None:
            gen = torch.Generator(device=device).manual_seed(1234 + rank)
            meshes = torch.randn(n_meshes, nv, 3, device=device, generator=gen)
        # the bench owns the set: normalised in place (one resident copy)
        self.data = E.ResidentData(meshes, bs=4, shuffle=True, norm=norm, inplace=True)
        self.avg = cdist.GradientAverager(world)
        if world > 1:
            cdist.broadcast_parameters(self.eng.params.data, 0)
            self.eng.sync_shadow()
        self.ts = TrainStep(self.eng, self.data, self.avg)
        self.b = self.ts.b
        self.use_graph = use_graph

    def eager_step(self):
        self.ts.eager_step()

    def capture(self):
        self.ts.capture()
        self.ts.capture_multi()  # the multi-step graph the timed run(k) replays, recorded before timing

    def step(self):
        self.ts.step()

    def run(self, k):
        self.ts.run(k)


# ------------------------------------------------------------------ roofline
def launch_cost(name, a):
    """(flop, algorithmic HBM bytes, peak TFLOP/s) of one libcfsd launch from
    its ABI arguments (include/cfsd.h); (0, 0, None) for bookkeeping launches
    that do no work the algorithm requires (step counter, latent head,
    loss finalisation, slab reduction, gradient scaling)."""
    f4 = 4

    def sz(dt):  # bytes per element of a storage descriptor (type | CFSD_VM)
        return 4 if (dt & 0xf) == 0 else 2

    if name == "cfsd_spiral_conv_fwd":
        B, vs, rows, S, ci, co = a[7:13]
        return 2.0 * B * rows * S * ci * co, f4 * (B * vs * ci + B * rows * co + co * S * ci) + 4 * rows * S, FP32_PEAK_TFLOPS
    if name == "cfsd_spiral_conv_bwd_data":
        B, vs, rows, S, ci, co = a[9:15]
        elu = a[5] is not None
        return (2.0 * B * rows * S * ci * co,
                f4 * (B * rows * co + B * vs * ci * (2 if elu else 1) + co * S * ci) + 16 * vs * S, FP32_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_bwd_weight":
        B, vs, rows, S, ci, co = a[7:13]
        return 2.0 * B * rows * S * ci * co, f4 * (B * vs * ci + B * rows * co + co * S * ci) + 4 * rows * S, FP32_PEAK_TFLOPS
    if name == "cfsd_spiral_conv_bwd":
        B, vs, rows, S, ci, co = a[13:19]
        dx, elu = a[8] is not None, a[7] is not None
        fl = 2.0 * B * rows * S * ci * co * (2 if dx else 1)
        by = f4 * (B * vs * ci + B * rows * co + co * S * ci) + 4 * rows * S
        if dx:
            by += f4 * B * vs * ci * (2 if elu else 1) + 16 * vs * S
        return fl, by, FP32_PEAK_TFLOPS
    if name == "cfsd_spiral_conv_bwd_rowsub":  # dx (dG + gather) and dW of a row-subset conv
        B, vs, rows, S, ci, co = a[12:18]
        elu = a[6] is not None
        return (4.0 * B * rows * S * ci * co,
                f4 * (B * vs * ci * (2 if elu else 1) + B * vs * ci + B * rows * co + co * S * ci) + 4 * rows * S
                + 4 * vs * a[4], FP32_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_bwd_data_rowsub":
        B, vs, rows, S, ci, co = a[9:15]
        sd = sz(a[6])
        elu = a[4] is not None
        return (2.0 * B * rows * S * ci * co, f4 * (B * rows * co + co * S * ci) + sd * B * vs * ci * (2 if elu else 1)
                + 4 * vs * a[2], FP32_PEAK_TFLOPS)
    if name in ("cfsd_spmm_csr_sched", "cfsd_spmm_sched_csr"):
        sx, sy = sz(a[5]), sz(a[8])
        B, m, n, c = a[9:13]
        elu = a[6] is not None
        return 0.0, B * c * (sx * n + sy * m * (2 if elu else 1)), None
    if name == "cfsd_spiral_conv_fwd_x":
        sx, sy = sz(a[1]), sz(a[7])
        B, vs, rows, S, ci, co = a[8:14]
        peak = BF16_PEAK_TFLOPS if (ci >= 16 and co >= 16 and sx == 2) else FP32_PEAK_TFLOPS
        return 2.0 * B * rows * S * ci * co, sx * B * vs * ci + sy * B * rows * co + 2 * co * S * ci + 4 * rows * S, peak
    if name == "cfsd_spiral_conv_bwd_data_x":
        sd = sz(a[1])
        B, vs, rows, S, ci, co = a[9:15]
        elu = a[6] is not None
        return (2.0 * B * rows * S * ci * co, sd * B * rows * co + 2 * B * vs * ci * (2 if elu else 1)
                + 2 * co * S * ci + 16 * vs * S, BF16_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_bwd_data_flat":
        sd, sx = sz(a[1]), sz(a[7])
        B, vs, rows, S, ci, co = a[8:14]
        elu = a[5] is not None
        return (2.0 * B * rows * S * ci * co, sd * B * rows * co + sx * B * vs * ci * (2 if elu else 1)
                + sx * co * S * ci + 4 * vs * a[3], BF16_PEAK_TFLOPS if sx == 2 else FP32_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_bwd_weight_x":
        sx, sd = sz(a[1]), sz(a[4])
        B, vs, rows, S, ci, co = a[9:15]
        peak = BF16_PEAK_TFLOPS if (ci >= 16 and sx == 2) else FP32_PEAK_TFLOPS
        return 2.0 * B * rows * S * ci * co, sx * B * vs * ci + sd * B * rows * co + 4 * co * S * ci + 4 * rows * S, peak
    if name == "cfsd_spiral_conv_bwd_x":
        sx = sz(a[1])  # x, elu_y, dx storage
        B, vs, rows, S, ci, co = a[15:21]
        dx, elu = a[10] is not None, a[9] is not None
        fl = 2.0 * B * rows * S * ci * co * (2 if dx else 1)
        by = sx * B * vs * ci + 4 * B * rows * co + 4 * co * S * ci + (sx * B * vs * ci * (2 if elu else 1) if dx else 0)
        return fl, by, FP32_PEAK_TFLOPS
    if name in ("cfsd_spmm_csr_x", "cfsd_spmm_uniform"):
        sx, sy = sz(a[4]), sz(a[7])
        B, m, n, c = a[8:12]
        elu = a[5] is not None
        return 0.0, B * c * (sx * n + sy * m * (2 if elu else 1)), None
    if name == "cfsd_spmm_csr":
        B, m, n, c = a[6:10]
        elu = a[4] is not None
        return 0.0, f4 * B * c * (n + m * (2 if elu else 1)), None
    if name == "cfsd_spiral_conv_bwd_flat_pair":  # flat-list dx + vm32 dW of one vertex-major conv
        B, vs, rows, S, ci, co = a[12:18]
        elu = a[6] is not None
        return (4.0 * B * rows * S * ci * co,
                f4 * (B * rows * co + B * vs * ci * (2 + int(elu)) + 2 * co * S * ci) + 4 * rows * S
                + 4 * vs * a[4], FP32_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_bwd_flat_pair_bf16":  # the same pair on bf16 operands
        B, vs, rows, S, ci, co = a[10:16]
        elu = a[6] is not None
        return (4.0 * B * rows * S * ci * co,
                2.0 * (B * rows * co + B * vs * ci * (2 + int(elu)) + co * S * ci) + 4 * rows * S + 4 * vs * a[4],
                BF16_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_bwd_rowsub_pair_bf16":  # bf16 Enblock: fp32-product dx + bf16 dW
        B, vs, rows, S, ci, co = a[10:16]
        elu = a[6] is not None
        return (4.0 * B * rows * S * ci * co,
                f4 * (B * rows * co + co * S * ci) + 2.0 * B * vs * ci * (2 + int(elu)) + 4 * rows * S
                + 4 * vs * a[4], FP32_PEAK_TFLOPS)
    if name == "cfsd_spiral_conv_fwd_in_swap":  # the swap + the xyz input conv (spiral length 9)
        bs, vs, rows, ci, co = a[4], a[14], a[15], a[16], a[17]
        B, S = bs * bs, 9
        return (2.0 * B * rows * S * ci * co,
                f4 * (bs * vs * ci + B * vs * ci) + vs + sz(a[13]) * B * rows * co + f4 * co * S * ci + 4 * rows * S,
                FP32_PEAK_TFLOPS)
    if name in ("cfsd_swap_features", "cfsd_swap_features_x"):
        bs, nv, c = a[5:8] if name == "cfsd_swap_features" else a[6:9]
        return 0.0, f4 * (bs * nv * c + bs * bs * nv * c) + nv, None
    if name in ("cfsd_recon_lap_fwd", "cfsd_recon_lap_fwd_x"):
        B, nv, c = a[7:10]
        return 0.0, f4 * 3 * B * nv * c, None
    if name in ("cfsd_recon_lap_bwd", "cfsd_recon_lap_bwd_finalize", "cfsd_recon_lap_bwd_x",
                "cfsd_recon_lap_bwd_finalize_x"):
        B, nv, c = a[7:10]
        return 0.0, f4 * 4 * B * nv * c, None
    if name == "cfsd_linear_fwd":
        m, k, n = a[6:9]
        return 2.0 * m * k * n, f4 * (m * k + n * k + m * n), FP32_PEAK_TFLOPS
    if name == "cfsd_linear_bwd":
        m, k, n = a[9:12]
        dx, dw, elu = a[4] is not None, a[5] is not None, a[3] is not None
        fl = 2.0 * m * k * n * (int(dx) + int(dw))
        by = f4 * (m * n + n * k + m * k * (int(dx) + int(dw) + int(elu)) + n * k * int(dw))
        return fl, by, FP32_PEAK_TFLOPS
    if name == "cfsd_linear_bwd_split":
        m, k, n = a[6:9]
        return 4.0 * m * k * n, f4 * (m * n + 2 * n * k + m * k), FP32_PEAK_TFLOPS
    if name == "cfsd_spiral_conv_bwd_out_flat":  # xyz output conv: dx (with ELU') + dW in one pass
        sx = sz(a[1])  # x, elu_y, dx storage
        B, vs, rows, S, ci, co = a[14:20]
        dx, elu = a[9] is not None, a[8] is not None
        fl = 2.0 * B * rows * S * ci * co * (2 if dx else 1)
        by = (sx * B * vs * ci + 4 * B * rows * co + 4 * co * S * ci + 4 * vs * a[6]
              + (sx * B * vs * ci * (2 if elu else 1) if dx else 0))
        return fl, by, FP32_PEAK_TFLOPS
    if name == "cfsd_spiral_conv_fwd_up":  # Deblock: Pool(up) inside the conv gather
        B, nc, rows, S, ci, co = a[8:14]
        up_out = a[7] is not None
        fl = 2.0 * B * rows * S * ci * co + 2.0 * 3 * B * rows * ci
        by = (f4 * (B * nc * ci + B * rows * co + co * S * ci + (B * rows * ci if up_out else 0))
              + 4 * rows * S + 8 * 3 * rows)  # idx + the up matrix (3 entries per row: col + val)
        return fl, by, FP32_PEAK_TFLOPS
    if name == "cfsd_spiral_conv_bwd_rowsub_x":  # row-subset dx + dW, x / dx / elu_y in x_dt
        sx = sz(a[1])
        B, vs, rows, S, ci, co = a[13:19]
        elu = a[7] is not None
        return (4.0 * B * rows * S * ci * co,
                sx * B * vs * ci * (2 if elu else 1) + sx * B * vs * ci + f4 * (B * rows * co + co * S * ci)
                + 4 * rows * S + 4 * vs * a[5], FP32_PEAK_TFLOPS)
    if name == "cfsd_latent_linear_fwd":  # latent head (KL, LC, reparameterisation) + decoder Linear
        bsz, lat, n = a[6], a[7], a[19]
        nin = 2 * lat if a[10] else lat
        return (2.0 * bsz * lat * n + 10.0 * bsz * lat,
                f4 * (bsz * nin + bsz * lat * 4 + n * lat + n + bsz * n), FP32_PEAK_TFLOPS)
    if name in ("cfsd_latent_bwd", "cfsd_latent_bwd_parts"):  # latent head backward
        bsz, lat = (a[6], a[7]) if name == "cfsd_latent_bwd" else (a[7], a[8])
        return 10.0 * bsz * lat, f4 * bsz * lat * 8, FP32_PEAK_TFLOPS
    if name == "cfsd_dw_reduce_batch_adam":  # the slab reduction is bookkeeping; Adam's 7 streams are not
        n = a[7].value if hasattr(a[7], "value") else a[7]
        return 0.0, 7.0 * f4 * n, None
    if name == "cfsd_adam":
        n = a[5].value if hasattr(a[5], "value") else a[5]
        return 0.0, 7.0 * f4 * n, None
    if name == "cfsd_adam_scaled":  # + the scaled gradient written back
        n = a[5].value if hasattr(a[5], "value") else a[5]
        return 0.0, 8.0 * f4 * n, None
    if name == "cfsd_bottleneck_bwd":  # Pool(up)^T + decoder Linear + latent head + encoder Linear
        n_up, cup, nd = a[4], a[5], a[11]
        ke, ne, B, lat = a[25], a[26], a[29], a[30]
        elu = a[21] is not None
        fl = 4.0 * B * lat * nd + 10.0 * B * lat + 4.0 * B * ke * ne
        by = (f4 * B * cup * n_up + 12 * nd // cup * 3      # fine gradient + the CSR (dh never stored)
              + f4 * (2 * nd * lat + B * lat)               # W_d, dW_d, z
              + f4 * B * lat * 8                            # latent head
              + f4 * (2 * ne * ke + B * ke * (2 + int(elu)) + B * ne))  # W_e, dW_e, x_e, dx_e (elu_y), dmulv
        return fl, by, FP32_PEAK_TFLOPS
    return 0.0, 0.0, None


# Launches that do no work the algorithm requires (priced at zero by
# launch_cost): step counter / noise / batch pick, loss reduction, the
# deferred weight-gradient slab reduction, gradient scaling.
BOOKKEEPING = ("cfsd_step_begin", "cfsd_loss_finalize", "cfsd_dw_reduce_batch", "cfsd_scale")


def step_roofline(runner, ms_per_step):
    """Time-weighted roofline of one training step: every launch of an eager
    step is timed with a HIP event pair on its stream (queued behind a sleep
    kernel so the device runs them back-to-back, as in the graph) and scaled
    to the graph step (the pairs' own overhead makes the eager sum exceed it),
    priced at its roofline time max(flop/peak, bytes/8 TB/s) from the work the
    algorithm requires (Enblock row subset applied), and the sum of those
    ideal times is divided by the measured time."""
    torch.cuda.synchronize()
    torch.cuda._sleep(50_000_000)
    with _abi.trace_launches() as rec:
        runner.eager_step()
    torch.cuda.synchronize()
    rows, t_sum, ideal_sum, flop_sum, byte_sum = [], 0.0, 0.0, 0.0, 0.0
    for name, args, e0, e1 in rec:
        t = e0.elapsed_time(e1) * 1e-3
        fl, by, peak = launch_cost(name, args)
        ideal = max(fl / (peak * 1e12) if peak else 0.0, by / (HBM_PEAK_GBS * 1e9))
        rows.append((name, t, fl, by, ideal))
        t_sum += t
        ideal_sum += ideal
        flop_sum += fl
        byte_sum += by
    # The eager event pairs add per-launch overhead the graph replay does not
    # pay (their sum exceeds the graph step): every launch time is scaled by
    # one factor so that they sum to at most the measured (graph) step.
    raw_sum = t_sum
    scale = min(1.0, (ms_per_step * 1e-3) / t_sum) if t_sum else 1.0
    rows = [(n, t * scale, fl, by, i) for n, t, fl, by, i in rows]
    t_sum *= scale
    top = sorted(rows, key=lambda r: -r[1])[:8]
    return {
        "launches": len(rows), "kernel_time_us": t_sum * 1e6,
        "eager_kernel_time_us": raw_sum * 1e6, "eager_to_graph_scale": scale,
        "required_gflop_per_step": flop_sum / 1e9, "algorithmic_mb_per_step": byte_sum / 1e6,
        "ideal_time_us": ideal_sum * 1e6,
        "frac_of_kernel_time": ideal_sum / t_sum if t_sum else None,
        "frac_of_step_time": ideal_sum / (ms_per_step * 1e-3),
        "achieved_tflops_step": flop_sum / (ms_per_step * 1e-3) / 1e12,
        "note": "per-launch times: eager HIP event pairs, scaled by eager_to_graph_scale so that they sum to "
                "at most the graph-replayed step; "
                "frac = sum over launches of max(flop/peak, bytes/HBM) / measured time; "
                "bookkeeping launches (" + ", ".join(BOOKKEEPING) + ") count as time with no required "
                "work; cfsd_dw_reduce_batch_adam is priced at Adam's 7 x 4 B per parameter only",
        "unpriced_work_launches": sorted({n for n, _, fl, by, _ in rows if fl == 0 and by == 0
                                          and n not in BOOKKEEPING}),
        "top_launches": [{"name": n, "us": t * 1e6, "frac": (i / t if t else None)}
                         for n, t, _, _, i in top],
    }


def kernel_probe(runner, n_iter=20):
    """Per-kernel device time of the dominant kernels, HIP events on the
    launch stream (eager replays of the same step, same inputs)."""
    eng, b, T = runner.eng, runner.b, runner.topo
    st = torch.cuda.current_stream()
    res = {}

    def timed(name, fn, reps=3):
        # best of `reps` back-to-back batches after 3 warm-up launches (the
        # first batch after an idle gap can catch the clock ramping up)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            e0.record(st)
            for _ in range(n_iter):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / n_iter * 1e-3  # seconds per launch
            best = t if best is None else min(best, t)
        res[name] = best

    dec = eng.spec.dec_layers()
    i3 = len(dec) - 1
    w3, bias3 = eng._dec_w(i3)
    wname = f"de_layers.{i3 + 1}.conv.layer.weight"
    # the D3 kernels exactly as the step launches them (dW deferred: slab
    # kernel only, reduced by the batched reduce)
    if 0 in b.xl:  # vertex-major level 0 (bf16, or fp32 at batch % 16 == 0)
        w16 = eng._w16(wname) if runner.precision == "bf16" else None
        wx = eng._wx(wname)
        timed("conv_fwd_D3", lambda: ops.spiral_conv_fwd_x(b.dec_up[i3], T.spiral[0], w3, w16, bias3, 1,
                                                            b.dec_out[i3]))
        if eng._flat_dx(b, 0, 32, 32):
            timed("conv_dx_D3", lambda: ops.spiral_conv_bwd_data_flat(b.dpre_dec[i3], T.spiral_flat[0], wx,
                                                                      T.n_verts[0], out=b.g_dec_up[i3]))
        else:
            timed("conv_dx_D3", lambda: ops.spiral_conv_bwd_data_x(b.dpre_dec[i3], T.spiral_inv[0], w16,
                                                                   T.n_verts[0], out=b.g_dec_up[i3]))
        timed("conv_dw_D3", lambda: ops.spiral_conv_bwd_weight_x(b.dec_up[i3], T.spiral[0], b.dpre_dec[i3],
                                                                 None, None, b.ws_dw[("dec", i3)]))
        if b.vm_pair.get(("dec", i3)) and runner.precision == "bf16":  # the step runs dx + dW as one launch
            timed("conv_pair_D3", lambda: ops.spiral_conv_bwd_flat_pair_bf16(
                b.dec_up[i3], T.spiral[0], b.dpre_dec[i3], T.spiral_flat[0], wx, b.g_dec_up[i3],
                workspace=b.ws_dw[("dec", i3)]))
    else:
        timed("conv_fwd_D3", lambda: ops.spiral_conv_fwd(b.dec_up[i3], T.spiral[0], w3, bias3, 1,
                                                          out=b.dec_out[i3]))
        # the D3 backward kernels exactly as the step launches them (dW
        # deferred: slab kernel only, reduced by the batched reduce)
        timed("conv_dx_D3", lambda: ops.spiral_conv_bwd_data(b.dpre_dec[i3], T.spiral_inv[0], w3,
                                                             T.n_verts[0], out=b.g_dec_up[i3], workspace=b.ws))
        timed("conv_dw_D3", lambda: ops.spiral_conv_bwd_weight(b.dec_up[i3], T.spiral[0], b.dpre_dec[i3],
                                                               None, None, b.ws_dw[("dec", i3)]))
    g = torch.empty(16, T.n_verts[0], 9 * 32, device=b.x.device)
    xg = b.dec_up[i3].float().contiguous()  # batch-major fp32 copy
    timed("spiral_gather_L0", lambda: ops.spiral_gather(xg, T.spiral[0], out=g))
    del g
    return res


def pmc_traffic(key="conv_fwd_d3"):
    """HBM bytes per launch of a D3 kernel from the newest PMC pass under
    profiles/ (tools/pmc_traffic.py: FETCH_SIZE and WRITE_SIZE in separate
    rocprofv3 runs, gfx950 FETCH_SIZE x2 correction).  Newest = the largest
    "created" stamp written by the tool (files without one rank by mtime)."""
    import glob
    best = None
    for f in glob.glob(os.path.join(PROFILES, f"*_pmc_traffic_{key}.json")):
        with open(f) as fh:
            d = json.load(fh)
        if not d.get("hbm_bytes_per_launch"):  # a pass that matched no launch
            continue
        rank = (d.get("created", 0), os.path.getmtime(f))
        if best is None or rank > best[0]:
            best = (rank, d, f)
    if best is None:
        return None, None
    return best[1].get("hbm_bytes_per_launch"), os.path.relpath(best[2], ROOT)


def _bits_checksum(t):
    """Order-sensitive checksum of a float buffer's bit patterns (int64,
    wrapping): equal on two ranks iff (up to a 2^-64 collision) the buffers
    are bit-identical."""
    bits = t.detach().contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(bits.numel(), device=t.device, dtype=torch.int64) % 65521 + 1
    return int((bits * w).sum().item())


def dist_check(runner, el, steps, backend, shared_device):
    """Self-verification of an N > 1 line (every rank calls it): the world
    size and backend the process group really has, each rank's GPU (PCI
    domain:bus:device, all-gathered; distinct unless the one-GPU rehearsal
    CFSD_SHARE_DEVICE shares it on purpose), each rank's own ms per step, and
    bit checksums of the parameters, the gradient and both Adam moments after
    the timed steps, which data-parallel training keeps identical on every
    rank (model_manager.py:360-393: each rank's swap groups are independent,
    the averaged gradient and Adam are the same everywhere)."""
    P = runner.eng.params
    dev = P.data.device
    props = torch.cuda.get_device_properties(dev)
    mine = {"rank": dist.get_rank(), "device": str(dev),
            "pci": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
            "ms_per_step": el / steps * 1e3, "adam_t": int(P.step.item()),
            "params": _bits_checksum(P.data), "grad": _bits_checksum(P.grad),
            "exp_avg": _bits_checksum(P.exp_avg), "exp_avg_sq": _bits_checksum(P.exp_avg_sq)}
    if P.shadow is not None:
        mine["shadow"] = _bits_checksum(P.shadow.view(torch.int16).to(torch.int32).float())
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, mine)
    keys = [k for k in ("params", "grad", "exp_avg", "exp_avg_sq", "shadow", "adam_t") if k in mine]
    pcis = [r["pci"] for r in allr]
    ms = [r["ms_per_step"] for r in allr]
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
            "shared_device_rehearsal": bool(shared_device),
            "pci_bus_ids": pcis, "distinct_devices": len(set(pcis)) == len(pcis),
            "ms_per_step_min": min(ms), "ms_per_step_max": max(ms),
            "ranks_in_sync": all(r[k] == allr[0][k] for r in allr for k in keys),
            "checksums_rank0": {k: allr[0][k] for k in keys}}


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


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                return ln.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cpus():
    """CPUs this process may actually use: the cgroup CPU quota (cpu.max)
    when one is set, else the scheduler affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, min(aff, int(float(quota) / float(period))))
    except (OSError, ValueError):
        pass
    return aff


def cpu_baseline(budget_s):
    """Oracle (PyTorch-CPU restatement of the reference step, the same ATen
    ops) on the host: with the CPUs this process may use (cgroup quota /
    affinity; also OMP_NUM_THREADS when set) and with one thread; ``value`` =
    the fastest.  With os.cpu_count() threads on a quota-limited box the run
    is oversubscribed (measured on the 256-CPU GPU host with a 16-CPU share:
    0.56 meshes/s, 28.5 s for ONE step, profiles/r02e_bench.json), so that
    configuration is reported, not re-run by default."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle import cfsd_oracle as O
    import recipe
    T = O.Topology(dict(np.load(TOPO_NPZ)))
    P = O.make_params(recipe.golden_weights())
    opt = O.Adam(P)
    rs = np.random.RandomState(0)
    x4 = rs.randn(4, T.n_verts[0], 3).astype(np.float32)
    eps = rs.randn(16, 75).astype(np.float32)
    host = os.cpu_count() or 1
    usable = usable_cpus()
    cand = {usable}
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cand.add(min(int(os.environ["OMP_NUM_THREADS"]), host))
    if os.environ.get("CFSD_CPU_ALL_THREADS"):
        cand.add(host)
    multi = sorted(cand, reverse=True)
    plan = [(t, budget_s * 0.65 / len(multi)) for t in multi] + [(1, budget_s * 0.35)]
    runs = []
    for threads, budget in plan:
        torch.set_num_threads(threads)
        O.train_step(P, opt, x4, T, 0, eps)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            O.train_step(P, opt, x4, T, n % 15, eps)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= 200:
                break
        runs.append({"threads": threads, "steps": n, "seconds": el, "meshes_per_s": 16 * n / el})
    best = max(runs, key=lambda r: r["meshes_per_s"])
    return {"value": best["meshes_per_s"], "unit": "meshes/s", "cores": best["threads"], "kind": "port",
            "sample": f"{best['steps']} full train steps (16 swapped meshes each, fp32, "
                      f"oracle/cfsd_oracle.py torch-CPU restatement) in {best['seconds']:.1f} s",
            "one_thread": runs[-1]["meshes_per_s"], "host_cpus": host, "usable_cpus": usable,
            "cpu_model": cpu_model(), "runs": runs}


def synth5k_line(device, steps=500, warmup=20):
    """Secondary throughput line (north_star's "~5k verts, 4 levels"): the
    same step on a synthetic 5120/1280/320/80/20 hierarchy built by the
    product's own topology precompute (craniofacialsd_vae_amd.precompute)."""
    r = Runner(1, 0, device, 256, True, "synth5k")
    r.capture()
    r.run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.run(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"workload": "synthetic 4-level hierarchy, same model/step, 16 meshes/GPU, fp32",
            "levels": r.topo.n_verts, "value": 16 * steps / el, "unit": "meshes/s",
            "ms_per_step": el / steps * 1e3, "steps": steps}


def d3_roofline(runner, probe, topo_name):
    """Per-launch roofline of the three D3 (decoder level 0, 32 -> 32) conv
    kernels, 5.02 GFLOP each, from their live HIP-event times (``probe``);
    returns (kernels, dominant key, kernel names).  fp32: MFMA bound (AI 72
    flop/B > ridge 19.7); bf16: HBM bound (AI ~140 flop/B < ridge 312),
    priced on algorithmic bytes (input + output once + indices)."""
    nv = runner.topo.n_verts[0]
    flops = 2.0 * 16 * nv * 9 * 32 * 32
    bf = runner.precision == "bf16"
    s_act = 2 if bf else 4
    d3_bytes = {"conv_fwd_D3": s_act * 16 * nv * 64 + nv * 36,
                "conv_dx_D3": s_act * 16 * nv * 64 + nv * 9 * 16,
                "conv_dw_D3": s_act * 16 * nv * 64 + nv * 36}
    d3 = {}
    vm0 = 0 in runner.b.xl  # level-0 tensors vertex-major (the kernels below)
    for name, key in (("conv_fwd_D3", "conv_fwd_d3"), ("conv_dx_D3", "conv_dx_d3"), ("conv_dw_D3", "conv_dw_d3")):
        t = probe[name]
        key = key + ("_bf16" if bf else "") + ("_vm" if vm0 else "")
        traffic, traffic_src = pmc_traffic(key) if topo_name == "craniofacial" else (None, None)
        if bf:
            d3[name] = {"us_per_launch": t * 1e6, "bound": "hbm", "achieved": d3_bytes[name] / t / 1e9,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": d3_bytes[name] / t / 1e9 / HBM_PEAK_GBS, "tflops": flops / t / 1e12,
                        "algorithmic_bytes": d3_bytes[name], "traffic": traffic, "traffic_source": traffic_src}
        else:
            d3[name] = {"us_per_launch": t * 1e6, "bound": "mfma", "achieved": flops / t / 1e12,
                        "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": flops / t / 1e12 / FP32_PEAK_TFLOPS, "algorithmic_flop": flops,
                        "traffic": traffic, "traffic_source": traffic_src}
    if "conv_pair_D3" in probe:  # bf16: the step runs D3's dx + dW as one launch (ABI 4.11)
        t = probe["conv_pair_D3"]
        pb = 3 * s_act * 16 * nv * 32 + 2 * 32 * 288 + nv * 9 * 4 + nv * 20 * 4
        ptr_, psrc = pmc_traffic("conv_pair_d3_bf16_vm") if topo_name == "craniofacial" else (None, None)
        d3["conv_pair_D3"] = {"us_per_launch": t * 1e6, "bound": "hbm", "achieved": pb / t / 1e9,
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": pb / t / 1e9 / HBM_PEAK_GBS,
                              "tflops": 2 * flops / t / 1e12, "algorithmic_bytes": pb, "traffic": ptr_,
                              "traffic_source": psrc}
        for k in ("conv_dx_D3", "conv_dw_D3"):
            d3[k]["in_step"] = False  # measured standalone; the step runs the pair
    dom = max((k for k in d3 if d3[k].get("in_step", True)), key=lambda k: d3[k]["us_per_launch"])
    if bf:
        kern_names = {"conv_fwd_D3": "conv_fwd_vm16<32,32> (decoder level 0 forward, bf16, vertex-major)",
                      "conv_dx_D3": "conv_dx_flat_vm16<32,32> (decoder level 0 data gradient, bf16, "
                                    "vertex-major flat list)",
                      "conv_dw_D3": "conv_dw_vm16 (decoder level 0 weight gradient, bf16, vertex-major)",
                      "conv_pair_D3": "conv_bwd_vm16_pair (decoder level 0 dx + dW slabs, bf16, vertex-major, "
                                      "one launch)"}
    elif vm0:
        kern_names = {"conv_fwd_D3": "conv_fwd_vm32<32,32> (decoder level 0 forward, vertex-major)",
                      "conv_dx_D3": "conv_dx_flat_vm32<32,32> (decoder level 0 data gradient, vertex-major "
                                    "flat list)",
                      "conv_dw_D3": "conv_dw_vm32 (decoder level 0 weight gradient, vertex-major)"}
    else:
        kern_names = {"conv_fwd_D3": "conv_fwd_mfma<32,32> (decoder level 0 forward)",
                      "conv_dx_D3": "conv_dx_mfma<32,32> (decoder level 0 data gradient)",
                      "conv_dw_D3": "conv_dw_mfma<32,32> (decoder level 0 weight gradient)"}
    return d3, dom, dict({"kernel": "cfsd " + kern_names[dom]}, **d3[dom])


def timed(runner, steps, warmup, world, device):
    """Capture, W untimed warm-up steps, then EXACTLY K steps between a
    barrier + synchronize on both sides; returns (this rank's seconds, the
    max over ranks)."""
    if runner.use_graph:
        runner.capture()
    runner.run(warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.run(steps)  # exactly `steps` training steps (steps_per_graph per replay of the multi-step graph)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el_rank = time.perf_counter() - t0
    return el_rank, cdist.max_over_ranks(el_rank, device)


def bf16_block(args, world, rank, device):
    """Configs C3 / C5's precision in the same run: the same step (same
    workload, per-GPU batch and parallelism) with bf16 level-0/1 tensors on
    bf16 MFMA, its own timed region, its own D3 roofline (against HBM)."""
    runner = Runner(world, rank, device, args.dataset, not args.no_graph, args.topology, "bf16")
    el_rank, el = timed(runner, args.steps, args.warmup, world, device)
    losses = runner.eng.loss_acc.cpu().numpy()
    runner.eng.check_health()
    probe = kernel_probe(runner)
    d3, _, roof = d3_roofline(runner, probe, args.topology)
    out = {"metric": METRIC, "value": 16 * world * args.steps / el, "unit": "meshes/s",
           "ms_per_step": el / args.steps * 1e3, "steps": args.steps, "warmup": args.warmup, "dtype": "bf16",
           "config": "the main line's workload and parallelism; levels 0-1 bf16 vertex-major, coarse levels, "
                     "losses, gradients, Adam and master weights fp32",
           "roofline": roof, "d3_kernels": d3, "losses_finite": bool(np.isfinite(losses).all())}
    del runner
    torch.cuda.empty_cache()
    return out


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
    aug_info, meshes, norm = None, None, None
    if args.augmented:
        per_rank = args.augmented // world
        meshes, norm, aug_info = augmented_set(per_rank, device, seed=77 + rank)
    runner = Runner(world, rank, device, args.dataset, not args.no_graph, args.topology, args.precision,
                    meshes=meshes, norm=norm, vertex_major=not args.batch_major)
    del meshes
    el_rank, el = timed(runner, args.steps, args.warmup, world, device)
    dcheck = dist_check(runner, el_rank, args.steps, backend, os.environ.get("CFSD_SHARE_DEVICE")) \
        if world > 1 else None
    meshes = 16 * world * args.steps
    ms_per_step = el / args.steps * 1e3
    losses = runner.eng.loss_acc.cpu().numpy()
    finite = bool(np.isfinite(losses).all())
    runner.eng.check_health()  # the one-launch bottleneck backward never gave up waiting
    probe = kernel_probe(runner)
    steprf = None if args.no_extras else step_roofline(runner, ms_per_step)
    bf = runner.precision == "bf16"
    bfb = None
    if not (bf or args.no_extras or args.no_bf16 or args.augmented or args.batch_major):
        bfb = bf16_block(args, world, rank, device)
    if rank == 0:
        nv = runner.topo.n_verts[0]
        gather_bytes = 16 * nv * (32 + 9 * 32) * 4 + nv * 9 * 4
        t_g = probe["spiral_gather_L0"]
        parity = c1_parity(device)
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline(args.cpu_seconds)  # N=1 only
        s5k = None
        if not (args.no_extras or world > 1 or args.topology != "craniofacial" or bf):
            try:
                s5k = synth5k_line(device)
            except (ImportError, AttributeError) as e:  # precompute not available
                s5k = {"error": str(e)}
        d3, _, roof = d3_roofline(runner, probe, args.topology)
        out = {
            "metric": METRIC, "value": meshes / el, "unit": "meshes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if bf else "fp32",
            "data": ("spectral-interpolation augmented meshes generated on the device, resident in HBM, "
                     "random-init weights" if aug_info else
                     "synthetic N(0,1) meshes resident in HBM, random-init weights"),
            "augmented_set": aug_info,
            "config": {"workload": "craniofacial.yaml SD-VAE train step (swap bs 4->16, fwd, "
                                   "MSE+Laplacian+KL+latent-consistency, bwd, Adam)",
                       "precision": runner.precision,
                       "layout": "vertex-major levels 0-1" if 0 in runner.b.xl else "batch-major",
                       "topology": args.topology, "template_vertices": nv, "levels": runner.topo.n_verts,
                       "global_batch": 16 * world, "per_gpu_batch": 16,
                       "resident_meshes_per_gpu": runner.data.n_items,
                       "parallelism": f"dp{world}", "graph": runner.use_graph,
                       "step_graph": ("one graph per step" if runner.ts.one_graph else "three graphs") +
                                     (", collectives captured" if (world > 1 and runner.ts.one_graph) else ""),
                       "step_graph_fallback": runner.ts.fallback,
                       "collective": None if world == 1 else
                       (("rccl" if backend == "nccl" else backend) + " all_reduce, 2 buckets overlapped")},
            "roofline": roof,
            "d3_kernels": d3,
            "bf16": bfb,
            "step_roofline": steprf,
            "gather_roofline": {"kernel": "cfsd spiral_gather_k (level 0, 32 ch, 16 meshes)",
                                "bound": "hbm", "achieved": gather_bytes / t_g / 1e9,
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": gather_bytes / t_g / 1e9 / HBM_PEAK_GBS,
                                "us_per_launch": t_g * 1e6},
            "dist_check": dcheck,
            "synthetic_5k": s5k,
            "parity": parity,
            "cpu_baseline": cpu,
            "losses_mean": (losses[:5] / max(losses[5], 1)).tolist(), "losses_finite": finite,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
