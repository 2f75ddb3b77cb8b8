"""A/B of the union-staged bf16 forward against conv_fwd_vm16 (bit-identity +
HIP-event timing) at the C2 shapes: levels 0 and 1, 16 meshes, 32 -> 32.
usage: python tools/union_ab.py [iters]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import ops, topology  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda")
npz = np.load(os.path.join(ROOT, "tests", "golden", "topology_craniofacial.npz"))
g = torch.Generator(device=dev).manual_seed(0)
B = int(os.environ.get("UA_BATCH", "16"))


def timed(fn, n=20):
    """Device time per launch: ``n`` launches captured in one graph, replayed."""
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            fn()
    for _ in range(3):
        gr.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    reps = max(1, iters // n)
    for _ in range(reps):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (reps * n)


for lev in (0, 1):
    sp = npz[f"spiral_{lev}"]
    if os.environ.get("UA_RCM"):  # locality (reverse Cuthill-McKee) vertex order
        from scipy.sparse import coo_matrix
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        v = sp.shape[0]
        a = coo_matrix((np.ones(sp.size), (np.repeat(np.arange(v), sp.shape[1]), sp.ravel())), shape=(v, v)).tocsr()
        order = np.asarray(reverse_cuthill_mckee((a + a.T).tocsr(), symmetric_mode=True), np.int64)
        inv = np.empty(v, np.int64)
        inv[order] = np.arange(v)
        sp = inv[np.asarray(sp, np.int64)[order]]
    nv = sp.shape[0]
    idx = torch.from_numpy(sp.astype(np.int32)).to(dev)
    cap = int(os.environ.get("UA_CAP", "56"))
    tiles, urows, lidx = (torch.from_numpy(a).to(dev) for a in topology.union_tiles(sp, cap))
    x = ops.vm_empty(B, nv, 32, torch.bfloat16)
    x.copy_(torch.randn(B, nv, 32, generator=g, device=dev).to(torch.bfloat16))
    w = (torch.randn(32, 9 * 32, generator=g, device=dev) * 0.06)
    wb = w.to(torch.bfloat16)
    b = torch.randn(32, generator=g, device=dev) * 0.1
    for act in (1, 0):
        for ydt in ("bf16_vm", "f32_bm"):
            if ydt == "bf16_vm":
                y0, y1 = ops.vm_empty(B, nv, 32, torch.bfloat16), ops.vm_empty(B, nv, 32, torch.bfloat16)
            else:
                y0, y1 = (torch.empty(B, nv, 32, device=dev) for _ in range(2))
            y0.fill_(1.0)
            y1.fill_(-1.0)
            f0 = lambda: ops.spiral_conv_fwd_x(x, idx, w, wb, b, act, y0)  # noqa: E731
            f1 = lambda: ops.spiral_conv_fwd_union(x, idx, (tiles, urows, lidx, cap), wb, b, act, y1)  # noqa: E731
            f0()
            f1()
            torch.cuda.synchronize()
            same = torch.equal(y0.contiguous().view(torch.int16) if y0.dtype == torch.bfloat16 else y0.contiguous(),
                               y1.contiguous().view(torch.int16) if y1.dtype == torch.bfloat16 else y1.contiguous())
            diff = (y0.float() - y1.float()).abs().max().item()
            t0, t1 = timed(f0), timed(f1)
            print(f"level {lev} act {act} y {ydt}: bitequal {same} maxdiff {diff:.3g}  vm16 {t0:.2f} us  union {t1:.2f} us"
                  f"  tiles {tiles.shape[0]} cap {cap}", flush=True)
