"""Diagnostic: lat dW (cfsd_spiral_conv_bwd_weight, few-row geometry) vs a
torch reference on the device; prints the error pattern per slot / row."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "tests/golden")
import cfsd_loader  # noqa: E402

cfsd_loader.load()
import recipe  # noqa: E402
from craniofacialsd_vae_amd import ops, topology  # noqa: E402

T = topology.DeviceTopology.from_npz(recipe.load_topology(), device="cuda")
for (cin, cout, level, bsz) in [(32, 32, 3, 3), (32, 32, 2, 16), (64, 64, 2, 3)]:
    idx = T.spiral[level]
    v = idx.shape[0]
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(bsz, v, cin, device="cuda", generator=g)
    dpre = torch.randn(bsz, v, cout, device="cuda", generator=g)
    G = x[:, idx.long()].reshape(bsz * v, 9 * cin)
    ref = dpre.reshape(-1, cout).t().double() @ G.double()
    dw = torch.empty(cout, 9 * cin, device="cuda")
    db = torch.empty(cout, device="cuda")
    ws = torch.zeros(ops.spiral_conv_bwd_weight_workspace(bsz, v, 9, cin, cout) // 4 + 1, device="cuda")
    ops.spiral_conv_bwd_weight(x, idx, dpre, dw, db, ws)
    torch.cuda.synchronize()
    err = (dw.double() - ref).abs()
    print(f"cin {cin} cout {cout} level {level} bsz {bsz} rows {bsz * v}: max err {err.max():.3e} "
          f"max ref {ref.abs().max():.3e}")
    print("  err per slot:", [f"{err[:, s * cin:(s + 1) * cin].max():.2e}" for s in range(9)])
    print("  err per o (first 8):", [f"{err[o].max():.2e}" for o in range(8)])
    r = (dw.double() / ref)
    print("  ratio sample:", r[0, :6].tolist())
    print("  db err", (db.double() - dpre.reshape(-1, cout).sum(0).double()).abs().max().item())
