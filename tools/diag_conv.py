"""Locate wrong rows of a spiral-conv forward vs the oracle (GPU diagnostic)."""
import sys
import os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import cfsd_loader  # noqa
cfsd_loader.load()
from craniofacialsd_vae_amd import ops  # noqa
from oracle import cfsd_oracle as O  # noqa

z = np.load(os.path.join(ROOT, "tests", "golden", "topology_craniofacial.npz"))
for (cin, cout, level, bsz) in [(32, 32, 1, 2), (64, 32, 2, 3), (64, 32, 0, 4), (32, 32, 0, 4)]:
    sp = z[f"spiral_{level}"]
    g = torch.Generator().manual_seed(1)
    x = torch.randn(bsz, sp.shape[0], cin, generator=g)
    w = torch.randn(cout, 9 * cin, generator=g) * 0.1
    b = torch.randn(cout, generator=g) * 0.1
    ref = O.spiral_conv(x, sp, w, b).reshape(-1, cout).numpy()
    y = ops.spiral_conv_fwd(x.cuda(), torch.from_numpy(sp.astype(np.int32)).cuda(), w.cuda(), b.cuda(), 0)
    y = y.reshape(-1, cout).cpu().numpy()
    err = np.abs(y - ref).max(1)
    bad = np.nonzero(err > 1e-3)[0]
    tiles = np.unique(bad // 32)
    print(f"case {(cin, cout, level, bsz)} rows {len(ref)} bad rows {len(bad)} bad tiles {len(tiles)} of {(len(ref) + 31) // 32}")
    if len(bad):
        print("  first bad tiles", tiles[:20].tolist())
        t0 = tiles[0]
        rows = bad[bad // 32 == t0] % 32
        print("  rows-in-tile bad (tile %d):" % t0, rows.tolist())
        colbad = np.nonzero(np.abs(y - ref)[bad[0]] > 1e-3)[0]
        print("  cols bad in first bad row:", colbad.tolist()[:40])
        print("  sample y/ref:", y[bad[0], :4], ref[bad[0], :4])
