import sys, numpy as np, torch
sys.path[:0] = ['tests/golden', '.']
import recipe, cfsd_loader
from oracle import cfsd_oracle as O
cfsd_loader.load()
from craniofacialsd_vae_amd import ops, topology
torch.set_num_threads(1)
print("threads", torch.get_num_threads(), torch.__config__.parallel_info().splitlines()[:6])
npz = recipe.load_topology()
T = O.Topology(npz)
D = topology.DeviceTopology.from_npz(npz)
for lv in [3, 0]:
    row, col, val, (m, n) = T.up[lv]
    g = torch.Generator().manual_seed(lv)
    x = torch.randn(2, n, 32, generator=g)
    out = O.pool(x, T.up[lv]).numpy()
    xs = x.numpy()
    seq = np.zeros((2, m, 32), np.float32)
    for k in range(len(row)):
        seq[:, row[k]] += xs[:, col[k]] * val[k]
    y = ops.spmm(D.up_csr[lv], x.cuda(), m).cpu().numpy()
    print(lv, "oracle!=seq", (seq != out).mean(), "hip!=seq", (y != seq).mean(), "hip!=oracle", (y != out).mean())
    bad = np.argwhere(y != seq)[:3]
    for b_, r, c in bad:
        ks = np.nonzero(row == r)[0]
        terms = [xs[b_, col[k], c] * val[k] for k in ks]
        print("  row", r, "ks", ks, "terms", terms, "seq", seq[b_, r, c], "hip", y[b_, r, c], "fma-ish", np.float32(np.float64(terms[0]) + terms[1]))
