"""Time the C5 augmentation pieces at full template size (GPU)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import cfsd_loader  # noqa: E402
import recipe  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import augment as A  # noqa: E402

z = recipe.load_topology()
t0 = time.perf_counter()
s, u = A.laplacian_eigendecomposition(z["face_0"].astype(np.int64), 17039, k=1000, device="cuda")
torch.cuda.synchronize()
print(f"eigh 17039 (k=1000): {time.perf_counter() - t0:.1f} s, s[:4] {s[:4]}, s[999] {s[999]:.4f}", flush=True)
m = torch.from_numpy(recipe.load_meshes()["verts"]).float().cuda()
labels = list("nnnaaacccmmm") * 1
for reps in (1, 3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    aug, cls, _ = A.augment(u, m, labels * 400, aug_factor=11, balanced=True, seed=2, batch=1024) \
        if False else A.augment(u, m.repeat(400, 1, 1), labels * 400, aug_factor=11, balanced=True, seed=2, batch=1024)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"augment: {aug.shape[0]} meshes in {el:.2f} s = {aug.shape[0] / el:.0f} meshes/s", flush=True)
