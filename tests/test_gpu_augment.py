"""Spectral-interpolation augmentation on the GPU (reference
utils.py:238-267, data_loading.py:292-374).

* eigendecomposition: the device eigenpairs of the template's combinatorial
  Laplacian satisfy L U = U diag(s) and U^T U = I (fp32 1e-4), and the
  smallest eigenvalues equal scipy's ARPACK shift-invert solve (rel 1e-6);
* the batched GEMM + cfsd_spectral_blend path equals the oracle's float64
  restatement of ``spectral_interpolation`` on the demo meshes with the same
  U and the same random coefficients (rel 1e-4 of the mesh scale; fp32);
* ``augment`` produces the reference's per-class counts (balanced mode).
Level-1 template (4260 vertices) keeps the dense eigensolve in test time."""
import numpy as np
import pytest
import scipy.sparse.linalg as sla
import torch

import cfsd_loader
import recipe
from oracle import cfsd_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    cfsd_loader.load()
    from craniofacialsd_vae_amd import augment, precompute
    return augment, precompute


@pytest.fixture(scope="module")
def eig(mods, topo_npz):
    A, P = mods
    faces = topo_npz["face_1"].astype(np.int64)
    n = int(topo_npz["pos_1"].shape[0])
    s, u = A.laplacian_eigendecomposition(faces, n, k=200, device="cuda")
    return faces, n, s, u


def test_eigenpairs(mods, eig):
    A, P = mods
    faces, n, s, u = eig
    L = P.combinatorial_laplacian(faces, n)
    U = u.double().cpu().numpy()
    res = np.abs(L @ U - U * s[None]).max()
    assert res <= 1e-4 * max(1.0, float(np.abs(s).max()))
    assert np.abs(U.T @ U - np.eye(U.shape[1])).max() <= 1e-4
    ref = np.sort(sla.eigsh(L.astype(np.float64), k=12, sigma=-1e-3, which="LM")[0])
    np.testing.assert_allclose(s[:12], ref, rtol=1e-6, atol=1e-9)


def test_spectral_interpolation_vs_oracle(mods, eig, topo_npz):
    A, _ = mods
    faces, n, s, u = eig
    # demo meshes restricted to the level-1 vertices (the level-1 template's graph)
    sel = topo_npz["down_0_col"][np.argsort(topo_npz["down_0_row"])]
    m = recipe.load_meshes()["verts"][:, sel]
    rs = np.random.RandomState(0)
    pairs = [(0, 1), (2, 3), (4, 5), (6, 11)]
    vals = rs.normal(0.5, 0.5, size=(len(pairs), u.shape[1])).astype(np.float32)
    x1 = torch.from_numpy(np.stack([m[a] for a, _ in pairs])).float().cuda()
    x2 = torch.from_numpy(np.stack([m[b] for _, b in pairs])).float().cuda()
    got = A.spectral_interpolation(u, x1, x2, torch.from_numpy(vals).cuda()).cpu().numpy()
    U = u.double().cpu().numpy()
    for i, (a, b) in enumerate(pairs):
        ref = O.spectral_interpolation(U, m[a], m[b], vals[i])
        err = np.abs(got[i] - ref).max() / np.abs(ref).max()
        assert err <= 1e-4, f"pair {i}: rel {err}"
    # values == 0: the projection of x1 onto the spectral subspace
    z = A.spectral_interpolation(u, x1, x2, torch.zeros_like(torch.from_numpy(vals)).cuda()).cpu().numpy()
    ref = (U @ (U.T @ m[0].astype(np.float64)))
    assert np.abs(z[0] - ref).max() / np.abs(ref).max() <= 1e-4


def test_augment_counts(mods, eig, topo_npz):
    A, _ = mods
    faces, n, s, u = eig
    sel = topo_npz["down_0_col"][np.argsort(topo_npz["down_0_row"])]
    m = torch.from_numpy(recipe.load_meshes()["verts"][:, sel]).float().cuda()
    labels = list("nnnaaacccmmm")
    aug, cls, (i1, i2, _, _) = A.augment(u, m, labels, aug_factor=5, balanced=True, seed=1, batch=7)
    exp = A.balanced_counts(labels, 5, True)
    assert {c: cls.count(c) for c in set(cls)} == {c: v for c, v in exp.items() if v}
    assert aug.shape == (len(cls), n, 3) and torch.isfinite(aug).all()
    assert all(labels[a] == labels[b] and a != b for a, b in zip(i1, i2))


# ------------------------------------------------ full template, k = 1000 (C5)
@pytest.fixture(scope="module")
def eig_full(mods, topo_npz, tmp_path_factory):
    """The reference's eigendecomposition size (data_loading.py:309-310:
    k = 1000 of the 17 039-vertex template), device fp64, cached in a file
    and read back from the cache."""
    A, _ = mods
    faces = topo_npz["face_0"].astype(np.int64)
    n = int(topo_npz["pos_0"].shape[0])
    cache = str(tmp_path_factory.mktemp("eig") / "laplacian_eig_k1000.npz")
    s, u = A.laplacian_eigendecomposition(faces, n, k=1000, device="cuda", cache=cache)
    s2, u2 = A.laplacian_eigendecomposition(faces, n, k=1000, device="cuda", cache=cache)
    assert np.array_equal(s, s2) and torch.equal(u.cpu(), u2.cpu())
    return faces, n, s, u


def test_full_template_eigenpairs(mods, eig_full):
    A, P = mods
    faces, n, s, u = eig_full
    assert u.shape == (17039, 1000)
    L = P.combinatorial_laplacian(faces, n)
    U = u.double().cpu().numpy()
    res = np.abs(L @ U - U * s[None]).max()
    assert res <= 1e-4 * max(1.0, float(np.abs(s).max())), res
    assert np.abs(U.T @ U - np.eye(U.shape[1])).max() <= 1e-4
    ref = np.sort(sla.eigsh(L.astype(np.float64), k=12, sigma=-1e-3, which="LM")[0])
    np.testing.assert_allclose(s[:12], ref, rtol=1e-6, atol=1e-9)
    assert np.all(np.diff(s) >= -1e-9)  # ascending: the k SMALLEST (eigsh which='SM')


def test_full_template_spectral_interpolation_vs_oracle(mods, eig_full):
    """C5's generator at full size: batched GEMMs + cfsd_spectral_blend ==
    the oracle's float64 spectral_interpolation (utils.py:256-267) with the
    same U and coefficients, on demo pairs of the 17 039-vertex template."""
    A, _ = mods
    faces, n, s, u = eig_full
    m = recipe.load_meshes()["verts"]
    rs = np.random.RandomState(1)
    pairs = [(0, 1), (2, 3), (4, 5), (6, 11), (7, 9)]
    vals = rs.normal(0.5, 0.5, size=(len(pairs), u.shape[1])).astype(np.float32)
    x1 = torch.from_numpy(np.stack([m[a] for a, _ in pairs])).float().cuda()
    x2 = torch.from_numpy(np.stack([m[b] for _, b in pairs])).float().cuda()
    got = A.spectral_interpolation(u, x1, x2, torch.from_numpy(vals).cuda()).cpu().numpy()
    U = u.double().cpu().numpy()
    for i, (a, b) in enumerate(pairs):
        ref = O.spectral_interpolation(U, m[a], m[b], vals[i])
        err = np.abs(got[i] - ref).max() / np.abs(ref).max()
        assert err <= 1e-4, f"pair {i}: rel {err}"
