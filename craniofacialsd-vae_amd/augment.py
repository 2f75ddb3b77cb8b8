"""Spectral-interpolation data augmentation on the GPU (the
source of config C5's 50k synthetic meshes).

Reference: ``utils.compute_laplacian_eigendecomposition`` (utils.py:238-241:
``eigsh`` of the combinatorial Laplacian D - A of the template graph, the k
smallest eigenpairs), ``spectral_interpolation`` / ``spectral_combination``
(utils.py:244-267) and ``MeshInMemoryDataset._augment`` (data_loading.py:
292-374: pairs drawn within a class and age group, balanced per class).

MI355X design: the eigenvectors U [V, k] are computed once (dense symmetric
eigensolver on the device, fp64, cached in the precomputed folder) and stay
resident; a batch of P pairs is then two plain GEMMs on hipBLASLt
(S = U^T [X1 | X2], out = U S4) around libcfsd's ``cfsd_spectral_blend``
(the per-coefficient alpha-blend of the first 30 components), so 50 000
augmented meshes are ~50 batched launches instead of 50 000 host loops.
"""
import os

import numpy as np
import torch

from . import ops
from .precompute import combinatorial_laplacian


def laplacian_eigendecomposition(faces, n, k=1000, device="cuda", cache=None):
    """The k smallest eigenpairs of the template's combinatorial Laplacian
    (utils.py:238-241).  Returns (eigenvalues [k] float64, U [n, k] float32,
    device).  ``eigsh(which='SM')`` is replaced by a dense fp64 eigensolve on
    the device (eigenvectors of repeated eigenvalues are a basis choice; each
    is unit-norm and L U = U diag(s))."""
    if cache is not None and os.path.exists(cache):
        d = np.load(cache)
        if d["u"].shape == (n, k):
            return d["s"], torch.from_numpy(d["u"]).to(device)
    L = torch.from_numpy(combinatorial_laplacian(faces, n).toarray()).to(device)
    s, u = torch.linalg.eigh(L)
    s, u = s[:k].cpu().numpy(), u[:, :k].float().contiguous()
    del L
    if cache is not None:
        np.savez(cache, s=s, u=u.cpu().numpy())
    return s, u


def spectral_interpolation(u, x1, x2, values, n_interp=30):
    """``spectral_interpolation`` (utils.py:256-267) for a batch of pairs:
    x1, x2 [P, V, 3] device fp32, values [P, k] (the reference draws
    N(0.5, 0.5) per coefficient); returns U S4, [P, V, 3]."""
    p, v, c = x1.shape
    k = u.shape[1]
    ut = u.t()
    s1 = torch.matmul(ut, x1.permute(1, 0, 2).reshape(v, p * c)).view(k, p, c).permute(1, 0, 2).contiguous()
    s2 = torch.matmul(ut, x2.permute(1, 0, 2).reshape(v, p * c)).view(k, p, c).permute(1, 0, 2).contiguous()
    s4 = ops.spectral_blend(s1, s2, values.contiguous(), n_interp)
    out = torch.matmul(u, s4.permute(1, 0, 2).reshape(k, p * c)).view(v, p, c).permute(1, 0, 2)
    return out.contiguous()


def spectral_combination_values(rng, pairs, k, swap_until=30):
    """0/1 coefficient selector of ``spectral_combination`` (utils.py:244-253):
    a third of the first 30 components taken from x2."""
    vals = np.zeros((pairs, k), np.float32)
    for i in range(pairs):
        vals[i, rng.choice(swap_until, swap_until // 3, replace=False)] = 1.0
    return vals


def choose_pairs(labels, ages, n_aug, rng, split_3years=True):
    """Pair draws of ``_augment`` (data_loading.py:314-358) as indices: for
    each class, ``n_aug[class]`` pairs of distinct meshes of the same class,
    from one age group (< 48 / >= 48 months, picked at random) when ages are
    known and both groups hold >= 2 meshes (the reference would fail on a
    group of < 2 at ``np.random.choice(len(group), 2, replace=False)``; here
    the whole class is used instead).  Returns (i1, i2, class, i) arrays,
    ``i`` = the draw's index within its class (the reference's name suffix,
    data_loading.py:342-371)."""
    labels = np.asarray(labels)
    ages = np.asarray(ages, np.float64) if ages is not None else None
    out = []
    for cl, n in n_aug.items():
        members = np.nonzero(labels == cl)[0]
        groups = [members]
        if split_3years and ages is not None:
            g = [members[ages[members] < 48], members[ages[members] >= 48]]
            if all(len(x) >= 2 for x in g):
                groups = g
        if n > 0 and len(members) < 2:
            raise ValueError(f"class {cl!r} has {len(members)} mesh(es): augmentation pairs need 2")
        for i in range(n):
            grp = groups[rng.randint(len(groups))]
            a, b = rng.choice(len(grp), 2, replace=False)
            out.append((grp[a], grp[b], cl, i))
    if not out:
        e = np.zeros(0, np.int64)
        return e, e, np.zeros(0, labels.dtype), e
    i1, i2, cls, idx = zip(*out)
    return np.asarray(i1), np.asarray(i2), np.asarray(cls), np.asarray(idx)


def balanced_counts(labels, aug_factor, balanced=True):
    """Augmented meshes per class (data_loading.py:314-335).  The classes are
    the merged ones ('b' paediatric folded into 'n', :322-324), but the
    balanced target divides by the number of class letters BEFORE the merge
    (``data_classes``, :314, :332), exactly as the reference does."""
    n_letters = len(set(labels))
    merged = ["n" if y == "b" else y for y in labels]
    classes = sorted(set(merged))
    cnt = {c: merged.count(c) for c in classes}
    if balanced:
        target = aug_factor * len(merged) // n_letters
        return {c: target - cnt[c] for c in classes}
    return {c: (aug_factor - 1) * cnt[c] for c in classes}


def augment(u, meshes, labels, ages=None, aug_factor=5, balanced=True, mode="spectral_interp", seed=0,
            batch=1024, n_interp=30, split_3years=True):
    """The augmented training meshes ``_augment`` writes to disk, produced on
    the device: meshes [N, V, 3] (raw, un-normalised, device fp32), labels [N]
    class letters.  Returns (augmented [M, V, 3] device, labels [M],
    (i1, i2, i, t)) with ``i`` the index of each draw within its class and
    ``t`` the interpolation values of mode 'interpolate' (else None).
    A negative balanced count (a class already above the target) draws
    nothing, as ``range(negative)`` does in the reference."""
    rng = np.random.RandomState(seed)
    counts = {c: max(0, n) for c, n in balanced_counts(labels, aug_factor, balanced).items()}
    i1, i2, cls, idx = choose_pairs(["n" if y == "b" else y for y in labels], ages, counts, rng,
                                    split_3years)
    aug, tv = _generate(u, meshes, i1, i2, mode, rng, batch, n_interp)
    return aug, list(cls), (i1, i2, idx, tv)


def _generate(u, meshes, i1, i2, mode, rng, batch=1024, n_interp=30):
    """The meshes of the pairs (i1, i2), ``batch`` pairs per launch group;
    coefficients drawn from ``rng`` batch by batch."""
    k = u.shape[1] if u is not None else 0
    outs, tvals = [], []
    for s in range(0, len(i1), batch):
        a, b = i1[s:s + batch], i2[s:s + batch]
        x1 = meshes[torch.as_tensor(a, device=meshes.device)]
        x2 = meshes[torch.as_tensor(b, device=meshes.device)]
        if mode == "spectral_interp":
            vals = rng.normal(loc=0.5, scale=0.5, size=(len(a), k)).astype(np.float32)
        elif mode == "spectral_comb":
            vals = spectral_combination_values(rng, len(a), k, n_interp)
        elif mode == "interpolate":  # utils.py:234-235: one value per pair, whole mesh
            tv = rng.uniform(size=(len(a), 1, 1)).astype(np.float32)
            tvals.append(tv.ravel())
            t = torch.as_tensor(tv, device=meshes.device)
            outs.append(x1 + t * (x2 - x1))
            continue
        else:
            raise ValueError(f"unknown augmentation_mode {mode!r}")
        outs.append(spectral_interpolation(u, x1, x2, torch.from_numpy(vals).to(meshes.device), n_interp))
    aug = torch.cat(outs) if outs else meshes[:0]
    return aug, (np.concatenate(tvals) if tvals else None)


def synthesize(u, meshes, labels, n, seed=0, mode="spectral_interp", batch=1024):
    """``n`` augmented meshes drawn as ``_augment`` draws them (same-class
    pairs, spectral interpolation) with the classes taking turns -- the
    generator of configuration C5's synthetic set (50 000 meshes from the
    demo meshes).  Returns (meshes [n, V, 3] device, class letters)."""
    rng = np.random.RandomState(seed)
    merged = ["n" if y == "b" else y for y in labels]
    classes = sorted(set(merged))
    per = {c: n // len(classes) + (1 if i < n % len(classes) else 0) for i, c in enumerate(classes)}
    i1, i2, cls, _ = choose_pairs(merged, None, per, rng, split_3years=False)
    aug, _ = _generate(u, meshes, i1, i2, mode, rng, batch)
    return aug, list(cls)
