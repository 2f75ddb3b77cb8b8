"""Convert the reference's demo geometry into plain-array fixtures.

TEST INFRASTRUCTURE — runs only in the build container (it reads
``/root/reference``, which does not exist on the GPU box).  Output:

* ``topology_craniofacial.npz`` — everything the training step consumes that
  the reference precomputes once (``model_manager.py:176-238``,
  ``utils.py:77-144``):
    - ``spiral_{l}``      int32 [V_l, 9], bit-exact copy of ``spirals.pkl``
    - ``down_{l}_{row,col,val,shape}`` COO of ``transforms.pkl`` in FILE order
    - ``up_{l}_{row,col,val,shape}``
    - ``face_{l}`` int32 [F_l, 3] (level 0 from ``template.ply``), ``pos_{l}``
    - ``template_colors`` uint8 [V, 4]
    - ``region_keys`` (15 colour strings, first-appearance order),
      ``region_{i}_feature`` / ``region_{i}_contour`` int32
    - ``lap_{row,col,val}`` the random-walk Laplacian COO (``utils.py:88-89``)
* ``demo_meshes.npz`` — the 12 demo OBJ vertex arrays (sorted file names)
  and ``norm_mean``/``norm_std`` from ``norm.pt``.

Pickles are read with :mod:`safe_unpickle` (no code from the file runs) and
``norm.pt`` with ``torch.load(weights_only=True)``.

Restated (the third-party code is absent from the image):
* trimesh ``edges_unique`` (version unpinned in ``install_env.sh``): sorted
  face edges, de-duplicated and ordered by trimesh's row hash
  ``min ^ (max << 32)``, i.e. by (max, min).
* torch_geometric ``FaceToEdge`` + ``get_laplacian(normalization='rw')``:
  undirected coalesced edges, off-diagonal ``-1/deg(row)``, then the
  ``N`` unit diagonal entries appended (``add_self_loops``).
Both are "parity unpinned" against the reference's own runs (no reference
test pins them); the region key order is checked against
``region_ldas.pkl``'s key order by ``make_golden.py``.
"""
import os
import sys
from collections import Counter

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import refcache as safe_unpickle  # noqa: E402

REF = os.environ.get("CFSD_REFERENCE", "/root/reference")
DEMO = os.path.join(REF, "demo_files")


def read_ply(path):
    """Binary little-endian PLY as written by trimesh (template.ply header)."""
    with open(path, "rb") as f:
        raw = f.read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    header = raw[:end].decode("ascii").splitlines()
    nv = nf = 0
    for ln in header:
        if ln.startswith("element vertex"):
            nv = int(ln.split()[-1])
        if ln.startswith("element face"):
            nf = int(ln.split()[-1])
    assert "format binary_little_endian 1.0" in header
    vdt = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                    ("r", "u1"), ("g", "u1"), ("b", "u1"), ("a", "u1")])
    v = np.frombuffer(raw, dtype=vdt, count=nv, offset=end)
    off = end + nv * vdt.itemsize
    fdt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
    f = np.frombuffer(raw, dtype=fdt, count=nf, offset=off)
    assert (f["n"] == 3).all()
    pos = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float32)
    col = np.stack([v["r"], v["g"], v["b"], v["a"]], 1).astype(np.uint8)
    return pos, f["i"].astype(np.int64), col


def trimesh_edges_unique(faces):
    e = faces[:, [0, 1, 1, 2, 2, 0]].reshape(-1, 2)
    e = np.sort(e, axis=1)
    h = e[:, 0].astype(np.int64) ^ (e[:, 1].astype(np.int64) << 32)
    _, first = np.unique(h, return_index=True)
    return e[first]


def feature_and_contour(colors, faces):
    """Restatement of ``utils.extract_feature_and_contour_from_colour``
    (``utils.py:93-135``) including the early ``break`` quirk (:128-129)."""
    edges = trimesh_edges_unique(faces)
    nbrs = [dict() for _ in range(len(colors))]  # networkx adjacency order
    for a, b in edges.tolist():
        nbrs[a][b] = None
        nbrs[b][a] = None
    rings = [list(d.keys()) for d in nbrs]
    keys = [str(c) for c in colors]
    features = {}
    for index in range(len(colors)):
        k = keys[index]
        if k not in features:
            features[k] = {"feature": [], "contour": []}
        contour = any(not np.array_equal(colors[index], colors[r])
                      for r in rings[index])
        features[k]["contour" if contour else "feature"].append(index)
    remove = []
    for key, feat in features.items():
        if len(feat["feature"]) < 3:
            remove.append(key)
            for idx in feat["feature"]:
                counts = Counter([keys[r] for r in rings[idx]])
                mc = counts.most_common(1)[0][0]
                if mc == key:
                    break
                features[mc]["feature"].append(idx)
                features[mc]["contour"].append(idx)
    for e in remove:
        features.pop(e, None)
    return features


def rw_laplacian(faces, n):
    e = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [0, 2]]])
    e = np.concatenate([e, e[:, ::-1]])  # to_undirected
    lin = np.unique(e[:, 0].astype(np.int64) * n + e[:, 1])  # coalesce
    row, col = lin // n, lin % n
    keep = row != col
    row, col = row[keep], col[keep]
    deg = np.bincount(row, minlength=n).astype(np.float32)
    dinv = (np.float32(1.0) / deg).astype(np.float32)
    dinv[np.isinf(dinv)] = 0
    w = -(dinv[row] * np.float32(1.0))
    ar = np.arange(n)
    return (np.concatenate([row, ar]).astype(np.int32),
            np.concatenate([col, ar]).astype(np.int32),
            np.concatenate([w, np.ones(n, np.float32)]).astype(np.float32))


def read_obj_vertices(path):
    vs = []
    with open(path) as f:
        for ln in f:
            if ln.startswith("v "):
                vs.append([float(t) for t in ln.split()[1:4]])
    return np.asarray(vs, dtype=np.float32)


def main():
    out = {}
    pos, faces, colors = read_ply(os.path.join(DEMO, "template.ply"))
    spirals = safe_unpickle.load(os.path.join(DEMO, "spirals.pkl"))
    low, down, up = safe_unpickle.load(os.path.join(DEMO, "transforms.pkl"))
    assert len(spirals) == len(down) == len(up) == len(low)
    out["n_levels"] = np.int32(len(spirals))
    out["pos_0"] = pos
    out["face_0"] = faces.astype(np.int32)
    out["template_colors"] = colors
    for l in range(len(spirals)):
        out[f"spiral_{l}"] = spirals[l].numpy().astype(np.int32)
        assert (out[f"spiral_{l}"].astype(np.int64) == spirals[l].numpy()).all()
        for name, tr in (("down", down[l]), ("up", up[l])):
            idx = tr["indices"].numpy()
            out[f"{name}_{l}_row"] = idx[0].astype(np.int32)
            out[f"{name}_{l}_col"] = idx[1].astype(np.int32)
            out[f"{name}_{l}_val"] = tr["values"].numpy().astype(np.float32)
            out[f"{name}_{l}_shape"] = np.asarray(tr["size"], np.int64)
        out[f"pos_{l + 1}"] = low[l]["pos"].numpy().astype(np.float32)
        out[f"face_{l + 1}"] = low[l]["face"].numpy().T.astype(np.int32)
    feats = feature_and_contour(colors, faces)
    keys = list(feats.keys())
    out["region_keys"] = np.asarray(keys)
    for i, k in enumerate(keys):
        out[f"region_{i}_feature"] = np.asarray(feats[k]["feature"], np.int32)
        out[f"region_{i}_contour"] = np.asarray(feats[k]["contour"], np.int32)
    r, c, v = rw_laplacian(faces, len(pos))
    out["lap_row"], out["lap_col"], out["lap_val"] = r, c, v
    np.savez_compressed(os.path.join(HERE, "topology_craniofacial.npz"), **out)

    names = sorted(f for f in os.listdir(os.path.join(DEMO, "meshes"))
                   if f.endswith(".obj"))
    meshes = np.stack([read_obj_vertices(os.path.join(DEMO, "meshes", f))
                       for f in names])
    norm = torch.load(os.path.join(DEMO, "norm.pt"), weights_only=True)
    np.savez_compressed(os.path.join(HERE, "demo_meshes.npz"),
                        names=np.asarray(names), verts=meshes,
                        norm_mean=norm["mean"].numpy(),
                        norm_std=norm["std"].numpy())
    print("levels", [out[f"spiral_{l}"].shape for l in range(len(spirals))])
    print("regions", len(keys), [len(feats[k]["feature"]) for k in keys])
    print("laplacian nnz", len(r), "meshes", meshes.shape)


if __name__ == "__main__":
    main()
