"""Topology precompute against the reference's own cached
outputs (``spirals.pkl`` / ``transforms.pkl``, bit-exact copies in
``tests/golden/topology_craniofacial.npz``).  CPU only.

* spirals: OpenMesh half-edge restatement, ``np.array_equal`` on all 4
  levels (compute_spirals.py:11-73; includes 4 non-manifold faces OpenMesh
  rejects at level 2);
* quadric edge collapse: kept-vertex set (the 0/1 down matrix) and the
  decimated faces identical on all 4 levels (mesh_simplification.py:43-188);
* up matrix (mesh_simplification.py:214-247): every row whose closest face
  is unique is identical (columns; values within 4 ulp); rows where several
  faces are exactly equally close pick by trimesh's R-tree traversal order
  (libspatialindex, unpinned) -- for the kept vertices (distance 0) every
  choice up-samples to the identical position, the few off-surface ties are
  counted and bounded.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import cfsd_loader

cfsd_loader.load()
from craniofacialsd_vae_amd import precompute as PC  # noqa: E402
from craniofacialsd_vae_amd import topology  # noqa: E402


@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_spirals_bit_exact(topo_npz, level):
    m = PC.HalfedgeMesh(topo_npz[f"pos_{level}"], topo_npz[f"face_{level}"])
    sp_ = PC.extract_spirals(m, 9)
    assert np.array_equal(sp_, topo_npz[f"spiral_{level}"].astype(np.int64))
    if level == 2:
        assert len(m.rejected) == 4  # non-manifold faces OpenMesh refuses


def test_preprocess_spiral_kdtree_fallback():
    """A mesh too small for 9-long rings takes the KD-tree branch
    (compute_spirals.py:54-59): k nearest points, the vertex itself first."""
    pos = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 1]], np.float64)
    faces = np.array([[0, 1, 2], [0, 2, 3], [0, 3, 1], [1, 3, 2]])
    s = PC.preprocess_spiral(faces, 5, pos)
    assert s.shape == (5, 5)
    assert (s[:, 0] == np.arange(5)).all()


@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_quadric_collapse_matches_transforms(topo_npz, level):
    faces, kept = PC.quadric_edge_collapse(topo_npz[f"pos_{level}"], topo_npz[f"face_{level}"], 4)
    ref = topo_npz[f"down_{level}_col"][np.argsort(topo_npz[f"down_{level}_row"])]
    assert np.array_equal(kept, ref)
    assert np.array_equal(faces, topo_npz[f"face_{level + 1}"])
    assert np.array_equal(topo_npz[f"pos_{level}"][kept], topo_npz[f"pos_{level + 1}"])


@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_upsampling_matrix(topo_npz, level):
    z = topo_npz
    r, c, v, shape = PC.upsampling_matrix(z[f"pos_{level}"], z[f"pos_{level + 1}"], z[f"face_{level + 1}"])
    assert tuple(shape) == tuple(z[f"up_{level}_shape"])
    # the reference's CSC entry order: by column, then row
    assert np.all(np.diff(c) >= 0)
    A = sp.csr_matrix((v, (r, c)), shape=shape)
    B = sp.csr_matrix((z[f"up_{level}_val"], (z[f"up_{level}_row"], z[f"up_{level}_col"])), shape=shape)
    same = np.array([np.array_equal(A.indices[A.indptr[i]:A.indptr[i + 1]],
                                    B.indices[B.indptr[i]:B.indptr[i + 1]]) for i in range(shape[0])])
    kept = np.zeros(shape[0], bool)
    kept[z[f"down_{level}_col"]] = True
    assert np.abs((A - B)[same]).max() <= 4.8e-7
    P = z[f"pos_{level + 1}"].astype(np.float64)
    d = np.abs(A @ P - B @ P).max(1)
    assert d[kept].max() == 0.0                     # distance-0 ties: same position
    assert (~same & ~kept).sum() <= 8                # off-surface ties (8/2/3/1 on the 4 levels)
    assert same.mean() > 0.78


def test_rw_laplacian_and_regions_match_fixture(topo_npz):
    z = topo_npz
    r, c, v = PC.rw_laplacian(z["face_0"], 17039)
    assert np.array_equal(r, z["lap_row"]) and np.array_equal(c, z["lap_col"])
    assert np.array_equal(v, z["lap_val"])
    fc = PC.feature_and_contour(z["template_colors"], z["face_0"].astype(np.int64))
    keys = [str(k) for k in z["region_keys"]]
    assert list(fc.keys()) == keys
    for i, k in enumerate(keys):
        assert fc[k]["feature"] == z[f"region_{i}_feature"].tolist()
        assert fc[k]["contour"] == z[f"region_{i}_contour"].tolist()


def test_ply_round_trip_and_template(tmp_path, topo_npz):
    z = topo_npz
    p = tmp_path / "t.ply"
    PC.write_ply(p, z["pos_0"], z["face_0"], z["template_colors"])
    tpl = PC.load_template(str(p))
    assert np.array_equal(tpl.pos, z["pos_0"]) and np.array_equal(tpl.faces, z["face_0"])
    assert len(tpl.feat_and_cont) == 15
    assert np.array_equal(tpl.laplacian[2], z["lap_val"])


def test_synthetic_hierarchy_builds():
    h = PC.build_hierarchy(*PC.torus())
    assert [h[f"pos_{l}"].shape[0] for l in range(5)] == [5120, 1280, 320, 80, 20]
    T = topology.DeviceTopology.from_npz(h, device="cpu")
    assert all(T.enc_select) and T.n_regions == 15
    for l in range(4):
        s = h[f"spiral_{l}"]
        assert s.shape == (T.n_verts[l], 9) and (s[:, 0] == np.arange(T.n_verts[l])).all()
        # every up row is a barycentric combination (rows sum to 1)
        u = sp.csr_matrix((h[f"up_{l}_val"], (h[f"up_{l}_row"], h[f"up_{l}_col"])),
                          shape=tuple(h[f"up_{l}_shape"]))
        assert np.abs(np.asarray(u.sum(1)).ravel() - 1).max() < 1e-5


def test_sampling_variants_r_weighted_and_edge_length():
    """f2 sampling variants (parity unpinned: trimesh/torch_geometric absent,
    no reference cache for these modes).  ``r_weighted`` (model_manager.py:191,
    mesh_simplification.py:50-59): region-weighted collapse costs, and the
    template's swap regions become feature + contour (the reference's in-place
    ``extend``); ``edge_length_weighted`` (:157-158) adds the edge length to
    each cost.  Both keep the level sizes and change which vertices survive."""
    pos, faces, col = PC.torus(n_major=40, n_minor=32)
    kw = dict(sampling_factors=(4, 4), seq_lengths=(9, 9))
    base = PC.build_hierarchy(pos, faces, col, **kw)
    rw = PC.build_hierarchy(pos, faces, col, sampling_type="r_weighted", **kw)
    el = PC.build_hierarchy(pos, faces, col, edge_length_weighted=True, **kw)
    tpl = PC.Template(pos, faces, col)
    for i, k in enumerate(base["region_keys"]):
        fc = tpl.feat_and_cont[k]
        assert list(base[f"region_{i}_feature"]) == list(fc["feature"])
        assert list(rw[f"region_{i}_feature"]) == list(fc["feature"]) + list(fc["contour"])
        assert list(rw[f"region_{i}_contour"]) == list(fc["contour"])
    for h in (rw, el):
        assert [h[f"pos_{l}"].shape[0] for l in range(3)] == [1280, 320, 80]
    assert not np.array_equal(rw["down_0_col"], base["down_0_col"])
    assert not np.array_equal(el["down_0_col"], base["down_0_col"])
