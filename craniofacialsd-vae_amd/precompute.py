"""Topology precompute without OpenMesh / trimesh / torch_geometric.

The reference builds its static geometry once, through third-party packages
that are absent from this image, and caches it in ``spirals.pkl`` /
``transforms.pkl`` (``model_manager.py:176-230``):

* spirals: ``compute_spirals.py:11-73`` walks OpenMesh one-rings
  (``mesh.vv()``) ring by ring, with a KD-tree fallback;
* down/up-sampling: ``mesh_simplification.py:43-247`` (quadric edge
  collapse -> 0/1 down matrix; barycentric projection on the closest face of
  the decimated mesh -> 3-tap up matrix);
* template: ``utils.py:77-144`` (PLY load, colour segmentation into swap
  regions, FaceToEdge edges, random-walk Laplacian).

This module restates all of it in NumPy so a new template (e.g. the body
topology of config C4, or the synthetic ~5k hierarchy the bench reports)
can be prepared on a host with no third-party mesh library.  The spiral
walk reproduces OpenMesh's half-edge connectivity exactly -- the order in
which ``PolyConnectivity::add_face`` links half-edges and picks each
vertex's outgoing half-edge decides where every clockwise one-ring starts --
so the spirals are bit-exact to ``spirals.pkl`` (``tests/test_precompute.py``).
"""
import heapq
import math
from collections import Counter

import numpy as np

from .topology import DeviceTopology


# ============================================================== half-edge mesh
class HalfedgeMesh:
    """OpenMesh ``TriMesh(points, faces)`` connectivity (ArrayKernel +
    PolyConnectivity), restated: the same half-edge numbering (edge e owns
    half-edges 2e, 2e+1), the same ``add_face`` linking, boundary handling,
    and rejection of non-manifold faces ("complex vertex/edge", "patch
    re-linking failed": the face is skipped, as OpenMesh does)."""

    def __init__(self, points, faces):
        self.points = np.asarray(points, np.float64)
        n = len(self.points)
        self.v_he = [-1] * n          # outgoing half-edge of each vertex
        self.to = []                  # to-vertex of each half-edge
        self.nxt = []
        self.prv = []
        self.fac = []                 # face of each half-edge (-1: boundary)
        self.n_faces = 0
        self.rejected = []
        for f in np.asarray(faces, np.int64).tolist():
            vs = [v for v in f if v >= 0]
            if len(vs) >= 3 and not self.add_face(vs):
                self.rejected.append(f)

    # -- basic queries
    def _boundary_v(self, v):
        h = self.v_he[v]
        return not (h != -1 and self.fac[h] != -1)

    def _cw(self, h):                 # cw_rotated_halfedge_handle
        return self.nxt[h ^ 1]

    def _outgoing(self, v):
        """Outgoing half-edges of v, clockwise from v_he[v] (OpenMesh voh)."""
        start = self.v_he[v]
        if start == -1:
            return
        h = start
        while True:
            yield h
            h = self._cw(h)
            if h == start or h == -1:
                return

    def _find(self, a, b):
        for h in self._outgoing(a):
            if self.to[h] == b:
                return h
        return -1

    def _new_edge(self, a, b):
        h0 = len(self.to)
        self.to += [b, a]
        self.nxt += [-1, -1]
        self.prv += [-1, -1]
        self.fac += [-1, -1]
        return h0

    def _set_next(self, h, n):
        self.nxt[h] = n
        self.prv[n] = h

    def _adjust_outgoing(self, v):
        for h in self._outgoing(v):
            if self.fac[h] == -1:
                self.v_he[v] = h
                return

    def add_face(self, vh):
        n = len(vh)
        he = [-1] * n
        new = [False] * n
        adj = [False] * n
        for i in range(n):
            ii = (i + 1) % n
            if not self._boundary_v(vh[i]):
                return False                                   # complex vertex
            he[i] = self._find(vh[i], vh[ii])
            new[i] = he[i] == -1
            if not new[i] and self.fac[he[i]] != -1:
                return False                                   # complex edge
        cache = []
        for i in range(n):
            ii = (i + 1) % n
            if not new[i] and not new[ii]:
                inner_prev, inner_next = he[i], he[ii]
                if self.nxt[inner_prev] != inner_next:
                    # re-link a whole patch: find a free gap
                    outer_prev = inner_next ^ 1
                    bprev = outer_prev
                    while True:
                        bprev = self.nxt[bprev] ^ 1
                        if self.fac[bprev] == -1:
                            break
                    bnext = self.nxt[bprev]
                    if bprev == inner_prev:
                        return False                           # re-linking failed
                    patch_start = self.nxt[inner_prev]
                    patch_end = self.prv[inner_next]
                    cache += [(bprev, patch_start), (patch_end, bnext), (inner_prev, inner_next)]
        for i in range(n):
            if new[i]:
                he[i] = self._new_edge(vh[i], vh[(i + 1) % n])
        fh = self.n_faces
        self.n_faces += 1
        for i in range(n):
            ii = (i + 1) % n
            v = vh[ii]
            inner_prev, inner_next = he[i], he[ii]
            kind = (1 if new[i] else 0) | (2 if new[ii] else 0)
            if kind:
                outer_prev, outer_next = inner_next ^ 1, inner_prev ^ 1
                if kind == 1:      # prev is new, next is old
                    bprev = self.prv[inner_next]
                    cache.append((bprev, outer_next))
                    self.v_he[v] = outer_next
                elif kind == 2:    # next is new, prev is old
                    bnext = self.nxt[inner_prev]
                    cache.append((outer_prev, bnext))
                    self.v_he[v] = bnext
                else:              # both new
                    if self.v_he[v] == -1:
                        self.v_he[v] = outer_next
                        cache.append((outer_prev, outer_next))
                    else:
                        bnext = self.v_he[v]
                        bprev = self.prv[bnext]
                        cache += [(bprev, outer_next), (outer_prev, bnext)]
                cache.append((inner_prev, inner_next))
            else:
                adj[ii] = self.v_he[v] == inner_next
            self.fac[he[i]] = fh
        for h, nx in cache:
            self._set_next(h, nx)
        for i in range(n):
            if adj[i]:
                self._adjust_outgoing(vh[i])
        return True

    def vv(self, v):
        """One-ring of v, clockwise from the outgoing half-edge (``mesh.vv``)."""
        return [self.to[h] for h in self._outgoing(v)]


# ============================================================== spirals
def _next_ring(mesh, rings, last_ring, other):
    """``compute_spirals._next_ring`` (compute_spirals.py:11-31)."""
    res = []
    last_set, other_set, res_set = set(last_ring), set(other), set()

    def is_new(i):
        return i not in last_set and i not in other_set and i not in res_set

    for vh1 in last_ring:
        ring = rings[vh1]
        after_last_ring = False
        for vh2 in ring:
            if after_last_ring and is_new(vh2):
                res.append(vh2)
                res_set.add(vh2)
            if vh2 in last_set:
                after_last_ring = True
        for vh2 in ring:
            if vh2 in last_set:
                break
            if is_new(vh2):
                res.append(vh2)
                res_set.add(vh2)
    return res


def _kdtree_query(points, p, k):
    """sklearn ``KDTree(points).query(p, k)`` (exact k nearest, nearest first,
    squared distances summed in coordinate order; equal distances keep index
    order -- ties are unpinned by the reference)."""
    d = np.zeros(len(points))
    for c in range(points.shape[1]):
        d += (points[:, c] - p[c]) ** 2
    return np.argsort(d, kind="stable")[:k].tolist()


def extract_spirals(mesh, seq_length, dilation=1):
    """``compute_spirals.extract_spirals`` (compute_spirals.py:34-61)."""
    n = len(mesh.points)
    rings = [mesh.vv(v) for v in range(n)]
    spirals = []
    for vh0 in range(n):
        spiral = [vh0]
        last_ring = list(rings[vh0])
        next_ring = _next_ring(mesh, rings, last_ring, spiral)
        spiral.extend(last_ring)
        while len(spiral) + len(next_ring) < seq_length * dilation:
            if len(next_ring) == 0:
                break
            last_ring = next_ring
            next_ring = _next_ring(mesh, rings, last_ring, spiral)
            spiral.extend(last_ring)
        if len(next_ring) > 0:
            spiral.extend(next_ring)
        else:
            spiral = _kdtree_query(mesh.points, mesh.points[spiral[0]], seq_length * dilation)
        spirals.append(spiral[:seq_length * dilation][::dilation])
    return np.asarray(spirals, np.int64)


def preprocess_spiral(face, seq_length, vertices=None, dilation=1):
    """``compute_spirals.preprocess_spiral`` (compute_spirals.py:64-73):
    int64 ``[V, seq_length]`` spiral indices."""
    face = np.asarray(face)
    assert face.shape[1] == 3
    if vertices is None:
        vertices = np.ones([int(face.max()) + 1, 3])
    return extract_spirals(HalfedgeMesh(vertices, face), seq_length, dilation)


# ============================================================== edges / Laplacian
def face_to_edge(faces, n):
    """torch_geometric ``FaceToEdge`` + ``to_undirected``: both directions of
    every face edge, coalesced (sorted by (row, col), duplicates removed).
    Returns ``edge_index`` [2, E]."""
    f = np.asarray(faces, np.int64)
    e = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [0, 2]]])
    e = np.concatenate([e, e[:, ::-1]])
    lin = np.unique(e[:, 0] * n + e[:, 1])
    return np.stack([lin // n, lin % n])


def rw_laplacian(faces, n):
    """``get_laplacian(edge_index, normalization='rw')`` of the FaceToEdge
    graph (utils.py:88-89): off-diagonal -1/deg(row) in coalesced edge order,
    then the n unit diagonal entries.  COO (row, col, val) fp32."""
    row, col = face_to_edge(faces, n)
    keep = row != col
    row, col = row[keep], col[keep]
    deg = np.bincount(row, minlength=n).astype(np.float32)
    with np.errstate(divide="ignore"):
        dinv = (np.float32(1.0) / deg).astype(np.float32)
    dinv[np.isinf(dinv)] = 0
    w = -(dinv[row] * np.float32(1.0))
    ar = np.arange(n)
    return (np.concatenate([row, ar]).astype(np.int32), np.concatenate([col, ar]).astype(np.int32),
            np.concatenate([w, np.ones(n, np.float32)]).astype(np.float32))


def combinatorial_laplacian(faces, n):
    """``get_laplacian(edge_index, normalization=None)`` = D - A (utils.py:240),
    as a scipy CSR matrix (float64) for the spectral eigendecomposition."""
    import scipy.sparse as sp
    row, col = face_to_edge(faces, n)
    keep = row != col
    a = sp.csr_matrix((np.ones(int(keep.sum())), (row[keep], col[keep])), shape=(n, n))
    return (sp.diags(np.asarray(a.sum(1)).ravel()) - a).tocsr()


# ============================================================== template + regions
def read_ply(path):
    """Binary little-endian PLY with float xyz + uchar RGBA vertices and
    triangle faces (the reference's ``template.ply`` layout, loaded by
    ``trimesh.load_mesh(path, 'ply', process=False)`` at utils.py:78).
    Returns (pos float32 [V,3], faces int64 [F,3], colors uint8 [V,4])."""
    with open(path, "rb") as f:
        raw = f.read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    header = raw[:end].decode("ascii").splitlines()
    if "format binary_little_endian 1.0" not in header:
        raise ValueError(f"{path}: only binary little-endian PLY is supported")
    nv = nf = 0
    vprops = []
    in_vertex = False
    for ln in header:
        t = ln.split()
        if ln.startswith("element"):
            in_vertex = t[1] == "vertex"
            if t[1] == "vertex":
                nv = int(t[2])
            elif t[1] == "face":
                nf = int(t[2])
        elif ln.startswith("property") and in_vertex:
            vprops.append((t[-1], {"float": "<f4", "float32": "<f4", "double": "<f8", "uchar": "u1",
                                   "uint8": "u1"}[t[1]]))
    vdt = np.dtype(vprops)
    v = np.frombuffer(raw, dtype=vdt, count=nv, offset=end)
    off = end + nv * vdt.itemsize
    fdt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
    f = np.frombuffer(raw, dtype=fdt, count=nf, offset=off)
    if not (f["n"] == 3).all():
        raise ValueError(f"{path}: only triangle faces are supported")
    pos = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float32)
    names = v.dtype.names
    if "red" in names:
        col = np.stack([v["red"], v["green"], v["blue"], v["alpha"] if "alpha" in names else
                        np.full(nv, 255, np.uint8)], 1)
    elif "r" in names:
        col = np.stack([v["r"], v["g"], v["b"], v["a"] if "a" in names else np.full(nv, 255, np.uint8)], 1)
    else:
        col = np.full((nv, 4), 255, np.uint8)
    return pos, f["i"].astype(np.int64), col.astype(np.uint8)


def edges_unique(faces):
    """trimesh ``edges_unique``: sorted face edges de-duplicated in trimesh's
    row-hash order (``min ^ (max << 32)``, i.e. by (max, min)) -- the graph the
    colour segmentation walks (utils.py:105)."""
    e = np.asarray(faces, np.int64)[:, [0, 1, 1, 2, 2, 0]].reshape(-1, 2)
    e = np.sort(e, axis=1)
    h = e[:, 0] ^ (e[:, 1] << 32)
    _, first = np.unique(h, return_index=True)
    return e[first]


def feature_and_contour(colors, faces):
    """``utils.extract_feature_and_contour_from_colour`` (utils.py:93-135):
    region per distinct vertex colour (first-appearance order), split into
    feature and contour vertices; regions with < 3 feature vertices are
    folded into their neighbours' -- including the reference's early
    ``break`` (utils.py:128-129).  Returns {str(colour): {'feature': [...],
    'contour': [...]}} in the reference's key order."""
    colors = np.asarray(colors)
    nbrs = [dict() for _ in range(len(colors))]   # networkx adjacency order
    for a, b in edges_unique(faces).tolist():
        nbrs[a][b] = None
        nbrs[b][a] = None
    rings = [list(d.keys()) for d in nbrs]
    keys = [str(c) for c in colors]
    features = {}
    for index in range(len(colors)):
        k = keys[index]
        if k not in features:
            features[k] = {"feature": [], "contour": []}
        contour = any(not np.array_equal(colors[index], colors[r]) for r in rings[index])
        features[k]["contour" if contour else "feature"].append(index)
    remove = []
    for key, feat in features.items():
        if len(feat["feature"]) < 3:
            remove.append(key)
            for idx in feat["feature"]:
                mc = Counter([keys[r] for r in rings[idx]]).most_common(1)[0][0]
                if mc == key:
                    break
                features[mc]["feature"].append(idx)
                features[mc]["contour"].append(idx)
    for e in remove:
        features.pop(e, None)
    return features


class Template:
    """What ``utils.load_template`` (utils.py:77-90) returns, as arrays:
    pos [V,3] fp32, faces [F,3], colors [V,4], ``feat_and_cont`` (swap
    regions), ``laplacian`` (rw COO) and ``edge_index``."""

    def __init__(self, pos, faces, colors=None):
        self.pos = np.asarray(pos, np.float32)
        self.faces = np.asarray(faces, np.int64)
        n = len(self.pos)
        self.colors = None if colors is None else np.asarray(colors)
        self.feat_and_cont = feature_and_contour(self.colors, self.faces) if colors is not None else None
        self.edge_index = face_to_edge(self.faces, n)
        self.laplacian = rw_laplacian(self.faces, n)

    @property
    def num_nodes(self):
        return len(self.pos)


def load_template(path):
    """``utils.load_template`` (utils.py:77-90) without trimesh/torch_geometric."""
    pos, faces, colors = read_ply(path)
    return Template(pos, faces, colors)


# ============================================================== mesh simplification
def vertex_quadrics(pos, faces):
    """``MeshSimplifier._vertex_quadrics`` (mesh_simplification.py:122-141):
    per-face plane (SVD null vector of [v | 1], normalised by its normal),
    outer products accumulated per vertex in face order."""
    q = np.zeros((len(pos), 4, 4))
    pos = np.asarray(pos)
    for f in np.asarray(faces):
        verts = np.hstack((pos[f], np.array([1, 1, 1]).reshape(-1, 1)))
        _, _, v = np.linalg.svd(verts)
        eq = v[-1, :].reshape(-1, 1)
        eq = eq / (np.linalg.norm(eq[0:3]))
        o = np.outer(eq, eq)
        for k in range(3):
            q[f[k], :, :] += o
    return q


def quadric_edge_collapse(pos, faces, sampling_factor, region_weights=None, edge_length_weighted=False):
    """``MeshSimplifier.quadric_edge_collapse`` with ``_quadric_edge_collapse``
    and ``_edge_collapse_cost`` (mesh_simplification.py:43-167): greedy
    lowest-cost edge collapse (lazy heap, stale costs re-pushed) down to
    ceil(V / factor) vertices.  ``edge_length_weighted`` adds the edge's fp32
    length to the collapse cost before the region weighting (:157-160; an
    option of MeshSimplifier that ModelManager never sets).  Returns
    (new_faces [F',3], kept vertex indices ascending = the 0/1 down matrix's
    columns)."""
    pos = np.asarray(pos, np.float32)
    n = len(pos)
    desired = math.ceil(n / sampling_factor)
    quadrics = vertex_quadrics(pos, faces)
    ei = face_to_edge(faces, n).T
    edges = ei[ei[:, 0] < ei[:, 1]].copy()
    f = np.asarray(faces, np.int64).T.copy()           # [3, F] as the reference
    ones = np.array([1]).reshape(-1, 1)

    def cost(e0, e1):
        qs = quadrics[e0] + quadrics[e1]
        p0 = np.vstack((pos[e0].reshape(-1, 1), ones))
        p1 = np.vstack((pos[e1].reshape(-1, 1), ones))
        d0 = p0.T.dot(qs).dot(p0).item()
        d1 = p1.T.dot(qs).dot(p1).item()
        c = min([d0, d1])
        if edge_length_weighted:
            c += np.linalg.norm(pos[e0] - pos[e1])
        if region_weights is not None:
            c *= (region_weights[e0] + region_weights[e1]) / 2
        return c, d0, d1, qs

    h = [(cost(e[0], e[1])[0], i) for i, e in enumerate(edges)]
    heapq.heapify(h)
    nverts = n
    while nverts > desired:
        top_cost, idx = heapq.heappop(h)
        e0, e1 = edges[idx]
        if e0 == e1:
            continue
        c, d0, d1, qs = cost(e0, e1)
        if c > top_cost:
            heapq.heappush(h, (c, idx))
            continue
        keep, destroy = (e0, e1) if d0 < d1 else (e1, e0)
        np.place(f, f == destroy, keep)
        np.place(edges, edges == destroy, keep)
        quadrics[keep] = qs
        quadrics[destroy] = qs
        nverts -= 1
    a, b, c = f[0] == f[1], f[1] == f[2], f[2] == f[0]
    f = f[:, ~(a | b | c)]
    ft = f.T
    verts_left = np.unique(ft.flatten())
    mp = np.arange(0, ft.max() + 1)
    mp[verts_left] = np.arange(len(verts_left))
    return mp[ft.flatten()].reshape(-1, 3), verts_left


def _closest_on_triangles(tri, p):
    """Closest point on each triangle ``tri`` [K,3,3] to the matching point
    ``p`` [K,3] (Ericson's region test, as trimesh.triangles.closest_point)."""
    a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
    ab, ac, ap = b - a, c - a, p - a
    dot = lambda x, y: (x * y).sum(1)  # noqa: E731
    d1, d2 = dot(ab, ap), dot(ac, ap)
    bp = p - b
    d3, d4 = dot(ab, bp), dot(ac, bp)
    cp = p - c
    d5, d6 = dot(ab, cp), dot(ac, cp)
    vc = d1 * d4 - d3 * d2
    vb = d5 * d2 - d1 * d6
    va = d3 * d6 - d5 * d4
    with np.errstate(divide="ignore", invalid="ignore"):
        denom = 1.0 / (va + vb + vc)
        out = a + ab * (vb * denom)[:, None] + ac * (vc * denom)[:, None]
        done = np.zeros(len(p), bool)

        def put(mask, val):
            m = mask & ~done
            out[m] = val[m]
            done[m] = True

        put((d1 <= 0) & (d2 <= 0), a)
        put((d3 >= 0) & (d4 <= d3), b)
        put((vc <= 0) & (d1 >= 0) & (d3 <= 0), a + (d1 / (d1 - d3))[:, None] * ab)
        put((d6 >= 0) & (d5 <= d6), c)
        put((vb <= 0) & (d2 >= 0) & (d6 <= 0), a + (d2 / (d2 - d6))[:, None] * ac)
        put((va <= 0) & ((d4 - d3) >= 0) & ((d5 - d6) >= 0),
            b + ((d4 - d3) / ((d4 - d3) + (d5 - d6)))[:, None] * (c - b))
    return out


def closest_faces(pos, faces, points, merge_tol=1e-8, chunk=512):
    """``trimesh.proximity.closest_point(mesh, points)[2]`` restated: the
    candidate faces of each point are those whose bounding box meets the box
    of radius (distance to the nearest mesh vertex + tol.merge); the closest
    one wins, and when the best two are equally far (within tol.merge) and
    not on the surface, the one whose normal points most toward the query.
    Candidates are ranked in face order (trimesh's R-tree order is unpinned,
    so exact ties on the surface may pick a different, equivalent face)."""
    from scipy.spatial import cKDTree
    pos = np.asarray(pos, np.float64)
    pts = np.asarray(points, np.float64)
    tri = pos[np.asarray(faces)]
    lo, hi = tri.min(1), tri.max(1)
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    ln = np.linalg.norm(nrm, axis=1)
    nrm = nrm / np.where(ln > 0, ln, 1)[:, None]
    dv = cKDTree(pos).query(pts)[0] + merge_tol
    out = np.empty(len(pts), np.int64)
    for s in range(0, len(pts), chunk):
        p = pts[s:s + chunk]
        r = dv[s:s + chunk, None]
        hit = ((lo[None] <= (p + r)[:, None]) & (hi[None] >= (p - r)[:, None])).all(2)
        qi, fi = np.nonzero(hit)                       # face-ascending per point
        close = _closest_on_triangles(tri[fi], p[qi])
        vec = p[qi] - close
        d2 = (vec * vec).sum(1)
        starts = np.searchsorted(qi, np.arange(len(p)))
        ends = np.searchsorted(qi, np.arange(len(p)), side="right")
        for k in range(len(p)):
            seg = slice(starts[k], ends[k])
            dd = d2[seg]
            order = np.argsort(dd, kind="stable")[:2]
            best = order[0]
            if len(order) > 1:
                t = dd[order]
                if np.ptp(t) < merge_tol and np.all(np.abs(t) > merge_tol):
                    v = vec[seg][order] / np.sqrt(t)[:, None]
                    dots = (nrm[fi[seg][order]] * v).sum(1)
                    best = order[int(np.argmax(dots))]
            out[s + k] = fi[seg][best]
    return out


def upsampling_matrix(fine_pos, coarse_pos, coarse_faces):
    """``MeshSimplifier._get_upsampling_transformation``
    (mesh_simplification.py:214-247): every fine vertex is written in
    barycentric coordinates (Heidrich 2005, fp32 as the reference) of its
    closest coarse face.  COO (row, col, val) in the reference's CSC order
    (by column, then row) and shape (V_fine, V_coarse)."""
    fine_pos = np.asarray(fine_pos, np.float32)
    coarse_pos = np.asarray(coarse_pos, np.float32)
    coarse_faces = np.asarray(coarse_faces, np.int64)
    fids = closest_faces(coarse_pos, coarse_faces, fine_pos)
    tri = coarse_pos[coarse_faces[fids]]                    # [V, 3, 3] fp32
    u = tri[:, 1] - tri[:, 0]
    v = tri[:, 2] - tri[:, 0]
    n = np.cross(u, v)
    w = fine_pos - tri[:, 0]
    nn = (n * n).sum(1, dtype=np.float32)
    gamma = (np.cross(u, w) * n).sum(1, dtype=np.float32) / nn
    beta = (np.cross(w, v) * n).sum(1, dtype=np.float32) / nn
    alpha = np.float32(1) - gamma - beta
    rows = np.repeat(np.arange(len(fine_pos)), 3)
    cols = coarse_faces[fids].reshape(-1)
    vals = np.stack([alpha, beta, gamma], 1).reshape(-1).astype(np.float32)
    order = np.lexsort((rows, cols))
    return rows[order], cols[order], vals[order], (len(fine_pos), len(coarse_pos))


# ============================================================== hierarchy
def build_hierarchy(pos, faces, colors=None, sampling_factors=(4, 4, 4, 4), seq_lengths=(9, 9, 9, 9),
                    dilations=None, sampling_type="basic", edge_length_weighted=False):
    """The reference's precompute chain (``ModelManager._precompute_transformations``
    + ``_precompute_spirals``, model_manager.py:176-230) from a template:
    per sampling factor one quadric-edge-collapse level (0/1 down matrix) and
    its barycentric up matrix, then spirals of every level but the coarsest.
    Returns a dict in the ``topology_craniofacial.npz`` layout (``spiral_l``,
    ``down_l_{row,col,val,shape}``, ``up_l_*``, ``pos_l``, ``face_l``,
    ``region_*``, ``lap_*``) that ``DeviceTopology.from_npz`` consumes.

    ``sampling_type='r_weighted'`` weights the collapse costs by 1/|region|
    (mesh_simplification.py:50-59, model_manager.py:191).  The reference's
    weighting loop also extends each region's feature list by its contour in
    place (``feat_and_cont.extend``, :56-58) on the template object the
    ModelManager keeps, so after a fresh r_weighted precompute the swap
    regions (``region_i_feature``) are feature + contour; that is reproduced
    here (a run that loads a cached ``transforms.pkl`` has no such effect).
    ``edge_length_weighted`` is MeshSimplifier's length term (:157-158)."""
    n_lv = len(sampling_factors)
    dilations = dilations or [1] * n_lv
    tpl = Template(pos, faces, colors)
    out = {"n_levels": np.int32(n_lv), "pos_0": tpl.pos, "face_0": tpl.faces.astype(np.int32)}
    if colors is not None:
        out["template_colors"] = np.asarray(colors, np.uint8)
        keys = list(tpl.feat_and_cont.keys())
        out["region_keys"] = np.asarray(keys)
        for i, k in enumerate(keys):
            feat = list(tpl.feat_and_cont[k]["feature"])
            if sampling_type != "basic":  # the in-place extend of mesh_simplification.py:56-58
                feat = feat + list(tpl.feat_and_cont[k]["contour"])
            out[f"region_{i}_feature"] = np.asarray(feat, np.int32)
            out[f"region_{i}_contour"] = np.asarray(tpl.feat_and_cont[k]["contour"], np.int32)
    out["lap_row"], out["lap_col"], out["lap_val"] = tpl.laplacian
    cur_pos, cur_faces, cur_col = tpl.pos, tpl.faces, tpl.colors
    for l, factor in enumerate(sampling_factors):
        rw = None
        if sampling_type != "basic":
            if cur_col is None:
                raise ValueError("region-weighted sampling needs vertex colours")
            fc = feature_and_contour(cur_col, cur_faces)
            rw = np.ones(len(cur_pos))
            for k, f in fc.items():
                rw[f["feature"] + f["contour"]] = 1 / (len(f["feature"]) + len(f["contour"]))
        new_faces, kept = quadric_edge_collapse(cur_pos, cur_faces, factor, region_weights=rw,
                                                edge_length_weighted=edge_length_weighted)
        m = len(kept)
        out[f"down_{l}_row"] = np.arange(m, dtype=np.int32)
        out[f"down_{l}_col"] = kept.astype(np.int32)
        out[f"down_{l}_val"] = np.ones(m, np.float32)
        out[f"down_{l}_shape"] = np.asarray([m, len(cur_pos)], np.int64)
        new_pos = cur_pos[kept]
        r, c, v, shape = upsampling_matrix(cur_pos, new_pos, new_faces)
        out[f"up_{l}_row"], out[f"up_{l}_col"], out[f"up_{l}_val"] = (r.astype(np.int32), c.astype(np.int32), v)
        out[f"up_{l}_shape"] = np.asarray(shape, np.int64)
        out[f"spiral_{l}"] = preprocess_spiral(cur_faces, seq_lengths[l], cur_pos, dilations[l]).astype(np.int32)
        out[f"pos_{l + 1}"], out[f"face_{l + 1}"] = new_pos, new_faces.astype(np.int32)
        cur_pos, cur_faces = new_pos, new_faces
        cur_col = None if cur_col is None else cur_col[kept]
    return out


def torus(n_major=80, n_minor=64, r_major=1.0, r_minor=0.35, bumps=0.04, seed=0):
    """A closed, bumpy torus grid (n_major x n_minor vertices, 2 triangles per
    cell, consistent winding) with vertex colours that cut it into
    ``n_major // (n_major // 15)``-ish angular sectors -- a synthetic stand-in
    for a coloured template (vertex colour = swap region, utils.py:93-135)."""
    rs = np.random.RandomState(seed)
    u = np.arange(n_major) * 2 * np.pi / n_major
    v = np.arange(n_minor) * 2 * np.pi / n_minor
    uu, vv = np.meshgrid(u, v, indexing="ij")
    rr = r_minor * (1 + bumps * rs.randn(n_major, n_minor))
    x = (r_major + rr * np.cos(vv)) * np.cos(uu)
    y = (r_major + rr * np.cos(vv)) * np.sin(uu)
    zz = rr * np.sin(vv)
    pos = np.stack([x, y, zz], -1).reshape(-1, 3).astype(np.float32)
    idx = np.arange(n_major * n_minor).reshape(n_major, n_minor)
    i0 = idx
    i1 = np.roll(idx, -1, axis=0)
    i2 = np.roll(idx, -1, axis=1)
    i3 = np.roll(np.roll(idx, -1, axis=0), -1, axis=1)
    faces = np.concatenate([np.stack([i0, i1, i3], -1).reshape(-1, 3),
                            np.stack([i0, i3, i2], -1).reshape(-1, 3)]).astype(np.int64)
    sector = (np.arange(n_major) * 15 // n_major)
    palette = np.stack([(37 * np.arange(15)) % 256, (91 * np.arange(15) + 40) % 256,
                        (53 * np.arange(15) + 100) % 256, np.full(15, 255)], 1).astype(np.uint8)
    colors = palette[np.repeat(sector, n_minor)]
    return pos, faces, colors


_SYNTH_CACHE = {}


def synthetic_hierarchy(n_major=80, n_minor=64, device="cuda"):
    """The north-star's synthetic ~5k-vertex, 4-level hierarchy (5120 / 1280 /
    320 / 80 / 20 vertices, spiral length 9, 15 colour regions), built by this
    module from a bumpy torus, as a ``DeviceTopology``."""
    key = (n_major, n_minor)
    if key not in _SYNTH_CACHE:
        _SYNTH_CACHE[key] = build_hierarchy(*torus(n_major, n_minor))
    return DeviceTopology.from_npz(_SYNTH_CACHE[key], device=device)


def write_ply(path, pos, faces, colors=None):
    """Binary little-endian PLY (float xyz [+ uchar RGBA], int32 triangles)."""
    pos = np.asarray(pos, np.float32)
    faces = np.asarray(faces, np.int32)
    props = [("x", "<f4"), ("y", "<f4"), ("z", "<f4")]
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {len(pos)}",
            "property float x", "property float y", "property float z"]
    if colors is not None:
        props += [("red", "u1"), ("green", "u1"), ("blue", "u1"), ("alpha", "u1")]
        head += ["property uchar red", "property uchar green", "property uchar blue", "property uchar alpha"]
    head += [f"element face {len(faces)}", "property list uchar int vertex_indices", "end_header"]
    v = np.zeros(len(pos), np.dtype(props))
    v["x"], v["y"], v["z"] = pos[:, 0], pos[:, 1], pos[:, 2]
    if colors is not None:
        c = np.asarray(colors, np.uint8)
        v["red"], v["green"], v["blue"], v["alpha"] = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    f = np.zeros(len(faces), np.dtype([("n", "u1"), ("i", "<i4", (3,))]))
    f["n"], f["i"] = 3, faces
    with open(path, "wb") as fh:
        fh.write(("\n".join(head) + "\n").encode("ascii"))
        fh.write(v.tobytes())
        fh.write(f.tobytes())
