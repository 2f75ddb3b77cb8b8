"""Synthetic mesh hierarchies for the configurations whose template is not in
the reference snapshot.

TEST INFRASTRUCTURE (parity cases, not the product).  SURVEY §8d C4: the body
template (``configurations/body.yaml``: ``precomputed_bodies/star_template.ply``)
is absent, so C4 runs on a closed 130 x 53 torus grid of 6 890 vertices with
the body configuration's shape: sampling factors [4, 4, 4] -> levels
6890 / 1723 / 431 / 108, spiral length 9 at every level (``body.yaml:42-45``).

The arrays follow the schema of ``topology_craniofacial.npz`` (what
``spirals.pkl`` / ``transforms.pkl`` / the template hold in the reference):

* ``spiral_l`` [V_l, 9]: the vertex itself, then its neighbours ring by ring
  (level 0: the triangulated grid's 1-ring then 2-ring, nearest first; coarser
  levels: nearest kept vertices) -- the shape ``compute_spirals.py`` produces;
* ``down_l``: a 0/1 row selection keeping every 4th vertex (the QEM decimation
  matrices of ``mesh_simplification.py`` are 0/1 selections too);
* ``up_l``: 3 barycentric-like taps per fine vertex (inverse-distance weights
  of the 3 nearest coarse vertices, summing to 1), emitted in COLUMN order so
  rows are unsorted, as in the reference's transforms;
* ``lap``: the random-walk Laplacian I - D^-1 A of the level-0 edge graph
  (``utils.py:88-89`` semantics);
* 11 feature regions (latent 33 = 11 x 3 dims, ``_compute_latent_regions``).

Everything is a deterministic function of the grid size: no RNG, no files.
"""
import numpy as np

NU, NV = 130, 53
R_MAJOR, R_MINOR = 1.0, 0.4
SEQ = 9
N_REGIONS = 11


def torus_grid(nu=NU, nv=NV):
    """Vertex positions [nu*nv, 3] (id = i*nv + j) and triangle faces."""
    i, j = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    th, ph = 2 * np.pi * i / nu, 2 * np.pi * j / nv
    pos = np.stack([(R_MAJOR + R_MINOR * np.cos(ph)) * np.cos(th),
                    (R_MAJOR + R_MINOR * np.cos(ph)) * np.sin(th),
                    R_MINOR * np.sin(ph)], -1).reshape(-1, 3)
    a = (i * nv + j)
    b = (((i + 1) % nu) * nv + j)
    c = (((i + 1) % nu) * nv + (j + 1) % nv)
    d = (i * nv + (j + 1) % nv)
    faces = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3),
                            np.stack([a, c, d], -1).reshape(-1, 3)])
    return pos.astype(np.float64), faces.astype(np.int64)


def edges_of(faces):
    e = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]])
    e = np.sort(e, axis=1)
    return np.unique(e, axis=0)


def mesh_spirals(pos, faces, seq=SEQ):
    """Vertex, 1-ring, 2-ring (each ring nearest first, ties by index)."""
    n = len(pos)
    e = edges_of(faces)
    nbr = [[] for _ in range(n)]
    for a, b in e:
        nbr[a].append(b)
        nbr[b].append(a)
    out = np.empty((n, seq), np.int64)
    for v in range(n):
        ring1 = sorted(set(nbr[v]))
        ring2 = sorted(set(u for w in ring1 for u in nbr[w]) - set(ring1) - {v})
        order = [v]
        for ring in (ring1, ring2):
            d = np.linalg.norm(pos[ring] - pos[v], axis=1)
            order += [ring[k] for k in np.lexsort((ring, d))]
        out[v] = order[:seq]
    return out


def knn(pos_q, pos_ref, k):
    d = ((pos_q[:, None, :] - pos_ref[None, :, :]) ** 2).sum(-1)
    idx = np.argsort(d, axis=1, kind="stable")[:, :k]
    return idx, np.sqrt(np.take_along_axis(d, idx, 1))


def rw_laplacian(edges, n):
    """COO of I - D^-1 A (torch_geometric ``get_laplacian(..., 'rw')``)."""
    row = np.concatenate([edges[:, 0], edges[:, 1]])
    col = np.concatenate([edges[:, 1], edges[:, 0]])
    deg = np.bincount(row, minlength=n).astype(np.float64)
    val = -1.0 / deg[row]
    row = np.concatenate([row, np.arange(n)])
    col = np.concatenate([col, np.arange(n)])
    val = np.concatenate([val, np.ones(n)])
    return row, col, val.astype(np.float32)


def torus_topology(nu=NU, nv=NV, factors=(4, 4, 4), seq=SEQ, n_regions=N_REGIONS):
    pos, faces = torus_grid(nu, nv)
    levels = [np.arange(len(pos))]          # level l vertex -> level-0 vertex id
    for f in factors:
        levels.append(levels[-1][::f])
    npz = {"n_levels": np.int64(len(factors))}
    for l in range(len(factors)):
        p_l = pos[levels[l]]
        if l == 0:
            sp = mesh_spirals(pos, faces, seq)
        else:
            sp, _ = knn(p_l, p_l, seq)
            sp[:, 0] = np.arange(len(p_l))   # self first (distance 0 ties)
        npz[f"spiral_{l}"] = sp.astype(np.int64)
        m, n = len(levels[l + 1]), len(levels[l])
        # down: keep every factor-th vertex of level l
        npz[f"down_{l}_row"] = np.arange(m, dtype=np.int64)
        npz[f"down_{l}_col"] = np.arange(m, dtype=np.int64) * factors[l]
        npz[f"down_{l}_val"] = np.ones(m, np.float32)
        npz[f"down_{l}_shape"] = np.array([m, n], np.int64)
        # up: 3 inverse-distance taps from the coarse level, column-major COO
        idx, d = knn(p_l, pos[levels[l + 1]], 3)
        w = 1.0 / (d + 1e-3)
        w = (w / w.sum(1, keepdims=True)).astype(np.float32)
        rows = np.repeat(np.arange(n), 3)
        cols = idx.reshape(-1)
        vals = w.reshape(-1)
        o = np.lexsort((rows, cols))
        npz[f"up_{l}_row"], npz[f"up_{l}_col"], npz[f"up_{l}_val"] = rows[o], cols[o], vals[o]
        npz[f"up_{l}_shape"] = np.array([n, m], np.int64)
    lr, lc, lv = rw_laplacian(edges_of(faces), len(pos))
    npz["lap_row"], npz["lap_col"], npz["lap_val"] = lr, lc, lv
    # regions: n_regions bands around the major circle, on the outer half of
    # the tube, of varying width
    i, j = np.divmod(np.arange(len(pos)), nv)
    keys = []
    for k in range(n_regions):
        lo, hi = k * nu // n_regions, (k + 1) * nu // n_regions
        band = (i >= lo) & (i < hi) & ((j < nv // 4 + k) | (j > 3 * nv // 4))
        npz[f"region_{k}_feature"] = np.nonzero(band)[0].astype(np.int64)
        keys.append(f"band{k}")
    npz["region_keys"] = np.array(keys)
    return npz


def torus_meshes(n, nu=NU, nv=NV, seed=0):
    """``n`` deformed tori (smooth random bumps), normalised-scale fp32."""
    pos, _ = torus_grid(nu, nv)
    rs = np.random.RandomState(seed)
    i, j = np.divmod(np.arange(len(pos)), nv)
    th, ph = 2 * np.pi * i / nu, 2 * np.pi * j / nv
    out = []
    for _ in range(n):
        a = rs.randn(4) * 0.05
        bump = (a[0] * np.cos(2 * th) + a[1] * np.sin(3 * ph) + a[2] * np.cos(th + ph)
                + a[3] * np.sin(5 * th))
        p = pos * (1.0 + bump)[:, None] + rs.randn(len(pos), 3) * 0.01
        out.append((p - p.mean(0)) / p.std())
    return np.stack(out).astype(np.float32)
