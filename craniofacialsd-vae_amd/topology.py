"""Mesh-hierarchy index tables, laid out for the gfx950 kernels.

The reference keeps its static geometry as int64 spiral tensors
(``spirals.pkl``), torch sparse-COO down/up transforms (``transforms.pkl``)
and a COO random-walk Laplacian (``utils.py:88-89``), and consumes them with
``index_select`` / ``scatter_add`` / ``sparse.mm`` every step
(``model_manager.py:176-230``).  Here they are converted ONCE into the int32
tables the kernels read:

* spirals -> int32 ``[V, S]`` plus the inverse-spiral CSR (rows r with
  ``idx[r, s] == u`` for every (u, s)) that makes the spiral backward a
  deterministic gather instead of an atomic scatter;
* a down transform that is a 0/1 row selection (the QEM decimation matrices,
  one nnz of value 1.0 per row) becomes a *row subset*: the Enblock conv is
  evaluated only at the kept vertices, bit-identical to conv -> Pool(down);
* other transforms -> CSR (row-sorted, per-row order = COO file order, i.e.
  the reference's sequential ``scatter_add`` order) and the transpose CSR
  for the backward;
* the Laplacian -> CSR in coalesced (row, col) order + transpose CSR;
* the feature-swap regions -> a ``[n_regions, V]`` uint8 membership mask.
"""
import numpy as np
import torch


def _i32(a):
    a = np.asarray(a)
    if a.size and (a.min() < np.iinfo(np.int32).min or a.max() > np.iinfo(np.int32).max):
        raise ValueError("index out of int32 range")
    return np.ascontiguousarray(a, dtype=np.int32)


def csr_from_coo(row, col, val, m):
    """Row-sorted CSR keeping, inside each row, the COO (file) order."""
    row = np.asarray(row, np.int64)
    order = np.argsort(row, kind="stable")
    ptr = np.zeros(m + 1, np.int64)
    np.add.at(ptr, row + 1, 1)
    ptr = np.cumsum(ptr)
    return _i32(ptr), _i32(np.asarray(col)[order]), np.ascontiguousarray(np.asarray(val, np.float32)[order])


def csr_transpose_from_coo(row, col, val, n):
    """CSR of the transpose (grouped by column), per-group order = COO order.
    Matches the accumulation order of ``index_add_`` over the nnz sequence
    (the autograd of ``index_select`` at ``model.py:53``)."""
    return csr_from_coo(col, row, val, n)


INV_HEAD = 4  # list entries kept inline per (u, s) key (CFSD_INV_HEAD)


def inverse_spiral(idx, vsrc):
    """CSR over keys (u, s): rows r with ``idx[r, s] == u``, r ascending.
    Returns (ptr [vsrc*S + 1], rows [R*S], head [vsrc*S, 4]) where ``head``
    holds the first four rows of every list (-1 when absent): one 16-B load
    per key covers 99.7 % of the lists of the craniofacial template (fan-in
    distribution per key at level 0: 0: 27 %, 1: 51 %, 2: 19 %, 3: 3.3 %,
    4: 0.25 %, more: 0.03 %), so the kernels rarely walk the CSR."""
    idx = np.asarray(idx, np.int64)
    r_count, s_len = idx.shape
    if idx.size and (idx.min() < 0 or idx.max() >= vsrc):
        raise ValueError("spiral index out of range")
    keys = (idx * s_len + np.arange(s_len)[None, :]).reshape(-1)  # r-major
    rows = np.repeat(np.arange(r_count), s_len)
    order = np.argsort(keys, kind="stable")
    ptr = np.zeros(vsrc * s_len + 1, np.int64)
    np.add.at(ptr, keys + 1, 1)
    ptr = np.cumsum(ptr)
    rows_sorted = rows[order]
    cnt = np.diff(ptr)
    head = -np.ones((vsrc * s_len, INV_HEAD), np.int64)
    for j in range(INV_HEAD):
        has = cnt > j
        head[has, j] = rows_sorted[ptr[:-1][has] + j]
    return _i32(ptr), _i32(rows_sorted), _i32(head)


def inverse_flat(idx, vsrc, max_width=16):
    """Per source vertex u, the flattened spiral positions p = r*S + s with
    ``idx[r, s] == u`` in ascending p (the order the reference's
    ``index_add_`` -- the autograd of ``index_select``, model.py:34 -- adds
    them), padded with -1 to a width that is a multiple of 4.  Returns
    ([vsrc, width] int32, width), or (None, 0) when some fan-in exceeds
    ``max_width`` (the row-subset backward then uses the inverse CSR)."""
    idx = np.asarray(idx, np.int64)
    flat = idx.reshape(-1)
    cnt = np.bincount(flat, minlength=vsrc)
    width = max(4, int(-(-cnt.max() // 4) * 4)) if flat.size else 4
    if width > max_width:
        return None, 0
    order = np.argsort(flat, kind="stable")  # p ascending inside each u
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    slot = np.arange(flat.size) - np.repeat(start, cnt)
    out = -np.ones((vsrc, width), np.int64)
    out[flat[order], slot] = order
    return _i32(out), width


def row_schedule(ptr, min_max_len=16):
    """Rows by decreasing length (stable), the visiting order of
    ``cfsd_spmm_csr_sched``; None when no row is longer than ``min_max_len``
    (the plain kernel then has no long fold to start early)."""
    cnt = np.diff(np.asarray(ptr, np.int64))
    if cnt.size == 0 or cnt.max() <= min_max_len:
        return None
    return _i32(np.argsort(-cnt, kind="stable"))


def scheduled_csr(ptr, col, val, order):
    """The CSR re-stored in visiting order ``order`` (``row_schedule``): returns
    (ptr_s [m+1], col_s, val_s, rows_s [m]) with slot i = row order[i], its
    entries in the original per-row order (``cfsd_spmm_sched_csr``)."""
    ptr = np.asarray(ptr, np.int64)
    order = np.asarray(order, np.int64)
    cnt = np.diff(ptr)[order]
    ptr_s = np.concatenate([[0], np.cumsum(cnt)])
    take = np.concatenate([np.arange(ptr[r], ptr[r + 1]) for r in order]) if len(order) else np.zeros(0, np.int64)
    return (_i32(ptr_s), _i32(np.asarray(col)[take]), np.ascontiguousarray(np.asarray(val, np.float32)[take]),
            _i32(order))


def uniform_rows(ptr, max_k=4):
    """k when every CSR row holds exactly k <= max_k entries (the barycentric
    up-sampling matrices: 3), else 0 (``cfsd_spmm_uniform`` needs no row_ptr)."""
    cnt = np.diff(np.asarray(ptr, np.int64))
    if cnt.size == 0 or cnt[0] < 1 or cnt[0] > max_k or not np.all(cnt == cnt[0]):
        return 0
    return int(cnt[0])


def selection_rows(row, col, val, m):
    """Return the kept-vertex list if the COO transform is a 0/1 row
    selection (exactly one entry of value 1.0 per row), else None."""
    row = np.asarray(row)
    if len(row) != m:
        return None
    if not np.array_equal(np.sort(row), np.arange(m)):
        return None
    if not np.all(np.asarray(val) == 1.0):
        return None
    sel = np.empty(m, np.int64)
    sel[row] = np.asarray(col)
    return sel


def coalesced_csr(row, col, val, n):
    """torch ``coalesce`` order (row, then col), duplicates summed."""
    row = np.asarray(row, np.int64)
    col = np.asarray(col, np.int64)
    lin = row * n + col
    uniq, inv = np.unique(lin, return_inverse=True)
    v = np.zeros(len(uniq), np.float32)
    np.add.at(v, inv, np.asarray(val, np.float32))
    r, c = uniq // n, uniq % n
    return r, c, v


class Level:
    """Device tables of one resolution level."""


def _dev(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


class DeviceTopology:
    """All static tables of a mesh hierarchy, resident on one device.

    ``spirals[l]`` int [V_l, S]; ``down[l]``/``up[l]`` COO triples
    ``(row, col, val, (M, N))``; ``lap`` optional COO triple of level 0;
    ``regions`` optional list of feature-vertex index arrays (swap keys).
    """

    def __init__(self, spirals, down, up, lap=None, regions=None, region_keys=None,
                 device="cuda"):
        self.device = torch.device(device)
        self.n_levels = len(spirals)
        self.seq = [int(np.asarray(s).shape[1]) for s in spirals]
        self.n_verts = [int(np.asarray(spirals[0]).shape[0])] + [int(d[3][0]) for d in down]
        self.region_keys = list(region_keys) if region_keys is not None else None
        self.spiral = []        # full spiral tables [V_l, S]
        self.spiral_inv = []    # inverse CSR of the full table
        self.spiral_flat = []   # (inverse_flat of the full table, width) or None (fan-in > 20)
        self.enc_rows = []      # per Enblock: evaluated spiral table (subset or full)
        self.enc_inv = []
        self.enc_select = []    # True when Pool(down) folds into the row subset
        self.enc_flat = []      # per Enblock on a row subset: (inverse_flat table, width)
        self.down_csr, self.downT_csr = [], []
        self.up_csr, self.upT_csr = [], []
        self.upT_order = []     # row schedule of each up transpose (None: short rows)
        self.up_uniform = []    # entries per row of each up matrix when uniform (else 0)
        self.upT_sched = []     # each up transpose stored in its visiting order (None: short rows)
        self.upT_nat = []       # the same in natural row order (vertex-major x: XCD-contiguous row ranges)
        self.np_spirals = [np.asarray(s, np.int64) for s in spirals]
        for l in range(self.n_levels):
            sp = np.asarray(spirals[l], np.int64)
            v = sp.shape[0]
            self.spiral.append(_dev(_i32(sp), self.device))
            self.spiral_inv.append(tuple(_dev(a, self.device) for a in inverse_spiral(sp, v)))
            fl, width = inverse_flat(sp, v, max_width=20)
            self.spiral_flat.append((_dev(fl, self.device), width) if fl is not None else None)
            drow, dcol, dval, dshape = down[l]
            sel = selection_rows(drow, dcol, dval, dshape[0])
            if dshape[1] != v:
                raise ValueError(f"down[{l}] has {dshape[1]} columns, level has {v} vertices")
            if sel is not None:
                sub = sp[sel]
                self.enc_select.append(True)
                self.enc_rows.append(_dev(_i32(sub), self.device))
                self.enc_inv.append(tuple(_dev(a, self.device) for a in inverse_spiral(sub, v)))
                fl, width = inverse_flat(sub, v)
                self.enc_flat.append((_dev(fl, self.device), width) if fl is not None else None)
            else:
                self.enc_select.append(False)
                self.enc_rows.append(self.spiral[-1])
                self.enc_inv.append(self.spiral_inv[-1])
                self.enc_flat.append(None)
            self.down_csr.append(self._csr(csr_from_coo(drow, dcol, dval, dshape[0])))
            self.downT_csr.append(self._csr(csr_transpose_from_coo(drow, dcol, dval, dshape[1])))
            urow, ucol, uval, ushape = up[l]
            up_l = csr_from_coo(urow, ucol, uval, ushape[0])
            self.up_uniform.append(uniform_rows(up_l[0]))
            self.up_csr.append(self._csr(up_l))
            self.upT_csr.append(self._csr(csr_transpose_from_coo(urow, ucol, uval, ushape[1])))
            upT = csr_transpose_from_coo(urow, ucol, uval, ushape[1])
            sched = row_schedule(upT[0])
            self.upT_order.append(_dev(sched, self.device) if sched is not None else None)
            self.upT_sched.append(tuple(_dev(a, self.device) for a in scheduled_csr(*upT, sched))
                                  if sched is not None else None)
            self.upT_nat.append(tuple(_dev(a, self.device) for a in
                                      scheduled_csr(*upT, np.arange(len(upT[0]) - 1)))
                                if sched is not None else None)
        # composite up-sampling rows of every spiral position (the Deblock
        # forward's fused Pool(up) gather, cfsd_spiral_conv_fwd_up): for up
        # matrix ui (level ui+1 -> level ui, uniform 3-entry rows) and spiral
        # position (r, s) of level ui, the 3 columns / values of up row
        # spiral[r, s], in the row's CSR (file) order; None when the rows are
        # not uniform or a spiral does not start at its own vertex
        self.up_comp = []
        for ui in range(self.n_levels):
            sp = self.np_spirals[ui]
            ok = (self.up_uniform[ui] == 3 and sp.shape[0] == self.up_csr[ui][0].numel() - 1
                  and np.array_equal(sp[:, 0], np.arange(sp.shape[0])))
            if not ok:
                self.up_comp.append(None)
                continue
            ucol = self.up_csr[ui][1].cpu().numpy().reshape(-1, 3)
            uval = self.up_csr[ui][2].cpu().numpy().reshape(-1, 3)
            self.up_comp.append((_dev(_i32(ucol[sp]), self.device),
                                 _dev(np.ascontiguousarray(uval[sp], np.float32), self.device)))
        self.lap_csr = self.lapT_csr = None
        if lap is not None:
            lr, lc, lv, lshape = lap
            r, c, v = coalesced_csr(lr, lc, lv, lshape[1])
            self.lap_csr = self._csr(csr_from_coo(r, c, v, lshape[0]))
            self.lapT_csr = self._csr(csr_transpose_from_coo(r, c, v, lshape[1]))
        self.region_mask = None
        self.n_regions = 0
        if regions is not None:
            mask = np.zeros((len(regions), self.n_verts[0]), np.uint8)
            for k, feat in enumerate(regions):
                mask[k, np.asarray(feat, np.int64)] = 1
            self.region_mask = _dev(mask, self.device)
            self.n_regions = len(regions)

    def _csr(self, t):
        ptr, col, val = t
        return (_dev(ptr, self.device), _dev(col, self.device), _dev(val, self.device))

    # ------------------------------------------------------------- builders
    @classmethod
    def from_npz(cls, npz, device="cuda"):
        """From the arrays of ``tests/golden/topology_craniofacial.npz``."""
        n = int(npz["n_levels"])
        spirals = [npz[f"spiral_{l}"] for l in range(n)]

        def coo(name, l):
            return (npz[f"{name}_{l}_row"], npz[f"{name}_{l}_col"], npz[f"{name}_{l}_val"],
                    tuple(int(s) for s in npz[f"{name}_{l}_shape"]))

        down = [coo("down", l) for l in range(n)]
        up = [coo("up", l) for l in range(n)]
        nv = spirals[0].shape[0]
        lap = None
        if "lap_row" in npz:
            lap = (npz["lap_row"], npz["lap_col"], npz["lap_val"], (nv, nv))
        regions = keys = None
        if "region_keys" in npz:
            keys = [str(k) for k in npz["region_keys"]]
            regions = [npz[f"region_{i}_feature"] for i in range(len(keys))]
        return cls(spirals, down, up, lap, regions, keys, device)

    @classmethod
    def from_torch(cls, spiral_indices, down_transform, up_transform, laplacian=None,
                   feat_and_cont=None, device="cuda"):
        """From the objects the reference passes to ``Model`` (int64 spiral
        tensors, torch sparse-COO transforms) and, optionally, the template's
        ``laplacian`` and ``feat_and_cont`` (``utils.load_template``)."""
        def coo_of(t):
            t = t.cpu()
            idx = t._indices().numpy()
            return (idx[0], idx[1], t._values().numpy(), tuple(t.shape))

        spirals = [s.cpu().numpy() for s in spiral_indices]
        down = [coo_of(d) for d in down_transform]
        up = [coo_of(u) for u in up_transform]
        lap = coo_of(laplacian) if laplacian is not None else None
        regions = keys = None
        if feat_and_cont is not None:
            keys = list(feat_and_cont.keys())
            regions = [np.asarray(feat_and_cont[k]["feature"]) for k in keys]
        return cls(spirals, down, up, lap, regions, keys, device)
