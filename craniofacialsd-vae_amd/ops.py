"""Typed host wrappers over the libcfsd C ABI.

Every wrapper validates shapes/dtypes/devices on the host BEFORE launching
(an out-of-range launch on the GPU would fault the device), then launches on
the current torch stream with no synchronisation.  Outputs may be passed in
(pre-allocated, graph-capture friendly) or are allocated with ``torch.empty``.
"""
import ctypes

import torch

from . import _abi
from ._abi import call, ptr, stream_ptr
from .topology import INV_HEAD

ACT_NONE = 0
ACT_ELU = 1
DT_F32 = 0    # CFSD_DT_F32
DT_BF16 = 1   # CFSD_DT_BF16
_DTYPES = {torch.float32: DT_F32, torch.bfloat16: DT_BF16}


def _need(t, shape, dtype=torch.float32, name="tensor"):
    if t is None:
        raise ValueError(f"{name} is required")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
    return t


def _dt(t, name="tensor"):
    if t.dtype not in _DTYPES:
        raise ValueError(f"{name}: dtype {t.dtype}, expected float32 or bfloat16")
    return _DTYPES[t.dtype]


def _needx(t, shape, name="tensor"):
    """_need for a mixed-precision operand (fp32 or bf16)."""
    if t is None:
        raise ValueError(f"{name} is required")
    return _need(t, shape, t.dtype if t.dtype in _DTYPES else torch.float32, name)


# ------------------------------------------------------------------ layouts
VM = 0x10  # CFSD_VM: vertex-major storage flag of a *_dt argument (include/cfsd.h)


def is_vm(t):
    """True for a logical [B, V, C] view of a VERTEX-MAJOR [V, B, C] buffer
    (``vm_empty`` / ``to_vm``): element (b, v, c) at (v*B + b)*C + c, the
    rows of one vertex in every mesh of the batch contiguous."""
    if t is None or t.dim() != 3 or t.is_contiguous():
        return False
    b, v, c = t.shape
    return t.stride() == (c, b * c, 1)


def vm_empty(bsz, nv, c, dtype=torch.float32, device="cuda"):
    """Uninitialised vertex-major tensor, seen as [bsz, nv, c]."""
    return torch.empty((nv, bsz, c), dtype=dtype, device=device).permute(1, 0, 2)


def to_vm(t):
    """Vertex-major copy of a [B, V, C] tensor (same logical values)."""
    return t.transpose(0, 1).contiguous().transpose(0, 1)


def _needl(t, shape, name="tensor", dtype=None):
    """A mixed-precision [B, V, C] operand in either layout: batch-major
    (contiguous) or vertex-major (``is_vm``)."""
    if t is None:
        raise ValueError(f"{name} is required")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    want = dtype if dtype is not None else (t.dtype if t.dtype in _DTYPES else torch.float32)
    if t.dtype != want:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {want}")
    if not (t.is_contiguous() or is_vm(t)):
        raise ValueError(f"{name} must be contiguous (batch-major) or a vertex-major view")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
    return t


def _st(t, name="tensor"):
    """Storage descriptor of a mixed-precision operand: type | CFSD_VM."""
    return _dt(t, name) | (VM if is_vm(t) else 0)


def _same_layout(a, b, what):
    if a is not None and b is not None and is_vm(a) != is_vm(b):
        raise ValueError(f"{what} must share one layout")


def _out(out, shape, like, name="out"):
    if out is None:
        return torch.empty(shape, dtype=torch.float32, device=like.device)
    return _need(out, shape, name=name)


# ------------------------------------------------------------------ spiral conv
def spiral_conv_workspace(bsz, vsrc, rows, seq, cin, cout):
    return int(_abi.lib().cfsd_spiral_conv_workspace(bsz, vsrc, rows, seq, cin, cout))


def _conv_ws(workspace, device, need):
    if workspace is None:
        workspace = torch.empty(need // 4 + 1, dtype=torch.float32, device=device)
    _need(workspace, None, name="workspace")
    nbytes = workspace.numel() * workspace.element_size()
    if nbytes < need:
        raise ValueError(f"conv workspace {nbytes} < {need} bytes")
    return workspace, nbytes


def spiral_conv_fwd(x, idx, w, b, act=ACT_NONE, out=None, workspace=None):
    """y[b, r] = act(b + W . concat_s x[b, idx[r, s]])  (model.py:27-41)."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = w.shape[0]
    _need(x, None, name="x")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(w, (cout, seq * cin), name="w")
    if b is not None:
        _need(b, (cout,), name="bias")
    y = _out(out, (bsz, rows, cout), x)
    ws, nb = _conv_ws(workspace, x.device, spiral_conv_workspace(bsz, vsrc, rows, seq, cin, cout))
    call("cfsd_spiral_conv_fwd", ptr(x), ptr(idx), ptr(w), ptr(b), ptr(y), ptr(ws),
         ctypes.c_size_t(nb), bsz, vsrc, rows, seq, cin, cout, act, stream_ptr())
    return y


def spiral_conv_bwd_data(dpre, inv, w, vsrc, elu_y=None, out=None, workspace=None):
    """dx[b, u] = g * sum_{(r,s) in inv(u)} W_s^T dpre[b, r]; ``inv`` is the
    (inv_ptr, inv_row, inv_head) triple of ``topology.inverse_spiral``."""
    bsz, rows, cout = dpre.shape
    inv_ptr, inv_row, inv_head = inv
    seq = (inv_ptr.numel() - 1) // vsrc
    cin = w.shape[1] // seq
    _need(dpre, None, name="dpre")
    _need(inv_ptr, (vsrc * seq + 1,), torch.int32, "inv_ptr")
    _need(inv_row, (rows * seq,), torch.int32, "inv_row")
    _need(inv_head, (vsrc * seq, INV_HEAD), torch.int32, "inv_head")
    _need(w, (cout, seq * cin), name="w")
    if elu_y is not None:
        _need(elu_y, (bsz, vsrc, cin), name="elu_y")
    dx = _out(out, (bsz, vsrc, cin), dpre)
    ws, nb = _conv_ws(workspace, dpre.device, spiral_conv_workspace(bsz, vsrc, rows, seq, cin, cout))
    call("cfsd_spiral_conv_bwd_data", ptr(dpre), ptr(inv_ptr), ptr(inv_row), ptr(inv_head), ptr(w),
         ptr(elu_y), ptr(dx), ptr(ws), ctypes.c_size_t(nb), bsz, vsrc, rows, seq, cin, cout,
         stream_ptr())
    return dx


def spiral_conv_bwd_weight_workspace(bsz, rows, seq, cin, cout):
    return int(_abi.lib().cfsd_spiral_conv_bwd_weight_workspace(bsz, rows, seq, cin, cout))


def spiral_conv_bwd_weight(x, idx, dpre, dw, db, workspace):
    """dW/db of one SpiralConv.  With ``dw is db is None`` the reduction is
    deferred: the partials stay in ``workspace`` and a DeferredDw descriptor
    is returned for ``dw_reduce_batch`` (which must get the real dw/db)."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    _need(x, None, name="x")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(dpre, (bsz, rows, cout), name="dpre")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    _need(workspace, None, name="workspace")
    need = spiral_conv_bwd_weight_workspace(bsz, rows, seq, cin, cout)
    nbytes = workspace.numel() * workspace.element_size()
    if nbytes < need:
        raise ValueError(f"workspace {nbytes} < {need} bytes")
    call("cfsd_spiral_conv_bwd_weight", ptr(x), ptr(idx), ptr(dpre), ptr(dw), ptr(db),
         ptr(workspace), ctypes.c_size_t(nbytes), bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    if dw is None:
        return DeferredDw(workspace, bsz, vsrc, rows, cin, cout, False)
    return None


class DeferredDw:
    """Slab set left by a deferred weight-gradient call (see dw_reduce_batch)."""

    def __init__(self, workspace, batch, vsrc, rows, cin, cout, fused):
        self.workspace = workspace
        self.sizes = (batch, vsrc, rows, cin, cout, int(fused))

    def desc(self, dw, db):
        _need(dw, (self.sizes[4], 9 * self.sizes[3]), name="dw")
        _need(db, (self.sizes[4],), name="db")
        return _abi.DwSlabs(self.workspace.data_ptr(), dw.data_ptr(), db.data_ptr(), *self.sizes)


def dw_reduce_batch(items, adam=None):
    """Reduce several deferred weight gradients in ONE launch.
    ``items``: list of (DeferredDw, dw, db).  ``adam``: optional dict(param,
    grad, m, v, step, lr, beta1, beta2, eps, weight_decay, shadow) -- the Adam
    step over the whole flat buffers fused into the same launch (the items'
    dw/db must be views of ``grad``)."""
    if not items and adam is None:
        return
    arr = (_abi.DwSlabs * max(len(items), 1))(*[d.desc(dw, db) for d, dw, db in items])
    if adam is None:
        call("cfsd_dw_reduce_batch", arr, len(items), stream_ptr())
        return
    a = adam
    n = a["param"].numel()
    for t, nm in ((a["param"], "param"), (a["grad"], "grad"), (a["m"], "m"), (a["v"], "v")):
        _need(t, (n,), name=nm)
    _need(a["step"], (1,), torch.int32, "step")
    if a.get("shadow") is not None:
        _need(a["shadow"], (n,), torch.bfloat16, "shadow")
    call("cfsd_dw_reduce_batch_adam", arr, len(items), ptr(a["param"]), ptr(a["grad"]), ptr(a["m"]),
         ptr(a["v"]), ptr(a["step"]), ctypes.c_size_t(n), float(a["lr"]), float(a["beta1"]),
         float(a["beta2"]), float(a["eps"]), float(a["weight_decay"]), ptr(a.get("shadow")), stream_ptr())


def spiral_conv_bwd_workspace(bsz, vsrc, rows, seq, cin, cout):
    return int(_abi.lib().cfsd_spiral_conv_bwd_workspace(bsz, vsrc, rows, seq, cin, cout))


def spiral_conv_bwd_paired(bsz, vsrc, rows, seq, cin, cout):
    """True when spiral_conv_bwd (with dx) runs dx and dW as one paired launch."""
    return bool(_abi.lib().cfsd_spiral_conv_bwd_paired(bsz, vsrc, rows, seq, cin, cout))


def spiral_conv_bwd(x, idx, dpre, inv, w, dw, db, dx=None, elu_y=None, workspace=None):
    """Fused dX (skipped when ``dx`` is None) + dW/db of one SpiralConv; same
    results as spiral_conv_bwd_data followed by spiral_conv_bwd_weight."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    inv_ptr, inv_row, inv_head = inv
    _need(x, None, name="x")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(dpre, (bsz, rows, cout), name="dpre")
    _need(inv_ptr, (vsrc * seq + 1,), torch.int32, "inv_ptr")
    _need(inv_row, (rows * seq,), torch.int32, "inv_row")
    _need(inv_head, (vsrc * seq, INV_HEAD), torch.int32, "inv_head")
    _need(w, (cout, seq * cin), name="w")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    if dx is not None:
        _need(dx, (bsz, vsrc, cin), name="dx")
    if elu_y is not None:
        _need(elu_y, (bsz, vsrc, cin), name="elu_y")
    ws, nb = _conv_ws(workspace, x.device, spiral_conv_bwd_workspace(bsz, vsrc, rows, seq, cin, cout))
    call("cfsd_spiral_conv_bwd", ptr(x), ptr(idx), ptr(dpre), ptr(inv_ptr), ptr(inv_row),
         ptr(inv_head), ptr(w), ptr(elu_y), ptr(dx), ptr(dw), ptr(db), ptr(ws), ctypes.c_size_t(nb),
         bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    if dw is None:  # deferred weight gradient
        return dx, DeferredDw(ws, bsz, vsrc, rows, cin, cout, True)
    return dx


def spiral_conv_bwd_rowsub_workspace(bsz, vsrc, rows, seq, cin, cout):
    """0 when the shape has no row-subset backward (cin != 32)."""
    return int(_abi.lib().cfsd_spiral_conv_bwd_rowsub_workspace(bsz, vsrc, rows, seq, cin, cout))


def spiral_conv_bwd_rowsub(x, idx, dpre, flat, w, dw, db, dx, elu_y=None, workspace=None):
    """dX + dW/db of a conv evaluated on a row subset (an Enblock conv):
    dG = dpre.W at the kept rows, then the ascending-order gather-sum of dG
    through ``flat`` = ``topology.inverse_flat``'s (table, width)."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    table, width = flat
    if is_vm(x):  # vertex-major fp32 x (the fp32 step's E1): cfsd_spiral_conv_bwd_rowsub_x
        _needl(x, (bsz, vsrc, cin), "x", torch.float32)
    else:
        _need(x, None, name="x")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(dpre, (bsz, rows, cout), name="dpre")
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w, (cout, seq * cin), name="w")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    if is_vm(x):  # x, dx and elu_y share the source level's layout
        _needl(dx, (bsz, vsrc, cin), "dx", torch.float32)
        _same_layout(x, dx, "x and dx")
        if elu_y is not None:
            _needl(elu_y, (bsz, vsrc, cin), "elu_y", torch.float32)
            _same_layout(x, elu_y, "x and elu_y")
    else:
        _need(dx, (bsz, vsrc, cin), name="dx")
        if elu_y is not None:
            _need(elu_y, (bsz, vsrc, cin), name="elu_y")
    need = spiral_conv_bwd_rowsub_workspace(bsz, vsrc, rows, seq, cin, cout)
    if need == 0:
        raise ValueError(f"no row-subset backward for {cin} -> {cout} channels")
    ws, nb = _conv_ws(workspace, x.device, need)
    if is_vm(x):
        call("cfsd_spiral_conv_bwd_rowsub_x", ptr(x), _st(x), ptr(idx), ptr(dpre), ptr(table), width, ptr(w),
             ptr(elu_y), ptr(dx), ptr(dw), ptr(db), ptr(ws), ctypes.c_size_t(nb), bsz, vsrc, rows, seq,
             cin, cout, stream_ptr())
    else:
        call("cfsd_spiral_conv_bwd_rowsub", ptr(x), ptr(idx), ptr(dpre), ptr(table), width, ptr(w),
             ptr(elu_y), ptr(dx), ptr(dw), ptr(db), ptr(ws), ctypes.c_size_t(nb), bsz, vsrc, rows, seq,
             cin, cout, stream_ptr())
    if dw is None:  # deferred weight gradient (slabs at the workspace start)
        return dx, DeferredDw(ws, bsz, vsrc, rows, cin, cout, True)
    return dx


def spiral_conv_bwd_data_rowsub_workspace(bsz, rows, seq, cin):
    return int(_abi.lib().cfsd_spiral_conv_bwd_data_rowsub_workspace(bsz, rows, seq, cin))


def spiral_conv_bwd_data_rowsub(dpre, flat, w, vsrc, elu_y=None, out=None, workspace=None):
    """dx of a row-subset conv (dG = dpre.W at the kept rows, then the
    ascending flat gather); ``out``/``elu_y`` fp32 or bf16 (bf16 path)."""
    bsz, rows, cout = dpre.shape
    table, width = flat
    cin = w.shape[1] // 9
    _need(dpre, None, name="dpre")
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w, (cout, 9 * cin), name="w")
    _needl(out, (bsz, vsrc, cin), "out")
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", out.dtype)
        _same_layout(out, elu_y, "out and elu_y")
    need = spiral_conv_bwd_data_rowsub_workspace(bsz, rows, 9, cin)
    if need == 0:
        raise ValueError(f"no row-subset backward for {cin} -> {cout} channels")
    ws, nb = _conv_ws(workspace, dpre.device, need)
    call("cfsd_spiral_conv_bwd_data_rowsub", ptr(dpre), ptr(table), width, ptr(w), ptr(elu_y), ptr(out),
         _st(out), ptr(ws), ctypes.c_size_t(nb), bsz, vsrc, rows, 9, cin, cout, stream_ptr())
    return out


def spiral_gather(x, idx, out=None):
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    _need(x, None, name="x")
    _need(idx, (rows, seq), torch.int32, "idx")
    g = _out(out, (bsz, rows, seq * cin), x)
    call("cfsd_spiral_gather", ptr(x), ptr(idx), ptr(g), bsz, vsrc, rows, seq, cin, stream_ptr())
    return g


# ------------------------------------------------------------------ pool / swap
def spmm(csr, x, m, elu_y=None, out=None, order=None, uniform=0, sched=None):
    """y[b, r] = g * sum_{k in row r} val[k] x[b, col[k]]   (Pool, model.py:50-55).
    ``order``: optional row schedule (a permutation of the rows by decreasing
    length, for matrices with long skewed rows); ``uniform``: every row holds
    exactly that many entries (``topology.uniform_rows``; no row_ptr walk);
    ``sched``: the CSR re-stored in a visiting order (``topology.scheduled_csr``,
    replaces ``csr``/``order``).  Same results bit for bit in every form."""
    row_ptr, col, val = csr
    bsz, n, c = x.shape
    _need(x, None, name="x")
    _need(row_ptr, (m + 1,), torch.int32, "row_ptr")
    _need(col, None, torch.int32, "col")
    _need(val, (col.numel(),), name="val")
    if elu_y is not None:
        _need(elu_y, (bsz, m, c), name="elu_y")
    y = _out(out, (bsz, m, c), x)
    if sched is not None:
        _spmm_sched_csr(sched, x, elu_y, y, bsz, m, n, c)
        return y
    if order is not None:
        _spmm_sched(row_ptr, col, val, order, x, elu_y, y, bsz, m, n, c)
        return y
    if uniform:
        _spmm_uniform(uniform, col, val, x, elu_y, y, bsz, m, n, c)
        return y
    call("cfsd_spmm_csr", ptr(row_ptr), ptr(col), ptr(val), ptr(x), ptr(elu_y), ptr(y), bsz, m, n,
         c, stream_ptr())
    return y


def _spmm_uniform(k, col, val, x, elu_y, y, bsz, m, n, c):
    """cfsd_spmm_uniform: every row holds exactly ``k`` entries."""
    if col.numel() != m * k:
        raise ValueError(f"uniform SpMM: {col.numel()} entries != {m} rows x {k}")
    call("cfsd_spmm_uniform", int(k), ptr(col), ptr(val), ptr(x), _st(x), ptr(elu_y), ptr(y), _st(y),
         bsz, m, n, c, stream_ptr())


def _spmm_sched_csr(sched, x, elu_y, y, bsz, m, n, c):
    """cfsd_spmm_sched_csr over a CSR stored in visiting order."""
    ptr_s, col_s, val_s, rows_s = sched
    _need(ptr_s, (m + 1,), torch.int32, "ptr_s")
    _need(rows_s, (m,), torch.int32, "rows_s")
    _need(col_s, None, torch.int32, "col_s")
    _need(val_s, (col_s.numel(),), name="val_s")
    call("cfsd_spmm_sched_csr", ptr(ptr_s), ptr(col_s), ptr(val_s), ptr(rows_s), ptr(x), _st(x), ptr(elu_y),
         ptr(y), _st(y), bsz, m, n, c, stream_ptr())


def _spmm_sched(row_ptr, col, val, order, x, elu_y, y, bsz, m, n, c):
    """cfsd_spmm_csr_sched: rows visited in ``order`` (``topology.row_schedule``)."""
    _need(order, (m,), torch.int32, "order")
    call("cfsd_spmm_csr_sched", ptr(row_ptr), ptr(col), ptr(val), ptr(order), ptr(x), _st(x),
         ptr(elu_y), ptr(y), _st(y), bsz, m, n, c, stream_ptr())


def swap_features(x_all, batch_idx, region_mask, key, bs, out=None):
    """``SwapFeatures.__call__`` (swap_batch_transform.py:13-42) on device."""
    n_meshes, nv, c = x_all.shape
    _need(x_all, None, name="x_all")
    _need(batch_idx, (bs,), torch.int32, "batch_idx")
    if region_mask is None or region_mask.dim() != 2:
        raise ValueError("region_mask [n_regions, nv] is required")
    _need(region_mask, (region_mask.shape[0], nv), torch.uint8, "region_mask")
    _need(key, (1,), torch.int32, "key")
    if out is not None and is_vm(out):  # vertex-major output (the fp32 step's level-0 input)
        _needl(out, (bs * bs, nv, c), "out", torch.float32)
        call("cfsd_swap_features_x", ptr(x_all), ptr(batch_idx), ptr(region_mask), ptr(key), ptr(out),
             _st(out), bs, nv, c, n_meshes, int(region_mask.shape[0]), stream_ptr())
        return out
    y = _out(out, (bs * bs, nv, c), x_all)
    call("cfsd_swap_features", ptr(x_all), ptr(batch_idx), ptr(region_mask), ptr(key), ptr(y), bs,
         nv, c, n_meshes, int(region_mask.shape[0]), stream_ptr())
    return y


def spiral_conv_fwd_in_swap(x_all, batch_idx, region_mask, key, bs, x_out, idx, w, bias, act, out):
    """:func:`swap_features` into ``x_out`` and the xyz input conv of the first
    Enblock (``out`` = act(conv(x_out)) at the rows of ``idx``) in one launch
    (``cfsd_spiral_conv_fwd_in_swap``): the conv gathers through the swap
    straight from ``x_all``.  ``x_out`` fp32, either layout; ``out`` fp32 or
    bf16, either layout."""
    n_meshes, nv, c = x_all.shape
    rows, seq = idx.shape
    cout = w.shape[0]
    _need(x_all, None, name="x_all")
    _need(batch_idx, (bs,), torch.int32, "batch_idx")
    if region_mask is None or region_mask.dim() != 2:
        raise ValueError("region_mask [n_regions, nv] is required")
    _need(region_mask, (region_mask.shape[0], nv), torch.uint8, "region_mask")
    _need(key, (1,), torch.int32, "key")
    _needl(x_out, (bs * bs, nv, c), "x_out", torch.float32)
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(w, (cout, seq * c), name="w")
    _needl(out, (bs * bs, rows, cout), "out", out.dtype)
    call("cfsd_spiral_conv_fwd_in_swap", ptr(x_all), ptr(batch_idx), ptr(region_mask), ptr(key), bs, n_meshes,
         int(region_mask.shape[0]), ptr(x_out), _st(x_out), ptr(idx), ptr(w), ptr(bias), ptr(out), _st(out), nv, rows,
         c, cout, int(act), stream_ptr())
    return out


def spiral_conv_fwd_up_supported(bsz, rows, seq, cin, cout):
    return bool(_abi.lib().cfsd_spiral_conv_fwd_up_supported(bsz, rows, seq, cin, cout))


def spiral_conv_fwd_up(xc, comp, idx, w, bias, act, out, up_out=None):
    """SpiralDeblock forward (``model.py:80-82``) with Pool(up) fused into
    the gather: ``comp`` = the level's composite up table
    (``DeviceTopology.up_comp``); ``up_out`` receives Pool(xc, up) (the
    input the weight gradient reads), bit-identical to :func:`spmm`."""
    bsz, n_coarse, cin = xc.shape
    rows, seq = idx.shape
    cout = w.shape[0]
    _need(xc, None, name="xc")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(comp[0], (rows, seq, 3), torch.int32, "comp_col")
    _need(comp[1], (rows, seq, 3), torch.float32, "comp_val")
    _need(w, (cout, seq * cin), name="w")
    _need(out, (bsz, rows, cout), name="out")
    if up_out is not None:
        _need(up_out, (bsz, rows, cin), name="up_out")
    call("cfsd_spiral_conv_fwd_up", ptr(xc), ptr(comp[0]), ptr(comp[1]), ptr(idx), ptr(w), ptr(bias), ptr(out),
         ptr(up_out), bsz, n_coarse, rows, seq, cin, cout, int(act), stream_ptr())
    return out


def gather_meshes(x_all, batch_idx, bs, out=None):
    """The un-swapped batch of a ``swap_features: False`` configuration
    (``data_loading.py:38, 81-82``: MeshCollater without a feature swapper):
    ``out[b] = x_all[batch_idx[b]]`` on device (``cfsd_gather_meshes``)."""
    n_meshes, nv, c = x_all.shape
    _need(x_all, None, name="x_all")
    _need(batch_idx, (bs,), torch.int32, "batch_idx")
    if out is not None and is_vm(out):
        _needl(out, (bs, nv, c), "out", torch.float32)
        y = out
    else:
        y = _out(out, (bs, nv, c), x_all)
    call("cfsd_gather_meshes", ptr(x_all), ptr(batch_idx), ptr(y), _st(y), bs, nv, c, n_meshes, stream_ptr())
    return y


def spectral_blend(s1, s2, values, n_blend, out=None):
    """Augmentation coefficients s1 + v * (s2 - s1) on the first ``n_blend``
    spectral components (utils.py:256-267); s1/s2 [pairs, k, c], values [pairs, k]."""
    _need(s1, None, name="s1")
    if s1.dim() != 3:
        raise ValueError(f"s1: shape {tuple(s1.shape)}, expected [pairs, k, c]")
    p, k, c = s1.shape
    _need(s2, (p, k, c), name="s2")
    _need(values, (p, k), name="values")
    y = _out(out, (p, k, c), s1)
    call("cfsd_spectral_blend", ptr(s1), ptr(s2), ptr(values), ptr(y), p, k, c, int(n_blend), stream_ptr())
    return y


def normalize(x, mean, std, out=None):
    """``(x - mean) / std`` per vertex (data_loading.py:259-260), bit-exact."""
    _need(x, None, name="x")
    if x.dim() != 3:
        raise ValueError(f"x: shape {tuple(x.shape)}, expected [n_meshes, nv, c]")
    n, nv, c = x.shape
    _need(mean, (nv, c), name="mean")
    _need(std, (nv, c), name="std")
    y = _out(out, (n, nv, c), x)
    call("cfsd_normalize", ptr(x), ptr(mean), ptr(std), ptr(y), n, nv, c, stream_ptr())
    return y


def elu_bwd(dy, y, out=None):
    _need(dy, None, name="dy")
    _need(y, tuple(dy.shape), name="y")
    dx = _out(out, tuple(dy.shape), dy)
    call("cfsd_elu_bwd", ptr(dy), ptr(y), ptr(dx), ctypes.c_size_t(dy.numel()), stream_ptr())
    return dx


# ------------------------------------------------------------------ dense
def linear_workspace(m, k, n):
    return int(_abi.lib().cfsd_linear_workspace(m, k, n))


def _ws(workspace, need):
    if need == 0:
        return None, 0
    if workspace is None:
        raise ValueError(f"linear: workspace of {need} bytes required")
    nbytes = workspace.numel() * workspace.element_size()
    if nbytes < need:
        raise ValueError(f"linear: workspace {nbytes} < {need} bytes")
    return workspace, nbytes


def linear_fwd(x, w, b, out=None, workspace=None):
    m, k = x.shape
    n = w.shape[0]
    _need(x, None, name="x")
    _need(w, (n, k), name="w")
    if b is not None:
        _need(b, (n,), name="b")
    y = _out(out, (m, n), x)
    if workspace is None and linear_workspace(m, k, n):
        workspace = torch.empty(linear_workspace(m, k, n) // 4, device=x.device)
    ws, nb = _ws(workspace, linear_workspace(m, k, n))
    call("cfsd_linear_fwd", ptr(x), ptr(w), ptr(b), ptr(y), ptr(ws), ctypes.c_size_t(nb), m, k, n,
         stream_ptr())
    return y


def linear_bwd(x, w, dy, dx=None, dw=None, db=None, elu_y=None, accumulate=False, workspace=None):
    m, n = dy.shape
    k = w.shape[1] if w is not None else x.shape[1]
    _need(dy, None, name="dy")
    if dx is not None:
        _need(dx, (m, k), name="dx")
        _need(w, (n, k), name="w")
    if dw is not None:
        _need(dw, (n, k), name="dw")
        _need(x, (m, k), name="x")
    if db is not None:
        _need(db, (n,), name="db")
    if elu_y is not None:
        _need(elu_y, (m, k), name="elu_y")
    need = linear_workspace(m, k, n) if dx is not None else 0
    if workspace is None and need:
        workspace = torch.empty(need // 4, device=dy.device)
    ws, nb = _ws(workspace, need)
    call("cfsd_linear_bwd", ptr(x), ptr(w), ptr(dy), ptr(elu_y), ptr(dx), ptr(dw), ptr(db),
         ptr(ws), ctypes.c_size_t(nb), m, k, n, int(accumulate), stream_ptr())


# ------------------------------------------------------------------ losses
def recon_lap_blocks(bsz, nv):
    return int(_abi.lib().cfsd_recon_lap_blocks(bsz, nv))


def _loss_layout(*ts):
    """Storage flag of the loss operands: all batch-major or all vertex-major."""
    vm = [is_vm(t) for t in ts]
    if any(vm) and not all(vm):
        raise ValueError("loss operands must share one layout (batch-major or vertex-major)")
    for t in ts:
        _needl(t, tuple(ts[0].shape), "loss operand", torch.float32)
    return VM if vm[0] else 0


def recon_lap_fwd(pred, gt, lap_csr, unit, partials):
    bsz, nv, c = pred.shape
    lay = _loss_layout(pred, gt, unit)
    _need(partials, (2 * recon_lap_blocks(bsz, nv),), name="partials")
    _need(lap_csr[0], (nv + 1,), torch.int32, "l_ptr")
    call("cfsd_recon_lap_fwd_x", ptr(pred), ptr(gt), ptr(lap_csr[0]), ptr(lap_csr[1]),
         ptr(lap_csr[2]), ptr(unit), ptr(partials), bsz, nv, c, lay, stream_ptr())


def recon_lap_bwd(pred, gt, unit, lapT_csr, dpred, w_rec, w_lap):
    bsz, nv, c = pred.shape
    lay = _loss_layout(pred, gt, unit, dpred)
    _need(lapT_csr[0], (nv + 1,), torch.int32, "lt_ptr")
    call("cfsd_recon_lap_bwd_x", ptr(pred), ptr(gt), ptr(unit), ptr(lapT_csr[0]),
         ptr(lapT_csr[1]), ptr(lapT_csr[2]), ptr(dpred), bsz, nv, c, float(w_rec), float(w_lap), lay,
         stream_ptr())


def recon_lap_bwd_finalize(pred, gt, unit, lapT_csr, dpred, w_rec, w_lap, partials, terms, out, acc,
                           w_kl, w_lc):
    """recon_lap_bwd + loss_finalize in one launch (the last workgroup
    finalises the losses of the preceding recon_lap_fwd)."""
    bsz, nv, c = pred.shape
    lay = _loss_layout(pred, gt, unit, dpred)
    _need(lapT_csr[0], (nv + 1,), torch.int32, "lt_ptr")
    _need(out, (5,), name="out")
    if acc is not None:
        _need(acc, (6,), name="acc")
    call("cfsd_recon_lap_bwd_finalize_x", ptr(pred), ptr(gt), ptr(unit), ptr(lapT_csr[0]),
         ptr(lapT_csr[1]), ptr(lapT_csr[2]), ptr(dpred), bsz, nv, c, float(w_rec), float(w_lap),
         ptr(partials), partials.numel() // 2, ptr(terms), ptr(out), ptr(acc), float(w_kl),
         float(w_lc), lay, stream_ptr())


def latent_fwd(mulv, eps, key, z, dlat, terms, latent, region_size, train, is_vae, sigmoid,
               w_kl, w_lc, eta1, eta2):
    bsz = z.shape[0]
    _need(mulv, (bsz, 2 * latent if is_vae else latent), name="mulv")
    _need(z, (bsz, latent), name="z")
    _need(dlat, (bsz, 3 * latent), name="dlat")
    _need(terms, (2,), name="terms")
    if eps is not None:
        _need(eps, (bsz, latent), name="eps")
    if key is not None:
        _need(key, (1,), torch.int32, "key")
    call("cfsd_latent_fwd", ptr(mulv), ptr(eps), ptr(key), ptr(z), ptr(dlat), ptr(terms), bsz,
         latent, region_size, int(train), int(is_vae), int(sigmoid), float(w_kl), float(w_lc),
         float(eta1), float(eta2), stream_ptr())


def latent_linear_fwd_supported(batch, latent, n):
    return bool(_abi.lib().cfsd_latent_linear_fwd_supported(int(batch), int(latent), int(n)))


def latent_linear_fwd(mulv, eps, key, z, dlat, terms, latent, region_size, train, is_vae, sigmoid,
                      w_kl, w_lc, eta1, eta2, w, bias, out):
    """latent_fwd, then the decoder Linear out = z w^T + bias, in one launch
    (cfsd_latent_linear_fwd: z, dlat, out bit-identical to the two calls)."""
    bsz = z.shape[0]
    n = w.shape[0]
    _need(mulv, (bsz, 2 * latent if is_vae else latent), name="mulv")
    _need(z, (bsz, latent), name="z")
    _need(dlat, (bsz, 3 * latent), name="dlat")
    _need(terms, (2,), name="terms")
    _need(w, (n, latent), name="w")
    _need(out, (bsz, n), name="out")
    if bias is not None:
        _need(bias, (n,), name="bias")
    if eps is not None:
        _need(eps, (bsz, latent), name="eps")
    if key is not None:
        _need(key, (1,), torch.int32, "key")
    call("cfsd_latent_linear_fwd", ptr(mulv), ptr(eps), ptr(key), ptr(z), ptr(dlat), ptr(terms), bsz,
         latent, region_size, int(train), int(is_vae), int(sigmoid), float(w_kl), float(w_lc),
         float(eta1), float(eta2), ptr(w), ptr(bias), ptr(out), n, stream_ptr())


def latent_bwd(mulv, eps, z, dz_dec, dlat, dmulv, latent, train, is_vae, sigmoid):
    """``dz_dec`` [B, latent], or [parts, B, latent] partial products (summed
    in part order: cfsd_latent_bwd_parts)."""
    _need(dmulv, tuple(mulv.shape), name="dmulv")
    if dz_dec.dim() == 3:
        parts, bsz = dz_dec.shape[:2]
        _need(dz_dec, (parts, bsz, latent), name="dz_parts")
        call("cfsd_latent_bwd_parts", ptr(mulv), ptr(eps), ptr(z), ptr(dz_dec), parts, ptr(dlat),
             ptr(dmulv), bsz, latent, int(train), int(is_vae), int(sigmoid), stream_ptr())
        return
    bsz = dz_dec.shape[0]
    _need(dz_dec, (bsz, latent), name="dz_dec")
    call("cfsd_latent_bwd", ptr(mulv), ptr(eps), ptr(z), ptr(dz_dec), ptr(dlat), ptr(dmulv), bsz,
         latent, int(train), int(is_vae), int(sigmoid), stream_ptr())


BN_SYNC_INTS = 608  # cfsd_bottleneck_bwd's counters and flags (19 x one 128-B line)
BN_SYNC_ERR = 65    # CFSD_BN_SYNC_ERR: the sticky timed-out-wait word inside them


def bottleneck_exchange_floats(batch, latent, nd, ne):
    """Size of cfsd_bottleneck_bwd's exchange workspace (device floats)."""
    return int(_abi.lib().cfsd_bottleneck_bwd_exchange_floats(batch, latent, nd, ne))


def bottleneck_check(sync):
    """Raise CfsdError if any cfsd_bottleneck_bwd launch that used ``sync``
    gave up waiting (its values are then wrong).  Reads one device int (a
    host sync): call it at a cadence, e.g. once per epoch, not per step."""
    err = int(sync[BN_SYNC_ERR].item())
    if err:
        raise _abi.CfsdError(f"cfsd_bottleneck_bwd: a wait timed out (roles {err:#x}); the step's "
                             f"bottleneck gradients are invalid")


def bottleneck_bwd(up_csr, g, z, wd, exchange, dwd, dbd, mulv, eps, dlat, dmulv, is_vae, sigmoid, xe, we, dxe,
                   dwe, dbe, sync, elu_y=None, accumulate=False, train=True):
    """The bottleneck backward in one launch (``cfsd_bottleneck_bwd``): the
    coarsest Pool(up) transpose over ``g`` [B, n_up, cup] (``up_csr`` =
    (row_ptr, col, val), plain per-row order), the decoder Linear backward
    (``wd`` [nd, latent]), the latent head backward (:func:`latent_bwd`) and
    the encoder Linear backward (:func:`linear_bwd` with ``xe`` [B, ke],
    ``we`` [ne, ke], dy = ``dmulv``).  ``exchange``: a device float buffer of
    :func:`bottleneck_exchange_floats` (the launch's line-exclusive hand-off
    area); ``sync``: BN_SYNC_INTS zeroed device int32, left zeroed (a timed-out
    wait sets ``sync[BN_SYNC_ERR]``: :func:`bottleneck_check`)."""
    row_ptr, col, val = up_csr
    bsz, n_up, cup = g.shape
    _need(g, None, name="g")
    if is_vm(g):
        raise ValueError("g must be batch-major")
    m, lat = z.shape
    nd, kd = wd.shape
    ne, ke = we.shape
    if kd != lat or m != bsz or nd % cup:
        raise ValueError(f"bottleneck_bwd: z {tuple(z.shape)}, wd {tuple(wd.shape)}, g {tuple(g.shape)}")
    _need(row_ptr, (nd // cup + 1,), torch.int32, "up_ptr")
    _need(col, None, torch.int32, "up_col")
    _need(val, (col.numel(),), name="up_val")
    _need(z, (m, lat), name="z")
    _need(exchange, (bottleneck_exchange_floats(m, lat, nd, ne),), name="exchange")
    _need(dwd, (nd, lat), name="dwd")
    _need(dbd, (nd,), name="dbd")
    _need(dmulv, tuple(mulv.shape), name="dmulv")
    _need(xe, (m, ke), name="xe")
    _need(dxe, (m, ke), name="dxe")
    if elu_y is not None:
        _need(elu_y, (m, ke), name="elu_y")
    _need(dwe, (ne, ke), name="dwe")
    _need(dbe, (ne,), name="dbe")
    _need(sync, (BN_SYNC_INTS,), torch.int32, "sync")
    call("cfsd_bottleneck_bwd", ptr(row_ptr), ptr(col), ptr(val), ptr(g), n_up, cup, ptr(z), ptr(wd), ptr(exchange),
         ptr(dwd), ptr(dbd), nd, ptr(mulv), ptr(eps), ptr(dlat), ptr(dmulv), int(train), int(is_vae), int(sigmoid),
         ptr(xe), ptr(we), ptr(elu_y), ptr(dxe), ptr(dwe), ptr(dbe), ke, ne, int(accumulate), ptr(sync), m, lat,
         stream_ptr())


def linear_bwd_split_parts(n):
    return int(_abi.lib().cfsd_linear_bwd_split_parts(n))


def linear_bwd_split(x, w, dy, dx_parts, dw, db):
    """Decoder-Linear backward in one launch: dW/db and dx as partial
    products over 64-row slices of W (``dx_parts`` [parts, m, k], summed by
    :func:`latent_bwd` with ``n_parts``)."""
    m, k = x.shape
    n = dy.shape[1]
    _need(x, (m, k), name="x")
    _need(w, (n, k), name="w")
    _need(dy, (m, n), name="dy")
    _need(dx_parts, (linear_bwd_split_parts(n), m, k), name="dx_parts")
    _need(dw, (n, k), name="dw")
    _need(db, (n,), name="db")
    call("cfsd_linear_bwd_split", ptr(x), ptr(w), ptr(dy), ptr(dx_parts), ptr(dw), ptr(db), m, k, n,
         stream_ptr())


def loss_finalize(partials, terms, out, acc, bsz, nv, c, w_kl, w_lc, w_lap):
    _need(out, (5,), name="out")
    if acc is not None:
        _need(acc, (6,), name="acc")
    call("cfsd_loss_finalize", ptr(partials), partials.numel() // 2, ptr(terms), ptr(out),
         ptr(acc), bsz, nv, c, float(w_kl), float(w_lc), float(w_lap), stream_ptr())


# ------------------------------------------------------------------ optimiser
def adam(param, grad, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
         shadow=None):
    """Adam over the flat fp32 buffers; ``shadow`` (bf16, same length) also
    receives the updated parameters (the bf16 path's weight copy)."""
    n = param.numel()
    for t, nm in ((param, "param"), (grad, "grad"), (m, "m"), (v, "v")):
        _need(t, (n,), name=nm)
    _need(step, (1,), torch.int32, "step")
    if shadow is not None:
        _need(shadow, (n,), torch.bfloat16, "shadow")
    call("cfsd_adam", ptr(param), ptr(grad), ptr(m), ptr(v), ptr(step), ctypes.c_size_t(n),
         float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), ptr(shadow),
         stream_ptr())


def adam_scaled(param, grad, m, v, step, grad_scale, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
                shadow=None):
    """``scale(grad, grad_scale)`` then :func:`adam` in one launch (the
    data-parallel step's 1/world averaging folded into the update); ``grad``
    receives the scaled gradient."""
    n = param.numel()
    for t, nm in ((param, "param"), (grad, "grad"), (m, "m"), (v, "v")):
        _need(t, (n,), name=nm)
    _need(step, (1,), torch.int32, "step")
    if shadow is not None:
        _need(shadow, (n,), torch.bfloat16, "shadow")
    call("cfsd_adam_scaled", ptr(param), ptr(grad), ptr(m), ptr(v), ptr(step), ctypes.c_size_t(n),
         float(grad_scale), float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), ptr(shadow),
         stream_ptr())


def step_begin(counter, seed, eps=None, key=None, n_regions=0, batch_idx=None, bs=0,
               n_batches=0, perm=None, adam_step=None, n_items=None, shuffle=False):
    """Per-step device bookkeeping (``cfsd_step_begin``): counter, swap key,
    VAE noise, the epoch-shuffled drop_last batch and Adam's t.  ``perm``
    (optional, int32) maps the ``n_items`` shuffled positions to dataset rows;
    its length and range are the caller's contract (validated once by
    ``engine.ResidentData``), not re-checked per step."""
    _need(counter, (1,), torch.int32, "counter")
    if adam_step is not None:
        _need(adam_step, (1,), torch.int32, "adam_step")
    if eps is not None:
        _need(eps, None, name="eps")
    if key is not None:
        _need(key, (1,), torch.int32, "key")
    if batch_idx is not None:
        _need(batch_idx, (bs,), torch.int32, "batch_idx")
        if n_items is None:
            n_items = perm.numel() if perm is not None else n_batches * bs
        if perm is not None:
            _need(perm, None, torch.int32, "perm")
            if perm.numel() < n_items:
                raise ValueError(f"perm has {perm.numel()} entries < n_items {n_items}")
        if n_items < n_batches * bs:
            raise ValueError(f"n_items {n_items} < n_batches {n_batches} x bs {bs}")
    call("cfsd_step_begin", ptr(counter), ctypes.c_ulonglong(seed), ptr(eps),
         eps.numel() if eps is not None else 0, ptr(key), n_regions, ptr(batch_idx), bs,
         n_batches, ptr(perm), int(n_items or 0), int(bool(shuffle)), ptr(adam_step), stream_ptr())


def scale(y, alpha):
    _need(y, None, name="y")
    call("cfsd_scale", ptr(y), ctypes.c_size_t(y.numel()), float(alpha), stream_ptr())


# ------------------------------------------------------------------ evaluation
def vertex_errors(out, gt, to_mm=89.11, mean=None, std=None, want_l1=False, want_mesh_mean=False):
    """``ModelManager.compute_vertex_errors`` (``model_manager.py:395-400``) on
    device: ``sqrt(sum_c (out - gt)^2) * to_mm`` per vertex, ``[B, V]``.

    ``mean``/``std`` ``[V, 3]`` un-normalise both inputs first
    (``Tester._unnormalize_verts``, ``test.py:81-84``).  ``want_l1`` also
    returns the per-vertex L1 ``sum_c |out - gt|``; ``want_mesh_mean`` the
    per-mesh mean used by ``Tester.reconstruction_errors`` (``test.py:297``).
    Returns ``err`` or a tuple ``(err, l1?, mesh_mean?)``."""
    _need(out, None, name="out")
    if out.dim() != 3 or out.shape[-1] != 3:
        raise ValueError(f"out: shape {tuple(out.shape)}, expected [B, V, 3]")
    bsz, nv = int(out.shape[0]), int(out.shape[1])
    _need(gt, tuple(out.shape), name="gt")
    if (mean is None) != (std is None):
        raise ValueError("mean and std go together")
    if mean is not None:
        _need(mean, (nv, 3), name="mean")
        _need(std, (nv, 3), name="std")
    err = torch.empty((bsz, nv), dtype=torch.float32, device=out.device)
    l1 = torch.empty_like(err) if want_l1 else None
    mm = torch.empty((bsz,), dtype=torch.float32, device=out.device) if want_mesh_mean else None
    call("cfsd_vertex_errors", ptr(out), ptr(gt), ptr(mean), ptr(std), ptr(err), ptr(l1),
         ptr(mm), bsz, nv, float(to_mm), stream_ptr())
    if not (want_l1 or want_mesh_mean):
        return err
    return (err,) + ((l1,) if want_l1 else ()) + ((mm,) if want_mesh_mean else ())


def reconstruction_error_stats(mesh_means):
    """The summary of ``Tester.reconstruction_errors`` (``test.py:298-301``)
    over the concatenated per-mesh means (device tensor, torch reductions)."""
    return {"mean": torch.mean(mesh_means).item(), "median": torch.median(mesh_means).item(),
            "max": torch.max(mesh_means).item(), "std": torch.std(mesh_means).item()}


# ------------------------------------------------------------------ bf16 path
# Mixed-precision entry points (include/cfsd.h "bf16 path"): activations /
# gradients are float32 or bfloat16 tensors, weights are the fp32 master view
# and its bf16 shadow view.
def cast(src, out):
    """fp32 <-> bf16 storage conversion (round to nearest even)."""
    _needx(src, None, "src")
    _needx(out, tuple(src.shape), "out")
    call("cfsd_cast", ptr(src), _dt(src), ptr(out), _dt(out), ctypes.c_size_t(src.numel()), stream_ptr())
    return out


def spiral_conv_fwd_x(x, idx, w, w_bf16, b, act, out):
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = w.shape[0]
    _needl(x, None, "x")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(w, (cout, seq * cin), name="w")
    if w_bf16 is not None:
        _need(w_bf16, (cout, seq * cin), torch.bfloat16, "w_bf16")
    if b is not None:
        _need(b, (cout,), name="bias")
    _needl(out, (bsz, rows, cout), "out")
    call("cfsd_spiral_conv_fwd_x", ptr(x), _st(x), ptr(idx), ptr(w), ptr(w_bf16), ptr(b), ptr(out),
         _st(out), bsz, vsrc, rows, seq, cin, cout, act, stream_ptr())
    return out


def spiral_conv_bwd_data_x(dpre, inv, w_bf16, vsrc, elu_y=None, out=None):
    bsz, rows, cout = dpre.shape
    inv_ptr, inv_row, inv_head = inv
    seq = (inv_ptr.numel() - 1) // vsrc
    cin = w_bf16.shape[1] // seq
    _needl(dpre, None, "dpre")
    _need(inv_ptr, (vsrc * seq + 1,), torch.int32, "inv_ptr")
    _need(inv_row, (rows * seq,), torch.int32, "inv_row")
    _need(inv_head, (vsrc * seq, INV_HEAD), torch.int32, "inv_head")
    _need(w_bf16, (cout, seq * cin), torch.bfloat16, "w_bf16")
    if out is None:
        out = torch.empty((bsz, vsrc, cin), dtype=torch.bfloat16, device=dpre.device)
    _needl(out, (bsz, vsrc, cin), "dx", torch.bfloat16)
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", torch.bfloat16)
        _same_layout(out, elu_y, "dx and elu_y")
    call("cfsd_spiral_conv_bwd_data_x", ptr(dpre), _st(dpre), ptr(inv_ptr), ptr(inv_row), ptr(inv_head),
         ptr(w_bf16), ptr(elu_y), ptr(out), _st(out), bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    return out


def spiral_conv_bwd_data_flat(dpre, flat, w, vsrc, elu_y=None, out=None):
    """dx of a vertex-major layer through the flat inverse list
    (``topology.spiral_flat``), batch a multiple of 16.  ``w`` bf16 (the
    shadow; dx / elu_y bf16) or fp32 (dx, elu_y and dpre fp32: the fp32
    step's vertex-major kernel)."""
    bsz, rows, cout = dpre.shape
    table, width = flat
    seq = 9
    cin = w.shape[1] // seq
    dt = w.dtype
    if dt not in (torch.float32, torch.bfloat16):
        raise ValueError(f"w must be fp32 or bf16, got {dt}")
    _needl(dpre, None, "dpre")
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w, (cout, seq * cin), dt, "w")
    if out is None:
        out = vm_empty(bsz, vsrc, cin, dtype=dt, device=dpre.device)
    _needl(out, (bsz, vsrc, cin), "dx", dt)
    if dt == torch.float32 and dpre.dtype != torch.float32:
        raise ValueError("fp32 dx needs fp32 dpre")
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", dt)
        _same_layout(out, elu_y, "dx and elu_y")
    call("cfsd_spiral_conv_bwd_data_flat", ptr(dpre), _st(dpre), ptr(table), width, ptr(w), ptr(elu_y),
         ptr(out), _st(out), bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    return out


def spiral_conv_bwd_weight_x_workspace(bsz, rows, seq, cin, cout, x_dtype=torch.bfloat16):
    """Workspace of :func:`spiral_conv_bwd_weight_x` (``x_dtype`` fp32: the
    fp32 kernels' slab geometry, as :func:`spiral_conv_bwd_weight_workspace`)."""
    if x_dtype == torch.float32:
        return spiral_conv_bwd_weight_workspace(bsz, rows, seq, cin, cout)
    return int(_abi.lib().cfsd_spiral_conv_bwd_weight_x_workspace(bsz, rows, seq, cin, cout))


def spiral_conv_bwd_weight_x(x, idx, dpre, dw, db, workspace):
    """dW/db of a bf16-path conv (x / dpre fp32 or bf16); ``dw is db is None``
    defers the reduction (returns a DeferredDw for dw_reduce_batch)."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    _needl(x, None, "x")
    _need(idx, (rows, seq), torch.int32, "idx")
    _needl(dpre, (bsz, rows, cout), "dpre")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    _need(workspace, None, name="workspace")
    need = spiral_conv_bwd_weight_x_workspace(bsz, rows, seq, cin, cout, x.dtype)
    nbytes = workspace.numel() * workspace.element_size()
    if nbytes < need:
        raise ValueError(f"workspace {nbytes} < {need} bytes")
    call("cfsd_spiral_conv_bwd_weight_x", ptr(x), _st(x), ptr(idx), ptr(dpre), _st(dpre), ptr(dw), ptr(db),
         ptr(workspace), ctypes.c_size_t(nbytes), bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    if dw is None:  # bf16 32/64-channel slabs are plain (kind 2); fp32 x: the fp32 kernels' slabs
        mfma = cin in (32, 64) and cout in (32, 64) and x.dtype == torch.bfloat16
        # fp32 32 -> 32 with vertex-major x and dpre: conv_dw_vm32's slabs (3)
        vm32 = (x.dtype == torch.float32 and is_vm(x) and is_vm(dpre) and cin == 32 and cout == 32
                and bsz % 16 == 0)
        return DeferredDw(workspace, bsz, vsrc, rows, cin, cout, 2 if mfma else (3 if vm32 else 0))
    return None


def spiral_conv_bwd_flat_pair_workspace(bsz, rows, seq, cin, cout):
    return int(_abi.lib().cfsd_spiral_conv_bwd_flat_pair_workspace(bsz, rows, seq, cin, cout))


def spiral_conv_bwd_flat_pair(x, idx, dpre, flat, w, dw, db, dx, elu_y=None, workspace=None):
    """Both gradients of a full 32 -> 32 conv whose x, dpre, dx (and elu_y)
    are all vertex-major fp32 (the fp32 step's level-0/1 Deblocks) in ONE
    launch (``cfsd_spiral_conv_bwd_flat_pair``, ABI 4.10): the flat-list dx
    of :func:`spiral_conv_bwd_data_flat` and coarse-geometry dW slabs.
    ``dw is db is None`` defers the reduction (returns a DeferredDw)."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    table, width = flat
    for t, nm, shp in ((x, "x", (bsz, vsrc, cin)), (dpre, "dpre", (bsz, rows, cout)), (dx, "dx", (bsz, vsrc, cin))):
        _needl(t, shp, nm, torch.float32)
        if not is_vm(t):
            raise ValueError(f"spiral_conv_bwd_flat_pair: {nm} must be vertex-major")
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", torch.float32)
        _same_layout(dx, elu_y, "dx and elu_y")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w, (cout, seq * cin), torch.float32, "w")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    need = spiral_conv_bwd_flat_pair_workspace(bsz, rows, seq, cin, cout)
    if need == 0:
        raise ValueError(f"no vertex-major pair for {cin} -> {cout} channels")
    ws, nb = _conv_ws(workspace, x.device, need)
    call("cfsd_spiral_conv_bwd_flat_pair", ptr(x), ptr(idx), ptr(dpre), ptr(table), width, ptr(w), ptr(elu_y),
         ptr(dx), ptr(dw), ptr(db), ptr(ws), ctypes.c_size_t(nb), bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    if dw is None:
        return DeferredDw(ws, bsz, vsrc, rows, cin, cout, 3)
    return None


def spiral_conv_bwd_flat_pair_bf16(x, idx, dpre, flat, w16, dx, elu_y=None, workspace=None):
    """:func:`spiral_conv_bwd_flat_pair` on the bf16 step's tensors (x, dpre,
    dx, elu_y bf16 vertex-major; ``w16`` the bf16 weight shadow), always
    deferred (``cfsd_spiral_conv_bwd_flat_pair_bf16``, ABI 4.11): the dx of
    :func:`spiral_conv_bwd_data_flat` and the slabs of
    :func:`spiral_conv_bwd_weight_x` in one launch; returns the DeferredDw."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    table, width = flat
    for t, nm, shp in ((x, "x", (bsz, vsrc, cin)), (dpre, "dpre", (bsz, rows, cout)), (dx, "dx", (bsz, vsrc, cin))):
        _needl(t, shp, nm, torch.bfloat16)
        if not is_vm(t):
            raise ValueError(f"spiral_conv_bwd_flat_pair_bf16: {nm} must be vertex-major")
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", torch.bfloat16)
        _same_layout(dx, elu_y, "dx and elu_y")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w16, (cout, seq * cin), torch.bfloat16, "w16")
    _need(workspace, None, name="workspace")
    nbytes = workspace.numel() * workspace.element_size()
    call("cfsd_spiral_conv_bwd_flat_pair_bf16", ptr(x), ptr(idx), ptr(dpre), ptr(table), width, ptr(w16),
         ptr(elu_y), ptr(dx), ptr(workspace), ctypes.c_size_t(nbytes), bsz, vsrc, rows, seq, cin, cout,
         stream_ptr())
    return DeferredDw(workspace, bsz, vsrc, rows, cin, cout, 2)


def spiral_conv_bwd_rowsub_pair_bf16(x, idx, dpre, flat, w, dx, elu_y=None, workspace=None):
    """The bf16 step's Enblock backward in ONE launch
    (``cfsd_spiral_conv_bwd_rowsub_pair_bf16``, ABI 4.11): the dx of
    :func:`spiral_conv_bwd_data_rowsub` (fp32 batch-major ``dpre`` at the kept
    rows, fp32 ``w``; bf16 vertex-major ``dx`` / ``elu_y``) and the deferred
    slabs of :func:`spiral_conv_bwd_weight_x` (bf16 vertex-major ``x``);
    returns the DeferredDw."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    table, width = flat
    for t, nm in ((x, "x"), (dx, "dx")):
        _needl(t, (bsz, vsrc, cin), nm, torch.bfloat16)
        if not is_vm(t):
            raise ValueError(f"spiral_conv_bwd_rowsub_pair_bf16: {nm} must be vertex-major")
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", torch.bfloat16)
        _same_layout(dx, elu_y, "dx and elu_y")
    _need(dpre, (bsz, rows, cout), torch.float32, "dpre")
    _need(idx, (rows, seq), torch.int32, "idx")
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w, (cout, seq * cin), torch.float32, "w")
    _need(workspace, None, name="workspace")
    nbytes = workspace.numel() * workspace.element_size()
    call("cfsd_spiral_conv_bwd_rowsub_pair_bf16", ptr(x), ptr(idx), ptr(dpre), ptr(table), width, ptr(w),
         ptr(elu_y), ptr(dx), ptr(workspace), ctypes.c_size_t(nbytes), bsz, vsrc, rows, seq, cin, cout,
         stream_ptr())
    return DeferredDw(workspace, bsz, vsrc, rows, cin, cout, 2)


def spiral_conv_bwd_x(x, idx, dpre, inv, w, dw, db, dx=None, elu_y=None, workspace=None):
    """Fused dx + dW of the xyz output conv with bf16 (or fp32) x / elu_y /
    dx in either layout."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    inv_ptr, inv_row, inv_head = inv
    xdt = x.dtype
    if xdt not in (torch.float32, torch.bfloat16):
        raise ValueError(f"x must be fp32 or bf16, got {xdt}")
    _needl(x, None, "x", xdt)
    _need(idx, (rows, seq), torch.int32, "idx")
    _needl(dpre, (bsz, rows, cout), "dpre", torch.float32)
    _need(inv_head, (vsrc * seq, INV_HEAD), torch.int32, "inv_head")
    _need(w, (cout, seq * cin), name="w")
    if dx is not None:
        _needl(dx, (bsz, vsrc, cin), "dx", xdt)
        _same_layout(x, dx, "x and dx")
    if elu_y is not None:
        _needl(elu_y, (bsz, vsrc, cin), "elu_y", xdt)
        _same_layout(x, elu_y, "x and elu_y")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    ws, nb = _conv_ws(workspace, x.device, spiral_conv_bwd_workspace(bsz, vsrc, rows, seq, cin, cout))
    call("cfsd_spiral_conv_bwd_x", ptr(x), _st(x), ptr(idx), ptr(dpre), _st(dpre), ptr(inv_ptr), ptr(inv_row),
         ptr(inv_head), ptr(w), ptr(elu_y), ptr(dx), ptr(dw), ptr(db), ptr(ws), ctypes.c_size_t(nb),
         bsz, vsrc, rows, seq, cin, cout, stream_ptr())
    if dw is None:
        return dx, DeferredDw(ws, bsz, vsrc, rows, cin, cout, 1)
    return dx


def spiral_conv_bwd_out_flat(x, idx, dpre, flat, w, dw, db, dx=None, elu_y=None, workspace=None):
    """Fused dx + dW of the xyz output conv (32 -> 3) with vertex-major x /
    elu_y / dx (fp32 or bf16) and dpre, through the flat inverse list
    (``topology.spiral_flat``); batch a multiple of 16."""
    bsz, vsrc, cin = x.shape
    rows, seq = idx.shape
    cout = dpre.shape[2]
    table, width = flat
    xdt = x.dtype
    if not (is_vm(x) and is_vm(dpre)):
        raise ValueError("x and dpre must be vertex-major")
    _needl(x, None, "x", xdt)
    _need(idx, (rows, seq), torch.int32, "idx")
    _needl(dpre, (bsz, rows, cout), "dpre", torch.float32)
    _need(table, (vsrc, width), torch.int32, "inv_flat")
    _need(w, (cout, seq * cin), name="w")
    for t, nm in ((dx, "dx"), (elu_y, "elu_y")):
        if t is not None:
            _needl(t, (bsz, vsrc, cin), nm, xdt)
            _same_layout(x, t, f"x and {nm}")
    if dw is not None or db is not None:
        _need(dw, (cout, seq * cin), name="dw")
        _need(db, (cout,), name="db")
    ws, nb = _conv_ws(workspace, x.device, spiral_conv_bwd_workspace(bsz, vsrc, rows, seq, cin, cout))
    call("cfsd_spiral_conv_bwd_out_flat", ptr(x), _st(x), ptr(idx), ptr(dpre), _st(dpre), ptr(table), width,
         ptr(w), ptr(elu_y), ptr(dx), ptr(dw), ptr(db), ptr(ws), ctypes.c_size_t(nb), bsz, vsrc, rows, seq, cin,
         cout, stream_ptr())
    if dw is None:
        return dx, DeferredDw(ws, bsz, vsrc, rows, cin, cout, 1)
    return dx


def spmm_x(csr, x, m, elu_y=None, out=None, order=None, uniform=0, sched=None):
    """Pool SpMM with fp32 or bf16 operands (fp32 sums, file order)."""
    row_ptr, col, val = csr
    bsz, n, c = x.shape
    _needl(x, None, "x")
    _need(row_ptr, (m + 1,), torch.int32, "row_ptr")
    _need(col, None, torch.int32, "col")
    _need(val, (col.numel(),), name="val")
    _needl(out, (bsz, m, c), "out")
    if elu_y is not None:
        _needl(elu_y, (bsz, m, c), "elu_y", out.dtype)
        _same_layout(out, elu_y, "out and elu_y")
    if sched is not None:
        _spmm_sched_csr(sched, x, elu_y, out, bsz, m, n, c)
        return out
    if order is not None:
        _spmm_sched(row_ptr, col, val, order, x, elu_y, out, bsz, m, n, c)
        return out
    if uniform:
        _spmm_uniform(uniform, col, val, x, elu_y, out, bsz, m, n, c)
        return out
    call("cfsd_spmm_csr_x", ptr(row_ptr), ptr(col), ptr(val), ptr(x), _st(x), ptr(elu_y), ptr(out),
         _st(out), bsz, m, n, c, stream_ptr())
    return out
