"""fp32 vertex-major path (the C2 step's level-0/1 tensors stored
[nv][batch][c], batch % 16 == 0): every kernel against the batch-major fp32
kernels and the float64 oracle on the same inputs, then the whole fp32 step
in both layouts.

Tolerances (stated per test): the vertex-major forward runs the batch-major
kernel's products in the same order (bit-identical, torch.equal); the data
gradient walks the flat inverse list (model.py:34's index_add_ order) instead
of per-slot row sums, and the weight gradient visits rows vertex-major, so
those agree with the float64 oracle to fp32 summation error (rel 1e-5 of the
largest magnitude) and with the batch-major kernels to the same bound.
Reference: model.py:27-55 (+ autograd), model_manager.py:274-326.
"""
import numpy as np
import pytest
import torch

import cfsd_loader
import recipe
from oracle import cfsd_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
torch.set_num_threads(1)


@pytest.fixture(scope="module")
def mods():
    cfsd_loader.load()
    from craniofacialsd_vae_amd import engine as E
    from craniofacialsd_vae_amd import ops, topology
    return E, ops, topology


@pytest.fixture(scope="module")
def dtopo(mods, topo_npz):
    return mods[2].DeviceTopology.from_npz(topo_npz, device=DEV)


def err_rel_max(got, ref):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return float((got - ref).abs().max() / (ref.abs().max() + 1e-30))


def gather(x, sp):
    idx = torch.as_tensor(np.asarray(sp), dtype=torch.long)
    return torch.index_select(x, 1, idx.reshape(-1)).view(x.shape[0], idx.shape[0], -1)


# (level, batch, cout): the C2 layers (16 meshes) plus a 32-mesh batch and a 64-wide output
FWD_CASES = [(0, 16, 32), (1, 16, 32), (1, 32, 32), (2, 16, 64), (3, 48, 32)]


@pytest.mark.parametrize("level,bsz,cout", FWD_CASES)
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("yvm", [True, False])
def test_fwd_vm32_bit_exact(mods, otopo, dtopo, level, bsz, cout, act, yvm):
    """Same products, same K order as the batch-major persistent kernel
    (conv_fwd_mfma, which the batch-major path runs at levels 0/1): torch.equal
    there; the coarse levels' batch-major kernels sum in a different order
    (rel 1e-5 of the largest magnitude)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(level * 31 + bsz + cout + act)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    x = torch.randn(bsz, v, 32, generator=g).to(DEV)
    w = (torch.randn(cout, 288, generator=g) * 0.1).to(DEV)
    bias = torch.randn(cout, generator=g).to(DEV)
    idx = dtopo.spiral[level]
    ref = ops.spiral_conv_fwd(x, idx, w, bias, act)
    y = ops.vm_empty(bsz, v, cout, device=DEV) if yvm else torch.empty(bsz, v, cout, device=DEV)
    ops.spiral_conv_fwd_x(ops.to_vm(x), idx, w, None, bias, act, y)
    assert ops.is_vm(y) == yvm
    if level <= 1:
        assert torch.equal(y.contiguous(), ref)
    else:
        assert err_rel_max(y, ref) <= 1e-5
    # and the float64 oracle
    r64 = gather(x.double().cpu(), sp) @ w.double().cpu().T + bias.double().cpu()
    if act:
        r64 = torch.nn.functional.elu(r64)
    assert err_rel_max(y, r64) <= 1e-5


def test_fwd_vm32_row_subset(mods, otopo, dtopo):
    """E1 at the kept rows: vertex-major level-1 x, batch-major level-2 y
    (model.py:50-55 with the 0/1 Pool folded in).  The batch-major path runs
    its latency-shaped kernel here (another summation order): rel 1e-5."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(5)
    x = torch.randn(16, dtopo.n_verts[1], 32, generator=g).to(DEV)
    w = (torch.randn(32, 288, generator=g) * 0.1).to(DEV)
    bias = torch.randn(32, generator=g).to(DEV)
    idx = dtopo.enc_rows[1]
    ref = ops.spiral_conv_fwd(x, idx, w, bias, 1)
    y = torch.empty_like(ref)
    ops.spiral_conv_fwd_x(ops.to_vm(x), idx, w, None, bias, 1, y)
    assert err_rel_max(y, ref) <= 1e-5


@pytest.mark.parametrize("level,bsz,cout", [(0, 16, 32), (1, 16, 32), (1, 32, 64), (2, 16, 32), (3, 48, 32)])
@pytest.mark.parametrize("with_elu", [False, True])
def test_dx_flat_vm32(mods, otopo, dtopo, level, bsz, cout, with_elu):
    """fp32 flat-list data gradient vs float64 autograd of gather + Linear and
    vs the batch-major fp32 kernel: rel 1e-5 of the largest magnitude."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(level * 7 + bsz + cout)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    y = torch.nn.functional.elu(torch.randn(bsz, v, 32, generator=g))
    w = torch.randn(cout, 288, generator=g) * 0.1
    dpre = torch.randn(bsz, v, cout, generator=g)
    xl = y.double().requires_grad_()
    (gather(xl, sp) @ w.double().T).backward(dpre.double())
    ref = xl.grad * (torch.where(y.double() > 0, 1.0, y.double() + 1.0) if with_elu else 1.0)
    dp = ops.to_vm(dpre.to(DEV))
    ey = ops.to_vm(y.to(DEV)) if with_elu else None
    dx = ops.spiral_conv_bwd_data_flat(dp, dtopo.spiral_flat[level], w.to(DEV), v, elu_y=ey)
    assert ops.is_vm(dx) and dx.dtype == torch.float32
    assert err_rel_max(dx, ref) <= 1e-5
    bm = ops.spiral_conv_bwd_data(dpre.to(DEV), dtopo.spiral_inv[level], w.to(DEV), v,
                                  elu_y=y.to(DEV) if with_elu else None)
    assert err_rel_max(dx, bm) <= 1e-5
    dx2 = ops.spiral_conv_bwd_data_flat(dp, dtopo.spiral_flat[level], w.to(DEV), v, elu_y=ey)
    assert torch.equal(dx, dx2)  # deterministic


@pytest.mark.parametrize("table,level,bsz,cout,dpvm", [("dec", 0, 16, 32, True), ("dec", 1, 16, 32, True),
                                                       ("dec", 1, 32, 64, True), ("dec", 3, 16, 32, True),
                                                       ("enc", 1, 16, 32, False), ("enc", 1, 16, 64, False)])
def test_dw_vm32(mods, otopo, dtopo, table, level, bsz, cout, dpvm):
    """Weight gradient with vertex-major x (persistent and latency-shaped
    geometries; E1's batch-major level-2 dpre) vs float64 and vs the
    batch-major fp32 kernel; deferred slabs through the batched reduce give
    the same values as the direct reduce."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(level * 3 + bsz + cout + dpvm)
    idx = dtopo.spiral[level] if table == "dec" else dtopo.enc_rows[level]  # Enblock: the kept rows
    sp = idx.cpu().numpy()
    v = dtopo.n_verts[level]
    rows = sp.shape[0]
    x = torch.randn(bsz, v, 32, generator=g)
    dpre = torch.randn(bsz, rows, cout, generator=g)
    gx = gather(x.double(), sp).reshape(bsz * rows, -1)
    dref = dpre.double().reshape(bsz * rows, cout)
    dw_ref, db_ref = dref.T @ gx, dref.sum(0)
    nb = ops.spiral_conv_bwd_weight_x_workspace(bsz, rows, 9, 32, cout, torch.float32)
    ws = torch.zeros(nb // 4 + 64, device=DEV)
    dw = torch.empty(cout, 288, device=DEV)
    db = torch.empty(cout, device=DEV)
    dp_dev = ops.to_vm(dpre.to(DEV)) if dpvm else dpre.to(DEV)
    ops.spiral_conv_bwd_weight_x(ops.to_vm(x.to(DEV)), idx, dp_dev, dw, db, ws)
    assert err_rel_max(dw, dw_ref) <= 1e-5 and err_rel_max(db, db_ref) <= 1e-5
    dw_bm, db_bm = torch.empty_like(dw), torch.empty_like(db)
    ops.spiral_conv_bwd_weight(x.to(DEV), idx, dpre.to(DEV), dw_bm, db_bm, ws)
    assert err_rel_max(dw, dw_bm) <= 1e-5 and err_rel_max(db, db_bm) <= 1e-5
    ws.zero_()
    d = ops.spiral_conv_bwd_weight_x(ops.to_vm(x.to(DEV)), idx, dp_dev, None, None, ws)
    dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
    ops.dw_reduce_batch([(d, dw2, db2)])
    assert torch.equal(dw2, dw) and torch.equal(db2, db)


@pytest.mark.parametrize("level,bsz", [(0, 16), (1, 16), (1, 32)])
@pytest.mark.parametrize("with_elu", [False, True])
def test_bwd_flat_pair_vm32(mods, otopo, dtopo, level, bsz, with_elu):
    """cfsd_spiral_conv_bwd_flat_pair (ABI 4.10: the flat-list dx and the
    vm32 dW slabs as interleaved workgroups of one launch, every operand
    vertex-major fp32): dx and dW / db bit-identical to
    cfsd_spiral_conv_bwd_data_flat + cfsd_spiral_conv_bwd_weight_x (same
    bodies, same slab split); dW vs float64 rel 1e-5; the deferred slabs
    through the batched reduce == the direct reduce."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(level * 5 + bsz + with_elu)
    idx = dtopo.spiral[level]
    sp = idx.cpu().numpy()
    v = dtopo.n_verts[level]
    x = torch.nn.functional.elu(torch.randn(bsz, v, 32, generator=g))
    w = torch.randn(32, 288, generator=g) * 0.1
    dpre = torch.randn(bsz, v, 32, generator=g)
    gx = gather(x.double(), sp).reshape(bsz * v, -1)
    dref = dpre.double().reshape(bsz * v, 32)
    dw_ref, db_ref = dref.T @ gx, dref.sum(0)
    xv, dpv = ops.to_vm(x.to(DEV)), ops.to_vm(dpre.to(DEV))
    ey = xv if with_elu else None
    flat = dtopo.spiral_flat[level]
    nb = ops.spiral_conv_bwd_flat_pair_workspace(bsz, v, 9, 32, 32)
    assert nb > 0
    ws = torch.zeros(nb // 4 + 64, device=DEV)
    dw, db = torch.empty(32, 288, device=DEV), torch.empty(32, device=DEV)
    dx = ops.vm_empty(bsz, v, 32, device=DEV)
    ops.spiral_conv_bwd_flat_pair(xv, idx, dpv, flat, w.to(DEV), dw, db, dx, elu_y=ey, workspace=ws)
    dx_ref = ops.spiral_conv_bwd_data_flat(dpv, flat, w.to(DEV), v, elu_y=ey)
    assert torch.equal(dx, dx_ref)
    assert err_rel_max(dw, dw_ref) <= 1e-5 and err_rel_max(db, db_ref) <= 1e-5
    nbx = ops.spiral_conv_bwd_weight_x_workspace(bsz, v, 9, 32, 32, torch.float32)
    wsx = torch.zeros(nbx // 4 + 64, device=DEV)
    dw_x, db_x = torch.empty_like(dw), torch.empty_like(db)
    ops.spiral_conv_bwd_weight_x(xv, idx, dpv, dw_x, db_x, wsx)
    assert torch.equal(dw, dw_x) and torch.equal(db, db_x)
    ws.zero_()
    dx2 = ops.vm_empty(bsz, v, 32, device=DEV)
    d = ops.spiral_conv_bwd_flat_pair(xv, idx, dpv, flat, w.to(DEV), None, None, dx2, elu_y=ey, workspace=ws)
    dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
    ops.dw_reduce_batch([(d, dw2, db2)])
    assert torch.equal(dx2, dx) and torch.equal(dw2, dw) and torch.equal(db2, db)


def test_xyz_layers_vm32(mods, otopo, dtopo):
    """The xyz input / output layers with fp32 vertex-major 32-channel
    operands: forwards bit-exact to batch-major; the fused output backward's
    dx and dW, and the input layer's dW, within fp32 summation error."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(11)
    bsz, v0, v1 = 16, dtopo.n_verts[0], dtopo.n_verts[1]
    x = torch.randn(bsz, v0, 3, generator=g).to(DEV)
    w_in = (torch.randn(32, 27, generator=g) * 0.3).to(DEV)
    b_in = torch.randn(32, generator=g).to(DEV)
    ref = ops.spiral_conv_fwd(x, dtopo.enc_rows[0], w_in, b_in, 1)
    y = ops.vm_empty(bsz, v1, 32, device=DEV)
    ops.spiral_conv_fwd_x(x, dtopo.enc_rows[0], w_in, None, b_in, 1, y)
    assert torch.equal(y.contiguous(), ref)
    h = torch.nn.functional.elu(torch.randn(bsz, v0, 32, generator=g)).to(DEV)
    w_out = (torch.randn(3, 288, generator=g) * 0.1).to(DEV)
    b_out = torch.randn(3, generator=g).to(DEV)
    ref = ops.spiral_conv_fwd(h, dtopo.spiral[0], w_out, b_out, 0)
    out = torch.empty_like(ref)
    hv = ops.to_vm(h)
    ops.spiral_conv_fwd_x(hv, dtopo.spiral[0], w_out, None, b_out, 0, out)
    assert torch.equal(out, ref)
    # fused output backward
    dout = torch.randn(bsz, v0, 3, generator=g).to(DEV)
    dx_bm = torch.empty(bsz, v0, 32, device=DEV)
    dw_bm, db_bm = torch.empty(3, 288, device=DEV), torch.empty(3, device=DEV)
    ops.spiral_conv_bwd(h, dtopo.spiral[0], dout, dtopo.spiral_inv[0], w_out, dw_bm, db_bm, dx=dx_bm, elu_y=h)
    dx = ops.vm_empty(bsz, v0, 32, device=DEV)
    dw, db = torch.empty_like(dw_bm), torch.empty_like(db_bm)
    ops.spiral_conv_bwd_x(hv, dtopo.spiral[0], dout, dtopo.spiral_inv[0], w_out, dw, db, dx=dx, elu_y=hv)
    assert err_rel_max(dx, dx_bm) <= 1e-5
    assert err_rel_max(dw, dw_bm) <= 1e-5 and err_rel_max(db, db_bm) <= 1e-5
    # input layer dW with a vertex-major fp32 dpre
    dpre = torch.randn(bsz, v1, 32, generator=g).to(DEV)
    nb = ops.spiral_conv_bwd_weight_x_workspace(bsz, v1, 9, 3, 32, torch.float32)
    ws = torch.zeros(nb // 4 + 64, device=DEV)
    dwi, dbi = torch.empty(32, 27, device=DEV), torch.empty(32, device=DEV)
    ops.spiral_conv_bwd_weight_x(x, dtopo.enc_rows[0], ops.to_vm(dpre), dwi, dbi, ws)
    dwi_bm, dbi_bm = torch.empty_like(dwi), torch.empty_like(dbi)
    ops.spiral_conv_bwd_weight(x, dtopo.enc_rows[0], dpre, dwi_bm, dbi_bm, ws)
    assert err_rel_max(dwi, dwi_bm) <= 1e-5 and err_rel_max(dbi, dbi_bm) <= 1e-5


def test_fp32_step_vertex_major_vs_batch_major(mods, dtopo):
    """Three C2 train steps (batch 16) in both fp32 layouts from the same
    weights and batches: the forward is bit-identical, the gradients differ
    only in fp32 summation order, so losses agree to 1e-5 relative and the
    parameters after three Adam steps to 1e-5 of their magnitude."""
    E, ops, _ = mods
    w = recipe.golden_weights()
    meshes = torch.from_numpy(recipe.normalized_meshes(12)).to(DEV)
    res = []
    for vm in (False, True):
        eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV, vertex_major=vm)
        eng.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
        b = eng.buffers(16)
        assert ops.is_vm(b.dec_out[-1]) == vm and eng.vm_levels(16) == ({0, 1} if vm else set())
        losses = []
        for step in range(3):
            eng.inject(b, recipe.train_key_index(step), torch.from_numpy(recipe.train_eps(step)))
            b.batch_idx.copy_(torch.arange(4 * step, 4 * step + 4, dtype=torch.int32))
            ops.swap_features(meshes, b.batch_idx, dtopo.region_mask, b.key, 4, out=b.x)
            if step == 0:  # forward only: bit-identical outputs
                eng.forward(b, train=True)
                out0 = b.out.clone()
            eng.train_step_on(b)
            torch.cuda.synchronize()
            losses.append(b.losses.cpu().clone())
        res.append((out0, torch.stack(losses), eng.params.data.cpu().clone(), eng.params.grad.cpu().clone()))
    (o_bm, l_bm, p_bm, g_bm), (o_vm, l_vm, p_vm, g_vm) = res
    assert torch.equal(o_bm, o_vm)  # every forward kernel: same products in the same order
    assert float(((l_vm - l_bm).abs() / l_bm.abs().clamp_min(1e-12)).max()) <= 1e-5
    assert err_rel_max(p_vm, p_bm) <= 1e-5
    assert err_rel_max(g_vm, g_bm) <= 1e-4


def test_fp32_vm_graph_step_matches_eager(mods, dtopo):
    """The resident fp32 vertex-major step captured in a hipGraph and replayed
    equals the same number of eager steps bit for bit."""
    E, _, _ = mods
    w = recipe.golden_weights()
    res = []
    for use_graph in (False, True):
        data = E.ResidentData(torch.from_numpy(recipe.normalized_meshes(12)).to(DEV), bs=4, shuffle=True)
        eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV)
        eng.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
        b = eng.buffers(16)
        step = lambda: eng.resident_step(b, data)  # noqa: E731
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                step()
            for _ in range(3):
                gr.replay()
        else:
            for _ in range(4):
                step()
        torch.cuda.synchronize()
        res.append((eng.params.data.cpu().clone(), b.losses.cpu().clone()))
        assert torch.isfinite(res[-1][1]).all()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_swap_and_losses_vertex_major(mods, dtopo):
    """Level-0 xyz tensors in the vertex-major layout: the feature swap
    (swap_batch_transform.py:13-42) and the MSE + Laplacian passes
    (model_manager.py:333-349) give the batch-major values element for
    element (same per-row arithmetic); the reduced losses are sums in another
    order (rel 1e-6)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(3)
    nv = dtopo.n_verts[0]
    data = torch.randn(12, nv, 3, generator=g).to(DEV)
    idx = torch.tensor([1, 5, 7, 9], dtype=torch.int32, device=DEV)
    key = torch.tensor([2], dtype=torch.int32, device=DEV)
    x_bm = ops.swap_features(data, idx, dtopo.region_mask, key, 4)
    x_vm = ops.vm_empty(16, nv, 3, device=DEV)
    ops.swap_features(data, idx, dtopo.region_mask, key, 4, out=x_vm)
    assert ops.is_vm(x_vm) and torch.equal(x_vm.contiguous(), x_bm)
    pred = torch.randn(16, nv, 3, generator=g).to(DEV)
    res = []
    for vm in (False, True):
        mk = (lambda: ops.vm_empty(16, nv, 3, device=DEV)) if vm else (lambda: torch.empty(16, nv, 3, device=DEV))
        p, x, unit, dout = mk(), mk(), mk(), mk()
        p.copy_(pred)
        x.copy_(x_bm)
        parts = torch.empty(2 * ops.recon_lap_blocks(16, nv), device=DEV)
        terms = torch.tensor([0.5, 0.25], device=DEV)
        losses = torch.empty(5, device=DEV)
        ops.recon_lap_fwd(p, x, dtopo.lap_csr, unit, parts)
        ops.recon_lap_bwd_finalize(p, x, unit, dtopo.lapT_csr, dout, 1.0, 0.1, parts, terms, losses, None,
                                   1e-4, 0.5)
        torch.cuda.synchronize()
        res.append((unit.contiguous().cpu(), dout.contiguous().cpu(), losses.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert err_rel_max(res[1][2], res[0][2]) <= 1e-6


@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("bsz", [16, 32])
def test_bwd_out_flat(mods, otopo, dtopo, xdt, bsz):
    """Vertex-major fused backward of the xyz output conv (model.py:172-173
    autograd) through the flat inverse list, against float64 autograd of
    gather + Linear on the same (storage-rounded) operands: dx rel 1e-5 (+ one
    bf16 rounding for bf16 storage), dW / db rel 1e-5; deferred slabs reduce
    to the same values."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(bsz + (7 if xdt == torch.bfloat16 else 0))
    sp = otopo.spirals[0]
    v = sp.shape[0]
    h = torch.nn.functional.elu(torch.randn(bsz, v, 32, generator=g)).to(xdt)
    w = torch.randn(3, 288, generator=g) * 0.1
    dout = torch.randn(bsz, v, 3, generator=g)
    hl = h.double().requires_grad_()
    wl = w.double().requires_grad_()
    (gather(hl, sp) @ wl.T).backward(dout.double())
    ref_dx = hl.grad * torch.where(h.double() > 0, 1.0, h.double() + 1.0)
    hv = ops.to_vm(h.to(DEV))
    dx = ops.vm_empty(bsz, v, 32, dtype=xdt, device=DEV)
    dw, db = torch.empty(3, 288, device=DEV), torch.empty(3, device=DEV)
    dv = ops.to_vm(dout.to(DEV))
    ops.spiral_conv_bwd_out_flat(hv, dtopo.spiral[0], dv, dtopo.spiral_flat[0], w.to(DEV), dw, db, dx=dx, elu_y=hv)
    tol = 1e-5 if xdt == torch.float32 else 2.0 ** -8
    assert err_rel_max(dx.float(), ref_dx) <= tol
    assert err_rel_max(dw, wl.grad) <= 1e-5
    assert err_rel_max(db, dout.double().sum((0, 1))) <= 1e-5
    dx2 = ops.vm_empty(bsz, v, 32, dtype=xdt, device=DEV)
    _, d = ops.spiral_conv_bwd_out_flat(hv, dtopo.spiral[0], dv, dtopo.spiral_flat[0], w.to(DEV), None, None,
                                        dx=dx2, elu_y=hv)
    dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
    ops.dw_reduce_batch([(d, dw2, db2)])
    assert torch.equal(dx2, dx) and torch.equal(dw2, dw) and torch.equal(db2, db)

