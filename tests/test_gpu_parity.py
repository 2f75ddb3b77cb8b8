"""HIP path vs the CPU oracle and the reference goldens (needs an MI355X).

Tolerances (fp32 everywhere):
* per-vertex L1 of reconstructions <= 1e-4 (BASELINE north_star), z <= 1e-4;
* per-op results: |hip - oracle| <= 1e-5 * (1 + max|oracle|) unless stated;
* Pool forward / backward and the feature swap: bit-exact (same fp32
  operation order as the reference's sequential scatter_add / index_add_).
"""
import numpy as np
import pytest
import torch

import cfsd_loader
import recipe
from oracle import cfsd_oracle as O

pytestmark = pytest.mark.gpu

cfsd_loader.load()
from craniofacialsd_vae_amd import engine as E  # noqa: E402
from craniofacialsd_vae_amd import ops, topology  # noqa: E402

DEV = "cuda"
torch.set_num_threads(1)


def close(a, b, rel=1e-5, what=""):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    tol = rel * (1.0 + np.abs(b).max())
    err = np.abs(a - b).max()
    assert err <= tol, f"{what}: max err {err:.3e} > tol {tol:.3e}"


@pytest.fixture(scope="module")
def dtopo(topo_npz):
    return topology.DeviceTopology.from_npz(topo_npz, device=DEV)


# --------------------------------------------------------------- spiral conv
# (cin, cout, level, batch): batches chosen so every slot-group split of the
# MFMA kernels is exercised (<400 tiles -> 1 slot/group, 400-2047 -> 3, >=2048 -> 9).
CONV_CASES = [(3, 32, 3, 3), (32, 32, 3, 3), (32, 64, 3, 3), (64, 32, 2, 3), (64, 64, 2, 3),
              (32, 3, 1, 2), (32, 32, 1, 2), (3, 32, 0, 2), (32, 3, 0, 2), (32, 32, 0, 2),
              (32, 32, 0, 4), (64, 32, 0, 4), (32, 64, 1, 16), (64, 64, 1, 16)]
# forward-only: the VALU 3-channel output kernel at its other input widths
FWD_ONLY_CASES = [(16, 3, 2, 2), (64, 3, 1, 2), (32, 3, 0, 16)]


@pytest.mark.parametrize("cin,cout,level,bsz", CONV_CASES + FWD_ONLY_CASES)
@pytest.mark.parametrize("act", [0, 1])
def test_spiral_conv_fwd(otopo, dtopo, cin, cout, level, bsz, act):
    g = torch.Generator().manual_seed(cin * 100 + cout + level)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    x = torch.randn(bsz, v, cin, generator=g)
    w = torch.randn(cout, 9 * cin, generator=g) * 0.1
    b = torch.randn(cout, generator=g) * 0.1
    ref = O.spiral_conv(x, sp, w, b)
    if act:
        ref = O.elu(ref)
    y = ops.spiral_conv_fwd(x.to(DEV), dtopo.spiral[level], w.to(DEV), b.to(DEV), act)
    close(y, ref, 1e-5, "conv fwd")


@pytest.mark.parametrize("cin,level,bsz", [(32, 0, 16), (64, 1, 3), (32, 3, 1), (4, 2, 2), (12, 4 - 1, 5)])
def test_spiral_gather_bit_exact(otopo, dtopo, cin, level, bsz):
    """Materialising gather (the HBM-roofline probe) == the reference's
    ``x.index_select(1, indices.view(-1)).view(B, V, -1)`` (model.py:34),
    bit-exact, including the ragged tail of the last block."""
    g = torch.Generator().manual_seed(7 + cin + level)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    x = torch.randn(bsz, v, cin, generator=g)
    ref = x.index_select(1, torch.as_tensor(sp, dtype=torch.long).reshape(-1)).view(bsz, v, -1)
    got = ops.spiral_gather(x.to(DEV), dtopo.spiral[level])
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("cin,cout,level,bsz", [c for c in CONV_CASES if c[0] != 3])
@pytest.mark.parametrize("use_elu_y", [False, True])
def test_spiral_conv_bwd(otopo, dtopo, cin, cout, level, bsz, use_elu_y):
    g = torch.Generator().manual_seed(7 + cin + cout + level)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    x = torch.randn(bsz, v, cin, generator=g).requires_grad_()
    xin = O.elu(x) if use_elu_y else x
    w = (torch.randn(cout, 9 * cin, generator=g) * 0.1).requires_grad_()
    b = (torch.randn(cout, generator=g) * 0.1).requires_grad_()
    xin_leaf = xin.detach().requires_grad_()
    y = O.spiral_conv(xin_leaf, sp, w, b)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    dx_ref = xin_leaf.grad
    if use_elu_y:
        dx_ref = torch.autograd.grad(xin, x, dx_ref)[0]
    dpre = dy.to(DEV)
    dx = ops.spiral_conv_bwd_data(dpre, dtopo.spiral_inv[level], w.detach().to(DEV), v,
                                  elu_y=xin.detach().to(DEV) if use_elu_y else None)
    close(dx, dx_ref, 1e-5, "conv dx")
    dw = torch.empty(cout, 9 * cin, device=DEV)
    db = torch.empty(cout, device=DEV)
    ws = torch.empty(ops.spiral_conv_bwd_weight_workspace(bsz, v, 9, cin, cout) // 4 + 1, device=DEV)
    ops.spiral_conv_bwd_weight(xin.detach().to(DEV).contiguous(), dtopo.spiral[level], dpre, dw, db, ws)
    close(dw, w.grad, 1e-5, "conv dw")
    close(db, b.grad, 1e-5, "conv db")


@pytest.mark.parametrize("cin,cout,level,bsz", [(32, 3, 0, 2), (32, 3, 0, 16), (64, 3, 1, 5),
                                                (32, 3, 3, 1), (32, 32, 1, 2), (64, 64, 2, 3),
                                                (32, 1, 1, 2), (32, 2, 0, 2), (64, 1, 2, 3),
                                                (64, 2, 1, 2)])
@pytest.mark.parametrize("with_dx", [False, True])
def test_spiral_conv_bwd_fused(otopo, dtopo, cin, cout, level, bsz, with_dx):
    """cfsd_spiral_conv_bwd (dX + dW/db in one call; source-row pass for 3-ch outputs)."""
    g = torch.Generator().manual_seed(11 + cin + cout + level + bsz)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    # reference in float64: dW sums up to 16*17039 products, so an fp32 oracle's
    # own rounding would dominate the comparison
    x = torch.randn(bsz, v, cin, generator=g).double().requires_grad_()
    xin = O.elu(x)
    xin_leaf = xin.detach().requires_grad_()
    w = (torch.randn(cout, 9 * cin, generator=g) * 0.1).float().double().requires_grad_()
    b = (torch.randn(cout, generator=g) * 0.1).double().requires_grad_()
    y = O.spiral_conv(xin_leaf, sp, w, b)
    dy = torch.randn(y.shape, generator=g).double()
    y.backward(dy)
    dx_ref = torch.autograd.grad(xin, x, xin_leaf.grad)[0]
    dw = torch.full((cout, 9 * cin), float("nan"), device=DEV)
    db = torch.full((cout,), float("nan"), device=DEV)
    dx = torch.full((bsz, v, cin), float("nan"), device=DEV) if with_dx else None
    xd = xin.detach().float().to(DEV).contiguous()
    ops.spiral_conv_bwd(xd, dtopo.spiral[level], dy.float().to(DEV), dtopo.spiral_inv[level],
                        w.detach().float().to(DEV), dw, db, dx=dx, elu_y=xd if with_dx else None)
    close(dw, w.grad, 1e-5, "fused dw")
    close(db, b.grad, 1e-5, "fused db")
    if with_dx:
        close(dx, dx_ref, 1e-5, "fused dx")


# (table, level, cin, cout, batch): decoder tables and the Enblock row-subset
# tables (E1 at batch 16 is the 2-column-tile dx shape)
PAIR_CASES = [("dec", 1, 32, 32, 2), ("dec", 2, 64, 32, 3), ("dec", 3, 64, 32, 16), ("dec", 2, 64, 32, 16),
              ("enc", 1, 32, 32, 16), ("enc", 2, 32, 32, 16), ("enc", 3, 32, 32, 16), ("enc", 1, 32, 32, 3)]


@pytest.mark.parametrize("table,level,cin,cout,bsz", PAIR_CASES)
def test_spiral_conv_bwd_paired_bit_exact(dtopo, table, level, cin, cout, bsz):
    """The paired dx+dW launch (coarse layers) == the separate dx and dW
    kernels, bit for bit, deferred slabs included."""
    idx = dtopo.spiral[level] if table == "dec" else dtopo.enc_rows[level]
    inv = dtopo.spiral_inv[level] if table == "dec" else dtopo.enc_inv[level]
    vsrc, rows = dtopo.n_verts[level], idx.shape[0]
    if not ops.spiral_conv_bwd_paired(bsz, vsrc, rows, 9, cin, cout):
        pytest.skip("coarse layer: dx on the slot-group kernel (cfsd_spiral_conv_bwd does not pair)")
    g = torch.Generator(device=DEV).manual_seed(level * 10 + cin + cout + bsz)
    x = torch.randn(bsz, vsrc, cin, device=DEV, generator=g)
    y = torch.nn.functional.elu(x)
    dpre = torch.randn(bsz, rows, cout, device=DEV, generator=g)
    w = torch.randn(cout, 9 * cin, device=DEV, generator=g) * 0.1
    ws_sz = ops.spiral_conv_bwd_workspace(bsz, vsrc, rows, 9, cin, cout)
    ws = torch.zeros(ws_sz // 4 + 1, device=DEV)
    dx_p = torch.full((bsz, vsrc, cin), float("nan"), device=DEV)
    dw_p, db_p = torch.empty(cout, 9 * cin, device=DEV), torch.empty(cout, device=DEV)
    ops.spiral_conv_bwd(y, idx, dpre, inv, w, dw_p, db_p, dx=dx_p, elu_y=y, workspace=ws)
    dx_s = ops.spiral_conv_bwd_data(dpre, inv, w, vsrc, elu_y=y)
    dw_s, db_s = torch.empty_like(dw_p), torch.empty_like(db_p)
    ws2 = torch.zeros(ops.spiral_conv_bwd_weight_workspace(bsz, rows, 9, cin, cout) // 4 + 1, device=DEV)
    ops.spiral_conv_bwd_weight(y, idx, dpre, dw_s, db_s, ws2)
    assert torch.equal(dx_p, dx_s)
    assert torch.equal(dw_p, dw_s) and torch.equal(db_p, db_s)
    # deferred: slabs reduced by the batched reduce
    ws.zero_()
    dx_d = torch.empty_like(dx_p)
    _, d = ops.spiral_conv_bwd(y, idx, dpre, inv, w, None, None, dx=dx_d, elu_y=y, workspace=ws)
    dw_d, db_d = torch.empty_like(dw_p), torch.empty_like(db_p)
    ops.dw_reduce_batch([(d, dw_d, db_d)])
    assert torch.equal(dx_d, dx_s) and torch.equal(dw_d, dw_s) and torch.equal(db_d, db_s)


@pytest.mark.parametrize("bsz", [2, 16])
def test_spiral_conv_e0_weight_grad(otopo, dtopo, bsz):
    g = torch.Generator().manual_seed(3)
    sp = otopo.spirals[0]
    x = torch.randn(bsz, sp.shape[0], 3, generator=g)
    w = (torch.randn(32, 27, generator=g) * 0.1).requires_grad_()
    b = torch.zeros(32).requires_grad_()
    sel = torch.from_numpy(otopo.down[0][1])
    y = O.spiral_conv(x, sp, w, b)[:, sel]
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    dw = torch.empty(32, 27, device=DEV)
    db = torch.empty(32, device=DEV)
    ws = torch.empty(ops.spiral_conv_bwd_weight_workspace(bsz, 4260, 9, 3, 32) // 4 + 1, device=DEV)
    ops.spiral_conv_bwd_weight(x.to(DEV), dtopo.enc_rows[0], dy.to(DEV), dw, db, ws)
    close(dw, w.grad, 1e-5, "E0 dw")
    close(db, b.grad, 1e-5, "E0 db")


def test_enblock_row_subset_equals_conv_then_pool(otopo, dtopo):
    """Pool(down) of a selection transform == conv evaluated at kept rows."""
    g = torch.Generator().manual_seed(5)
    for level in range(4):
        sp = otopo.spirals[level]
        cin = 3 if level == 0 else 32
        x = torch.randn(2, sp.shape[0], cin, generator=g)
        w = torch.randn(32, 9 * cin, generator=g) * 0.1
        b = torch.randn(32, generator=g) * 0.1
        ref = O.pool(O.elu(O.spiral_conv(x, sp, w, b)), otopo.down[level])
        y = ops.spiral_conv_fwd(x.to(DEV), dtopo.enc_rows[level], w.to(DEV), b.to(DEV), 1)
        close(y, ref, 1e-5, f"enblock level {level}")


# --------------------------------------------------------------- pool
@pytest.mark.parametrize("level", [0, 1, 2, 3])
@pytest.mark.parametrize("kind", ["up", "down"])
def test_pool_bit_exact(otopo, dtopo, level, kind):
    coo = (otopo.up if kind == "up" else otopo.down)[level]
    csr = (dtopo.up_csr if kind == "up" else dtopo.down_csr)[level]
    csrT = (dtopo.upT_csr if kind == "up" else dtopo.downT_csr)[level]
    m, n = coo[3]
    g = torch.Generator().manual_seed(level)
    x = torch.randn(2, n, 32, generator=g).requires_grad_()
    out = O.pool(x, coo)
    dout = torch.randn(out.shape, generator=g)
    out.backward(dout)
    y = ops.spmm(csr, x.detach().to(DEV), m)
    np.testing.assert_array_equal(y.cpu().numpy(), out.detach().numpy())
    dx = ops.spmm(csrT, dout.to(DEV), n)
    np.testing.assert_array_equal(dx.cpu().numpy(), x.grad.numpy())
    if kind == "up":  # uniform-row forward and long-row schedule of the transpose: same bits
        assert dtopo.up_uniform[level] == 3
        yu = ops.spmm(csr, x.detach().to(DEV), m, uniform=dtopo.up_uniform[level])
        np.testing.assert_array_equal(yu.cpu().numpy(), out.detach().numpy())
        assert dtopo.upT_order[level] is not None
        dxs = ops.spmm(csrT, dout.to(DEV), n, order=dtopo.upT_order[level])
        np.testing.assert_array_equal(dxs.cpu().numpy(), x.grad.numpy())


@pytest.mark.parametrize("bsz", [16, 3])
@pytest.mark.parametrize("dts", [("f32", "f32"), ("bf16", "bf16"), ("bf16", "f32")])
def test_pool_scheduled_transpose(dtopo, bsz, dts):
    """cfsd_spmm_csr_sched and cfsd_spmm_sched_csr == cfsd_spmm_csr(_x) bit for bit (every level, with the
    ELU-backward epilogue, XCD mesh groups and the single-group fallback)."""
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}
    g = torch.Generator().manual_seed(bsz)
    for level in range(4):
        m, n = dtopo.n_verts[level + 1], dtopo.n_verts[level]
        x = torch.randn(bsz, n, 32, generator=g).to(DEV, dt[dts[0]])
        ey = O.elu(torch.randn(bsz, m, 32, generator=g)).to(DEV, dt[dts[1]])
        a = torch.empty(bsz, m, 32, device=DEV, dtype=dt[dts[1]])
        b = torch.empty_like(a)
        ops.spmm_x(dtopo.upT_csr[level], x, m, elu_y=ey, out=a)
        ops.spmm_x(dtopo.upT_csr[level], x, m, elu_y=ey, out=b, order=dtopo.upT_order[level])
        assert torch.equal(a, b), f"level {level}"
        b.zero_()
        ops.spmm_x(dtopo.upT_csr[level], x, m, elu_y=ey, out=b, sched=dtopo.upT_sched[level])
        assert torch.equal(a, b), f"level {level} (visiting-order CSR)"
        # vertex-major source (the engine's levels 0/1): XCD-contiguous row ranges, either order
        xv, eyv = ops.to_vm(x), ops.to_vm(ey)
        for sch in (dtopo.upT_sched[level], dtopo.upT_nat[level]):
            if sch is None:
                continue
            c = ops.vm_empty(bsz, m, 32, dtype=dt[dts[1]], device=DEV)
            ops.spmm_x(dtopo.upT_csr[level], xv, m, elu_y=eyv, out=c, sched=sch)
            assert torch.equal(a, c), f"level {level} (vertex-major)"


@pytest.mark.parametrize("bsz", [16, 3])
@pytest.mark.parametrize("dts", [("f32", "f32"), ("bf16", "bf16"), ("f32", "bf16"), ("bf16", "f32")])
def test_pool_uniform_rows(dtopo, bsz, dts):
    """cfsd_spmm_uniform == cfsd_spmm_csr(_x) bit for bit on the 3-tap up-sampling
    matrices (every level, with and without the ELU-backward epilogue, ragged
    thread tails at bsz 3)."""
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}
    g = torch.Generator().manual_seed(100 + bsz)
    for level in range(4):
        m, n = dtopo.n_verts[level], dtopo.n_verts[level + 1]
        k = dtopo.up_uniform[level]
        assert k == 3
        x = torch.randn(bsz, n, 32, generator=g).to(DEV, dt[dts[0]])
        ey = O.elu(torch.randn(bsz, m, 32, generator=g)).to(DEV, dt[dts[1]])
        for e in (None, ey):
            a = torch.empty(bsz, m, 32, device=DEV, dtype=dt[dts[1]])
            b = torch.empty_like(a)
            ops.spmm_x(dtopo.up_csr[level], x, m, elu_y=e, out=a)
            ops.spmm_x(dtopo.up_csr[level], x, m, elu_y=e, out=b, uniform=k)
            assert torch.equal(a, b), f"level {level} elu {e is not None}"


def test_pool_golden(dtopo):
    gops = np.load(f"{recipe.HERE}/golden_ops.npz")
    for name, level, kind in (("down3", 3, "down"), ("up3", 3, "up"), ("up2", 2, "up")):
        csr = (dtopo.up_csr if kind == "up" else dtopo.down_csr)[level]
        csrT = (dtopo.upT_csr if kind == "up" else dtopo.downT_csr)[level]
        x = torch.from_numpy(gops[f"pool_{name}_x"]).to(DEV)
        out = gops[f"pool_{name}_out"]
        y = ops.spmm(csr, x, out.shape[1])
        np.testing.assert_array_equal(y.cpu().numpy(), out)
        dx = ops.spmm(csrT, torch.from_numpy(gops[f"pool_{name}_dout"]).to(DEV), x.shape[1])
        close(dx, gops[f"pool_{name}_dx"], 1e-6, "pool golden dx")


def test_conv_golden(dtopo):
    gops = np.load(f"{recipe.HERE}/golden_ops.npz")
    x = torch.from_numpy(gops["conv_x"]).to(DEV)
    w = torch.from_numpy(gops["conv_w"]).to(DEV)
    b = torch.from_numpy(gops["conv_b"]).to(DEV)
    y = ops.spiral_conv_fwd(x, dtopo.spiral[3], w, b, 0)
    close(y, gops["conv_y"], 1e-5, "golden conv y")
    dy = torch.from_numpy(gops["conv_dy"]).to(DEV)
    dx = ops.spiral_conv_bwd_data(dy, dtopo.spiral_inv[3], w, 267)
    close(dx, gops["conv_dx"], 1e-5, "golden conv dx")
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    ws = torch.empty(ops.spiral_conv_bwd_weight_workspace(2, 267, 9, 32, 64) // 4 + 1, device=DEV)
    ops.spiral_conv_bwd_weight(x, dtopo.spiral[3], dy, dw, db, ws)
    close(dw, gops["conv_dw"], 1e-5, "golden conv dw")
    close(db, gops["conv_db"], 1e-5, "golden conv db")


# --------------------------------------------------------------- swap
def test_swap_bit_exact(otopo, dtopo):
    gsw = np.load(f"{recipe.HERE}/golden_swap.npz")
    base = torch.from_numpy(recipe.normalized_meshes(4)).to(DEV)
    bidx = torch.arange(4, dtype=torch.int32, device=DEV)
    key = torch.zeros(1, dtype=torch.int32, device=DEV)
    for k in range(dtopo.n_regions):
        key.fill_(k)
        out = ops.swap_features(base, bidx, dtopo.region_mask, key, 4)
        assert recipe.sha256(out.cpu().numpy()) == str(gsw["sha"][k]), k


# --------------------------------------------------------------- full model
def make_engine(dtopo, weights, bs=4, precision="fp32", vertex_major=True):
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(), swap_bs=bs, device=DEV, precision=precision,
                        vertex_major=vertex_major)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in weights.items()})
    return eng


def test_state_dict_keys_match_reference(dtopo):
    eng = make_engine(dtopo, recipe.golden_weights())
    assert list(eng.state_dict().keys()) == [k for k, _ in recipe.param_shapes()]


def test_eval_c1_golden(dtopo):
    """C1: encode+decode of the first 8 demo meshes, eval mode (z = mu)."""
    g = np.load(f"{recipe.HERE}/golden_eval.npz")
    eng = make_engine(dtopo, recipe.golden_weights())
    b = eng.set_batch(torch.from_numpy(recipe.normalized_meshes(8)).to(DEV))
    eng.forward(b, train=False)
    torch.cuda.synchronize()
    d = np.abs(b.out.cpu().numpy() - g["recon"]).sum(-1)
    assert d.max() <= 1e-4, f"max per-vertex L1 {d.max():.3e}"
    assert np.abs(b.z.cpu().numpy() - g["z"]).max() <= 1e-4
    assert np.abs(b.mulv[:, 75:].cpu().numpy() - g["mu"]).max() <= 1e-4
    assert np.abs(b.mulv[:, :75].cpu().numpy() - g["logvar"]).max() <= 1e-4


def test_train_three_steps_golden(otopo, dtopo):
    """C2: three reference train steps (swap, fwd, 4 losses, bwd, Adam)."""
    g = np.load(f"{recipe.HERE}/golden_train.npz")
    w = recipe.golden_weights()
    eng = make_engine(dtopo, w)
    # oracle in lock-step for full-tensor gradient comparison
    P = O.make_params(w)
    opt = O.Adam(P)
    meshes = recipe.normalized_meshes(12)
    data = torch.from_numpy(meshes).to(DEV)
    for step in range(3):
        p = f"s{step}_"
        key = recipe.train_key_index(step)
        eps = torch.from_numpy(recipe.train_eps(step))
        out, grads, x16 = O.train_step(P, opt, meshes[4 * step:4 * step + 4], otopo, key, eps.numpy())
        b = eng.inject(eng.buffers(16), key, eps)
        b.batch_idx.copy_(torch.arange(4 * step, 4 * step + 4, dtype=torch.int32))
        ops.swap_features(data, b.batch_idx, dtopo.region_mask, b.key, 4, out=b.x)
        eng.train_step_on(b)
        torch.cuda.synchronize()
        assert recipe.sha256(b.x.cpu().numpy()) == str(g[p + "x_sha"])
        got = b.losses.cpu().numpy()
        np.testing.assert_allclose(got, g[p + "losses"], rtol=1e-4)
        np.testing.assert_allclose(b.z.cpu().numpy(), g[p + "z"], atol=1e-4)
        hip_grads = {k: v.cpu() for k, v in eng.grads().items()}
        for name in w:
            close(hip_grads[name], grads[name], 1e-4, f"step {step} grad {name}")
        sd = eng.state_dict()
        for name in w:
            close(sd[name], P[name].detach(), 2e-5, f"step {step} param {name}")
            ps = sd[name].cpu().numpy().ravel()
            np.testing.assert_allclose(ps[recipe.sample_idx(ps.size)], g[p + "param_sample_" + name],
                                       atol=2e-5)


@pytest.mark.parametrize("bs", [4, 1])
def test_train_steps_without_swap(otopo, dtopo, bs):
    """data config ``swap_features: False`` (data_loading.py:38, 81-82: no
    SwapFeatures in the collater): the step's batch is the bs picked meshes
    (cfsd_gather_meshes, bit-exact), latent consistency is 0
    (model_manager.py:290-293) -- also at bs = 1, where a swapped group would
    have bs^2 = bs rows -- and two steps (losses, every gradient, parameters
    after Adam) match the oracle's un-swapped _do_iteration.  Through
    step.TrainStep (the object the driver and the bench run)."""
    from craniofacialsd_vae_amd.step import TrainStep
    w = recipe.golden_weights()
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(), swap_bs=bs, device=DEV, swap_features=False)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    assert eng.step_rows == bs
    meshes = recipe.normalized_meshes(12)
    data = E.ResidentData(torch.from_numpy(meshes).to(DEV), bs=bs, shuffle=True)
    ts = TrainStep(eng, data)
    assert ts.b.bsz == bs
    P = O.make_params(w)
    opt = O.Adam(P)
    for step in range(2):
        ts.step()
        torch.cuda.synchronize()
        b = ts.b
        picked = b.batch_idx.cpu().numpy()
        assert len(set(picked.tolist())) == bs
        np.testing.assert_array_equal(b.x.cpu().numpy(), meshes[picked])
        out, grads, _ = O.train_step(P, opt, meshes[picked], otopo, None, b.eps.cpu().numpy(), swap=False)
        got = b.losses.cpu().numpy()
        assert got[2] == 0.0
        np.testing.assert_allclose(got, [out[k].item() for k in ("rec", "kl", "lc", "lap", "tot")],
                                   rtol=1e-4, atol=1e-7)
        hip_grads = {k: v.cpu() for k, v in eng.grads().items()}
        for name in w:
            close(hip_grads[name], grads[name], 1e-4, f"step {step} grad {name}")
        sd = eng.state_dict()
        for name in w:
            close(sd[name], P[name].detach(), 2e-5, f"step {step} param {name}")


def test_gather_meshes_layouts(dtopo):
    """cfsd_gather_meshes into either level-0 layout equals the host gather."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(7, dtopo.n_verts[0], 3, generator=g).to(DEV)
    idx = torch.tensor([5, 0, 6, 2] * 4, dtype=torch.int32, device=DEV)
    ref = x.cpu()[idx.cpu().long()]
    y = ops.gather_meshes(x, idx, 16)
    assert torch.equal(y.cpu(), ref)
    yv = ops.vm_empty(16, dtopo.n_verts[0], 3, dtype=torch.float32, device=DEV)
    ops.gather_meshes(x, idx, 16, out=yv)
    assert torch.equal(yv.cpu(), ref)


def test_train_step_deterministic(dtopo):
    w = recipe.golden_weights()
    outs = []
    for _ in range(2):
        eng = make_engine(dtopo, w)
        b = eng.set_batch(torch.from_numpy(
            O.swap_features(recipe.normalized_meshes(4), [np.asarray(r) for r in
                                                          O.Topology(recipe.load_topology()).region_features], 2)).to(DEV),
            key_index=2, eps=torch.from_numpy(recipe.train_eps(0)).to(DEV))
        eng.train_step_on(b)
        torch.cuda.synchronize()
        outs.append((eng.params.data.cpu().clone(), eng.params.grad.cpu().clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("precision,vertex_major", [("fp32", True), ("fp32", False), ("bf16", True)])
def test_fused_reduce_adam_matches_separate(dtopo, precision, vertex_major):
    """The single-process step's fused update (cfsd_dw_reduce_batch_adam)
    == cfsd_dw_reduce_batch + cfsd_adam, bit for bit: parameters, gradients,
    both Adam moments and (bf16) the weight shadow after two steps; in bf16
    also the bf16-MFMA weight-gradient items."""
    w = recipe.golden_weights()
    x = torch.from_numpy(O.swap_features(recipe.normalized_meshes(4), [np.asarray(r) for r in
                                         O.Topology(recipe.load_topology()).region_features], 2)).to(DEV)
    eps = torch.from_numpy(recipe.train_eps(0)).to(DEV)
    outs = []
    for mode in ("fused", "separate"):
        eng = make_engine(dtopo, w, precision=precision, vertex_major=vertex_major)
        for _ in range(2):
            b = eng.set_batch(x, key_index=2, eps=eps)
            if mode != "separate":
                eng.train_step_on(b)
            else:
                eng.advance_step(b)
                eng.forward(b, train=True, finalize=False)
                eng.backward(b)
                eng.adam_step()
        torch.cuda.synchronize()
        P = eng.params
        bufs = [P.data, P.grad, P.exp_avg, P.exp_avg_sq] + ([P.shadow] if P.shadow is not None else [])
        outs.append([t.cpu().clone() for t in bufs])
    assert len(outs[0]) == (5 if precision == "bf16" else 4)
    for other in outs[1:]:
        for a, c in zip(outs[0], other):
            assert torch.equal(a, c)


@pytest.mark.parametrize("precision,vertex_major", [("fp32", True), ("fp32", False), ("bf16", True)])
def test_fused_bottleneck_matches_four_launches(dtopo, precision, vertex_major):
    """cfsd_bottleneck_bwd (ABI 4.8: coarsest Pool(up)^T + decoder Linear +
    latent head + encoder Linear in one launch, later workgroups waiting on
    device counters) == spmm + linear_bwd_split + latent_bwd + linear_bwd,
    bit for bit over two whole training steps: parameters, gradients, Adam
    moments, dmulv and the encoder-Linear data gradient; the counters are
    left zero."""
    w = recipe.golden_weights()
    x = torch.from_numpy(O.swap_features(recipe.normalized_meshes(4), [np.asarray(r) for r in
                                         O.Topology(recipe.load_topology()).region_features], 2)).to(DEV)
    eps = torch.from_numpy(recipe.train_eps(0)).to(DEV)
    outs = []
    for fused in (False, True):
        eng = make_engine(dtopo, w, precision=precision, vertex_major=vertex_major)
        eng.fuse_bottleneck = fused
        for _ in range(2):
            b = eng.set_batch(x, key_index=2, eps=eps)
            assert eng._fused_bottleneck_ok(b) == fused
            eng.train_step_on(b)
        torch.cuda.synchronize()
        P = eng.params
        last = eng.spec.enc_layers()[-1][2]
        outs.append([t.cpu().clone() for t in (P.data, P.grad, P.exp_avg, P.exp_avg_sq, b.dmulv,
                                               b.dpre_enc[last])])
        if fused:
            assert not b.bn_sync.any()
    for a, c in zip(*outs):
        assert torch.equal(a, c)


@pytest.mark.parametrize("precision,vertex_major", [("fp32", True), ("fp32", False), ("bf16", True)])
def test_swap_in_first_conv_matches_two_launches(dtopo, precision, vertex_major):
    """cfsd_spiral_conv_fwd_in_swap (ABI 4.9: the feature swap and the first
    Enblock's xyz conv as two roles of one launch, the conv gathering through
    the swap from the resident set) == swap_features + the conv launch, bit
    for bit over two resident-data training steps: the swapped batch, the
    first Enblock's output, parameters and gradients."""
    from craniofacialsd_vae_amd.step import TrainStep
    data_meshes = torch.from_numpy(recipe.normalized_meshes(12)).to(DEV)
    outs = []
    for fused in (False, True):
        eng = make_engine(dtopo, recipe.golden_weights(), precision=precision, vertex_major=vertex_major)
        eng.fuse_swap = fused
        data = E.ResidentData(data_meshes.clone(), bs=4, shuffle=True)
        ts = TrainStep(eng, data)
        assert eng._swap_in_conv_ok(ts.b, data) == fused
        for _ in range(2):
            ts.step()
        torch.cuda.synchronize()
        grads = eng.grads()
        outs.append([ts.b.x.cpu().clone(), ts.b.enc_out[0].float().cpu()]
                    + [v.cpu().clone() for v in eng.state_dict().values()] + [grads[k].cpu().clone() for k in grads])
    assert len(outs[0]) == len(outs[1])
    for a, c in zip(*outs):
        assert torch.equal(a, c)


@pytest.mark.parametrize("is_vae,select,sigmoid", [(1, True, 0), (0, True, 1), (1, False, 0)])
def test_bottleneck_bwd_op_vs_separate(is_vae, select, sigmoid):
    """The op on random operands (batch 16, the craniofacial bottleneck: 267
    -> 67 coarse vertices x 64 channels, latent 75, encoder flat 4288) ==
    the four separate launches, bit for bit, three calls in a row (the
    counters reset themselves); VAE / plain-AE-with-sigmoid latent heads, with
    and without the encoder-Linear ELU."""
    g = torch.Generator().manual_seed(7 + is_vae + 2 * select)
    rnd = lambda *s: torch.randn(*s, generator=g).to(DEV)
    B, L, cup, n_up, nv, ke = 16, 75, 64, 267, 67, 4288
    ne = 2 * L if is_vae else L
    # a Pool(up)^T-shaped CSR: each fine vertex feeds 3 coarse vertices
    cols = [[] for _ in range(nv)]
    for f in range(n_up):
        for k in range(3):
            cols[(f * 7 + k * 11) % nv].append((f, 0.1 + 0.3 * k))
    row_ptr = torch.tensor([0] + list(np.cumsum([len(c) for c in cols])), dtype=torch.int32, device=DEV)
    col = torch.tensor([f for c in cols for f, _ in c], dtype=torch.int32, device=DEV)
    val = torch.tensor([v for c in cols for _, v in c], dtype=torch.float32, device=DEV)
    gfine0, z, wd = rnd(B, n_up, cup), rnd(B, L), rnd(nv * cup, L)
    mulv, epsv, dlat0 = rnd(B, ne), rnd(B, L), rnd(B, 3 * L)
    zval = torch.sigmoid(z)
    xe, we = rnd(B, ke), rnd(ne, ke)
    elu_y = torch.nn.functional.elu(rnd(B, ke)) if select else None
    parts_n = ops.linear_bwd_split_parts(nv * cup)
    hist_s, hist_f = [], []
    res = []
    for fused in (False, True):
        gfine, dlat = gfine0.clone(), dlat0.clone()
        out = dict(dwd=torch.zeros(nv * cup, L, device=DEV),
                   dbd=torch.zeros(nv * cup, device=DEV), dmulv=torch.zeros(B, ne, device=DEV),
                   dxe=torch.zeros(B, ke, device=DEV), dwe=torch.zeros(ne, ke, device=DEV),
                   dbe=torch.zeros(ne, device=DEV))
        sync = torch.zeros(ops.BN_SYNC_INTS, dtype=torch.int32, device=DEV)
        parts = torch.zeros(parts_n, B, L, device=DEV)
        xchg = torch.full((ops.bottleneck_exchange_floats(B, L, nv * cup, ne),), float("nan"), device=DEV)
        zin = zval if (sigmoid and not is_vae) else z
        for it in range(3):  # fresh operands per call: a stale cached value from the previous call would show
            gfine.mul_(0.5 + it)
            dlat.add_(0.25)
            if fused:
                ops.bottleneck_bwd((row_ptr, col, val), gfine, zin, wd, xchg, out["dwd"], out["dbd"], mulv,
                                   epsv, dlat, out["dmulv"], is_vae, sigmoid, xe, we, out["dxe"], out["dwe"],
                                   out["dbe"], sync, elu_y=elu_y)
            else:
                dh = ops.spmm((row_ptr, col, val), gfine, nv)
                ops.linear_bwd_split(zin, wd, dh.view(B, -1), parts, out["dwd"], out["dbd"])
                ops.latent_bwd(mulv, epsv, zin, parts, dlat, out["dmulv"], L, True, is_vae, sigmoid)
                ops.linear_bwd(xe, we, out["dmulv"], dx=out["dxe"], dw=out["dwe"], db=out["dbe"], elu_y=elu_y)
            res_it = {k: v.cpu().clone() for k, v in out.items()}
            res.append(res_it) if it == 2 else None
            (hist_f if fused else hist_s).append(res_it)
        torch.cuda.synchronize()
        if fused:
            assert not sync.any()
    for a_, c_ in zip(hist_s, hist_f):  # every call, not only the last
        for k in a_:
            assert torch.equal(a_[k], c_[k]), k
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k


# (batch, latent, is_vae, sigmoid, coarse vertices, cup, fine vertices, encoder width, ELU)
BN_STRESS = [(16, 75, 1, 0, 67, 64, 267, 4288, True), (1, 75, 1, 0, 67, 64, 267, 4288, False),
             (3, 33, 0, 1, 27, 64, 108, 1728, True), (7, 80, 1, 0, 20, 128, 80, 2560, True),
             (16, 128, 0, 0, 80, 64, 320, 5120, True), (5, 16, 1, 0, 80, 64, 320, 1000, False),
             (16, 2, 0, 1, 1, 64, 4, 64, True), (9, 75, 1, 0, 67, 64, 267, 4288, True)]


def test_bottleneck_bwd_stress_varied_shapes():
    """the one-launch bottleneck backward's counter hand-offs,
    run many times in ONE process over varied batch / latent / grid sizes
    (so its workgroups land on different XCDs and CUs from case to case)
    against the four separate launches -- bit for bit on every call, the
    counters left zero and the sticky timed-out-wait word never set."""
    for case_i, (B, L, is_vae, sigmoid, nv, cup, n_up, ke, select) in enumerate(BN_STRESS):
        g = torch.Generator().manual_seed(100 + case_i)
        rnd = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
        ne = 2 * L if is_vae else L
        cols = [[] for _ in range(nv)]
        for f in range(n_up):
            for k in range(3):
                cols[(f * 7 + k * 11) % nv].append((f, 0.1 + 0.3 * k))
        row_ptr = torch.tensor([0] + list(np.cumsum([len(c) for c in cols])), dtype=torch.int32, device=DEV)
        col = torch.tensor([f for c in cols for f, _ in c], dtype=torch.int32, device=DEV)
        val = torch.tensor([v for c in cols for _, v in c], dtype=torch.float32, device=DEV)
        z, wd, mulv, epsv = rnd(B, L), rnd(nv * cup, L), rnd(B, ne), rnd(B, L)
        zin = torch.sigmoid(z) if (sigmoid and not is_vae) else z
        xe, we = rnd(B, ke), rnd(ne, ke)
        elu_y = torch.nn.functional.elu(rnd(B, ke)) if select else None
        parts = torch.zeros(ops.linear_bwd_split_parts(nv * cup), B, L, device=DEV)
        xchg = torch.zeros(ops.bottleneck_exchange_floats(B, L, nv * cup, ne), device=DEV)
        sync = torch.zeros(ops.BN_SYNC_INTS, dtype=torch.int32, device=DEV)
        outs = [{k: torch.zeros(*s, device=DEV) for k, s in
                 (("dwd", (nv * cup, L)), ("dbd", (nv * cup,)), ("dmulv", (B, ne)), ("dxe", (B, ke)),
                  ("dwe", (ne, ke)), ("dbe", (ne,)))} for _ in range(2)]
        for it in range(12):
            gfine, dlat = rnd(B, n_up, cup), rnd(B, 3 * L)
            s_, f_ = outs
            dh = ops.spmm((row_ptr, col, val), gfine, nv)
            ops.linear_bwd_split(zin, wd, dh.view(B, -1), parts, s_["dwd"], s_["dbd"])
            ops.latent_bwd(mulv, epsv, zin, parts, dlat, s_["dmulv"], L, True, is_vae, sigmoid)
            ops.linear_bwd(xe, we, s_["dmulv"], dx=s_["dxe"], dw=s_["dwe"], db=s_["dbe"], elu_y=elu_y)
            ops.bottleneck_bwd((row_ptr, col, val), gfine, zin, wd, xchg, f_["dwd"], f_["dbd"], mulv, epsv, dlat,
                               f_["dmulv"], is_vae, sigmoid, xe, we, f_["dxe"], f_["dwe"], f_["dbe"], sync,
                               elu_y=elu_y)
            for k in s_:
                assert torch.equal(s_[k], f_[k]), (case_i, it, k)
        assert not sync.any(), case_i
        ops.bottleneck_check(sync)
    # the sticky word is what the host refuses
    sync[ops.BN_SYNC_ERR] = 2
    with pytest.raises(RuntimeError, match="timed out"):
        ops.bottleneck_check(sync)


# --------------------------------------------------------------- dense Linears
# Both bottleneck shapes of the model (encoder [m x 4288] -> 150 stacked
# mu/logvar, decoder 75 -> 4288) plus ragged m (not a multiple of the 4-row /
# 16-row groups).  Torch fp32 reference, tolerance rel 1e-5 (k <= 4288 terms).
LINEAR_CASES = [(16, 4288, 150), (16, 75, 4288), (5, 4288, 150), (3, 75, 4288), (1, 600, 7),
                (20, 64, 33), (18, 1000, 600)]


@pytest.mark.parametrize("m,k,n", LINEAR_CASES)
def test_linear_fwd(m, k, n):
    g = torch.Generator().manual_seed(m * 7 + k + n)
    x, w, b = torch.randn(m, k, generator=g), torch.randn(n, k, generator=g) * 0.05, torch.randn(n, generator=g)
    y = ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV))
    close(y, x.double() @ w.double().T + b.double(), 1e-5, "linear fwd")


@pytest.mark.parametrize("m,k,n", LINEAR_CASES)
@pytest.mark.parametrize("elu,accumulate", [(False, False), (True, False), (False, True)])
def test_linear_bwd(m, k, n, elu, accumulate):
    g = torch.Generator().manual_seed(m + k * 3 + n)
    x, w = torch.randn(m, k, generator=g), torch.randn(n, k, generator=g) * 0.05
    dy = torch.randn(m, n, generator=g)
    ey = O.elu(torch.randn(m, k, generator=g)) if elu else None
    dx0 = torch.randn(m, k, generator=g)
    dx_ref = dy.double() @ w.double()
    if elu:
        dx_ref = dx_ref * torch.where(ey > 0, torch.ones_like(ey), ey + 1).double()
    if accumulate:
        dx_ref = dx_ref + dx0.double()
    dx = dx0.clone().to(DEV) if accumulate else torch.empty(m, k, device=DEV)
    dw, db = torch.empty(n, k, device=DEV), torch.empty(n, device=DEV)
    ops.linear_bwd(x.to(DEV), w.to(DEV), dy.to(DEV), dx=dx, dw=dw, db=db,
                   elu_y=ey.to(DEV) if elu else None, accumulate=accumulate)
    close(dx, dx_ref, 1e-5, "linear dx")
    close(dw, dy.double().T @ x.double(), 1e-5, "linear dw")
    close(db, dy.double().sum(0), 1e-5, "linear db")


@pytest.mark.parametrize("m,k,n", [(16, 75, 4288), (3, 33, 200), (16, 128, 65)])
def test_linear_bwd_split(m, k, n):
    """Decoder-Linear backward in one launch: dW/db exact-order sums, dx as
    64-row-slice partial products that sum (in slice order) to dy.W."""
    g = torch.Generator().manual_seed(m + k + n)
    x, w = torch.randn(m, k, generator=g), torch.randn(n, k, generator=g) * 0.05
    dy = torch.randn(m, n, generator=g)
    parts = torch.empty(ops.linear_bwd_split_parts(n), m, k, device=DEV)
    dw, db = torch.empty(n, k, device=DEV), torch.empty(n, device=DEV)
    ops.linear_bwd_split(x.to(DEV), w.to(DEV), dy.to(DEV), parts, dw, db)
    close(parts.sum(0), dy.double() @ w.double(), 1e-5, "split dx")
    close(dw, dy.double().T @ x.double(), 1e-5, "split dw")
    close(db, dy.double().sum(0), 1e-5, "split db")
    # the latent head's backward sums the parts like one dz
    L = k
    mulv = torch.randn(m, 2 * L, generator=g).to(DEV)
    eps = torch.randn(m, L, generator=g).to(DEV)
    dlat = torch.randn(m, 3 * L, generator=g).to(DEV)
    a, b = torch.empty(m, 2 * L, device=DEV), torch.empty(m, 2 * L, device=DEV)
    z = torch.zeros(m, L, device=DEV)
    ops.latent_bwd(mulv, eps, z, parts, dlat, a, L, True, True, False)
    dz = torch.zeros(m, L, device=DEV)
    for p in range(parts.shape[0]):
        dz += parts[p]
    ops.latent_bwd(mulv, eps, z, dz, dlat, b, L, True, True, False)
    assert torch.equal(a, b)


# --------------------------------------------------------------- latent head
@pytest.mark.parametrize("key,bs", [(0, 4), (7, 4), (14, 4), (3, 9), (11, 16)])
def test_latent_head_vs_oracle(key, bs):
    """Reparameterisation + KL + latent consistency (fwd terms and dz/dmu/dlogvar);
    bs 9 and 16 (batch 81 / 256) run the head with > 64 KB of dynamic LDS."""
    g = torch.Generator().manual_seed(key)
    L = 75
    B = bs * bs
    mu = torch.randn(B, L, generator=g).double().requires_grad_()
    lv = (torch.randn(B, L, generator=g) * 0.3).double().requires_grad_()
    eps = torch.randn(B, L, generator=g)
    z = mu + eps.double() * torch.exp(0.5 * lv)
    regions = O.latent_regions(15, L)
    kl = O.kl_loss(mu, lv)
    lc = O.latent_consistency(z, regions[key], bs)
    (1e-4 * kl + 0.5 * lc).backward()
    mulv = torch.cat([lv, mu], 1).detach().float().to(DEV)
    zz, dlat, terms = torch.empty(B, L, device=DEV), torch.empty(B, 3 * L, device=DEV), torch.empty(2, device=DEV)
    keyt = torch.full((1,), key, dtype=torch.int32, device=DEV)
    ops.latent_fwd(mulv, eps.to(DEV), keyt, zz, dlat, terms, L, 5, True, True, False, 1e-4, 0.5, 0.5, 0.5)
    close(zz, z.detach(), 1e-5, "z")
    close(terms[0], kl.detach(), 1e-5, "kl")
    close(terms[1], lc.detach(), 1e-5, "lc")
    dmulv = torch.empty_like(mulv)
    ops.latent_bwd(mulv, eps.to(DEV), zz, torch.zeros(B, L, device=DEV), dlat, dmulv, L, True, True, False)
    close(dmulv[:, L:], mu.grad, 1e-5, "dmu")
    close(dmulv[:, :L], lv.grad, 1e-5, "dlogvar")


def test_graph_replay_matches_eager(dtopo):
    """The hipGraph-captured resident step (device-side batch pick, key and
    noise) gives bit-identical parameters and losses to eager launches."""
    w = recipe.golden_weights()
    res = []
    for use_graph in (False, True):
        data = E.ResidentData(torch.from_numpy(recipe.normalized_meshes(12)).to(DEV), bs=4,
                              rows=list(range(11, -1, -1)), shuffle=True)
        eng = make_engine(dtopo, w)
        b = eng.buffers(16)
        step = lambda: eng.resident_step(b, data)  # noqa: E731
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            for _ in range(3):
                g.replay()
        else:
            for _ in range(4):
                step()
        torch.cuda.synchronize()
        res.append((eng.params.data.cpu().clone(), b.losses.cpu().clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


def test_deferred_weight_grads_batch_reduce(otopo, dtopo):
    """Deferred dW (partials left in per-layer workspaces) reduced by ONE
    cfsd_dw_reduce_batch launch == the per-layer reductions, bit for bit
    (same fixed summation order); covers MFMA, 3-channel and fused kinds."""
    g = torch.Generator().manual_seed(21)
    cases = [(32, 32, 0, 4, otopo.spirals[0]), (64, 64, 2, 3, otopo.spirals[2]),
             (3, 32, 1, 2, otopo.spirals[1]), (32, 3, 1, 2, otopo.spirals[1])]
    items, refs = [], []
    for cin, cout, level, bsz, sp in cases:
        v = sp.shape[0]
        x = torch.randn(bsz, v, cin, generator=g).to(DEV)
        dpre = torch.randn(bsz, v, cout, generator=g).to(DEV)
        nb = ops.spiral_conv_bwd_weight_workspace(bsz, v, 9, cin, cout)
        dw, db = torch.empty(cout, 9 * cin, device=DEV), torch.empty(cout, device=DEV)
        ops.spiral_conv_bwd_weight(x, dtopo.spiral[level], dpre, dw, db,
                                   torch.empty(nb // 4 + 1, device=DEV))
        refs.append((dw, db))
        d = ops.spiral_conv_bwd_weight(x, dtopo.spiral[level], dpre, None, None,
                                       torch.empty(nb // 4 + 1, device=DEV))
        items.append((d, torch.full_like(dw, float("nan")), torch.full_like(db, float("nan"))))
    # fused xyz-output backward, deferred
    sp = otopo.spirals[0]
    x = torch.randn(2, sp.shape[0], 32, generator=g).to(DEV)
    dpre = torch.randn(2, sp.shape[0], 3, generator=g).to(DEV)
    w = torch.randn(3, 288, generator=g).to(DEV)
    dw, db = torch.empty(3, 288, device=DEV), torch.empty(3, device=DEV)
    ops.spiral_conv_bwd(x, dtopo.spiral[0], dpre, dtopo.spiral_inv[0], w, dw, db)
    refs.append((dw, db))
    _, d = ops.spiral_conv_bwd(x, dtopo.spiral[0], dpre, dtopo.spiral_inv[0], w, None, None,
                               workspace=torch.empty(ops.spiral_conv_bwd_workspace(2, sp.shape[0], sp.shape[0], 9, 32, 3) // 4 + 1, device=DEV))
    items.append((d, torch.full_like(dw, float("nan")), torch.full_like(db, float("nan"))))
    ops.dw_reduce_batch(items)
    torch.cuda.synchronize()
    for (d, dw, db), (rw, rb) in zip(items, refs):
        assert torch.equal(dw, rw) and torch.equal(db, rb)


@pytest.mark.parametrize("n,wd", [(1, 0.0), (4099, 0.0), (1082403, 0.0), (1027, 1e-2)])
def test_adam_matches_torch(n, wd):
    """cfsd_adam == torch.optim.Adam (the reference's optimiser,
    model_manager.py: torch.optim.Adam(lr, weight_decay)), 3 steps, vectorised
    body + n % 4 tail."""
    g = torch.Generator().manual_seed(n)
    p0 = torch.randn(n, generator=g)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=1e-3, weight_decay=wd, foreach=False)
    p, m, v = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    for _ in range(3):
        gr = torch.randn(n, generator=g)
        ref.grad = gr.clone()
        opt.step()
        step += 1
        ops.adam(p, gr.to(DEV), m, v, step, 1e-3, weight_decay=wd)
    close(p, ref.detach(), 1e-6, "adam param")
    close(m, opt.state[ref]["exp_avg"], 1e-6, "adam m")


@pytest.mark.parametrize("n,world", [(1081881, 2), (1023, 8), (7, 3)])
def test_adam_scaled_equals_scale_then_adam(n, world):
    """cfsd_adam_scaled (the data-parallel step's 1/world averaging folded into
    Adam) == cfsd_scale then cfsd_adam, bit for bit: parameters, both moments,
    the bf16 shadow and the scaled gradient left in `grad`."""
    g = torch.Generator().manual_seed(n + world)
    p0, gr0 = torch.randn(n, generator=g).to(DEV), torch.randn(n, generator=g).to(DEV)
    step = torch.full((1,), 3, dtype=torch.int32, device=DEV)
    outs = []
    for fused in (False, True):
        p, gr = p0.clone(), gr0.clone()
        m, v = torch.full((n,), 0.1, device=DEV), torch.full((n,), 0.2, device=DEV)
        sh = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        if fused:
            ops.adam_scaled(p, gr, m, v, step, 1.0 / world, 1e-3, weight_decay=1e-4, shadow=sh)
        else:
            ops.scale(gr, 1.0 / world)
            ops.adam(p, gr, m, v, step, 1e-3, weight_decay=1e-4, shadow=sh)
        outs.append((p, gr, m, v, sh))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


# --------------------------------------------------------------- evaluation (a17, f4)
@pytest.mark.parametrize("bsz,nv,normalise", [(1, 67, False), (3, 1065, True), (16, 17039, False)])
def test_vertex_errors_vs_oracle(bsz, nv, normalise):
    """cfsd_vertex_errors vs ``compute_vertex_errors`` (model_manager.py:395-400,
    oracle.vertex_errors) and the per-mesh mean of test.py:297.  Tolerance:
    rel. 1e-6 per vertex (same fp32 operation order, contraction off), 1e-6 for
    the mesh mean (fixed-order tree vs torch's CPU reduction)."""
    g = torch.Generator().manual_seed(bsz * 7 + nv)
    out = torch.randn(bsz, nv, 3, generator=g)
    gt = torch.randn(bsz, nv, 3, generator=g)
    mean = torch.randn(nv, 3, generator=g) if normalise else None
    std = torch.rand(nv, 3, generator=g) + 0.5 if normalise else None
    ro, rg = (out * std + mean, gt * std + mean) if normalise else (out, gt)
    ref = O.vertex_errors(ro, rg, to_mm=89.11)
    dev = (lambda t: None if t is None else t.to(DEV))
    err, l1, mm = ops.vertex_errors(out.to(DEV), gt.to(DEV), to_mm=89.11, mean=dev(mean),
                                    std=dev(std), want_l1=True, want_mesh_mean=True)
    torch.cuda.synchronize()
    close(err, ref, rel=1e-6, what="vertex err (mm)")
    close(l1, (ro - rg).abs().sum(-1), rel=1e-6, what="per-vertex L1")
    close(mm, torch.mean(ref, dim=1), rel=1e-6, what="per-mesh mean")


def test_reconstruction_errors_c1(dtopo):
    """Tester.reconstruction_errors (test.py:280-301) on the C1 demo batch:
    device recon + un-normalised device errors vs the oracle's errors of the
    reference's golden reconstruction (mm, 1e-2 mm absolute: the recon itself
    differs by <= 1e-4 normalised units per vertex)."""
    m = np.load(f"{recipe.HERE}/demo_meshes.npz")
    g = np.load(f"{recipe.HERE}/golden_eval.npz")
    eng = make_engine(dtopo, recipe.golden_weights())
    x = torch.from_numpy(recipe.normalized_meshes(8)).to(DEV)
    b = eng.set_batch(x)
    eng.forward(b, train=False)
    mean = torch.from_numpy(m["norm_mean"]).float().contiguous()
    std = torch.from_numpy(m["norm_std"]).float().contiguous()
    err, l1, mm = ops.vertex_errors(b.out.contiguous(), x, mean=mean.to(DEV), std=std.to(DEV),
                                    want_l1=True, want_mesh_mean=True)
    stats = ops.reconstruction_error_stats(mm)
    xr = torch.from_numpy(recipe.normalized_meshes(8))
    rec = torch.from_numpy(g["recon"])
    ref = O.vertex_errors(rec * std + mean, xr * std + mean)
    ref_mm = torch.mean(ref, dim=1)
    assert np.abs(err.cpu().numpy() - ref.numpy()).max() <= 1e-2
    assert abs(stats["mean"] - torch.mean(ref_mm).item()) <= 1e-3
    assert abs(stats["max"] - torch.max(ref_mm).item()) <= 1e-3
    assert abs(stats["median"] - torch.median(ref_mm).item()) <= 1e-3
    assert np.isfinite(stats["std"])
    # the same kernel's L1 term on normalised units against the golden recon
    _, l1n = ops.vertex_errors(b.out.contiguous(), rec.to(DEV), want_l1=True)
    assert l1n.max().item() <= 1e-4


def _golden_step(eng, dtopo, data, step):
    b = eng.inject(eng.buffers(16), recipe.train_key_index(step),
                   torch.from_numpy(recipe.train_eps(step)))
    b.batch_idx.copy_(torch.arange(4 * step, 4 * step + 4, dtype=torch.int32))
    ops.swap_features(data, b.batch_idx, dtopo.region_mask, b.key, 4, out=b.x)
    eng.train_step_on(b)
    torch.cuda.synchronize()


def test_checkpoint_resume_and_torch_adam_interop(dtopo, tmp_path):
    """f4: save_weights / resume (model_manager.py:682-706).  (1) A resumed
    engine continues bit-identically to the uninterrupted one.  (2) The saved
    optimizer.pt loads into torch.optim.Adam over the reference parameter order
    (model_manager.py:69-72) and its next step, given the device gradient,
    matches the device Adam (1e-6)."""
    w = recipe.golden_weights()
    data = torch.from_numpy(recipe.normalized_meshes(12)).to(DEV)
    a = make_engine(dtopo, w)
    for s in range(2):
        _golden_step(a, dtopo, data, s)
    name = a.save_weights(str(tmp_path), epoch=1)
    assert name.endswith("model_00000002.pt")
    b = make_engine(dtopo, w)
    b.params.data.zero_()
    assert b.resume(str(tmp_path)) == 2
    for buf in ("data", "exp_avg", "exp_avg_sq", "step"):
        assert torch.equal(getattr(a.params, buf), getattr(b.params, buf)), buf
    # torch Adam from the checkpoint, reference parameter order
    ck = torch.load(tmp_path / "model_00000002.pt", weights_only=True)["model"]
    ref = [ck[k].clone().requires_grad_() for k in ck]
    opt = torch.optim.Adam(ref, lr=1e-4, weight_decay=0.0, foreach=False)
    opt.load_state_dict(torch.load(tmp_path / "optimizer.pt", weights_only=True)["optimizer"])
    _golden_step(a, dtopo, data, 2)
    _golden_step(b, dtopo, data, 2)
    assert torch.equal(a.params.data, b.params.data)
    grads = a.grads()
    for p, k in zip(ref, ck):
        p.grad = grads[k].detach().cpu().clone()
    opt.step()
    sd = a.state_dict()
    for p, k in zip(ref, ck):
        close(sd[k], p.detach(), 1e-6, f"adam after resume {k}")


def test_encode_all_and_latent_stats_c1(dtopo):
    """f4: encode_all in ragged batches (3, 3, 2) of the C1 meshes vs the
    reference's golden mu (model_manager.py:244-246, 1e-4) and
    compute_latent_stats (test.py:95-117) vs the same statistics of the golden
    latents (1e-4)."""
    g = np.load(f"{recipe.HERE}/golden_eval.npz")
    eng = make_engine(dtopo, recipe.golden_weights())
    x = torch.from_numpy(recipe.normalized_meshes(8)).to(DEV)
    z = eng.encode_all(x, batch_size=3)
    torch.cuda.synchronize()
    assert tuple(z.shape) == (8, 75)
    assert np.abs(z.cpu().numpy() - g["mu"]).max() <= 1e-4
    st = eng.latent_stats(z)
    ref = torch.from_numpy(g["mu"])
    for k, v in {"means": ref.mean(0), "stds": ref.std(0), "mins": ref.min(0)[0],
                 "maxs": ref.max(0)[0]}.items():
        assert np.abs(st[k].cpu().numpy() - v.numpy()).max() <= 1e-4, k


@pytest.mark.parametrize("level,cout,bsz", [(1, 32, 2), (1, 32, 16), (2, 32, 16), (3, 64, 16), (3, 64, 3)])
@pytest.mark.parametrize("elu,deferred", [(False, False), (True, True)])
def test_rowsub_backward(otopo, dtopo, level, cout, bsz, elu, deferred):
    """Enblock backward on the kept rows (dG = dpre.W, then the ascending
    flat-list gather) vs autograd of conv -> row subset (model.py:34,40)."""
    g = torch.Generator().manual_seed(level * 10 + cout + bsz)
    sp = otopo.spirals[level]
    sel = torch.from_numpy(otopo.down[level][1])
    v = sp.shape[0]
    x = torch.randn(bsz, v, 32, generator=g).requires_grad_()
    w = (torch.randn(cout, 288, generator=g) * 0.1).requires_grad_()
    b = (torch.randn(cout, generator=g) * 0.1).requires_grad_()
    y = O.spiral_conv(x, sp, w, b)[:, sel]
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    ey = O.elu(torch.randn(bsz, v, 32, generator=g))
    ref_dx = x.grad * torch.where(ey > 0, torch.ones_like(ey), ey + 1) if elu else x.grad
    rows = sel.numel()
    need = ops.spiral_conv_bwd_rowsub_workspace(bsz, v, rows, 9, 32, cout)
    assert need > 0 and dtopo.enc_flat[level] is not None
    ws = torch.empty(need // 4 + 1, device=DEV)
    dx = torch.full((bsz, v, 32), float("nan"), device=DEV)
    dw = torch.empty(cout, 288, device=DEV)
    db = torch.empty(cout, device=DEV)
    args = (x.detach().to(DEV), dtopo.enc_rows[level], dy.to(DEV), dtopo.enc_flat[level], w.detach().to(DEV))
    if deferred:
        _, d = ops.spiral_conv_bwd_rowsub(*args, None, None, dx, elu_y=ey.to(DEV) if elu else None,
                                          workspace=ws)
        ops.dw_reduce_batch([(d, dw, db)])
    else:
        ops.spiral_conv_bwd_rowsub(*args, dw, db, dx, elu_y=ey.to(DEV) if elu else None, workspace=ws)
    close(dx, ref_dx, 1e-5, f"rowsub dx L{level}")
    close(dw, w.grad, 1e-5, f"rowsub dw L{level}")
    close(db, b.grad, 1e-5, f"rowsub db L{level}")
    # run-to-run bit-identical (fixed summation order, no atomics)
    dx2 = torch.empty_like(dx)
    ops.spiral_conv_bwd_rowsub(*args, dw, db, dx2, elu_y=ey.to(DEV) if elu else None, workspace=ws)
    assert torch.equal(dx, dx2)



@pytest.mark.parametrize("level,cout", [(1, 32), (2, 32), (3, 64)])
@pytest.mark.parametrize("deferred", [False, True])
def test_rowsub_backward_vertex_major(otopo, dtopo, level, cout, deferred):
    """Row-subset backward with vertex-major x / dx / elu_y (the fp32 step's
    E1 layout; batch-major dpre): dx by the flat-list MFMA kernel straight from
    dpre, dW slabs by the lat body -- vs autograd of conv -> row subset."""
    bsz = 16
    g = torch.Generator().manual_seed(level * 100 + cout)
    sp = otopo.spirals[level]
    sel = torch.from_numpy(otopo.down[level][1])
    v = sp.shape[0]
    x = torch.randn(bsz, v, 32, generator=g).requires_grad_()
    w = (torch.randn(cout, 288, generator=g) * 0.1).requires_grad_()
    b = (torch.randn(cout, generator=g) * 0.1).requires_grad_()
    y = O.spiral_conv(x, sp, w, b)[:, sel]
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    ey = O.elu(torch.randn(bsz, v, 32, generator=g))
    ref_dx = x.grad * torch.where(ey > 0, torch.ones_like(ey), ey + 1)
    rows = sel.numel()
    ws = torch.empty(ops.spiral_conv_bwd_rowsub_workspace(bsz, v, rows, 9, 32, cout) // 4 + 1, device=DEV)
    xv = ops.to_vm(x.detach().to(DEV))
    eyv = ops.to_vm(ey.to(DEV))
    dx = ops.vm_empty(bsz, v, 32, device=DEV)
    dw = torch.empty(cout, 288, device=DEV)
    db = torch.empty(cout, device=DEV)
    args = (xv, dtopo.enc_rows[level], dy.to(DEV), dtopo.enc_flat[level], w.detach().to(DEV))
    if deferred:
        _, d = ops.spiral_conv_bwd_rowsub(*args, None, None, dx, elu_y=eyv, workspace=ws)
        ops.dw_reduce_batch([(d, dw, db)])
    else:
        ops.spiral_conv_bwd_rowsub(*args, dw, db, dx, elu_y=eyv, workspace=ws)
    assert ops.is_vm(dx)
    close(dx, ref_dx, 1e-5, f"rowsub vm dx L{level}")
    close(dw, w.grad, 1e-5, f"rowsub vm dw L{level}")
    close(db, b.grad, 1e-5, f"rowsub vm db L{level}")
    dx2 = ops.vm_empty(bsz, v, 32, device=DEV)
    ops.spiral_conv_bwd_rowsub(*args, dw, db, dx2, elu_y=eyv, workspace=ws)
    assert torch.equal(dx, dx2)


@pytest.mark.parametrize("level,cout", [(1, 32), (2, 32), (3, 64)])
def test_rowsub_data_bf16_storage(dtopo, level, cout):
    """dx-only row-subset backward: bf16 storage = one rounding of the fp32
    result (the same fp32 sums: flat-list MFMA at 32 -> 32, dG + gather at
    32 -> 64), so it equals the fp32 call cast."""
    bsz = 16
    g = torch.Generator().manual_seed(level + cout)
    v, rows = dtopo.n_verts[level], dtopo.n_verts[level + 1]
    dpre = torch.randn(bsz, rows, cout, generator=g).to(DEV)
    w = (torch.randn(cout, 288, generator=g) * 0.1).to(DEV)
    ey16 = O.elu(torch.randn(bsz, v, 32, generator=g)).to(DEV, torch.bfloat16)
    d32 = torch.empty(bsz, v, 32, device=DEV)
    d16 = torch.empty(bsz, v, 32, device=DEV, dtype=torch.bfloat16)
    ops.spiral_conv_bwd_data_rowsub(dpre, dtopo.enc_flat[level], w, v, elu_y=ey16.float(), out=d32)
    ops.spiral_conv_bwd_data_rowsub(dpre, dtopo.enc_flat[level], w, v, elu_y=ey16, out=d16)
    assert torch.equal(d16, d32.to(torch.bfloat16))
    # vertex-major dx / elu_y (the bf16 step's E1 layout): the same values
    dvm = ops.vm_empty(bsz, v, 32, dtype=torch.bfloat16, device=DEV)
    ops.spiral_conv_bwd_data_rowsub(dpre, dtopo.enc_flat[level], w, v, elu_y=ops.to_vm(ey16), out=dvm)
    assert ops.is_vm(dvm) and torch.equal(dvm, d16)
    # and the fp32 dx equals the fused rowsub backward's dx (at batch 16 that
    # one multiplies each list entry into one MFMA accumulator: fp32 rounding)
    x = torch.randn(bsz, v, 32, generator=g).to(DEV)
    dxf = torch.empty_like(d32)
    ops.spiral_conv_bwd_rowsub(x, dtopo.enc_rows[level], dpre, dtopo.enc_flat[level], w, None, None, dxf,
                               elu_y=ey16.float())
    close(dxf, d32, 1e-5, "fused rowsub dx vs dG + gather")


@pytest.mark.parametrize("i,bsz", [(0, 16), (0, 3), (1, 4)])
def test_deblock_fused_up_matches_spmm_then_conv(dtopo, i, bsz):
    """cfsd_spiral_conv_fwd_up (coarse Deblock: Pool(up) inside the conv
    gather, model.py:80-82) == cfsd_spmm_uniform then the conv: the
    up-sampled input bit for bit, the ELU output within 1e-5 (same slot
    partials, possibly another slot grouping)."""
    eng = make_engine(dtopo, recipe.golden_weights(), bs=4)
    cin, cout, lv, ui = eng.spec.dec_layers()[i]
    assert dtopo.up_comp[ui] is not None
    assert ops.spiral_conv_fwd_up_supported(bsz, dtopo.n_verts[lv], 9, cin, cout)
    # (the fused form covers the few-tile layers only: D1 at batch 16 = 1065 tiles is not fused)
    assert not ops.spiral_conv_fwd_up_supported(16, dtopo.n_verts[2], 9, 64, 32)
    g = torch.Generator(device=DEV).manual_seed(i + bsz)
    xc = torch.randn(bsz, dtopo.n_verts[lv + 1], cin, device=DEV, generator=g)
    w, bias = eng._dec_w(i)
    up = ops.spmm(dtopo.up_csr[ui], xc, dtopo.n_verts[lv], uniform=dtopo.up_uniform[ui])
    ref = ops.spiral_conv_fwd(up, dtopo.spiral[lv], w, bias, 1)
    y = torch.empty(bsz, dtopo.n_verts[lv], cout, device=DEV)
    yup = torch.full((bsz, dtopo.n_verts[lv], cin), float("nan"), device=DEV)
    ops.spiral_conv_fwd_up(xc, dtopo.up_comp[ui], dtopo.spiral[lv], w, bias, 1, out=y, up_out=yup)
    assert torch.equal(yup, up)
    close(y, ref, 1e-5, "fused Deblock forward")
    # and against the oracle (float64 of the same up-sampled input)
    sp = dtopo.spiral[lv].long().cpu()
    r64 = O.spiral_conv(up.double().cpu(), sp, w.double().cpu(), bias.double().cpu())
    close(y, torch.nn.functional.elu(r64), 1e-5, "fused Deblock forward vs float64")


def test_engine_forward_fused_up_equals_unfused(dtopo):
    """The step's forward with the fused coarse Deblocks equals the unfused
    forward (reconstruction within 1e-5, the decoder's up-sampled inputs
    bit-identical)."""
    outs = []
    x = torch.from_numpy(recipe.normalized_meshes(8)).to(DEV)
    for fuse in (True, False):
        eng = make_engine(dtopo, recipe.golden_weights())
        eng.fuse_up = fuse
        b = eng.set_batch(x)
        eng.forward(b, train=False)
        torch.cuda.synchronize()
        outs.append((b.out.clone(), [u.clone() for u in b.dec_up[:2]]))
    close(outs[0][0], outs[1][0], 1e-5, "reconstruction")
    for a, c in zip(outs[0][1], outs[1][1]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("bs,vae,train,n", [(4, True, True, 4288), (3, True, True, 300), (9, True, True, 4288),
                                            (4, True, False, 4288), (4, False, True, 1000)])
def test_latent_linear_fused_equals_two_launches(bs, vae, train, n):
    """cfsd_latent_linear_fwd (latent head + decoder Linear in one launch):
    z, dlat and the Linear output bit-identical to cfsd_latent_fwd followed by
    cfsd_linear_fwd, terms included."""
    g = torch.Generator().manual_seed(bs * 7 + n)
    L, B = 75, bs * bs
    mulv = torch.randn(B, (2 if vae else 1) * L, generator=g).to(DEV) * 0.5
    eps = torch.randn(B, L, generator=g).to(DEV)
    w = torch.randn(n, L, generator=g).to(DEV) * 0.1
    bias = torch.randn(n, generator=g).to(DEV)
    keyt = torch.full((1,), 2, dtype=torch.int32, device=DEV)
    res = []
    for fused in (True, False):
        zz, dlat = torch.full((B, L), 7.0, device=DEV), torch.full((B, 3 * L), 7.0, device=DEV)
        terms, h = torch.full((2,), 7.0, device=DEV), torch.full((B, n), 7.0, device=DEV)
        args = (mulv, eps if (vae and train) else None, keyt, zz, dlat, terms, L, 5, train, vae, False,
                1e-4, 0.5, 0.5, 0.5)
        if fused:
            assert ops.latent_linear_fwd_supported(B, L, n)
            ops.latent_linear_fwd(*args, w, bias, out=h)
        else:
            ops.latent_fwd(*args)
            ops.linear_fwd(zz, w, bias, out=h, workspace=None)
        torch.cuda.synchronize()
        res.append((zz, dlat, terms, h))
    for name, a, c in zip(("z", "dlat", "terms", "h"), res[0], res[1]):
        assert torch.equal(a, c), name


def test_engine_forward_fused_latent_equals_unfused(dtopo):
    """The step's forward with the latent head and decoder Linear in one launch
    equals the two-launch forward bit for bit (z, decoder input, output)."""
    outs = []
    x = torch.from_numpy(recipe.normalized_meshes(12)).to(DEV)
    x = torch.cat([x, x[:4]])  # 16 = bs^2: latent consistency on
    for fuse in (True, False):
        eng = make_engine(dtopo, recipe.golden_weights())
        eng.fuse_latent = fuse
        assert eng._lc_on(eng.buffers(16))
        eps = torch.randn(16, eng.spec.latent, generator=torch.Generator().manual_seed(5)).to(DEV)
        b = eng.set_batch(x, key_index=3, eps=eps)
        eng.forward(b, train=True)
        torch.cuda.synchronize()
        outs.append((b.z.clone(), b.h.clone(), b.out.clone(), b.dlat.clone(), b.terms.clone()))
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)


def test_trainstep_multi_step_graph_matches_eager(dtopo):
    """TrainStep.run(k) on a captured single-GPU runner replays the
    steps_per_graph-step graph k // steps_per_graph times (+ the one-step
    graph): the parameters, moments and losses of k eager steps, bit for bit
    (epoch boundaries inside the multi-step graph included: 3 batches per
    epoch)."""
    from craniofacialsd_vae_amd import step as ST
    res = []
    for captured in (False, True):
        data = E.ResidentData(torch.from_numpy(recipe.normalized_meshes(12)).to(DEV), bs=4,
                              rows=list(range(12)), shuffle=True)
        eng = make_engine(dtopo, recipe.golden_weights())
        ts = ST.TrainStep(eng, data)
        n = ts.steps_per_graph
        if captured:
            ts.capture()  # (runs one real step eagerly first)
            ts.run(2 * n + 3)
        else:
            ts.run(2 * n + 4)
        torch.cuda.synchronize()
        P = eng.params
        res.append([t.clone() for t in (P.data, P.exp_avg, P.exp_avg_sq, eng.loss_acc)])
    for a, c in zip(*res):
        assert torch.equal(a, c)
