"""bf16 path (BASELINE.json configs C3/C5): every bf16 kernel against the
oracle run in float64 on the SAME bf16-rounded inputs, then the full bf16
train step against the fp32 reference goldens.

Tolerances (stated per test): a product of two bf16 values is exact in fp32
and every sum is fp32, so fp32 outputs carry only fp32 summation error
(rel 1e-5 of the largest magnitude); bf16 outputs add one rounding (half a
bf16 ulp = 2^-9 relative); the dx kernel also rounds the inverse-spiral
gather-sum A to bf16 once before the MFMA (1e-2 of the largest magnitude).
The Pool SpMM sums fp32 products in file order exactly like the oracle, so
its bf16 output is bit-exact to the oracle's fp32 result rounded to bf16.
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
BF = torch.bfloat16
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


def rb(t):
    """bf16-rounded copy (as float64 for the reference)."""
    return t.to(BF).double()


def err_rel_max(got, ref):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return float((got - ref).abs().max() / (ref.abs().max() + 1e-30))


def lay(ops, t, vm):
    """The operand in the requested layout: batch-major (contiguous) or
    vertex-major (CFSD_VM, ``ops.to_vm``) -- same logical values."""
    return ops.to_vm(t) if vm else t.contiguous()


def empty(ops, shape, dtype, vm):
    return ops.vm_empty(*shape, dtype=dtype, device=DEV) if vm else torch.empty(shape, dtype=dtype, device=DEV)


def gather(x, sp):
    idx = torch.as_tensor(sp, dtype=torch.long)
    return torch.index_select(x, 1, idx.reshape(-1)).view(x.shape[0], idx.shape[0], -1)


# (cin, cout, level, batch) of the 32/64-channel bf16 MFMA kernels
MFMA_CASES = [(32, 32, 0, 2), (32, 32, 1, 16), (32, 32, 3, 3), (32, 64, 2, 3), (64, 32, 2, 3),
              (64, 64, 3, 2), (32, 32, 0, 16), (32, 64, 3, 32), (32, 32, 2, 48)]


# layouts of (x, y): batch-major / vertex-major / mixed (E1 reads a
# vertex-major level-1 tensor and writes a batch-major level-2 one)
LAYOUTS = [(False, False), (True, True), (True, False), (False, True)]


@pytest.mark.parametrize("cin,cout,level,bsz", MFMA_CASES)
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("out_bf16", [True, False])
@pytest.mark.parametrize("xvm,yvm", LAYOUTS)
def test_conv_fwd_bf16(mods, otopo, dtopo, cin, cout, level, bsz, act, out_bf16, xvm, yvm):
    """Also: every layout gives the bit-identical result (same per-output
    MFMA K order; only the addressing differs)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(cin + cout + level + act)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    x = torch.randn(bsz, v, cin, generator=g)
    w = torch.randn(cout, 9 * cin, generator=g) * 0.1
    b = torch.randn(cout, generator=g) * 0.1
    ref = gather(rb(x), sp) @ rb(w).T + b.double()
    if act:
        ref = torch.nn.functional.elu(ref)
    odt = BF if out_bf16 else torch.float32
    out = empty(ops, (bsz, v, cout), odt, yvm)
    assert ops.is_vm(out) == (yvm and bsz > 1)
    args = (dtopo.spiral[level], w.to(DEV), w.to(BF).to(DEV), b.to(DEV), act)
    ops.spiral_conv_fwd_x(lay(ops, x.to(BF).to(DEV), xvm), *args, out)
    tol = 2.0 ** -8 if out_bf16 else 1e-5
    assert err_rel_max(out.float(), ref) <= tol
    if xvm or yvm:  # layouts agree (the vertex-major batch-16 kernel: to one bf16 rounding)
        base = torch.empty(bsz, v, cout, dtype=odt, device=DEV)
        ops.spiral_conv_fwd_x(x.to(BF).to(DEV), *args, base)
        if xvm and bsz % 16 == 0:
            assert err_rel_max(out.float(), base.float()) <= (2.0 ** -8 if out_bf16 else 1e-6)
        else:
            assert torch.equal(out, base)


@pytest.mark.parametrize("table,cin,cout,level,bsz", [("dec", 32, 32, 0, 2), ("dec", 32, 32, 1, 16),
                                                      ("enc", 32, 32, 1, 16), ("dec", 64, 32, 2, 3),
                                                      ("dec", 32, 64, 3, 3), ("dec", 64, 64, 2, 2),
                                                      ("dec", 32, 32, 0, 16), ("dec", 32, 64, 2, 32)])
@pytest.mark.parametrize("dpre_f32", [False, True])
@pytest.mark.parametrize("xvm,dpvm", [(False, False), (True, True), (True, False)])
def test_conv_bwd_bf16(mods, otopo, dtopo, table, cin, cout, level, bsz, dpre_f32, xvm, dpvm):
    """dx (bf16, with elu') and dW/db (fp32) of the bf16 MFMA kernels, on the
    full spiral table and on the Enblock row subset (E1's shape), with x /
    dx / elu_y and dpre in either layout (dx bit-identical across layouts)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(5 + cin + cout + level)
    sp = otopo.spirals[level]
    if table == "enc":
        sp = sp[np.asarray(otopo.down[level][1])[np.argsort(otopo.down[level][0])]]
        idx, inv = dtopo.enc_rows[level], dtopo.enc_inv[level]
    else:
        idx, inv = dtopo.spiral[level], dtopo.spiral_inv[level]
    vsrc, rows = otopo.spirals[level].shape[0], sp.shape[0]
    y = torch.nn.functional.elu(torch.randn(bsz, vsrc, cin, generator=g))  # the conv input (an ELU output)
    w = torch.randn(cout, 9 * cin, generator=g) * 0.1
    dpre = torch.randn(bsz, rows, cout, generator=g)
    yb, wb = rb(y), rb(w)
    # dx sums fp32 dpre rows in fp32 before rounding the sum; dW rounds every
    # dpre value to bf16 as its MFMA operand -> two references
    dpb = dpre.double() if dpre_f32 else rb(dpre)
    xl = yb.clone().requires_grad_()
    (gather(xl, sp) @ wb.T).backward(dpb)
    dx_ref = xl.grad * torch.where(yb > 0, 1.0, yb + 1.0)
    wl = wb.clone().requires_grad_()
    bl = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    (gather(yb, sp) @ wl.T + bl).backward(rb(dpre))
    dpre_dev = lay(ops, (dpre if dpre_f32 else dpre.to(BF)).to(DEV), dpvm)
    y_dev = lay(ops, y.to(BF).to(DEV), xvm)
    dx = empty(ops, (bsz, vsrc, cin), BF, xvm)
    ops.spiral_conv_bwd_data_x(dpre_dev, inv, w.to(BF).to(DEV), vsrc, elu_y=y_dev, out=dx)
    assert err_rel_max(dx.float(), dx_ref) <= 1e-2
    if xvm or dpvm:
        base = ops.spiral_conv_bwd_data_x(dpre_dev.contiguous(), inv, w.to(BF).to(DEV), vsrc,
                                          elu_y=y_dev.contiguous())
        if xvm and dpvm and bsz % 16 == 0:  # vertex-major batch-16 kernel: one bf16 rounding
            assert err_rel_max(dx.float(), base.float()) <= 2.0 ** -8
        else:
            assert torch.equal(dx, base)
    dw = torch.empty(cout, 9 * cin, device=DEV)
    db = torch.empty(cout, device=DEV)
    ws = torch.empty(ops.spiral_conv_bwd_weight_x_workspace(bsz, rows, 9, cin, cout) // 4 + 1, device=DEV)
    ops.spiral_conv_bwd_weight_x(y_dev, idx, dpre_dev, dw, db, ws)
    assert err_rel_max(dw, wl.grad) <= 1e-4
    assert err_rel_max(db, bl.grad) <= 1e-4
    # deferred slabs through the batched reduce: identical
    ws.zero_()
    d = ops.spiral_conv_bwd_weight_x(y_dev, idx, dpre_dev, None, None, ws)
    dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
    ops.dw_reduce_batch([(d, dw2, db2)])
    assert torch.equal(dw2, dw) and torch.equal(db2, db)


@pytest.mark.parametrize("level,bsz,cout", [(0, 16, 32), (1, 16, 32), (1, 32, 64), (2, 16, 32), (3, 48, 32)])
@pytest.mark.parametrize("dpre_f32", [False, True])
@pytest.mark.parametrize("with_elu", [False, True])
def test_conv_dx_flat_bf16(mods, otopo, dtopo, level, bsz, cout, dpre_f32, with_elu):
    """Flat-list data gradient (vertex-major, batch % 16): exact bf16 products
    summed in fp32 over the ascending flat list (model.py:34's index_add_
    order), so it matches the float64 oracle on the same bf16 operands to fp32
    summation error plus the output's bf16 rounding (2^-8 of the largest)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(level * 7 + bsz + cout)
    sp = otopo.spirals[level]
    v = sp.shape[0]
    assert dtopo.spiral_flat[level] is not None
    y = torch.nn.functional.elu(torch.randn(bsz, v, 32, generator=g))
    w = torch.randn(cout, 288, generator=g) * 0.1
    dpre = torch.randn(bsz, v, cout, generator=g)
    dpb = rb(dpre)  # each row is an MFMA operand: bf16-rounded, fp32 or bf16 storage alike
    xl = rb(y).requires_grad_()
    (gather(xl, sp) @ rb(w).T).backward(dpb)
    ref = xl.grad * (torch.where(rb(y) > 0, 1.0, rb(y) + 1.0) if with_elu else 1.0)
    dp = ops.to_vm((dpre if dpre_f32 else dpre.to(BF)).to(DEV))
    ey = ops.to_vm(y.to(BF).to(DEV)) if with_elu else None
    dx = ops.spiral_conv_bwd_data_flat(dp, dtopo.spiral_flat[level], w.to(BF).to(DEV), v, elu_y=ey)
    assert ops.is_vm(dx)
    assert err_rel_max(dx.float(), ref) <= 2.0 ** -8
    # deterministic: a second launch is bit-identical
    dx2 = ops.spiral_conv_bwd_data_flat(dp, dtopo.spiral_flat[level], w.to(BF).to(DEV), v, elu_y=ey)
    assert torch.equal(dx, dx2)


@pytest.mark.parametrize("level,kind,x_bf16,y_bf16", [(0, "up", True, True), (1, "up", False, True),
                                                       (0, "upT", True, True), (1, "upT", True, False),
                                                       (2, "down", True, True)])
@pytest.mark.parametrize("with_elu", [False, True])
@pytest.mark.parametrize("xvm,yvm", LAYOUTS)
def test_spmm_bf16_bit_exact(mods, otopo, dtopo, level, kind, x_bf16, y_bf16, with_elu, xvm, yvm):
    """Bit-exact in every layout and in each of the step's SpMM forms (CSR,
    uniform-row, visiting-order CSR)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(level * 3 + len(kind))
    coo = otopo.up[level] if kind != "down" else otopo.down[level]
    m, n = coo[3]
    if kind == "upT":
        row, col, val, _ = coo
        coo, (m, n) = (col, row, val, (n, m)), (n, m)
        csr = dtopo.upT_csr[level]
    else:
        csr = dtopo.up_csr[level] if kind == "up" else dtopo.down_csr[level]
    x = torch.randn(4, n, 32, generator=g)
    if x_bf16:
        x = x.to(BF).float()
    ref = O.pool(x, coo)
    ey = torch.nn.functional.elu(torch.randn(4, m, 32, generator=g))
    if with_elu:
        eyq = ey.to(BF).float() if y_bf16 else ey
        ref = ref * torch.where(eyq > 0, torch.ones_like(eyq), eyq + 1.0)
    ydt = BF if y_bf16 else torch.float32
    xd = lay(ops, (x.to(BF) if x_bf16 else x).to(DEV), xvm)
    eyd = lay(ops, (ey.to(BF) if y_bf16 else ey).to(DEV), yvm) if with_elu else None
    exp = ref.to(BF) if y_bf16 else ref
    forms = [{}]
    if kind == "up":
        forms.append({"uniform": dtopo.up_uniform[level]})
    if kind == "upT":
        forms.append({"sched": dtopo.upT_sched[level]})
    for f in forms:
        if not all(f.values()):
            continue
        out = empty(ops, (4, m, 32), ydt, yvm)
        ops.spmm_x(csr, xd, m, elu_y=eyd, out=out, **f)
        assert torch.equal(out.cpu(), exp), f


@pytest.mark.parametrize("bsz", [2, 16])
@pytest.mark.parametrize("vm", [False, True])
def test_xyz_layers_bf16(mods, otopo, dtopo, bsz, vm):
    """The xyz layers of the bf16 step: input conv (fp32 x -> bf16 y) and
    its dW with bf16 dpre; output conv (bf16 x -> fp32 y) and its fused
    dx (bf16) + dW.  ``vm``: the 32-channel operands vertex-major (the
    step's layout), the xyz tensors batch-major."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(bsz)
    sp0 = otopo.spirals[0]
    sel = np.asarray(otopo.down[0][1])[np.argsort(otopo.down[0][0])]
    x = torch.randn(bsz, sp0.shape[0], 3, generator=g)
    w0 = torch.randn(32, 27, generator=g) * 0.1
    b0 = torch.randn(32, generator=g) * 0.1
    ref = torch.nn.functional.elu(gather(x.double(), sp0[sel]) @ w0.double().T + b0.double())
    y = empty(ops, (bsz, len(sel), 32), BF, vm)
    ops.spiral_conv_fwd_x(x.to(DEV), dtopo.enc_rows[0], w0.to(DEV), None, b0.to(DEV), 1, y)
    assert err_rel_max(y.float(), ref) <= 2.0 ** -8
    dpre = torch.randn(bsz, len(sel), 32, generator=g)
    dw, db = torch.empty(32, 27, device=DEV), torch.empty(32, device=DEV)
    ws = torch.empty(ops.spiral_conv_bwd_weight_x_workspace(bsz, len(sel), 9, 3, 32) // 4 + 1, device=DEV)
    ops.spiral_conv_bwd_weight_x(x.to(DEV), dtopo.enc_rows[0], lay(ops, dpre.to(BF).to(DEV), vm), dw, db, ws)
    gx = gather(x.double(), sp0[sel])
    assert err_rel_max(dw, torch.einsum("bro,brk->ok", rb(dpre), gx)) <= 1e-5
    assert err_rel_max(db, rb(dpre).sum((0, 1))) <= 1e-5
    # output conv
    h = torch.nn.functional.elu(torch.randn(bsz, sp0.shape[0], 32, generator=g))
    w5 = torch.randn(3, 288, generator=g) * 0.1
    b5 = torch.randn(3, generator=g) * 0.1
    out = torch.empty(bsz, sp0.shape[0], 3, device=DEV)
    hd = lay(ops, h.to(BF).to(DEV), vm)
    ops.spiral_conv_fwd_x(hd, dtopo.spiral[0], w5.to(DEV), None, b5.to(DEV), 0, out)
    hl = rb(h).requires_grad_()
    wl = w5.double().requires_grad_()
    bl = b5.double().requires_grad_()
    ref = gather(hl, sp0) @ wl.T + bl
    assert err_rel_max(out, ref) <= 1e-5
    dout = torch.randn(ref.shape, generator=g)
    ref.backward(dout.double())
    dx_ref = hl.grad * torch.where(rb(h) > 0, 1.0, rb(h) + 1.0)
    dx = empty(ops, (bsz, sp0.shape[0], 32), BF, vm)
    dw, db = torch.empty(3, 288, device=DEV), torch.empty(3, device=DEV)
    ops.spiral_conv_bwd_x(hd, dtopo.spiral[0], dout.to(DEV), dtopo.spiral_inv[0], w5.to(DEV), dw, db,
                          dx=dx, elu_y=hd)
    assert err_rel_max(dx.float(), dx_ref) <= 2.0 ** -8
    assert err_rel_max(dw, wl.grad) <= 1e-5
    assert err_rel_max(db, bl.grad) <= 1e-5


def test_adam_writes_bf16_shadow(mods):
    _, ops, _ = mods
    n = 1000003
    g = torch.Generator().manual_seed(1)
    p, gr = torch.randn(n, generator=g).to(DEV), torch.randn(n, generator=g).to(DEV)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    step = torch.ones(1, dtype=torch.int32, device=DEV)
    sh = torch.empty(n, dtype=BF, device=DEV)
    ops.adam(p, gr, m, v, step, 1e-3, shadow=sh)
    assert torch.equal(sh, p.to(BF))
    back = torch.empty(n, device=DEV)
    ops.cast(sh, back)
    assert torch.equal(back, sh.float())


# bf16 step vs (a) the oracle emulating the bf16 storage points (levels 0/1
# rounded to bf16, bf16 weights on the MFMA layers), layer by layer with the
# engine's own input fed to each decoder layer: mean abs error <= 1e-6 and
# max <= one bf16 ulp of the layer's largest value (only rare rounding-tie
# flips from the fp32 summation order differ) -- the bf16 pipeline itself;
# end to end the flips propagate (mean per-vertex L1 <= 5e-3; measured 1.4e-3);
# and (b) the fp32 reference goldens (tests/golden/golden_train.npz): losses
# rel 2e-2, mean per-vertex L1 <= 2e-2, every gradient cosine >= 0.99 --
# what the bf16 precision costs.
def test_bf16_layers_vs_bf16_emulating_oracle(mods, otopo, dtopo):
    E, _, _ = mods
    w = recipe.golden_weights()
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV, precision="bf16")
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    P = O.make_params(w)
    key, eps = recipe.train_key_index(0), torch.from_numpy(recipe.train_eps(0))
    x16 = torch.from_numpy(O.swap_features(recipe.normalized_meshes(4), otopo.region_features, key))
    b = eng.set_batch(x16.to(DEV), key_index=key, eps=eps.to(DEV))
    eng.forward(b, train=True)
    torch.cuda.synchronize()

    def check(got, ref, what):
        d = (got.float().cpu() - ref).abs()
        ulp = 2.0 ** (np.floor(np.log2(float(ref.abs().max()))) - 7)
        assert float(d.mean()) <= 1e-6 and float(d.max()) <= ulp, f"{what}: mean {float(d.mean())} max {float(d.max())}"

    with torch.no_grad():
        h = x16
        for i in range(4):  # encoder, each layer from the engine's input
            low = i in (0, 1) and h.shape[-1] >= 16
            r = O.pool(O.elu(O.spiral_conv(h, otopo.spirals[i], O._w(P, f"en_layers.{i}.conv.layer.weight", low),
                                           P[f"en_layers.{i}.conv.layer.bias"])), otopo.down[i])
            r = O._q(r) if i + 1 in (0, 1) else r
            check(b.enc_out[i], r, f"enc_out[{i}]")
            h = b.enc_out[i].float().cpu()
        hh = b.h.cpu()
        for i in range(1, 5):
            lv = 4 - i
            hu = O.pool(hh, otopo.up[lv])
            hu = O._q(hu) if lv in (0, 1) else hu
            check(b.dec_up[i - 1], hu, f"dec_up[{i - 1}]")
            r = O.elu(O.spiral_conv(b.dec_up[i - 1].float().cpu(), otopo.spirals[lv],
                                    O._w(P, f"de_layers.{i}.conv.layer.weight", lv in (0, 1)),
                                    P[f"de_layers.{i}.conv.layer.bias"]))
            check(b.dec_out[i - 1], O._q(r) if lv in (0, 1) else r, f"dec_out[{i - 1}]")
            hh = b.dec_out[i - 1].float().cpu()
        out = O.spiral_conv(hh, otopo.spirals[0], P["de_layers.5.layer.weight"], P["de_layers.5.layer.bias"])
        check(b.out, out, "out")
        emu = O.losses(P, x16, otopo, key, eps, lp={0, 1})
    l1 = (b.out.cpu() - emu["out"]).abs().sum(-1)
    assert float(l1.mean()) <= 5e-3, f"end to end mean per-vertex L1 {float(l1.mean())}"


def test_bf16_train_three_steps_vs_fp32_golden(mods, otopo, dtopo):
    E, ops, _ = mods
    g = np.load(f"{recipe.HERE}/golden_train.npz")
    w = recipe.golden_weights()
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV, precision="bf16")
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    P = O.make_params(w)
    opt = O.Adam(P)
    meshes = recipe.normalized_meshes(12)
    data = torch.from_numpy(meshes).to(DEV)
    report = []
    for step in range(3):
        key = recipe.train_key_index(step)
        eps = torch.from_numpy(recipe.train_eps(step))
        out, grads, _ = O.train_step(P, opt, meshes[4 * step:4 * step + 4], otopo, key, eps.numpy())
        b = eng.inject(eng.buffers(16), key, eps)
        b.batch_idx.copy_(torch.arange(4 * step, 4 * step + 4, dtype=torch.int32))
        ops.swap_features(data, b.batch_idx, dtopo.region_mask, b.key, 4, out=b.x)
        eng.train_step_on(b)
        torch.cuda.synchronize()
        got = b.losses.cpu().numpy()
        rel = np.abs(got - g[f"s{step}_losses"]) / np.abs(g[f"s{step}_losses"])
        l1 = np.abs(b.out.cpu().numpy() - out["out"].detach().numpy()).sum(-1)
        cos = {}
        for name, gd in eng.grads().items():
            a, r = gd.detach().cpu().double().ravel(), grads[name].double().ravel()
            cos[name] = float(a @ r / (a.norm() * r.norm() + 1e-30))
        report.append((step, float(rel.max()), float(l1.mean()), float(l1.max()), min(cos.values())))
        assert rel.max() <= 2e-2, f"step {step} loss rel {rel}"
        assert l1.mean() <= 2e-2, f"step {step} mean per-vertex L1 {l1.mean()}"
        assert min(cos.values()) >= 0.99, f"step {step} grad cosine {sorted(cos.items(), key=lambda kv: kv[1])[:3]}"
    print("bf16 vs fp32 golden (step, loss rel, mean / max per-vertex L1, min grad cosine):", report)


def test_bf16_graph_step_runs(mods, dtopo):
    """The resident bf16 step captures into a hipGraph and replays with
    identical results to eager launches."""
    E, _, _ = mods
    w = recipe.golden_weights()
    res = []
    for use_graph in (False, True):
        data = E.ResidentData(torch.from_numpy(recipe.normalized_meshes(12)).to(DEV), bs=4, shuffle=True)
        eng = E.SDVAEEngine(dtopo, E.ModelSpec(), device=DEV, precision="bf16")
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
        res.append((eng.params.data.cpu().clone(), b.losses.cpu().clone(), eng.params.shadow.cpu().clone()))
        assert torch.isfinite(res[-1][1]).all()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("level", [0, 1])
@pytest.mark.parametrize("with_elu", [False, True])
def test_bwd_flat_pair_bf16(mods, dtopo, level, with_elu):
    """cfsd_spiral_conv_bwd_flat_pair_bf16 (ABI 4.11: the bf16 flat-list dx
    and the conv_dw_vm16 slabs as two workgroup roles of one launch) == the
    deferred cfsd_spiral_conv_bwd_weight_x + cfsd_spiral_conv_bwd_data_flat
    on the same bf16 operands, bit for bit (dx, and dW / db through the
    batched reduce)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(31 + level + with_elu)
    bsz, v = 16, dtopo.n_verts[level]
    idx = dtopo.spiral[level]
    x = ops.to_vm(torch.randn(bsz, v, 32, generator=g).to(DEV).bfloat16())
    dpre = ops.to_vm(torch.randn(bsz, v, 32, generator=g).to(DEV).bfloat16())
    ey = ops.to_vm(torch.nn.functional.elu(torch.randn(bsz, v, 32, generator=g)).to(DEV).bfloat16()) if with_elu else None
    w16 = (torch.randn(32, 288, generator=g) * 0.1).to(DEV).bfloat16()
    flat = dtopo.spiral_flat[level]
    nb = ops.spiral_conv_bwd_weight_x_workspace(bsz, v, 9, 32, 32)
    ws_a = torch.zeros(nb // 4 + 64, device=DEV)
    ws_b = torch.zeros_like(ws_a)
    dx_a = ops.vm_empty(bsz, v, 32, dtype=torch.bfloat16, device=DEV)
    d_a = ops.spiral_conv_bwd_flat_pair_bf16(x, idx, dpre, flat, w16, dx_a, elu_y=ey, workspace=ws_a)
    dx_b = ops.spiral_conv_bwd_data_flat(dpre, flat, w16, v, elu_y=ey)
    d_b = ops.spiral_conv_bwd_weight_x(x, idx, dpre, None, None, ws_b)
    dw_a, db_a = torch.empty(32, 288, device=DEV), torch.empty(32, device=DEV)
    dw_b, db_b = torch.empty_like(dw_a), torch.empty_like(db_a)
    ops.dw_reduce_batch([(d_a, dw_a, db_a), (d_b, dw_b, db_b)])
    assert torch.equal(dx_a, dx_b)
    assert torch.equal(dw_a, dw_b) and torch.equal(db_a, db_b)


@pytest.mark.parametrize("with_elu", [False, True])
def test_bwd_rowsub_pair_bf16(mods, dtopo, with_elu):
    """cfsd_spiral_conv_bwd_rowsub_pair_bf16 (ABI 4.11: the bf16 step's E1
    backward -- fp32-product flat dx from fp32 batch-major dpre at the kept
    rows, and the conv_dw_vm16<float> slabs -- in one launch) == the deferred
    cfsd_spiral_conv_bwd_weight_x + cfsd_spiral_conv_bwd_data_rowsub, bit for
    bit (dx, and dW / db through the batched reduce)."""
    _, ops, _ = mods
    g = torch.Generator().manual_seed(41 + with_elu)
    bsz, lv = 16, 1
    v, rows_tab, flat = dtopo.n_verts[lv], dtopo.enc_rows[lv], dtopo.enc_flat[lv]
    rows = rows_tab.shape[0]
    x = ops.to_vm(torch.randn(bsz, v, 32, generator=g).to(DEV).bfloat16())
    dpre = torch.randn(bsz, rows, 32, generator=g).to(DEV)
    ey = ops.to_vm(torch.nn.functional.elu(torch.randn(bsz, v, 32, generator=g)).to(DEV).bfloat16()) if with_elu else None
    w = (torch.randn(32, 288, generator=g) * 0.1).to(DEV)
    nb = ops.spiral_conv_bwd_weight_x_workspace(bsz, rows, 9, 32, 32)
    ws_a = torch.zeros(nb // 4 + 64, device=DEV)
    ws_b = torch.zeros_like(ws_a)
    dx_a = ops.vm_empty(bsz, v, 32, dtype=torch.bfloat16, device=DEV)
    dx_b = ops.vm_empty(bsz, v, 32, dtype=torch.bfloat16, device=DEV)
    d_a = ops.spiral_conv_bwd_rowsub_pair_bf16(x, rows_tab, dpre, flat, w, dx_a, elu_y=ey, workspace=ws_a)
    d_b = ops.spiral_conv_bwd_weight_x(x, rows_tab, dpre, None, None, ws_b)
    wsg = torch.empty(ops.spiral_conv_bwd_data_rowsub_workspace(bsz, rows, 9, 32) // 4 + 64, device=DEV)
    ops.spiral_conv_bwd_data_rowsub(dpre, flat, w, v, elu_y=ey, out=dx_b, workspace=wsg)
    dw_a, db_a = torch.empty(32, 288, device=DEV), torch.empty(32, device=DEV)
    dw_b, db_b = torch.empty_like(dw_a), torch.empty_like(db_a)
    ops.dw_reduce_batch([(d_a, dw_a, db_a), (d_b, dw_b, db_b)])
    assert torch.equal(dx_a, dx_b)
    assert torch.equal(dw_a, dw_b) and torch.equal(db_a, db_b)

