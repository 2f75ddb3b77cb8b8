"""Micro-benchmark of individual step kernels at the C2 shapes (for rocprofv3 / PMC).

python tools/kbench.py [names...]   names: fwd_d3 dx_d3 dw_d3 dout_fwd dout_dx dout_dw spmm_up0 spmm_up0T step
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd import engine as E  # noqa: E402
from craniofacialsd_vae_amd import ops, topology  # noqa: E402


def locality_orders(spirals, n_coarsest=None):
    """Experiment (measured: no kernel changed by more than noise, so the
    product keeps the template numbering).  Per-level vertex orders with small spiral bandwidth (reverse
    Cuthill-McKee on the spiral adjacency).  ``order[l][i]`` is the original
    vertex stored at position i.  The template's own numbering spreads a
    32-row tile's spiral neighbours over ~10k rows, so a level-0 sweep touches
    the whole mesh and its L2 lines are evicted between reuses; in RCM order
    the neighbours of a tile lie within ~1k rows."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    orders = []
    for sp in spirals:
        sp = np.asarray(sp, np.int64)
        v = sp.shape[0]
        a = coo_matrix((np.ones(sp.size), (np.repeat(np.arange(v), sp.shape[1]), sp.ravel())),
                       shape=(v, v)).tocsr()
        orders.append(np.asarray(reverse_cuthill_mckee((a + a.T).tocsr(), symmetric_mode=True), np.int64))
    if n_coarsest is not None:
        orders.append(np.arange(n_coarsest, dtype=np.int64))
    return orders


def relabel_npz(npz, orders):
    """The arrays of a topology npz with level l's vertices renumbered so that
    new vertex i is original vertex ``orders[l][i]`` (COO entries keep their
    file order, so every per-row summation order is unchanged)."""
    n = int(npz["n_levels"])
    inv = []
    for o in orders:
        iv = np.empty(len(o), np.int64)
        iv[o] = np.arange(len(o))
        inv.append(iv)
    out = dict(npz)
    for l in range(n):
        out[f"spiral_{l}"] = inv[l][np.asarray(npz[f"spiral_{l}"], np.int64)[orders[l]]]
        out[f"down_{l}_row"] = inv[l + 1][np.asarray(npz[f"down_{l}_row"], np.int64)]
        out[f"down_{l}_col"] = inv[l][np.asarray(npz[f"down_{l}_col"], np.int64)]
        out[f"up_{l}_row"] = inv[l][np.asarray(npz[f"up_{l}_row"], np.int64)]
        out[f"up_{l}_col"] = inv[l + 1][np.asarray(npz[f"up_{l}_col"], np.int64)]
    if "lap_row" in npz:
        out["lap_row"] = inv[0][np.asarray(npz["lap_row"], np.int64)]
        out["lap_col"] = inv[0][np.asarray(npz["lap_col"], np.int64)]
    for k in list(npz.keys()):
        if k.startswith("region_") and (k.endswith("_feature") or k.endswith("_contour")):
            out[k] = inv[0][np.asarray(npz[k], np.int64)]
    return out


def build_cases(names=()):
    names = list(names)
    npz = dict(np.load(os.path.join(ROOT, "tests", "golden", "topology_craniofacial.npz")))
    if os.environ.get("KB_REORDER"):  # locality (RCM) vertex order on every level
        n = int(npz["n_levels"])
        orders = locality_orders([npz[f"spiral_{l}"] for l in range(n)], int(npz[f"down_{n - 1}_shape"][0]))
        npz = relabel_npz(npz, orders)
    T = topology.DeviceTopology.from_npz(npz, device="cuda")
    eng = E.SDVAEEngine(T, E.ModelSpec(), device="cuda", vertex_major=False)
    b = eng.buffers(16)
    g = torch.Generator(device="cuda").manual_seed(0)
    for t in (b.x, b.dec_up[3], b.dec_out[3], b.dpre_dec[3], b.dout, b.dec_out[2], b.g_dec_up[3]):
        t.copy_(torch.randn(t.shape, device="cuda", generator=g))
    b.dec_out[3].copy_(torch.nn.functional.elu(b.dec_out[3]))
    w3, b3 = eng._dec_w(3)
    wout = eng.params.view("de_layers.5.layer.weight")
    bout = eng.params.view("de_layers.5.layer.bias")
    P = eng.params
    cases = {
        "fwd_d3": lambda: ops.spiral_conv_fwd(b.dec_up[3], T.spiral[0], w3, b3, 1, out=b.dec_out[3], workspace=b.ws),
        "dx_d3": lambda: ops.spiral_conv_bwd_data(b.dpre_dec[3], T.spiral_inv[0], w3, T.n_verts[0], out=b.g_dec_up[3], workspace=b.ws),
        "dw_d3": lambda: ops.spiral_conv_bwd_weight(b.dec_up[3], T.spiral[0], b.dpre_dec[3],
                                                   P.gview("de_layers.4.conv.layer.weight"),
                                                   P.gview("de_layers.4.conv.layer.bias"), b.ws),
        "dout_fwd": lambda: ops.spiral_conv_fwd(b.dec_out[3], T.spiral[0], wout, bout, 0, out=b.out, workspace=b.ws),
        "dout_dx": lambda: ops.spiral_conv_bwd_data(b.dout, T.spiral_inv[0], wout, T.n_verts[0], elu_y=b.dec_out[3],
                                                    out=b.dpre_dec[3], workspace=b.ws),
        "dout_dw": lambda: ops.spiral_conv_bwd_weight(b.dec_out[3], T.spiral[0], b.dout,
                                                     P.gview("de_layers.5.layer.weight"),
                                                     P.gview("de_layers.5.layer.bias"), b.ws),
        "dout_bwd": lambda: ops.spiral_conv_bwd(b.dec_out[3], T.spiral[0], b.dout, T.spiral_inv[0], wout,
                                                P.gview("de_layers.5.layer.weight"),
                                                P.gview("de_layers.5.layer.bias"), dx=b.dpre_dec[3],
                                                elu_y=b.dec_out[3], workspace=b.ws),
        "spmm_up0": lambda: ops.spmm(T.up_csr[0], b.dec_out[2], T.n_verts[0], out=b.dec_up[3]),
        "spmm_up1": lambda: ops.spmm(T.up_csr[1], b.dec_out[1], T.n_verts[1], out=b.dec_up[2]),
        "spmm_up0u": lambda: ops.spmm(T.up_csr[0], b.dec_out[2], T.n_verts[0], out=b.dec_up[3],
                                      uniform=T.up_uniform[0]),
        "spmm_up1u": lambda: ops.spmm(T.up_csr[1], b.dec_out[1], T.n_verts[1], out=b.dec_up[2],
                                      uniform=T.up_uniform[1]),
        "spmm_up2": lambda: ops.spmm(T.up_csr[2], b.dec_out[0], T.n_verts[2], out=b.dec_up[1]),
        "spmm_up3": lambda: ops.spmm(T.up_csr[3], b.h, T.n_verts[3], out=b.dec_up[0]),
        "spmm_up1T": lambda: ops.spmm(T.upT_csr[1], b.g_dec_up[2], T.n_verts[2], elu_y=b.dec_out[1],
                                      out=b.dpre_dec[1]),
        "spmm_up2T": lambda: ops.spmm(T.upT_csr[2], b.g_dec_up[1], T.n_verts[3], elu_y=b.dec_out[0],
                                      out=b.dpre_dec[0]),
        "spmm_up3T": lambda: ops.spmm(T.upT_csr[3], b.g_dec_up[0], T.n_verts[4], out=b.dh),
        "spmm_up0T": lambda: ops.spmm(T.upT_csr[0], b.g_dec_up[3], T.n_verts[1], elu_y=b.dec_out[2],
                                      out=b.dpre_dec[2]),
        "e0_fwd": lambda: ops.spiral_conv_fwd(b.x, T.enc_rows[0], *eng._enc_w(0), 1, out=b.enc_out[0], workspace=b.ws),
        "e0_dw": lambda: ops.spiral_conv_bwd_weight(b.x, T.enc_rows[0], b.dpre_enc[0],
                                                   P.gview("en_layers.0.conv.layer.weight"),
                                                   P.gview("en_layers.0.conv.layer.bias"), b.ws),
    }
    for lv, (gin, outb, ey) in enumerate([(b.g_dec_up[3], b.dpre_dec[2], b.dec_out[2]),
                                           (b.g_dec_up[2], b.dpre_dec[1], b.dec_out[1]),
                                           (b.g_dec_up[1], b.dpre_dec[0], b.dec_out[0]),
                                           (b.g_dec_up[0], b.dh, None)]):
        cases[f"spmm_up{lv}T_s"] = (lambda lv=lv, gin=gin, outb=outb, ey=ey: ops.spmm(
            T.upT_csr[lv], gin, T.n_verts[lv + 1], elu_y=ey, out=outb, order=T.upT_order[lv]))
        cases[f"spmm_up{lv}T_c"] = (lambda lv=lv, gin=gin, outb=outb, ey=ey: ops.spmm(
            T.upT_csr[lv], gin, T.n_verts[lv + 1], elu_y=ey, out=outb, sched=T.upT_sched[lv]))
    w2d, b2d = eng._dec_w(2)
    for t in (b.dpre_dec[2], b.g_dec_up[2]):
        t.copy_(torch.randn(t.shape, device="cuda", generator=g))
    cases["dx_d2"] = lambda: ops.spiral_conv_bwd_data(b.dpre_dec[2], T.spiral_inv[1], w2d, T.n_verts[1],
                                                      out=b.g_dec_up[2], workspace=b.ws)
    cases["dw_d2"] = lambda: ops.spiral_conv_bwd_weight(b.dec_up[2], T.spiral[1], b.dpre_dec[2],
                                                       P.gview("de_layers.3.conv.layer.weight"),
                                                       P.gview("de_layers.3.conv.layer.bias"), b.ws)
    cases["fwd_d2"] = lambda: ops.spiral_conv_fwd(b.dec_up[2], T.spiral[1], *eng._dec_w(2), 1, out=b.dec_out[2],
                                                  workspace=b.ws)
    # coarse decoder / encoder layers (latency-shaped kernels)
    w0, b0 = eng._dec_w(0)
    w1, b1 = eng._dec_w(1)
    for t in (b.dec_up[0], b.dec_up[1], b.dpre_dec[0], b.dpre_dec[1], b.enc_out[0], b.dpre_enc[1]):
        t.copy_(torch.randn(t.shape, device="cuda", generator=g))
    cases["fwd_d0"] = lambda: ops.spiral_conv_fwd(b.dec_up[0], T.spiral[3], w0, b0, 1, out=b.dec_out[0], workspace=b.ws)
    cases["dx_d0"] = lambda: ops.spiral_conv_bwd_data(b.dpre_dec[0], T.spiral_inv[3], w0, T.n_verts[3],
                                                      out=b.g_dec_up[0], workspace=b.ws)
    cases["dw_d0"] = lambda: ops.spiral_conv_bwd_weight(b.dec_up[0], T.spiral[3], b.dpre_dec[0],
                                                       P.gview("de_layers.1.conv.layer.weight"),
                                                       P.gview("de_layers.1.conv.layer.bias"), b.ws)
    cases["pair_d0"] = lambda: ops.spiral_conv_bwd(b.dec_up[0], T.spiral[3], b.dpre_dec[0], T.spiral_inv[3], w0,
                                                   None, None, dx=b.g_dec_up[0], workspace=b.ws_dw[("dec", 0)])
    cases["fwd_d1"] = lambda: ops.spiral_conv_fwd(b.dec_up[1], T.spiral[2], w1, b1, 1, out=b.dec_out[1], workspace=b.ws)
    cases["pair_d1"] = lambda: ops.spiral_conv_bwd(b.dec_up[1], T.spiral[2], b.dpre_dec[1], T.spiral_inv[2], w1,
                                                   P.gview("de_layers.2.conv.layer.weight"),
                                                   P.gview("de_layers.2.conv.layer.bias"), dx=b.g_dec_up[1],
                                                   workspace=b.ws_dw[("dec", 1)])
    cases["dx_d1"] = lambda: ops.spiral_conv_bwd_data(b.dpre_dec[1], T.spiral_inv[2], w1, T.n_verts[2],
                                                      out=b.g_dec_up[1], workspace=b.ws)
    cases["dw_d1"] = lambda: ops.spiral_conv_bwd_weight(b.dec_up[1], T.spiral[2], b.dpre_dec[1], None, None,
                                                       b.ws_dw[("dec", 1)])
    we1, be1 = eng._enc_w(1)
    cases["dw_e1"] = lambda: ops.spiral_conv_bwd_weight(b.enc_out[0], T.enc_rows[1], b.dpre_enc[1], None, None,
                                                       b.ws_dw[("enc", 1)])
    for lv in (2, 3):
        cases[f"fwd_e{lv}"] = (lambda lv=lv: ops.spiral_conv_fwd(b.enc_out[lv - 1], T.enc_rows[lv], *eng._enc_w(lv), 1,
                                                                 out=b.enc_out[lv], workspace=b.ws))
    cases["fwd_e1"] = lambda: ops.spiral_conv_fwd(b.enc_out[0], T.enc_rows[1], we1, be1, 1, out=b.enc_out[1], workspace=b.ws)
    cases["rowsub_e1"] = lambda: ops.spiral_conv_bwd_rowsub(b.enc_out[0], T.enc_rows[1], b.dpre_enc[1], T.enc_flat[1],
                                                            we1, None, None, dx=b.dpre_enc[0], elu_y=b.enc_out[0],
                                                            workspace=b.ws_dw[("enc", 1)])
    self_idx = torch.arange(T.n_verts[0], dtype=torch.int32, device="cuda").view(-1, 1).repeat(1, 9).contiguous()
    shift_idx = ((torch.arange(T.n_verts[0], device="cuda").view(-1, 1) + torch.arange(9, device="cuda").view(1, -1))
                 % T.n_verts[0]).to(torch.int32).contiguous()
    cases["fwd_d3_self"] = lambda: ops.spiral_conv_fwd(b.dec_up[3], self_idx, w3, b3, 1, out=b.dec_out[3], workspace=b.ws)
    cases["fwd_d3_shift"] = lambda: ops.spiral_conv_fwd(b.dec_up[3], shift_idx, w3, b3, 1, out=b.dec_out[3], workspace=b.ws)
    cases["fwd_d3_noact"] = lambda: ops.spiral_conv_fwd(b.dec_up[3], T.spiral[0], w3, b3, 0, out=b.dec_out[3], workspace=b.ws)
    ip, ir, ipair = T.spiral_inv[0]
    inv_noovf = (torch.zeros_like(ip), ir, ipair)
    pair1 = ipair.clone()
    pair1[:, 1:] = -1
    inv_nomore = (ip, ir, pair1)
    pair3 = ipair.clone()
    pair3[:, 3] = -1
    inv_now = (ip, ir, pair3)  # timing only: no rows 3.. (no exec branch)
    cases["dx_d3_now"] = lambda: ops.spiral_conv_bwd_data(b.dpre_dec[3], inv_now, w3, T.n_verts[0], out=b.g_dec_up[3], workspace=b.ws)
    cases["dx_d3_noovf"] = lambda: ops.spiral_conv_bwd_data(b.dpre_dec[3], inv_noovf, w3, T.n_verts[0], out=b.g_dec_up[3], workspace=b.ws)
    cases["dx_d3_nomore"] = lambda: ops.spiral_conv_bwd_data(b.dpre_dec[3], inv_nomore, w3, T.n_verts[0], out=b.g_dec_up[3], workspace=b.ws)
    cases["dout_bwd_noovf"] = lambda: ops.spiral_conv_bwd(b.dec_out[3], T.spiral[0], b.dout, inv_noovf, wout,
                                                         P.gview("de_layers.5.layer.weight"),
                                                         P.gview("de_layers.5.layer.bias"), dx=b.dpre_dec[3],
                                                         elu_y=b.dec_out[3], workspace=b.ws)
    cases["dout_bwd_nodx"] = lambda: ops.spiral_conv_bwd(b.dec_out[3], T.spiral[0], b.dout, T.spiral_inv[0], wout,
                                                        P.gview("de_layers.5.layer.weight"),
                                                        P.gview("de_layers.5.layer.bias"), workspace=b.ws)
    for lv in (1, 2, 3):  # Enblock data gradients (latency-shaped kernels)
        cases[f"dx_e{lv}"] = (lambda lv=lv: ops.spiral_conv_bwd_data(
            b.dpre_enc[lv], T.enc_inv[lv], eng._enc_w(lv)[0], T.n_verts[lv], elu_y=b.enc_out[lv - 1],
            out=b.dpre_enc[lv - 1], workspace=b.ws))
    # the fused bottleneck backward on the engine's buffers (kprof with CFSD_BN_EXP phases)
    cases["bneck"] = lambda: eng._bottleneck_bwd_fused(b)
    W_enc, B_enc = eng._enc_lin()
    gW_enc, gB_enc = eng._enc_lin(P.grad)
    flat = b.enc_out[3].view(16, -1)
    flat.copy_(torch.randn(flat.shape, device="cuda", generator=g))
    Wd, Bd = P.view("de_layers.0.weight"), P.view("de_layers.0.bias")
    cases["lin_enc_fwd"] = lambda: ops.linear_fwd(flat, W_enc, B_enc, out=b.mulv)
    cases["lin_dec_fwd"] = lambda: ops.linear_fwd(b.z, Wd, Bd, out=b.h.view(16, -1))
    cases["lin_dec_dx"] = lambda: ops.linear_bwd(b.z, Wd, b.dh.view(16, -1), dx=b.dz)
    cases["lin_dec_dw"] = lambda: ops.linear_bwd(b.z, None, b.dh.view(16, -1), dw=P.gview("de_layers.0.weight"),
                                                 db=P.gview("de_layers.0.bias"))
    cases["lin_enc_dx"] = lambda: ops.linear_bwd(flat, W_enc, b.dmulv, dx=b.dpre_enc[3].view(16, -1), elu_y=flat)
    cases["lin_enc_dw"] = lambda: ops.linear_bwd(flat, None, b.dmulv, dw=gW_enc.view(W_enc.shape), db=gB_enc)
    # bf16 D3 kernels (configs C3/C5), the step's own launch arguments
    e16 = E.SDVAEEngine(T, E.ModelSpec(), device="cuda", precision="bf16")
    c = e16.buffers(16)
    for t in (c.dec_up[3], c.dec_out[3], c.dpre_dec[3]):
        t.copy_(torch.randn(t.shape, device="cuda", generator=g))
    w3h, b3h = e16._dec_w(3)
    w16 = e16._w16("de_layers.4.conv.layer.weight")
    cases["fwd_d3_b16"] = lambda: ops.spiral_conv_fwd_x(c.dec_up[3], T.spiral[0], w3h, w16, b3h, 1, c.dec_out[3])
    cases["dx_d3_b16"] = lambda: ops.spiral_conv_bwd_data_x(c.dpre_dec[3], T.spiral_inv[0], w16, T.n_verts[0],
                                                            out=c.g_dec_up[3])
    cases["dxf_d3_b16"] = lambda: ops.spiral_conv_bwd_data_flat(c.dpre_dec[3], T.spiral_flat[0], w16, T.n_verts[0],
                                                                out=c.g_dec_up[3])
    cases["dw_d3_b16"] = lambda: ops.spiral_conv_bwd_weight_x(c.dec_up[3], T.spiral[0], c.dpre_dec[3], None, None,
                                                              c.ws_dw[("dec", 3)])
    cases["pair_d3_b16"] = lambda: ops.spiral_conv_bwd_flat_pair_bf16(c.dec_up[3], T.spiral[0], c.dpre_dec[3],
                                                                      T.spiral_flat[0], w16, c.g_dec_up[3],
                                                                      workspace=c.ws_dw[("dec", 3)])
    cases["spmm_up0T_b16"] = lambda: ops.spmm_x(T.upT_csr[0], c.g_dec_up[3], T.n_verts[1], elu_y=c.dec_out[2],
                                                out=c.dpre_dec[2], sched=T.upT_nat[0])
    cases["spmm_up0_b16"] = lambda: ops.spmm_x(T.up_csr[0], c.dec_out[2], T.n_verts[0], out=c.dec_up[3],
                                               uniform=T.up_uniform[0])
    cases["spmm_up1_b16"] = lambda: ops.spmm_x(T.up_csr[1], c.dec_out[1], T.n_verts[1], out=c.dec_up[2],
                                               uniform=T.up_uniform[1])
    cases["dw_e1_b16"] = lambda: ops.spiral_conv_bwd_weight_x(c.enc_out[0], T.enc_rows[1], c.dpre_enc[1], None, None,
                                                              c.ws_dw[("enc", 1)])
    cases["dw_d2_b16"] = lambda: ops.spiral_conv_bwd_weight_x(c.dec_up[2], T.spiral[1], c.dpre_dec[2], None, None,
                                                              c.ws_dw[("dec", 2)])
    c.dout.copy_(torch.randn(c.dout.shape, device="cuda", generator=g))
    wo16 = e16.params.view("de_layers.5.layer.weight")
    cases["dout_bwd_flat_b16"] = lambda: ops.spiral_conv_bwd_out_flat(c.dec_out[3], T.spiral[0], c.dout,
                                                                      T.spiral_flat[0], wo16, None, None,
                                                                      dx=c.dpre_dec[3], elu_y=c.dec_out[3],
                                                                      workspace=c.ws_dw["out"])
    bm_up, bm_out = c.dec_up[3].contiguous(), c.dec_out[3].contiguous()
    bm_dp, bm_g = c.dpre_dec[3].contiguous(), c.g_dec_up[3].contiguous()
    cases["fwd_d3_b16_bm"] = lambda: ops.spiral_conv_fwd_x(bm_up, T.spiral[0], w3h, w16, b3h, 1, bm_out)
    cases["dx_d3_b16_bm"] = lambda: ops.spiral_conv_bwd_data_x(bm_dp, T.spiral_inv[0], w16, T.n_verts[0], out=bm_g)
    cases["dw_d3_b16_bm"] = lambda: ops.spiral_conv_bwd_weight_x(bm_up, T.spiral[0], bm_dp, None, None,
                                                                 c.ws_dw[("dec", 3)])
    for mult in (2, 4):  # work scaling of the vertex-major forward (fixed-cost check)
        xin = ops.to_vm(torch.randn(16 * mult, T.n_verts[0], 32, device="cuda", generator=g).to(torch.bfloat16))
        yout = ops.vm_empty(16 * mult, T.n_verts[0], 32, dtype=torch.bfloat16, device="cuda")
        cases[f"fwd_d3_b16_x{mult}"] = (lambda xin=xin, yout=yout:
                                        ops.spiral_conv_fwd_x(xin, T.spiral[0], w3h, w16, b3h, 1, yout))
    cases["fwd_d3_b16_self"] = lambda: ops.spiral_conv_fwd_x(c.dec_up[3], self_idx, w3h, w16, b3h, 1, c.dec_out[3])
    cases["fwd_d3_b16_shift"] = lambda: ops.spiral_conv_fwd_x(c.dec_up[3], shift_idx, w3h, w16, b3h, 1, c.dec_out[3])
    # fp32 vertex-major kernels (the fp32 step's level-0/1 layers at batch 16)
    ev = E.SDVAEEngine(T, E.ModelSpec(), device="cuda", vertex_major=True)
    v = ev.buffers(16)
    for t in (v.dec_up[3], v.dec_out[3], v.dpre_dec[3], v.dec_up[2], v.dpre_dec[2], v.enc_out[0],
              v.dpre_enc[0], v.dpre_enc[1]):
        t.copy_(torch.randn(t.shape, device="cuda", generator=g))
    v.dec_out[3].copy_(torch.nn.functional.elu(v.dec_out[3]))
    w3v, b3v = ev._dec_w(3)
    cases["fwd_d3_vm"] = lambda: ops.spiral_conv_fwd_x(v.dec_up[3], T.spiral[0], w3v, None, b3v, 1, v.dec_out[3])
    # diagnosis of the D3 forward: gathers that hit L1 (self), neighbours in
    # index order (shift), no ELU epilogue, and twice the meshes (fixed costs)
    cases["fwd_d3_vm_self"] = lambda: ops.spiral_conv_fwd_x(v.dec_up[3], self_idx, w3v, None, b3v, 1, v.dec_out[3])
    cases["fwd_d3_vm_shift"] = lambda: ops.spiral_conv_fwd_x(v.dec_up[3], shift_idx, w3v, None, b3v, 1, v.dec_out[3])
    cases["fwd_d3_vm_noact"] = lambda: ops.spiral_conv_fwd_x(v.dec_up[3], T.spiral[0], w3v, None, b3v, 0, v.dec_out[3])
    x32 = ops.to_vm(torch.randn(32, T.n_verts[0], 32, device="cuda", generator=g))
    y32 = ops.vm_empty(32, T.n_verts[0], 32, dtype=torch.float32, device="cuda")
    cases["fwd_d3_vm_x2"] = lambda: ops.spiral_conv_fwd_x(x32, T.spiral[0], w3v, None, b3v, 1, y32)
    cases["dxf_d3_vm"] = lambda: ops.spiral_conv_bwd_data_flat(v.dpre_dec[3], T.spiral_flat[0], w3v, T.n_verts[0],
                                                               out=v.g_dec_up[3])
    cases["dw_d3_vm"] = lambda: ops.spiral_conv_bwd_weight_x(v.dec_up[3], T.spiral[0], v.dpre_dec[3], None, None,
                                                             v.ws_dw[("dec", 3)])
    w2v, b2v = ev._dec_w(2)
    cases["fwd_d2_vm"] = lambda: ops.spiral_conv_fwd_x(v.dec_up[2], T.spiral[1], w2v, None, b2v, 1, v.dec_out[2])
    cases["dxf_d2_vm"] = lambda: ops.spiral_conv_bwd_data_flat(v.dpre_dec[2], T.spiral_flat[1], w2v, T.n_verts[1],
                                                               out=v.g_dec_up[2])
    cases["dw_d2_vm"] = lambda: ops.spiral_conv_bwd_weight_x(v.dec_up[2], T.spiral[1], v.dpre_dec[2], None, None,
                                                             v.ws_dw[("dec", 2)])
    # the fp32 step's D2 backward: flat dx + vm32 dW slabs in one launch (conv_bwd_vm_pair)
    cases["pair_d2_vm"] = lambda: ops.spiral_conv_bwd_flat_pair(v.dec_up[2], T.spiral[1], v.dpre_dec[2],
                                                                T.spiral_flat[1], w2v, None, None, v.g_dec_up[2],
                                                                workspace=v.ws_dw[("dec", 2)])
    wov, bov = ev.params.view("de_layers.5.layer.weight"), ev.params.view("de_layers.5.layer.bias")
    cases["dout_fwd_vm"] = lambda: ops.spiral_conv_fwd_x(v.dec_out[3], T.spiral[0], wov, None, bov, 0, v.out)
    cases["dout_bwd_vm"] = lambda: ops.spiral_conv_bwd_x(v.dec_out[3], T.spiral[0], v.dout, T.spiral_inv[0], wov,
                                                         None, None, dx=v.dpre_dec[3], elu_y=v.dec_out[3],
                                                         workspace=v.ws_dw["out"])
    cases["dout_bwd_flat"] = lambda: ops.spiral_conv_bwd_out_flat(v.dec_out[3], T.spiral[0], v.dout, T.spiral_flat[0],
                                                                  wov, None, None, dx=v.dpre_dec[3],
                                                                  elu_y=v.dec_out[3], workspace=v.ws_dw["out"])
    cases["e0_fwd_vm"] = lambda: ops.spiral_conv_fwd_x(v.x, T.enc_rows[0], *ev._enc_w(0)[:1], None, ev._enc_w(0)[1],
                                                       1, v.enc_out[0])
    cases["e0_dw_vm"] = lambda: ops.spiral_conv_bwd_weight_x(v.x, T.enc_rows[0], v.dpre_enc[0], None, None,
                                                             v.ws_dw[("enc", 0)])
    cases["fwd_e1_vm"] = lambda: ops.spiral_conv_fwd_x(v.enc_out[0], T.enc_rows[1], ev._enc_w(1)[0], None,
                                                       ev._enc_w(1)[1], 1, v.enc_out[1])
    cases["dw_e1_vm"] = lambda: ops.spiral_conv_bwd_weight_x(v.enc_out[0], T.enc_rows[1], v.dpre_enc[1], None, None,
                                                             v.ws_dw[("enc", 1)])
    we1v = ev._enc_w(1)[0]
    cases["rowsub_e1_vm"] = lambda: ops.spiral_conv_bwd_rowsub(v.enc_out[0], T.enc_rows[1], v.dpre_enc[1],
                                                               T.enc_flat[1], we1v, None, None, dx=v.dpre_enc[0],
                                                               elu_y=v.enc_out[0], workspace=v.ws_dw[("enc", 1)])
    cases["dgonly_e1_vm"] = lambda: ops.spiral_conv_bwd_data_rowsub(v.dpre_enc[1], T.enc_flat[1], we1v, T.n_verts[1],
                                                                    elu_y=v.enc_out[0], out=v.dpre_enc[0],
                                                                    workspace=v.ws)
    cases["spmm_up0_vm"] = lambda: ops.spmm_x(T.up_csr[0], v.dec_out[2], T.n_verts[0], out=v.dec_up[3],
                                              uniform=T.up_uniform[0])
    cases["spmm_up0T_vm"] = lambda: ops.spmm_x(T.upT_csr[0], v.g_dec_up[3], T.n_verts[1], elu_y=v.dec_out[2],
                                               out=v.dpre_dec[2], sched=T.upT_nat[0])
    # the coarse chain exactly as the fp32 vertex-major step launches it
    for t in (v.h, v.dec_up[0], v.dec_up[1], v.dpre_dec[0], v.dpre_dec[1], v.g_dec_up[1], v.g_dec_up[0],
              v.enc_out[1], v.enc_out[2], v.enc_out[3], v.dpre_enc[2], v.dpre_enc[3], v.dh, v.z, v.mulv):
        t.copy_(torch.randn(t.shape, device="cuda", generator=g))
    w0v, b0v = ev._dec_w(0)
    w1v, b1v = ev._dec_w(1)
    Pv = ev.params
    cases["fwd_d0_up"] = lambda: ops.spiral_conv_fwd_up(v.h, T.up_comp[3], T.spiral[3], w0v, b0v, 1,
                                                        out=v.dec_out[0], up_out=v.dec_up[0])
    cases["fwd_d1_vm"] = lambda: ops.spiral_conv_fwd(v.dec_up[1], T.spiral[2], w1v, b1v, 1, out=v.dec_out[1],
                                                     workspace=v.ws)
    cases["pair_d1_vm"] = lambda: ops.spiral_conv_bwd(v.dec_up[1], T.spiral[2], v.dpre_dec[1], T.spiral_inv[2], w1v,
                                                      None, None, dx=v.g_dec_up[1], workspace=v.ws_dw[("dec", 1)])
    cases["pair_d0_vm"] = lambda: ops.spiral_conv_bwd(v.dec_up[0], T.spiral[3], v.dpre_dec[0], T.spiral_inv[3], w0v,
                                                      None, None, dx=v.g_dec_up[0], workspace=v.ws_dw[("dec", 0)])
    for lv in (2, 3):
        cases[f"fwd_e{lv}_vm"] = (lambda lv=lv: ops.spiral_conv_fwd(v.enc_out[lv - 1], T.enc_rows[lv], *ev._enc_w(lv), 1,
                                                                    out=v.enc_out[lv], workspace=v.ws))
    cases["rowsub_e2_vm"] = lambda: ops.spiral_conv_bwd_rowsub(v.enc_out[1], T.enc_rows[2], v.dpre_enc[2], T.enc_flat[2],
                                                               ev._enc_w(2)[0], None, None, dx=v.dpre_enc[1],
                                                               elu_y=v.enc_out[1], workspace=v.ws_dw[("enc", 2)])
    cases["rowsub_e3_vm"] = lambda: ops.spiral_conv_bwd_rowsub(v.enc_out[2], T.enc_rows[3], v.dpre_enc[3], T.enc_flat[3],
                                                               ev._enc_w(3)[0], None, None, dx=v.dpre_enc[2],
                                                               elu_y=v.enc_out[2], workspace=v.ws_dw[("enc", 3)])
    for lv, (gin, outb, ey) in enumerate([(v.g_dec_up[2], v.dpre_dec[1], v.dec_out[1]),
                                          (v.g_dec_up[1], v.dpre_dec[0], v.dec_out[0]),
                                          (v.g_dec_up[0], v.dh, None)], start=1):
        cases[f"spmm_up{lv}T_vm"] = (lambda lv=lv, gin=gin, outb=outb, ey=ey: ops.spmm_x(
            T.upT_csr[lv], gin, T.n_verts[lv + 1], elu_y=ey, out=outb,
            sched=T.upT_nat[lv] if lv == 1 else T.upT_sched[lv]))  # level 1 is vertex-major (engine.backward_head)
    Wdv, Bdv = Pv.view("de_layers.0.weight"), Pv.view("de_layers.0.bias")
    W_encv, _ = ev._enc_lin()
    gW_encv, gB_encv = ev._enc_lin(Pv.grad)
    flatv = v.enc_out[3].view(16, -1)
    cases["lin_dec_split"] = lambda: ops.linear_bwd_split(v.z, Wdv, v.dh.view(16, -1), v.dz_parts,
                                                          Pv.gview("de_layers.0.weight"), Pv.gview("de_layers.0.bias"))
    cases["latent_bwd"] = lambda: ops.latent_bwd(v.mulv, v.eps, v.z, v.dz_parts, v.dlat, v.dmulv, 75, True, True, False)
    cases["lin_enc_pair"] = lambda: ops.linear_bwd(flatv, W_encv, v.dmulv, dx=v.dpre_enc[3].view(16, -1),
                                                   dw=gW_encv.view(W_encv.shape), db=gB_encv, elu_y=flatv)
    cases["lin_enc_fwd_vm"] = lambda: ops.linear_fwd(flatv, W_encv, ev._enc_lin()[1], out=v.mulv, workspace=v.lin_ws)
    if "red_items" in names:  # the step's batched slab reduce, item by item (HIP events)
        cap = []
        orig = ops.dw_reduce_batch
        ops.dw_reduce_batch = lambda items, adam=None: (cap.append((list(items), adam)), orig(items, adam=adam))[1]
        ev.set_batch(b.x, key_index=3)
        ev.train_step_on(v)
        ops.dw_reduce_batch = orig
        items, adam = cap[-1]
        for i, it in enumerate(items):
            cases[f"red_item{i}"] = (lambda it=it: orig([it]))
            print(f"red_item{i}: sizes {it[0].sizes}", flush=True)
        cases["red_all"] = lambda: orig(items)
        cases["red_all_adam"] = lambda: orig(items, adam=adam)
        names = [n for n in names if n != "red_items"] + [f"red_item{i}" for i in range(len(items))] + [
            "red_all", "red_all_adam"]
    if "step_vm" in names:
        ev.set_batch(b.x, key_index=3)
        cases["step_vm"] = lambda: ev.train_step_on(v)
    if "step" in names:
        eng.set_batch(b.x, key_index=3)
        cases["step"] = lambda: eng.train_step_on(b)
    return cases, names, b


def main():
    names = sys.argv[1:] or ["fwd_d3", "dx_d3", "dw_d3", "dout_fwd", "dout_dx", "dout_dw", "spmm_up0",
                             "spmm_up0T", "e0_fwd", "e0_dw"]
    iters = int(os.environ.get("KB_ITERS", "50"))
    cases, names, b = build_cases(names)
    if os.environ.get("KB_PTSTAMPS"):  # -DCFSD_LAT_STAMPS build: conv_fwd_pt first-tile phases (wave 0)
        import ctypes
        from craniofacialsd_vae_amd import _abi
        case = os.environ["KB_PTSTAMPS"]
        for _ in range(5):
            cases[case]()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (2048 * 6))()
        rc = _abi.lib().cfsd_debug_pt_stamps(buf)
        st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 6).astype(np.int64)
        st = st[st[:, 0] > 0]
        t0 = st[:, 0].min()
        print(f"{case} conv_fwd_pt stamps rc {rc}: {len(st)} workgroups (us from the first start; min p10 p50 p90 max)")
        for c, nm in enumerate(["start", "W slice in", "tables in", "x taps in", "tile 1 done", "end"]):
            print(f"  {nm:12s} {np.round(np.percentile((st[:, c] - t0) / 100.0, [0, 10, 50, 90, 100]), 2)}")
        return
    if os.environ.get("KB_LATSTAMPS"):  # library built with -DCFSD_LAT_STAMPS: conv_bwd_lat_pair roles
        import ctypes
        from craniofacialsd_vae_amd import _abi
        case = os.environ["KB_LATSTAMPS"]
        for _ in range(5):
            cases[case]()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4096 * 3))()
        fn = os.environ.get("KB_STAMPFN", "cfsd_debug_lat_stamps")  # cfsd_debug_ks_stamps: the coarse ks pair
        rc = getattr(_abi.lib(), fn)(buf)
        st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3).astype(np.int64)
        st = st[st[:, 0] > 0]
        t0 = st[:, 1].min()
        print(f"{case} lat-pair stamps rc {rc}: {len(st)} workgroups, span {(st[:, 2].max() - t0) / 100:.2f} us")
        for role, nm in ((1, "dx"), (2, "dW")):
            r = st[st[:, 0] == role]
            q = lambda c: np.round(np.percentile((r[:, c] - t0) / 100.0, [0, 10, 50, 90, 100]), 2)
            print(f"  {nm} n={len(r)}  start {q(1)}  end {q(2)}  dur p50 {np.median((r[:, 2] - r[:, 1]) / 100):.2f}")
        return
    if os.environ.get("KB_BNSTAMPS"):  # diagnostic library built with -DCFSD_BN_STAMPS
        import ctypes
        from craniofacialsd_vae_amd import _abi
        bn_case = os.environ.get("KB_BNCASE", "bneck")
        for _ in range(5):
            cases[bn_case]()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4096 * 5))()
        rc = _abi.lib().cfsd_debug_bn_stamps(buf)
        st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 5).astype(np.int64)
        st = st[st[:, 1] > 0]
        t0 = st[:, 1].min()
        print(f"bneck stamps rc {rc}: {len(st)} workgroups, span {(st[:, 4].max() - t0) / 100:.2f} us (100 MHz clock)")
        for role, nm in enumerate(["A dz parts", "L latent", "D dW_d", "E dx", "E dW"]):
            r = st[st[:, 0] == role]
            if len(r) == 0:
                continue
            q = lambda c: np.percentile((r[:, c] - t0) / 100.0, [0, 50, 100])
            print(f"  {nm:11s} n={len(r):4d}  start {q(1)}  mark1 {q(2)}  mark2 {q(3)}  end {q(4)}")
        return
    if os.environ.get("KB_STAMPS"):
        for n in names:
            b.ws.zero_()
            cases[n]()
            torch.cuda.synchronize()
            st = b.ws.view(torch.int64)[: (b.ws.numel() // 2) // 8 * 8].view(-1, 8).cpu()
            st = st[st[:, 7] == 1].double()
            if len(st) == 0:
                print(n, "no stamps")
                continue
            tiles = st[:, 5].sum()
            print(f"{n}: waves {len(st)} tiles/wave {st[:, 5].mean():.2f} | per wave (cycles): prologue {st[:, 0].mean():.0f} "
                  f"total {st[:, 6].mean():.0f} max {st[:, 6].max():.0f} | per tile: idx {st[:, 1].sum() / tiles:.0f} "
                  f"slot0-wait {st[:, 2].sum() / tiles:.0f} slots {st[:, 3].sum() / tiles:.0f} epilogue {st[:, 4].sum() / tiles:.0f}")
        return
    for n in names:
        fn = cases[n]
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{n:10s} {e0.elapsed_time(e1) / iters * 1e3:9.2f} us", flush=True)


if __name__ == "__main__":
    main()
