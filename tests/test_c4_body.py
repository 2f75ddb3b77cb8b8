"""C4: the body configuration (``configurations/body.yaml``) on a
synthetic 6 890-vertex torus hierarchy -- 3 Enblocks [32, 32, 64], latent 33,
kl_weight 0 (AE, ``model_manager.py:58,67``), laplacian_weight 1,
latent_consistency_weight 1, spiral length 9, sampling factors [4, 4, 4].

The body template is not in the reference snapshot, so there is no reference
output for this topology: parity here is HIP path vs the oracle (whose
per-op semantics are pinned on the craniofacial goldens), same tolerances as
C2 (losses rtol 1e-4, per-vertex L1 <= 1e-4, gradients rel 1e-4).
"""
import numpy as np
import pytest
import torch

import recipe
import synthetic_topology as ST
from oracle import cfsd_oracle as O

W_BODY = {"kl": 0.0, "lc": 1.0, "lap": 1.0}
OUT_CH = [32, 32, 64]
LATENT = 33


@pytest.fixture(scope="module")
def c4():
    npz = ST.torus_topology()
    return npz, O.Topology(npz)


def body_weights():
    shapes = recipe.param_shapes(num_vert=108, out_ch=OUT_CH, latent=LATENT, is_vae=False)
    return recipe.golden_weights(shapes, seed=4)


def test_c4_hierarchy_shape(c4):
    npz, T = c4
    assert T.n_verts == [6890, 1723, 431, 108]
    for l, sp in enumerate(T.spirals):
        assert sp.shape == (T.n_verts[l], 9)
        assert np.array_equal(sp[:, 0], np.arange(T.n_verts[l])), "spiral starts at the vertex"
        assert all(len(set(r)) == 9 for r in sp), "spiral entries distinct"
        row, col, val, shape = T.up[l]
        s = np.zeros(shape[0])
        np.add.at(s, row, val)
        np.testing.assert_allclose(s, 1.0, atol=1e-6)  # barycentric-like rows
        assert not np.all(np.diff(row) >= 0), "up COO must be row-unsorted (column order)"
    row, col, val, (n, _) = T.lap
    s = np.zeros(n)
    np.add.at(s, row, val)
    np.testing.assert_allclose(s, 0.0, atol=1e-6)     # rw Laplacian rows sum to 0
    assert len(T.region_keys) == 11


def test_c4_oracle_step_cpu(c4):
    """The oracle runs the AE step (no KL term, z = mu) on C4."""
    _, T = c4
    torch.manual_seed(0)
    P = O.make_params(body_weights())
    out, grads, x16 = O.train_step(P, O.Adam(P), ST.torus_meshes(4), T, 5, None, w=W_BODY,
                                   is_vae=False)
    assert out["kl"].item() == 0.0 and out["logvar"] is None
    assert torch.equal(out["z"], out["mu"])
    assert all(torch.isfinite(g).all() for g in grads.values())
    assert x16.shape == (16, 6890, 3)


# ----------------------------------------------------------------- GPU
def _engine(c4):
    from craniofacialsd_vae_amd import engine as E
    from craniofacialsd_vae_amd import topology
    npz, _ = c4
    dtopo = topology.DeviceTopology.from_npz(npz, device="cuda")
    eng = E.SDVAEEngine(dtopo, E.ModelSpec(3, OUT_CH, LATENT, is_vae=False), w_kl=W_BODY["kl"],
                        w_lc=W_BODY["lc"], w_lap=W_BODY["lap"], swap_bs=4, device="cuda")
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in body_weights().items()})
    return dtopo, eng


def _close(a, b, rel, what):
    a = a.detach().cpu().double().numpy()
    b = b.detach().cpu().double().numpy()
    err, tol = np.abs(a - b).max(), rel * (1.0 + np.abs(b).max())
    assert err <= tol, f"{what}: max err {err:.3e} > tol {tol:.3e}"


@pytest.mark.gpu
def test_c4_eval_per_vertex_l1(c4):
    import cfsd_loader
    cfsd_loader.load()
    torch.set_num_threads(1)
    _, T = c4
    _, eng = _engine(c4)
    meshes = ST.torus_meshes(8, seed=1)
    b = eng.set_batch(torch.from_numpy(meshes).cuda())
    eng.forward(b, train=False)
    torch.cuda.synchronize()
    P = O.make_params(body_weights())
    with torch.no_grad():
        rec, z, mu, _ = O.forward(P, torch.from_numpy(meshes), T, train=False, is_vae=False)
    d = np.abs(b.out.cpu().numpy() - rec.numpy()).sum(-1)
    assert d.max() <= 1e-4, f"max per-vertex L1 {d.max():.3e}"
    assert np.abs(b.z.cpu().numpy() - z.numpy()).max() <= 1e-4


@pytest.mark.gpu
def test_c4_train_three_steps(c4):
    """Swap (bit-exact), forward, MSE + Laplacian + latent consistency (AE:
    no KL), backward and Adam, three steps in lock-step with the oracle."""
    import cfsd_loader
    cfsd_loader.load()
    from craniofacialsd_vae_amd import ops
    torch.set_num_threads(1)
    _, T = c4
    dtopo, eng = _engine(c4)
    w = body_weights()
    P = O.make_params(w)
    opt = O.Adam(P)
    shadow = {k: torch.from_numpy(v.copy()) for k, v in w.items()}
    shadow_opt = O.Adam(shadow)
    meshes = ST.torus_meshes(12, seed=2)
    data = torch.from_numpy(meshes).cuda()
    for step in range(3):
        key = (2 + 4 * step) % 11
        out, grads, x16 = O.train_step(P, opt, meshes[4 * step:4 * step + 4], T, key, None,
                                       w=W_BODY, is_vae=False)
        b = eng.buffers(16)
        b.key.fill_(key)
        b.batch_idx.copy_(torch.arange(4 * step, 4 * step + 4, dtype=torch.int32))
        ops.swap_features(data, b.batch_idx, dtopo.region_mask, b.key, 4, out=b.x)
        eng.train_step_on(b)
        torch.cuda.synchronize()
        assert np.array_equal(b.x.cpu().numpy(), x16.numpy()), f"step {step}: swap differs"
        ref = np.array([out[k].item() for k in ("rec", "kl", "lc", "lap", "tot")])
        np.testing.assert_allclose(b.losses.cpu().numpy(), ref, rtol=1e-4, atol=1e-7)
        d = np.abs(b.out.cpu().numpy() - out["out"].detach().numpy()).sum(-1)
        assert d.max() <= 1e-4, f"step {step}: max per-vertex L1 {d.max():.3e}"
        hip_grads = {k: g.detach().cpu().clone() for k, g in eng.grads().items()}
        for name, g in hip_grads.items():
            _close(g, grads[name], 1e-4, f"step {step} grad {name}")
        # Adam: the device update equals the restated torch.optim.Adam rule
        # applied to the device's own gradients (1e-6).  Against the oracle's
        # parameters only |diff| <= 2*lr*(step+1) holds: Adam's first steps
        # move every element by ~lr*sign(g), so gradient entries below the
        # gradient tolerance (the 6912-wide AE Linear has many) may flip sign.
        shadow_opt.step(shadow, hip_grads)
        sd = eng.state_dict()
        for name in w:
            _close(sd[name], shadow[name], 1e-6, f"step {step} adam {name}")
            assert (sd[name].cpu() - P[name].detach()).abs().max() <= 2e-4 * (step + 1) + 1e-6
