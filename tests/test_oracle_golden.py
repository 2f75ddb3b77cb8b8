"""Pin the CPU oracle against vectors produced by the reference itself
(``tests/golden/make_golden.py``).  CPU only."""
import numpy as np
import pytest
import torch

import recipe
from oracle import cfsd_oracle as O

torch.set_num_threads(1)  # goldens were generated single-threaded


@pytest.fixture(scope="module")
def ops():
    return dict(np.load(f"{recipe.HERE}/golden_ops.npz"))


def test_spiral_conv_fwd_bwd(ops, otopo):
    x = torch.from_numpy(ops["conv_x"]).requires_grad_()
    w = torch.from_numpy(ops["conv_w"]).requires_grad_()
    b = torch.from_numpy(ops["conv_b"]).requires_grad_()
    y = O.spiral_conv(x, otopo.spirals[3], w, b)
    y.backward(torch.from_numpy(ops["conv_dy"]))
    np.testing.assert_allclose(y.detach().numpy(), ops["conv_y"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(x.grad.numpy(), ops["conv_dx"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(w.grad.numpy(), ops["conv_dw"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(b.grad.numpy(), ops["conv_db"], rtol=1e-5, atol=1e-5)
    y2 = O.spiral_conv(x.detach()[0], otopo.spirals[3], w.detach(), b.detach())
    np.testing.assert_allclose(y2.numpy(), ops["conv2d_y"], rtol=0, atol=2e-6)


def test_spiral_conv_rank_error(otopo):
    with pytest.raises(RuntimeError):
        O.spiral_conv(torch.zeros(1, 1, 267, 3), otopo.spirals[3], torch.zeros(2, 27), None)


@pytest.mark.parametrize("name,level,kind", [("down3", 3, "down"), ("up3", 3, "up"), ("up2", 2, "up")])
def test_pool_fwd_bwd(ops, otopo, name, level, kind):
    coo = (otopo.down if kind == "down" else otopo.up)[level]
    x = torch.from_numpy(ops[f"pool_{name}_x"]).requires_grad_()
    out = O.pool(x, coo)
    out.backward(torch.from_numpy(ops[f"pool_{name}_dout"]))
    np.testing.assert_array_equal(out.detach().numpy(), ops[f"pool_{name}_out"])
    np.testing.assert_allclose(x.grad.numpy(), ops[f"pool_{name}_dx"], rtol=0, atol=1e-5)


def test_swap_bit_exact(otopo):
    g = np.load(f"{recipe.HERE}/golden_swap.npz")
    base = recipe.normalized_meshes(4)
    for k in range(len(otopo.region_keys)):
        assert recipe.sha256(O.swap_features(base, otopo.region_features, k)) == str(g["sha"][k])
    k = otopo.region_keys.index(str(g["call_key"]))
    assert recipe.sha256(O.swap_features(base, otopo.region_features, k)) == str(g["call_x_sha"])
    ny, na, nage, ng = O.swap_labels(4, ["a", "b", "c", "n"], np.zeros((4, 1), np.float32),
                                     np.arange(4, dtype=np.float32).reshape(4, 1),
                                     ["M", "F", "M", "F"])
    np.testing.assert_array_equal(na, g["call_aug"])
    np.testing.assert_array_equal(nage, g["call_age"])
    assert [str(v) for v in ny] == list(g["call_y"])
    assert ng == list(g["call_gender"])


def test_eval_c1(otopo):
    g = np.load(f"{recipe.HERE}/golden_eval.npz")
    w = recipe.golden_weights()
    assert recipe.weights_sha256(w) == str(g["weights_sha"])
    P = {k: torch.from_numpy(v) for k, v in w.items()}
    with torch.no_grad():
        out, z, mu, lv = O.forward(P, torch.from_numpy(recipe.normalized_meshes(8)), otopo, train=False)
    d = np.abs(out.numpy() - g["recon"]).sum(-1)
    assert d.max() <= 1e-5, d.max()
    np.testing.assert_allclose(mu.numpy(), g["mu"], atol=1e-5)
    np.testing.assert_allclose(lv.numpy(), g["logvar"], atol=1e-5)


def test_train_three_steps(otopo):
    g = np.load(f"{recipe.HERE}/golden_train.npz")
    w = recipe.golden_weights()
    P = O.make_params(w)
    opt = O.Adam(P)
    names = list(w.keys())
    meshes = recipe.normalized_meshes(12)
    for step in range(3):
        p = f"s{step}_"
        out, grads, x16 = O.train_step(P, opt, meshes[4 * step:4 * step + 4], otopo,
                                       recipe.train_key_index(step), recipe.train_eps(step))
        assert recipe.sha256(x16.numpy()) == str(g[p + "x_sha"])
        got = np.array([out[k].item() for k in ("rec", "kl", "lc", "lap", "tot")])
        np.testing.assert_allclose(got, g[p + "losses"], rtol=2e-5)
        np.testing.assert_allclose(out["z"].detach().numpy(), g[p + "z"], atol=2e-5)
        for n in names:
            gs = grads[n].double().numpy().ravel()
            ref = g[p + "grad_stats_" + n]
            np.testing.assert_allclose(np.abs(gs).sum(), ref[1], rtol=1e-3)
            scale = np.abs(g[p + "grad_sample_" + n]).max() + 1e-12
            np.testing.assert_allclose(gs[recipe.sample_idx(gs.size)], g[p + "grad_sample_" + n],
                                       atol=2e-3 * scale)
            ps = P[n].detach().numpy().ravel()
            np.testing.assert_allclose(ps[recipe.sample_idx(ps.size)], g[p + "param_sample_" + n],
                                       atol=2e-6)
