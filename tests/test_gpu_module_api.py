"""Drop-in module API (reference model.py signatures) on the HIP path."""
import numpy as np
import pytest
import torch

import cfsd_loader
import recipe
from oracle import cfsd_oracle as O

pytestmark = pytest.mark.gpu

cfsd_loader.load()
from craniofacialsd_vae_amd import model as M  # noqa: E402

DEV = "cuda"


def ref_inputs(npz):
    """What the reference passes to Model: int64 spirals + sparse COO transforms."""
    n = int(npz["n_levels"])
    spirals = [torch.from_numpy(npz[f"spiral_{l}"].astype(np.int64)).to(DEV) for l in range(n)]

    def sp(name, l):
        idx = np.stack([npz[f"{name}_{l}_row"], npz[f"{name}_{l}_col"]]).astype(np.int64)
        return torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(npz[f"{name}_{l}_val"]),
                                       tuple(npz[f"{name}_{l}_shape"].tolist())).to(DEV)

    return spirals, [sp("down", l) for l in range(n)], [sp("up", l) for l in range(n)]


@pytest.fixture(scope="module")
def model(topo_npz):
    spirals, down, up = ref_inputs(topo_npz)
    m = M.Model(3, [32, 32, 32, 64], 75, spirals, down, up, pre_z_sigmoid=False, is_vae=True).to(DEV)
    w = recipe.golden_weights()
    assert list(m.state_dict().keys()) == list(w.keys())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    return m


def test_repr_and_errors(topo_npz):
    spirals, _, _ = ref_inputs(topo_npz)
    conv = M.SpiralConv(32, 64, spirals[3]).to(DEV)
    assert repr(conv) == "SpiralConv(32, 64, seq_length=9)"
    with pytest.raises(RuntimeError):
        conv(torch.zeros(1, 1, 267, 32, device=DEV))


def test_eval_matches_golden(model):
    g = np.load(f"{recipe.HERE}/golden_eval.npz")
    model.eval()
    with torch.no_grad():
        out, z, mu, lv = model(torch.from_numpy(recipe.normalized_meshes(8)).to(DEV))
    d = np.abs(out.cpu().numpy() - g["recon"]).sum(-1)
    assert d.max() <= 1e-4
    assert np.abs(mu.cpu().numpy() - g["mu"]).max() <= 1e-4
    assert np.abs(lv.cpu().numpy() - g["logvar"]).max() <= 1e-4


def test_unbatched_spiral_conv(topo_npz):
    gops = np.load(f"{recipe.HERE}/golden_ops.npz")
    spirals, _, _ = ref_inputs(topo_npz)
    conv = M.SpiralConv(32, 64, spirals[3]).to(DEV)
    conv.layer.weight.data.copy_(torch.from_numpy(gops["conv_w"]))
    conv.layer.bias.data.copy_(torch.from_numpy(gops["conv_b"]))
    y = conv(torch.from_numpy(gops["conv_x"][0]).to(DEV))
    np.testing.assert_allclose(y.detach().cpu().numpy(), gops["conv2d_y"], atol=2e-5)


def test_train_backward_matches_oracle(model, otopo):
    """Gradients of a random linear functional of (out, z) vs the oracle."""
    model.train()
    w = recipe.golden_weights()
    x = torch.from_numpy(recipe.normalized_meshes(4))
    x16 = torch.cat([x, x, x, x])
    eps = torch.from_numpy(recipe.train_eps(0))
    g = torch.Generator().manual_seed(11)
    r_out = torch.randn(16, 17039, 3, generator=g)
    r_z = torch.randn(16, 75, generator=g)
    model.zero_grad()
    out, z, mu, lv = model(x16.to(DEV), eps=eps.to(DEV))
    ((out * r_out.to(DEV)).sum() + (z * r_z.to(DEV)).sum()).backward()
    P = O.make_params(w)
    oo, oz, _, _ = O.forward(P, x16, otopo, eps=eps, train=True)
    ((oo * r_out).sum() + (oz * r_z).sum()).backward()
    for name, p in model.named_parameters():
        ref = P[name].grad.numpy()
        got = p.grad.cpu().numpy()
        err = np.abs(got - ref).max() / (1 + np.abs(ref).max())
        assert err < 1e-4, (name, err)
